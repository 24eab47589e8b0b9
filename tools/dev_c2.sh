cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/c2t; export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --host-fed-steps 0 > gpurun_out/c2t/prof$i.json 2> gpurun_out/c2t/prof$i.err || exit 1
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --host-fed-steps 0 --no-profile > gpurun_out/c2t/noprof$i.json 2> gpurun_out/c2t/noprof$i.err || exit 1
done
python3 - <<'PY'
import json
for f in ["prof1","noprof1","prof2","noprof2"]:
    d=json.loads([l for l in open(f"gpurun_out/c2t/{f}.json") if l.startswith("{")][-1])
    print(f, "%.4g"%d["value"], d["ms_per_step"], {k:round(v["avg_ms"],4) for k,v in (d.get("kernels") or {}).items()}, d["roofline"]["frac"] if d.get("roofline") else None)
PY
WORKLOADS="c2" S=12 W=2 bash tools/evidence.sh
