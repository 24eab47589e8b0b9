cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/hll; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "hll or HLL or hyperloglog or pool or snapshot" > gpurun_out/hll/tests.log 2>&1 || { echo tests rc=$?; tail -30 gpurun_out/hll/tests.log; exit 1; }
tail -2 gpurun_out/hll/tests.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/hll/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c5 --steps 14 --warmup 2 --no-cpu-baseline --host-fed-steps 0 --no-profile --sync-input > "$GRAFT_REPO_ROOT/gpurun_out/hll/prof.log" 2>&1) || { echo prof rc=$?; exit 1; }
grep '^{' gpurun_out/hll/prof.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/hll/prof/run_kernel_stats.csv")):
    if float(r["TotalDurationNs"])/1e6 > 1: print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1000,1))
PY
