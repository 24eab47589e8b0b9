#!/usr/bin/env bash
# Round evidence: full GPU parity suite, then the C2 headline bench, the C3/C4/C5 benches and a
# rocprofv3 kernel trace of the C2 bench.  Each GPU step has its own limit; a failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py > gpurun_out/bench_c2.log 2>&1 || exit $?
for w in c3 c4 c5; do
  timeout -k 10 240 python -u bench.py --workload $w --steps 20 --warmup 3 > gpurun_out/bench_$w.log 2>&1 || exit $?
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" \
    -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline \
    > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
cd "$GRAFT_REPO_ROOT" && python3 - <<'PY'
import json
for w in ("c2", "c3", "c4", "c5"):
    for l in open(f"gpurun_out/bench_{w}.log"):
        if l.startswith("{"):
            d = json.loads(l)
            print(w, "%.4g" % d["value"], d["roofline"]["kernel"], d["roofline"]["frac"],
                  d["path_roofline"]["frac"], (d["cpu_baseline"] or {}).get("value"))
PY
exit $rc
