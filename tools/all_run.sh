#!/usr/bin/env bash
# Round evidence: full GPU parity suite, smoke(), the C2 headline bench, the C3/C4/C5 benches, a
# rocprofv3 kernel trace of the C2 bench and of the C3 bench, and the C5 PMC traffic passes.
# Each GPU step has its own limit; a failure ends the session.  SKIP_TESTS=1 / SKIP_BENCH=1 skip parts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" = "0" ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
if [ "${SKIP_BENCH:-0}" = "0" ]; then
  timeout -k 10 240 python -u bench.py > gpurun_out/bench_c2.log 2>&1 || exit $?
  for w in c3 c4 c5; do
    timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 3 > gpurun_out/bench_$w.log 2>&1 || exit $?
  done
fi
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" \
    -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline \
    > "$R/gpurun_out/prof.log" 2>&1) || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c3" \
    -o run --output-format csv -- python3 "$R/bench.py" --workload c3 --steps 10 --warmup 3 --no-cpu-baseline \
    > "$R/gpurun_out/prof_c3.log" 2>&1) || exit $?
echo "rocprof ok"
WORKLOADS=c5 bash tools/pmc_all.sh > gpurun_out/pmc_c5.log 2>&1 || exit $?
echo "pmc c5 ok"
python3 - <<'PY'
import json, os
for w in ("c2", "c3", "c4", "c5"):
    f = f"gpurun_out/bench_{w}.log"
    if not os.path.exists(f):
        continue
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(w, "%.4g" % d["value"], d["roofline"]["kernel"], d["roofline"]["frac"],
                  d["path_roofline"]["frac"], (d["cpu_baseline"] or {}).get("value"))
PY
