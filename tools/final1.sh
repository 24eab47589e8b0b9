#!/usr/bin/env bash
# Round evidence, part 1: GPU parity suite, smoke(), C2 PMC traffic passes, bench lines C2 / C1 / C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
WORKLOADS="c2 c4" bash tools/pmc_all.sh > gpurun_out/pmc.log 2>&1 || { tail -5 gpurun_out/pmc.log; exit 1; }
echo "pmc ok"
for w in c2 c1 c4; do
  tr=""; [ -f gpurun_out/traffic_$w.json ] && tr="--traffic gpurun_out/traffic_$w.json"
  timeout -k 10 300 python -u bench.py --workload $w $tr > gpurun_out/bench_$w.log 2>&1
  rc=$?; echo "bench $w rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$w.log; exit $rc; }
done
