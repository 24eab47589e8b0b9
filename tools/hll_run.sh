#!/usr/bin/env bash
# HLL GPU check: the HLL parity tests, then the C5 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "hll" > gpurun_out/hll_tests.log 2>&1
rc=$?; echo "hll tests rc=$rc"; tail -8 gpurun_out/hll_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench_c5.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench_c5.log | head -c 3000; tail -3 gpurun_out/bench_c5.log; exit $rc
