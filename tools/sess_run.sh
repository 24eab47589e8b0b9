#!/usr/bin/env bash
# GPU parity tests, then the C2 bench and a short C4 (sessions) bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2.log | cut -c1-300
timeout -k 10 300 python -u bench.py --workload c4 --steps 5 --warmup 2 > gpurun_out/bench_c4.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c4.log
