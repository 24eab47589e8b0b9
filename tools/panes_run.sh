#!/usr/bin/env bash
# Pane-mode GPU check: the sliding parity tests, then the whole GPU suite, then the C3 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "panes or burst" > gpurun_out/panes_tests.log 2>&1
rc=$?; echo "pane tests rc=$rc"; tail -5 gpurun_out/panes_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench_c3.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench_c3.log | head -c 2500; exit $rc
