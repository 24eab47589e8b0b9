#!/usr/bin/env bash
# Pane-mode check: pane/sliding parity tests, then the steady-state C3 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "panes or sliding or kats or burst or rescale" > gpurun_out/c3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/c3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} \
    > gpurun_out/b3.log 2>&1 || exit $?
grep "^{" gpurun_out/b3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel'], d['roofline']['frac'], d['path_roofline']['frac'], {k:round(v['avg_ms'],3) for k,v in d['kernels'].items()})"
