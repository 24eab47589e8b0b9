#!/usr/bin/env bash
# t-digest GPU tests, then a C5t rocprof kernel summary with sync input (k_td_* durations)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
LIMIT=300 FILES="tests/test_gpu_tdigest.py tests/test_gpu_pool_state.py" bash tools/gpu_tests.sh || exit 1
R=$PWD; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p5t5 -o run --output-format csv \
  -- python3 $R/bench.py --workload c5t --steps 12 --warmup 2 --no-cpu-baseline --host-fed-steps 0 --no-profile --sync-input > $R/gpurun_out/p5t5.log 2>&1
