#!/usr/bin/env bash
# list-path GPU tests, then the list bench (apply) and a rocprof kernel summary of it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
FILES="tests/test_gpu_list.py tests/test_gpu_heapstate.py" LIMIT=300 bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python3 -u tools/bench_list.py --no-cpu-baseline > gpurun_out/bench_list.json 2> gpurun_out/bench_list.err || { tail -5 gpurun_out/bench_list.err; exit 1; }
tail -1 gpurun_out/bench_list.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_list -o run --output-format csv -- python3 $R/tools/bench_list.py --no-cpu-baseline > $R/gpurun_out/prof_list.log 2>&1; echo "rocprof rc=$?"
