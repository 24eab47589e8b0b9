#!/usr/bin/env bash
# list-path GPU tests, then the list bench with apply and with CountEvictor 8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
FILES="tests/test_gpu_list.py tests/test_gpu_heapstate.py" LIMIT=300 bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python3 -u tools/bench_list.py > gpurun_out/bench_list.json 2> gpurun_out/bench_list.err || { tail -5 gpurun_out/bench_list.err; exit 1; }
tail -1 gpurun_out/bench_list.json
timeout -k 10 300 python3 -u tools/bench_list.py --evictor count:8 --no-cpu-baseline > gpurun_out/bench_list_evict.json 2> gpurun_out/bench_list_evict.err || { tail -5 gpurun_out/bench_list_evict.err; exit 1; }
tail -1 gpurun_out/bench_list_evict.json
