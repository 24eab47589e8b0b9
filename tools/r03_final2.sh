#!/usr/bin/env bash
# Round-3 close-out, part 1: the whole GPU parity suite, the list benches, C2 and C1 evidence (each step under its
# own limit; stop at the first failure).  Part 2: WORKLOADS="c3 c4 c5 c5t" S=24 bash tools/evidence.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
LIMIT=600 bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python3 -u tools/bench_list.py > gpurun_out/bench_list.json 2> gpurun_out/bench_list.err || { tail -5 gpurun_out/bench_list.err; exit 1; }
tail -1 gpurun_out/bench_list.json
timeout -k 10 300 python3 -u tools/bench_list.py --evictor count:8 --no-cpu-baseline > gpurun_out/bench_list_evict.json 2> gpurun_out/bench_list_evict.err || { tail -5 gpurun_out/bench_list_evict.err; exit 1; }
tail -1 gpurun_out/bench_list_evict.json
WORKLOADS="c2 c1" S=24 bash tools/evidence.sh
