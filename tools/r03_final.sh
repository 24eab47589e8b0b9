#!/usr/bin/env bash
# Round-3 close-out on the final tree: the whole GPU parity suite, the list bench and the C2 evidence
# (each step under its own limit; stop at the first failure)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
LIMIT=600 bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python3 -u tools/bench_list.py > gpurun_out/bench_list.json 2> gpurun_out/bench_list.err || { tail -5 gpurun_out/bench_list.err; exit 1; }
tail -1 gpurun_out/bench_list.json
WORKLOADS="${WORKLOADS:-c2}" S=24 bash tools/evidence.sh
