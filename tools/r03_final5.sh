#!/usr/bin/env bash
# Round-3 close-out after the HLL read change: the whole GPU parity suite, smoke, C5 evidence
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
LIMIT=600 bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
WORKLOADS="c5" S=24 bash tools/evidence.sh
