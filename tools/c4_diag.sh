#!/usr/bin/env bash
# k_aggregate phase clocks (FW_DIAG=256) for C4 with uniform keys vs C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/c4_diag.log
for a in "--workload c4 --zipf 0" "--workload c2"; do
  echo "== $a" >> gpurun_out/c4_diag.log
  FW_DIAG=256 timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline $a >> gpurun_out/c4_diag.log 2>&1 || exit $?
done
grep -E "^==|agg timing|session flush" gpurun_out/c4_diag.log
