#!/usr/bin/env bash
# Ablation / sweep timing.  FW_DIAG bits (fw_internal.h) price stages of k_scatter / k_aggregate
# (results are wrong under them); SUBS sweeps the state partitions per key group.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for d in ${DIAGS:-0}; do
  for s in ${SUBS:-0}; do
    echo "== FW_DIAG=$d SUB=$s" >> gpurun_out/diag.log
    FW_DIAG=$d timeout -k 10 120 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --sub-partitions $s \
        >> gpurun_out/diag.log 2>&1 || exit $?
  done
done
