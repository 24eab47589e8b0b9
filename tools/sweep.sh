#!/usr/bin/env bash
# Batch-size sweep of the bench (one process per point, short runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for b in ${BATCHES:-16777216}; do
  echo "== BATCH=$b $EXTRA" >> gpurun_out/sweep.log
  timeout -k 10 120 python -u bench.py --steps ${STEPS:-12} --warmup 3 --no-cpu-baseline --batch $b $EXTRA \
      >> gpurun_out/sweep.log 2>&1 || exit $?
done
