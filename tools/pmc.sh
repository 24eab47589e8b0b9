#!/usr/bin/env bash
# PMC passes over a short bench (one pass per counter group; never combined with trace domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $counters -d "$R/gpurun_out/pmc/p$i" -o run --output-format csv \
      -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-profile $BENCH_ARGS \
      > "$R/gpurun_out/pmc/p$i.log" 2>&1) || { echo "pass $i rc=$?"; exit 1; }
  echo "pass $i ok: $counters"
done <<< "${PASSES}"
