#!/usr/bin/env bash
# PMC HBM-traffic passes (FETCH_SIZE, WRITE_SIZE: one rocprofv3 run each) for the C2, C3 and C5 benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; export TMPDIR=/tmp
for w in ${WORKLOADS:-c2 c3 c5}; do
  d="$R/gpurun_out/pmc_$w"; mkdir -p "$d"
  i=0
  for counters in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $counters -d "$d/p$i" -o run --output-format csv \
        -- python3 "$R/bench.py" --workload $w --steps ${PMC_STEPS:-3} --warmup 1 --no-cpu-baseline --no-profile --host-fed-steps 0 \
        > "$d/p$i.log" 2>&1) || { echo "$w pass $i rc=$?"; tail -5 "$d/p$i.log"; exit 1; }
    echo "$w pass $i ok: $counters"
  done
  python3 tools/traffic.py "$d" --workload $w --last ${PMC_STEPS:-3} --out "gpurun_out/traffic_$w.json" | tail -12
done
