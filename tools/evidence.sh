#!/usr/bin/env bash
# Round evidence for one or more workloads (WORKLOADS, default c2): for each, with S timed steps (>= one firing
# period) after W warmup steps:
#   PMC passes FETCH_SIZE and WRITE_SIZE (one rocprofv3 run each, no trace domains) -> traffic_${ROUND:-r06}_$w.json
#   rocprofv3 --kernel-trace --stats of the bench with async input and with --sync-input (no HIP-event pass)
#   the bench line itself (default flags, the traffic file above)
#   tools/roofline_check.py: the line's frac / isolated frac recomputed from the traces
# Everything under gpurun_out/ev/$w/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; export TMPDIR=/tmp
S=${S:-12}; W=${W:-2}
for w in ${WORKLOADS:-c2}; do
  d="$R/gpurun_out/ev/$w"; mkdir -p "$d"
  ba="--workload $w --steps $S --warmup $W --no-cpu-baseline --host-fed-steps 0 ${EXTRA:-}"
  i=0
  for counters in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $counters -d "$d/pmc/p$i" -o run --output-format csv \
        -- python3 "$R/bench.py" $ba --no-profile > "$d/pmc_p$i.log" 2>&1) || { echo "$w pmc $i rc=$?"; tail -5 "$d/pmc_p$i.log"; exit 1; }
  done
  python3 tools/traffic.py "$d/pmc" --workload $w --steps $S --warmup $W --out "$d/traffic_${ROUND:-r06}_$w.json" > "$d/traffic.txt" || exit 1
  for mode in async sync; do
    extra=""; [ $mode = sync ] && extra="--sync-input"
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d/prof_$mode" -o run --output-format csv \
        -- python3 "$R/bench.py" $ba --no-profile $extra > "$d/prof_$mode.log" 2>&1) || { echo "$w prof $mode rc=$?"; tail -5 "$d/prof_$mode.log"; exit 1; }
  done
  timeout -k 10 400 python3 -u bench.py $ba --traffic "$d/traffic_${ROUND:-r06}_$w.json" > "$d/bench.json" 2> "$d/bench.err" || { echo "$w bench rc=$?"; tail -5 "$d/bench.err"; exit 1; }
  python3 tools/roofline_check.py "$d/bench.json" --async-trace "$d/prof_async/run_kernel_trace.csv" \
      --sync-trace "$d/prof_sync/run_kernel_trace.csv" --steps $S --warmup $W --out "$d/roofline_check.json" > /dev/null || exit 1
  python3 - "$d" <<'PY'
import json, sys
d = sys.argv[1]
b = json.loads([l for l in open(d + "/bench.json") if l.startswith("{")][-1])
c = json.load(open(d + "/roofline_check.json"))
print(d.split("/")[-1], "value %.4g" % b["value"], "ms %.4f" % b["ms_per_step"], "frac", b["roofline"]["frac"],
      "iso", (b["roofline"].get("isolated") or {}).get("frac"), "rocprof", c["rocprof"]["frac"], c["rocprof"]["isolated_frac"],
      "traffic/rec", b["roofline"].get("traffic_per_record"))
PY
  tail -1 "$d/traffic.txt"
done
