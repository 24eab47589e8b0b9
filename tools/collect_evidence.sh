#!/usr/bin/env bash
# Copy tools/evidence.sh outputs (gpurun_out/ev/<workload>/) into profiles/<round>_<v>/ under the names the docs cite,
# and each workload's PMC traffic summary to profiles/ (where bench.py looks for it).
cd "$(dirname "$0")/.."
out=profiles/${1:?profiles subdirectory, e.g. r05_v1}; mkdir -p "$out"
for d in gpurun_out/ev/*/; do
  w=$(basename "$d"); [ -f "$d/bench.json" ] || continue
  cp "$d/bench.json" "$out/bench_$w.json"
  cp "$d/prof_async/run_kernel_stats.csv" "$out/kernel_stats_${w}_async.csv"
  cp "$d/prof_sync/run_kernel_stats.csv" "$out/kernel_stats_${w}_sync.csv"
  cp "$d/roofline_check.json" "$out/roofline_check_$w.json"
  cp "$d/traffic.txt" "$out/traffic_$w.txt"
  for t in "$d"/traffic_r*_"$w".json; do cp "$t" "$out/"; cp "$t" profiles/; done
  echo "$w -> $out"
done
