#!/usr/bin/env bash
# Copies the judged parts of gpurun_out/ev/<workload>/ (tools/evidence.sh) into profiles/$1/:
# the bench line, rocprof kernel stats (async / sync input), PMC traffic and the roofline recomputation.
set -e
cd "$(dirname "$0")/.."
dst=profiles/$1; mkdir -p "$dst"
for d in gpurun_out/ev/*/; do
  w=$(basename "$d")
  [ -f "$d/bench.json" ] || continue
  grep '^{' "$d/bench.json" | tail -1 > "$dst/bench_$w.json"
  for m in async sync; do
    [ -f "$d/prof_$m/run_kernel_stats.csv" ] && cp "$d/prof_$m/run_kernel_stats.csv" "$dst/kernel_stats_${w}_$m.csv"
  done
  cp "$d"/traffic_r03_*.json "$dst/" 2>/dev/null || true
  [ -f "$d/traffic.txt" ] && cp "$d/traffic.txt" "$dst/traffic_$w.txt"
  [ -f "$d/roofline_check.json" ] && cp "$d/roofline_check.json" "$dst/roofline_check_$w.json"
done
[ -f gpurun_out/gpu_tests.log ] && tail -3 gpurun_out/gpu_tests.log > "$dst/gpu_tests_tail.txt"
[ -f gpurun_out/smoke.log ] && tail -1 gpurun_out/smoke.log > "$dst/smoke.txt"
ls "$dst"
