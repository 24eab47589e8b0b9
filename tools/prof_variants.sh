#!/usr/bin/env bash
# rocprofv3 kernel stats of the bench under each build variant (diagnostics): VARIANTS="a b" W=c5t bash tools/prof_variants.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; export TMPDIR=/tmp
for v in $VARIANTS; do
  d="$R/gpurun_out/pv/$v"; mkdir -p "$d"
  lib="$R/flink_amd/_lib/variants/lib_$v.so"; [ "$v" = main ] && lib="$R/flink_amd/_lib/libflinkwin.so"
  (cd /tmp && FW_LIB="$lib" timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$d" -o run --output-format csv \
      -- python3 "$R/bench.py" --workload ${W:-c5t} --steps ${S:-6} --warmup 2 --no-cpu-baseline --host-fed-steps 0 \
      --no-profile --sync-input > "$d/log" 2>&1) || { echo "$v rc=$?"; tail -5 "$d/log"; exit 1; }
  echo "== $v"; python3 tools/kstats.py "$d/run_kernel_stats.csv" | head -${TOP:-16}
done
