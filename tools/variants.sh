#!/usr/bin/env bash
# Build-variant timing (diagnostics): for each "name:EXTRA flags" in VARIANTS (built here on the CPU
# into flink_amd/_lib/variants/), run the bench with FW_LIB pointing at it.  Usage on the GPU box:
#   VARIANTS="a:-DFW_RPT=4 b:..." bash tools/variants.sh run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ "${1:-}" = "build" ]; then
  for v in $VARIANTS; do
    name=${v%%:*}; flags=${v#*:}; flags=${flags//,/ }
    make -s -j4 -C flink_amd/csrc OUT=../_lib/variants LIBNAME=lib_$name.so EXTRA="$flags" || exit 1
  done
  exit 0
fi
mkdir -p gpurun_out; export TMPDIR=/tmp; : > gpurun_out/variants.log
for v in $VARIANTS; do
  name=${v%%:*}
  for d in ${DIAGS:-0}; do
    echo "== $v FW_DIAG=$d" >> gpurun_out/variants.log
    FW_DIAG=$d FW_LIB=$PWD/flink_amd/_lib/variants/lib_$name.so timeout -k 10 120 python -u bench.py --steps ${STEPS:-10} \
        --warmup 3 --no-cpu-baseline $BENCH_ARGS >> gpurun_out/variants.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/variants.log"):
    if l.startswith("=="): print(l.strip())
    if l.startswith("{"):
        d = json.loads(l)
        print("%.4g rec/s  %.4f ms/step" % (d["value"], d["ms_per_step"]),
              {k: round(v["avg_ms"], 4) for k, v in d["kernels"].items()})
PY
