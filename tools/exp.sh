#!/usr/bin/env bash
# Optional GPU parity suite, then the bench once per variant (VARIANTS: ';'-separated env assignments,
# "-" = none, optionally '|' then extra bench arguments), each summarised as records/s, ms/step and per-kernel average ms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" = "0" ]; then
  timeout -k 10 ${TEST_LIMIT:-480} python -u -m pytest ${FILES:-tests} -m gpu -x -q --timeout 120 --timeout-method thread \
      ${K:+-k "$K"} > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
: > gpurun_out/exp.log
IFS=';' read -ra VS <<< "${VARIANTS:--}"
for v in "${VS[@]}"; do
  echo "== $v $BENCH_ARGS" >> gpurun_out/exp.log
  a=""; case "$v" in *"|"*) a="${v#*|}"; v="${v%%|*}";; esac   # "ENV=.. | --bench-arg .."
  [ "$v" = "-" ] && v=""
  env $v timeout -k 10 150 python -u bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --host-fed-steps 0 \
      $BENCH_ARGS $a >> gpurun_out/exp.log 2>&1 || exit $?
done
python3 - <<'PY'
import json
for l in open("gpurun_out/exp.log"):
    if l.startswith("=="): print(l.strip())
    if l.startswith("{"):
        d = json.loads(l)
        print("%.4g rec/s  %.4f ms/step" % (d["value"], d["ms_per_step"]),
              {k: round(v["avg_ms"], 4) for k, v in d["kernels"].items()})
PY
