#!/usr/bin/env bash
# GPU parity tests, then bench timings under FW_DIAG values (DIAGS, default "0"), summarised.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" = "0" ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} \
      > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
: > gpurun_out/diag.log
for d in ${DIAGS:-0}; do
  echo "== FW_DIAG=$d $BENCH_ARGS" >> gpurun_out/diag.log
  FW_DIAG=$d timeout -k 10 120 python -u bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline $BENCH_ARGS \
      >> gpurun_out/diag.log 2>&1 || exit $?
done
python3 - <<'PY'
import json
for l in open("gpurun_out/diag.log"):
    if l.startswith("=="): print(l.strip())
    if l.startswith("{"):
        d = json.loads(l)
        print("%.4g rec/s  %.4f ms/step" % (d["value"], d["ms_per_step"]),
              {k: round(v["avg_ms"], 4) for k, v in d["kernels"].items()})
PY
