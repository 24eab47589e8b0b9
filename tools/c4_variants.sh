#!/usr/bin/env bash
# C4 and related variants (session vs tumbling, Zipf vs uniform keys): per-kernel timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/c4_variants.log
run() {
  echo "== $*" >> gpurun_out/c4_variants.log
  timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" >> gpurun_out/c4_variants.log 2>&1 || exit $?
}
run --workload c4
run --workload c4 --zipf 0
run --workload c4 --sub-partitions 64
run --workload c2 --zipf 1.1
run --workload c2 --zipf 1.1 --rate 100000 --bound 1000 --jitter 1000
python3 - <<'PY'
import json
for l in open("gpurun_out/c4_variants.log"):
    if l.startswith("=="): print(l.strip())
    if l.startswith("{"):
        d = json.loads(l)
        print("%.4g rec/s  %.4f ms/step" % (d["value"], d["ms_per_step"]),
              {k: round(v["avg_ms"], 4) for k, v in d["kernels"].items()})
PY
