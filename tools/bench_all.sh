#!/usr/bin/env bash
# Bench lines for the given workloads (WORKLOADS, default all), each under its own limit; a failure ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for w in ${WORKLOADS:-c2 c1 c3 c4 c5 c5t}; do
  timeout -k 10 300 python -u bench.py --workload $w ${BENCH_ARGS:-} > gpurun_out/bench_$w.log 2>&1
  rc=$?; echo "bench $w rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$w.log; exit $rc; }
done
python3 - <<'PY'
import json, os
for w in ("c2", "c1", "c3", "c4", "c5", "c5t"):
    f = f"gpurun_out/bench_{w}.log"
    if not os.path.exists(f):
        continue
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            r = d["roofline"] or {}
            print(w, "%.4g" % d["value"], "ms/step", d["ms_per_step"], r.get("kernel"), "frac", r.get("frac"),
                  "path", d["path_roofline"]["frac"], "host_fed %.4g" % (d["host_fed"] or {}).get("value", 0),
                  "cpu", (d["cpu_baseline"] or {}).get("value"),
                  {k: v["avg_ms"] for k, v in d["kernels"].items()})
PY
