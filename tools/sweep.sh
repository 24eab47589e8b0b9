#!/usr/bin/env bash
# Parameter sweep of bench.py (one line per configuration) into gpurun_out/sweep.log.
# ARGS_LIST: ';'-separated bench argument sets; COMMON: arguments added to each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/sweep.log
IFS=';' read -ra SETS <<< "$ARGS_LIST"
for a in "${SETS[@]}"; do
  echo "== $a" >> gpurun_out/sweep.log
  timeout -k 10 ${LIMIT:-180} python3 bench.py $a ${COMMON:---steps 10 --warmup 3 --no-cpu-baseline --host-fed-steps 0} \
      > gpurun_out/sweep_one.log 2>&1 || { echo "rc=$? for $a"; tail -5 gpurun_out/sweep_one.log; exit 1; }
  python3 - >> gpurun_out/sweep.log <<'PY'
import json
for line in open("gpurun_out/sweep_one.log"):
    if line.startswith("{"):
        d = json.loads(line)
        ks = d.get("kernels", {})
        print(f"value={d['value']:.4g} ms={d['ms_per_step']:.4f} frac={d['roofline']['frac']} path={d.get('path_roofline',{}).get('frac')} " +
              " ".join(f"{k}={v['avg_ms']:.4f}" for k, v in ks.items()))
PY
done
cat gpurun_out/sweep.log
