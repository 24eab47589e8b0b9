#!/usr/bin/env bash
# Prices kernel stages with FW_DIAG ablation bits (results are wrong under them): one bench line per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/diag.log
for d in ${DIAGS:-0 1 2 16}; do
  echo "== FW_DIAG=$d" >> gpurun_out/diag.log
  FW_DIAG=$d timeout -k 10 120 python3 bench.py ${ARGS:---workload c2} --steps 10 --warmup 3 --no-cpu-baseline --host-fed-steps 0 \
      > gpurun_out/diag_one.log 2>&1 || { echo "rc=$? diag $d"; tail -5 gpurun_out/diag_one.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/diag_one.log'):
    if l.startswith('{'):
        d=json.loads(l); print('ms', d['ms_per_step'], ' '.join(f\"{k}={v['avg_ms']:.4f}\" for k,v in d['kernels'].items()))" >> gpurun_out/diag.log
done
cat gpurun_out/diag.log
