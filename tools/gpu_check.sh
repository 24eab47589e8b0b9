#!/bin/bash
# GPU round trip used during development: the GPU test suite, then (only when pytest ended normally, i.e. passed or
# reported failures) one C2 bench line.  Everything goes to gpurun_out/.
# usage: tools/gpu_check.sh TAG [pytest -k expression]
tag=${1:-chk}
kexpr=${2:-}
mkdir -p gpurun_out
if [ -n "$kexpr" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail=30 -k "$kexpr" \
    > gpurun_out/gt_$tag.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail=30 \
    > gpurun_out/gt_$tag.log 2>&1
fi
rc=$?
tail -5 gpurun_out/gt_$tag.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
brc=$?
python3 -c "
import json,sys
d=json.load(open('gpurun_out/bench_$tag.json'))
print('value %.3e ms %.4f' % (d['value'], d['ms_per_step']))
for k,v in d.get('kernels_isolated',{}).items(): print('  iso', k, v['avg_ms'])
for k,v in d.get('kernels',{}).items(): print('  ovl', k, v['avg_ms'])
" || true
exit $brc
