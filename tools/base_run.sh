cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/base; export TMPDIR=/tmp
timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/base/bench_c2.log 2>&1 || exit $?
for w in c4 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/base/bench_$w.log 2>&1 || exit $?
done
grep -h '^{' gpurun_out/base/*.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config']['workload'][:3], '%.4g'%d['value'], d['ms_per_step'], {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()})"
