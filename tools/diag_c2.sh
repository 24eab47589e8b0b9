# C2 stage pricing with FW_DIAG ablation bits (results are wrong under any bit; timing only)
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/diag; export TMPDIR=/tmp
for d in 0 1 2 4 8 16 128; do
  FW_DIAG=$d timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/diag/d$d.log 2>&1 || exit $?
  echo -n "diag $d: "; grep '^{' gpurun_out/diag/d$d.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('%.4g'%d['value'], d['ms_per_step'], {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()})"
done
