cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/c3p; export TMPDIR=/tmp
for sp in 0 16 8; do
timeout -k 10 200 python -u bench.py --workload c3 --steps 24 --warmup 4 --no-cpu-baseline --host-fed-steps 0 --sub-partitions $sp > gpurun_out/c3p/sp$sp.json 2> gpurun_out/c3p/sp$sp.err || exit 1
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/c3p/sp$sp.json') if l.startswith('{')][-1]); print($sp, '%.4g'%d['value'], d['ms_per_step'], {k:round(v['avg_ms'],4) for k,v in d['kernels'].items()})"
done
