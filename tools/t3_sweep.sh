mkdir -p gpurun_out
for t in default 1024 2048 4096; do
  if [ $t = default ]; then unset FW_LIB; else export FW_LIB=$PWD/flink_amd/_lib/libflinkwin_t$t.so; fi
  timeout -k 10 200 python3 -u bench.py --workload c5t --steps 12 --warmup 2 --no-cpu-baseline --host-fed-steps 0 --sync-input > gpurun_out/t3_$t.json 2> gpurun_out/t3_$t.err || { echo "rc $t"; tail -3 gpurun_out/t3_$t.err; exit 1; }
  python3 -c "
import json,sys;b=json.loads([l for l in open('gpurun_out/t3_$t.json') if l.startswith('{')][-1]);print('$t', b['ms_per_step'], '%.4g'%b['value'], b['kernels']['k_tdigest']['avg_ms'])"
done
export FW_LIB=$PWD/flink_amd/_lib/libflinkwin_t2048.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_tdigest.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/t3_tests.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/t3_tests.log
