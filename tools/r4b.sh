cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench/lds_ubench > gpurun_out/lds.txt 2>&1; echo "lds rc=$?"
FW_LIB=$PWD/flink_amd/_lib/variants/lib_timing.so timeout -k 10 120 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --sync-input --host-fed-steps 0 > gpurun_out/timing.txt 2>&1; echo "timing rc=$?"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_heapstate.py > gpurun_out/heap.txt 2>&1; echo "heap rc=$?"
