tools/gpu_check.sh dt3 "tumbling or combine or restore or rescal or c2 or full or word or snapshot or exchange or smoke or size" || exit $?
VARIANTS="tim" STEPS=10 BENCH_ARGS="--sync-input --host-fed-steps 0" bash tools/variants.sh run > gpurun_out/var_dt3.txt 2>&1
grep "dt timing" gpurun_out/variants.log | tail -5
