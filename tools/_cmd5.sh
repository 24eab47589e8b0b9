tools/gpu_check.sh dt2 || exit $?
VARIANTS="t512r4 t512r2" STEPS=20 BENCH_ARGS="--sync-input --host-fed-steps 0" bash tools/variants.sh run > gpurun_out/var_dt2a.txt 2>&1 || exit $?
VARIANTS="base" DIAGS="0 2048" STEPS=20 BENCH_ARGS="--sync-input --host-fed-steps 0" bash tools/variants.sh run > gpurun_out/var_dt2b.txt 2>&1 || exit $?
