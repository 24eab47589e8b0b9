cd "${GRAFT_REPO_ROOT}"
STEPS=8 VARIANTS="-;-|--workload c4;-|--workload c4 --sub-partitions 32;-|--workload c5;-|--workload c5 --sub-partitions 32" bash tools/exp.sh || exit $?
cp gpurun_out/exp.log gpurun_out/exp_parts.log
VARIANTS="tim" DIAGS=256 bash tools/variants.sh run || exit $?
cp gpurun_out/variants.log gpurun_out/var_tim_c2.log
BENCH_ARGS="--workload c4" VARIANTS="tim" DIAGS=256 bash tools/variants.sh run || exit $?
cp gpurun_out/variants.log gpurun_out/var_tim_c4.log
VARIANTS="cwg" bash tools/variants.sh run
cp gpurun_out/variants.log gpurun_out/var_cwg.log
VARIANTS="r4 t16 t16r4w2" bash tools/variants.sh run
