cd "$GRAFT_REPO_ROOT"
VARIANTS="pipe deep2 deep3" STEPS=24 BENCH_ARGS="--workload c3 --sync-input --host-fed-steps 0" timeout -k 10 700 bash tools/variants.sh run || exit 1
cp gpurun_out/variants.log gpurun_out/var_c3.log
VARIANTS="pipe cur" STEPS=14 BENCH_ARGS="--workload c5 --sync-input --host-fed-steps 0" timeout -k 10 300 bash tools/variants.sh run || exit 1
cp gpurun_out/variants.log gpurun_out/var_c5.log
VARIANTS="pipe cur" STEPS=14 BENCH_ARGS="--workload c4 --sync-input --host-fed-steps 0" timeout -k 10 300 bash tools/variants.sh run || exit 1
