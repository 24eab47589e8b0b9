cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
VARIANTS="r4w4:x r4w6:x r1:x" bash tools/variants.sh run
