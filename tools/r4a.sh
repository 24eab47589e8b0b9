cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
VARIANTS="base rpt4 pf pfr4 s1344 s1344r4 s896t512" STEPS=20 timeout -k 10 400 bash tools/variants.sh run > gpurun_out/var.txt 2>&1; echo "variants rc=$?"
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sharded.py "tests/test_gpu_exchange.py::test_gpu_exchange_world2_operator_kinds" > gpurun_out/shard.txt 2>&1; echo "tests rc=$?"
