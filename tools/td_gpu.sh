cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tdigest.py -x -v --timeout 180 --timeout-method thread > gpurun_out/td_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/td_tests.log; exit $rc
