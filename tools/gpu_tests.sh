#!/usr/bin/env bash
# GPU tests under one time limit; K = pytest -k expression (default: all), FILES = test paths (default tests)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 ${LIMIT:-600} python -u -m pytest ${FILES:-tests} -m gpu -x -q --timeout 180 --timeout-method thread \
    ${K:+-k "$K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/gpu_tests.log | tail -15; exit $rc
