#!/usr/bin/env bash
# One GPU-box session: parity tests, then (only if they did not crash or hang) a short bench and a
# rocprofv3 kernel trace.  Every GPU step runs under its own time limit; a crash, abort or time limit
# (124/134/137/139) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }

timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
if fatal $rc; then exit $rc; fi

if [ "${SKIP_BENCH:-0}" = "0" ]; then
  timeout -k 10 240 python -u bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-3} ${BENCH_ARGS:-} \
      > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
  if fatal $rc; then exit $rc; fi
fi
if [ "${PROFILE:-0}" = "1" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" \
      -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline \
      --no-profile > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
fi
exit 0
