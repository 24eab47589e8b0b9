#!/usr/bin/env bash
# One workload (W, default c5t): the bench line, then a rocprofv3 kernel trace of the same run with sync input
# (each kernel alone), into gpurun_out/quick/$W.  Optional TESTS = pytest files run first (gpu_tests.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; export TMPDIR=/tmp
W=${W:-c5t}; S=${S:-12}; d="$R/gpurun_out/quick/$W"; mkdir -p "$d"
if [ -n "$TESTS" ]; then FILES="$TESTS" LIMIT=${LIMIT:-500} bash tools/gpu_tests.sh || exit 1; fi
ba="--workload $W --steps $S --warmup 2 --no-cpu-baseline --host-fed-steps 0 ${EXTRA:-}"
timeout -k 10 240 python3 -u bench.py $ba > "$d/bench.json" 2> "$d/bench.err" || { echo "bench rc=$?"; tail -5 "$d/bench.err"; exit 1; }
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$d/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" $ba --no-profile --sync-input > "$d/prof.log" 2>&1) || { echo "prof rc=$?"; tail -5 "$d/prof.log"; exit 1; }
python3 - "$d" <<'PY'
import json, sys
d = sys.argv[1]
b = json.loads([l for l in open(d + "/bench.json") if l.startswith("{")][-1])
print(d.split("/")[-1], "value %.4g" % b["value"], "ms %.4f" % b["ms_per_step"], {k: v["avg_ms"] for k, v in b.get("kernels_isolated", {}).items()})
PY
python3 tools/kstats.py "$d/prof/run_kernel_stats.csv" | head -24
