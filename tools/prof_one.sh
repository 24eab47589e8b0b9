#!/usr/bin/env bash
# rocprofv3 kernel trace + stats of one bench workload (W, default c2) -> gpurun_out/prof_$W
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
W=${W:-c2}
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$W" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload $W --steps ${STEPS:-10} --warmup ${WARMUP:-3} --no-cpu-baseline --host-fed-steps 0 \
    ${BENCH_ARGS:-} > "$R/gpurun_out/prof_$W.log" 2>&1) || exit $?
python3 - "$R/gpurun_out/prof_$W" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:25]:
    print("%-90s %5s %10.1f us" % (r["Name"][:90], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
