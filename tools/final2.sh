#!/usr/bin/env bash
# Round evidence, part 2: C5 PMC passes, bench lines C3 / C5 / C5t, rocprofv3 kernel summaries of C2 (async and
# sync input).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
WORKLOADS="c5" bash tools/pmc_all.sh > gpurun_out/pmc5.log 2>&1 || { tail -5 gpurun_out/pmc5.log; exit 1; }
echo "pmc c5 ok"
for w in c5 c5t c3; do
  tr=""; [ -f gpurun_out/traffic_$w.json ] && tr="--traffic gpurun_out/traffic_$w.json"
  timeout -k 10 400 python -u bench.py --workload $w $tr > gpurun_out/bench_$w.log 2>&1
  rc=$?; echo "bench $w rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$w.log; exit $rc; }
done
W=c2 BENCH_ARGS="--no-profile" bash tools/prof_one.sh > gpurun_out/prof_c2_summary.txt || exit $?
mv gpurun_out/prof_c2 gpurun_out/prof_c2_async
W=c2 BENCH_ARGS="--sync-input" bash tools/prof_one.sh > gpurun_out/prof_c2_sync_summary.txt || exit $?
echo "prof ok"
