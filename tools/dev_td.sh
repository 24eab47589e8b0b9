cd "$GRAFT_REPO_ROOT"; R=$PWD; export TMPDIR=/tmp; mkdir -p gpurun_out/td
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_tdigest.py > gpurun_out/td/tests.log 2>&1 || { echo tests rc=$?; tail -30 gpurun_out/td/tests.log; exit 1; }
tail -3 gpurun_out/td/tests.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/td/prof" -o run --output-format csv -- python3 "$R/bench.py" --workload c5t --steps 12 --warmup 2 --no-cpu-baseline --host-fed-steps 0 --no-profile --sync-input > "$R/gpurun_out/td/prof.log" 2>&1) || { echo prof rc=$?; tail -20 gpurun_out/td/prof.log; exit 1; }
grep '^{' gpurun_out/td/prof.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
VARIANTS="base t3k sr8 sr32" STEPS=12 BENCH_ARGS="--workload c5t --sync-input --host-fed-steps 0" timeout -k 10 600 bash tools/variants.sh run
cp gpurun_out/variants.log gpurun_out/td/variants_c5t.log
VARIANTS="base hu8 hu8c8" STEPS=12 BENCH_ARGS="--workload c5 --sync-input --host-fed-steps 0" timeout -k 10 400 bash tools/variants.sh run
