#!/usr/bin/env bash
# One rocprofv3 PMC pass of SQ counters (instruction mix, LDS waits and bank conflicts) over a short bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; export TMPDIR=/tmp; mkdir -p gpurun_out
W=${W:-c4}
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS \
    SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$R/gpurun_out/pmc_sq_$W" -o run --output-format csv \
    -- python3 "$R/bench.py" --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-profile --host-fed-steps 0 \
    > "$R/gpurun_out/pmc_sq_$W.log" 2>&1) || { echo "pmc rc=$?"; tail -5 "$R/gpurun_out/pmc_sq_$W.log"; exit 1; }
python3 - "$R/gpurun_out/pmc_sq_$W" <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0]
v = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
    v[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
for k, c in sorted(v.items(), key=lambda x: -x[1].get("SQ_BUSY_CYCLES", 0))[:8]:
    d = len(n[k])
    print(k, d, {x: "%.3g" % (y / d) for x, y in sorted(c.items())})
PY
