#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc_all.sh, tools/evidence.sh) into per-kernel, per-launch HBM bytes.

Reads gpurun_out/pmc/p*/run_counter_collection.csv, averages each counter over the dispatches of
each kernel, and derives HBM bytes as MI355X_MICROARCH.md §HBM prescribes:
  read  bytes = FETCH_SIZE (KiB) * 1024 * 2   (gfx950 tallies a 128-B request of a wide coalesced
                                               read as 64 B: the counter reads half the bytes)
  write bytes = WRITE_SIZE (KiB) * 1024       (exact for 16-B-per-lane streaming stores)
The correction factor for reads is checked against k_classify_hist, whose reads are known exactly
(16 B per record: key + ts), and the calibration is printed beside the result.

Bytes are per bench step (one push + one watermark), summed per bench timing bucket (BUCKETS), over the timed
steps only (the dispatches between the bench's stats reads around its timed loop), so a run of steps >= one firing
period averages the firings in.

usage: tools/traffic.py [pmc_dir] --steps S --warmup W [--records N] [--out profiles/traffic_rNN_W.json]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    return n.split("(")[0].replace("void ", "").split("<")[0].strip()  # k_aggregate<2, false> -> k_aggregate


# bench.py's timing buckets (fw_kernel_name) and the kernels each one launches
BUCKETS = {
    "k_classify_hist": ("k_classify_hist", "k_taint"),
    "k_scan": ("k_scan_blocks", "k_scan_top", "k_scan_add"),
    "k_scatter": ("k_scatter_rsv", "k_scatter_staged", "k_scatter", "k_scatter_ordered", "k_stage"),
    "k_aggregate": ("k_aggregate", "k_dt_aggregate", "k_hll_update", "k_chunk_plan", "k_pmerge"),
    "k_slow": ("k_slow",),
    "k_fire": ("k_fire", "k_fire_panes", "k_dt_fire"),
    "k_tdigest": ("k_td_", "rocprim"),
}


def bucket_of(kernel):
    for b, members in BUCKETS.items():
        for m in members:
            if kernel == m or (m.endswith("_") and kernel.startswith(m)) or (m == "rocprim" and kernel.startswith(m)):
                return b
    return None


def timed_window(ordered):
    """(lo, hi): bench.py reads the operator's stats (fw_get_stats -> one k_table_stats dispatch) right before and
    right after its timed steps, so the timed dispatches are the ones strictly between the last two k_table_stats.
    ordered: (order key, kernel short name) in dispatch order."""
    st = [key for key, n in ordered if n == "k_table_stats"]
    if len(st) < 2:
        raise SystemExit("no k_table_stats pair in the trace: not a bench.py run?")
    return st[-2], st[-1]


def load(pmc_dir):
    """kernel -> counter -> summed value over the timed steps' dispatches (timed_window), and their count."""
    vals = defaultdict(lambda: defaultdict(float))
    for f in sorted(glob.glob(os.path.join(pmc_dir, "p*", "run_counter_collection.csv"))):
        per = defaultdict(float)
        names = {}
        with open(f) as fh:
            for r in csv.DictReader(fh):
                key = (int(r["Dispatch_Id"]), r["Counter_Name"])
                per[key] += float(r["Counter_Value"])  # sum over dimensions (XCDs / instances)
                names[int(r["Dispatch_Id"])] = short(r["Kernel_Name"])
        lo, hi = timed_window(sorted(names.items()))
        seen = defaultdict(set)
        for (d, cn), v in per.items():
            if lo < d < hi:
                vals[names[d]][cn] += v
                seen[names[d]].add(d)
        for k, ds in seen.items():
            vals[k]["_n"] = len(ds)
    return {k: dict(v) for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir", nargs="?", default="gpurun_out/pmc")
    ap.add_argument("--records", type=int, default=1 << 24, help="records per push (bench --batch)")
    ap.add_argument("--steps", type=int, required=True, help="the bench's timed steps (bench --steps)")
    ap.add_argument("--warmup", type=int, required=True, help="the bench's warmup steps (bench --warmup)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--workload", default="c2", help="bench --workload the passes ran (recorded for bench.py)")
    a = ap.parse_args()
    k = load(a.pmc_dir)
    res, per_step = {}, defaultdict(float)
    for name, c in sorted(k.items()):
        rd, wr = c.get("FETCH_SIZE"), c.get("WRITE_SIZE")
        r = {"dispatches": int(c["_n"]), "dispatches_per_step": round(c["_n"] / a.steps, 3),
             "read_bytes_per_step": None if rd is None else rd * 1024 * 2 / a.steps,
             "write_bytes_per_step": None if wr is None else wr * 1024 / a.steps}
        if rd is not None and wr is not None:
            r["hbm_bytes_per_step"] = r["read_bytes_per_step"] + r["write_bytes_per_step"]
            b = bucket_of(name)
            r["bucket"] = b
            if b:
                per_step[b] += r["hbm_bytes_per_step"]
        res[name] = r
    # the path's kernels only (not the bench's generator, the runtime's copies or a stats query)
    total = sum(r.get("hbm_bytes_per_step", 0) for r in res.values() if r.get("bucket"))
    other = sum(r.get("hbm_bytes_per_step", 0) for r in res.values() if not r.get("bucket"))
    cal = None
    if "k_classify_hist" in res and res["k_classify_hist"]["read_bytes_per_step"] and "k_scatter_rsv" not in res:
        cal = res["k_classify_hist"]["read_bytes_per_step"] / (16.0 * a.records)
    out = {"note": "HBM bytes per bench step (= per launch of each timing bucket: one push and one watermark per "
                   "step), over the last `steps` steps' dispatches of each kernel; read = FETCH_SIZE*1024*2 (gfx950 "
                   "half-count correction), write = WRITE_SIZE*1024; Infinity-Cache hits are counted by these "
                   "counters",
           "records_per_launch": a.records, "steps": a.steps, "warmup": a.warmup,
           "read_calibration_k_classify_hist": cal,
           "workload": a.workload,
           "bytes_per_record_all_kernels": round(total / a.records, 2),
           "bytes_per_record_outside_the_path": round(other / a.records, 2),
           "per_launch_bytes": dict(per_step),
           "kernels": res}
    for n, r in res.items():
        hb = r.get("hbm_bytes_per_step") or 0
        print(f"{n:28s} x{r['dispatches_per_step']:5.2f}/step read={r['read_bytes_per_step'] or 0:14.0f} "
              f"write={r['write_bytes_per_step'] or 0:14.0f} per_rec={hb / a.records:7.2f} B")
    print(f"path kernels: {total / a.records:.2f} B per record over {a.steps} steps "
          f"(outside the path: {other / a.records:.2f})")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
