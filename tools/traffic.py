#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) into per-kernel, per-launch HBM bytes.

Reads gpurun_out/pmc/p*/run_counter_collection.csv, averages each counter over the dispatches of
each kernel, and derives HBM bytes as MI355X_MICROARCH.md §HBM prescribes:
  read  bytes = FETCH_SIZE (KiB) * 1024 * 2   (gfx950 tallies a 128-B request of a wide coalesced
                                               read as 64 B: the counter reads half the bytes)
  write bytes = WRITE_SIZE (KiB) * 1024       (exact for 16-B-per-lane streaming stores)
The correction factor for reads is checked against k_classify_hist, whose reads are known exactly
(16 B per record: key + ts), and the calibration is printed beside the result.

usage: tools/traffic.py [pmc_dir] [--records N] [--out profiles/traffic_rNN.json]
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


def load(pmc_dir, last=0):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch values]
    for f in sorted(glob.glob(os.path.join(pmc_dir, "p*", "run_counter_collection.csv"))):
        per = defaultdict(float)
        names = {}
        with open(f) as fh:
            for r in csv.DictReader(fh):
                key = (r["Dispatch_Id"], r["Counter_Name"])
                per[key] += float(r["Counter_Value"])  # sum over dimensions (XCDs / instances)
                names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
        for (d, cn), v in per.items():
            vals[names[d]][cn].append(v)
    # `last`: average only each kernel's last dispatches (the bench's timed steps follow its warmup)
    cut = (lambda v: v[-last:]) if last else (lambda v: v)
    return {k: {c: sum(cut(v)) / len(cut(v)) for c, v in cs.items()} | {"_dispatches": max(len(cut(v)) for v in cs.values())}
            | {"_total_dispatches": max(len(v) for v in cs.values())} | {"_sum_" + c: sum(v) for c, v in cs.items()}
            for k, cs in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir", nargs="?", default="gpurun_out/pmc")
    ap.add_argument("--records", type=int, default=1 << 24, help="records per push (bench --batch)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--workload", default="c2", help="bench --workload the passes ran (recorded for bench.py)")
    ap.add_argument("--last", type=int, default=0, help="average only each kernel's last N dispatches")
    a = ap.parse_args()
    k = load(a.pmc_dir, a.last)
    res = {}
    for name, c in sorted(k.items()):
        rd = c.get("FETCH_SIZE")
        wr = c.get("WRITE_SIZE")
        res[name] = {
            "dispatches": c["_dispatches"],
            "fetch_size_kib": rd,
            "write_size_kib": wr,
            "read_bytes": None if rd is None else rd * 1024 * 2,
            "write_bytes": None if wr is None else wr * 1024,
        }
        for extra in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"):
            if extra in c:
                res[name][extra] = c[extra]
        r = res[name]
        if r["read_bytes"] is not None and r["write_bytes"] is not None:
            r["hbm_bytes"] = r["read_bytes"] + r["write_bytes"]
    # bench.py's timing buckets: the HLL register update is timed with k_aggregate, the pane fire is k_fire,
    # the t-digest compression (k_td_* and its rocPRIM radix sorts) is k_tdigest
    per_launch = {n: r.get("hbm_bytes") for n, r in res.items()}
    td_parts = tuple(n for n in res if n.startswith("k_td_") or n.startswith("rocprim"))
    if "k_td_keys" in k:  # several dispatches per push (the radix sorts' passes): bytes per push over all pushes
        pushes = k["k_td_keys"]["_total_dispatches"]
        per_launch["k_tdigest"] = sum(k[x].get("_sum_FETCH_SIZE", 0) * 2048 + k[x].get("_sum_WRITE_SIZE", 0) * 1024
                                      for x in td_parts) / pushes
    for bucket, parts in (("k_aggregate", ("k_aggregate", "k_hll_update")), ("k_fire", ("k_fire", "k_fire_panes"))):
        vals = [per_launch[x] for x in parts if per_launch.get(x) is not None]
        if vals:
            per_launch[bucket] = sum(vals)
    cal = None
    if "k_classify_hist" in res and res["k_classify_hist"]["read_bytes"]:
        cal = res["k_classify_hist"]["read_bytes"] / (16.0 * a.records)
    out = {"note": "per-launch averages; read = FETCH_SIZE*1024*2 (gfx950 half-count correction), "
                   "write = WRITE_SIZE*1024; Infinity-Cache hits are counted by these counters",
           "records_per_launch": a.records,
           "read_calibration_k_classify_hist": cal,
           "workload": a.workload,
           "per_launch_bytes": per_launch,
           "kernels": res}
    for n, r in res.items():
        hb = r.get("hbm_bytes")
        print(f"{n:28s} n={r['dispatches']:3d} read={r['read_bytes'] or 0:14.0f} write={r['write_bytes'] or 0:14.0f}"
              f" per_rec={(hb or 0) / a.records:7.2f} B")
    print("read calibration (k_classify_hist measured / 16 B per record):", cal)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
