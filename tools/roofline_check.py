#!/usr/bin/env python3
"""Recompute a bench line's roofline from the rocprofv3 kernel traces under profiles/ (VERDICT r02 item 3).

A bench line prices its dominant timing bucket (bench.py `roofline.kernel`, one of fw_kernel_name's buckets) at
its own algorithmic bytes per launch (bench.py kernel_share) over the bucket's average HIP-event duration, and every
other bucket the same way (`kernels[*].frac`); `roofline.isolated` does the same over
a pass with synchronous input.  Here the same figures come from rocprofv3 kernel traces of the same command:
the bucket's kernels (tools/traffic.py BUCKETS), their dispatches in the timed steps (between the bench's stats
reads around its timed loop), durations summed and divided by the timed steps.  Under async input a HIP-event interval also holds
the launch's dispatch latency and its wait for CUs held by the other stream's kernel, so the line's async figure
reads a few percent below the trace's.

usage: tools/roofline_check.py BENCH_JSON --async-trace CSV --sync-trace CSV --steps S --warmup W
"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from traffic import bucket_of, short, timed_window  # noqa: E402


def bucket_ms(trace, steps):
    """per bucket: the summed durations of its kernels' dispatches in the timed steps (traffic.timed_window) / steps"""
    rows = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    lo, hi = timed_window([(i, r[2]) for i, r in enumerate(rows)])
    out = defaultdict(float)
    for s, e, k in rows[lo + 1:hi]:
        b = bucket_of(k)
        if b:
            out[b] += (e - s) / 1e6 / steps
    return dict(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("bench_json")
    ap.add_argument("--async-trace", required=True)
    ap.add_argument("--sync-trace", required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    line = json.loads([l for l in open(a.bench_json) if l.startswith("{")][-1])
    rf = line["roofline"]
    alg, peak, dom = rf["alg_bytes_per_launch"], rf["peak"], rf["kernel"]
    ms_a = bucket_ms(a.async_trace, a.steps)
    ms_s = bucket_ms(a.sync_trace, a.steps)
    frac = lambda ms: alg / (ms * 1e-3) / 1e9 / peak  # noqa: E731
    res = {"workload": line["config"]["workload"], "dominant_bucket": dom, "alg_bytes_per_launch": alg,
           "line": {"frac": rf["frac"], "avg_ms": line["kernels"][dom]["avg_ms"],
                    "isolated_frac": rf.get("isolated", {}).get("frac"),
                    "isolated_avg_ms": rf.get("isolated", {}).get("avg_ms")},
           "rocprof": {"async_bucket_ms": ms_a, "sync_bucket_ms": ms_s,
                       "frac": round(frac(ms_a[dom]), 4), "isolated_frac": round(frac(ms_s[dom]), 4)}}
    res["rel_diff"] = {"frac": round(res["rocprof"]["frac"] / rf["frac"] - 1, 4) if rf["frac"] else None,
                       "isolated_frac": (round(res["rocprof"]["isolated_frac"] / rf["isolated"]["frac"] - 1, 4)
                                         if rf.get("isolated") and rf["isolated"]["frac"] else None)}
    # every bucket's own share (bench.py kernel_share), line vs trace
    per = {}
    for b, k in line["kernels"].items():
        a_b = k.get("alg_bytes_per_launch")
        if not a_b or b not in ms_a:
            continue
        fb = lambda ms: a_b / (ms * 1e-3) / 1e9 / peak  # noqa: E731
        per[b] = {"line_frac": k.get("frac"), "rocprof_frac": round(fb(ms_a[b]), 4),
                  "rocprof_isolated_frac": round(fb(ms_s[b]), 4) if b in ms_s else None,
                  "rel_diff": round(fb(ms_a[b]) / k["frac"] - 1, 4) if k.get("frac") else None}
    res["per_bucket"] = per
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
