#!/usr/bin/env python3
"""Benchmark of the window-contents (ListState) path, f4 (fw_list_*: WindowedStream.apply / process and the
EvictingWindowOperator) on one MI355X, on the C2 stream shape: 1 s tumbling event-time windows, 1M uniform Long
keys, bounded out-of-orderness 200 ms, 1e8 records per event-second, a punctuated watermark after every batch of
2^24 records.  The Iterable window function's input — every fired window's elements (timestamp, value, ordinal) in
list order — is materialised in HBM and discarded (the sink); `--evictor count:N` / `time:MS` adds the evictor.

Algorithmic bytes per record (this build's figure; SURVEY §8d prices only the aggregating state): the input
24 B, the element stored once (timestamp + value 16 B) and read once when its window fires (16 B), and emitted
to the function once (24 B with its ordinal): 80 B.  `path_roofline` = 80 B x records/s / 8 TB/s over the whole
step.  The CPU baseline is the ListState restatement (oracle/list_oracle.cpp) on a bounded sample, 1 thread.
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
B_ALG = 80


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--rate", type=int, default=100_000_000)
    ap.add_argument("--window", type=int, default=1000)
    ap.add_argument("--evictor", default="none", help="none | count:N | time:MS")
    ap.add_argument("--cpu-sample", type=int, default=1 << 22)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import numpy as np
    import torch
    from flink_amd import CountEvictor, TimeEvictor, TumblingEventTimeWindows
    from flink_amd.datagen import generate_device
    from flink_amd.listwindow import GpuListWindowOperator

    ev = None
    if args.evictor.startswith("count:"):
        ev = CountEvictor.of(int(args.evictor[6:]))
    elif args.evictor.startswith("time:"):
        ev = TimeEvictor.of(int(args.evictor[5:]))
    per_window = args.rate * args.window // 1000
    op = GpuListWindowOperator(TumblingEventTimeWindows.of(args.window), evictor=ev, max_batch=args.batch,
                               expected_elements=int(per_window * 1.3))
    dev = torch.device("cuda", 0)
    batches, wms, m = [], [], -(1 << 63)
    for s in range(args.warmup + args.steps):
        k, t, v, mx = generate_device(0x5EED, s * args.batch, args.batch, args.keys, ts_base=0, rate=args.rate,
                                      jitter=200, device=0)
        batches.append((k, t, v))
        m = max(m, int(mx.item()))
        wms.append(m - 200)
    torch.cuda.synchronize()
    fired = elems = 0

    def step(s):
        nonlocal fired, elems
        k, t, v = batches[s]
        op.process_batch(k, t, v)
        op.advance_watermark(wms[s])
        nr, ne, _ = op.pending()
        fired += nr
        elems += ne
        op.clear_pending()  # discarding sink: the fired rows and elements were materialised in HBM

    for s in range(args.warmup):
        step(s)
    fired = elems = 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.warmup, args.warmup + args.steps):
        step(s)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = args.steps * args.batch
    value = n / dt
    st = op.stats()
    cpu = None
    if not args.no_cpu_baseline:
        from flink_amd.datagen import generate_host
        from oracle import oracle as orc
        hk, ht, hv = generate_host(0x5EED, 0, args.cpu_sample, args.keys, ts_base=0, rate=args.rate, jitter=200)
        ref = orc.ListWindowOracle(assigner="tumbling", size=args.window,
                                   evictor="none" if ev is None else ("count" if args.evictor.startswith("count")
                                                                      else "time"),
                                   evict_arg=0 if ev is None else int(args.evictor.split(":")[1]))
        c0 = time.perf_counter()
        bs = min(args.batch, args.cpu_sample)
        mm = -(1 << 63)
        for b in range(0, args.cpu_sample, bs):
            ref.process(hk[b:b + bs], ht[b:b + bs], hv[b:b + bs])
            mm = max(mm, int(ht[b:b + bs].max()))
            ref.watermark(mm - 200)
        ref.watermark((1 << 63) - 1)
        cdt = time.perf_counter() - c0
        cpu = {"value": round(args.cpu_sample / cdt, 1), "unit": "records/s", "cores": 1, "kind": "port",
               "sample": f"first {args.cpu_sample} records of the same stream through the ListState restatement "
                         f"(oracle/list_oracle.cpp, std::map lists), 1 thread, final watermark included"}
    line = {
        "metric": "records/sec keyed window-contents (ListState apply/process) path, 1 GPU", "value": round(value, 1),
        "unit": "records/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True, "dtype": "int64",
        "data": "synthetic (splitmix64 counter stream)",
        "config": {"workload": f"f4: tumbling {args.window} ms apply over ListState, evictor {args.evictor}, "
                               f"{args.keys} uniform Long keys, {args.rate} records per event-second, 2^24 per step",
                   "fired_rows": fired, "fired_elements": elems, "table_grows": st["table_grows"]},
        "path_roofline": {"b_alg_bytes_per_record": B_ALG, "frac": round(B_ALG * value / 8e12, 4),
                          "basis": "input 24 + element stored 16 + read at its firing 16 + emitted 24 B"},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    op.close()
    del np


if __name__ == "__main__":
    main()
