#!/usr/bin/env python3
"""Benchmark of the keyed event-time window aggregation path (BASELINE.json metric:
"records/sec keyed windowed aggregation at 1/2/4/8 GPUs; % of HBM roofline").

Workload (BASELINE.json configs[1]): 1 s tumbling event-time windows, 1M uniform
Long keys, built-in count/sum/min/max AggregateFunction, bounded out-of-orderness watermarks (200 ms,
punctuated after every batch), synthetic counter-based stream at 1e8 records per event-second.
One step = one micro-batch of `--batch` records per GPU pushed through the operator plus the
watermark that follows it (every window whose end passed fires).  Inputs are generated into HBM
before the timed region.  With N > 1 (torchrun, one process per GPU over RCCL) each rank owns the
KeyGroupRange computeKeyGroupRangeForOperatorIndex(128, N, rank), generates `--batch` records of the
global stream per step and the keyBy exchange (route + RCCL all_to_all) and the watermark min
(all_reduce) run inside the timed region: weak scaling.

--workload c3 runs SURVEY §8d C3 (SlidingEventTimeWindows 60 s / 1 s, 60 windows per record, 2M uniform
keys per GPU = 16M at 8 GPUs, 1e8 records per event-second per GPU, bound 200 ms); --workload c4 runs C4
(EventTimeSessionWindows gap 30 s, 1M Zipf(1.1) keys, 1e5 records per event-second, bound 1 s).  The
default line is C2.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md §Chip-level parameters

# SURVEY.md §8d workloads.  c2 is BASELINE.json configs[1] (the default, the headline line); c4 is the
# session-window config, benchmarked on request (--workload c4).
PRESETS = {
    "c2": dict(rate=100_000_000, bound=200, jitter=200, zipf=None, keys=1_000_000, cpu_sample=1 << 24,
               workload="C2 tumbling 1s event-time window, count/sum/min/max, 1M uniform Long keys, "
                        "bounded out-of-orderness 200 ms"),
    "c3": dict(rate=100_000_000, bound=200, jitter=200, zipf=None, keys=2_000_000, cpu_sample=1 << 19,
               workload="C3 sliding 60s/1s event-time windows (60x fan-out), count/sum/min/max, 2M uniform Long keys "
                        "per GPU (16M at 8 GPUs), bounded out-of-orderness 200 ms"),
    "c5": dict(rate=100_000_000, bound=200, jitter=200, zipf=1.1, keys=1_000_000, cpu_sample=1 << 20,
               workload="C5 tumbling 1s event-time window, HyperLogLog (p=14) distinct count per key and window, "
                        "1M Zipf(1.1) Long keys, bounded out-of-orderness 200 ms"),
    "c4": dict(rate=100_000, bound=1000, jitter=1000, zipf=1.1, keys=1_000_000, cpu_sample=1 << 22,
               workload="C4 EventTimeSessionWindows gap 30 s, count/sum/min/max, 1M Zipf(1.1) Long keys, "
                        "bounded out-of-orderness 1 s"),
}


def kernel_bytes(name, n, merged, fired=0, hll_p=0, panes_per_window=0):
    """Algorithmic bytes of one launch.  `fired` = rows fired per launch."""
    if name == "k_fire":
        if hll_p:  # per fired (key, window): the 64-B entry, read + zero its 2^p register block, the 56-B row
            return fired * (64 + 2 * (1 << hll_p) + 56)
        if panes_per_window:  # per fired window: its size/slide 64-B panes read, one 56-B row written
            return fired * (64 * panes_per_window + 56)
        return fired * (64 + 56)  # per fired window: its entry read, its row written
    if name == "k_classify_hist":
        return 16 * n                      # key + ts
    if name == "k_scatter":
        return 24 * n + 32 * n             # read key/ts/val, write the 32-B partitioned record
    if name == "k_aggregate":
        return 32 * n + 128 * merged       # read the partitioned records, RMW one 64-B entry per delta
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--workload", choices=sorted(PRESETS), default="c2")
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--keys", type=int, default=None)
    ap.add_argument("--rate", type=int, default=None, help="records per event-second (whole job)")
    ap.add_argument("--bound", type=int, default=None, help="out-of-orderness bound (ms)")
    ap.add_argument("--jitter", type=int, default=None)
    ap.add_argument("--window", type=int, default=1000, help="tumbling window (ms, c2)")
    ap.add_argument("--gap", type=int, default=30_000, help="session gap (ms, c4)")
    ap.add_argument("--size", type=int, default=60_000, help="sliding window size (ms, c3)")
    ap.add_argument("--slide", type=int, default=1000, help="sliding window slide (ms, c3)")
    ap.add_argument("--hll-p", type=int, default=14, help="HyperLogLog precision (c5)")
    ap.add_argument("--no-steady", dest="steady", action="store_false",
                    help="c3: do not extend the warmup to one window size of event time")
    ap.add_argument("--cpu-sample", type=int, default=None)
    ap.add_argument("--zipf", type=float, default=None, help="Zipf exponent of the keys (0 = uniform)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-kernel HIP-event timing")
    ap.add_argument("--traffic", default=None,
                    help="PMC traffic summary (tools/traffic.py); default profiles/traffic_r01[_<workload>].json")
    ap.add_argument("--sub-partitions", type=int, default=0, help="state partitions per key group (0 = auto)")
    args = ap.parse_args()
    preset = PRESETS[args.workload]
    if args.traffic is None:
        args.traffic = os.path.join(ROOT, "profiles", "traffic_r01.json" if args.workload == "c2"
                                    else f"traffic_r01_{args.workload}.json")
    for name in ("keys", "rate", "bound", "jitter", "cpu_sample"):
        if getattr(args, name) is None:
            setattr(args, name, preset[name])
    if args.zipf is None:
        args.zipf = preset["zipf"]
    args.zipf = args.zipf or None
    sessions = args.workload == "c4"
    sliding = args.workload == "c3"
    hll = args.workload == "c5"

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from flink_amd import (CountSumMinMax, EventTimeSessionWindows, HyperLogLog, SlidingEventTimeWindows,
                           TumblingEventTimeWindows)
    from flink_amd import _native as N
    from flink_amd.datagen import generate_device, zipf_cdf
    from flink_amd.exchange import KeyGroupExchange
    from flink_amd.operator import GpuWindowOperator

    max_par = 128
    exch = KeyGroupExchange(max_par, world, rank)
    if sliding:
        # weak scaling: the key space and the event rate grow with the GPU count (16M keys at 8 GPUs)
        args.keys *= world
        args.rate *= world
    if sessions:
        assigner = EventTimeSessionWindows.with_gap(args.gap)
    elif sliding:
        assigner = SlidingEventTimeWindows.of(args.size, args.slide)
    else:
        assigner = TumblingEventTimeWindows.of(args.window)
    live_windows = (args.size // args.slide + 1) if sliding else 2
    cdf = torch.from_numpy(zipf_cdf(args.keys, args.zipf)).to(dev) if args.zipf else None
    op = GpuWindowOperator(assigner, HyperLogLog(args.hll_p) if hll else CountSumMinMax(),
                           key_group_range=exch.key_group_range,
                           device=local_rank, max_parallelism=max_par,
                           expected_entries=live_windows * args.keys // world,
                           max_batch=args.batch if world == 1 else 2 * args.batch,
                           sub_partitions=args.sub_partitions)
    if sliding and args.steady:
        # steady state: the warmup covers one window size of event time, so the timed steps see the
        # full pane population (size/slide + 1 panes per key) and windows merging size/slide panes
        event_ms_per_step = args.batch * world * 1000.0 / args.rate
        args.warmup = max(args.warmup, int(args.size / event_ms_per_step) + 2)
    steps_total = args.warmup + args.steps
    seed = 0x5EED

    def generate(s):
        first = (s * world + rank) * args.batch  # global record index of this rank's slice of step s
        return generate_device(seed, first, args.batch, args.keys, ts_base=0, rate=args.rate,
                               jitter=args.jitter, cdf_dev=cdf, device=local_rank)

    # warmup batches are generated step by step (untimed); the timed ones are staged in HBM up front.
    # punctuated watermark of this rank's source after each batch: max ts so far - bound
    batches, local_wm = {}, {}
    m = -(1 << 63)
    for s in range(args.warmup, steps_total):
        k, t, v, mx = generate(s)
        batches[s] = (k, t, v)
        local_wm[s] = int(mx.item())  # this batch's max; made cumulative once the warmup's is known
    torch.cuda.synchronize()

    def step(s):
        nonlocal m
        if s < args.warmup:
            k, t, v, mx = generate(s)
            m = max(m, int(mx.item()))
            wm = m - args.bound
        else:
            k, t, v = batches[s]
            wm = local_wm[s]
        if world > 1:
            k, t, v = exch.exchange(k, t, v)
            wm = exch.combine_watermark(wm, device=dev)
        op.process_batch(k, t, v)          # queued; settles the previous step's sequence
        op.advance_watermark(wm, wait=False)  # queued behind the push
        op.clear_pending()  # discarding sink: fired rows were materialised in HBM

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    for s in range(args.warmup):
        step(s)
    for j in range(args.warmup, steps_total):  # fold the warmup's running max into the staged batch maxima
        m = max(m, local_wm[j])
        local_wm[j] = m - args.bound
    L = N.lib()
    if not args.no_profile:
        L.fw_profile(op._h, 1)
        L.fw_profile_read(op._h, None, None, 1)
    st0 = op.stats()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.warmup, steps_total):
        step(s)
    op.synchronize()  # settles the last step (resumes it if it suspended)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    st1 = op.stats()

    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    records = args.batch * world * args.steps
    value = records / elapsed
    fired = st1["fired_rows_total"] - st0["fired_rows_total"]

    roofline = None
    kernels = {}
    if not args.no_profile:
        import ctypes
        ms = (ctypes.c_double * N.FW_NUM_KERNELS)()
        nl = (ctypes.c_int64 * N.FW_NUM_KERNELS)()
        L.fw_profile_read(op._h, ms, nl, 1)
        merged = st1["state_merges"] - st0["state_merges"]
        for i in range(N.FW_NUM_KERNELS):
            name = L.fw_kernel_name(i).decode()
            if nl[i]:
                kernels[name] = {"launches": int(nl[i]), "avg_ms": ms[i] / nl[i], "total_ms": ms[i]}
        per_launch_records = records / world / args.steps
        # the dominant kernel among those with an algorithmic byte count (all but the tiny scan/slow ones)
        b = None
        for dom in sorted(kernels, key=lambda k: -kernels[k]["total_ms"]):
            b = kernel_bytes(dom, per_launch_records, merged / args.steps,
                             fired=fired / kernels[dom]["launches"], hll_p=args.hll_p if hll else 0,
                             panes_per_window=args.size // args.slide if sliding else 0)
            if b is not None:
                break
        traffic = None
        if os.path.exists(args.traffic):
            with open(args.traffic) as f:
                tr = json.load(f)
            # PMC bytes per launch were measured on one workload (tools/traffic.py); other workloads: null
            if tr.get("workload", "c2") == args.workload:
                traffic = tr.get("per_launch_bytes", {}).get(dom)
        if b is not None:
            achieved = b / (kernels[dom]["avg_ms"] * 1e-3) / 1e9
            roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                        "traffic": traffic, "alg_bytes_per_launch": int(b)}
    # whole-path roofline with SURVEY §8d's B_alg: C2 24 + 104 F/N, C4 24 + 112 F/N bytes per record;
    # C3 (pane model) 24 + 96 + (60*48 + 56) F/N, plus the exchange 2*24*(G-1)/G
    fpr = fired / max(1, records / world)
    if sliding:
        b_alg = 24 + 96 + (args.size // args.slide * 48 + 56) * fpr + 48 * (world - 1) / world
    elif hll:  # C5-HLL: 24 + B_x + 2 + (2^p + 56) F/N
        b_alg = 24 + 48 * (world - 1) / world + 2 + ((1 << args.hll_p) + 56) * fpr
    else:
        b_alg = 24 + (112 if sessions else 104) * fpr
    path_frac = value * b_alg / (world * HBM_PEAK_GBS * 1e9)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)

    if rank == 0:
        line = {
            "metric": "records/sec keyed windowed aggregation at 1/2/4/8 GPUs; % of HBM roofline",
            "value": round(value, 1), "unit": "records/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int64", "data": "synthetic (splitmix64 counter stream)",
            "config": {"workload": preset["workload"],
                       "records_per_step_per_gpu": args.batch, "keys": args.keys,
                       **({"gap_ms": args.gap, "zipf_s": args.zipf} if sessions else
                          {"size_ms": args.size, "slide_ms": args.slide} if sliding else
                          {"window_ms": args.window, "hll_precision": args.hll_p, "zipf_s": args.zipf} if hll else
                          {"window_ms": args.window}),
                       "records_per_event_second": args.rate, "watermark_bound_ms": args.bound,
                       "max_parallelism": 128, "parallelism": f"keygroup{world}"},
            "roofline": roofline,
            "path_roofline": {"b_alg_bytes_per_record": round(b_alg, 3), "frac": round(path_frac, 4),
                              "fired_rows": int(fired)},
            "cpu_baseline": cpu,
            "kernels": kernels,
            "state": {"table_slots": int(st1["table_capacity"]), "table_grows_in_timed_region":
                      int(st1["table_grows"] - st0["table_grows"]), "live_entries": int(st1["keyed_state_entries"])},
        }
        print(json.dumps(line), flush=True)
    op.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def cpu_baseline(args):
    """CPU restatement of WindowOperator (oracle/, kind "port"): p threads = p subtasks over their
    KeyGroupRanges, the same generator and punctuated watermarks, on a bounded sample."""
    import numpy as np
    from flink_amd.datagen import generate_host
    from oracle import oracle as orc
    n = args.cpu_sample
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    k, t, v = generate_host(0x5EED, 0, n, args.keys, ts_base=0, rate=args.rate, jitter=args.jitter, zipf_s=args.zipf)
    batch = min(args.batch, n)
    wms, m = [], -(1 << 63)
    for b in range(0, n, batch):
        m = max(m, int(t[b:b + batch].max()))
        wms.append(m - args.bound)
    t0 = time.perf_counter()
    if args.workload == "c4":
        cfg = dict(assigner="session", gap=args.gap)
    elif args.workload == "c3":
        cfg = dict(assigner="sliding", size=args.size, slide=args.slide)
    elif args.workload == "c5":
        cfg = dict(assigner="tumbling", size=args.window, hll_p=args.hll_p)
    else:
        cfg = dict(assigner="tumbling", size=args.window)
    orc.run_parallel(cfg, k, t, v, batch, np.array(wms), 128, threads)
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 1), "unit": "records/s", "cores": threads, "kind": "port",
            "sample": f"first {n} records of the same {args.workload.upper()} stream, {threads} subtasks (threads), watermark every "
                      f"{batch} records; CPU restatement of WindowOperator semantics (oracle/), not the Java "
                      f"reference (no JDK on the box)"}


if __name__ == "__main__":
    main()
