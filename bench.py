#!/usr/bin/env python3
"""Benchmark of the keyed event-time window aggregation path (BASELINE.json metric:
"records/sec keyed windowed aggregation at 1/2/4/8 GPUs; % of HBM roofline").

Workload (BASELINE.json configs[1]): 1 s tumbling event-time windows, 1M uniform
Long keys, built-in count/sum/min/max AggregateFunction, bounded out-of-orderness watermarks (200 ms,
punctuated after every batch), synthetic counter-based stream at 1e8 records per event-second.
One step = one micro-batch of `--batch` records per GPU pushed through the operator plus the
watermark that follows it (every window whose end passed fires; the sink discards the fired rows,
which stay materialised in HBM).  Inputs are generated into HBM before the timed region.  With N > 1
(torchrun, one process per GPU over RCCL) each rank owns the KeyGroupRange
computeKeyGroupRangeForOperatorIndex(128, N, rank), generates `--batch` records of the global stream
per step and the keyBy exchange (route + RCCL all_to_all) and the watermark min (all_reduce) run
inside the timed region: weak scaling.

Other SURVEY §8d configs (--workload):
  c1   WindowWordCount (configs[0]): String keys from WordCountData's 287 tokens (170 words), hashed by the
       host, window(Tumbling 5 s).sum(1), 10M tokens per step; CPU baseline = the oracle at p = 1 for both
       C1 pipelines (countWindow(10, 5).sum(1) and the tumbling sum)
  c3   SlidingEventTimeWindows 60 s / 1 s (60 windows per record), 2M uniform keys per GPU
  c4   EventTimeSessionWindows gap 30 s, 1M Zipf(1.1) keys, 1e5 records per event-second
  c5   HyperLogLog (p = 14) per key and 1 s tumbling window, 1M Zipf(1.1) keys
  c5t  t-digest (delta = 100) quantiles per key and 1 s tumbling window, 1M Zipf(1.1) keys

Roofline: `roofline` prices the dominant kernel at its own share of the algorithmic bytes
(`kernel_share`: the partitioning, the aggregate, the t-digest compression and the firing each charged what they
must move of B_alg) x the records one launch processes, over that kernel's average HIP-event duration (the kernel
launches once per step); `impl_bytes` is what the kernel itself must move as built, `traffic` the PMC-measured
HBM bytes per launch (profiles/traffic_*.json).  `path_roofline` is B_alg x records/s over the whole step.
A `host_fed` leg (rank 0, N = 1) pushes further batches from pinned host memory through fw_push_batch and
drains the fired rows to the host: the PCIe-inclusive rate of the JNI drop-in, reported beside `value`.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md §Chip-level parameters
XGMI_LINK_GBS = 153.0  # one xGMI link per peer pair, per direction

# SURVEY.md §8d workloads.  c2 is BASELINE.json configs[1] (the default, the headline line).
PRESETS = {
    "c1": dict(rate=2_000_000, bound=0, jitter=0, zipf=None, keys=287, cpu_sample=10_000_000, batch=10_000_000,
               workload="C1 WindowWordCount: keyBy(word).window(Tumbling 5 s).sum(1), String keys (WordCountData, "
                        "287 tokens / 170 words) hashed by the host, 10M tokens per step, 2000 tokens per ms"),
    "c2": dict(rate=100_000_000, bound=200, jitter=200, zipf=None, keys=1_000_000, cpu_sample=1 << 24,
               workload="C2 tumbling 1s event-time window, count/sum/min/max, 1M uniform Long keys, "
                        "bounded out-of-orderness 200 ms"),
    "c3": dict(rate=100_000_000, bound=200, jitter=200, zipf=None, keys=2_000_000, cpu_sample=1 << 19,
               workload="C3 sliding 60s/1s event-time windows (60x fan-out), count/sum/min/max, 2M uniform Long keys "
                        "per GPU (16M at 8 GPUs), bounded out-of-orderness 200 ms"),
    "c5": dict(rate=100_000_000, bound=200, jitter=200, zipf=1.1, keys=1_000_000, cpu_sample=1 << 20,
               workload="C5 tumbling 1s event-time window, HyperLogLog (p=14) distinct count per key and window, "
                        "1M Zipf(1.1) Long keys, bounded out-of-orderness 200 ms"),
    "c5t": dict(rate=100_000_000, bound=200, jitter=200, zipf=1.1, keys=1_000_000, cpu_sample=1 << 22,
                workload="C5 tumbling 1s event-time window, t-digest (delta=100) quantiles p50/p95/p99 of a Double "
                         "field per key and window, 1M Zipf(1.1) Long keys, bounded out-of-orderness 200 ms"),
    "c4": dict(rate=100_000, bound=1000, jitter=1000, zipf=1.1, keys=1_000_000, cpu_sample=1 << 22,
               workload="C4 EventTimeSessionWindows gap 30 s, count/sum/min/max, 1M Zipf(1.1) Long keys, "
                        "bounded out-of-orderness 1 s"),
}


def b_alg(workload, fired_per_record, world, hll_p=14, panes=60, centroids_per_record=0.0):
    """SURVEY §8d algorithmic HBM bytes per record (the figure `roofline` and `path_roofline` use):
    input 24 B (+ 4 B key hash at C1), the keyBy exchange 2 x 24 (G-1)/G, state RMW where §8d counts it,
    and the fired rows' entry reads + 56-B rows."""
    bx = 48 * (world - 1) / world
    f = fired_per_record
    if workload == "c1":
        return 28 + 104 * f + bx
    if workload == "c3":  # pane model: one pane update per record, size/slide pane reads per fired window
        return 24 + bx + 96 + (panes * 48 + 56) * f
    if workload == "c4":
        return 24 + bx + 112 * f
    if workload == "c5":  # HLL: one register byte RMW per record, the 2^p register block read per fired row
        return 24 + bx + 2 + ((1 << hll_p) + 56) * f
    if workload == "c5t":  # t-digest: 16 B per record into the digest, 16 B per fired centroid + the row
        return 24 + bx + 16 + 16 * centroids_per_record + 56 * f
    return 24 + bx + 104 * f  # c2


def kernel_share(name, workload, f, hll_p=14, panes=60, centroids_per_record=0.0):
    """Per record, the bytes each timing bucket must move in this build's data flow (its own share, VERDICT r03
    item 7): the partitioning reads the input (B_in) and writes each record once into its partition's
    run (16-B CRec, 32-B PRec for sessions); the aggregate reads that record back and does §8d's state
    read-modify-write (C3: one 48-B pane RMW; C5: the HLL register byte; 0 where §8d counts the table as
    cache-resident); the t-digest compression adds §8d's 16 B per value; the firing reads what fires and writes
    the rows (§8d B_fire).  The design-independent figure is `path_roofline` (B_alg x records/s)."""
    rec = 32 if workload == "c4" else 16
    b_in = 28 if workload == "c1" else 24
    if name == "k_scatter":
        return b_in + rec
    if name == "k_aggregate":
        return rec + {"c3": 96, "c5": 2}.get(workload, 0)
    if name == "k_tdigest":
        return 16
    if name == "k_fire":
        if workload == "c3":
            return (panes * 48 + 56) * f
        if workload == "c4":
            return 112 * f
        if workload == "c5":
            return ((1 << hll_p) + 56) * f
        if workload == "c5t":
            return 16 * centroids_per_record + 56 * f
        return 104 * f
    return 0.0


def impl_bytes(name, n, merged, fired=0, hll_p=0, panes_per_window=0, compact=True, single=False):
    """What one launch of a kernel moves as built, for the `impl_bytes` field.  single: the
    batches took the single-pass scatter (k_scatter_rsv), behind which classify / scan / scatter only check a flag."""
    rec = 16 if compact else 32  # partitioned record: CRec {key hash | window, val} or PRec
    if single and name in ("k_classify_hist", "k_scan"):
        return 0
    if name == "k_fire":
        if hll_p:
            return fired * (64 + 2 * (1 << hll_p) + 56)
        if panes_per_window:
            return fired * (64 * panes_per_window + 56)
        return fired * (64 + 56)
    if name == "k_classify_hist":
        return 16 * n
    if name == "k_scatter":
        return 24 * n + rec * n
    if name == "k_aggregate":
        return rec * n + 128 * merged
    if name == "k_tdigest":  # grouping (read the record; digest, rank and value key written, the rank rewritten),
        # placement into the digests' runs (16 B read, 12 B written), the run sorts (8 B read and written; the hot
        # keys' runs once more through a sample-sort pass, about half the values), the tiers (24)
        return rec * n + 16 * n + 8 * n + 28 * n + 16 * n + 8 * n + 24 * n
    return None


def cpu_info():
    model = platform.processor() or "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model, os.cpu_count()


def wordcount_stream(first, n):
    """C1 tokens: token i = WordCountData's token splitmix64(0x5EED ^ 4i) mod 287; key = the word's id among
    the 170 distinct words, key_hash = String.hashCode(word), value = 1, ts = i // 2000 ms."""
    import numpy as np
    from flink_amd.datagen import generate_host
    from flink_amd.keygroups import string_hash_code
    toks = json.load(open(os.path.join(ROOT, "tests", "golden", "wordcount_tokens.json")))["tokens"]
    words = sorted(set(toks))
    wid = np.array([words.index(t) for t in toks], dtype=np.int64)
    hashes = np.array([string_hash_code(w) for w in words], dtype=np.int32)
    idx, _, _ = generate_host(0x5EED, first, n, len(toks), ts_base=0, rate=2_000_000, jitter=0)
    keys = wid[idx]
    ts = (np.arange(first, first + n, dtype=np.int64) // 2000)
    return keys, ts, np.ones(n, dtype=np.int64), hashes[keys]


def job_cpu_share():
    """The host cores this job may use: the CPU affinity mask, capped by OMP_NUM_THREADS when the box sets it (the
    GPU box shows all of its cores to every job and declares the job's share there: 16 for one GPU)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and 0 < int(omp) < aff:
        return int(omp), f"OMP_NUM_THREADS={omp} (the job's CPU share; affinity mask {aff} cores)"
    return aff, f"the CPU affinity mask ({aff} cores)"


def visible_gpus(topology="/sys/class/kfd/kfd/topology/nodes"):
    """GPUs this node offers the ranks, counted WITHOUT any HIP call (the launcher must not initialise the GPU: a
    process that did must never be replaced, and torch.cuda.device_count() falls back to hipGetDeviceCount when the
    amdsmi discovery fails).  The KFD topology lists one node per agent; GPU agents have a non-zero
    gfx_target_version.  A *_VISIBLE_DEVICES list narrows the count.  None when the count is unavailable (the
    ranks then find out for themselves)."""
    import glob
    n = 0
    try:
        for props in glob.glob(os.path.join(topology, "*", "properties")):
            with open(props) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    if k == "gfx_target_version" and v.strip() not in ("", "0"):
                        n += 1
                        break
    except OSError:
        return None
    if n == 0:
        return None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        lst = os.environ.get(var)
        if lst is not None:
            n = min(n, len([x for x in lst.split(",") if x.strip()]))
    return n


def launch_ranks(args, argv):
    """`--gpus N` (N > 1) without a torch.distributed launcher around it: start one rank per GPU with
    `python -m torch.distributed.run` (rendezvous on 127.0.0.1, one process per GPU, RCCL between them) and pass
    its exit status on; rank 0 prints the JSON line.  This process makes no HIP call (it counts GPUs from the KFD
    topology, visible_gpus(); torch is not even imported) and never exec()s: the ranks are children."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + \
        [a for a in argv if a != "--dry-run-launch"]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (the host driver has no legacy IPC)
    env["MASTER_ADDR"] = "127.0.0.1"
    if args.dry_run_launch:
        print(json.dumps({"launch": cmd, "nproc": args.gpus,
                          "env": {k: env[k] for k in ("HSA_ENABLE_IPC_MODE_LEGACY", "MASTER_ADDR")}}), flush=True)
        return 0
    have = visible_gpus()
    need = 1 if args.rehearse_gloo else args.gpus
    if have is not None and have < need:
        print(f"bench.py: --gpus {args.gpus} needs {need} visible GPUs, this node shows {have}", file=sys.stderr,
              flush=True)
        return 2
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node, one rank each (default 1; N > 1 starts N ranks with torch.distributed.run "
                         "unless already launched by it)")
    ap.add_argument("--dry-run-launch", action="store_true",
                    help="with --gpus N > 1: print the rank launcher's command and environment, start nothing")
    ap.add_argument("--steps", type=int, default=64)  # 64 x 2^24 = 2^30 records
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--workload", choices=sorted(PRESETS), default="c2")
    ap.add_argument("--batch", type=int, default=None, help="records per step per GPU (default 2^24; C1 10M)")
    ap.add_argument("--keys", type=int, default=None)
    ap.add_argument("--rate", type=int, default=None, help="records per event-second (whole job)")
    ap.add_argument("--bound", type=int, default=None, help="out-of-orderness bound (ms)")
    ap.add_argument("--jitter", type=int, default=None)
    ap.add_argument("--window", type=int, default=None, help="tumbling window (ms; c2/c5 1000, c1 5000)")
    ap.add_argument("--gap", type=int, default=30_000, help="session gap (ms, c4)")
    ap.add_argument("--size", type=int, default=60_000, help="sliding window size (ms, c3)")
    ap.add_argument("--slide", type=int, default=1000, help="sliding window slide (ms, c3)")
    ap.add_argument("--hll-p", type=int, default=14, help="HyperLogLog precision (c5)")
    ap.add_argument("--delta", type=int, default=100, help="t-digest compression (c5t)")
    ap.add_argument("--no-steady", dest="steady", action="store_false",
                    help="c3: do not extend the warmup to one window size of event time")
    ap.add_argument("--cpu-sample", type=int, default=None)
    ap.add_argument("--zipf", type=float, default=None, help="Zipf exponent of the keys (0 = uniform)")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU baseline subtasks (default: the job's CPU share, job_cpu_share())")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-fed-steps", type=int, default=None,
                    help="steps of the host-fed leg (0 = skip; default: enough event time to cross a window end, so "
                         "fw_drain_rows moves rows)")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-kernel HIP-event timing")
    ap.add_argument("--traffic", default=None,
                    help="PMC traffic summary (tools/traffic.py); default the newest profiles/traffic_*<workload>.json")
    ap.add_argument("--sub-partitions", type=int, default=0, help="state partitions per key group (0 = auto)")
    ap.add_argument("--combine", action="store_true",
                    help="pre-shuffle combining (SURVEY §8e): partial accumulators instead of records cross the "
                         "exchange (C2: tumbling count/sum/min/max; C5: HyperLogLog partial rows + non-zero registers)")
    ap.add_argument("--rehearse-gloo", action="store_true",
                    help="N > 1 on ONE GPU: every rank on cuda:0 and the Python exchange over gloo (exercises the "
                         "multi-rank bench path; RCCL cannot put two ranks on one GPU)")
    ap.add_argument("--sync-input", action="store_true",
                    help="partition each batch on the operator's own stream (no overlap with the previous batch)")
    args = ap.parse_args()
    if args.combine and args.rehearse_gloo:
        ap.error("--combine with --rehearse-gloo: the gloo rehearsal exchanges records through the Python exchange "
                 "and would not combine (the line would claim a combining run)")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    if args.gpus is not None and env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks")
    preset = PRESETS[args.workload]
    w = args.workload
    for name in ("keys", "rate", "bound", "jitter", "cpu_sample", "batch"):
        if getattr(args, name) is None:
            setattr(args, name, preset.get(name, 1 << 24))
    if args.window is None:
        args.window = 5000 if w == "c1" else 1000
    if args.zipf is None:
        args.zipf = preset["zipf"]
    args.zipf = args.zipf or None
    if args.traffic is None:
        for cand in (f"traffic_r06_{w}.json", f"traffic_r05_{w}.json", f"traffic_r04_{w}.json", f"traffic_r03_{w}.json",
                     f"traffic_r02_{w}.json", f"traffic_r01_{w}.json" if w != "c2" else "traffic_r01.json"):
            args.traffic = os.path.join(ROOT, "profiles", cand)
            if os.path.exists(args.traffic):
                break
    sessions, sliding, hll, tdig, c1 = w == "c4", w == "c3", w == "c5", w == "c5t", w == "c1"

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    gloo = world > 1 and args.rehearse_gloo
    if gloo:  # rehearsal of the N > 1 path on one GPU: every rank on cuda:0, the Python exchange over gloo
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    coll_dev = torch.device("cpu") if gloo else dev  # where the bench's own collectives' tensors live
    if world > 1:
        import torch.distributed as dist
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from flink_amd import (CountSumMinMax, EventTimeSessionWindows, HyperLogLog, SlidingEventTimeWindows, TDigest,
                           TumblingEventTimeWindows)
    from flink_amd import _native as N
    from flink_amd.datagen import generate_device, zipf_cdf
    from flink_amd.exchange import KeyGroupExchange
    from flink_amd.operator import GpuWindowOperator

    max_par = 128
    exch = KeyGroupExchange(max_par, world, rank, key_type="hashed" if c1 else "long")
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
    agg = (HyperLogLog(args.hll_p) if hll else TDigest(args.delta) if tdig else CountSumMinMax("int") if c1
           else CountSumMinMax())
    op = GpuWindowOperator(assigner, agg, key_group_range=exch.key_group_range, key_type="hashed" if c1 else "long",
                           device=local_rank, max_parallelism=max_par,
                           expected_entries=(1000 if c1 else live_windows * args.keys // world),
                           max_batch=args.batch if world == 1 else 2 * args.batch,
                           sub_partitions=args.sub_partitions, async_input=not args.sync_input)
    nx = None
    if world > 1 and not gloo:
        # the keyBy exchange a JNI host calls: fw_keyby_push_device over the library's own RCCL communicator
        # (route, count all-to-all, per-peer ncclSend / ncclRecv, push), rank 0's id handed to the others
        import torch.distributed as dist
        from flink_amd.exchange import NativeKeyByExchange
        uid = [NativeKeyByExchange.new_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        nx = NativeKeyByExchange(op, world, rank, uid[0])
    cx = comb = None
    if args.combine:
        if w not in ("c2", "c5"):
            raise SystemExit("--combine: C2 (tumbling count/sum/min/max) and C5 (tumbling HyperLogLog) combine")
        from flink_amd.exchange import CombiningExchange
        # the combiner sees this rank's whole slice of the key space
        comb = GpuWindowOperator(assigner, agg, device=local_rank, max_parallelism=max_par,
                                 expected_entries=live_windows * args.keys, max_batch=args.batch,
                                 sub_partitions=args.sub_partitions)
        cx = CombiningExchange(exch, comb)
    if sliding and args.steady:
        # steady state: the warmup covers one window size of event time, so the timed steps see the
        # full pane population (size/slide + 1 panes per key) and windows merging size/slide panes
        event_ms_per_step = args.batch * world * 1000.0 / args.rate
        args.warmup = max(args.warmup, int(args.size / event_ms_per_step) + 2)
    steps_total = args.warmup + args.steps
    seed = 0x5EED

    def generate(s):
        first = (s * world + rank) * args.batch  # global record index of this rank's slice of step s
        if c1:
            k, t, v, h = wordcount_stream(first, args.batch)
            dk, dt, dv, dh = (torch.from_numpy(x).to(dev) for x in (k, t, v, h))
            return dk, dt, dv, torch.tensor([int(t.max())], device=dev), dh
        k, t, v, mx = generate_device(seed, first, args.batch, args.keys, ts_base=0, rate=args.rate,
                                      jitter=args.jitter, cdf_dev=cdf, device=local_rank)
        if tdig:
            v = v.to(torch.float64)  # the Double field: the generator's int32 values
        return k, t, v, mx, None

    # warmup batches are generated step by step (untimed); the timed ones are staged in HBM up front.
    # punctuated watermark of this rank's source after each batch: max ts so far - bound
    batches, local_wm = {}, {}
    m = -(1 << 63)
    # with async input the timed region overlaps each batch's partitioning with the previous batch's aggregation,
    # so the kernels' own durations are also measured in an isolated pass of as many steps after it
    iso_steps = args.steps if (not args.no_profile and not args.sync_input) else 0
    for s in range(args.warmup, steps_total + iso_steps):
        k, t, v, mx, h = generate(s)
        batches[s] = (k, t, v, h)
        local_wm[s] = int(mx.item())  # this batch's max; made cumulative once the warmup's is known
    torch.cuda.synchronize()

    def step(s):
        nonlocal m
        if s < args.warmup:
            k, t, v, mx, h = generate(s)
            m = max(m, int(mx.item()))
            wm = m - args.bound
        else:
            k, t, v, h = batches[s]
            wm = local_wm[s]
        if nx is not None and comb is not None:  # combine, exchange the partials, merge them (fw_keyby_combine_push_device)
            wm = nx.push_combined(comb, k, t, v, wm)
        elif nx is not None:  # route, exchange, push (fw_keyby_push_device); wm = min over the subtasks
            wm = nx.push(k, t, v, wm, h)
        elif gloo:  # rehearsal: fw_route_device + gloo all-to-alls through host memory (KeyGroupExchange)
            got = exch.exchange(k, t, v, h)
            wm = exch.combine_watermark(wm)
            op.process_batch(*got)
        elif cx is not None:  # world 1: combine and merge through the Python exchange
            wm = cx.push(op, k, t, v, wm)
        else:
            op.process_batch(k, t, v, h)            # queued; settles the previous step's sequence
        op.advance_watermark(wm, wait=False)  # queued behind the push
        op.clear_pending()  # discarding sink: fired rows were materialised in HBM

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    L = N.lib()
    if not args.no_profile and args.warmup:  # the warmup times every kernel kind to find the dominant one
        L.fw_profile(op._h, 1)
    for s in range(args.warmup):
        step(s)
    for j in range(args.warmup, steps_total + iso_steps):  # fold the warmup's running max into the staged batch maxima
        m = max(m, local_wm[j])
        local_wm[j] = m - args.bound
    if not args.no_profile:
        import ctypes
        # the timed region records events around the warmup's two dominant kernels only: every timed launch adds two
        # markers to its stream, and timing every kind cost C2 ~10 % of its step
        mask = 1
        if args.warmup:
            ms_w = (ctypes.c_double * N.FW_NUM_KERNELS)()
            L.fw_profile_read(op._h, ms_w, None, 1)
            top = sorted(range(N.FW_NUM_KERNELS), key=lambda i: -ms_w[i])[:2]  # (the two largest: a firing-bound
            mask = N.FW_PROFILE_KINDS | (1 << top[0]) | (1 << top[1])  # workload may not fire in the warmup)
        L.fw_profile(op._h, mask)
        L.fw_profile_read(op._h, None, None, 1)
    st0 = op.stats()
    def exchange_stats():
        if nx is not None:
            return nx.stats()
        return {"world": world, "rank": rank, "bytes_sent": exch.bytes_sent, "items_sent": exch.items_sent,
                "bytes_received": exch.bytes_received, "recv_reallocs": 0}

    xs0 = exchange_stats() if world > 1 else None
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

    exchange = None
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        xs1 = exchange_stats()
        sent = [xs1[f] - xs0[f] for f in ("bytes_sent", "items_sent", "bytes_received", "recv_reallocs")]
        allr = [torch.zeros(4, dtype=torch.float64, device=coll_dev) for _ in range(world)]
        dist.all_gather(allr, torch.tensor(sent, dtype=torch.float64, device=coll_dev))
        allr = [[float(x) for x in r.tolist()] for r in allr]
        total_sent = sum(r[0] for r in allr)
        xgmi_peak = world * (world - 1) * XGMI_LINK_GBS * 1e9  # G (G-1) links of 153 GB/s
        exchange = {"impl": ("fw_keyby_push_device" + ("/combine" if comb is not None else "") +
                             " (RCCL: count all-to-all + watermark MIN + batch SUM, grouped per-peer "
                             "ncclSend/ncclRecv)") if nx is not None else
                            "REHEARSAL: fw_route_device + torch.distributed gloo all-to-alls, every rank on cuda:0 "
                            "(not a multi-GPU measurement)",
                    "rccl_ranks": int(xs1["world"]) if nx is not None else None, "rccl_rank0": int(xs1["rank"]),
                    "bytes_sent_per_rank": [int(r[0]) for r in allr],
                    "items_sent_per_rank": [int(r[1]) for r in allr],
                    "bytes_received_per_rank": [int(r[2]) for r in allr],
                    "recv_reallocs_in_timed_region": int(sum(r[3] for r in allr)),
                    "shuffled_bytes_per_s": round(total_sent / elapsed, 1),
                    "xgmi_frac": round(total_sent / elapsed / xgmi_peak, 4),
                    "xgmi_basis": f"bytes sent to other ranks in the timed region / time / (G (G-1) x "
                                  f"{XGMI_LINK_GBS:.0f} GB/s), SURVEY §8d"}
    records = args.batch * world * args.steps
    value = records / elapsed
    fired = st1["fired_rows_total"] - st0["fired_rows_total"]
    per_gpu_records = records / world
    fpr = fired / max(1, per_gpu_records)
    cpr = (st1["digest_centroids_fired"] - st0["digest_centroids_fired"]) / max(1, per_gpu_records)
    balg = b_alg(w, fpr, world, args.hll_p, args.size // args.slide, cpr)
    path_frac = value * balg / (world * HBM_PEAK_GBS * 1e9)

    roofline = None
    kernels = {}
    if not args.no_profile:
        import ctypes
        ms = (ctypes.c_double * N.FW_NUM_KERNELS)()
        nl = (ctypes.c_int64 * N.FW_NUM_KERNELS)()
        L.fw_profile_read(op._h, ms, nl, 1)
        merged = (st1["state_merges"] - st0["state_merges"]) / args.steps
        single = st1["single_pass_batches"] - st0["single_pass_batches"] == args.steps
        per_launch_records = per_gpu_records / args.steps
        tr, tr_all, tr_src = {}, None, None
        if os.path.exists(args.traffic):
            with open(args.traffic) as f:
                t = json.load(f)
            if t.get("workload", "c2") == w:  # PMC bytes per launch of this workload (tools/traffic.py)
                tr = t.get("per_launch_bytes", {})
                tr_all = t.get("bytes_per_record_all_kernels")
                tr_src = os.path.relpath(args.traffic, ROOT)
        alg_path = balg * per_launch_records
        share = {}
        for i in range(N.FW_NUM_KERNELS):
            name = L.fw_kernel_name(i).decode()
            if not nl[i]:
                continue
            avg = ms[i] / nl[i]
            ib = impl_bytes(name, per_launch_records, merged, fired=fired / nl[i], hll_p=args.hll_p if hll else 0,
                            panes_per_window=args.size // args.slide if sliding else 0, single=single)
            # the bucket's own algorithmic bytes per launch: its share per record x the records of one launch (a
            # watermark's firing: the records of the steps it follows)
            sh = kernel_share(name, w, fpr, args.hll_p, args.size // args.slide, cpr)
            share[name] = sh * per_gpu_records / nl[i]
            kernels[name] = {"launches": int(nl[i]), "avg_ms": round(avg, 5), "total_ms": round(ms[i], 4),
                             "alg_bytes_per_record": round(sh, 3), "alg_bytes_per_launch": int(share[name]),
                             "frac": round(share[name] / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                             "impl_bytes": None if ib is None else int(ib),
                             "impl_frac": None if not ib else round(ib / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                             "traffic": tr.get(name)}
        dom = max(kernels, key=lambda k: kernels[k]["total_ms"])
        kd = kernels[dom]
        alg = share[dom]
        achieved = alg / (kd["avg_ms"] * 1e-3) / 1e9
        traffic = tr.get(dom)
        # the WHOLE step's algorithmic bytes (B_alg x records per launch) over the dominant
        # kernel's duration alone: design-independent, an upper bound on any one kernel's frac
        sec8d = alg_path / (kd["avg_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "sec8d_frac": round(sec8d, 4),
                    "sec8d_basis": "SURVEY §8d B_alg x records per launch / the dominant kernel's average duration",
                    "traffic": traffic,
                    "alg_bytes_per_launch": int(alg), "alg_bytes_per_record": kd["alg_bytes_per_record"],
                    "path_alg_bytes_per_launch": int(alg_path),
                    "impl_bytes_per_launch": kd["impl_bytes"], "impl_frac": kd["impl_frac"],
                    "traffic_over_alg": None if (traffic is None or not alg) else round(traffic / alg, 3),
                    "traffic_per_record": None if traffic is None else round(traffic / per_launch_records, 2),
                    "traffic_all_kernels_per_record": tr_all, "traffic_source": tr_src,
                    "basis": "the dominant bucket's own share (bench.py kernel_share: input + partitioned-record "
                             "write for the partitioning, record read + SURVEY §8d state RMW for the aggregate, "
                             "§8d B_fire for the firing) x records per launch / its average HIP-event duration "
                             "(on the stream it runs on); path_roofline prices the whole step at §8d B_alg"}
    kernels_iso = None
    if iso_steps:
        import ctypes
        kernels_iso = {}
        op.set_async_input(False)  # (synchronizes)
        L.fw_profile(op._h, 1)  # every kind in the isolated pass
        L.fw_profile_read(op._h, None, None, 1)
        for s in range(steps_total, steps_total + iso_steps):
            step(s)
        op.synchronize()
        ms_i = (ctypes.c_double * N.FW_NUM_KERNELS)()
        nl_i = (ctypes.c_int64 * N.FW_NUM_KERNELS)()
        L.fw_profile_read(op._h, ms_i, nl_i, 1)
        for i in range(N.FW_NUM_KERNELS):
            if nl_i[i]:
                kernels_iso[L.fw_kernel_name(i).decode()] = {"launches": int(nl_i[i]),
                                                             "avg_ms": round(ms_i[i] / nl_i[i], 5)}
    if kernels_iso and roofline:
        # the same kernel's own duration: the isolated pass (its batch partitioned on the operator's stream)
        ki = kernels_iso.get(roofline["kernel"])
        if ki:
            a_i = alg / (ki["avg_ms"] * 1e-3) / 1e9
            roofline["isolated"] = {"avg_ms": ki["avg_ms"], "achieved": round(a_i, 1),
                                    "frac": round(a_i / HBM_PEAK_GBS, 4),
                                    "sec8d_frac": round(alg_path / (ki["avg_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                    "basis": f"{iso_steps} further steps after the timed region with --sync-input "
                                             "(no overlap): the kernel's duration alone on the GPU"}

    count_gpu = None
    if c1 and world == 1:
        count_gpu = count_window_leg(args, batches, local_rank)

    host_fed = None
    if args.host_fed_steps is None:
        # enough steps that the watermark passes a window end (a 1 s / 5 s window, C3's 1 s slide; sessions of C4 end
        # every step at its 1e5 records per event-second), so the leg drains fired rows (WindowOperator.java:544-548)
        period = args.slide if sliding else (1 if sessions else args.window)
        event_ms = args.batch * 1000.0 / args.rate
        args.host_fed_steps = int(min(12, max(3, (period + args.bound) / event_ms + 2)))
    if rank == 0 and world == 1 and args.host_fed_steps > 0:
        host_fed = host_fed_leg(args, op, generate, steps_total + iso_steps, m, c1)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)

    if rank == 0:
        line = {
            "metric": "records/sec keyed windowed aggregation at 1/2/4/8 GPUs; % of HBM roofline",
            "value": round(value, 1), "unit": "records/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            **({"rccl_ranks": exchange["rccl_ranks"]} if exchange else {}),
            **({"rehearsal": "gloo, all ranks on one GPU: checks the N > 1 code path, not a scaling number"}
               if gloo else {}),
            "dtype": "f64" if tdig else "int64", "data": "synthetic (splitmix64 counter stream)",
            "config": {"workload": preset["workload"],
                       "records_per_step_per_gpu": args.batch, "keys": args.keys,
                       **({"gap_ms": args.gap, "zipf_s": args.zipf} if sessions else
                          {"size_ms": args.size, "slide_ms": args.slide} if sliding else
                          {"window_ms": args.window, "hll_precision": args.hll_p, "zipf_s": args.zipf} if hll else
                          {"window_ms": args.window, "tdigest_delta": args.delta, "zipf_s": args.zipf} if tdig else
                          {"window_ms": args.window}),
                       "records_per_event_second": args.rate, "watermark_bound_ms": args.bound,
                       "max_parallelism": 128, "parallelism": f"keygroup{world}",
                       "sink": "discarding (fired rows materialised in HBM)",

                       **({"combine": "pre-shuffle partial accumulators (SURVEY §8e)"} if cx is not None else {})},
            "roofline": roofline,
            "path_roofline": {"b_alg_bytes_per_record": round(balg, 3), "frac": round(path_frac, 4),
                              "fired_rows": int(fired)},
            **({"exchange": exchange} if exchange else {}),
            "host_fed": host_fed,
            **({"count_window_gpu": count_gpu} if count_gpu else {}),
            "cpu_baseline": cpu,
            "kernels": kernels,
            **({"kernels_isolated": kernels_iso} if kernels_iso else {}),
            "state": {"single_pass_batches": int(st1["single_pass_batches"] - st0["single_pass_batches"]),
                      "single_pass_redone": int(st1["single_pass_redone"] - st0["single_pass_redone"]),
                      "table_slots": int(st1["table_capacity"]), "table_grows_in_timed_region":
                      int(st1["table_grows"] - st0["table_grows"]), "live_entries": int(st1["keyed_state_entries"])},
        }
        print(json.dumps(line), flush=True)
    if nx is not None:
        nx.close()
    op.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def count_window_leg(args, batches, device):
    """C1's other pipeline on the GPU: keyBy(word).countWindow(10, 5).sum(1) (WindowWordCount.java:74-81;
    EvictingWindowOperator + CountTrigger + CountEvictor) over the same device-resident token batches, the
    rows materialised in HBM; timed like the main leg (the batches' pushes between synchronisations)."""
    import torch
    from flink_amd import CountWindows
    from flink_amd.operator import GpuWindowOperator
    from flink_amd.windowing import FirstElementReduce
    op = GpuWindowOperator(CountWindows.of(10, 5), FirstElementReduce("int", "sum"), device=device,
                           expected_entries=1000, max_batch=args.batch)
    keys = sorted(batches)
    k, t, v, _ = batches[keys[0]]
    op.process_batch(k, t, v)  # warm (slot map, allocations)
    op.synchronize()
    op.clear_pending()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rows = 0
    for s in keys:
        k, t, v, _ = batches[s]
        op.process_batch(k, t, v)
        n_rows = op.advance_watermark(0)  # settles: the count windows fired while the batch was processed
        rows += n_rows
        op.clear_pending()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    op.close()
    n = args.batch * len(keys)
    return {"value": round(n / dt, 1), "unit": "records/s", "steps": len(keys), "fired_rows": int(rows),
            "ms_per_step": round(dt / len(keys) * 1e3, 3),
            "pipeline": "countWindow(10, 5).sum(1) on the GPU (k_cnt_*: key slots, stable sort, fire, ring update)"}


def host_fed_leg(args, op, generate, first_step, m, c1):
    """The JNI drop-in path end to end: batches in pinned host memory (a Java DirectByteBuffer's role) pushed
    with fw_push_batch (H2D copy, processed before the call returns), the watermark, and the fired rows drained
    to host memory.  Continues the same stream after the timed steps."""
    import torch
    staged = []
    for s in range(first_step, first_step + args.host_fed_steps):
        k, t, v, mx, h = generate(s)
        m = max(m, int(mx.item()))
        cols = [x.cpu().pin_memory() for x in (k, t, v) + ((h,) if h is not None else ())]
        staged.append((cols, m - args.bound))
    torch.cuda.synchronize()
    op.synchronize()
    op.clear_pending()
    rows = 0
    t0 = time.perf_counter()
    for cols, wm in staged:
        k, t, v = (x.numpy() for x in cols[:3])
        op.process_batch(k, t, v, cols[3].numpy() if len(cols) > 3 else None)
        op.advance_watermark(wm)
        rows += len(op.drain_rows())
    dt = time.perf_counter() - t0
    n = args.batch * args.host_fed_steps
    return {"value": round(n / dt, 1), "unit": "records/s", "steps": args.host_fed_steps, "fired_rows": rows,
            "ms_per_step": round(dt / args.host_fed_steps * 1e3, 3),
            "path": "fw_push_batch from pinned host buffers (H2D inside the call) + fw_advance_watermark + "
                    "fw_drain_rows to host: PCIe-inclusive, not the headline value"}


def cpu_baseline(args):
    """CPU restatement of WindowOperator (oracle/, kind "port"): p threads = p subtasks over their
    KeyGroupRanges, the same generator and punctuated watermarks, on a bounded sample.  C1 runs at p = 1
    (LocalStreamEnvironment parallelism 1, BASELINE configs[0]) for both WindowWordCount pipelines."""
    import numpy as np
    from flink_amd.datagen import generate_host
    from oracle import oracle as orc
    model, nproc = cpu_info()
    n = args.cpu_sample
    if args.workload == "c1":
        k, t, v, _ = wordcount_stream(0, n)
        t0 = time.perf_counter()
        cw = orc.CountWindowOracle(10, 5, value_type="i32")  # countWindow(10, 5).sum(1), WindowWordCount.java:74-81
        cw.process(k, v)
        dt_count = time.perf_counter() - t0
        t0 = time.perf_counter()
        tw = orc.WindowOperatorOracle(assigner="tumbling", size=args.window, value_type="i32")
        tw.process(k, t, v)
        tw.watermark((1 << 63) - 1)
        dt = time.perf_counter() - t0
        return {"value": round(n / dt, 1), "unit": "records/s", "cores": 1, "kind": "port",
                "count_window_value": round(n / dt_count, 1), "cpu_model": model, "nproc": nproc, "parallelism": 1,
                "sample": f"all {n} tokens of C1 at p = 1: value = window(Tumbling {args.window} ms).sum(1) (the GPU "
                          f"line's pipeline), count_window_value = countWindow(10, 5).sum(1); CPU restatement of "
                          f"WindowOperator / EvictingWindowOperator semantics (oracle/), not the Java reference "
                          f"(no JDK on the box)"}
    share, why = job_cpu_share()
    threads = args.cpu_threads or share
    why = why if not args.cpu_threads else f"--cpu-threads {args.cpu_threads}"
    k, t, v = generate_host(0x5EED, 0, n, args.keys, ts_base=0, rate=args.rate, jitter=args.jitter, zipf_s=args.zipf)
    if args.workload == "c5t":
        v = v.astype(np.float64)
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
    elif args.workload == "c5t":
        cfg = dict(assigner="tumbling", size=args.window, tdigest=args.delta)
    else:
        cfg = dict(assigner="tumbling", size=args.window)
    orc.run_parallel(cfg, k, t, v, batch, np.array(wms), 128, threads)
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 1), "unit": "records/s", "cores": threads, "kind": "port", "cpu_model": model,
            "nproc": nproc, "parallelism": threads, "parallelism_basis": why,
            "sample": f"first {n} records of the same {args.workload.upper()} stream, {threads} subtasks (threads; "
                      f"p = the host cores this job may use: {why}; nproc = {nproc}), watermark every {batch} "
                      f"records; CPU "
                      f"restatement of WindowOperator semantics (oracle/, C++ -O2), not the Java reference (no JDK "
                      f"on the box)"}


if __name__ == "__main__":
    main()
