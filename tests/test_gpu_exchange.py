"""The keyBy exchange with the library's own kernels on the GPU:

* world size 2 over gloo, both subtasks on cuda:0: fw_route_device groups each subtask's batch by destination
  (computeOperatorIndexForKeyGroup, KeyGroupRangeAssignment.java:115-117), the columns (and the key hashes of
  String keys) go through all_to_all_single, each subtask's GpuWindowOperator owns its KeyGroupRange, and the
  watermark is the minimum over subtasks (StatusWatermarkValve.java:173-191).  The union of both subtasks'
  rows must equal one oracle operator over the whole stream.  Long keys, Integer keys with negative values
  (Integer.hashCode differs from Long.hashCode) and String keys hashed by the host.
* fw_keyby_push_device (the C-ABI exchange over the library's RCCL communicator) at world size 1, and at world
  size 2 with a skewed send (two GPUs).
"""
import os
import socket

import numpy as np
import pytest

from flink_amd.datagen import generate_host
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

MAX_PAR, WORLD, BATCH, STEPS, KEYS = 128, 2, 20_000, 5, 3000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# operator kinds through the exchange: (assigner, oracle kwargs, key distribution); the session and HLL streams
# draw Zipf(1.1) keys (BASELINE configs[3] / [4] shapes at parity size), panes are sliding 60 s / 1 s (configs[2])
KINDS = {
    "tumbling": dict(oracle=dict(assigner="tumbling", size=1000), zipf=None),
    "sessions": dict(oracle=dict(assigner="session", gap=30_000), zipf=1.1),
    "panes": dict(oracle=dict(assigner="sliding", size=60_000, slide=1000), zipf=None),
    "hll": dict(oracle=dict(assigner="tumbling", size=1000, hll_p=12), zipf=1.1),
    "tdigest": dict(oracle=dict(assigner="tumbling", size=1000, tdigest=100), zipf=1.1),
}


def _operator(kind, key_type, kgr):
    from flink_amd import (EventTimeSessionWindows, HyperLogLog, SlidingEventTimeWindows, TDigest,
                           TumblingEventTimeWindows)
    from flink_amd.operator import GpuWindowOperator
    from flink_amd.windowing import CountSumMinMax
    assigner = {"tumbling": TumblingEventTimeWindows.of(1000), "sessions": EventTimeSessionWindows.with_gap(30_000),
                "panes": SlidingEventTimeWindows.of(60_000, 1000), "hll": TumblingEventTimeWindows.of(1000),
                "tdigest": TumblingEventTimeWindows.of(1000)}[kind]
    agg = HyperLogLog(12) if kind == "hll" else TDigest(100) if kind == "tdigest" else CountSumMinMax()
    return GpuWindowOperator(assigner, agg, key_type=key_type, max_parallelism=MAX_PAR, key_group_range=kgr,
                             device=0, expected_entries=20_000 if kind in ("hll", "tdigest") else 0)


def _slice(rank, step, key_type, kind="tumbling"):
    from flink_amd.keygroups import string_hash_code
    first = (step * WORLD + rank) * BATCH
    k, t, v = generate_host(0x5EED, first, BATCH, KEYS, ts_base=0, rate=100_000, jitter=300,
                            zipf_s=KINDS[kind]["zipf"])
    h = None
    if key_type == "int":
        k = k - KEYS // 2  # negative Integer keys
    elif key_type == "hashed":
        h = np.array([string_hash_code(f"word-{x}") for x in range(KEYS)], dtype=np.int32)[k]
    if kind == "tdigest":  # a Double field: distinct-ish values of both signs
        v = (v & 0xFFFFFF).astype(np.float64) / 7.0 - 1.0e6
    return k, t, v, h


def _worker(rank, port, out_dir, key_type, kind="tumbling"):
    import torch
    import torch.distributed as dist
    from flink_amd.exchange import KeyGroupExchange
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    ex = KeyGroupExchange(MAX_PAR, WORLD, rank, key_type=key_type)
    op = _operator(kind, key_type, ex.key_group_range)
    mx = -(1 << 63)
    dev = torch.device("cuda", 0)
    for s in range(STEPS):
        k, t, v, h = _slice(rank, s, key_type, kind)
        mx = max(mx, int(t.max()))
        cols = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (k, t, v)]
        hk = torch.from_numpy(h).to(dev) if h is not None else None
        got = ex.exchange(*cols, key_hash=hk)
        wm = ex.combine_watermark(mx - 300)
        op.process_batch(got[0], got[1], got[2], got[3] if hk is not None else None)
        op.watermark(wm)
    op.watermark((1 << 63) - 1)
    np.save(os.path.join(out_dir, f"rows_{rank}.npy"), op.rows())
    op.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("key_type", ["long", "int", "hashed"])
def test_gpu_exchange_world2_library_route(tmp_path, key_type):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(_free_port(), str(tmp_path), key_type), nprocs=WORLD, join=True)
    rows = np.concatenate([np.load(tmp_path / f"rows_{r}.npy") for r in range(WORLD)])
    # one operator over the whole stream, fed in the exchange's per-step source-major order, global watermarks
    if key_type == "hashed":
        return _check_hashed(rows)
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=1000)
    mx = [-(1 << 63)] * WORLD
    for s in range(STEPS):
        parts = [_slice(r, s, key_type) for r in range(WORLD)]
        for r in range(WORLD):
            mx[r] = max(mx[r], int(parts[r][1].max()))
        for src in range(WORLD):
            ref.process(*parts[src][:3])
        ref.watermark(min(m - 300 for m in mx))
    ref.watermark((1 << 63) - 1)
    _same(rows, ref.rows())


def _same(rows, r):
    key = lambda a: np.lexsort((a["start"], a["key"], a["epoch"]))  # noqa: E731
    a, b = rows[key(rows)], r[key(r)]
    assert len(a) == len(b) > 0
    for f in ("epoch", "key", "start", "end", "count", "sum", "min", "max"):
        np.testing.assert_array_equal(a[f], b[f])


def _check_hashed(rows):
    # String keys: per-word totals over the stream (the oracle keys by the dictionary id as a Long)
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=1000)
    mx = [-(1 << 63)] * WORLD
    for s in range(STEPS):
        parts = [_slice(r, s, "hashed") for r in range(WORLD)]
        for r in range(WORLD):
            mx[r] = max(mx[r], int(parts[r][1].max()))
        for src in range(WORLD):
            ref.process(*parts[src][:3])
        ref.watermark(min(m - 300 for m in mx))
    ref.watermark((1 << 63) - 1)
    _same(rows, ref.rows())


def test_gpu_native_keyby_world1():
    # the C-ABI exchange over the library's own RCCL communicator, one subtask: route, counts, self send/recv, push
    import torch
    from flink_amd import TumblingEventTimeWindows
    from flink_amd.exchange import NativeKeyByExchange
    from flink_amd.operator import GpuWindowOperator
    op = GpuWindowOperator(TumblingEventTimeWindows.of(1000), max_parallelism=MAX_PAR, device=0)
    ex = NativeKeyByExchange(op, 1, 0, NativeKeyByExchange.new_unique_id())
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=1000)
    mx = -(1 << 63)
    dev = torch.device("cuda", 0)
    for s in range(STEPS):
        k, t, v, _ = _slice(0, s, "long")
        mx = max(mx, int(t.max()))
        wm = ex.push(*(torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (k, t, v)), mx - 300)
        assert wm == mx - 300
        op.watermark(wm)
        ref.process(k, t, v)
        ref.watermark(mx - 300)
    op.watermark((1 << 63) - 1)
    ref.watermark((1 << 63) - 1)
    _same(op.rows(), ref.rows())
    ex.close()
    op.close()


@pytest.mark.parametrize("kind", ["sessions", "panes", "hll", "tdigest"])
def test_gpu_exchange_world2_operator_kinds(tmp_path, kind):
    """Sessions (gap 30 s, Zipf keys: MergingWindowSet merges per key on its owning subtask), panes (sliding
    60 s / 1 s), HyperLogLog and t-digest (delta 100; Zipf keys, BASELINE configs[4]) through the world-size-2
    exchange: the union of both subtasks' rows equals one oracle operator over the whole stream, fed each step's
    records in the exchange's source-major order as one batch (a t-digest compresses once per push), under the
    global watermarks.  t-digest rows (count, min / max, the p50 / p95 / p99 bits) are bit-exact."""
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(_free_port(), str(tmp_path), "long", kind), nprocs=WORLD, join=True)
    rows = np.concatenate([np.load(tmp_path / f"rows_{r}.npy") for r in range(WORLD)])
    ref = orc.WindowOperatorOracle(**KINDS[kind]["oracle"])
    mx = [-(1 << 63)] * WORLD
    for s in range(STEPS):
        parts = [_slice(r, s, "long", kind) for r in range(WORLD)]
        for r in range(WORLD):
            mx[r] = max(mx[r], int(parts[r][1].max()))
        ref.process(*(np.concatenate([p[i] for p in parts]) for i in range(3)))
        ref.watermark(min(m - 300 for m in mx))
    ref.watermark((1 << 63) - 1)
    r = ref.rows()
    if kind == "hll":  # registers, zero count and checksum bit-exact; the estimate's log within an ulp
        key = lambda a: np.lexsort((a["start"], a["key"], a["epoch"]))  # noqa: E731
        a, b = rows[key(rows)], r[key(r)]
        assert len(a) == len(b) > 0
        for f in ("epoch", "key", "start", "end", "count", "min", "max"):
            np.testing.assert_array_equal(a[f], b[f])
        np.testing.assert_allclose(a["sum"].view(np.float64), b["sum"].view(np.float64), rtol=1e-9)
    else:
        _same(rows, r)


def _native_worker(rank, port, out_dir):
    # one subtask per GPU: fw_keyby_push_device over the library's RCCL communicator.  Subtask 1 sends a quarter of
    # subtask 0's records, so it receives more than it sent (the receive columns grow).
    import torch
    import torch.distributed as dist
    from flink_amd import TumblingEventTimeWindows
    from flink_amd.exchange import KeyGroupExchange, NativeKeyByExchange
    from flink_amd.operator import GpuWindowOperator
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(rank)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    uid = [NativeKeyByExchange.new_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    kgr = KeyGroupExchange(MAX_PAR, WORLD, rank).key_group_range
    op = GpuWindowOperator(TumblingEventTimeWindows.of(1000), max_parallelism=MAX_PAR, key_group_range=kgr,
                           device=rank)
    ex = NativeKeyByExchange(op, WORLD, rank, uid[0])
    dev = torch.device("cuda", rank)
    mx = -(1 << 63)
    for s in range(STEPS):
        k, t, v = _native_slice(rank, s)
        mx = max(mx, int(t.max()))
        wm = ex.push(*(torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (k, t, v)), mx - 300)
        op.watermark(wm)
    op.watermark((1 << 63) - 1)
    np.save(os.path.join(out_dir, f"rows_{rank}.npy"), op.rows())
    ex.close()
    op.close()
    dist.destroy_process_group()


def _native_slice(rank, step):
    n = BATCH if rank == 0 else BATCH // 4
    first = step * 2 * BATCH + rank * BATCH
    return generate_host(0x5EED, first, n, KEYS, ts_base=0, rate=100_000, jitter=300)


def test_gpu_native_keyby_world2_skewed(tmp_path):
    """fw_keyby_push_device at world size 2 (per-peer ncclSend / ncclRecv offsets, the receive columns growing on
    the subtask that receives more than it sent): the union of both subtasks' rows equals one oracle operator.
    RCCL refuses two ranks on one device, so this needs two GPUs."""
    import torch
    if torch.cuda.device_count() < WORLD:
        pytest.skip("needs 2 GPUs (RCCL: one rank per device)")
    import torch.multiprocessing as mp
    mp.spawn(_native_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    rows = np.concatenate([np.load(tmp_path / f"rows_{r}.npy") for r in range(WORLD)])
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=1000)
    mx = [-(1 << 63)] * WORLD
    for s in range(STEPS):
        parts = [_native_slice(r, s) for r in range(WORLD)]
        for r in range(WORLD):
            mx[r] = max(mx[r], int(parts[r][1].max()))
        for src in range(WORLD):
            ref.process(*parts[src])
        ref.watermark(min(m - 300 for m in mx))
    ref.watermark((1 << 63) - 1)
    _same(rows, ref.rows())
