"""BASELINE configs[2] as sharded as one GPU allows: sliding 60 s / 1 s event-time windows over 16M keys, key-group
sharded over 8 subtasks (world size 8 over gloo, all on cuda:0).  Subtask r owns
computeKeyGroupRangeForOperatorIndex(128, 8, r) = 16 key groups (KeyGroupRangeAssignment.java:85-117); each
subtask's slice of the global stream goes through the library's fw_route_device and the all-to-all exchange
(RecordWriter.emit -> KeyGroupStreamPartitioner.selectChannels, RecordWriter.java:88-115), and the watermark is
the minimum over the subtasks (StatusWatermarkValve.java:173-191).  The 8-GPU RCCL transport is the driver's
(bench.py --gpus 8); this covers G = 8 key-group ranges and configs[2]'s key count.

* full size: 2^24 records per subtask and step (2^27 per step in all), 16M uniform keys, two steps, then the final
  watermark fires every window.  Size-independent properties: every record counted in exactly 60 windows, sums
  likewise, one row per (key, window), each subtask's rows only from its own key groups, no late record;
* reduced size: the same topology against one oracle operator over the whole stream, row for row.
"""
import json
import os
import socket

import numpy as np
import pytest

from flink_amd.datagen import generate_host
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

MAX_PAR, WORLD = 128, 8
SEED = 0xC3C3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, port):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)


def _full_worker(rank, port, out_dir, n, steps, keys):
    import torch
    import torch.distributed as dist
    from flink_amd import SlidingEventTimeWindows
    from flink_amd.datagen import generate_device
    from flink_amd.exchange import KeyGroupExchange
    from flink_amd.operator import GpuWindowOperator
    _init(rank, port)
    ex = KeyGroupExchange(MAX_PAR, WORLD, rank)
    kgr = ex.key_group_range
    assert kgr.get_number_of_key_groups() == MAX_PAR // WORLD
    op = GpuWindowOperator(SlidingEventTimeWindows.of(60_000, 1000), max_parallelism=MAX_PAR, key_group_range=kgr,
                           device=0)
    dev = torch.device("cuda", 0)
    vsum = torch.zeros((), dtype=torch.int64, device=dev)
    got_cnt = torch.zeros((), dtype=torch.int64, device=dev)
    got_sum = torch.zeros((), dtype=torch.int64, device=dev)
    codes, kg_bad, received, mx = [], 0, 0, -(1 << 63)

    def drain():
        nonlocal got_cnt, got_sum, kg_bad
        r = op.drain_rows_torch(("key", "start", "end", "count", "sum"))
        if r["key"].numel() == 0:
            return
        assert bool(((r["end"] - r["start"]) == 60_000).all()) and bool((r["start"] % 1000 == 0).all())
        got_cnt += r["count"].sum()
        got_sum += r["sum"].sum()
        kg = torch.empty(r["key"].numel(), dtype=torch.int32, device=dev)
        from flink_amd import _native as N
        N.check(N.lib().fw_key_groups_device(r["key"].data_ptr(), None, N.FW_KEY_LONG, r["key"].numel(), MAX_PAR,
                                             kg.data_ptr(), None))
        torch.cuda.synchronize()
        kg_bad += int(((kg < kgr.start_key_group) | (kg > kgr.end_key_group)).sum())
        # (key, window start) as one word: keys < 2^24, starts within 2^20 s of the base
        codes.append((r["key"] << 20) | ((r["start"] - 900_000) // 1000))

    for s in range(steps):
        k, t, v, m = generate_device(SEED, (s * WORLD + rank) * n, n, keys, ts_base=1_000_000, rate=100_000_000,
                                     jitter=200)
        vsum += v.sum()
        mx = max(mx, int(m.item()))
        kk, tt, vv = ex.exchange(k, t, v)
        received += kk.numel()
        op.process_batch(kk, tt, vv)
        op.advance_watermark(ex.combine_watermark(mx - 200))
        drain()
    op.advance_watermark((1 << 63) - 1)
    drain()
    allc = torch.cat(codes)
    rows = allc.numel()
    distinct = torch.unique(allc).numel()
    res = dict(rank=rank, received=received, vsum=int(vsum), cnt=int(got_cnt), sum=int(got_sum), rows=rows,
               distinct=distinct, kg_bad=kg_bad, late=op.late_dropped)
    op.close()
    with open(os.path.join(out_dir, f"res_{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


def test_gpu_c3_world8_full_size_properties(tmp_path):
    import torch.multiprocessing as mp
    n, steps, keys = 1 << 24, 2, 16_000_000
    mp.spawn(_full_worker, args=(_free_port(), str(tmp_path), n, steps, keys), nprocs=WORLD, join=True)
    res = [json.load(open(tmp_path / f"res_{r}.json")) for r in range(WORLD)]
    total = WORLD * steps * n
    assert sum(r["received"] for r in res) == total  # nothing lost or duplicated in the exchange
    assert all(r["late"] == 0 and r["kg_bad"] == 0 for r in res), res
    assert all(r["rows"] == r["distinct"] for r in res), res  # one row per (key, window) on its subtask
    assert sum(r["cnt"] for r in res) == 60 * total  # every record in exactly 60 sliding windows
    wrap = lambda x: (x + (1 << 63)) % (1 << 64) - (1 << 63)  # noqa: E731  (Long sums wrap)
    assert wrap(sum(r["sum"] for r in res)) == wrap(60 * sum(r["vsum"] for r in res))
    assert all(r["received"] > 0 and r["rows"] > 0 for r in res)


def _small_slice(rank, step, n, keys):
    return generate_host(SEED, (step * WORLD + rank) * n, n, keys, ts_base=1_000_000, rate=100_000, jitter=300)


def _small_worker(rank, port, out_dir, n, steps, keys):
    import torch
    import torch.distributed as dist
    from flink_amd import SlidingEventTimeWindows
    from flink_amd.exchange import KeyGroupExchange
    from flink_amd.operator import GpuWindowOperator
    _init(rank, port)
    ex = KeyGroupExchange(MAX_PAR, WORLD, rank)
    op = GpuWindowOperator(SlidingEventTimeWindows.of(60_000, 1000), max_parallelism=MAX_PAR,
                           key_group_range=ex.key_group_range, device=0)
    dev = torch.device("cuda", 0)
    mx = -(1 << 63)
    for s in range(steps):
        k, t, v = _small_slice(rank, s, n, keys)
        mx = max(mx, int(t.max()))
        cols = ex.exchange(*(torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (k, t, v)))
        op.process_batch(*cols)
        op.watermark(ex.combine_watermark(mx - 300))
    op.watermark((1 << 63) - 1)
    np.save(os.path.join(out_dir, f"rows_{rank}.npy"), op.rows())
    op.close()
    dist.destroy_process_group()


def test_gpu_c3_world8_vs_oracle(tmp_path):
    import torch.multiprocessing as mp
    from flink_amd.keygroups import (assign_to_key_group, compute_key_group_range_for_operator_index,
                                     long_hash_code)
    n, steps, keys = 8_000, 4, 5_000
    mp.spawn(_small_worker, args=(_free_port(), str(tmp_path), n, steps, keys), nprocs=WORLD, join=True)
    per = [np.load(tmp_path / f"rows_{r}.npy") for r in range(WORLD)]
    for r, rows in enumerate(per):  # a subtask emits only its own key groups
        kgr = compute_key_group_range_for_operator_index(MAX_PAR, WORLD, r)
        assert all(kgr.contains(assign_to_key_group(long_hash_code(int(k)), MAX_PAR)) for k in np.unique(rows["key"]))
    rows = np.concatenate(per)
    ref = orc.WindowOperatorOracle(assigner="sliding", size=60_000, slide=1000)
    mx = [-(1 << 63)] * WORLD
    for s in range(steps):
        parts = [_small_slice(r, s, n, keys) for r in range(WORLD)]
        for r in range(WORLD):
            mx[r] = max(mx[r], int(parts[r][1].max()))
        ref.process(*(np.concatenate([p[i] for p in parts]) for i in range(3)))
        ref.watermark(min(m - 300 for m in mx))
    ref.watermark((1 << 63) - 1)
    r = ref.rows()
    key = lambda a: np.lexsort((a["start"], a["key"], a["epoch"]))  # noqa: E731
    a, b = rows[key(rows)], r[key(r)]
    assert len(a) == len(b) > 0
    for f in ("epoch", "key", "start", "end", "count", "sum", "min", "max"):
        np.testing.assert_array_equal(a[f], b[f])
