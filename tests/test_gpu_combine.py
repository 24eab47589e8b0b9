"""Pre-shuffle combining on the GPU: a combiner GpuWindowOperator aggregates each batch, is drained
into partial accumulators in key-group order (fw_combine_extract_device), and the receiving operator merges them
(fw_push_partials_device).  Rows must equal the oracle fed with the records themselves — bit-exact for keys,
windows, counts and integer sum/min/max, f64 sums within 1e-6 — and late partials count all of their records
(WindowOperator.java:402-418 with allowed lateness 0).

* world size 1: combiner -> partials -> operator on one GPU, including a table far too small (the merge suspends
  and resumes after growth) and keys outside the receiver's KeyGroupRange rejected;
* fw_keyby_combine_push_device (the C-ABI exchange over the library's RCCL communicator) at world size 1;
* world size 2 over gloo, both subtasks on cuda:0: CombiningExchange (combine, per-destination slices through
  all_to_all_single, merge), the union of both subtasks' rows against one oracle operator.
"""
import os
import socket

import numpy as np
import pytest

from flink_amd import KeyGroupRange, TumblingEventTimeWindows
from flink_amd.datagen import generate_host
from flink_amd.windowing import CountSumMinMax
from oracle import oracle as orc
from tests.parity_util import assert_rows_equal

pytestmark = pytest.mark.gpu

_VT = {"i64": "long", "i32": "int", "f64": "double"}


def _stream(n, batch, keys, bound, jitter, rate, value_type="i64"):
    k, t, v = generate_host(0x5EED, 0, n, keys, ts_base=1_000_000, rate=rate, jitter=jitter)
    if value_type == "f64":
        v = (v & 0xFFFFF).astype(np.float64) / 7.0
    out, mx = [], -(1 << 63)
    for b in range(0, n, batch):
        sl = slice(b, min(n, b + batch))
        mx = max(mx, int(t[sl].max()))
        out.append((k[sl], t[sl], v[sl], mx - bound))
    return out


def _ops(value_type, expected, kgr=None):
    from flink_amd.operator import GpuWindowOperator
    agg = CountSumMinMax(_VT[value_type])
    comb = GpuWindowOperator(TumblingEventTimeWindows.of(1000), agg, device=0, expected_entries=expected)
    op = GpuWindowOperator(TumblingEventTimeWindows.of(1000), agg, device=0, expected_entries=expected,
                           key_group_range=kgr)
    return comb, op


@pytest.mark.parametrize("value_type,keys,n,batch,expected", [
    ("i64", 2000, 600_000, 40_000, 0), ("i32", 2000, 600_000, 40_000, 0), ("f64", 2000, 600_000, 40_000, 0),
    ("i64", 1 << 20, 2 << 20, 1 << 20, 1000)], ids=["long", "int", "double", "table-grows"])
def test_gpu_combine_world1_vs_oracle(value_type, keys, n, batch, expected):
    import torch
    # out-of-order records (jitter 900 ms against a 300 ms bound): late windows arrive as late partials
    batches = _stream(n, batch, keys, bound=300, jitter=900, rate=200_000, value_type=value_type)
    comb, op = _ops(value_type, expected)
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=1000, value_type=value_type)
    rows = []
    sent = 0
    for k, t, v, wm in batches:
        cols = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (k, t, v)]
        comb.process_batch(*cols)
        parts, counts = comb.combine_extract(1)
        assert counts == [parts[0].numel()]
        sent += parts[0].numel()
        op.push_partials(*(c.clone() for c in parts), config=parts.config)
        ref.process(k, t, v)
        rows.append(op.process_watermark(wm))
        ref.watermark(wm)
    rows.append(op.process_watermark((1 << 63) - 1))
    ref.watermark((1 << 63) - 1)
    assert_rows_equal(np.concatenate(rows), ref.rows(), _VT[value_type])
    assert op.late_dropped == ref.late_dropped
    assert op.stats()["records_in"] == n  # numRecordsIn counts the records inside the partials
    if expected:
        assert op.stats()["table_grows"] >= 1
    else:
        assert ref.late_dropped > 0
        assert sent < n // 4  # one partial per (key, window) of a batch instead of one per record
    comb.close()
    op.close()


@pytest.mark.parametrize("value_type", ["i64", "f64"])
def test_gpu_combine_panes_world1_vs_oracle(value_type):
    # sliding windows kept as panes (size % slide == 0, no lateness): the combiner's partials are (key, pane)
    # accumulators, a pane's partial is late exactly when its elements are (they share the pane's newest window),
    # and the receiver merges them into its panes; rows vs the oracle fed the records (60 s / 1 s shape scaled down)
    import torch
    from flink_amd import SlidingEventTimeWindows
    from flink_amd.operator import GpuWindowOperator
    batches = _stream(400_000, 40_000, 2000, bound=300, jitter=9000, rate=100_000, value_type=value_type)
    agg = CountSumMinMax(_VT[value_type])
    comb = GpuWindowOperator(SlidingEventTimeWindows.of(6000, 1000), agg, device=0)
    op = GpuWindowOperator(SlidingEventTimeWindows.of(6000, 1000), agg, device=0)
    ref = orc.WindowOperatorOracle(assigner="sliding", size=6000, slide=1000, value_type=value_type)
    rows, sent, n = [], 0, 0
    for k, t, v, wm in batches:
        cols = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (k, t, v)]
        comb.process_batch(*cols)
        parts, _ = comb.combine_extract(1)
        sent += parts[0].numel()
        n += len(k)
        op.push_partials(*(c.clone() for c in parts), config=parts.config)
        ref.process(k, t, v)
        rows.append(op.process_watermark(wm))
        ref.watermark(wm)
    rows.append(op.process_watermark((1 << 63) - 1))
    ref.watermark((1 << 63) - 1)
    assert_rows_equal(np.concatenate(rows), ref.rows(), _VT[value_type])
    assert op.late_dropped == ref.late_dropped > 0
    assert op.stats()["records_in"] == n
    assert sent < n // 2  # (a batch spans the 9 s of jitter: about ten panes per key)
    comb.close()
    op.close()


def _hll_rows_equal(g, r):
    ks = lambda a: a[np.lexsort((a["start"], a["key"], a["epoch"]))]  # noqa: E731
    g, r = ks(g), ks(r)
    assert len(g) == len(r) > 0
    for f in ("epoch", "key", "start", "end", "count", "min", "max"):
        assert np.array_equal(g[f], r[f]), f
    np.testing.assert_allclose(g["sum"].view(np.float64), r["sum"].view(np.float64), rtol=1e-9)


@pytest.mark.parametrize("zipf,p", [(1.1, 12), (None, 6)], ids=["zipf-p12", "uniform-p6"])
def test_gpu_combine_hll_world1_vs_oracle(zipf, p):
    # HyperLogLog combines before the shuffle -- a combined window is its count and its non-zero
    # registers, the receiver takes the register max (AggregateFunction.merge, AggregateFunction.java:160); rows
    # (count, zero registers, the register checksum, the estimate) equal the oracle fed the records; late partials
    # count their records
    import torch
    from flink_amd import HyperLogLog
    from flink_amd.operator import GpuWindowOperator
    k, t, v = generate_host(0x5EED, 0, 400_000, 3000, ts_base=1_000_000, rate=200_000, jitter=900, zipf_s=zipf)
    comb = GpuWindowOperator(TumblingEventTimeWindows.of(1000), HyperLogLog(p), device=0, expected_entries=8000)
    op = GpuWindowOperator(TumblingEventTimeWindows.of(1000), HyperLogLog(p), device=0, expected_entries=8000)
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=1000, hll_p=p)
    rows, sent, regs_sent, mx = [], 0, 0, -(1 << 63)
    for b in range(0, len(k), 40_000):
        sl = slice(b, b + 40_000)
        mx = max(mx, int(t[sl].max()))
        comb.process_batch(*(torch.from_numpy(np.ascontiguousarray(x[sl])).cuda() for x in (k, t, v)))
        cols, counts, regs, rcounts = comb.combine_extract_hll(1)
        assert counts == [cols[0].numel()] and rcounts == [regs.numel()] == [int(cols[3].sum())]
        sent += cols[0].numel()
        regs_sent += regs.numel()
        op.push_hll_partials(*(c.clone() for c in cols), regs=regs.clone(), config=cols.config)
        ref.process(k[sl], t[sl], v[sl])
        rows.append(op.process_watermark(mx - 300))
        ref.watermark(mx - 300)
    rows.append(op.process_watermark((1 << 63) - 1))
    ref.watermark((1 << 63) - 1)
    _hll_rows_equal(np.concatenate(rows), ref.rows())
    assert op.late_dropped == ref.late_dropped > 0
    assert op.stats()["records_in"] == len(k)
    assert sent < len(k) // 4 and regs_sent <= len(k)  # a register per distinct item at most
    comb.close()
    op.close()


def test_gpu_combine_rejects_foreign_key_groups_and_ineligible_configs():
    import torch
    from flink_amd import _native as N
    from flink_amd import SlidingEventTimeWindows
    from flink_amd.operator import GpuWindowOperator
    comb, op = _ops("i64", 0, kgr=KeyGroupRange(0, 63))
    k = torch.arange(1000, dtype=torch.int64, device="cuda")
    comb.process_batch(k, k + 1_000_000, k)
    parts, _ = comb.combine_extract(1)
    op.push_partials(*(c.clone() for c in parts), config=parts.config)
    with pytest.raises(N.NativeError):  # keys of key groups 64..127 reach a subtask owning 0..63
        op.process_watermark(0)
    bad = GpuWindowOperator(SlidingEventTimeWindows.of(2500, 1000), device=0)  # (no panes: size % slide != 0)
    with pytest.raises(N.NativeError):
        bad.combine_extract(1)
    for o in (comb, op, bad):
        o.close()


MAX_PAR, WORLD, BATCH, STEPS, KEYS = 128, 2, 40_000, 5, 3000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _slice(rank, step):
    first = (step * WORLD + rank) * BATCH
    return generate_host(0x5EED, first, BATCH, KEYS, ts_base=0, rate=100_000, jitter=300)


def _assigner(kind):
    from flink_amd import SlidingEventTimeWindows
    return SlidingEventTimeWindows.of(5000, 1000) if kind == "panes" else TumblingEventTimeWindows.of(1000)


def _worker(rank, port, out_dir, kind="tumbling"):
    import torch
    import torch.distributed as dist
    from flink_amd import HyperLogLog
    from flink_amd.exchange import CombiningExchange, KeyGroupExchange
    from flink_amd.operator import GpuWindowOperator
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    ex = KeyGroupExchange(MAX_PAR, WORLD, rank)
    agg = HyperLogLog(10) if kind == "hll" else CountSumMinMax()
    op = GpuWindowOperator(_assigner(kind), agg, max_parallelism=MAX_PAR, key_group_range=ex.key_group_range, device=0)
    comb = GpuWindowOperator(_assigner(kind), agg, max_parallelism=MAX_PAR, device=0)
    cx = CombiningExchange(ex, comb)
    mx = -(1 << 63)
    dev = torch.device("cuda", 0)
    for s in range(STEPS):
        k, t, v = _slice(rank, s)
        mx = max(mx, int(t.max()))
        cols = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (k, t, v)]
        wm = cx.push(op, *cols, mx - 300)
        op.watermark(wm)
    op.watermark((1 << 63) - 1)
    np.save(os.path.join(out_dir, f"rows_{rank}.npy"), op.rows())
    np.save(os.path.join(out_dir, f"sent_{rank}.npy"), np.array([cx.partials_sent, op.late_dropped]))
    comb.close()
    op.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["tumbling", "panes", "hll"])
def test_gpu_combining_exchange_world2(kind):
    import tempfile

    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(_free_port(), d, kind), nprocs=WORLD, join=True)
        rows = np.concatenate([np.load(os.path.join(d, f"rows_{r}.npy")) for r in range(WORLD)])
        sent = [np.load(os.path.join(d, f"sent_{r}.npy")) for r in range(WORLD)]
    ref = (orc.WindowOperatorOracle(assigner="sliding", size=5000, slide=1000) if kind == "panes"
           else orc.WindowOperatorOracle(assigner="tumbling", size=1000, hll_p=10 if kind == "hll" else 0))
    mx = [-(1 << 63)] * WORLD
    for s in range(STEPS):
        sl = [_slice(r, s) for r in range(WORLD)]
        for r in range(WORLD):
            ref.process(*sl[r])
            mx[r] = max(mx[r], int(sl[r][1].max()))
        ref.watermark(min(mx) - 300)
    ref.watermark((1 << 63) - 1)
    if kind == "hll":
        _hll_rows_equal(rows, ref.rows())
    else:
        assert_rows_equal(rows, ref.rows())
    assert sum(int(x[1]) for x in sent) == ref.late_dropped
    assert 0 < sum(int(x[0]) for x in sent) < WORLD * STEPS * BATCH // 4


@pytest.mark.parametrize("hll", [False, True], ids=["count_sum", "hll"])
def test_gpu_native_keyby_combine_world1(hll):
    # the C-ABI combining exchange over the library's own RCCL communicator, one subtask: combiner push, drain,
    # counts, self send/recv of the partials (and, for HyperLogLog, of their registers), merge
    import torch
    from flink_amd import HyperLogLog
    from flink_amd.exchange import NativeKeyByExchange
    from flink_amd.operator import GpuWindowOperator
    agg = HyperLogLog(10) if hll else CountSumMinMax()
    op = GpuWindowOperator(TumblingEventTimeWindows.of(1000), agg, max_parallelism=MAX_PAR, device=0)
    comb = GpuWindowOperator(TumblingEventTimeWindows.of(1000), agg, max_parallelism=MAX_PAR, device=0)
    ex = NativeKeyByExchange(op, 1, 0, NativeKeyByExchange.new_unique_id())
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=1000, hll_p=10 if hll else 0)
    mx = -(1 << 63)
    dev = torch.device("cuda", 0)
    for s in range(2 * STEPS):
        k, t, v = _slice(0, s)
        mx = max(mx, int(t.max()))
        wm = ex.push_combined(comb, *(torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (k, t, v)), mx - 300)
        assert wm == mx - 300
        op.watermark(wm)
        ref.process(k, t, v)
        ref.watermark(mx - 300)
    op.watermark((1 << 63) - 1)
    ref.watermark((1 << 63) - 1)
    if hll:
        _hll_rows_equal(op.rows(), ref.rows())
        assert ex.stats()["batches"] == 2 * STEPS
    else:
        assert_rows_equal(op.rows(), ref.rows())
    assert op.late_dropped == ref.late_dropped
    ex.close()
    comb.close()
    op.close()


@pytest.mark.parametrize("what", ["size", "value_type"])
def test_gpu_combine_rejects_mismatched_combiner(what):
    """Partials carry their combiner's configuration tag: a receiver with another window size (its window starts
    would be re-bucketed) or value type (f64 min/max are kept in sortable form) refuses them instead of misreading."""
    import torch
    from flink_amd import _native as N
    from flink_amd import TumblingEventTimeWindows
    from flink_amd.operator import GpuWindowOperator
    comb = GpuWindowOperator(TumblingEventTimeWindows.of(1000), device=0)
    op = GpuWindowOperator(TumblingEventTimeWindows.of(2000 if what == "size" else 1000),
                           CountSumMinMax(_VT["f64" if what == "value_type" else "i64"]), device=0)
    k = torch.arange(1000, dtype=torch.int64, device="cuda")
    comb.process_batch(k, k + 1_000_000, k)
    parts, _ = comb.combine_extract(1)
    with pytest.raises(N.NativeError, match="configured differently"):
        op.push_partials(*(c.clone() for c in parts), config=parts.config)
    for o in (comb, op):
        o.close()
