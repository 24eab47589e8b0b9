"""Keyed-state snapshot / restore of the aggregates whose accumulator lives in a pool block (HyperLogLog registers,
t-digest centroids): fw_snapshot_key_group_blocks / fw_restore_key_group_blocks.

The heap backend writes an AggregatingState's accumulator per (key, window) mapping through the accumulator
serializer (HeapAggregatingState.java:73-93, HeapKeyedStateBackend.java:370-381); here the accumulator is the
block beside the row (include/flink_window.h).  A run cut by a snapshot and restored over a different parallelism
must fire exactly the rows (and, for the t-digest, the centroids bit for bit) of an uninterrupted run — the
oracle's (oracle/window_oracle.h OR_AGG_HLL / OR_AGG_TDIGEST, pinned by test_oracle_hll / test_oracle_tdigest)."""
import ctypes

import numpy as np
import pytest

from flink_amd import HyperLogLog, TDigest, TumblingEventTimeWindows
from flink_amd.datagen import generate_host
from flink_amd.keygroups import (assign_to_key_group, compute_key_group_range_for_operator_index, long_hash_code)
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
MAXP = 128


def _stream(n, batch, num_keys, rate, f64=False, zipf=None, bound=200, jitter=200, seed=0x51A7):
    keys, ts, raw = generate_host(seed, 0, n, num_keys, ts_base=1_000_000, rate=rate, jitter=jitter, zipf_s=zipf)
    vals = ((raw & 0xFFFFFF).astype(np.float64) / 7.0 - 1.0e6) if f64 else raw
    batches, wms, mx = [], [], -(1 << 63)
    for b in range(0, n, batch):
        sl = slice(b, min(n, b + batch))
        batches.append((keys[sl], ts[sl], vals[sl]))
        mx = max(mx, int(ts[sl].max()))
        wms.append(mx - bound)
    batches.append((keys[:0], ts[:0], vals[:0]))
    wms.append((1 << 63) - 1)
    return batches, wms


def _fire(op, wm, epoch, digests):
    op.advance_watermark(wm)
    d = op.drain_digests() if digests else []
    r = op.drain_rows(epoch)
    return r, d


def _cut_and_rescale(agg_factory, batches, wms, new_par, digests, expected_entries):
    """Runs the first half on one operator over all key groups, snapshots every key group, restores the snapshot
    onto new_par operators (one KeyGroupRange each) and feeds them the rest; returns the rows (and digests)."""
    from flink_amd.operator import GpuWindowOperator
    cut = len(batches) // 2
    a = GpuWindowOperator(TumblingEventTimeWindows.of(1000), agg_factory(), max_parallelism=MAXP,
                          expected_entries=expected_entries)
    rows, digs = [], []
    for e, ((k, t, v), wm) in enumerate(zip(batches[:cut], wms[:cut])):
        if len(k):
            a.process(k, t, v)
        r, d = _fire(a, wm, e, digests)
        rows.append(r)
        digs += d
    entries = a.num_keyed_state_entries
    snap = a.snapshot_state()
    assert sum(len(r) for r in snap.values()) == entries > 0
    bb = next(len(r["acc"][0]) for r in snap.values() if len(r))
    a.close()
    parts = []
    for idx in range(new_par):
        kgr = compute_key_group_range_for_operator_index(MAXP, new_par, idx)
        op = GpuWindowOperator(TumblingEventTimeWindows.of(1000), agg_factory(), max_parallelism=MAXP,
                               key_group_range=kgr, expected_entries=expected_entries)
        op.initialize_state(snap)
        parts.append((kgr, op))
    assert sum(op.num_keyed_state_entries for _, op in parts) == entries
    for e, ((k, t, v), wm) in enumerate(zip(batches[cut:], wms[cut:]), start=cut):
        kg = np.array([assign_to_key_group(long_hash_code(int(x)), MAXP) for x in k], dtype=np.int64)
        for kgr, op in parts:
            m = (kg >= kgr.start_key_group) & (kg <= kgr.end_key_group)
            if m.any():
                op.process(k[m], t[m], v[m])
            r, d = _fire(op, wm, e, digests)
            rows.append(r)
            digs += d
    for _, op in parts:
        op.close()
    return np.concatenate(rows), digs, bb


def _oracle(batches, wms, **cfg):
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=1000, **cfg)
    for (k, t, v), wm in zip(batches, wms):
        if len(k):
            ref.process(k, t, v)
        ref.watermark(wm)
    return ref


def _order(a):
    return np.lexsort((a["start"], a["key"], a["epoch"]))


@pytest.mark.parametrize("p,new_par", [(14, 2), (6, 3)])
def test_gpu_hll_snapshot_restore_rescale(p, new_par):
    batches, wms = _stream(240_000, 30_000, 8_000, rate=200_000, zipf=1.1)
    got, _, bb = _cut_and_rescale(lambda: HyperLogLog(p), batches, wms, new_par, False, 40_000)
    assert bb == 1 << p
    exp = _oracle(batches, wms, hll_p=p).rows()
    g, r = got[_order(got)], exp[_order(exp)]
    assert len(g) == len(r) > 0
    for f in ("epoch", "key", "start", "end", "count", "min", "max"):
        assert np.array_equal(g[f], r[f]), f
    np.testing.assert_allclose(g["sum"].view(np.float64), r["sum"].view(np.float64), rtol=1e-9)


def test_gpu_hll_restore_merges_registers():
    # the same snapshot restored twice into one handle: the windows merge (AggregateFunction.merge: register max,
    # counts added), so every estimate equals the single restore's and every count doubles
    from flink_amd.operator import GpuWindowOperator
    batches, wms = _stream(60_000, 30_000, 2_000, rate=100_000, zipf=1.1)
    a = GpuWindowOperator(TumblingEventTimeWindows.of(1000), HyperLogLog(10), expected_entries=20_000)
    a.process(*batches[0])
    snap = a.snapshot_state()
    a.close()
    regs = np.concatenate([r["acc"] for r in snap.values() if len(r)])
    assert regs.max() > 0 and regs.max() <= 65 - 10
    out = []
    for times in (1, 2):
        op = GpuWindowOperator(TumblingEventTimeWindows.of(1000), HyperLogLog(10), expected_entries=20_000)
        for _ in range(times):
            op.initialize_state(snap)
        op.watermark((1 << 63) - 1)
        out.append(op.rows()[_order(op.rows())])
        assert op.stats()["keyed_state_entries"] == 0
        op.close()
    one, two = out
    assert len(one) == len(two) > 0
    for f in ("key", "start", "sum", "min", "max"):
        assert np.array_equal(one[f], two[f]), f
    assert np.array_equal(two["count"], 2 * one["count"])


@pytest.mark.parametrize("delta,new_par", [(100, 2), (30, 3)])
def test_gpu_tdigest_snapshot_restore_rescale(delta, new_par):
    # bit-exact centroids across the cut: the restored digests continue exactly as the uninterrupted ones
    batches, wms = _stream(240_000, 40_000, 3_000, rate=100_000, f64=True, zipf=1.1)
    q = (0.5, 0.95, 0.99)
    got, digs, bb = _cut_and_rescale(lambda: TDigest(delta, q, export=True), batches, wms, new_par, True, 20_000)
    assert bb == 8 * (1 + 2 * (delta // 2))
    ref = _oracle(batches, wms, tdigest=delta, quantiles=q)
    exp = ref.rows()
    rdig = [ref.digest(i) for i in range(len(exp))]
    go, ro = _order(got), _order(exp)
    assert len(got) == len(exp) > 0
    for f in ("epoch", "key", "start", "end", "count", "sum", "min", "max"):
        assert np.array_equal(got[f][go], exp[f][ro]), f
    for a, b in zip(go, ro):
        (gs, gw), (rs, rw) = digs[a], rdig[b]
        assert np.array_equal(gw, rw)
        assert np.array_equal(gs.view(np.int64), rs.view(np.int64))


def test_gpu_tdigest_snapshot_block_layout_and_refusals():
    from flink_amd import _native as N
    from flink_amd.operator import GpuWindowOperator
    batches, wms = _stream(20_000, 20_000, 500, rate=100_000, f64=True)
    a = GpuWindowOperator(TumblingEventTimeWindows.of(1000), TDigest(20, export=True), expected_entries=4000)
    a.process(*batches[0])
    snap = {kg: r for kg, r in a.snapshot_state().items() if len(r)}
    # the plain row calls refuse a pool aggregate (its accumulator is not in fw_state_rows)
    n = ctypes.c_int64()
    assert N.lib().fw_snapshot_key_group(a._h, 0, None, 0, ctypes.byref(n)) == N.FW_ERR_UNSUPPORTED
    a.close()
    rows = np.concatenate(list(snap.values()))
    w = rows["acc"].view(np.int64)  # n, then (sum bits, weight) per centroid, zero-padded
    assert np.all((w[:, 0] >= 1) & (w[:, 0] <= 10))
    for i in range(len(rows)):
        c = int(w[i, 0])
        assert w[i, 2:2 + 2 * c:2].sum() == rows["count"][i]
        assert not w[i, 1 + 2 * c:].any()
    kg, part = next(iter(snap.items()))
    op = GpuWindowOperator(TumblingEventTimeWindows.of(1000), TDigest(20), expected_entries=4000)
    op.restore_key_group(kg, part)
    with pytest.raises(N.NativeError) as e:  # a digest already present is not re-compressed
        op.restore_key_group(kg, part[:1])
    assert e.value.code == N.FW_ERR_STATE
    bad = part[:1].copy()
    bad["acc"].view(np.int64)[0, 0] = 11  # more centroids than delta / 2
    op2 = GpuWindowOperator(TumblingEventTimeWindows.of(1000), TDigest(20), expected_entries=4000)
    with pytest.raises(N.NativeError) as e:
        op2.restore_key_group(kg, bad)
    assert e.value.code == N.FW_ERR_STATE
    # the refused row changed nothing: the key group restores whole afterwards
    op2.restore_key_group(kg, part)
    assert op2.num_keyed_state_entries == len(part)
    with pytest.raises(ValueError):
        op2.restore_key_group(kg, np.zeros(1, dtype=np.dtype([(f, "<i8") for f in ("key", "start", "end", "count",
                                                                                   "sum", "min", "max", "timer")])))
    op.close()
    op2.close()
