"""GPU t-digest (FW_AGG_TDIGEST, BASELINE configs[4] / SURVEY §8d C5) against the oracle's restatement
(oracle/window_oracle.h OR_AGG_TDIGEST, itself pinned by tests/test_oracle_tdigest.py).

The bar is bit-exact: every fired row's centroids (sum bits and weights, via TDigest(export=True)) and its
three quantile estimates equal the oracle's, for digests merged serially and for the hot ones merged
bucket-parallel (more than FW_TD_T3 = 2048 values + centroids in one push); over tumbling, sliding and session
windows (merged sessions' digests: the centroid union), and under allowed lateness (late firings: the digest with
the push's values so far).  At the full C5 batch size
(2^24 records per push, generated in HBM) the checks are size-independent: every record is counted once and
the quantiles of the hottest keys lie within 1% in rank of the exact ones.
"""
import numpy as np
import pytest

from flink_amd import TDigest, TumblingEventTimeWindows
from flink_amd.datagen import generate_host
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _stream(n, batch, num_keys, rate, zipf=None, values="spread", seed=0x7D16, bound=200, jitter=200):
    keys, ts, raw = generate_host(seed, 0, n, num_keys, ts_base=1_000_000, rate=rate, jitter=jitter, zipf_s=zipf)
    if values == "spread":
        vals = (raw & 0xFFFFFF).astype(np.float64) / 7.0 - 1.0e6  # distinct-ish, negative and positive
    elif values == "lowbits":
        # 16 bases of both signs whose values differ only in their 10 lowest mantissa bits: they tie in the
        # sort key's high bits and are ordered by its low bits (k_td_fix_*; long runs in the hot digests)
        base = np.array([-1.0e6, -3.5, -0.75, -1e-3, 0.0, 1e-3, 0.625, 2.25, 9.0, 1e2, 3.3e3, 7e5, 1e6, -7e5, 4e9, -4e9])
        bits = base.view(np.int64)[(raw >> 12) & 15] ^ (raw & 0x3FF)
        vals = bits.view(np.float64)
    else:
        vals = (raw & 0x3F).astype(np.float64) * 0.5  # 64 distinct values: ties with each other and with means
    batches, wms, mx = [], [], -(1 << 63)
    for b in range(0, n, batch):
        sl = slice(b, min(n, b + batch))
        batches.append((keys[sl], ts[sl], vals[sl]))
        mx = max(mx, int(ts[sl].max()))
        wms.append(mx - bound)
    batches.append((keys[:0], ts[:0], vals[:0]))
    wms.append((1 << 63) - 1)
    return batches, wms


def _run(batches, wms, delta, quantiles=(0.5, 0.95, 0.99), sliding=None, gap=None, lateness=0, purging=False, **kw):
    from flink_amd import EventTimeSessionWindows, EventTimeTrigger, PurgingTrigger, SlidingEventTimeWindows
    from flink_amd.operator import GpuWindowOperator
    assigner = (SlidingEventTimeWindows.of(*sliding) if sliding else EventTimeSessionWindows.with_gap(gap) if gap
                else TumblingEventTimeWindows.of(1000))
    if purging:
        kw["trigger"] = PurgingTrigger.of(EventTimeTrigger.create())
    gpu = GpuWindowOperator(assigner, TDigest(delta, quantiles, export=True), allowed_lateness=lateness, **kw)
    ref = (orc.WindowOperatorOracle(assigner="sliding", size=sliding[0], slide=sliding[1], tdigest=delta,
                                    quantiles=quantiles, lateness=lateness, purging=purging) if sliding else
           orc.WindowOperatorOracle(assigner="session", gap=gap, tdigest=delta, quantiles=quantiles,
                                    lateness=lateness, purging=purging) if gap else
           orc.WindowOperatorOracle(assigner="tumbling", size=1000, tdigest=delta, quantiles=quantiles,
                                    lateness=lateness, purging=purging))
    g_rows, g_dig = [], []
    for epoch, ((k, t, v), wm) in enumerate(zip(batches, wms)):
        if len(k):
            gpu.process(k, t, v)
            ref.process(k, t, v)
        gpu.advance_watermark(wm)
        g_dig += gpu.drain_digests()
        g_rows.append(gpu.drain_rows(epoch))
        ref.watermark(wm)
    assert gpu.late_dropped == ref.late_dropped
    gpu.close()
    r_rows = ref.rows()
    r_dig = [ref.digest(i) for i in range(len(r_rows))]
    return np.concatenate(g_rows), g_dig, r_rows, r_dig


def _assert_same(g_rows, g_dig, r_rows, r_dig, delta):
    assert len(g_rows) == len(r_rows) > 0
    go = np.lexsort((g_rows["start"], g_rows["key"], g_rows["epoch"]))
    ro = np.lexsort((r_rows["start"], r_rows["key"], r_rows["epoch"]))
    for f in ("epoch", "key", "start", "end", "count", "sum", "min", "max"):  # quantiles as f64 bits
        bad = np.nonzero(g_rows[f][go] != r_rows[f][ro])[0]
        assert bad.size == 0, f"{f} differs at {bad[:5]}: {g_rows[go][bad[:3]]} vs {r_rows[ro][bad[:3]]}"
    for a, b in zip(go, ro):
        gs, gw = g_dig[a]
        rs, rw = r_dig[b]
        assert len(gs) == len(rs) <= delta // 2
        assert np.array_equal(gw, rw), (gw, rw)
        assert np.array_equal(gs.view(np.int64), rs.view(np.int64)), (gs, rs)
        assert int(gw.sum()) == g_rows["count"][a]


@pytest.mark.parametrize("delta", [100, 20])
@pytest.mark.parametrize("values", ["spread", "lowbits"])
def test_gpu_tdigest_serial_digests(delta, values):
    # uniform keys: every digest gets a few values per push (the serial merge)
    batches, wms = _stream(300_000, 60_000, 20_000, rate=200_000, values=values)
    out = _run(batches, wms, delta, expected_entries=60_000)
    _assert_same(*out, delta)


@pytest.mark.parametrize("delta,values", [(100, "spread"), (100, "ties"), (30, "spread"), (100, "lowbits")])
def test_gpu_tdigest_hot_digests(delta, values):
    # Zipf(1.1) over 1000 keys in 200K-record pushes: the hottest digests take tens of thousands of values per
    # push and are merged bucket-parallel; "ties" draws 64 distinct values, so values tie with each other and
    # with centroid means (a value goes before an equal mean)
    batches, wms = _stream(800_000, 200_000, 1000, rate=100_000, zipf=1.1, values=values)
    out = _run(batches, wms, delta, expected_entries=4000)
    _assert_same(*out, delta)
    assert max(len(s) for s, _ in out[1]) > delta // 4  # hot digests fill their buckets


@pytest.mark.parametrize("size,slide,zipf,jitter", [(3000, 1000, 1.1, 200), (2000, 500, None, 900), (1000, 300, 1.1, 600)],
                         ids=["3s-1s-zipf", "2s-500ms-uniform-late", "1s-300ms-zipf-uneven"])
def test_gpu_tdigest_sliding_vs_oracle(size, slide, zipf, jitter):
    # t-digest over sliding windows (WindowedStream.aggregate takes any assigner, WindowedStream.java:687-852;
    # SlidingEventTimeWindows.assignWindows, SlidingEventTimeWindows.java:67-81): one digest per window, every
    # element sorted into each of its windows that is not late (jitter past the bound makes elements partially
    # late: their oldest windows are skipped, WindowOperator.java:379-407), centroids and quantiles bit-exact
    batches, wms = _stream(200_000, 25_000, 2000, rate=100_000, zipf=zipf, jitter=jitter, bound=200)
    out = _run(batches, wms, 40, sliding=(size, slide), expected_entries=30_000)
    _assert_same(*out, 40)
    assert any(len(s) > 10 for s, _ in out[1])


@pytest.mark.parametrize("gap,zipf,jitter,lateness", [(300, 1.1, 200, 0), (100, None, 900, 0), (2000, 1.3, 400, 0),
                                                      (300, 1.1, 1200, 800), (100, None, 900, 2000),
                                                      (1000, 1.3, 1500, 3000)],
                         ids=["zipf", "uniform-out-of-order", "long-gap-hot", "zipf-lateness", "uniform-lateness",
                              "hot-long-lateness"])
def test_gpu_tdigest_sessions_vs_oracle(gap, zipf, jitter, lateness):
    # a10: t-digest over EventTimeSessionWindows.  Sessions merge (MergingWindowSet.java:150-225) and their digests
    # with them (AbstractHeapMergingState.mergeNamespaces, AbstractHeapMergingState.java:67-93; AggregateFunction.merge,
    # AggregateFunction.java:160; this build's merge = the union of the centroids, compressed with the push's values,
    # oracle td_union) -- in the parallel session flush, in the ordered replay of elements that arrive behind the
    # watermark and bridge in-flight sessions, and across pushes.  Under allowed lateness a session that an element
    # reaches behind the watermark fires again at once (WindowOperator.java:352-360) with getResult over its digest --
    # the union of the digests merged into it in the push and the push's values so far (the oracle compresses a copy).
    # Centroids and quantiles bit-exact.
    batches, wms = _stream(200_000, 20_000, 3000, rate=100_000, zipf=zipf, jitter=jitter, bound=200)
    g_rows, g_dig, r_rows, r_dig = _run(batches, wms, 40, gap=gap, lateness=lateness, expected_entries=30_000)
    _assert_same(g_rows, g_dig, r_rows, r_dig, 40)
    assert (g_rows["end"] - g_rows["start"] > gap).any()  # sessions merged
    if lateness:
        keys = np.stack([g_rows["key"], g_rows["start"]], axis=1)
        assert len(np.unique(keys, axis=0)) < len(keys)  # sessions fired more than once


@pytest.mark.parametrize("sliding,lateness,zipf,jitter",
                         [(None, 500, None, 900), (None, 3000, 1.1, 1500), ((2000, 500), 300, 1.1, 900),
                          ((1000, 300), 1000, None, 1200)],
                         ids=["tumbling", "tumbling-hot-long", "sliding-zipf", "sliding-uneven"])
def test_gpu_tdigest_lateness_vs_oracle(sliding, lateness, zipf, jitter):
    # allowed lateness (WindowedStream.allowedLateness; WindowOperator.java:379-420, 588-598): a window fired at its
    # maxTimestamp keeps its digest until cleanupTime, and every element that reaches it behind the watermark fires
    # it again (EventTimeTrigger.onElement -> FIRE) with getResult over every value so far -- this push's values
    # still buffered (the oracle compresses a copy, window_oracle.cpp emit; the ordered path the window's sorted
    # chain of them into a scratch digest).  Late firings, the digests exported with them, the on-time rows and the
    # dropped elements are bit-exact with the oracle.
    batches, wms = _stream(200_000, 20_000, 2000, rate=100_000, zipf=zipf, jitter=jitter, bound=200)
    g_rows, g_dig, r_rows, r_dig = _run(batches, wms, 40, sliding=sliding, lateness=lateness, expected_entries=60_000)
    _assert_same(g_rows, g_dig, r_rows, r_dig, 40)
    keys = np.stack([g_rows["key"], g_rows["start"]], axis=1)
    assert len(np.unique(keys, axis=0)) < len(keys)  # windows fired more than once


@pytest.mark.parametrize("sliding,gap,lateness,zipf,jitter",
                         [(None, 300, 0, 1.1, 200), (None, 300, 800, 1.1, 1200), (None, 100, 2000, None, 900),
                          (None, None, 500, None, 900), (None, None, 3000, 1.1, 1500), ((2000, 500), None, 300, 1.1, 900)],
                         ids=["sessions", "sessions-lateness", "sessions-uniform-lateness", "tumbling-lateness",
                              "tumbling-hot-long", "sliding-lateness"])
def test_gpu_tdigest_purging_vs_oracle(sliding, gap, lateness, zipf, jitter):
    # PurgingTrigger (FIRE_AND_PURGE: WindowOperator.java:391-403, 454-463) with t-digests: a firing clears the
    # window's state -- the centroids, and on the ordered path the push's values so far, which leave the push's
    # compression (td_purge) -- and the window stays until its cleanup time: a session in its MergingWindowSet (an
    # empty digest that later elements and merges fill again), a time window as empty state that a late element
    # fills and fires again with only its own values.  Bit-exact against the oracle's state.erase.
    batches, wms = _stream(200_000, 20_000, 3000, rate=100_000, zipf=zipf, jitter=jitter, bound=200)
    g_rows, g_dig, r_rows, r_dig = _run(batches, wms, 40, sliding=sliding, gap=gap, lateness=lateness, purging=True,
                                        expected_entries=60_000)
    _assert_same(g_rows, g_dig, r_rows, r_dig, 40)
    if lateness:
        keys = np.stack([g_rows["key"], g_rows["start"]], axis=1)
        assert len(np.unique(keys, axis=0)) < len(keys)  # windows fired (and purged) more than once


@pytest.mark.parametrize("purging", [False, True], ids=["fire", "fire-and-purge"])
def test_gpu_tdigest_lateness_grows_mid_push(monkeypatch, purging):
    # a burst of late elements for new windows within the allowed lateness, each key four times across the batch:
    # every element creates or joins a window on the ordered path and fires it, the regions (FW_TABLE_SLACK=1: sized
    # at the expected entries, ~196 per 256-slot region against a load limit of 192) run out of room, the ordered
    # path suspends and the table grows mid-push -- the push's sorted chains of buffered values follow the moved
    # slots (k_td_relink / k_td_resort)
    from flink_amd.operator import GpuWindowOperator
    monkeypatch.setenv("FW_TABLE_SLACK", "1")
    n, m = 200_000, 200_000
    rng = np.random.default_rng(7)
    k1 = np.arange(n, dtype=np.int64)
    k2 = np.tile(np.arange(1_000_000, 1_000_000 + m, dtype=np.int64), 4)
    batches = [(k1, k1 % 1000, rng.normal(size=n)), (k2, k2 % 997, rng.normal(size=4 * m)),
               (k1[:0], k1[:0], np.zeros(0))]
    wms = [5000, 6000, (1 << 63) - 1]
    # (purging: every firing empties the window, so each of a key's four late elements fires alone, and the
    # purged values' items must stay out of the chains the grow rebuilds)
    from flink_amd import EventTimeTrigger, PurgingTrigger
    trig = PurgingTrigger.of(EventTimeTrigger.create()) if purging else None
    gpu = GpuWindowOperator(TumblingEventTimeWindows.of(1000), TDigest(40, export=True), allowed_lateness=1 << 40,
                            expected_entries=n + m, trigger=trig)
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=1000, tdigest=40, quantiles=(0.5, 0.95, 0.99),
                                   lateness=1 << 40, purging=purging)
    g_rows, g_dig = [], []
    for epoch, ((k, t, v), wm) in enumerate(zip(batches, wms)):
        if len(k):
            gpu.process(k, t, v)
            ref.process(k, t, v)
        gpu.advance_watermark(wm)
        g_dig += gpu.drain_digests()
        g_rows.append(gpu.drain_rows(epoch))
        ref.watermark(wm)
    st = gpu.stats()
    gpu.close()
    r_rows = ref.rows()
    assert st["table_grows"] >= 1 and st["slow_path_records"] >= 4 * m
    assert len(r_rows) == n + 4 * m
    _assert_same(np.concatenate(g_rows), g_dig, r_rows, [ref.digest(i) for i in range(len(r_rows))], 40)


def test_gpu_tdigest_blocks_are_recycled():
    # many short windows over few keys with a pool sized for one window's digests: fired blocks are reused
    batches, wms = _stream(400_000, 10_000, 500, rate=100_000, bound=50, jitter=50)
    from flink_amd.operator import GpuWindowOperator
    gpu = GpuWindowOperator(TumblingEventTimeWindows.of(100), TDigest(40, (0.1, 0.5, 0.9)), expected_entries=1500)
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=100, tdigest=40, quantiles=(0.1, 0.5, 0.9))
    for (k, t, v), wm in zip(batches, wms):
        if len(k):
            gpu.process(k, t, v)
            ref.process(k, t, v)
        gpu.watermark(wm)
        ref.watermark(wm)
    g, r = gpu.rows(), ref.rows()
    gpu.close()
    assert len(g) == len(r) > 1000
    go = np.lexsort((g["start"], g["key"], g["epoch"]))
    ro = np.lexsort((r["start"], r["key"], r["epoch"]))
    for f in ("key", "start", "count", "sum", "min", "max"):
        assert np.array_equal(g[f][go], r[f][ro]), f


def test_gpu_tdigest_refuses_unsupported_shapes():
    from flink_amd import SlidingEventTimeWindows
    from flink_amd import _native as N
    from flink_amd.operator import GpuWindowOperator
    from flink_amd import EventTimeSessionWindows, EventTimeTrigger, PurgingTrigger
    purge = PurgingTrigger.of(EventTimeTrigger.create())
    for kw in (dict(assigner=EventTimeSessionWindows.with_gap(1000), trigger=purge),
               dict(assigner=EventTimeSessionWindows.with_gap(1000), allowed_lateness=10, trigger=purge),
               dict(allowed_lateness=10, trigger=purge),
               dict(assigner=SlidingEventTimeWindows.of(3000, 1000), allowed_lateness=10, trigger=purge)):
        GpuWindowOperator(kw.pop("assigner", TumblingEventTimeWindows.of(1000)), TDigest(100), **kw).close()  # offered
    with pytest.raises(N.NativeError) as e:
        GpuWindowOperator(TumblingEventTimeWindows.of(1000), TDigest(99))
    assert e.value.code == N.FW_ERR_ARG
    # the digest is not in fw_state_rows: the row-only snapshot call refuses it (test_gpu_pool_state covers the
    # block variant)
    import ctypes
    op = GpuWindowOperator(TumblingEventTimeWindows.of(1000), TDigest(100))
    n = ctypes.c_int64()
    assert N.lib().fw_snapshot_key_group(op._h, 0, None, 0, ctypes.byref(n)) == N.FW_ERR_UNSUPPORTED
    op.close()


def test_gpu_tdigest_full_size():
    # SURVEY §8d C5 shape: 2^24 records per push generated in HBM (Zipf(1.1) over 1M keys, 1e8 records per
    # event-second, values = the generator's int32 column as doubles), 3 pushes, then the final watermark
    import torch
    from flink_amd.datagen import generate_device, generate_host, zipf_cdf
    from flink_amd.operator import GpuWindowOperator
    n, steps, keys = 1 << 24, 3, 1_000_000
    cdf = torch.tensor(zipf_cdf(keys, 1.1), dtype=torch.float64, device="cuda")
    gpu = GpuWindowOperator(TumblingEventTimeWindows.of(1000), TDigest(100, (0.5, 0.9, 0.99)),
                            expected_entries=2_000_000)
    for s in range(steps):
        k, t, v, mx = generate_device(0x5EED, s * n, n, keys, ts_base=1_000_000, rate=100_000_000, jitter=200,
                                      cdf_dev=cdf)
        gpu.process_batch(k, t, v.to(torch.float64))
        gpu.watermark(int(mx.item()) - 200)
    gpu.watermark((1 << 63) - 1)
    rows = gpu.rows()
    assert gpu.late_dropped == 0
    gpu.close()
    assert int(rows["count"].sum()) == n * steps
    q = {f: rows[f].view(np.float64) for f in ("sum", "min", "max")}
    assert np.all(q["sum"] <= q["min"]) and np.all(q["min"] <= q["max"])
    # exact quantiles of the three hottest (key, window) rows from the same stream generated on the host
    hk, ht, hv = generate_host(0x5EED, 0, n * steps, keys, ts_base=1_000_000, rate=100_000_000, jitter=200,
                               zipf_s=1.1)
    hv = hv.astype(np.float64)
    for i in np.argsort(-rows["count"])[:3]:
        r = rows[i]
        sel = np.sort(hv[(hk == r["key"]) & (ht >= r["start"]) & (ht < r["end"])])
        assert len(sel) == r["count"]
        for f, qv in (("sum", 0.5), ("min", 0.9), ("max", 0.99)):
            rank = np.searchsorted(sel, q[f][i]) / len(sel)
            assert abs(rank - qv) < 0.01, (r["key"], qv, rank)
