"""HyperLogLog AggregateFunction of the oracle (definition in oracle/window_oracle.h).

No reference file holds an HLL (Flink 1.5 ships none; C5 names it as a user AggregateFunction), so the
oracle's HLL is pinned two ways: (1) against an independent numpy restatement of the same definition,
register by register through the exact checksum S and the zero count V, and (2) by the estimator's
published accuracy (standard error 1.04 / sqrt(m), Flajolet et al. 2007) against exact distinct counts."""
import numpy as np

from oracle import oracle as orc

M64 = (1 << 64) - 1


def _fmix64(x):
    x = x.astype(np.uint64)
    x ^= x >> np.uint64(33)
    x *= np.uint64(0xff51afd7ed558ccd)
    x ^= x >> np.uint64(33)
    x *= np.uint64(0xc4ceb9fe1a85ec53)
    x ^= x >> np.uint64(33)
    return x


def _np_hll(items, p):
    h = _fmix64(items.view(np.uint64))
    j = (h >> np.uint64(64 - p)).astype(np.int64)
    w = (h << np.uint64(p)) | np.uint64(1 << (p - 1))
    # clz64 + 1 via the position of the highest set bit
    hb = np.floor(np.log2(w.astype(np.float64))).astype(np.int64)
    # float rounding near powers of two: fix with exact shifts
    hb = np.where((w >> hb.astype(np.uint64)) == 0, hb - 1, hb)
    hb = np.where((w >> (hb + 1).astype(np.uint64)) != 0, hb + 1, hb)
    rank = 64 - hb
    regs = np.zeros(1 << p, dtype=np.int64)
    np.maximum.at(regs, j, rank)
    S = sum(1 << (65 - p - int(r)) for r in regs)
    return regs, S, int((regs == 0).sum())


def _run(keys, ts, items, p, size=1000):
    o = orc.WindowOperatorOracle(assigner="tumbling", size=size, hll_p=p)
    o.process(keys, ts, items)
    o.watermark((1 << 63) - 1)
    r = o.rows()
    o.close()
    return r


def test_hll_registers_match_independent_restatement():
    rng = np.random.default_rng(7)
    for p, n in ((4, 50), (10, 5000), (14, 200_000)):
        items = rng.integers(-(1 << 63), (1 << 63) - 1, size=n, dtype=np.int64)
        rows = _run(np.zeros(n, np.int64), np.zeros(n, np.int64), items, p)
        assert len(rows) == 1
        _, S, V = _np_hll(items, p)
        assert rows["count"][0] == n
        assert rows["min"][0] == V
        assert (int(rows["max"][0]) & M64) == (S & M64)


def test_hll_estimate_accuracy():
    rng = np.random.default_rng(11)
    p = 14
    for distinct in (100, 10_000, 1_000_000):
        pool = rng.integers(-(1 << 63), (1 << 63) - 1, size=distinct, dtype=np.int64)
        items = np.concatenate([pool, pool[: distinct // 2]])  # duplicates do not count
        rows = _run(np.zeros(len(items), np.int64), np.zeros(len(items), np.int64), items, p)
        est = rows["sum"].view(np.float64)[0]
        assert abs(est - distinct) <= 4 * 1.04 / np.sqrt(1 << p) * distinct + 1, (distinct, est)


def test_hll_per_key_and_window():
    # keys x tumbling windows: each (key, window) gets its own registers
    rng = np.random.default_rng(3)
    n = 20_000
    keys = rng.integers(0, 5, size=n, dtype=np.int64)
    ts = rng.integers(0, 3000, size=n, dtype=np.int64)
    items = rng.integers(0, 1000, size=n, dtype=np.int64)
    rows = _run(keys, ts, items, 8)
    assert len(rows) == 15
    for r in rows:
        sel = (keys == r["key"]) & (ts >= r["start"]) & (ts < r["end"])
        _, S, V = _np_hll(items[sel], 8)
        assert r["count"] == sel.sum() and r["min"] == V and (int(r["max"]) & M64) == (S & M64)
