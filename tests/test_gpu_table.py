"""f3 on the GPU: the Table API's group-window aggregates (FW_AGG_ROW; DataStreamGroupWindowAggregate.scala:197-294)
against the reference's own ITCases and the oracle's restatement of flink-table's built-in aggregate functions
(oracle/window_oracle.h OR_AGG_ROW).  Bar: keys, window bounds, COUNT(*), COUNT(col), integral SUM / MIN / MAX /
AVG and floating MIN / MAX bit-exact (NULLs included); Double SUM / AVG within 1e-9 relative (positive values: the
GPU's atomics add in another order than the reference's arrival order); Float SUM within the recursive-summation
bound (n + 1) 2^-24 sum|x| of the reference's float additions (DESIGN §2 "Float sums"); Float AVG within one float
ulp."""
import numpy as np
import pytest

from flink_amd.datagen import generate_host
from flink_amd.windowing import RowAggregate
from oracle import oracle as orc
from tests.kat_util import load_kats
from tests.table_util import case_cfg, case_events, expected_rows, rows_with_values

pytestmark = pytest.mark.gpu

CASES = load_kats()["table_group_windows"]
_T = {"i64": "long", "i32": "int", "f64": "double", "i16": "short", "i8": "byte", "f32": "float"}


def _op(cfg, types, specs, **kw):
    from flink_amd import EventTimeSessionWindows, SlidingEventTimeWindows, TumblingEventTimeWindows
    from flink_amd.operator import GpuWindowOperator
    a = cfg["assigner"]
    asg = (TumblingEventTimeWindows.of(cfg["size"], cfg.get("offset", 0)) if a == "tumbling"
           else SlidingEventTimeWindows.of(cfg["size"], cfg["slide"], cfg.get("offset", 0)) if a == "sliding"
           else EventTimeSessionWindows.with_gap(cfg["gap"]))
    return GpuWindowOperator(asg, RowAggregate(tuple(_T[t] for t in types), tuple(tuple(s) for s in specs)), **kw)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_gpu_table_group_window_kats(case):
    names, steps = case_events(case)
    op = _op(case_cfg(case), case["types"], case["specs"])
    for keys, ts, cols, nulls, wm in steps:
        op.process_row_batch(keys, ts, cols, nulls)
        op.watermark(wm)
    vals, nm = op.row_results()
    got = rows_with_values(op.rows(), vals, nm)
    op.close()
    assert got == expected_rows(case, names)


TYPES = ["i64", "i32", "f64", "f32", "i8"]
SPECS = [("count_star", 0), ("count", 0), ("sum", 0), ("avg", 0), ("min", 0), ("max", 0),  # (16: the ABI's limit)
         ("sum", 1), ("avg", 1), ("min", 1),
         ("sum", 2), ("avg", 2), ("min", 2), ("max", 2),
         ("sum", 3), ("max", 3), ("avg", 4)]


def _stream(n, batch, keys, bound, jitter, rate, seed=0x5EED, zipf=1.1, null_frac=0.15):
    k, t, v = generate_host(seed, 0, n, keys, ts_base=1_000_000, rate=rate, jitter=jitter, zipf_s=zipf)
    rng = np.random.default_rng(seed)
    cols = [v << 31,                                              # Long: window sums pass 64 bits (AVG exact)
            v % 100_003,                                          # Int
            ((v & 0xFFFFF) + 1).astype(np.float64) / 7.0,        # Double, positive
            np.float32((v & 0xFFF) + 1).astype(np.float64) / 3.0,  # (the double of) a Float, positive
            (v % 200) - 100]                                      # Byte: SUM wraps to 8 bits
    cols[3] = np.float32(cols[3]).astype(np.float64)
    nulls = np.zeros(n, dtype=np.uint8)
    for j in range(len(cols)):
        nulls |= ((rng.random(n) < null_frac).astype(np.uint8) << j)
    out, mx = [], -(1 << 63)
    for b in range(0, n, batch):
        sl = slice(b, min(n, b + batch))
        mx = max(mx, int(t[sl].max()))
        out.append((k[sl], t[sl], [c[sl] for c in cols], nulls[sl], mx - bound))
    e = np.zeros(0, dtype=np.int64)
    out.append((e, e, [e.astype(np.float64) if TYPES[j] in ("f64", "f32") else e for j in range(len(cols))],
                np.zeros(0, dtype=np.uint8), (1 << 63) - 1))
    return out


def _compare(g_rows, g_vals, g_nm, r_rows, r_vals, r_nm):
    key = lambda rows: np.lexsort((rows["start"], rows["key"], rows["epoch"]))  # noqa: E731
    gi, ri = key(g_rows), key(r_rows)
    assert len(gi) == len(ri) > 0
    for f in ("epoch", "key", "start", "end", "count"):
        assert np.array_equal(g_rows[f][gi], r_rows[f][ri]), f
    assert np.array_equal(g_nm[gi], r_nm[ri])
    gv, rv = g_vals[gi], r_vals[ri]
    live = (g_nm[gi, None] >> np.arange(len(SPECS))[None, :]) & 1 == 0
    for q, (fn, c) in enumerate(SPECS):
        t = TYPES[c]
        m = live[:, q]
        a, b = gv[m, q], rv[m, q]
        if t not in ("f64", "f32") or fn in ("count", "count_star", "min", "max"):
            assert np.array_equal(a, b), (fn, c, np.flatnonzero(a != b)[:5])
            continue
        x, y = a.view(np.float64), b.view(np.float64)
        if t == "f64":
            assert np.allclose(x, y, rtol=1e-9, atol=0), (fn, c)
        elif fn == "sum":  # the reference adds in float (positive values: sum|x| = |S|)
            cnt = g_rows["count"][gi][m].astype(np.float64)
            assert np.all(np.abs(x - y) <= (cnt + 1) * 2.0 ** -24 * np.abs(y) * 1.001), (fn, c)
        else:  # float AVG: (float)(double sum / count), the double sums in different orders
            assert np.all(np.abs(x - y) <= 2.0 ** -23 * np.abs(y)), (fn, c)


CFGS = [dict(assigner="tumbling", size=1000), dict(assigner="sliding", size=3000, slide=1000),
        dict(assigner="sliding", size=2500, slide=1000, offset=300), dict(assigner="session", gap=400)]


@pytest.mark.parametrize("small_table", [False, True], ids=["sized", "grows"])
@pytest.mark.parametrize("cfg", CFGS, ids=["tumbling", "sliding", "sliding-split", "session"])
def test_gpu_table_vs_oracle(cfg, small_table):
    # Zipf(1.1) keys, out-of-order timestamps (jitter 900 ms against a 300 ms bound: late records are dropped and, for
    # sessions, arrive behind in-flight sessions: the ordered path), NULLs in every column; "grows": the table
    # starts small (4 regions), so the aggregate suspends mid-push, the table and the Row accumulators' block pool
    # grow and the push resumes (the per-record column adds, which are not idempotent, must still count every record
    # once)
    steps = _stream(1 << 17, 1 << 14, 20_000, bound=300, jitter=900, rate=200_000)
    small = dict(expected_entries=2000, max_parallelism=4, sub_partitions=1) if small_table else {}
    gpu = _op(cfg, TYPES, SPECS, max_batch=1 << 14, **small)
    ref = orc.WindowOperatorOracle(**cfg, row=(TYPES, SPECS))
    for k, t, cols, nulls, wm in steps:
        gpu.process_row_batch(k, t, cols, nulls)
        ref.process_rows(k, t, cols, nulls)
        gpu.watermark(wm)
        ref.watermark(wm)
    g_vals, g_nm = gpu.row_results()
    r_vals, r_nm = ref.row_results()
    st = gpu.stats()
    _compare(gpu.rows(), g_vals, g_nm, ref.rows(), r_vals, r_nm)
    assert st["late_records_dropped"] == ref.late_dropped
    if small_table:
        assert st["table_grows"] > 0
    gpu.close()


def test_gpu_table_device_push_async():
    # the device entry point (fw_push_row_batch_device): columns and NULL masks as HBM tensors, async input
    import torch
    cfg = dict(assigner="tumbling", size=1000)
    steps = _stream(1 << 17, 1 << 15, 5_000, bound=200, jitter=200, rate=1_000_000)
    gpu = _op(cfg, TYPES, SPECS, max_batch=1 << 15)
    ref = orc.WindowOperatorOracle(**cfg, row=(TYPES, SPECS))
    rows, vals, nms = [], [], []
    for e, (k, t, cols, nulls, wm) in enumerate(steps):
        dev = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (k, t, nulls)]
        dcols = torch.from_numpy(np.stack([np.asarray(c).view(np.int64) for c in cols])).cuda()
        gpu.process_rows(dev[0], dev[1], dcols, dev[2])
        gpu.advance_watermark(wm, wait=False)
        v, m = gpu.drain_row_results()
        r = gpu.drain_rows(e)
        rows.append(r), vals.append(v), nms.append(m)
        ref.process_rows(k, t, cols, nulls)
        ref.watermark(wm)
    r_vals, r_nm = ref.row_results()
    _compare(np.concatenate(rows), np.concatenate(vals), np.concatenate(nms), ref.rows(), r_vals, r_nm)
    gpu.close()


def test_gpu_table_host_mirror_group_window():
    # flink_amd.table.GroupWindowAggregate (the host side of DataStreamGroupWindowAggregate): GroupWindowITCase's
    # tumbling select list, decoded to SQL values
    from flink_amd.table import GroupWindowAggregate, Tumble
    case = next(c for c in CASES if c["name"] == "table_tumble_builtins")
    names, steps = case_events(case)
    g = GroupWindowAggregate(Tumble.over(5), ["int"], [tuple(s) for s in case["specs"]])
    out = []
    for keys, ts, cols, nulls, wm in steps:
        g.process(keys, ts, cols, nulls)
        out += g.watermark(wm)
    g.close()
    assert sorted((k, s, e, tuple(v)) for k, v, s, e in out) == expected_rows(case, names)


def test_gpu_table_snapshot_restore():
    # keyed-state snapshot of the Row accumulators by key group (fw_snapshot_key_group_blocks), restored into a
    # fresh operator that then continues the stream: the same rows as one operator over the whole stream
    cfg = dict(assigner="session", gap=400)
    steps = _stream(1 << 16, 1 << 13, 3_000, bound=300, jitter=600, rate=100_000)
    half = len(steps) // 2
    a = _op(cfg, TYPES, SPECS, max_batch=1 << 13)
    ref = orc.WindowOperatorOracle(**cfg, row=(TYPES, SPECS))
    for k, t, cols, nulls, wm in steps[:half]:
        a.process_row_batch(k, t, cols, nulls)
        a.watermark(wm)
        ref.process_rows(k, t, cols, nulls)
        ref.watermark(wm)
    snap = {kg: a.snapshot_key_group(kg) for kg in range(128)}
    rows0, (v0, m0) = a.rows(), a.row_results()
    b = _op(cfg, TYPES, SPECS, max_batch=1 << 13)
    for kg, s in snap.items():
        b.restore_key_group(kg, s)
    b.advance_watermark(steps[half - 1][4])  # the restored operator's watermark (no window is due at it)
    b.clear_pending()
    for k, t, cols, nulls, wm in steps[half:]:
        b.process_row_batch(k, t, cols, nulls)
        b.watermark(wm)
        ref.process_rows(k, t, cols, nulls)
        ref.watermark(wm)
    r1, (v1, m1) = b.rows(), b.row_results()
    r1["epoch"] += half - 1  # (b's first watermark was the restore's)
    r_vals, r_nm = ref.row_results()
    _compare(np.concatenate([rows0, r1]), np.concatenate([v0, v1]), np.concatenate([m0, m1]), ref.rows(), r_vals,
             r_nm)
    a.close()
    b.close()
