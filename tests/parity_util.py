"""Row-multiset comparison between the GPU operator and the oracle (TestHarnessUtil.assertOutputEqualsSorted:
watermark epochs exact, rows sorted inside an epoch; flink-streaming-java/src/test/java/org/apache/flink/
streaming/util/TestHarnessUtil.java:70-108)."""
import numpy as np

F64_RTOL = 1e-6  # north_star: floating-point sums within 1e-6 relative
F32_U = 2.0 ** -24  # unit roundoff of float


def f32_sum_bound(rows, sums=()):
    """north_star exception for Float fields (DESIGN §2 "Float sums"): FloatSum rounds every partial sum to float in
    arrival order (SumFunction.java:92-99), so the reference's sum S_java of a window's n elements x_i carries the
    recursive-summation error |S_java - S| <= (n - 1) u sum|x_i| (u = 2^-24), which depends on the order and is not
    within 1e-6 of S for long or cancelling windows.  The GPU sums in f64 and rounds once (|S_gpu - S| <= u |S| +
    n 2^-53 sum|x_i|).  So the two agree within (n + 1) u sum|x_i|, with sum|x_i| <= n max(|min|, |max|) from the
    row itself: the bound checked here, per row (not a relative tolerance).  A passthrough row (FW_AGG_FIRST) keeps
    the first element's ordinal in `max`, so there the magnitude is also taken from the sums (`sums`): |S| =
    sum|x_i| for a field of one sign, which is what the passthrough tests feed."""
    n = rows["count"].astype(np.float64)
    amax = np.maximum(np.abs(rows["min"].view(np.float64)), np.abs(rows["max"].view(np.float64)))
    mag = n * amax
    for sm in sums:
        mag = np.maximum(mag, np.abs(sm))
    return (n + 1.0) * F32_U * mag * 1.001


def assert_f32_sums_near_exact(rows, keys, ts, vals, windows_of, size=None, wm_prev=None):
    """The tight half of the Float-sum check: the GPU sums a Float field in f64 and rounds once, so
    against the exact sum S of the window's elements |S_gpu - S| <= u |S| + n 2^-53 sum|x_i| -- linear in n, unlike
    the recursive-summation bound above, so a wrong element in a long window does not pass.  `windows_of(ts)` gives
    each element's window starts (a list of arrays, one per window it belongs to; tumbling / sliding assigners);
    with `size` and `wm_prev` (the watermark in effect when each element was processed) an element joins only the
    windows that are not late for it (WindowOperator.isWindowLate, allowed lateness 0: maxTimestamp <= watermark).
    The exact sums are f64 sums of float32 values of bounded magnitude (exact when they fit 53 bits, as in the
    tests that call this).  Every row's (key, window) element count must then equal the row's count."""
    k_all, s_all, x_all = [], [], []
    for starts in windows_of(ts):
        keep = np.ones(len(ts), dtype=bool) if wm_prev is None else starts + size - 1 > wm_prev
        k_all.append(keys[keep])
        s_all.append(starts[keep])
        x_all.append(vals[keep])
    k_all, s_all, x_all = np.concatenate(k_all), np.concatenate(s_all), np.concatenate(x_all)
    grp, inv = np.unique(np.stack([k_all, s_all], axis=1), axis=0, return_inverse=True)
    inv = inv.ravel()
    exact = np.zeros(len(grp))
    absum = np.zeros(len(grp))
    cnt = np.zeros(len(grp), dtype=np.int64)
    np.add.at(exact, inv, x_all)
    np.add.at(absum, inv, np.abs(x_all))
    np.add.at(cnt, inv, 1)
    idx = {(int(a), int(b)): i for i, (a, b) in enumerate(grp)}
    checked = 0
    for r in rows:
        i = idx.get((int(r["key"]), int(r["start"])))
        assert i is not None and cnt[i] == r["count"], (r, None if i is None else cnt[i])
        got = float(np.int64(r["sum"]).view(np.float64))
        n = float(cnt[i])
        assert abs(got - exact[i]) <= F32_U * abs(exact[i]) + n * 2.0 ** -53 * absum[i], (r, exact[i])
        checked += 1
    assert checked == len(rows) > 0


def _sorted(rows):
    order = np.lexsort((rows["end"], rows["start"], rows["key"], rows["epoch"]))
    return rows[order]


def assert_rows_equal(gpu, ref, value_type="long"):
    assert len(gpu) == len(ref), f"row count {len(gpu)} != {len(ref)}"
    if len(gpu) == 0:
        return
    g, r = _sorted(gpu), _sorted(ref)
    for f in ("epoch", "key", "start", "end", "count"):
        bad = np.nonzero(g[f] != r[f])[0]
        assert bad.size == 0, f"field {f} differs at {bad[:5]}: gpu={g[bad[:5]]} ref={r[bad[:5]]}"
    if value_type in ("double", "float"):
        for f in ("min", "max"):
            gb, rb = g[f].view(np.float64), r[f].view(np.float64)
            same = (gb == rb) | (np.isnan(gb) & np.isnan(rb))
            bad = np.nonzero(~same)[0]
            assert bad.size == 0, f"field {f} differs at {bad[:5]}"
        gs, rs = g["sum"].view(np.float64), r["sum"].view(np.float64)
        if value_type == "float":
            with np.errstate(invalid="ignore"):
                ok = (np.abs(gs - rs) <= f32_sum_bound(r, (gs, rs))) | (gs == rs) | (np.isnan(gs) & np.isnan(rs))
        else:
            ok = np.isclose(gs, rs, rtol=F64_RTOL, atol=0.0) | (np.isnan(gs) & np.isnan(rs))
        bad = np.nonzero(~ok)[0]
        assert bad.size == 0, f"sum differs beyond rtol at {bad[:5]}: {gs[bad[:5]]} vs {rs[bad[:5]]}"
    else:
        for f in ("sum", "min", "max"):
            bad = np.nonzero(g[f] != r[f])[0]
            assert bad.size == 0, f"field {f} differs at {bad[:5]}: gpu={g[bad[:5]]} ref={r[bad[:5]]}"


def assert_side_equal(gpu, ref):
    assert len(gpu) == len(ref)
    if len(gpu) == 0:
        return
    key = lambda a: a[np.lexsort((a["val"], a["ts"], a["key"], a["epoch"]))]  # noqa: E731
    g, r = key(gpu), key(ref)
    for f in ("epoch", "key", "ts", "val"):
        assert np.array_equal(g[f], r[f]), f"side field {f} differs"
