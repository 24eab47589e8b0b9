"""Row-multiset comparison between the GPU operator and the oracle (TestHarnessUtil.assertOutputEqualsSorted:
watermark epochs exact, rows sorted inside an epoch; flink-streaming-java/src/test/java/org/apache/flink/
streaming/util/TestHarnessUtil.java:70-108)."""
import numpy as np

F64_RTOL = 1e-6  # north_star: floating-point sums within 1e-6 relative
F32_RTOL = 1e-5  # Float fields: FloatSum rounds every partial sum to float (SumFunction.java:92-99)


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
        ok = (np.isclose(gs, rs, rtol=F32_RTOL if value_type == "float" else F64_RTOL, atol=0.0)
              | (np.isnan(gs) & np.isnan(rs)))
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
