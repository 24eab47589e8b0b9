"""f3 oracle: the Table API's group-window aggregates (OR_AGG_ROW, oracle/window_oracle.h) against the reference's
own ITCases (SqlITCase testRowTimeTumbleWindow; GroupWindowITCase tumbling / session / sliding tests), and the
built-in functions' semantics from their sources (flink-table .../functions/aggfunctions/*.scala) on edge values."""
import numpy as np
import pytest

from oracle import oracle as orc
from tests.kat_util import load_kats
from tests.table_util import case_cfg, case_events, expected_rows, rows_with_values

CASES = load_kats()["table_group_windows"]


def _run(case):
    names, steps = case_events(case)
    o = orc.WindowOperatorOracle(**case_cfg(case), row=(case["types"], case["specs"]))
    for keys, ts, cols, nulls, wm in steps:
        o.process_rows(keys, ts, cols, nulls)
        o.watermark(wm)
    vals, nm = o.row_results()
    return names, rows_with_values(o.rows(), vals, nm)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_table_group_window_kats(case):
    names, got = _run(case)
    assert got == expected_rows(case, names)


def _one_window(types, specs, cols, nulls=None):
    n = len(cols[0])
    o = orc.WindowOperatorOracle(assigner="tumbling", size=1000, row=(types, specs))
    o.process_rows(np.zeros(n, dtype=np.int64), np.arange(n, dtype=np.int64), cols, nulls)
    o.watermark((1 << 63) - 1)
    vals, nm = o.row_results()
    assert len(vals) == 1
    return [None if (int(nm[0]) >> q) & 1 else int(vals[0][q]) for q in range(len(specs))]


def test_oracle_table_sum_null_when_empty_and_avg_division():
    specs = [("count_star", 0), ("count", 0), ("sum", 0), ("min", 0), ("max", 0), ("avg", 0)]
    # every value NULL: COUNT(*) counts the records, COUNT(col) 0, SUM / MIN / MAX / AVG NULL
    assert _one_window(["i32"], specs, [np.array([5, 6, 7])], np.array([1, 1, 1], dtype=np.uint8)) == \
        [3, 0, None, None, None, None]
    # IntegralAvgAggFunction: Long sum / count with Java's truncating division, then toInt
    assert _one_window(["i32"], specs, [np.array([-7, 2, 0])]) == [3, 3, -5, -7, 2, -1]
    # Int SUM wraps at 32 bits (Scala Numeric[Int]); AVG uses the Long sum
    big = np.array([2**31 - 1, 2**31 - 1, 2], dtype=np.int64)
    assert _one_window(["i32"], specs, [big]) == [3, 3, 0, 2, 2**31 - 1, (2 * (2**31 - 1) + 2) // 3]
    # Long AVG divides the exact (BigInteger) sum: no 64-bit wrap; Long SUM wraps
    lng = np.array([2**63 - 1, 2**63 - 1, 2**63 - 1], dtype=np.int64)
    assert _one_window(["i64"], specs, [lng])[2] == (3 * (2**63 - 1) + 2**63) % 2**64 - 2**63
    assert _one_window(["i64"], specs, [lng])[5] == 2**63 - 1
    neg = np.array([-(2**63), -(2**63), -1], dtype=np.int64)
    assert _one_window(["i64"], [("avg", 0)], [neg]) == [-((2**64 + 1) // 3)]  # truncates toward zero
    # Byte / Short: SUM and AVG narrow to the type
    assert _one_window(["i8"], [("sum", 0), ("avg", 0)], [np.array([100, 100, 100])]) == [300 - 256, 100]


def test_oracle_table_double_and_float():
    f = np.array([1.5, -0.0, 0.0, 2.25])
    vals = _one_window(["f64"], [("sum", 0), ("min", 0), ("max", 0), ("avg", 0)], [f])
    d = np.array(vals, dtype=np.int64).view(np.float64)
    assert d[0] == 3.75 and np.signbit(d[1]) and d[1] == 0.0 and d[2] == 2.25 and d[3] == 3.75 / 4
    # Float: SUM adds in float, AVG in double (FloatingAvgAggFunction over doubleValue()), narrowed to float
    x = np.array([np.float32(0.1), np.float32(0.2), np.float32(0.3)], dtype=np.float64)
    s, a = np.array(_one_window(["f32"], [("sum", 0), ("avg", 0)], [x]), dtype=np.int64).view(np.float64)
    assert s == float(np.float32(np.float32(np.float32(0.1) + np.float32(0.2)) + np.float32(0.3)))
    assert a == float(np.float32((x[0] + x[1] + x[2]) / 3))


def test_oracle_table_session_merge_combines_columns():
    # two sessions of one key bridged by a later element: the merged accumulator is the merge of every column
    o = orc.WindowOperatorOracle(assigner="session", gap=15, row=(["i64", "f64"],
                                                                  [("count_star", 0), ("sum", 0), ("min", 1),
                                                                   ("count", 1), ("avg", 0)]))
    k = np.zeros(3, dtype=np.int64)
    o.process_rows(k, np.array([0, 30, 15]), [np.array([4, 5, 6]), np.array([1.0, -2.0, 0.5])],
                   np.array([0, 2, 0], dtype=np.uint8))
    o.watermark((1 << 63) - 1)
    r = o.rows()
    vals, nm = o.row_results()
    assert len(r) == 1 and r[0]["start"] == 0 and r[0]["end"] == 45 and r[0]["count"] == 3
    assert vals[0][1] == 15 and vals[0][3] == 2 and vals[0][4] == 5
    assert np.array([vals[0][2]]).view(np.float64)[0] == 0.5 and nm[0] == 0
