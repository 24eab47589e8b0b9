"""Pins the CPU oracle (oracle/) against the reference's own known-answer tests
(tests/golden/reference_kats.json, transcribed with provenance by tests/golden/make_golden.py)."""
from collections import Counter

import numpy as np
import pytest

from oracle import oracle as orc
from tests.kat_util import expected_counters, load_kats, replay, replay_list_phases, row_counters

KATS = load_kats()
KEYMAP = KATS["keys"]


def _make_oracle(cfg):
    return orc.WindowOperatorOracle(assigner=cfg["assigner"], size=cfg["size"], slide=cfg["slide"],
                                    offset=cfg["offset"], gap=cfg["gap"], lateness=cfg["lateness"],
                                    purging=cfg["purging"], side_output=cfg["side_output"],
                                    value_type=cfg["value_type"])


@pytest.mark.parametrize("case", KATS["operator_cases"], ids=[c["name"] for c in KATS["operator_cases"]])
def test_window_operator_kats(case):
    op = replay(case, KEYMAP, _make_oracle, flush_elements=False)
    got, got_side = row_counters(op.rows(), op.side_rows(), case, with_window=True)
    exp, exp_side = expected_counters(case, KEYMAP, with_window=True)
    assert got == exp
    assert got_side == exp_side
    if not case["cfg"]["side_output"]:
        # elements the KAT sends to a side output are counted as dropped when no tag is set
        assert op.late_dropped == 0 or case["expected_side"] == []


def test_key_group_kats():
    kg = KATS["key_groups"]
    L = orc.lib()
    for key, group in kg["key_group"]:
        # Integer.hashCode() == value
        assert L.oracle_key_group(key, kg["max_parallelism"]) == group
    for max_par, par, group, idx in kg["operator_index"]:
        assert L.oracle_operator_index(max_par, par, group) == idx


def test_window_start_kats():
    L = orc.lib()
    for ts, off, size, exp in KATS["window_start"]["cases"]:
        assert L.oracle_window_start(ts, off, size) == exp


def test_assigner_kats():
    for kind, size, slide, offset, ts, wins in KATS["assigners"]["cases"]:
        # assignment observed through the operator: one element, then a final watermark
        op = orc.WindowOperatorOracle(assigner=kind, size=size, slide=slide, offset=offset)
        op.process(np.array([1]), np.array([ts]), np.array([7]))
        op.watermark((1 << 63) - 1)
        rows = op.rows()
        got = sorted((int(r["start"]), int(r["end"])) for r in rows)
        assert got == sorted(tuple(w) for w in wins)
        assert all(r["count"] == 1 and r["sum"] == 7 for r in rows)


def test_session_example_kat():
    ex = KATS["session_example"]
    names = sorted({r[0] for r in ex["input"]})
    ids = {n: i for i, n in enumerate(names)}
    op = orc.WindowOperatorOracle(assigner="session", gap=ex["gap"], value_type="i32")
    for name, ts, val in ex["input"]:
        op.process(np.array([ids[name]]), np.array([ts]), np.array([val]))
        op.watermark(ts - 1)
    op.watermark((1 << 63) - 1)
    got = Counter((names[int(r["key"])], int(r["start"]), int(r["sum"])) for r in op.rows())
    assert got == Counter(tuple(e) for e in ex["expected"])


def test_session_example_sum_passthrough_kat():
    # a9: sum(2) keeps the session's FIRST element (SumAggregator.java:66-76); the first-element reduce
    # reports its arrival ordinal, from which the passthrough fields are taken
    from flink_amd.windowing import first_element_results
    ex = KATS["session_example"]
    names = sorted({r[0] for r in ex["input"]})
    ids = {n: i for i, n in enumerate(names)}
    op = orc.WindowOperatorOracle(assigner="session", gap=ex["gap"], value_type="i32", first=True)
    for name, ts, val in ex["input"]:
        op.process(np.array([ids[name]]), np.array([ts]), np.array([val]))
        op.watermark(ts - 1)
    op.watermark((1 << 63) - 1)
    got = first_element_results(op.rows(), [tuple(e) for e in ex["input"]], 2, "sum")
    assert sorted(got) == sorted(tuple(e) for e in ex["expected"])


def test_max_pos_keeps_first_element():
    # max(pos) (Comparator.MaxComparator, non-by aggregation): the first element with the field set to the max
    op = orc.WindowOperatorOracle(assigner="tumbling", size=10, first="max")
    op.process(np.array([1, 1, 1]), np.array([1, 2, 3]), np.array([4, 9, -2]))
    op.watermark((1 << 63) - 1)
    (r,) = op.rows()
    assert (int(r["min"]), int(r["max"]), int(r["count"])) == (9, 0, 3)


def test_first_element_reduce_keeps_first_across_merges():
    # tumbling: the ordinal is the first element added to each window; sessions: a bridging element
    # merges two sessions and the earlier first element survives
    op = orc.WindowOperatorOracle(assigner="tumbling", size=10, first=True)
    op.process(np.array([1, 2, 1, 1]), np.array([5, 3, 2, 15]), np.array([10, 20, 30, 40]))
    op.watermark((1 << 63) - 1)
    got = sorted((int(r["key"]), int(r["start"]), int(r["count"]), int(r["sum"]), int(r["min"]), int(r["max"]))
                 for r in op.rows())
    assert got == [(1, 0, 2, 40, 10, 0), (1, 10, 1, 40, 40, 3), (2, 0, 1, 20, 20, 1)]
    op = orc.WindowOperatorOracle(assigner="session", gap=30, first=True)
    op.process(np.array([7, 7, 7]), np.array([100, 50, 75]), np.array([1, 2, 3]))
    op.watermark((1 << 63) - 1)
    rows = op.rows()
    assert len(rows) == 1 and rows[0]["count"] == 3 and rows[0]["max"] == 0 and rows[0]["start"] == 50


@pytest.mark.parametrize("case", KATS["count_windows"], ids=[c["name"] for c in KATS["count_windows"]])
def test_count_window_kats(case):
    # a14: EvictingWindowOperatorTest count-trigger / count-evictor sequences, output compared as a sorted
    # multiset after each phase (TestHarnessUtil.assertOutputEqualsSorted)
    op = orc.CountWindowOracle(case["size"], case["slide"], case["evict_after"])
    ids = {"key1": 1, "key2": 2}
    names = {v: k for k, v in ids.items()}
    expected = Counter()
    for ph in case["phases"]:
        op.process(np.array([ids[k] for k, _ in ph["input"]]), np.array([v for _, v in ph["input"]]))
        expected.update(tuple(e) for e in ph["expected"])
        got = Counter((names[int(r["key"])], int(r["sum"])) for r in op.rows())
        assert got == expected
    assert all(r["end"] == (1 << 63) - 1 for r in op.rows())


def test_count_window_word_count_shape():
    # WindowWordCount (countWindow(10, 5).sum(1)): every 5th element of a key fires the sum of its last
    # <= 10 elements; the first reduced element is the oldest one kept by the evictor
    op = orc.CountWindowOracle(10, 5)
    keys = np.array([3] * 17)
    vals = np.arange(17)
    op.process(keys, vals)
    rows = op.rows()
    assert [int(r["sum"]) for r in rows] == [sum(range(5)), sum(range(10)), sum(range(5, 15))]
    assert [int(r["max"]) for r in rows] == [0, 0, 5]
    assert [int(r["count"]) for r in rows] == [5, 10, 10]


@pytest.mark.parametrize("by", ["min", "max"])
def test_min_by_max_by_first_tie_rule(by):
    # ComparableAggregator.reduce with byAggregate and first = true (ComparableAggregator.java:72-94):
    # a strictly better field replaces the element, an equal one keeps the earlier
    op = orc.WindowOperatorOracle(assigner="tumbling", size=10, value_type="i32", by=by)
    op.process(np.array([1] * 6), np.array([0, 1, 2, 3, 4, 5]), np.array([5, 3, 7, 3, 7, 4]))
    op.watermark((1 << 63) - 1)
    (r,) = op.rows()
    assert (int(r["min"]), int(r["max"])) == ((3, 1) if by == "min" else (7, 2))
    # sessions: two sessions bridged by a third element; the merged state keeps the earlier of equal fields
    op = orc.WindowOperatorOracle(assigner="session", gap=30, value_type="i32", by=by)
    op.process(np.array([7, 7, 7]), np.array([100, 50, 75]), np.array([2, 2, 9 if by == "min" else -9]))
    op.watermark((1 << 63) - 1)
    (r,) = op.rows()
    assert (int(r["min"]), int(r["max"]), int(r["count"])) == (2, 0, 3)


def _closed_form_stream(num_keys, n_per_key):
    keys, ts, vals, wms = [], [], [], []
    for nxt in range(n_per_key):
        for k in range(num_keys):
            keys.append(k)
            ts.append(nxt)
            vals.append(nxt)
        wms.append(nxt)
    return (np.array(keys, dtype=np.int64), np.array(ts, dtype=np.int64), np.array(vals, dtype=np.int64),
            wms)


@pytest.mark.parametrize("slide", [100, 50])
def test_closed_form_validator(slide):
    cf = KATS["closed_form"]
    nk, npk, size = cf["num_keys"], cf["num_elements_per_key"], cf["window_size"]
    keys, ts, vals, wms = _closed_form_stream(nk, npk)
    assigner = "tumbling" if slide == size else "sliding"
    op = orc.WindowOperatorOracle(assigner=assigner, size=size, slide=slide, value_type="i32")
    for i, wm in enumerate(wms):
        sl = slice(i * nk, (i + 1) * nk)
        op.process(keys[sl], ts[sl], vals[sl])
        op.watermark(wm)
    op.watermark((1 << 63) - 1)
    rows = op.rows()
    per_key = Counter()
    for r in rows:
        # closed form of EWC:713-719; windows past the last element (only with slide < size) are partial
        exp = sum(i for i in range(int(r["start"]), min(int(r["end"]), npk)) if i > 0)
        assert int(r["sum"]) == exp
        per_key[int(r["key"])] += 1
    # ValidatingSink: numElementsPerKey / windowSlide windows per key (full windows only, EWC:683);
    # sliding adds the (size/slide - 1) trailing partial windows that close at the final watermark.
    expected_windows = npk // slide + (size // slide - 1)
    assert set(per_key.values()) == {expected_windows}


def test_string_hash_matches_java():
    L = orc.lib()
    # "hello".hashCode() == 99162322 (JLS String.hashCode definition)
    assert L.oracle_string_hash(b"hello", 5) == 99162322
    assert L.oracle_string_hash(b"", 0) == 0


def test_long_hash_java():
    L = orc.lib()
    assert L.oracle_long_hash(0) == 0
    assert L.oracle_long_hash(-1) == 0
    assert L.oracle_long_hash(1 << 32) == 1
    assert L.oracle_long_hash(123456789) == 123456789


# ---- f4: window-contents (ListState) operators ----------------------------------------------------------
def _list_oracle(c, **over):
    kw = dict(assigner=c["assigner"], size=c["size"], trigger=c["trigger"], trigger_count=c["trigger_count"],
              evictor=c["evictor"], evict_after=c["evict_after"], evict_arg=c["evict_arg"],
              threshold=c["threshold"], value_type="i32")
    kw.update(over)
    return orc.ListWindowOracle(**kw)


@pytest.mark.parametrize("case", KATS["list_windows"], ids=[c["name"] for c in KATS["list_windows"]])
def test_list_window_kats(case):
    # EvictingWindowOperatorTest sequences through the ListState restatement (RichSumReducer = the row's sum)
    op = _list_oracle(case["cfg"])
    for got, exp in replay_list_phases(case, KEYMAP, op):
        assert got == exp


@pytest.mark.parametrize("name", sorted(KATS["list_apply_cases"]))
def test_list_apply_kats(name):
    # WindowedStream.apply over the plain WindowOperator (ListState, EventTimeTrigger, no evictor): the same rows
    # as the reduce KATs, with the contents of every firing in arrival order
    case = next(c for c in KATS["operator_cases"] if c["name"] == name)
    c = case["cfg"]
    op = replay(case, KEYMAP, lambda _: orc.ListWindowOracle(assigner=c["assigner"], size=c["size"],
                                                             slide=c["slide"], value_type="i32"),
                flush_elements=False)
    got, _ = row_counters(op.rows(), [], case, with_window=True)
    exp, _ = expected_counters(case, KEYMAP, with_window=True)
    assert got == exp
    for r, el in op.contents():
        assert len(el) == r["count"] and el["val"].sum() == r["sum"]
        assert np.all(np.diff(el["ord"]) > 0)  # list order = arrival order


def test_list_lateness_refires_contents():
    # allowed lateness: an element of a fired, not yet cleaned-up window fires the whole list again
    # (EventTimeTrigger.onElement: maxTimestamp <= watermark -> FIRE); the cleanup timer then drops it
    op = orc.ListWindowOracle(assigner="tumbling", size=10, lateness=20)
    op.process(np.array([1, 1]), np.array([1, 2]), np.array([5, 6]))
    op.watermark(12)
    op.process(np.array([1, 1]), np.array([3, 4]), np.array([7, 8]))
    assert [int(r["count"]) for r in op.rows()] == [2, 3, 4]
    assert op.num_state_entries == 1
    op.watermark(29)
    assert op.num_state_entries == 0 and op.num_timers == 0
    op.process(np.array([1]), np.array([5]), np.array([9]))
    assert op.late_dropped == 1


@pytest.mark.parametrize("name", sorted(KATS["list_session_cases"]))
def test_list_session_kats(name):
    # f4 merging: session windows over ListState (WindowOperator / EvictingWindowOperator merging branch) against
    # WindowOperatorTest's session sequences: the rows, and every firing's contents summing to its row
    case = next(c for c in KATS["operator_cases"] if c["name"] == name)
    c = case["cfg"]
    op = replay(case, KEYMAP, lambda _: orc.ListWindowOracle(assigner="session", gap=c["gap"], lateness=c["lateness"],
                                                             purging=c["purging"], side_output=c["side_output"],
                                                             value_type="i32"),
                flush_elements=False)
    side = op.side_rows()
    side_rows = [dict(key=k, ts=t, val=v, epoch=e) for k, t, v, e in zip(*side)]
    got, got_side = row_counters(op.rows(), side_rows, case, with_window=True)
    exp, exp_side = expected_counters(case, KEYMAP, with_window=True)
    assert got == exp
    assert got_side == exp_side
    for r, el in op.contents():
        assert len(el) == r["count"] and el["val"].sum() == r["sum"]


def _java_hashset_order(wins):
    """java.util.HashSet iteration order of TimeWindows added in order (an independent restatement for the test:
    TimeWindow.hashCode = longToIntWithBitMixing(start + end), bucket (h ^ h >>> 16) & 15)."""
    def mix(x):
        M = (1 << 64) - 1
        x &= M
        x = ((x ^ (x >> 30)) * 0xbf58476d1ce4e5b9) & M
        x = ((x ^ (x >> 27)) * 0x94d049bb133111eb) & M
        x ^= x >> 31
        return x & 0xffffffff
    b = [(mix(s + e) ^ (mix(s + e) >> 16)) & 15 for s, e in wins]
    return [w for _, _, w in sorted((b[i], i, w) for i, w in enumerate(wins))]


@pytest.mark.parametrize("first", [0, 1])
def test_list_session_bridge_order(first):
    # a bridging element merges two sessions: the merged list is the state window of the first merged window in
    # HashSet order followed by the other's list (MergingWindowSet.addWindow, MergingWindowSet.java:150-225;
    # HeapListState.mergeState = addAll), then the element; pick sessions so either one comes first
    gap = 10
    for a0 in range(0, 400):
        # the in-flight windows when the bridge arrives: A = [a0, a0 + gap + 1), B = [a0 + 2 gap, a0 + 3 gap + 1)
        A, B = (a0, a0 + gap + 1), (a0 + 2 * gap, a0 + 3 * gap + 1)
        order = _java_hashset_order([A, B])
        if (order[0] == A) == (first == 0):
            break
    op = orc.ListWindowOracle(assigner="session", gap=gap, value_type="i64")
    op.process(np.array([1, 1, 1, 1]), np.array([A[0], B[0], A[0] + 1, B[0] + 1]), np.array([1, 2, 3, 4]))
    op.process(np.array([1]), np.array([A[0] + gap]), np.array([5]))  # [a0 + gap, a0 + 2 gap) touches both
    op.watermark((1 << 63) - 1)
    (r, el), = op.contents()
    assert (r["start"], r["end"]) == (A[0], B[1]) and r["count"] == 5
    expect = [1, 3, 2, 4, 5] if order[0] == A else [2, 4, 1, 3, 5]
    assert list(el["val"]) == expect
