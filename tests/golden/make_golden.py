"""Writes tests/golden/reference_kats.json: known-answer vectors transcribed (as data) from the
reference's own tests.  Every case names the reference file:line it was read from.

Run:  python tests/golden/make_golden.py

Paths are relative to /root/reference.  Abbreviations:
  WOT = flink-streaming-java/src/test/java/org/apache/flink/streaming/runtime/operators/windowing/WindowOperatorTest.java
  TWT = flink-streaming-java/src/test/java/org/apache/flink/streaming/runtime/operators/windowing/TimeWindowTest.java
  TUT = .../windowing/TumblingEventTimeWindowsTest.java
  SLT = .../windowing/SlidingEventTimeWindowsTest.java
  CEP = flink-libraries/flink-cep/src/test/java/org/apache/flink/cep/operator/CEPRescalingTest.java
  SWD = flink-examples/flink-examples-streaming/src/main/java/org/apache/flink/streaming/examples/windowing/util/SessionWindowingData.java
  SWE = flink-examples/flink-examples-streaming/src/main/java/org/apache/flink/streaming/examples/windowing/SessionWindowing.java
  EWO = flink-streaming-java/src/test/java/org/apache/flink/streaming/runtime/operators/windowing/EvictingWindowOperatorTest.java
  EWC = flink-tests/src/test/java/org/apache/flink/test/checkpointing/AbstractEventTimeWindowCheckpointingITCase.java
  SIT = flink-libraries/flink-table/src/test/scala/org/apache/flink/table/runtime/stream/sql/SqlITCase.scala
  GWT = flink-libraries/flink-table/src/test/scala/org/apache/flink/table/runtime/stream/table/GroupWindowITCase.scala

Operator cases use the vocabulary of the harness: ("e", key, value, timestamp) is
processElement, ("w", t) is processWatermark.  Expected rows carry the output epoch (the
index of the first watermark that follows them in the output; TestHarnessUtil.java:70-108
compares watermark positions exactly and records sorted in between), the key, the aggregated
sum, the record timestamp (= window.maxTimestamp()) and, where the window function prints
them, the window start/end.  The harness keys are Strings; they are dictionary-encoded here
(key1 -> 1, key2 -> 2) — window results do not depend on the key's hash.
"""
import json
import os

MAX = (1 << 63) - 1


def E(k, v, t):
    return ["e", k, v, t]


def W(t):
    return ["w", t]


def row(epoch, key, s, ts, start=None, end=None):
    r = {"epoch": epoch, "key": key, "sum": s, "ts": ts}
    if start is not None:
        r["start"] = start
        r["end"] = end
    return r


def side(epoch, key, v, ts):
    return {"epoch": epoch, "key": key, "value": v, "ts": ts}


KEYS = {"key1": 1, "key2": 2}
ELEMS_8 = [E("key2", 1, 3999), E("key2", 1, 3000), E("key1", 1, 20), E("key1", 1, 0), E("key1", 1, 999),
           E("key2", 1, 1998), E("key2", 1, 1999), E("key2", 1, 1000)]

# Session sequence shared by WOT:1715-2266 (gap 3 s)
SESSION_PREFIX = [E("key2", 1, 1000), W(1999), E("key2", 1, 2000), W(4998), E("key2", 1, 4500), E("key2", 1, 8500),
                  W(7400), E("key2", 1, 7000), W(11501), E("key2", 1, 11600), W(14600)]
SESSION_PREFIX_ROWS = [row(3, "key2", 5, 11499, 1000, 11500), row(4, "key2", 1, 14599, 11600, 14600)]


def cfg(assigner, size=0, slide=0, gap=0, lateness=0, purging=False, side_output=False, offset=0):
    return {"assigner": assigner, "size": size, "slide": slide, "offset": offset, "gap": gap,
            "lateness": lateness, "purging": purging, "side_output": side_output, "value_type": "i32"}


CASES = [
    {"name": "sliding_3s_1s_reduce_sum", "source": "WOT:108-181,185-210",
     "cfg": cfg("sliding", size=3000, slide=1000),
     "events": ELEMS_8 + [W(999), W(1999), W(2999), W(3999), W(4999), W(5999), W(6999), W(7999)],
     "expected": [row(0, "key1", 3, 999),
                  row(1, "key1", 3, 1999), row(1, "key2", 3, 1999),
                  row(2, "key1", 3, 2999), row(2, "key2", 3, 2999),
                  row(3, "key2", 5, 3999), row(4, "key2", 2, 4999), row(5, "key2", 2, 5999)],
     "expected_side": []},
    {"name": "tumbling_3s_reduce_sum", "source": "WOT:241-308,312-335",
     "cfg": cfg("tumbling", size=3000),
     "events": ELEMS_8 + [W(999), W(1999), W(2999), W(3999), W(4999), W(5999), W(6999), W(7999)],
     "expected": [row(2, "key1", 3, 2999), row(2, "key2", 3, 2999), row(5, "key2", 2, 5999)],
     "expected_side": []},
    {"name": "session_3s_sum", "source": "WOT:368-442 (same rows as testReduceSessionWindows WOT:524-596)",
     "cfg": cfg("session", gap=3000),
     "events": [E("key2", 1, 0), E("key2", 2, 1000), E("key2", 3, 2500), E("key1", 1, 10), E("key1", 2, 1000),
                E("key1", 3, 2500), E("key2", 4, 5501), E("key2", 5, 6000), E("key2", 5, 6000), E("key2", 6, 6050),
                W(12000), E("key2", 10, 15000), E("key2", 20, 15000), W(17999)],
     "expected": [row(0, "key1", 6, 5499, 10, 5500), row(0, "key2", 6, 5499, 0, 5500),
                  row(0, "key2", 20, 9049, 5501, 9050), row(1, "key2", 30, 17999, 15000, 18000)],
     "expected_side": []},
    {"name": "lateness_tumbling_2s_purging", "source": "WOT:1434-1499",
     "cfg": cfg("tumbling", size=2000, lateness=500, purging=True, side_output=True),
     "events": [E("key2", 1, 500), W(1500), E("key2", 1, 1300), W(2300), E("key2", 1, 1997), W(6000),
                E("key2", 1, 1998), W(7000)],
     "expected": [row(1, "key2", 2, 1999), row(2, "key2", 1, 1999)],
     "expected_side": [side(3, "key2", 1, 1998)]},
    {"name": "cleanup_time_overflow", "source": "WOT:1502-1568",
     "cfg": cfg("tumbling", size=1000, lateness=2000),
     "events": [E("key2", 1, MAX - 1750), W(MAX - 1500), W(9223372036854774999)],
     "expected": [row(1, "key2", 1, 9223372036854774999, 9223372036854774000, 9223372036854775000)],
     "expected_side": []},
    {"name": "side_output_tumbling_2s", "source": "WOT:1571-1632",
     "cfg": cfg("tumbling", size=2000, side_output=True),
     "events": [E("key2", 1, 1000), W(1985), E("key2", 1, 1980), W(1999), E("key2", 1, 1998), E("key2", 1, 2001),
                W(2999), W(3999)],
     "expected": [row(1, "key2", 2, 1999), row(3, "key2", 1, 3999)],
     "expected_side": [side(2, "key2", 1, 1998)]},
    {"name": "side_output_sliding_3s_1s", "source": "WOT:1635-1712",
     "cfg": cfg("sliding", size=3000, slide=1000, side_output=True),
     "events": [E("key2", 1, 1000), W(1999), E("key2", 1, 2000), W(3000), E("key1", 1, 3001), E("key2", 1, 2400),
                E("key2", 1, 2400), E("key1", 1, 3001), E("key2", 1, 3900), W(6000), E("key1", 1, 3001), W(25000)],
     "expected": [row(0, "key2", 1, 1999), row(1, "key2", 2, 2999),
                  row(2, "key2", 5, 3999), row(2, "key1", 2, 3999), row(2, "key2", 4, 4999),
                  row(2, "key1", 2, 4999), row(2, "key2", 1, 5999), row(2, "key1", 2, 5999)],
     "expected_side": [side(3, "key1", 1, 3001)]},
    {"name": "session_zero_lateness_purging_side_output", "source": "WOT:1715-1804",
     "cfg": cfg("session", gap=3000, purging=True, side_output=True),
     "events": SESSION_PREFIX + [E("key2", 1, 10000), E("key2", 1, 10100), E("key2", 1, 14500), W(20000),
                                 W(100000)],
     "expected": SESSION_PREFIX_ROWS + [row(5, "key2", 1, 17499, 14500, 17500)],
     "expected_side": [side(5, "key2", 1, 10000), side(5, "key2", 1, 10100)]},
    {"name": "session_zero_lateness_side_output", "source": "WOT:1807-1890",
     "cfg": cfg("session", gap=3000, side_output=True),
     "events": SESSION_PREFIX + [E("key2", 1, 10000), E("key2", 1, 14500), W(20000), W(100000)],
     "expected": SESSION_PREFIX_ROWS + [row(5, "key2", 1, 17499, 14500, 17500)],
     "expected_side": [side(5, "key2", 1, 10000)]},
    {"name": "session_lateness_10_purging", "source": "WOT:1893-1977",
     "cfg": cfg("session", gap=3000, lateness=10, purging=True, side_output=True),
     "events": SESSION_PREFIX + [E("key2", 1, 10000), E("key2", 1, 14500), W(20000), W(100000)],
     "expected": SESSION_PREFIX_ROWS + [row(5, "key2", 1, 14599, 10000, 14600),
                                        row(5, "key2", 1, 17499, 10000, 17500)],
     "expected_side": []},
    {"name": "session_lateness_10_accumulating", "source": "WOT:1980-2081",
     "cfg": cfg("session", gap=3000, lateness=10),
     "events": SESSION_PREFIX + [E("key2", 1, 10000), E("key2", 1, 14500), W(20000), W(100000)],
     "expected": SESSION_PREFIX_ROWS + [row(5, "key2", 2, 14599, 10000, 14600),
                                        row(5, "key2", 3, 17499, 10000, 17500)],
     "expected_side": []},
    {"name": "session_huge_lateness_purging", "source": "WOT:2084-2173",
     "cfg": cfg("session", gap=3000, lateness=10000, purging=True),
     "events": SESSION_PREFIX + [E("key2", 1, 10000), E("key2", 1, 14500), W(20000), W(100000)],
     "expected": SESSION_PREFIX_ROWS + [row(5, "key2", 1, 14599, 1000, 14600),
                                        row(5, "key2", 1, 17499, 1000, 17500)],
     "expected_side": []},
    {"name": "session_huge_lateness_accumulating", "source": "WOT:2176-2266",
     "cfg": cfg("session", gap=3000, lateness=10000),
     "events": SESSION_PREFIX + [E("key2", 1, 10000), E("key2", 1, 14500), W(20000), W(100000)],
     "expected": SESSION_PREFIX_ROWS + [row(5, "key2", 7, 14599, 1000, 14600),
                                        row(5, "key2", 8, 17499, 1000, 17500)],
     "expected_side": []},
]

# SessionWindowing example: keyBy(0).window(EventTimeSessionWindows.withGap(3 ms)).sum(2), a watermark
# of (ts - 1) after every element and Long.MAX_VALUE at the end (SWE:57-83).  EXPECTED (SWD:26-27) is
# (key, f1 of the FIRST element of the session, sum) — for this input the first element of every
# session is also its earliest, so f1 == window start.
SESSION_EXAMPLE = {
    "source": "SWE:57-83, SWD:26-27",
    "gap": 3,
    "input": [["a", 1, 1], ["b", 1, 1], ["b", 3, 1], ["b", 5, 1], ["c", 6, 1], ["a", 10, 1], ["c", 11, 1]],
    "expected": [["a", 1, 1], ["c", 6, 1], ["c", 11, 1], ["b", 1, 3], ["a", 10, 1]],
}

# a14: EvictingWindowOperator over GlobalWindows with CountTrigger.of(slide) and CountEvictor.of(size[, after]);
# elements ("key", value) in order (timestamps are ignored by GlobalWindows); `expected` rows are
# (key, summed value) with timestamp Long.MAX_VALUE, compared as a sorted multiset after each phase.
_EW_INPUT = [["key2", 1], ["key2", 1], ["key1", 1], ["key1", 1], ["key1", 1], ["key2", 1], ["key2", 1],
             ["key2", 1]]
COUNT_WINDOWS = [
    {"name": "count_evictor_evict_after", "source": "EWO:73-142", "size": 4, "slide": 2, "evict_after": True,
     "phases": [{"input": _EW_INPUT, "expected": [["key2", 2], ["key2", 4], ["key1", 2]]},
                {"input": [["key1", 1], ["key2", 1]], "expected": [["key1", 4], ["key2", 6]]},
                {"input": [["key2", 1], ["key2", 1]], "expected": [["key2", 6]]}]},
    {"name": "count_trigger_evict_before", "source": "EWO:505-572", "size": 4, "slide": 2, "evict_after": False,
     "phases": [{"input": _EW_INPUT, "expected": [["key2", 2], ["key2", 4], ["key1", 2]]},
                {"input": [["key1", 1], ["key2", 1]], "expected": [["key1", 4], ["key2", 4]]}]},
]

# f4: window-contents (ListState) operators with an Iterable window function — RichSumReducer (EWO:720-760:
# output (key, sum of f1 over the contents)).  Each case is an EvictingWindowOperator; events as in CASES
# (timestamps None = a StreamRecord without timestamp); `expected` of a phase lists the rows (key, sum,
# timestamp) emitted up to its end, compared as a sorted multiset (TestHarnessUtil.assertOutputEqualsSorted).
def lcfg(assigner, trigger, trigger_count=0, evictor="none", evict_after=False, evict_arg=0, threshold=0.0, size=0):
    return {"assigner": assigner, "size": size, "trigger": trigger, "trigger_count": trigger_count,
            "evictor": evictor, "evict_after": evict_after, "evict_arg": evict_arg, "threshold": threshold}


def R(key, s, ts):
    return [key, s, ts]


_TE_A = [E("key2", 1, 1000), E("key2", 1, 4000), E("key1", 1, 20), E("key1", 1, 0), E("key1", 1, 999),
         E("key2", 1, 3500), E("key2", 1, 2001), E("key2", 1, 1001)]
_NO_TS = [E("key2", 1, None), E("key2", 1, None), E("key1", 1, None), E("key1", 1, None), E("key1", 1, None),
          E("key2", 1, None), E("key2", 1, None), E("key2", 1, None)]
_DELTA = [E("key2", 1, 3000), E("key2", 4, 3999), E("key1", 1, 20), E("key1", 1, 0), E("key1", 5, 999),
          E("key2", 5, 1998), E("key2", 6, 1999), E("key2", 1, 1000)]
LIST_WINDOWS = [
    {"name": "time_evictor_evict_after", "source": "EWO:148-212",
     "cfg": lcfg("global", "count", 2, "time", True, 2000),
     "phases": [{"events": _TE_A, "expected": [R("key2", 2, MAX), R("key1", 2, MAX), R("key2", 3, MAX)]},
                {"events": [E("key1", 1, 10999), E("key2", 1, 1002)],
                 "expected": [R("key2", 2, MAX), R("key1", 2, MAX), R("key2", 3, MAX), R("key1", 4, MAX),
                              R("key2", 5, MAX)]}]},
    {"name": "time_evictor_evict_before", "source": "EWO:218-283",
     "cfg": lcfg("tumbling", "count", 2, "time", False, 2000, size=4000),
     "phases": [{"events": [E("key2", 1, 1000), E("key2", 1, 3999), E("key1", 1, 20), E("key1", 1, 0),
                            E("key1", 1, 999), E("key1", 1, 5999), E("key2", 1, 3500), E("key2", 1, 2001),
                            E("key2", 1, 1001)],
                 "expected": [R("key2", 1, 3999), R("key1", 2, 3999), R("key2", 3, 3999)]},
                {"events": [E("key1", 1, 6500), E("key2", 1, 1002)],
                 "expected": [R("key2", 1, 3999), R("key1", 2, 3999), R("key2", 3, 3999), R("key1", 2, 7999),
                              R("key2", 3, 3999)]}]},
    {"name": "time_evictor_no_timestamp", "source": "EWO:289-352",
     "cfg": lcfg("global", "count", 2, "time", True, 2000),
     "phases": [{"events": _NO_TS, "expected": [R("key2", 2, MAX), R("key1", 2, MAX), R("key2", 4, MAX)]},
                {"events": [E("key1", 1, None), E("key2", 1, None)],
                 "expected": [R("key2", 2, MAX), R("key1", 2, MAX), R("key2", 4, MAX), R("key1", 4, MAX),
                              R("key2", 6, MAX)]}]},
    {"name": "delta_evictor_evict_before", "source": "EWO:357-428 (delta = new.f1 - old.f1)",
     "cfg": lcfg("global", "count", 2, "delta", False, threshold=2.0),
     "phases": [{"events": _DELTA, "expected": [R("key2", 4, MAX), R("key2", 11, MAX), R("key1", 2, MAX)]},
                {"events": [E("key1", 3, 10999), E("key2", 10, 1000)],
                 "expected": [R("key2", 4, MAX), R("key2", 11, MAX), R("key1", 2, MAX), R("key1", 8, MAX),
                              R("key2", 10, MAX)]}]},
    {"name": "delta_evictor_evict_after", "source": "EWO:432-500 (delta = new.f1 - old.f1)",
     "cfg": lcfg("global", "count", 2, "delta", True, threshold=2.0),
     "phases": [{"events": _DELTA, "expected": [R("key2", 5, MAX), R("key2", 15, MAX), R("key1", 2, MAX)]},
                {"events": [E("key1", 9, 10999), E("key2", 10, 1000)],
                 "expected": [R("key2", 5, MAX), R("key2", 15, MAX), R("key1", 2, MAX), R("key1", 16, MAX),
                              R("key2", 22, MAX)]}]},
    {"name": "count_evictor_evict_after", "source": "EWO:73-142",
     "cfg": lcfg("global", "count", 2, "count", True, 4),
     "phases": [{"events": [E(k, v, None) for k, v in _EW_INPUT],
                 "expected": [R("key2", 2, MAX), R("key2", 4, MAX), R("key1", 2, MAX)]},
                {"events": [E("key1", 1, None), E("key2", 1, None)],
                 "expected": [R("key2", 2, MAX), R("key2", 4, MAX), R("key1", 2, MAX), R("key1", 4, MAX),
                              R("key2", 6, MAX)]}]},
    {"name": "tumbling_with_apply_count_evictor", "source": "EWO:645-697",
     "cfg": lcfg("tumbling", "event_time", 0, "count", False, 4, size=4000),
     "phases": [{"events": [E("key1", 1, 10), E("key1", 1, 100), W(1999), E("key1", 1, 1997), E("key1", 1, 1998),
                            E("key1", 1, 2310), E("key1", 1, 2310), E("key2", 1, 2310), E("key2", 1, 2310),
                            W(3999)],
                 "expected": [R("key1", 4, 3999), R("key2", 2, 3999)]}]},
]
# WindowedStream.apply with the plain WindowOperator (ListState, no evictor): the WOT sequences of
# CASES "sliding_3s_1s_reduce_sum" (testSlidingEventTimeWindowsApply, WOT:213-238) and "tumbling_3s_reduce_sum"
# (testTumblingEventTimeWindowsApply, WOT:339-364) produce the same rows through RichSumReducer.
LIST_APPLY_CASES = {"sliding_3s_1s_reduce_sum": "WOT:213-238", "tumbling_3s_reduce_sum": "WOT:339-364"}
# f4 merging: session windows over ListState (WindowedStream.apply with EventTimeSessionWindows).  testSessionWindows
# (WOT:368-442) is that operator itself (ListStateDescriptor + SessionWindowFunction: key-sum over the contents); the
# lateness / purging / side-output session sequences (WOT:1715-2266) are written against a ReducingState sum, and
# WindowOperator's merging branch (WindowOperator.java:300-377) does not depend on the state kind, so a sum over the
# list's contents gives the same rows.
LIST_SESSION_CASES = {"session_3s_sum": "WOT:368-442", "session_zero_lateness_purging_side_output": "WOT:1715-1804",
                      "session_zero_lateness_side_output": "WOT:1807-1890",
                      "session_lateness_10_purging": "WOT:1893-1977",
                      "session_lateness_10_accumulating": "WOT:1980-2081",
                      "session_huge_lateness_purging": "WOT:2084-2173",
                      "session_huge_lateness_accumulating": "WOT:2176-2266"}

KEY_GROUPS = {
    "source": "CEP:71-82,170-215 (Integer keys: hashCode == value)",
    "max_parallelism": 10,
    "key_group": [[7, 1], [10, 9], [45, 6], [90, 2]],
    # [maxPar, parallelism, keyGroup, operatorIndex]
    "operator_index": [[10, 2, 1, 0], [10, 2, 9, 1], [10, 3, 1, 0], [10, 2, 6, 1], [10, 3, 6, 1],
                       [10, 3, 2, 0], [10, 2, 2, 0], [10, 3, 9, 2]],
}

WINDOW_START = {
    "source": "TWT:33-61",
    # [timestamp, offset, size, expected start]
    "cases": [[1, 0, 7, 0], [6, 0, 7, 0], [7, 0, 7, 7], [8, 0, 7, 7],
              [1, 3, 7, -4], [2, 3, 7, -4], [3, 3, 7, 3], [9, 3, 7, 3], [10, 3, 7, 10],
              [1, -2, 7, -2], [-2, -2, 7, -2], [3, -2, 7, -2], [4, -2, 7, -2], [7, -2, 7, 5], [12, -2, 7, 12],
              [1470902048450, -8 * 3600 * 1000, 24 * 3600 * 1000, 1470844800000]],
}

ASSIGNERS = {
    "source": "TUT:48-83, SLT:48-136",
    # [kind, size, slide, offset, timestamp, [[start, end], ...]]
    "cases": [
        ["tumbling", 5000, 0, 0, 0, [[0, 5000]]], ["tumbling", 5000, 0, 0, 4999, [[0, 5000]]],
        ["tumbling", 5000, 0, 0, 5000, [[5000, 10000]]],
        ["tumbling", 5000, 0, 100, 100, [[100, 5100]]], ["tumbling", 5000, 0, 100, 5099, [[100, 5100]]],
        ["tumbling", 5000, 0, 100, 5100, [[5100, 10100]]],
        ["tumbling", 5000, 0, 1000, 1000, [[1000, 6000]]], ["tumbling", 5000, 0, 1000, 5999, [[1000, 6000]]],
        ["tumbling", 5000, 0, 1000, 6000, [[6000, 11000]]],
        ["sliding", 5000, 1000, 0, 0, [[-4000, 1000], [-3000, 2000], [-2000, 3000], [-1000, 4000], [0, 5000]]],
        ["sliding", 5000, 1000, 0, 4999, [[0, 5000], [1000, 6000], [2000, 7000], [3000, 8000], [4000, 9000]]],
        ["sliding", 5000, 1000, 0, 5000, [[1000, 6000], [2000, 7000], [3000, 8000], [4000, 9000], [5000, 10000]]],
        ["sliding", 5000, 1000, 100, 100, [[-3900, 1100], [-2900, 2100], [-1900, 3100], [-900, 4100], [100, 5100]]],
        ["sliding", 5000, 1000, 100, 5099, [[100, 5100], [1100, 6100], [2100, 7100], [3100, 8100], [4100, 9100]]],
        ["sliding", 5000, 1000, 100, 5100,
         [[1100, 6100], [2100, 7100], [3100, 8100], [4100, 9100], [5100, 10100]]],
        ["sliding", 5000, 1000, 500, 100, [[-4500, 500], [-3500, 1500], [-2500, 2500], [-1500, 3500], [-500, 4500]]],
        ["sliding", 5000, 1000, 500, 5499, [[500, 5500], [1500, 6500], [2500, 7500], [3500, 8500], [4500, 9500]]],
        ["sliding", 5000, 1000, 500, 5100, [[500, 5500], [1500, 6500], [2500, 7500], [3500, 8500], [4500, 9500]]],
    ],
}

# EWC:571-629 (FailingSource without the failure), EWC:659-740 (ValidatingSink), EWC:865-877 defaults:
# for next in 0..numElementsPerKey-1: for key in 0..numKeys-1: emit (key, next) at ts=next; then
# watermark(next).  Every window holds sum(i for i in [start, end) if i > 0), and every key sees
# exactly numElementsPerKey / windowSlide windows (tumbling: / windowSize).
CLOSED_FORM = {"source": "EWC:571-629,659-740,865-877", "num_keys": 20, "num_elements_per_key": 300,
               "window_size": 100, "window_slide": 100}


# f3: Table API group windows (DataStreamGroupWindowAggregate.scala:197-294) -- the built-in aggregates of the
# reference's own ITCases, with their inputs (rowtime = the first tuple field, a punctuated watermark of ts - offset
# after every element: TimestampAndWatermarkWithOffset, SIT:645-659 / GWT:449-463; Long.MAX_VALUE at the end of the
# input).  "cols" are the aggregated columns (null = SQL NULL), "specs" the select list's built-in aggregates as
# [function, column index]; "expected" rows are [key, window start, window end, [values (null = NULL)]] -- the
# ITCase's expected strings with the user-defined aggregates (WeightedAvg, CountDistinct) left out and the keys as
# strings (None = the null grouping key).  User AggregateFunctions of the tests (countFun = the test's
# CountAggFunction: the non-null count of its argument) are the built-in COUNT(col).
_GW_DATA = [[1, [1], "Hi"], [2, [2], "Hello"], [4, [2], "Hello"], [8, [3], "Hello world"], [16, [3], "Hello world"]]
_GW_DATA2 = [[1, [1], "Hi"], [2, [2], "Hallo"], [3, [2], "Hello"], [4, [5], "Hello"], [7, [3], "Hello"],
             [8, [3], "Hello world"], [16, [4], "Hello world"], [32, [4], None]]


def _slide_rows(rows):
    return [[k, s, e, [c]] for k, c, s, e in rows]


TABLE_GROUP_WINDOWS = [
    {"name": "sql_tumble_count_star_count_col", "source": "SIT:44-82 (testRowTimeTumbleWindow)",
     "assigner": "tumbling", "size": 5000, "offset": 0, "types": ["i64"],
     "specs": [["count_star", 0], ["count_star", 0], ["count", 0]],
     "input": [[1000, [1], "Hello"], [2000, [2], "Hello"], [3000, [None], "Hello"], [4000, [4], "Hello"],
               [5000, [None], "Hello"], [6000, [6], "Hello"], [7000, [7], "Hello World"], [8000, [8], "Hello World"],
               [20000, [20], "Hello World"]],
     "expected": [["Hello World", 5000, 10000, [2, 2, 2]], ["Hello World", 20000, 25000, [1, 1, 1]],
                  ["Hello", 0, 5000, [4, 4, 3]], ["Hello", 5000, 10000, [2, 2, 1]]]},
    {"name": "table_tumble_builtins", "source": "GWT:50-55,169-201 (testEventTimeTumblingWindow)",
     "assigner": "tumbling", "size": 5, "offset": 0, "types": ["i32"],
     "specs": [["count", 0], ["avg", 0], ["min", 0], ["max", 0], ["sum", 0]],
     "input": _GW_DATA,
     "expected": [["Hello world", 5, 10, [1, 3, 3, 3, 3]], ["Hello world", 15, 20, [1, 3, 3, 3, 3]],
                  ["Hello", 0, 5, [2, 2, 2, 2, 4]], ["Hi", 0, 5, [1, 1, 1, 1, 1]]]},
    {"name": "table_session_merge", "source": "GWT:97-138 (testEventTimeSessionGroupWindowOverTime)",
     "assigner": "session", "gap": 5, "offset": 10, "types": ["i32"], "specs": [["count", 0], ["avg", 0]],
     "input": [[1, [1], "Hello"], [2, [2], "Hello"], [8, [8], "Hello"], [9, [9], "Hello World"], [4, [4], "Hello"],
               [16, [16], "Hello"]],
     "expected": [["Hello World", 9, 14, [1, 9]], ["Hello", 16, 21, [1, 16]], ["Hello", 1, 13, [4, 3]]]},
    {"name": "table_slide_all_overlapping", "source": "GWT:57-65,240-277 (testAllEventTimeSlidingGroupWindowOverTime)",
     "assigner": "sliding", "size": 5, "slide": 2, "offset": 0, "types": ["i32"], "specs": [["count", 0]],
     "input": [[t, c, "all"] for t, c, _ in _GW_DATA2],
     "expected": _slide_rows([["all", 1, 8, 13], ["all", 1, 12, 17], ["all", 1, 14, 19], ["all", 1, 16, 21],
                              ["all", 2, -2, 3], ["all", 2, 6, 11], ["all", 3, 2, 7], ["all", 3, 4, 9],
                              ["all", 4, 0, 5], ["all", 1, 28, 33], ["all", 1, 30, 35], ["all", 1, 32, 37]])},
    {"name": "table_slide_overlapping_full_pane", "source": "GWT:57-65,279-317", "assigner": "sliding",
     "size": 10, "slide": 5, "offset": 0, "types": ["i32"], "specs": [["count", 0]], "input": _GW_DATA2,
     "expected": _slide_rows([["Hallo", 1, -5, 5], ["Hallo", 1, 0, 10], ["Hello world", 1, 0, 10],
                              ["Hello world", 1, 5, 15], ["Hello world", 1, 10, 20], ["Hello world", 1, 15, 25],
                              ["Hello", 1, 5, 15], ["Hello", 2, -5, 5], ["Hello", 3, 0, 10], ["Hi", 1, -5, 5],
                              ["Hi", 1, 0, 10], [None, 1, 25, 35], [None, 1, 30, 40]])},
    {"name": "table_slide_overlapping_split_pane", "source": "GWT:57-65,319-354", "assigner": "sliding",
     "size": 5, "slide": 4, "offset": 0, "types": ["i32"], "specs": [["count", 0]], "input": _GW_DATA2,
     "expected": _slide_rows([["Hallo", 1, 0, 5], ["Hello world", 1, 4, 9], ["Hello world", 1, 8, 13],
                              ["Hello world", 1, 12, 17], ["Hello world", 1, 16, 21], ["Hello", 2, 0, 5],
                              ["Hello", 2, 4, 9], ["Hi", 1, 0, 5], [None, 1, 28, 33], [None, 1, 32, 37]])},
    {"name": "table_slide_non_overlapping_full_pane", "source": "GWT:57-65,356-385", "assigner": "sliding",
     "size": 5, "slide": 10, "offset": 0, "types": ["i32"], "specs": [["count", 0]], "input": _GW_DATA2,
     "expected": _slide_rows([["Hallo", 1, 0, 5], ["Hello", 2, 0, 5], ["Hi", 1, 0, 5], [None, 1, 30, 35]])},
    {"name": "table_slide_non_overlapping_split_pane", "source": "GWT:57-65,387-415", "assigner": "sliding",
     "size": 3, "slide": 10, "offset": 0, "types": ["i32"], "specs": [["count", 0]], "input": _GW_DATA2,
     "expected": _slide_rows([["Hallo", 1, 0, 3], ["Hi", 1, 0, 3], [None, 1, 30, 33]])},
]


def main():
    out = {"keys": KEYS, "operator_cases": CASES, "session_example": SESSION_EXAMPLE, "count_windows": COUNT_WINDOWS,
           "list_windows": LIST_WINDOWS, "list_apply_cases": LIST_APPLY_CASES, "key_groups": KEY_GROUPS,
           "window_start": WINDOW_START, "assigners": ASSIGNERS, "closed_form": CLOSED_FORM,
           "table_group_windows": TABLE_GROUP_WINDOWS, "list_session_cases": LIST_SESSION_CASES}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
