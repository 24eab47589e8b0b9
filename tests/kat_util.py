"""Helpers that replay a reference KAT (tests/golden/reference_kats.json) through an operator."""
import json
import os
from collections import Counter

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_kats.json")


def load_kats():
    with open(GOLDEN) as f:
        return json.load(f)


def replay(case, keymap, make_op, flush_elements=True):
    """Replay ('e', key, value, ts) / ('w', t) events.  Consecutive elements are handed over as
    one batch (the GPU operator's micro-batch; the oracle processes them one by one).  Returns
    (rows as Counter of (epoch, key, sum, ts[, start, end]), side rows Counter)."""
    op = make_op(case["cfg"])
    rows, side = [], []
    pend = []
    epoch = 0

    def flush():
        if pend:
            k = np.array([keymap[p[1]] for p in pend], dtype=np.int64)
            v = np.array([p[2] for p in pend], dtype=np.int64)
            t = np.array([p[3] for p in pend], dtype=np.int64)
            op.process(k, t, v)
            pend.clear()

    for ev in case["events"]:
        if ev[0] == "e":
            pend.append(ev)
            if not flush_elements:
                flush()
        else:
            flush()
            op.watermark(ev[1])
            epoch += 1
    flush()
    return op


def expected_counters(case, keymap, with_window):
    exp = Counter()
    for r in case["expected"]:
        t = (r["epoch"], keymap[r["key"]], r["sum"], r["ts"])
        if with_window and "start" in r:
            t = t + (r["start"], r["end"])
        exp[t] += 1
    side = Counter((s["epoch"], keymap[s["key"]], s["value"], s["ts"]) for s in case["expected_side"])
    return exp, side


def row_counters(rows, side_rows, case, with_window):
    got = Counter()
    has_window = any("start" in r for r in case["expected"])
    for r in rows:
        t = (int(r["epoch"]), int(r["key"]), int(r["sum"]), int(r["end"]) - 1)
        if with_window and has_window:
            t = t + (int(r["start"]), int(r["end"]))
        got[t] += 1
    side = Counter((int(s["epoch"]), int(s["key"]), int(s["val"]), int(s["ts"])) for s in side_rows)
    return got, side


LMIN, LMAX = -(1 << 63), (1 << 63) - 1


def row_ts(start, end):
    """the row's record timestamp: window.maxTimestamp() (GlobalWindow: Long.MAX_VALUE)"""
    return LMAX if (start == LMIN and end == LMAX) else end - 1


def replay_list_phases(case, keymap, op, watermark_epochs=False):
    """f4 KATs (reference_kats.json "list_windows"): replays each phase's events through `op` (process(k, t, v),
    watermark(t), rows() with key / start / end / sum), consecutive elements as one batch; after each phase
    yields (got, expected) Counters of (key, sum, timestamp) over everything emitted so far (a missing
    timestamp is Long.MIN_VALUE: StreamRecord without one)."""
    for ph in case["phases"]:
        pend = []

        def flush():
            if pend:
                op.process(np.array([keymap[p[1]] for p in pend], dtype=np.int64),
                           np.array([LMIN if p[3] is None else p[3] for p in pend], dtype=np.int64),
                           np.array([p[2] for p in pend], dtype=np.int64))
                pend.clear()

        for ev in ph["events"]:
            if ev[0] == "e":
                pend.append(ev)
            else:
                flush()
                op.watermark(ev[1])
        flush()
        expected = Counter((keymap[k], s, t) for k, s, t in ph["expected"])  # cumulative, as in the test
        got = Counter((int(r["key"]), int(r["sum"]), row_ts(int(r["start"]), int(r["end"]))) for r in op.rows())
        yield got, expected
