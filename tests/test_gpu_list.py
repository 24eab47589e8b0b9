"""f4 GPU parity: GpuListWindowOperator (fw_list_*, libflinkwin.so) — WindowedStream.apply / process over
ListState and the EvictingWindowOperator — against the reference KATs (EvictingWindowOperatorTest,
WindowOperatorTest apply sequences) and against the ListState oracle (oracle/list_oracle.cpp) on seeded streams.
Bar: rows (key, window, count, integer sum / min / max, first ordinal) and the contents of every firing
bit-exact; f64 sums are summed in list order on both sides, so they are bit-exact too."""
from collections import Counter

import numpy as np
import pytest

from flink_amd import (CountEvictor, CountTrigger, DeltaEvictor, EventTimeSessionWindows, EventTimeTrigger,
                       GlobalWindows, PurgingTrigger, SlidingEventTimeWindows, TimeEvictor, TumblingEventTimeWindows)
from oracle import oracle as orc
from tests.kat_util import expected_counters, load_kats, replay, replay_list_phases, row_counters

pytestmark = pytest.mark.gpu

KATS = load_kats()
KEYMAP = KATS["keys"]
_VT = {"i64": "long", "i32": "int", "f64": "double", "i16": "short", "i8": "byte", "f32": "float"}


def _assigner(kind, size=0, slide=0, offset=0, gap=0):
    if kind == "global":
        return GlobalWindows.create()
    if kind == "session":
        return EventTimeSessionWindows.with_gap(gap)
    if kind == "tumbling":
        return TumblingEventTimeWindows.of(size, offset)
    return SlidingEventTimeWindows.of(size, slide, offset)


def _evictor(kind, after, arg, threshold):
    return {"none": None, "count": lambda: CountEvictor.of(arg, after), "time": lambda: TimeEvictor.of(arg, after),
            "delta": lambda: DeltaEvictor.of(threshold, after)}[kind]() if kind != "none" else None


def _pair(assigner="tumbling", size=0, slide=0, offset=0, lateness=0, trigger="event_time", trigger_count=0,
          purging=False, evictor="none", evict_after=False, evict_arg=0, threshold=0.0, side_output=False,
          value_type="i64", gap=0, **gpu_kw):
    """(GPU operator, oracle) of one configuration"""
    from flink_amd.listwindow import GpuListWindowOperator
    trig = CountTrigger.of(trigger_count) if trigger == "count" else EventTimeTrigger.create()
    if purging:
        trig = PurgingTrigger.of(trig)
    gpu = GpuListWindowOperator(_assigner(assigner, size, slide, offset, gap), trig,
                                _evictor(evictor, evict_after, evict_arg, threshold), allowed_lateness=lateness,
                                side_output=side_output, value_type=_VT[value_type], **gpu_kw)
    kw = dict(gap=gap) if assigner == "session" else dict(size=size, slide=slide, offset=offset)
    ref = orc.ListWindowOracle(assigner=assigner, lateness=lateness, trigger=trigger, trigger_count=trigger_count,
                               purging=purging, evictor=evictor, evict_after=evict_after, evict_arg=evict_arg,
                               threshold=threshold, side_output=side_output, value_type=value_type, **kw)
    return gpu, ref


def _firings(op, ordinals=True):
    """Counter of every firing: (epoch, key, start, end, count, sum, min, max[, first], contents)"""
    out = Counter()
    for r, el in op.contents():
        ords = "ordinal" if "ordinal" in el.dtype.names else "ord"
        cont = (tuple(zip(el["ts"].tolist(), el["val"].tolist(), el[ords].tolist())) if ordinals
                else tuple(zip(el["ts"].tolist(), el["val"].tolist())))
        out[(int(r["epoch"]), int(r["key"]), int(r["start"]), int(r["end"]), int(r["count"]), int(r["sum"]),
             int(r["min"]), int(r["max"])) + ((int(r["first"]),) if ordinals else ()) + (cont,)] += 1
    return out


def _assert_same(gpu, ref):
    g, r = _firings(gpu), _firings(ref)
    assert sum(g.values()) == sum(r.values()), (sum(g.values()), sum(r.values()))
    assert g == r, (list((g - r).items())[:3], list((r - g).items())[:3])


# ---------------------------------------------------------------- reference KATs
@pytest.mark.parametrize("case", KATS["list_windows"], ids=[c["name"] for c in KATS["list_windows"]])
def test_gpu_list_window_kats(case):
    c = case["cfg"]
    gpu, ref = _pair(c["assigner"], c["size"], trigger=c["trigger"], trigger_count=c["trigger_count"],
                     evictor=c["evictor"], evict_after=c["evict_after"], evict_arg=c["evict_arg"],
                     threshold=c["threshold"], value_type="i32")
    for (got, exp), (rgot, _) in zip(replay_list_phases(case, KEYMAP, gpu), replay_list_phases(case, KEYMAP, ref)):
        assert got == exp
        assert rgot == exp
    _assert_same(gpu, ref)  # and the contents of every firing
    gpu.close()


@pytest.mark.parametrize("name", sorted(KATS["list_apply_cases"]))
def test_gpu_list_apply_kats(name):
    # WindowedStream.apply over ListState (WOT:213-238, :339-364): RichSumReducer's sums = the rows' sums
    case = next(c for c in KATS["operator_cases"] if c["name"] == name)
    c = case["cfg"]
    sums = []
    gpu, ref = _pair(c["assigner"], c["size"], c["slide"], value_type="i32",
                     window_function=lambda k, w, el: sums.append((k, w, int(el["val"].sum()))))
    gpu = replay(case, KEYMAP, lambda _: gpu, flush_elements=True)
    ref = replay(case, KEYMAP, lambda _: ref, flush_elements=False)
    got, _ = row_counters(gpu.rows(), [], case, with_window=True)
    exp, _ = expected_counters(case, KEYMAP, with_window=True)
    assert got == exp
    assert sorted(s for _, _, s in sums) == sorted(int(r["sum"]) for r in gpu.rows())
    _assert_same(gpu, ref)
    gpu.close()


# ---------------------------------------------------------------- seeded streams vs the oracle
def _stream(seed, n, keys, span, jitter):
    rng = np.random.default_rng(seed)
    k = rng.integers(0, keys, n, dtype=np.int64)
    t = np.arange(n, dtype=np.int64) * span // n - rng.integers(0, jitter, n, dtype=np.int64)
    v = rng.integers(-1000, 1000, n, dtype=np.int64)
    return k, t, v


CONFIGS = [
    dict(assigner="tumbling", size=100),
    dict(assigner="tumbling", size=100, purging=True, lateness=50, side_output=True),
    dict(assigner="tumbling", size=100, lateness=60),
    dict(assigner="sliding", size=100, slide=25),
    dict(assigner="sliding", size=90, slide=30, lateness=40),
    dict(assigner="tumbling", size=100, evictor="count", evict_arg=3),
    dict(assigner="tumbling", size=100, evictor="count", evict_arg=2, evict_after=True, lateness=30),
    dict(assigner="tumbling", size=200, evictor="time", evict_arg=50),
    dict(assigner="sliding", size=100, slide=50, evictor="time", evict_arg=20, evict_after=True),
    dict(assigner="tumbling", size=100, evictor="delta", threshold=300.0),
    dict(assigner="tumbling", size=100, trigger="count", trigger_count=3),
    dict(assigner="tumbling", size=100, trigger="count", trigger_count=2, purging=True, evictor="count", evict_arg=5),
    dict(assigner="global", trigger="count", trigger_count=4, evictor="count", evict_arg=6),
    dict(assigner="global", trigger="count", trigger_count=3, evictor="delta", threshold=500.0, evict_after=True),
    dict(assigner="global", trigger="count", trigger_count=5, purging=True),
]


@pytest.mark.parametrize("cfg", CONFIGS, ids=[str(i) for i in range(len(CONFIGS))])
@pytest.mark.parametrize("value_type", ["i64", "f64"])
def test_gpu_list_vs_oracle(cfg, value_type):
    gpu, ref = _pair(value_type=value_type, **cfg)
    k, t, v = _stream(7 + len(str(cfg)), 20000, 37, 2000, 150)
    if value_type == "f64":
        v = (v.astype(np.float64) * 0.37).view(np.int64)
    wm = -10**9
    for b in range(10):
        sl = slice(b * 2000, (b + 1) * 2000)
        vals = v[sl].view(np.float64) if value_type == "f64" else v[sl]
        gpu.process(k[sl], t[sl], vals)
        ref.process(k[sl], t[sl], v[sl])
        wm = max(wm, int(t[sl].max()) - 100)
        if b % 3 != 1:
            gpu.watermark(wm)
            ref.watermark(wm)
    for w in (wm + 500, (1 << 63) - 1):
        gpu.watermark(w)
        ref.watermark(w)
    _assert_same(gpu, ref)
    assert gpu.late_dropped == ref.late_dropped
    if cfg.get("side_output"):
        gs = sorted(map(tuple, np.stack([gpu.side_rows()[f] for f in ("epoch", "key", "ts", "val")], 1).tolist()))
        e, kk, ts, vv = ref.side_rows()
        assert gs == sorted(zip(e.tolist(), kk.tolist(), ts.tolist(), vv.tolist()))
    st = gpu.stats()
    assert st["keyed_state_entries"] == ref.num_state_entries
    assert st["event_time_timers"] == ref.num_timers
    gpu.close()


def test_gpu_list_state_counters_mid_stream():
    # numKeyedStateEntries / numEventTimeTimers while windows are open (lateness keeps fired lists alive)
    gpu, ref = _pair(assigner="sliding", size=100, slide=50, lateness=30)
    k, t, v = _stream(3, 5000, 11, 1000, 80)
    for h in (gpu, ref):
        h.process(k, t, v)
        h.watermark(600)
    st = gpu.stats()
    assert st["keyed_state_entries"] == ref.num_state_entries > 0
    assert st["event_time_timers"] == ref.num_timers > 0
    _assert_same(gpu, ref)
    gpu.close()


def test_gpu_list_growth_and_compaction():
    # a log and a group map far smaller than the stream: grows, cleanups and compactions along the way
    gpu, ref = _pair(assigner="tumbling", size=50, evictor="count", evict_arg=4, trigger="count", trigger_count=3,
                     expected_elements=1024)
    k, t, v = _stream(11, 200000, 5000, 40000, 30)
    for b in range(20):
        sl = slice(b * 10000, (b + 1) * 10000)
        gpu.process(k[sl], t[sl], v[sl])
        ref.process(k[sl], t[sl], v[sl])
        gpu.watermark(int(t[sl].max()) - 40)
        ref.watermark(int(t[sl].max()) - 40)
    gpu.watermark((1 << 63) - 1)
    ref.watermark((1 << 63) - 1)
    _assert_same(gpu, ref)
    assert gpu.stats()["table_grows"] > 0
    gpu.close()


def test_gpu_list_device_columns_and_hashed_keys():
    import torch
    from flink_amd.keygroups import string_hash_code
    words = ["to", "be", "or", "not", "that", "is", "the", "question"]
    rng = np.random.default_rng(5)
    ids = rng.integers(0, len(words), 30000)
    kh = np.array([string_hash_code(words[i]) for i in ids], dtype=np.int32)
    t = np.arange(30000, dtype=np.int64) // 3
    v = np.ones(30000, dtype=np.int64)
    gpu, ref = _pair(assigner="tumbling", size=1000, evictor="count", evict_arg=100, value_type="i32",
                     key_type="hashed")
    d = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    gpu.process(d(ids.astype(np.int64)), d(t), d(v), d(kh))
    ref.process(ids, t, v)
    for h in (gpu, ref):
        h.watermark((1 << 63) - 1)
    _assert_same(gpu, ref)
    gpu.close()


def test_gpu_list_snapshot_restore_rescale():
    # snapshot every key group mid-stream, restore into two subtasks over halves of the key groups, continue;
    # the union of their firings equals one uninterrupted oracle
    from flink_amd import KeyGroupRange
    from flink_amd.listwindow import GpuListWindowOperator
    cfg = dict(assigner="tumbling", size=100, lateness=50, evictor="count", evict_arg=5, trigger="count",
               trigger_count=4)
    gpu, ref = _pair(**cfg)
    k, t, v = _stream(21, 40000, 200, 4000, 60)
    h = 20000
    gpu.process(k[:h], t[:h], v[:h])
    ref.process(k[:h], t[:h], v[:h])
    gpu.watermark(int(t[:h].max()) - 70)
    ref.watermark(int(t[:h].max()) - 70)
    snap = gpu.snapshot_state()
    assert sum(int((s[0]["n_elems"] > 0).sum()) for s in snap.values()) == ref.num_state_entries
    assert sum(len(s[1]) for s in snap.values()) == sum(int(s[0]["n_elems"].sum()) for s in snap.values())
    parts = []
    for r in (KeyGroupRange(0, 63), KeyGroupRange(64, 127)):
        op = GpuListWindowOperator(TumblingEventTimeWindows.of(100), CountTrigger.of(4), CountEvictor.of(5),
                                   allowed_lateness=50, key_group_range=r)
        op.initialize_state(snap)
        op.epoch = gpu.epoch
        op.advance_watermark(int(t[:h].max()) - 70)
        op.epoch -= 1
        kg = np.array([orc.lib().oracle_key_group(orc.lib().oracle_long_hash(int(x)), 128) for x in k[h:]])
        mine = (kg >= r.start_key_group) & (kg <= r.end_key_group)
        op.process(k[h:][mine], t[h:][mine], v[h:][mine])
        op.watermark((1 << 63) - 1)
        parts.append(op)
    ref.process(k[h:], t[h:], v[h:])
    ref.watermark((1 << 63) - 1)
    # ordinals number each handle's own records, so the restored subtasks' differ from one operator's
    got = _firings(gpu, ordinals=False)
    for op in parts:
        got += _firings(op, ordinals=False)
    exp = _firings(ref, ordinals=False)
    assert got == exp
    for op in parts:
        op.close()
    gpu.close()


def test_gpu_list_full_size_every_record_once():
    # 2^22 records, 1M keys, tumbling 1 s apply: after the final watermark every record is in exactly one
    # fired list, in arrival order (size-independent properties at a BASELINE-like scale)
    import torch
    from flink_amd.datagen import generate_device
    from flink_amd.listwindow import GpuListWindowOperator
    n = 1 << 22
    k, t, v, _ = generate_device(0x5EED, 0, n, 1_000_000, ts_base=0, rate=100_000_000, jitter=200)
    op = GpuListWindowOperator(TumblingEventTimeWindows.of(1000), max_batch=n, expected_elements=n)
    op.process(k, t, v)
    op.watermark((1 << 63) - 1)
    rows, el = op.rows(), op.elems()
    assert int(rows["count"].sum()) == n == len(el)
    assert np.array_equal(np.sort(el["ordinal"]), np.arange(n))
    vh = v.cpu().numpy()
    assert int(rows["sum"].sum()) == int(vh.sum())
    for r in rows[:: max(1, len(rows) // 1000)]:
        seg = el["ordinal"][r["elem_off"]:r["elem_off"] + r["count"]]
        assert np.all(np.diff(seg) > 0)
    assert op.stats()["keyed_state_entries"] == 0
    op.close()
    del torch


def test_gpu_list_errors_and_edges():
    from flink_amd import _native as N
    from flink_amd.listwindow import GpuListWindowOperator
    # Long.MIN_VALUE timestamps on an event-time assigner (TumblingEventTimeWindows.java:69-71): refused, state intact
    op = GpuListWindowOperator(TumblingEventTimeWindows.of(100), max_batch=8)
    with pytest.raises(N.NativeError) as e:
        op.process(np.array([1, 2]), np.array([5, -(1 << 63)]), np.array([1, 1]))
    assert e.value.code == N.FW_ERR_NO_TIMESTAMP
    op.process(np.array([], dtype=np.int64), np.array([], dtype=np.int64), np.array([], dtype=np.int64))
    with pytest.raises(N.NativeError) as e:  # a device batch beyond max_batch
        import torch
        z = torch.zeros(9, dtype=torch.int64, device="cuda")
        op.process_batch(z, z, z)
    assert e.value.code == N.FW_ERR_ARG
    op.process(np.array([1, 1]), np.array([5, 7]), np.array([3, 4]))
    op.watermark(50)
    op.process(np.array([1]), np.array([10]), np.array([9]))  # late (window [0, 100) fired? no: maxTs 99 > 50)
    op.watermark(200)
    op.process(np.array([1, 2]), np.array([20, 30]), np.array([7, 7]))  # every window late: dropped
    op.watermark(300)
    assert [int(r["sum"]) for r in op.rows()] == [16]
    assert op.late_dropped == 2
    op.close()
    # a key outside the KeyGroupRange
    from flink_amd import KeyGroupRange
    from flink_amd.keygroups import assign_to_key_group
    keys = [k for k in range(100) if assign_to_key_group(k, 128) >= 64][:1]
    op = GpuListWindowOperator(TumblingEventTimeWindows.of(100), key_group_range=KeyGroupRange(0, 63))
    with pytest.raises(N.NativeError) as e:
        op.process(np.array(keys), np.array([1]), np.array([1]))
    assert e.value.code == N.FW_ERR_KEY_GROUP
    op.close()


def test_gpu_list_map_growth_bounded():
    """A push of far more new (key, window) groups than the group map holds (1024 slots at creation, 2^20 distinct
    keys in one batch): the probe chains of an overfull map are capped and the map grows fourfold per retry, so the
    push finishes quickly (no walk over the whole map per insert) and every group fires once with its records."""
    import time
    from flink_amd.listwindow import GpuListWindowOperator
    n = 1 << 20
    keys = np.arange(n, dtype=np.int64) * 7919
    ts = np.arange(n, dtype=np.int64) % 1000
    vals = np.arange(n, dtype=np.int64)
    op = GpuListWindowOperator(TumblingEventTimeWindows.of(1000), emit_contents=False)
    t0 = time.perf_counter()
    op.process(keys, ts, vals)
    took = time.perf_counter() - t0
    op.watermark(2000)
    rows = op.rows()
    op.close()
    assert took < 20, took
    assert len(rows) == n and int(rows["count"].sum()) == n
    assert np.array_equal(np.sort(rows["key"]), np.sort(keys))


# ---------------------------------------------------------------- session windows (the merging branch)
@pytest.mark.parametrize("name", sorted(KATS["list_session_cases"]))
def test_gpu_list_session_kats(name):
    # WindowedStream.apply over EventTimeSessionWindows (EvictingWindowOperator / WindowOperator merging branch,
    # EvictingWindowOperator.java:110-170, WindowOperator.java:297-370) against WindowOperatorTest's session sequences
    # (lateness, purging, side output): the rows, and every firing's contents equal to the oracle's
    case = next(c for c in KATS["operator_cases"] if c["name"] == name)
    c = case["cfg"]
    gpu, ref = _pair("session", gap=c["gap"], lateness=c["lateness"], purging=c["purging"],
                     side_output=c["side_output"], value_type="i32")
    gpu = replay(case, KEYMAP, lambda _: gpu, flush_elements=True)
    ref = replay(case, KEYMAP, lambda _: ref, flush_elements=False)
    side = [dict(key=int(r["key"]), ts=int(r["ts"]), val=int(r["val"]), epoch=int(r["epoch"]))
            for r in gpu.side_rows()]
    got, got_side = row_counters(gpu.rows(), side, case, with_window=True)
    exp, exp_side = expected_counters(case, KEYMAP, with_window=True)
    assert got == exp
    assert got_side == exp_side
    _assert_same(gpu, ref)
    gpu.close()


def _hashset_first(wins):
    """the first of TimeWindows in java.util.HashSet order (TimeWindow.hashCode = longToIntWithBitMixing(start +
    end), bucket (h ^ h >>> 16) & 15; an independent restatement for the test)"""
    def mix(x):
        M = (1 << 64) - 1
        x &= M
        x = ((x ^ (x >> 30)) * 0xbf58476d1ce4e5b9) & M
        x = ((x ^ (x >> 27)) * 0x94d049bb133111eb) & M
        return (x ^ (x >> 31)) & 0xffffffff
    b = [(mix(s + e) ^ (mix(s + e) >> 16)) & 15 for s, e in wins]
    return min(range(len(wins)), key=lambda i: (b[i], i))


@pytest.mark.parametrize("first", [0, 1])
def test_gpu_list_session_bridge_order(first):
    # a bridging element merges two sessions: the merged list is the state window of the first merged window in
    # HashSet order, then the other's list (MergingWindowSet.addWindow, MergingWindowSet.java:150-225;
    # AbstractHeapMergingState.mergeNamespaces :67-93 with HeapListState's addAll), then the element
    gap = 10
    for a0 in range(0, 400):
        A, B = (a0, a0 + gap + 1), (a0 + 2 * gap, a0 + 3 * gap + 1)
        if (_hashset_first([A, B]) == 0) == (first == 0):
            break
    gpu, ref = _pair("session", gap=gap)
    for h in (gpu, ref):
        h.process(np.array([1, 1, 1, 1]), np.array([A[0], B[0], A[0] + 1, B[0] + 1]), np.array([1, 2, 3, 4]))
        h.process(np.array([1]), np.array([A[0] + gap]), np.array([5]))
        h.watermark((1 << 63) - 1)
    (r, el), = gpu.contents()
    assert (r["start"], r["end"]) == (A[0], B[1]) and r["count"] == 5
    assert list(el["val"]) == ([1, 3, 2, 4, 5] if first == 0 else [2, 4, 1, 3, 5])
    _assert_same(gpu, ref)
    gpu.close()


def _zipf_stream(seed, n, keys, span, jitter, s=1.1):
    rng = np.random.default_rng(seed)
    w = 1.0 / np.arange(1, keys + 1) ** s
    k = rng.choice(keys, n, p=w / w.sum()).astype(np.int64) * 7919 + 13
    t = np.arange(n, dtype=np.int64) * span // n - rng.integers(0, jitter, n, dtype=np.int64)
    v = rng.integers(-1000, 1000, n, dtype=np.int64)
    return k, t, v


SESSION_CONFIGS = [
    dict(gap=30),
    dict(gap=30, lateness=200),
    dict(gap=30, lateness=200, purging=True, side_output=True),
    dict(gap=50, purging=True),
    dict(gap=30, evictor="count", evict_arg=3),
    dict(gap=30, lateness=150, evictor="count", evict_arg=2, evict_after=True),
    dict(gap=40, evictor="time", evict_arg=25),
    dict(gap=40, lateness=100, evictor="time", evict_arg=10, evict_after=True, purging=True),
    dict(gap=30, evictor="delta", threshold=300.0),
    dict(gap=20, lateness=300, evictor="delta", threshold=600.0, evict_after=True, side_output=True),
]


@pytest.mark.parametrize("cfg", SESSION_CONFIGS, ids=[str(i) for i in range(len(SESSION_CONFIGS))])
@pytest.mark.parametrize("value_type,zipf", [("i64", False), ("f64", True)], ids=["i64-uniform", "f64-zipf"])
def test_gpu_list_sessions_vs_oracle(cfg, value_type, zipf):
    # f4 with merging windows: seeded streams (out of order by up to 150 ms against a 100 ms watermark bound, so
    # elements arrive behind in-flight sessions, bridge them, fire late sessions again under allowed lateness, or
    # are dropped / side-output), every firing's row and contents in list order bit-exact against the oracle
    gpu, ref = _pair("session", value_type=value_type, **cfg)
    k, t, v = (_zipf_stream if zipf else _stream)(23 + len(str(cfg)), 20000, 300 if zipf else 400, 20000, 150)
    if value_type == "f64":
        v = (v.astype(np.float64) * 0.37).view(np.int64)
    wm = -10**9
    for b in range(10):
        sl = slice(b * 2000, (b + 1) * 2000)
        vals = v[sl].view(np.float64) if value_type == "f64" else v[sl]
        gpu.process(k[sl], t[sl], vals)
        ref.process(k[sl], t[sl], v[sl])
        wm = max(wm, int(t[sl].max()) - 100)
        if b % 3 != 1:
            gpu.watermark(wm)
            ref.watermark(wm)
    for w in (wm + 500, (1 << 63) - 1):
        gpu.watermark(w)
        ref.watermark(w)
    _assert_same(gpu, ref)
    assert gpu.late_dropped == ref.late_dropped
    if cfg.get("side_output"):
        gs = sorted(map(tuple, np.stack([gpu.side_rows()[f] for f in ("epoch", "key", "ts", "val")], 1).tolist()))
        e, kk, ts, vv = ref.side_rows()
        assert gs == sorted(zip(e.tolist(), kk.tolist(), ts.tolist(), vv.tolist()))
    rows = gpu.rows()
    assert (rows["end"] - rows["start"] > cfg["gap"]).any()  # sessions merged
    gpu.close()


def test_gpu_list_sessions_state_counters_and_growth():
    # a map and a log far smaller than the stream (rebuilds, compactions, tombstones of merged sessions) with the
    # state counters checked mid-stream while sessions are open under allowed lateness
    gpu, ref = _pair("session", gap=25, lateness=100, evictor="count", evict_arg=5, expected_elements=1024)
    k, t, v = _stream(31, 100000, 3000, 50000, 60)
    for b in range(10):
        sl = slice(b * 10000, (b + 1) * 10000)
        gpu.process(k[sl], t[sl], v[sl])
        ref.process(k[sl], t[sl], v[sl])
        gpu.watermark(int(t[sl].max()) - 50)
        ref.watermark(int(t[sl].max()) - 50)
        st = gpu.stats()
        assert st["keyed_state_entries"] == ref.num_state_entries
        assert st["event_time_timers"] == ref.num_timers
    gpu.watermark((1 << 63) - 1)
    ref.watermark((1 << 63) - 1)
    _assert_same(gpu, ref)
    assert gpu.stats()["table_grows"] > 0
    gpu.close()


def test_gpu_list_sessions_refusals():
    from flink_amd import _native as N
    from flink_amd.listwindow import GpuListWindowOperator
    with pytest.raises(N.NativeError) as e:  # (CountTrigger over merging windows: not offered)
        GpuListWindowOperator(EventTimeSessionWindows.with_gap(10), CountTrigger.of(3))
    assert e.value.code == N.FW_ERR_UNSUPPORTED
    op = GpuListWindowOperator(EventTimeSessionWindows.with_gap(10))
    op.process(np.array([1, 2]), np.array([5, 6]), np.array([1, 2]))
    with pytest.raises(N.NativeError) as e:  # (the merging window set is not in fw_list_state)
        op.snapshot_key_group(0)
    assert e.value.code == N.FW_ERR_UNSUPPORTED
    op.close()
