"""GPU parity: GpuWindowOperator (libflinkwin.so, HIP gfx950) against the oracle and the reference KATs.
Bar: bit-exact keys, window bounds, counts and integer sum/min/max; f64 sums within 1e-6 relative."""
import numpy as np
import pytest

from flink_amd import (EventTimeSessionWindows, KeyGroupRange, PurgingTrigger, SlidingEventTimeWindows,
                       EventTimeTrigger, TumblingEventTimeWindows)
from flink_amd.datagen import generate_host
from flink_amd.windowing import CountSumMinMax, ExtremalElementReduce, FirstElementReduce, first_element_results
from oracle import oracle as orc
from tests.kat_util import expected_counters, load_kats, replay, row_counters
from tests.parity_util import assert_f32_sums_near_exact, assert_rows_equal, assert_side_equal

pytestmark = pytest.mark.gpu

KATS = load_kats()
_VT = {"i64": "long", "i32": "int", "f64": "double", "i16": "short", "i8": "byte", "f32": "float"}


def _gpu_op(assigner, size=0, slide=0, offset=0, gap=0, lateness=0, purging=False, side_output=False,
            value_type="i64", first=False, by=None, **kw):
    from flink_amd.operator import GpuWindowOperator
    if assigner == "tumbling":
        a = TumblingEventTimeWindows.of(size, offset)
    elif assigner == "sliding":
        a = SlidingEventTimeWindows.of(size, slide, offset)
    else:
        a = EventTimeSessionWindows.with_gap(gap)
    trig = PurgingTrigger.of(EventTimeTrigger.create()) if purging else EventTimeTrigger.create()
    agg = (FirstElementReduce(_VT[value_type], "max" if first == "max" else "sum") if first
           else ExtremalElementReduce(by, _VT[value_type]) if by
           else CountSumMinMax(_VT[value_type]))
    return GpuWindowOperator(a, agg, trig, allowed_lateness=lateness,
                             side_output=side_output, **kw)


def _from_case_cfg(cfg):
    return _gpu_op(cfg["assigner"], cfg["size"], cfg["slide"], cfg["offset"], cfg["gap"], cfg["lateness"],
                   cfg["purging"], cfg["side_output"], cfg["value_type"])


@pytest.mark.parametrize("case", KATS["operator_cases"], ids=[c["name"] for c in KATS["operator_cases"]])
def test_gpu_reference_kats(case):
    keymap = KATS["keys"]
    op = replay(case, keymap, _from_case_cfg, flush_elements=True)
    got, got_side = row_counters(op.rows(), op.side_rows(), case, with_window=True)
    exp, exp_side = expected_counters(case, keymap, with_window=True)
    assert got == exp
    assert got_side == exp_side
    op.close()


def _panes(cfg):
    """The operator keeps sliding windows as panes (fw_runtime.cpp fw_create: size % slide == 0, no lateness)."""
    return (cfg["assigner"] == "sliding" and not cfg.get("lateness") and cfg["size"] > cfg["slide"]
            and cfg["size"] % cfg["slide"] == 0)


def _run_both(cfg, batches, wms, **gpu_kw):
    gpu = _gpu_op(**cfg, **gpu_kw)
    ref = orc.WindowOperatorOracle(**cfg)
    for (k, t, v), wm in zip(batches, wms):
        gpu.process(k, t, v)
        ref.process(k, t, v)
        gpu.watermark(wm)
        ref.watermark(wm)
    out = gpu.rows(), ref.rows(), gpu.side_rows(), ref.side_rows(), gpu.late_dropped, ref.late_dropped
    st = gpu.stats()
    # with sliding windows kept as panes the state entries are panes, not (key, window) pairs
    assert (st["keyed_state_entries"] == ref.num_state_entries or cfg.get("purging") or cfg["assigner"] == "session"
            or _panes(cfg))
    gpu.close()
    return out


def _stream(n, batch, num_keys, bound, jitter, rate, seed=0x5EED, value_type="i64", zipf=None, final=True):
    keys, ts, vals = generate_host(seed, 0, n, num_keys, ts_base=1_000_000, rate=rate, jitter=jitter, zipf_s=zipf)
    if value_type == "f64":
        vals = ((vals & 0xFFFFF).astype(np.float64) / 7.0)
    batches, wms, mx = [], [], -(1 << 63)
    for b in range(0, n, batch):
        sl = slice(b, min(n, b + batch))
        batches.append((keys[sl], ts[sl], vals[sl]))
        mx = max(mx, int(ts[sl].max()))
        wms.append(mx - bound)
    if final:
        batches.append((keys[:0], ts[:0], vals[:0]))
        wms.append((1 << 63) - 1)
    return batches, wms


CONFIGS = [
    dict(assigner="tumbling", size=1000),
    dict(assigner="tumbling", size=1000, offset=250, value_type="i32"),
    dict(assigner="tumbling", size=1000, value_type="f64"),
    dict(assigner="sliding", size=3000, slide=1000),
    dict(assigner="sliding", size=2500, slide=1000, offset=300, value_type="f64"),
    dict(assigner="tumbling", size=1000, lateness=700),
    dict(assigner="tumbling", size=1000, lateness=700, purging=True, side_output=True),
    dict(assigner="sliding", size=2000, slide=500, lateness=300, side_output=True),
    # panes: size % slide == 0 and no allowed lateness (partially late elements go to their pane)
    dict(assigner="sliding", size=3000, slide=500, offset=200, value_type="i32", purging=True, side_output=True),
    dict(assigner="sliding", size=4000, slide=1000, value_type="f64"),
    dict(assigner="session", gap=300),
    dict(assigner="session", gap=300, lateness=200, purging=True, side_output=True),
    dict(assigner="session", gap=300, lateness=400, value_type="f64"),
]


@pytest.mark.parametrize("cfg", CONFIGS, ids=[str(i) for i in range(len(CONFIGS))])
def test_gpu_vs_oracle_out_of_order(cfg):
    # heavy disorder (jitter 1.5 s against a 0.4 s bound) exercises late drops, late firings and
    # partially late sliding records; rate 1e5/s over 5000 keys keeps sessions open and merging
    vt = cfg.get("value_type", "i64")
    batches, wms = _stream(120_000, 10_000, 5000, bound=400, jitter=1500, rate=100_000, value_type=vt)
    g, r, gs, rs, gl, rl = _run_both(cfg, batches, wms)
    assert_rows_equal(g, r, _VT[vt])
    assert_side_equal(gs, rs)
    assert gl == rl


@pytest.mark.parametrize("cfg", CONFIGS, ids=[str(i) for i in range(len(CONFIGS))])
@pytest.mark.parametrize("first", [True, "max"], ids=["sum_min", "max"])
def test_gpu_first_element_vs_oracle(cfg, first):
    # a9: sum(pos)/min(pos) keep the window's first element; the rows' max is its arrival ordinal,
    # carried through the parallel path (k_scatter -> k_aggregate), the ordered replay (late firings,
    # sessions of tainted keys), pane windows and session merges
    vt = cfg.get("value_type", "i64")
    batches, wms = _stream(120_000, 10_000, 5000, bound=400, jitter=1500, rate=100_000, value_type=vt)
    g, r, gs, rs, gl, rl = _run_both(dict(cfg, first=first), batches, wms)
    assert_rows_equal(g, r, _VT[vt])
    assert_side_equal(gs, rs)
    assert gl == rl


@pytest.mark.parametrize("cfg", [dict(assigner="tumbling", size=100), dict(assigner="session", gap=20),
                                 dict(assigner="sliding", size=400, slide=100)], ids=["tumbling", "session", "panes"])
def test_gpu_first_element_hot_keys(cfg):
    # Zipf keys over multi-batch pushes: hot partitions are split over aggregate workgroups and the
    # chunks' deltas merged, with the first element's ordinal surviving the merge
    batches, wms = _stream(1 << 20, 1 << 19, 10_000, bound=50, jitter=50, rate=1_000_000, zipf=1.1)
    g, r, gs, rs, gl, rl = _run_both(dict(cfg, first=True), batches, wms)
    assert_rows_equal(g, r)
    assert gl == rl


def test_gpu_session_example_sum_passthrough():
    # SessionWindowing example (SWE:57-83): keyBy(0).window(sessions, gap 3).sum(2) emits a copy of the
    # session's first element with field 2 summed; EXPECTED (SWD:26-27) pinned exactly
    ex = KATS["session_example"]
    names = sorted({r[0] for r in ex["input"]})
    ids = {n: i for i, n in enumerate(names)}
    op = _gpu_op("session", gap=ex["gap"], value_type="i32", first=True, key_type="int")
    rows = []
    for name, ts, val in ex["input"]:
        op.process(np.array([ids[name]], dtype=np.int64), np.array([ts], dtype=np.int64),
                   np.array([val], dtype=np.int64))
        op.watermark(ts - 1)
    op.watermark((1 << 63) - 1)
    got = first_element_results(op.rows(), [tuple(e) for e in ex["input"]], 2, "sum")
    op.close()
    assert sorted(got) == sorted(tuple(e) for e in ex["expected"])


BY_CONFIGS = [
    dict(assigner="tumbling", size=1000),
    dict(assigner="tumbling", size=1000, lateness=700),
    dict(assigner="sliding", size=3000, slide=500),
    dict(assigner="sliding", size=2000, slide=500, lateness=300, side_output=True),
    dict(assigner="session", gap=300),
    dict(assigner="session", gap=300, lateness=200, purging=True),
]


def _by_values(v, value_type):
    """Fields drawn from 5 values, so most windows break ties by arrival order; Long fields beyond 32 bits,
    Double fields with -0.0 and 0.0 (distinct under Double.compare)."""
    f = v % 5
    if value_type == "i64":
        return (f - 2) * (1 << 40)
    if value_type == "f64":
        return np.array([-0.0, 0.0, 1.5, -2.25, 1e300])[f]
    return f


@pytest.mark.parametrize("by", ["min", "max"])
@pytest.mark.parametrize("value_type", ["i32", "i64", "f64"])
@pytest.mark.parametrize("cfg", BY_CONFIGS, ids=[str(i) for i in range(len(BY_CONFIGS))])
def test_gpu_min_by_max_by_vs_oracle(cfg, value_type, by):
    # a9 minBy/maxBy (first = true) over Integer, Long and Double fields (ComparableAggregator.java:72-94,
    # Comparator.java:35-108): the selected element's field and arrival ordinal
    batches, wms = _stream(120_000, 10_000, 5000, bound=400, jitter=1500, rate=100_000)
    batches = [(k, t, _by_values(v, value_type)) for k, t, v in batches]
    cfg = dict(cfg, value_type=value_type, by=by)
    g, r, gs, rs, gl, rl = _run_both(cfg, batches, wms)
    assert_rows_equal(g, r, {"i32": "int", "i64": "long", "f64": "double"}[value_type])
    if value_type == "f64":  # the selected field bit for bit (-0.0 and 0.0 differ under Double.compare)
        go = np.lexsort((g["end"], g["start"], g["key"], g["epoch"]))
        ro = np.lexsort((r["end"], r["start"], r["key"], r["epoch"]))
        assert np.array_equal(g["min"][go], r["min"][ro])
    assert_side_equal(gs, rs)
    assert gl == rl


@pytest.mark.parametrize("by", ["min", "max"])
@pytest.mark.parametrize("value_type", ["i64", "f64"])
def test_gpu_min_by_max_by_panes_hot_keys(value_type, by):
    # minBy / maxBy over sliding windows kept as panes (a window's element = the smallest (field, ordinal) pair over
    # its panes, ComparableAggregator.java:72-94), Zipf keys so hot partitions split into chunks, 10 s / 1 s windows
    batches, wms = _stream(200_000, 25_000, 3000, bound=300, jitter=200, rate=10_000, zipf=1.1)
    batches = [(k, t, _by_values(v, value_type)) for k, t, v in batches]
    cfg = dict(assigner="sliding", size=10_000, slide=1000, value_type=value_type, by=by)
    assert _panes(cfg)
    g, r, gs, rs, gl, rl = _run_both(cfg, batches, wms)
    assert_rows_equal(g, r, {"i64": "long", "f64": "double"}[value_type])
    assert gl == rl


@pytest.mark.parametrize("by", ["min", "max"])
def test_gpu_min_by_ties_straddle_2_32(by):
    # ordinals are compared in full: a restore numbers later pushes after the restored ordinals, so the batch's
    # elements get ordinals 2^32 - 2000 ...; tied fields across 2^32 keep the earlier element
    # (ComparableAggregator.java:80-84 keeps the first of equal elements)
    from flink_amd.keygroups import assign_to_key_group, long_hash_code
    from flink_amd.operator import STATE_DTYPE
    base = (1 << 32) - 2000
    op = _gpu_op("tumbling", 1000, value_type="i32", by=by)
    kg = assign_to_key_group(long_hash_code(-7), 128)
    row = np.zeros(1, dtype=STATE_DTYPE)
    row["key"], row["start"], row["end"], row["count"], row["min"], row["max"] = -7, 0, 1000, 1, 3, base - 1
    op.restore_key_group(kg, row)
    n = 8000
    j = np.arange(n)
    k = j % 40
    t = np.full(n, 5000)
    # keys 20..39: the extremal field first appears before 2^32 and ties after it; keys 0..19: it first appears
    # after 2^32 (the elements before carry a worse field), then ties
    worse = 2 if by == "min" else 0
    v = np.where((j < 2000) & (k < 20), worse, 1)
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=1000, value_type="i32", by=by)
    op.process(k, t, v)
    ref.process(k, t, v)
    op.watermark((1 << 63) - 1)
    ref.watermark((1 << 63) - 1)
    g = op.rows()
    op.close()
    g = g[g["key"] != -7]
    r = ref.rows()
    r["max"] += base
    assert (g["max"] >= (1 << 32)).any() and (g["max"] < (1 << 32)).any()
    assert_rows_equal(g, r, "int")


def _word_stream(n, n_words, seed=0x5EED):
    """C1 shape: uniformly drawn words (String keys: the key column is the word's dictionary id,
    key_hash its String.hashCode), value 1 (Integer), ts = i / 2000 ms (5 s of event time per 1e7 tokens)."""
    from flink_amd.keygroups import string_hash_code
    words = [f"w{j}" for j in range(n_words)]
    hashes = np.array([string_hash_code(w) for w in words], dtype=np.int32)
    keys, _, _ = generate_host(seed, 0, n, n_words, ts_base=0, rate=1000, jitter=1)
    ts = np.arange(n, dtype=np.int64) // 2000
    return words, keys, hashes[keys], ts, np.ones(n, dtype=np.int64)


@pytest.mark.parametrize("first", [False, True], ids=["count_sum", "sum_passthrough"])
def test_gpu_word_count_hashed_keys(first):
    # C1 (ii): keyBy(word).window(TumblingEventTimeWindows.of(5 s)).sum(1) with String keys hashed by the host
    # (FW_KEY_HASHED: key groups from String.hashCode, KeyGroupRangeAssignment.java:58-71) on the GPU
    words, keys, kh, ts, vals = _word_stream(200_000, 170)
    gpu = _gpu_op("tumbling", size=5000, value_type="i32", first=first, key_type="hashed")
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=5000, value_type="i32", first=first)
    step = 25_000
    for b in range(0, len(keys), step):
        sl = slice(b, b + step)
        gpu.process(keys[sl], ts[sl], vals[sl], key_hash=kh[sl])
        ref.process(keys[sl], ts[sl], vals[sl])
        gpu.watermark(int(ts[sl].max()))
        ref.watermark(int(ts[sl].max()))
    gpu.watermark((1 << 63) - 1)
    ref.watermark((1 << 63) - 1)
    g, r = gpu.rows(), ref.rows()
    gpu.close()
    assert_rows_equal(g, r, "int")
    assert int(g["count"].sum()) == len(keys)
    if first:
        elements = [(words[k], 1) for k in keys]
        got = first_element_results(g, elements, 1, "sum")
        assert sorted(got) == sorted(first_element_results(r, elements, 1, "sum"))
        assert all(t[0] == words[int(row["key"])] for t, row in zip(got, g))


def test_gpu_word_count_real_tokens():
    # C1 (configs[0]) on WordCountData's own tokens (tests/golden/wordcount_tokens.json: 287 tokens, 170 words,
    # WordCount.java:102-117's toLowerCase().split("\\W+")), 2M of the bench's 10M-token stream: both pipelines of
    # WindowWordCount.java:74-81 / SideOutputExample.java:97-101 on the GPU against the oracle, rows bit-exact
    from bench import wordcount_stream
    n = 2_000_000
    keys, ts, vals, kh = wordcount_stream(0, n)
    assert len(np.unique(keys)) == 170
    gpu = _gpu_op("tumbling", size=5000, value_type="i32", key_type="hashed")
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=5000, value_type="i32")
    step = 1 << 19
    for b in range(0, n, step):
        sl = slice(b, b + step)
        gpu.process(keys[sl], ts[sl], vals[sl], key_hash=kh[sl])
        ref.process(keys[sl], ts[sl], vals[sl])
        gpu.watermark(int(ts[sl].max()))
        ref.watermark(int(ts[sl].max()))
    gpu.watermark((1 << 63) - 1)
    ref.watermark((1 << 63) - 1)
    g, r = gpu.rows(), ref.rows()
    gpu.close()
    assert_rows_equal(g, r, "int")
    assert int(g["count"].sum()) == n and int(g["sum"].sum()) == n
    # countWindow(10, 5).sum(1): every 5th token of a word fires over its last <= 10
    cw = _count_op(10, 5, value_type="i32", expected_entries=1024)
    cref = orc.CountWindowOracle(10, 5, value_type="i32")
    for b in range(0, n, step):
        sl = slice(b, b + step)
        cw.process(keys[sl], np.zeros(len(keys[sl]), dtype=np.int64), vals[sl])
        cref.process(keys[sl], vals[sl])
    gc, rc = cw.rows(), cref.rows()
    cw.close()
    assert len(gc) == len(rc) > n // 6
    assert _count_rows(gc) == _count_rows(rc)


def test_gpu_vs_oracle_c2_shape():
    # configs[1] shape at parity size: 2^22 records, 1M uniform Long keys, 1 s tumbling,
    # bounded out-of-orderness 200 ms, count/sum/min/max
    cfg = dict(assigner="tumbling", size=1000)
    batches, wms = _stream(1 << 22, 1 << 20, 1_000_000, bound=200, jitter=200, rate=100_000_000)
    g, r, gs, rs, gl, rl = _run_both(cfg, batches, wms)
    assert len(g) > 1_000_000
    assert_rows_equal(g, r)
    assert gl == rl == 0


def test_gpu_panes_c3_shape():
    # SURVEY §8d C3 shape at parity size: sliding 60 s / 1 s (60 windows per element, kept as panes),
    # 20K uniform keys, 2e5 records per event-second, bound 200 ms, a watermark every 2^15 records
    cfg = dict(assigner="sliding", size=60_000, slide=1000)
    batches, wms = _stream(1 << 18, 1 << 15, 20_000, bound=200, jitter=200, rate=200_000)
    g, r, gs, rs, gl, rl = _run_both(cfg, batches, wms)
    assert len(g) > 1_000_000
    assert_rows_equal(g, r)
    assert gl == rl


def test_gpu_panes_fire_suspends_and_resumes():
    # one element per key in a small table: the final watermark forms 60 windows per pane, more rows than
    # the fired-row buffer holds, so k_fire_panes suspends per (window, key-hash slice) and resumes
    cfg = dict(assigner="sliding", size=60_000, slide=1000)
    n = 30_000
    keys = np.arange(n, dtype=np.int64)
    ts = (np.arange(n, dtype=np.int64) * 37) % 50_000
    vals = np.arange(n, dtype=np.int64) * 3 - 7
    batches = [(keys, ts, vals), (keys[:0], ts[:0], vals[:0])]
    wms = [10_000, (1 << 63) - 1]
    g, r, *_ = _run_both(cfg, batches, wms, expected_entries=1000)
    assert len(g) == 60 * n
    assert_rows_equal(g, r)


def test_gpu_zipf_hot_keys():
    cfg = dict(assigner="tumbling", size=100)
    batches, wms = _stream(400_000, 50_000, 100_000, bound=50, jitter=100, rate=1_000_000, zipf=1.1)
    g, r, *_ = _run_both(cfg, batches, wms)
    assert_rows_equal(g, r)


@pytest.mark.parametrize("async_input", [False, True], ids=["host-push", "async-device-push"])
@pytest.mark.parametrize("value_type", ["i64", "f64"])
def test_gpu_single_pass_scatter_fallbacks(value_type, async_input):
    # dense tumbling windows take the single-pass scatter (each partition's run reserved piece by piece, no
    # histogram); a batch it cannot take goes through classify / scan / scatter instead: one with a record whose
    # window is too far ahead for a compact word, one whose hot key overfills its partition's reserved run.  Late
    # records and key counts must come out once either way.
    cfg = dict(assigner="tumbling", size=100, value_type=value_type)
    batches, wms = _stream(700_000, 100_000, 50_000, bound=20, jitter=200, rate=1_000_000, value_type=value_type)
    k, t, v = batches[2]
    t = t.copy()
    t[17] += 10**12  # (the watermarks stay those of the original stream)
    batches[2] = (k, t, v)
    k, t, v = batches[4]
    k = k.copy()
    k[: len(k) * 3 // 4] = 7
    batches[4] = (k, t, v)
    # (async device pushes: the batch is partitioned on the input stream, the gated classify / scan / scatter behind
    # a failed single pass included, beside the previous batch's aggregation)
    gpu = _gpu_op(**cfg, max_batch=1 << 17, async_input=async_input)
    ref = orc.WindowOperatorOracle(**cfg)
    drained = []
    for e, ((k, t, v), wm) in enumerate(zip(batches, wms)):
        if async_input:
            import torch
            gpu.process_batch(*(torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (k, t, v)))
            gpu.advance_watermark(wm, wait=False)
            drained.append(gpu.drain_rows(e))
        else:
            gpu.process(k, t, v)
            gpu.watermark(wm)
        ref.process(k, t, v)
        ref.watermark(wm)
    g = np.concatenate(drained) if async_input else gpu.rows()
    r, gl, rl = ref.rows(), gpu.late_dropped, ref.late_dropped
    st = gpu.stats()
    gpu.close()
    assert_rows_equal(g, r, _VT[value_type])
    assert gl == rl and gl > 0
    assert int(g["count"].sum()) + gl == 700_000
    # every batch after the first tried the single pass; the far-ahead and the hot-key batches were redone
    assert st["single_pass_batches"] >= len(batches) - 2 and st["single_pass_redone"] >= 2


@pytest.mark.parametrize("async_input", [False, True], ids=["host-push", "async-device-push"])
@pytest.mark.parametrize("wide", ["value", "key"])
def test_gpu_narrow_records_and_fallback(wide, async_input):
    # dense single-pass batches of an integer field write 8-byte records {key (29-bit signed), window delta, int32
    # value}.  The batches straddle what that form holds: batch 1 has values AT the int32 bounds
    # and keys at the edges of [-2^28, 2^28) (narrow); batch 3 has a value just outside int32 (wide="value") or a key
    # of 2^28 (wide="key"): that batch is redone through classify / scan / scatter with 16-byte records, and the
    # operator keeps 16-byte records from then on.  Every row bit-exact vs the oracle.
    cfg = dict(assigner="tumbling", size=100)
    batches, wms = _stream(600_000, 75_000, 50_000, bound=20, jitter=30, rate=1_000_000)
    k, t, v = (x.copy() for x in batches[1])
    v[5], v[6], v[7] = -(1 << 31), (1 << 31) - 1, 0
    k[8], k[9] = -(1 << 28), (1 << 28) - 1
    batches[1] = (k, t, v)
    k, t, v = (x.copy() for x in batches[3])
    if wide == "value":
        v[11], v[12] = 1 << 31, -(1 << 31) - 1
    else:
        k[11], k[12] = 1 << 28, -(1 << 28) - 1
    batches[3] = (k, t, v)
    gpu = _gpu_op(**cfg, max_batch=1 << 17, async_input=async_input)
    ref = orc.WindowOperatorOracle(**cfg)
    drained = []
    for e, ((k, t, v), wm) in enumerate(zip(batches, wms)):
        if async_input:
            import torch
            gpu.process_batch(*(torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (k, t, v)))
            gpu.advance_watermark(wm, wait=False)
            drained.append(gpu.drain_rows(e))
        else:
            gpu.process(k, t, v)
            gpu.watermark(wm)
        ref.process(k, t, v)
        ref.watermark(wm)
    g = np.concatenate(drained) if async_input else gpu.rows()
    r = ref.rows()
    st = gpu.stats()
    gpu.close()
    assert_rows_equal(g, r)
    assert int(g["count"].sum()) + st["late_records_dropped"] == 600_000
    assert int(g["max"].max()) >= (1 << 31) - 1 and int(g["min"].min()) <= -(1 << 31)
    # batches 1 .. 3 were narrow (the first batch has no watermark yet to base the windows on), batch 3 was redone
    assert st["narrow_pass_batches"] >= 2 and st["narrow_pass_redone"] == 1
    assert st["single_pass_batches"] > st["narrow_pass_batches"]


@pytest.mark.parametrize("cfg", [dict(assigner="tumbling", size=1000),
                                 dict(assigner="sliding", size=5000, slide=1000),
                                 dict(assigner="session", gap=50)], ids=["tumbling", "sliding", "session"])
def test_gpu_lds_flush_and_retry(cfg):
    # ~8K distinct (key, window) pairs per state partition and batch: the LDS pre-aggregation table
    # (1024 slots) fills many times inside one round, so flush-and-retry is exercised heavily
    batches, wms = _stream(1 << 20, 1 << 20, 1 << 40, bound=100, jitter=100, rate=1_000_000)
    g, r, *_ = _run_both(cfg, batches, wms, sub_partitions=1)
    assert_rows_equal(g, r)


@pytest.mark.parametrize("cfg", [dict(assigner="tumbling", size=10_000), dict(assigner="session", gap=100)],
                         ids=["tumbling", "session"])
def test_gpu_table_growth(cfg):
    # tiny initial table: regions run out of room mid-aggregate, the push suspends, the table grows
    # and the push resumes (several times per push)
    batches, wms = _stream(300_000, 100_000, 200_000, bound=100, jitter=100, rate=1_000_000)
    g, r, *_ = _run_both(cfg, batches, wms, expected_entries=1000)
    assert_rows_equal(g, r)


@pytest.mark.parametrize("async_input", [False, True], ids=["host-push", "async-device-push"])
def test_gpu_dense_growth_single_pass(async_input):
    # dense tumbling regions sized for the minimum (65536 entries) under 1M keys: the narrow single-pass batches
    # overfill their regions, the dense aggregate suspends, the table grows and the push resumes from the same
    # single-pass words; the scratch set's next batch must find them zeroed again (k_rsv_reset skips behind a
    # suspension, settle zeroes them)
    cfg = dict(assigner="tumbling", size=100)
    batches, wms = _stream(900_000, 100_000, 1_000_000, bound=20, jitter=30, rate=1_000_000)
    gpu = _gpu_op(**cfg, max_batch=1 << 17, expected_entries=65536, async_input=async_input)
    ref = orc.WindowOperatorOracle(**cfg)
    drained = []
    for e, ((k, t, v), wm) in enumerate(zip(batches, wms)):
        if async_input:
            import torch
            gpu.process_batch(*(torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (k, t, v)))
            gpu.advance_watermark(wm, wait=False)
            drained.append(gpu.drain_rows(e))
        else:
            gpu.process(k, t, v)
            gpu.watermark(wm)
        ref.process(k, t, v)
        ref.watermark(wm)
    g = np.concatenate(drained) if async_input else gpu.rows()
    st = gpu.stats()
    gpu.close()
    assert_rows_equal(g, ref.rows())
    assert st["table_grows"] >= 1 and st["push_resumptions"] >= 1 and st["single_pass_batches"] >= len(batches) - 3


@pytest.mark.parametrize("small_table", [False, True], ids=["table", "tiny-table"])
@pytest.mark.parametrize("cfg", [dict(assigner="tumbling", size=100), dict(assigner="session", gap=20),
                                 dict(assigner="tumbling", size=100, value_type="f64")],
                         ids=["tumbling", "session", "tumbling-f64"])
def test_gpu_hot_keys_split_partitions(cfg, small_table):
    # Zipf(1.3) over 100K keys: the hottest key is ~20% of a 2^20-record batch, so its state partition
    # is split into chunks that separate workgroups pre-aggregate and the last one merges (AggHot);
    # with a tiny table that merge runs out of region room, suspends and resumes after the growth
    vt = cfg.get("value_type", "i64")
    batches, wms = _stream(1 << 21, 1 << 20, 100_000, bound=50, jitter=50, rate=1_000_000, zipf=1.3, value_type=vt)
    g, r, *_ = _run_both(cfg, batches, wms, **(dict(expected_entries=1000) if small_table else {}))
    assert_rows_equal(g, r, _VT[vt])


def test_gpu_session_merges_across_flushes():
    # one state partition per key group and ~1500 keys per partition: the LDS table flushes several
    # times per batch, so a key's session is built from LDS intervals of different flushes that the
    # flush joins into the region's sessions (connected components); keys recur about every 10 ms
    # against a 50 ms gap, so sessions grow long and merge across batches too
    cfg = dict(assigner="session", gap=50)
    batches, wms = _stream(1 << 20, 1 << 18, 200_000, bound=100, jitter=100, rate=20_000_000)
    g, r, *_ = _run_both(cfg, batches, wms, sub_partitions=1)
    assert_rows_equal(g, r)


def test_gpu_sessions_take_parallel_path():
    # in-order enough (jitter < bound): every element's window ends after the watermark, no key is
    # tainted, and the ordered path replays nothing
    cfg = dict(assigner="session", gap=300)
    batches, wms = _stream(200_000, 20_000, 5000, bound=400, jitter=300, rate=100_000)
    gpu = _gpu_op(**cfg)
    ref = orc.WindowOperatorOracle(**cfg)
    for (k, t, v), wm in zip(batches, wms):
        gpu.process(k, t, v)
        ref.process(k, t, v)
        gpu.watermark(wm)
        ref.watermark(wm)
    assert gpu.stats()["slow_path_records"] == 0
    assert_rows_equal(gpu.rows(), ref.rows())
    gpu.close()


def test_gpu_session_taint_orders_mixed_keys():
    # key 7 has in-time elements and, in the same batch, one whose window [880, 980) ends before the
    # watermark 1000 but within the allowed lateness: it merges into the session the in-time elements
    # build, so all of key 7's elements are replayed in arrival order; key 8 stays on the parallel path
    cfg = dict(assigner="session", gap=100, lateness=1000, side_output=True)
    gpu = _gpu_op(**cfg)
    ref = orc.WindowOperatorOracle(**cfg)
    steps = [
        (np.array([7, 8], dtype=np.int64), np.array([500, 510], dtype=np.int64), 1000),
        (np.array([7, 8, 7, 8, 7, 7, 9], dtype=np.int64), np.array([950, 960, 1040, 1100, 880, 990, 20], dtype=np.int64),
         1200),
        (np.array([7, 8], dtype=np.int64), np.array([1150, 1250], dtype=np.int64), (1 << 63) - 1),
    ]
    for k, t, wm in steps:
        v = (k * 10 + t).astype(np.int64)
        gpu.process(k, t, v)
        ref.process(k, t, v)
        gpu.watermark(wm)
        ref.watermark(wm)
    assert gpu.stats()["slow_path_records"] > 0
    assert_rows_equal(gpu.rows(), ref.rows())
    assert_side_equal(gpu.side_rows(), ref.side_rows())
    assert gpu.late_dropped == ref.late_dropped
    gpu.close()


def _run_device(cfg, batches, wms, **gpu_kw):
    """Like _run_both, but the GPU side gets HBM-resident torch columns: pushes are asynchronous and
    are only settled by the watermark that follows them."""
    import torch
    gpu = _gpu_op(**cfg, **gpu_kw)
    ref = orc.WindowOperatorOracle(**cfg)
    rows = []
    for (k, t, v), wm in zip(batches, wms):
        if len(k):
            gpu.process_batch(*(torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (k, t, v)))
        ref.process(k, t, v)
        rows.append(gpu.process_watermark(wm))
        ref.watermark(wm)
    st = gpu.stats()
    gpu.close()
    return np.concatenate(rows), ref.rows(), st


@pytest.mark.parametrize("cfg", [dict(assigner="sliding", size=5000, slide=1000, lateness=1),
                                 dict(assigner="sliding", size=5000, slide=1000)], ids=["windows", "panes"])
def test_gpu_burst_suspends_and_resumes_async(cfg):
    # 2^20 distinct keys x 5 sliding windows (or one pane) in ONE asynchronous push into a table sized
    # for 1000 entries: k_aggregate suspends over and over; the watermark queued behind the push is
    # skipped on the device and fired again after the host grew the table and resumed the push
    batches, wms = _stream(1 << 20, 1 << 20, 1 << 40, bound=100, jitter=100, rate=1_000_000)
    g, r, st = _run_device(cfg, batches, wms, expected_entries=1000)
    assert st["table_grows"] >= (1 if _panes(cfg) else 3)
    assert_rows_equal(g, r)


@pytest.mark.parametrize("async_input", [True, False], ids=["async-input", "sync-input"])
@pytest.mark.parametrize("cfg", [dict(assigner="tumbling", size=1000),
                                 dict(assigner="sliding", size=3000, slide=1000, lateness=500),
                                 dict(assigner="sliding", size=3000, slide=1000),
                                 dict(assigner="session", gap=700)],
                         ids=["tumbling", "sliding-late", "panes", "sessions"])
def test_gpu_async_pipeline_deferred_clear(cfg, async_input):
    # the bench's step shape: device push, watermark queued without waiting, pending rows cleared
    # without waiting (applied when the next push settles the sequence).  Rows of odd epochs are
    # cleared, rows of even epochs kept; the kept rows must be exactly the oracle's rows of those epochs.
    # With async input each batch is partitioned on the input stream beside the previous batch's
    # aggregation (fw_set_async_input); without it everything runs on the operator's stream.
    import torch
    batches, wms = _stream(400_000, 20_000, 50_000, bound=300, jitter=900, rate=200_000)
    gpu = _gpu_op(**cfg, expected_entries=1000, async_input=async_input)
    ref = orc.WindowOperatorOracle(**cfg)
    kept = []
    for e, ((k, t, v), wm) in enumerate(zip(batches, wms)):
        if len(k):
            gpu.process_batch(*(torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (k, t, v)))
        ref.process(k, t, v)
        gpu.advance_watermark(wm, wait=False)
        ref.watermark(wm)
        if e % 2:
            gpu.clear_pending()
        else:
            kept.append(gpu.drain_rows(e))
    g = np.concatenate(kept)
    r = ref.rows()
    r = r[r["epoch"] % 2 == 0]
    assert_rows_equal(g, r)
    assert gpu.stats()["late_records_dropped"] == ref.late_dropped
    gpu.close()


def test_gpu_async_input_toggled_mid_stream():
    # fw_set_async_input switched off and on between device pushes (bench.py's isolated pass does this): the switch
    # synchronizes, and the rows equal the oracle's whatever stream each batch was partitioned on
    import torch
    cfg = dict(assigner="tumbling", size=1000)
    batches, wms = _stream(600_000, 25_000, 40_000, bound=300, jitter=900, rate=200_000)
    gpu = _gpu_op(**cfg, expected_entries=1000)
    ref = orc.WindowOperatorOracle(**cfg)
    rows = []
    for e, ((k, t, v), wm) in enumerate(zip(batches, wms)):
        if e % 5 == 2:
            gpu.set_async_input(e % 2 == 0)
        if len(k):
            gpu.process_batch(*(torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (k, t, v)))
        ref.process(k, t, v)
        gpu.advance_watermark(wm, wait=False)
        ref.watermark(wm)
        rows.append(gpu.drain_rows(e))
    assert_rows_equal(np.concatenate(rows), ref.rows())
    assert gpu.stats()["late_records_dropped"] == ref.late_dropped
    gpu.close()


def test_gpu_late_burst_suspends_ordered_path():
    # a burst of late records for new keys, all within the allowed lateness: each one creates a
    # window on the ordered path and fires it at once, so k_slow runs out of region room and of
    # fired-row buffer, suspends, and is resumed chunk-exactly after the host grows both
    cfg = dict(assigner="tumbling", size=1000, lateness=1 << 40)
    n = 1 << 20
    k1 = np.arange(n, dtype=np.int64)
    k2 = np.arange(n, 2 * n, dtype=np.int64) * 7919
    t1, t2 = k1 % 1000, (k2 % 997)
    batches = [(k1, t1, k1 & 0xFF), (k2, t2, k2 & 0xFFF), (k1[:0], t1[:0], k1[:0])]
    wms = [5000, 6000, (1 << 63) - 1]
    for device in (False, True):
        if device:
            g, r, st = _run_device(cfg, batches, wms, expected_entries=1000)
        else:
            g, r, *_ = _run_both(cfg, batches, wms, expected_entries=1000)
            st = None
        assert len(r) == 2 * n
        assert_rows_equal(g, r)
        if st is not None:
            assert st["slow_path_records"] == n and st["table_grows"] >= 1


def test_gpu_key_group_range_subtask():
    # one subtask of parallelism 4 (KeyedOneInputStreamOperatorTestHarness(maxPar, numSubtasks, idx))
    from flink_amd.keygroups import compute_key_group_range_for_operator_index
    from flink_amd.operator import GpuWindowOperator
    kgr = compute_key_group_range_for_operator_index(128, 4, 2)
    keys, ts, vals = generate_host(7, 0, 50_000, 10_000, ts_base=0, rate=100_000, jitter=0)
    kg = orc.key_groups_long(keys, 128)
    sel = (kg >= kgr.start_key_group) & (kg <= kgr.end_key_group)
    op = GpuWindowOperator(TumblingEventTimeWindows.of(100), key_group_range=kgr)
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=100)
    op.process(keys[sel], ts[sel], vals[sel])
    ref.process(keys[sel], ts[sel], vals[sel])
    op.watermark((1 << 63) - 1)
    ref.watermark((1 << 63) - 1)
    assert_rows_equal(op.rows(), ref.rows())
    # a key outside the range is an error, as in the heap backend
    bad = keys[~sel][:1]
    with pytest.raises(RuntimeError):
        op.process(bad, ts[:1], vals[:1])


def test_gpu_no_timestamp_marker():
    from flink_amd.operator import GpuWindowOperator
    op = GpuWindowOperator(TumblingEventTimeWindows.of(100))
    with pytest.raises(RuntimeError, match="Long.MIN_VALUE"):
        op.process(np.array([1]), np.array([-(1 << 63)]), np.array([1]))


def test_gpu_device_resident_push_and_generator():
    import torch
    from flink_amd.datagen import generate_device
    from flink_amd.operator import GpuWindowOperator
    n = 1 << 20
    k, t, v, mx = generate_device(0x5EED, 0, n, 1_000_000, ts_base=0, rate=100_000_000, jitter=200)
    hk, ht, hv = generate_host(0x5EED, 0, n, 1_000_000, ts_base=0, rate=100_000_000, jitter=200)
    assert np.array_equal(k.cpu().numpy(), hk) and np.array_equal(t.cpu().numpy(), ht)
    assert np.array_equal(v.cpu().numpy(), hv) and int(mx.item()) == int(ht.max())
    op = GpuWindowOperator(TumblingEventTimeWindows.of(1000))
    op.process(k, t, v)
    op.watermark((1 << 63) - 1)
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=1000)
    ref.process(hk, ht, hv)
    ref.watermark((1 << 63) - 1)
    assert_rows_equal(op.rows(), ref.rows())
    del torch


def test_gpu_key_groups_and_route():
    import ctypes
    import torch
    from flink_amd import _native as N
    from flink_amd.exchange import route_device
    keys, ts, vals = generate_host(11, 0, 300_001, 1 << 40, ts_base=0, rate=1000, jitter=0)
    dk = torch.from_numpy(keys).cuda()
    kg = torch.empty(len(keys), dtype=torch.int32, device="cuda")
    N.check(N.lib().fw_key_groups_device(dk.data_ptr(), None, N.FW_KEY_LONG, len(keys), 128, kg.data_ptr(), None))
    torch.cuda.synchronize()
    assert np.array_equal(kg.cpu().numpy(), orc.key_groups_long(keys, 128))
    for par in (1, 2, 3, 8):
        cols, counts = route_device(dk, torch.from_numpy(ts).cuda(), torch.from_numpy(vals).cuda(), 128, par)
        counts = counts.cpu().numpy()
        rk = cols[0].cpu().numpy()
        dest = orc.key_groups_long(keys, 128).astype(np.int64) * par // 128
        off = 0
        for d in range(par):
            sel = dest == d
            assert counts[d] == sel.sum()
            # stable: arrival order kept inside each destination
            assert np.array_equal(rk[off:off + counts[d]], keys[sel])
            off += counts[d]
    del ctypes


# ---- keyed-state snapshot / restore per key group, with rescaling.
# Reference: AbstractStreamOperator.snapshotState writes keyed state per key group
# (flink-runtime/.../state/heap/HeapKeyedStateBackend.java:289-399, :370-381) and a restore hands the key
# groups to the subtasks of the new parallelism (KeyGroupRangeAssignment.computeKeyGroupRangeForOperatorIndex,
# KeyGroupRangeAssignment.java:85-99).  The run split by a snapshot must emit exactly the rows of an
# uninterrupted run (here: the oracle's).
@pytest.mark.parametrize("cfg,new_par", [
    (dict(assigner="tumbling", size=100), 3),
    (dict(assigner="sliding", size=300, slide=100), 2),
    (dict(assigner="session", gap=40), 2),
    (dict(assigner="tumbling", size=100, lateness=150), 1),
    (dict(assigner="tumbling", size=100, value_type="f64", by="max"), 2),
    (dict(assigner="session", gap=40, value_type="i64", by="min"), 3),
])
def test_gpu_snapshot_restore_rescale(cfg, new_par):
    from flink_amd.keygroups import (assign_to_key_group, compute_key_group_range_for_operator_index,
                                     long_hash_code)
    batches, wms = _stream(120_000, 15_000, 3_000, bound=50, jitter=80, rate=200_000)
    if cfg.get("by"):
        batches = [(k, t, _by_values(v, cfg["value_type"])) for k, t, v in batches]
    ref = orc.WindowOperatorOracle(**cfg)
    for (k, t, v), wm in zip(batches, wms):
        ref.process(k, t, v)
        ref.watermark(wm)
    exp = ref.rows()
    cut = len(batches) // 2
    a = _gpu_op(**cfg, max_parallelism=128)
    for (k, t, v), wm in zip(batches[:cut], wms[:cut]):
        a.process(k, t, v)
        a.watermark(wm)
    first = a.rows()
    entries = a.num_keyed_state_entries
    snap = a.snapshot_state()
    assert sum(len(r) for r in snap.values()) == entries
    a.close()
    parts = []
    for idx in range(new_par):
        kgr = compute_key_group_range_for_operator_index(128, new_par, idx)
        op = _gpu_op(**cfg, max_parallelism=128, key_group_range=kgr)
        op.initialize_state(snap)
        # ordinal aggregates: the restored operator numbers its own records after the restored ordinals
        base = max([int(r["max"].max()) + 1 for kg, r in snap.items() if kg in kgr and len(r)] + [0])
        parts.append((kgr, op, base, []))
    assert sum(op.num_keyed_state_entries for _, op, _, _ in parts) == entries
    got = [first]
    off = sum(len(b[0]) for b in batches[:cut])
    for (k, t, v), wm in zip(batches[cut:], wms[cut:]):
        kg = np.array([assign_to_key_group(long_hash_code(int(x)), 128) for x in k], dtype=np.int64)
        for kgr, op, _, fed in parts:
            m = (kg >= kgr.start_key_group) & (kg <= kgr.end_key_group)
            op.process(k[m], t[m], v[m])
            op.watermark(wm)
            fed.extend((off + np.nonzero(m)[0]).tolist())
        off += len(k)
    for _, op, base, fed in parts:
        r = op.rows()
        r["epoch"] += cut
        if cfg.get("by"):  # minBy / maxBy rows: this operator's ordinals back to the stream's element indices
            late = r["max"] >= base
            r["max"][late] = np.array(fed, dtype=np.int64)[r["max"][late] - base]
        got.append(r)
        op.close()
    assert_rows_equal(np.concatenate(got), exp, "double" if cfg.get("value_type") == "f64" else "long")


@pytest.mark.parametrize("first", [True, "max"], ids=["sum_min", "max"])
@pytest.mark.parametrize("cfg", [dict(assigner="tumbling", size=100), dict(assigner="sliding", size=300, slide=100),
                                 dict(assigner="session", gap=40)], ids=["tumbling", "panes", "session"])
def test_gpu_first_element_snapshot_restore(cfg, first):
    # the first element's ordinal (and max(pos)'s maximum) survive fw_snapshot_key_group / fw_restore_key_group
    # onto two handles; the final watermark then fires the restored windows exactly as the oracle does
    from flink_amd.keygroups import compute_key_group_range_for_operator_index
    cfg = dict(cfg, first=first)
    batches, wms = _stream(60_000, 15_000, 3_000, bound=50, jitter=80, rate=200_000, final=False)
    ref = orc.WindowOperatorOracle(**cfg)
    a = _gpu_op(**cfg, max_parallelism=128)
    for (k, t, v), wm in zip(batches, wms):
        ref.process(k, t, v)
        ref.watermark(wm)
        a.process(k, t, v)
        a.watermark(wm)
    ref.watermark((1 << 63) - 1)
    exp = ref.rows()
    got = [a.rows()]
    snap = a.snapshot_state()
    a.close()
    for idx in range(2):
        op = _gpu_op(**cfg, max_parallelism=128,
                     key_group_range=compute_key_group_range_for_operator_index(128, 2, idx))
        op.initialize_state(snap)
        op.watermark((1 << 63) - 1)
        r = op.rows()
        r["epoch"] = len(batches)
        got.append(r)
        op.close()
    exp["epoch"] = np.minimum(exp["epoch"], len(batches))
    assert_rows_equal(np.concatenate(got), exp)


def test_gpu_restore_refuses_foreign_key_group():
    from flink_amd import _native as N
    from flink_amd.keygroups import assign_to_key_group
    from flink_amd.operator import STATE_DTYPE
    op = _gpu_op("tumbling", 100, max_parallelism=128, key_group_range=KeyGroupRange(0, 63))
    key = next(x for x in range(1000) if assign_to_key_group(x, 128) == 5)
    rows = np.zeros(1, dtype=STATE_DTYPE)
    rows["key"], rows["start"], rows["end"], rows["count"] = key, 0, 100, 1
    with pytest.raises(N.NativeError):
        op.restore_key_group(7, rows)   # the row's key belongs to key group 5
    with pytest.raises(N.NativeError):
        op.restore_key_group(100, rows)  # key group outside the operator's range
    op.restore_key_group(5, rows)
    assert op.num_keyed_state_entries == 1
    op.close()


def _hll_rows_equal(g, r):
    ks = lambda a: a[np.lexsort((a["start"], a["key"], a["epoch"]))]  # noqa: E731
    g, r = ks(g), ks(r)
    assert len(g) == len(r) and len(g) > 0
    for f in ("epoch", "key", "start", "end", "count", "min", "max"):
        assert np.array_equal(g[f], r[f]), f
    np.testing.assert_allclose(g["sum"].view(np.float64), r["sum"].view(np.float64), rtol=1e-9)


@pytest.mark.parametrize("p,zipf", [(14, 1.1), (8, None), (4, 1.1)], ids=["p14-zipf", "p8-uniform", "p4-zipf"])
def test_gpu_hll_vs_oracle(p, zipf):
    # SURVEY §8d C5 shape at parity size: tumbling windows, HyperLogLog per key and window over the value
    # column as items; Zipf keys put most records on a few hot (key, window) register blocks
    from flink_amd import HyperLogLog
    from flink_amd.operator import GpuWindowOperator
    batches, wms = _stream(300_000, 50_000, 20_000, bound=200, jitter=200, rate=200_000, zipf=zipf)
    gpu = GpuWindowOperator(TumblingEventTimeWindows.of(1000), HyperLogLog(p), expected_entries=60_000)
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=1000, hll_p=p)
    for (k, t, v), wm in zip(batches, wms):
        gpu.process(k, t, v)
        ref.process(k, t, v)
        gpu.watermark(wm)
        ref.watermark(wm)
    assert gpu.late_dropped == ref.late_dropped
    _hll_rows_equal(gpu.rows(), ref.rows())
    gpu.close()


@pytest.mark.parametrize("p,zipf", [(10, 1.1), (6, None)], ids=["p10-zipf", "p6-uniform"])
def test_gpu_hll_sliding_vs_oracle(p, zipf):
    # HyperLogLog over sliding windows (WindowedStream.aggregate takes any assigner, WindowedStream.java:687-852):
    # every element raises its register in each of its size / slide windows, each window's registers their own block;
    # registers bit-exact against the oracle's per-window accumulators, late elements dropped alike
    from flink_amd import HyperLogLog
    from flink_amd.operator import GpuWindowOperator
    batches, wms = _stream(120_000, 20_000, 3000, bound=300, jitter=600, rate=50_000, zipf=zipf)
    gpu = GpuWindowOperator(SlidingEventTimeWindows.of(3000, 1000), HyperLogLog(p), expected_entries=30_000)
    ref = orc.WindowOperatorOracle(assigner="sliding", size=3000, slide=1000, hll_p=p)
    for (k, t, v), wm in zip(batches, wms):
        gpu.process(k, t, v)
        ref.process(k, t, v)
        gpu.watermark(wm)
        ref.watermark(wm)
    assert gpu.late_dropped == ref.late_dropped
    _hll_rows_equal(gpu.rows(), ref.rows())
    gpu.close()


@pytest.mark.parametrize("cfg", [dict(assigner="tumbling", size=1000, lateness=700),
                                 dict(assigner="tumbling", size=1000, lateness=700, purging=True),
                                 dict(assigner="sliding", size=2000, slide=500, lateness=300)],
                         ids=["tumbling-lateness", "tumbling-lateness-purging", "sliding-lateness"])
def test_gpu_hll_allowed_lateness_vs_oracle(cfg):
    # HyperLogLog under allowed lateness (WindowOperator.java:379-420, 452-463): a window fires at its maxTimestamp
    # and keeps its registers until its cleanup time; late elements raise them and fire the window again (the
    # ordered replay path estimates from the block it keeps); PurgingTrigger frees the block at every firing
    from flink_amd import HyperLogLog, PurgingTrigger
    from flink_amd.operator import GpuWindowOperator
    batches, wms = _stream(120_000, 10_000, 2000, bound=400, jitter=1500, rate=100_000, zipf=1.1)
    assigner = (TumblingEventTimeWindows.of(cfg["size"]) if cfg["assigner"] == "tumbling"
                else SlidingEventTimeWindows.of(cfg["size"], cfg["slide"]))
    trig = PurgingTrigger.of(EventTimeTrigger.create()) if cfg.get("purging") else None
    gpu = GpuWindowOperator(assigner, HyperLogLog(8), trigger=trig, allowed_lateness=cfg["lateness"],
                            expected_entries=20_000)
    ref = orc.WindowOperatorOracle(**cfg, hll_p=8)
    for (k, t, v), wm in zip(batches, wms):
        gpu.process(k, t, v)
        ref.process(k, t, v)
        gpu.watermark(wm)
        ref.watermark(wm)
    assert gpu.late_dropped == ref.late_dropped
    _hll_rows_equal(gpu.rows(), ref.rows())
    gpu.close()


def test_gpu_hll_register_blocks_are_recycled():
    # many windows over few keys with a pool sized for one window's entries: every fired block must be
    # zeroed and reused, or the pool runs out (FW_ERR_CAPACITY) or stale registers inflate the estimates
    from flink_amd import HyperLogLog
    from flink_amd.operator import GpuWindowOperator
    batches, wms = _stream(400_000, 10_000, 500, bound=50, jitter=50, rate=100_000)
    gpu = GpuWindowOperator(TumblingEventTimeWindows.of(100), HyperLogLog(10), expected_entries=1500)
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=100, hll_p=10)
    for (k, t, v), wm in zip(batches, wms):
        gpu.process(k, t, v)
        ref.process(k, t, v)
        gpu.watermark(wm)
        ref.watermark(wm)
    _hll_rows_equal(gpu.rows(), ref.rows())
    gpu.close()


HLL_SESSION_CFGS = [dict(gap=300, lateness=0, zipf=1.1, bound=200, jitter=300),
                    dict(gap=300, lateness=500, zipf=1.1, bound=400, jitter=1500),
                    dict(gap=50, lateness=200, zipf=None, bound=100, jitter=400),
                    dict(gap=2000, lateness=0, zipf=1.3, bound=200, jitter=200),
                    dict(gap=300, lateness=0, zipf=1.1, bound=200, jitter=300, purging=True),
                    dict(gap=300, lateness=500, zipf=1.1, bound=400, jitter=1500, purging=True),
                    dict(gap=50, lateness=200, zipf=None, bound=100, jitter=400, purging=True)]


@pytest.mark.parametrize("cfg", HLL_SESSION_CFGS, ids=["zipf", "zipf-lateness", "uniform-lateness", "long-gap",
                                                       "zipf-purging", "zipf-lateness-purging",
                                                       "uniform-lateness-purging"])
def test_gpu_hll_sessions_vs_oracle(cfg):
    # a10: HyperLogLog over EventTimeSessionWindows (WindowedStream.aggregate with any assigner, WindowedStream.java:
    # 687-852).  Sessions merge (MergingWindowSet.addWindow, MergingWindowSet.java:150-225) and their accumulators with
    # them (AbstractHeapMergingState.mergeNamespaces, AbstractHeapMergingState.java:67-93; AggregateFunction.merge,
    # AggregateFunction.java:160): the register max of the merged sessions' blocks -- in the parallel flush, in the
    # ordered replay of late elements (late firings, lateness), and across batches.  Registers bit-exact.
    # PurgingTrigger (WindowOperator.java:391-403, 454-463): a firing clears the session's registers (zeroed block)
    # and the session stays in its MergingWindowSet, empty, until later elements or merges fill it again.
    from flink_amd import HyperLogLog, PurgingTrigger
    from flink_amd.operator import GpuWindowOperator
    batches, wms = _stream(200_000, 20_000, 3000, bound=cfg["bound"], jitter=cfg["jitter"], rate=100_000,
                           zipf=cfg["zipf"])
    purging = cfg.get("purging", False)
    trig = PurgingTrigger.of(EventTimeTrigger.create()) if purging else None
    gpu = GpuWindowOperator(EventTimeSessionWindows.with_gap(cfg["gap"]), HyperLogLog(10), trigger=trig,
                            allowed_lateness=cfg["lateness"], expected_entries=20_000)
    ref = orc.WindowOperatorOracle(assigner="session", gap=cfg["gap"], lateness=cfg["lateness"], hll_p=10,
                                   purging=purging)
    for (k, t, v), wm in zip(batches, wms):
        gpu.process(k, t, v)
        ref.process(k, t, v)
        gpu.watermark(wm)
        ref.watermark(wm)
    assert gpu.late_dropped == ref.late_dropped
    g, r = gpu.rows(), ref.rows()
    _hll_rows_equal(g, r)
    # sessions did merge (a session spans more than one element window)
    assert (g["end"] - g["start"] > cfg["gap"]).any()
    gpu.close()


def test_gpu_hll_sessions_hot_partition_split():
    # sessions of a few Zipf keys in 200K-record batches: the hottest partitions are split over several aggregate
    # workgroups, whose deltas merge into the sessions (and their register blocks) at the last chunk
    from flink_amd import HyperLogLog
    from flink_amd.operator import GpuWindowOperator
    batches, wms = _stream(600_000, 200_000, 1000, bound=200, jitter=300, rate=100_000, zipf=1.1)
    gpu = GpuWindowOperator(EventTimeSessionWindows.with_gap(100), HyperLogLog(12), expected_entries=10_000)
    ref = orc.WindowOperatorOracle(assigner="session", gap=100, hll_p=12)
    for (k, t, v), wm in zip(batches, wms):
        gpu.process(k, t, v)
        ref.process(k, t, v)
        gpu.watermark(wm)
        ref.watermark(wm)
    _hll_rows_equal(gpu.rows(), ref.rows())
    gpu.close()


def test_gpu_hll_refuses_unsupported_shapes():
    from flink_amd import HyperLogLog, PurgingTrigger
    from flink_amd import _native as N
    from flink_amd.operator import GpuWindowOperator
    # (sessions with PurgingTrigger are offered: test_gpu_hll_sessions_vs_oracle)
    GpuWindowOperator(EventTimeSessionWindows.with_gap(3000), HyperLogLog(12),
                      trigger=PurgingTrigger.of(EventTimeTrigger.create())).close()
    with pytest.raises(N.NativeError):
        GpuWindowOperator(TumblingEventTimeWindows.of(1000), HyperLogLog(20))


def test_gpu_panes_key_hash_slices():
    # one state region (maxParallelism 1, one sub-partition) holding 20K keys: a window has more keys
    # than k_fire_panes' LDS table, so it is formed in slices of the key-hash space
    cfg = dict(assigner="sliding", size=3000, slide=1000)
    batches, wms = _stream(200_000, 25_000, 20_000, bound=200, jitter=300, rate=50_000)
    g, r, *_ = _run_both(cfg, batches, wms, max_parallelism=1, sub_partitions=1, expected_entries=100_000)
    assert len(g) > 50_000
    assert_rows_equal(g, r)


def test_gpu_panes_hot_partition_split():
    # Zipf keys in 200K-record batches: the hottest partitions exceed one aggregate workgroup's chunk and
    # are split (chunk deltas merged by the last chunk) on the pane path
    cfg = dict(assigner="sliding", size=4000, slide=1000)
    batches, wms = _stream(600_000, 200_000, 1000, bound=200, jitter=300, rate=100_000, zipf=1.1)
    g, r, *_ = _run_both(cfg, batches, wms)
    assert_rows_equal(g, r)


def test_gpu_hll_hot_partition_split():
    # the same split path with HyperLogLog register blocks (blocks are assigned when the merged deltas
    # are claimed in the region)
    from flink_amd import HyperLogLog
    from flink_amd.operator import GpuWindowOperator
    batches, wms = _stream(600_000, 200_000, 1000, bound=200, jitter=300, rate=100_000, zipf=1.1)
    gpu = GpuWindowOperator(TumblingEventTimeWindows.of(1000), HyperLogLog(12), expected_entries=10_000)
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=1000, hll_p=12)
    for (k, t, v), wm in zip(batches, wms):
        gpu.process(k, t, v)
        ref.process(k, t, v)
        gpu.watermark(wm)
        ref.watermark(wm)
    _hll_rows_equal(gpu.rows(), ref.rows())
    gpu.close()


def test_gpu_c2_full_size_properties():
    # BASELINE configs[1] at full size (four 2^24-record batches generated in HBM, 1M keys, 1 s tumbling,
    # bounded out-of-orderness 200 ms), beyond what the oracle finishes in seconds: size-independent
    # properties instead of row-by-row parity.  Conservation of counts, checksum of sums, global min/max,
    # one row per distinct (key, window), and aligned window bounds.
    import torch
    from flink_amd.datagen import generate_device
    n, steps, num_keys, rate = 1 << 24, 4, 1_000_000, 100_000_000
    gpu = _gpu_op("tumbling", size=1000)
    total = 0
    vsum = 0
    vmin, vmax = 1 << 63, -(1 << 63)
    ids = []
    for s in range(steps):
        k, t, v, mx = generate_device(0x5EED, s * n, n, num_keys, ts_base=1_000_000, rate=rate, jitter=200)
        torch.cuda.synchronize()
        total += n
        vsum += int(v.sum().item())
        vmin, vmax = min(vmin, int(v.min().item())), max(vmax, int(v.max().item()))
        ids.append(k * 100_000 + (t - 1_000_000) // 1000)  # (key, window index): ts stays above the base
        gpu.process_batch(k, t, v)
        gpu.watermark(int(mx.item()) - 200)
    gpu.watermark((1 << 63) - 1)
    rows = gpu.rows()
    assert gpu.late_dropped == 0
    gpu.close()
    assert int(rows["count"].sum()) == total
    assert int(rows["sum"].astype(np.int64).sum()) == vsum
    assert int(rows["min"].min()) == vmin and int(rows["max"].max()) == vmax
    assert np.all(rows["end"] - rows["start"] == 1000) and np.all(rows["start"] % 1000 == 0)
    distinct = torch.unique(torch.cat(ids)).numel()
    assert len(rows) == distinct
    assert len(np.unique(rows["key"] * 100_000 + (rows["start"] - 1_000_000) // 1000)) == distinct


@pytest.mark.parametrize("workload", ["c3", "c4", "c5"])
def test_gpu_full_size_count_conservation(workload):
    # SURVEY §8d C3/C4/C5 shapes at full batch size (2^24 records per push, generated in HBM): every record
    # is counted once per window it belongs to (60 sliding windows at C3; one session or one tumbling window
    # at C4/C5) once the final watermark has fired everything; no record is late (bound >= jitter)
    import torch
    from flink_amd.datagen import generate_device, zipf_cdf
    from flink_amd.windowing import HyperLogLog
    n, steps = 1 << 24, 2
    if workload == "c3":
        cfg, keys, rate, jitter, per = dict(assigner="sliding", size=60_000, slide=1000), 2_000_000, 100_000_000, 200, 60
    elif workload == "c4":
        cfg, keys, rate, jitter, per = dict(assigner="session", gap=30_000), 1_000_000, 100_000, 1000, 1
    else:
        cfg, keys, rate, jitter, per = dict(assigner="tumbling", size=1000), 1_000_000, 100_000_000, 200, 1
    cdf = None if workload == "c3" else torch.tensor(zipf_cdf(keys, 1.1), dtype=torch.float64, device="cuda")
    if workload == "c5":
        from flink_amd.operator import GpuWindowOperator
        gpu = GpuWindowOperator(TumblingEventTimeWindows.of(1000, 0), HyperLogLog(14),
                                expected_entries=2_000_000)  # 2 live windows of up to 1M keys (40 GB pool)
    else:
        gpu = _gpu_op(**cfg)
    for s in range(steps):
        k, t, v, mx = generate_device(0x5EED, s * n, n, keys, ts_base=1_000_000, rate=rate, jitter=jitter,
                                      cdf_dev=cdf)
        gpu.process_batch(k, t, v)
        gpu.watermark(int(mx.item()) - jitter)
    gpu.watermark((1 << 63) - 1)
    rows = gpu.rows()
    assert gpu.late_dropped == 0
    gpu.close()
    assert int(rows["count"].sum()) == per * n * steps
    if workload == "c4":  # sessions of one key never overlap or touch (gap-separated)
        r = rows[np.lexsort((rows["start"], rows["key"]))]
        same = r["key"][1:] == r["key"][:-1]
        assert np.all(r["start"][1:][same] > r["end"][:-1][same])


def test_gpu_restore_merges_repeated_rows():
    # one restore call holding the same (key, window) twice merges the rows (AggregateFunction.merge), in order:
    # the windows come back with doubled count and sum, the same min and max
    batches, wms = _stream(40_000, 10_000, 500, bound=50, jitter=80, rate=200_000, final=False)
    a = _gpu_op("tumbling", 1000)
    for (k, t, v), wm in zip(batches, wms):
        a.process(k, t, v)
        a.watermark(wm)
    snap = a.snapshot_state()
    a.close()
    b = _gpu_op("tumbling", 1000)
    for kg, rows in snap.items():
        if len(rows):
            b.restore_key_group(kg, np.concatenate([rows, rows]))
    for kg, rows in snap.items():
        got = b.snapshot_key_group(kg)
        assert len(got) == len(rows)
        got = got[np.lexsort((got["start"], got["key"]))]
        exp = rows[np.lexsort((rows["start"], rows["key"]))]
        assert np.array_equal(got["count"], 2 * exp["count"])
        assert np.array_equal(got["sum"], 2 * exp["sum"])
        assert np.array_equal(got["min"], exp["min"]) and np.array_equal(got["max"], exp["max"])
    b.close()


@pytest.mark.parametrize("purging", [False, True])
def test_gpu_sessions_many_in_flight_per_key(purging):
    # one key holding hundreds of in-flight sessions (gap 10 ms, allowedLateness 10 s: a session stays in the
    # MergingWindowSet until maxTimestamp + 10 s), with late elements that fire them again and elements that
    # bridge two sessions, modelled on WindowOperatorTest's session lateness cases (WindowOperatorTest.java
    # :1980-2266).  The reference's MergingWindowSet has no bound on a key's windows.
    rng = np.random.default_rng(11)
    base = 1_000_000
    t0 = base + 18 * np.arange(700)                              # key 0: one session every 18 ms
    bridge = base + 18 * rng.integers(0, 700, 80) + 8            # [t + 8, t + 18) touches two sessions
    late = base + 18 * rng.integers(0, 700, 150) + rng.integers(0, 9, 150)
    k_other = rng.integers(1, 50, 4000)
    t_other = base + rng.integers(0, 13_000, 4000)
    keys = np.concatenate([np.zeros(700 + 80 + 150, dtype=np.int64), k_other])
    ts = np.concatenate([t0, bridge, late, t_other]).astype(np.int64)
    order = np.argsort(ts + rng.integers(-300, 300, len(ts)), kind="stable")  # mostly in order, 300 ms jitter
    keys, ts = keys[order], ts[order]
    vals = rng.integers(-1000, 1000, len(ts))
    batches, wms, mx = [], [], -(1 << 63)
    for b in range(0, len(ts), 400):
        sl = slice(b, b + 400)
        batches.append((keys[sl], ts[sl], vals[sl]))
        mx = max(mx, int(ts[sl].max()))
        wms.append(mx - 500)
    batches.append((keys[:0], ts[:0], vals[:0]))
    wms.append((1 << 63) - 1)
    cfg = dict(assigner="session", gap=10, lateness=10_000, purging=purging)
    g, r, gs, rs, gl, rl = _run_both(cfg, batches, wms, max_parallelism=1, sub_partitions=1)
    assert_rows_equal(g, r)
    assert gl == rl
    assert (r["key"] == 0).sum() > 600  # the hot key's sessions (and their late firings)


NARROW_CONFIGS = [
    dict(assigner="tumbling", size=1000),
    dict(assigner="sliding", size=3000, slide=1000),
    dict(assigner="session", gap=300, lateness=200),
]


@pytest.mark.parametrize("first", [False, True], ids=["count_sum", "sum_passthrough"])
@pytest.mark.parametrize("value_type", ["i16", "i8", "f32"])
@pytest.mark.parametrize("cfg", NARROW_CONFIGS, ids=[c["assigner"] for c in NARROW_CONFIGS])
def test_gpu_short_byte_float_fields(cfg, value_type, first):
    # a9: Short / Byte sums wrap to their width (SumFunction.ShortSum / ByteSum), Float sums add in float
    # (FloatSum), min/max by compareTo (SumFunction.java:34-107, ComparableAggregator.java:72-94)
    batches, wms = _stream(120_000, 15_000, 2000, bound=400, jitter=900, rate=100_000)
    if value_type == "i16":
        conv = lambda v: ((v & 0xFFFF) - 0x8000).astype(np.int64)  # noqa: E731
    elif value_type == "i8":
        conv = lambda v: ((v & 0xFF) - 0x80).astype(np.int64)  # noqa: E731
    else:
        # positive values: a float sum's error relative to the sum stays at float precision (no cancellation)
        conv = lambda v: ((v & 0xFFFFF).astype(np.float32) / np.float32(3.0) + 1).astype(np.float64)  # noqa: E731
    batches = [(k, t, conv(v)) for k, t, v in batches]
    cfg = dict(cfg, value_type=value_type, first=first)
    g, r, *_ = _run_both(cfg, batches, wms)
    assert_rows_equal(g, r, _VT[value_type])
    if value_type == "f32" and not first and cfg["assigner"] != "session":
        # and against the exact sums of the windows' elements, with the tight single-rounding bound
        size, slide = cfg["size"], cfg.get("slide", cfg["size"])
        windows_of = lambda t: [t - t % slide - j * slide for j in range(size // slide)]  # noqa: E731 (ts >= 0)
        keys, ts, vals = (np.concatenate(c) for c in zip(*batches))
        wm_prev = np.concatenate([np.full(len(b[0]), wms[i - 1] if i else -(1 << 63), dtype=np.int64)
                                  for i, b in enumerate(batches)])
        assert_f32_sums_near_exact(g, keys, ts, vals, windows_of, size, wm_prev)


def _count_op(size, slide, evict_after=False, value_type="i64", **kw):
    from flink_amd import CountWindows
    from flink_amd.operator import GpuWindowOperator
    return GpuWindowOperator(CountWindows.of(size, slide, evict_after), FirstElementReduce(_VT[value_type], "sum"),
                             **kw)


def _count_rows(rows):
    return sorted(tuple(int(r[f]) for f in ("key", "start", "end", "count", "sum", "min", "max")) for r in rows)


@pytest.mark.parametrize("case", KATS["count_windows"], ids=[c["name"] for c in KATS["count_windows"]])
def test_gpu_count_window_kats(case):
    # a14: EvictingWindowOperatorTest count-trigger / count-evictor sequences, compared as a sorted multiset
    # after each phase (TestHarnessUtil.assertOutputEqualsSorted)
    from collections import Counter
    op = _count_op(case["size"], case["slide"], case["evict_after"])
    ids = {"key1": 1, "key2": 2}
    names = {v: k for k, v in ids.items()}
    expected = Counter()
    for ph in case["phases"]:
        k = np.array([ids[x] for x, _ in ph["input"]], dtype=np.int64)
        op.process(k, np.zeros_like(k), np.array([v for _, v in ph["input"]], dtype=np.int64))
        expected.update(tuple(e) for e in ph["expected"])
        assert Counter((names[int(r["key"])], int(r["sum"])) for r in op.rows()) == expected
    assert all(r["end"] == (1 << 63) - 1 and r["start"] == -(1 << 63) for r in op.rows())
    op.close()


COUNT_CONFIGS = [(10, 5, False), (10, 10, False), (7, 3, False), (4, 6, False), (4, 2, True), (5, 3, True),
                 (1, 1, False)]


@pytest.mark.parametrize("value_type", ["i64", "i32", "f64", "i16", "f32"])
@pytest.mark.parametrize("size,slide,after", COUNT_CONFIGS, ids=[f"{a}_{b}_{c}" for a, b, c in COUNT_CONFIGS])
def test_gpu_count_windows_vs_oracle(size, slide, after, value_type):
    # WindowWordCount's countWindow(10, 5).sum(1) and its tumbling / evict-after variants over ragged batches
    # (a key's run straddles pushes, so fired windows read the ring of earlier elements); rows bit-exact
    keys, _, vals = generate_host(0xC0DE, 0, 60_000, 700, ts_base=0, rate=1_000_000, jitter=0, zipf_s=1.05)
    if value_type == "f64":
        vals = (vals & 0xFFFFF).astype(np.float64) / 7.0
    elif value_type == "f32":
        vals = ((vals & 0xFFFFF).astype(np.float32) / np.float32(3.0) + 1).astype(np.float64)
    elif value_type == "i16":
        vals = ((vals & 0xFFFF) - 0x8000).astype(np.int64)
    elif value_type == "i32":
        vals = ((vals & 0xFFFFFFFF) - (1 << 31)).astype(np.int64)
    gpu = _count_op(size, slide, after, value_type, expected_entries=1024)
    ref = orc.CountWindowOracle(size, slide, after, value_type=value_type)
    cuts = [0, 1, 17, 4096, 4097, 20_000, 20_001, 45_000, 60_000]
    for a, b in zip(cuts, cuts[1:]):
        gpu.process(keys[a:b], np.zeros(b - a, dtype=np.int64), vals[a:b])
        ref.process(keys[a:b], vals[a:b].view(np.int64) if vals.dtype == np.float64 else vals[a:b])
        gpu.watermark(b)  # watermarks fire nothing for GlobalWindows
    g, r = gpu.rows(), ref.rows()
    assert len(g) == len(r) > 0
    assert _count_rows(g) == _count_rows(r)
    gpu.close()


def test_gpu_count_windows_device_batches_and_capacity():
    # device-resident pushes of a larger stream; then a stream with more distinct keys than expected_entries
    # is refused with FW_ERR_CAPACITY rather than dropping elements
    import torch
    from flink_amd import _native as N
    keys, _, vals = generate_host(7, 0, 1 << 20, 50_000, ts_base=0, rate=1_000_000, jitter=0)
    gpu = _count_op(10, 5, expected_entries=1 << 16)
    ref = orc.CountWindowOracle(10, 5, value_type="i64")
    for b in range(0, len(keys), 1 << 18):
        sl = slice(b, b + (1 << 18))
        kd, vd = torch.from_numpy(keys[sl]).cuda(), torch.from_numpy(vals[sl]).cuda()
        gpu.process(kd, torch.zeros_like(kd), vd)
        ref.process(keys[sl], vals[sl])
    assert _count_rows(gpu.rows()) == _count_rows(ref.rows())
    gpu.close()
    small = _count_op(10, 5, expected_entries=100)
    with pytest.raises(N.NativeError) as ei:
        k = np.arange(1000, dtype=np.int64)
        small.process(k, k, k)
    assert ei.value.code == N.FW_ERR_CAPACITY
    small.close()
