"""f2 on the GPU: fw_wire_decode_device / fw_wire_encode_device (flink_amd/wire.py) against the oracle's
sequential restatement of StreamElementSerializer + SpanningRecordSerializer (oracle/wire_oracle.*): columns and
stats bit-exact on mixed streams (records with and without timestamps, watermarks, stream statuses, latency
markers), partial trailing elements at every kind of cut, corrupt tags, every field kind, a 64 MB stream, the
encoder byte-exact on fired rows, and decode -> GpuWindowOperator equal to the oracle operator."""
import struct

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

F3 = [("long", "key"), ("long", "skip"), ("int", "value")]


def _codec(fields, max_bytes=1 << 26):
    from flink_amd.wire import WireCodec, WireLayout
    return WireCodec(WireLayout(fields), max_bytes)


def _gpu_decode(codec, data):
    import torch
    t = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    (k, ts, v), st = codec.decode(t)
    return (k.cpu().numpy(), ts.cpu().numpy(), v.cpu().numpy()), st


def _mixed_stream(n, fields, seed):
    rng = np.random.default_rng(seed)
    w = orc.WireStream(fields)
    wm = 0
    for i in range(n):
        r = rng.random()
        if r < 0.80:
            vals = [int(x) for x in rng.integers(-(1 << 31), 1 << 31, len(fields))]
            w.record(vals, ts=int(rng.integers(0, 1 << 40)) if rng.random() < 0.9 else None)
        elif r < 0.92:
            wm += int(rng.integers(0, 1000))
            w.watermark(wm)
        elif r < 0.96:
            w.status(int(rng.integers(0, 2)) - 1 if rng.random() < 0.5 else 0)
        else:
            w.latency(int(rng.integers(0, 1 << 40)), int(rng.integers(-(1 << 62), 1 << 62)), 7, int(rng.integers(0, 64)))
    return w.bytes()


def _same(g, gs, r, rs):
    for a, b in zip(g, r):
        np.testing.assert_array_equal(a, b)
    for f in ("records", "watermarks", "latency_markers", "statuses", "consumed", "watermark", "status"):
        assert gs[f] == rs[f], f


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_wire_decode_mixed_streams(seed):
    data = _mixed_stream(60_000, F3, seed)
    c = _codec(F3)
    g, gs = _gpu_decode(c, data)
    r, rs, rc = orc.wire_decode(data, F3)
    assert rc == 0 and rs["records"] > 40_000
    _same(g, gs, r, rs)
    c.close()


def test_gpu_wire_decode_partial_tails_and_small_streams():
    data = _mixed_stream(3000, F3, 7)
    c = _codec(F3)
    # cuts inside the length prefix, inside an element, exactly at elements and around chunk boundaries
    for end in [0, 1, 3, 4, 5, 12, 13, 2047, 2048, 2049, 2048 * 5 + 17, 4096 + 63, len(data) - 1, len(data)]:
        g, gs = _gpu_decode(c, data[:end])
        r, rs, rc = orc.wire_decode(data[:end], F3)
        assert rc == 0
        _same(g, gs, r, rs)
    only_wm = orc.WireStream(F3)
    for i in range(500):
        only_wm.watermark(i)
    g, gs = _gpu_decode(c, only_wm.bytes())
    assert gs["records"] == 0 and gs["watermark"] == 499 and gs["watermarks"] == 500
    c.close()


def test_gpu_wire_corrupt_tag_fails_like_the_reference():
    from flink_amd import _native as N
    data = bytearray(_mixed_stream(20_000, F3, 11))
    r, rs, _ = orc.wire_decode(bytes(data), F3)
    # break the tag of the element that starts closest after byte 150000
    pos, starts = 0, []
    while pos + 4 <= len(data):
        starts.append(pos)
        pos += 4 + struct.unpack(">I", bytes(data[pos:pos + 4]))[0]
    at = next(s for s in starts if s >= 150_000)
    data[at + 4] = 9
    r, rs, rc = orc.wire_decode(bytes(data), F3)
    assert rc == -1 and rs["bad_tag"] == 9
    c = _codec(F3)
    import torch
    t = torch.from_numpy(np.frombuffer(bytes(data), dtype=np.uint8).copy()).cuda()
    with pytest.raises(N.NativeError) as ei:
        c.decode(t)
    assert ei.value.code == N.FW_ERR_STATE and "Corrupt stream, found tag: 9" in str(ei.value)
    c.close()


def test_gpu_wire_every_field_kind():
    fields = [("byte", "skip"), ("short", "key"), ("boolean", "skip"), ("float", "value"), ("double", "skip"),
              ("int", "skip"), ("long", "skip")]
    rng = np.random.default_rng(5)
    w = orc.WireStream(fields)
    for i in range(20_000):
        f = np.float32(rng.normal() * 1e3)
        w.record([int(rng.integers(-128, 128)), int(rng.integers(-32768, 32768)), int(rng.integers(0, 2)),
                  struct.unpack("<q", struct.pack("<d", float(f)))[0],
                  struct.unpack("<q", struct.pack("<d", float(rng.normal())))[0], int(rng.integers(-(1 << 31), 1 << 31)),
                  int(rng.integers(-(1 << 62), 1 << 62))], ts=i if i % 3 else None)
    c = _codec(fields)
    g, gs = _gpu_decode(c, w.bytes())
    r, rs, rc = orc.wire_decode(w.bytes(), fields)
    assert rc == 0
    _same(g, gs, r, rs)
    c.close()


def test_gpu_wire_decode_64mb():
    # 2M Tuple3<Long, Long, Integer> records with timestamps, a watermark every 1000 records (vectorised build)
    n, every = 2_000_000, 1000
    rng = np.random.default_rng(9)
    rec = np.zeros(n, dtype=[("len", ">u4"), ("tag", "u1"), ("ts", ">i8"), ("k", ">i8"), ("s", ">i8"), ("v", ">i4")])
    rec["len"], rec["tag"] = 29, 0
    rec["ts"] = np.arange(n) * 5
    rec["k"] = rng.integers(0, 1 << 20, n)
    rec["v"] = rng.integers(-(1 << 31), 1 << 31, n)
    wm = np.zeros(n // every, dtype=[("len", ">u4"), ("tag", "u1"), ("wm", ">i8")])
    wm["len"], wm["tag"], wm["wm"] = 9, 2, (np.arange(n // every) + 1) * every * 5 - 100
    parts = []
    for i in range(n // every):
        parts.append(rec[i * every:(i + 1) * every].tobytes())
        parts.append(wm[i:i + 1].tobytes())
    data = b"".join(parts)
    assert len(data) > 60 << 20
    c = _codec(F3, max_bytes=len(data))
    g, gs = _gpu_decode(c, data)
    assert gs["records"] == n and gs["watermarks"] == n // every and gs["consumed"] == len(data)
    np.testing.assert_array_equal(g[0], rec["k"].astype(np.int64))
    np.testing.assert_array_equal(g[1], rec["ts"].astype(np.int64))
    np.testing.assert_array_equal(g[2], rec["v"].astype(np.int64))
    assert gs["watermark"] == int(wm["wm"][-1])
    c.close()


def test_gpu_wire_encode_fired_rows_and_decode_into_the_operator():
    # decode a channel -> push -> fire -> encode the rows; rows and bytes equal the oracle's
    from flink_amd import TumblingEventTimeWindows
    from flink_amd.operator import GpuWindowOperator
    from flink_amd.windowing import CountSumMinMax
    rng = np.random.default_rng(21)
    w = orc.WireStream(F3)
    for i in range(50_000):
        w.record([int(rng.integers(0, 500)), 0, int(rng.integers(-1000, 1000))], ts=i * 3)
    data = w.bytes()
    c = _codec(F3)
    import torch
    t = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    (k, ts, v), st = c.decode(t)
    op = GpuWindowOperator(TumblingEventTimeWindows.of(1000), CountSumMinMax("int"))
    op.process_batch(k, ts, v)
    op.advance_watermark((1 << 63) - 1)
    view, nrows = op.rows_device()
    out_fields = [("long", "key"), ("long", "start"), ("long", "end"), ("long", "count"), ("long", "sum"),
                  ("long", "min"), ("long", "max")]
    c_out = _codec(out_fields)
    out = c_out.encode(view, nrows).cpu().numpy().tobytes()
    c_out.close()
    rows = op.drain_rows()
    (rk, rt, rv), rs, rc = orc.wire_decode(data, F3)
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=1000, value_type="i32")
    ref.process(rk, rt, rv)
    ref.watermark((1 << 63) - 1)
    rr = ref.rows()
    order = lambda a: np.lexsort((a["start"], a["key"]))  # noqa: E731
    g, r = rows[order(rows)], rr[order(rr)]
    for f in ("key", "start", "end", "count", "sum", "min", "max"):
        np.testing.assert_array_equal(g[f], r[f])
    assert out == orc.wire_encode(rows, out_fields)
    op.close()
    c.close()


# ---- String fields: WindowWordCount's Tuple2<String, Integer> channel
S2 = [("string", "key"), ("int", "value")]


def _word_channel(n, seed=3, every=5000, extra=()):
    """WordCountData's tokens (tests/golden/wordcount_tokens.json) as Tuple2<String, Integer>(word, 1) records with
    timestamps i // 2000 ms (C1), a watermark every `every` records."""
    import json
    import os
    toks = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "wordcount_tokens.json")))["tokens"]
    words = sorted(set(toks)) + list(extra)
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, len(words), n)
    w = orc.WireStream(S2)
    for i, j in enumerate(idx):
        w.record_str([words[j], 1], ts=i // 2000)
        if (i + 1) % every == 0:
            w.watermark(i // 2000)
    return w.bytes(), words, idx


def test_gpu_wire_string_keys_match_the_oracle():
    # ASCII words plus words with two- and three-byte chars, mixed with watermarks; columns and stats bit-exact
    data, words, idx = _word_channel(40_000, extra=("wörd", "日本", "€"))
    c = _codec(S2)
    import torch
    t = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    (k, ts, v, kh), gs = c.decode(t)
    (rk, rkh, rt, rv), rs, rc = orc.wire_decode_keyed(data, S2)
    assert rc == 0
    for a, b in ((k, rk), (kh, rkh), (ts, rt), (v, rv)):
        np.testing.assert_array_equal(a.cpu().numpy(), b)
    for f in ("records", "watermarks", "consumed", "watermark"):
        assert gs[f] == rs[f], f
    c.close()


def test_gpu_wire_word_count_channel_into_the_operator():
    # C1 (ii) from the wire: decode WindowWordCount's channel on the GPU, push (key id, String.hashCode) into a
    # hashed-key operator, window(Tumbling 5 s).sum(1); rows equal the C1 oracle keyed by the word
    from flink_amd import TumblingEventTimeWindows
    from flink_amd.keygroups import string_key_id
    from flink_amd.operator import GpuWindowOperator
    from flink_amd.windowing import CountSumMinMax
    import torch
    n = 120_000
    data, words, idx = _word_channel(n)
    c = _codec(S2)
    t = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    (k, ts, v, kh), st = c.decode(t)
    assert st["records"] == n
    op = GpuWindowOperator(TumblingEventTimeWindows.of(5000), CountSumMinMax("int"), key_type="hashed")
    op.process_batch(k, ts, v, kh)
    op.advance_watermark(st["watermark"])
    op.advance_watermark((1 << 63) - 1)
    g = op.drain_rows()
    op.close()
    c.close()
    ids = {string_key_id(w): j for j, w in enumerate(words)}
    assert len(ids) == len(words)
    g["key"] = [ids[int(x)] for x in g["key"]]
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=5000, value_type="i32")
    ref.process(idx.astype(np.int64), np.arange(n, dtype=np.int64) // 2000, np.ones(n, dtype=np.int64))
    ref.watermark(st["watermark"])
    ref.watermark((1 << 63) - 1)
    r = ref.rows()
    order = lambda a: np.lexsort((a["start"], a["key"]))  # noqa: E731
    g, r = g[order(g)], r[order(r)]
    for f in ("key", "start", "end", "count", "sum", "min", "max"):
        np.testing.assert_array_equal(g[f], r[f])
    assert int(g["count"].sum()) == n


def test_gpu_wire_string_errors():
    from flink_amd import _native as N
    import torch
    w = orc.WireStream(S2)
    w.record_str(["fine", 1], ts=1)
    w.record_str([None, 2], ts=2)  # a null key
    c = _codec(S2)
    with pytest.raises(N.NativeError) as ei:
        c.decode(torch.from_numpy(np.frombuffer(w.bytes(), dtype=np.uint8).copy()).cuda())
    assert ei.value.code == N.FW_ERR_STATE and "null String key" in str(ei.value)
    w = orc.WireStream(S2)
    w.record_str(["y" * 60, 1], ts=1)  # 78 bytes with its prefix: beyond the decoder's 64
    with pytest.raises(N.NativeError) as ei:
        c.decode(torch.from_numpy(np.frombuffer(w.bytes(), dtype=np.uint8).copy()).cuda())
    assert ei.value.code == N.FW_ERR_STATE
    c.close()
