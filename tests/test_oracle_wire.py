"""f2: the CPU restatement of Flink's wire format (oracle/wire_oracle.*), pinned by the reference's own bytes.

StreamElementSerializer (SJ/runtime/streamrecord/StreamElementSerializer.java:54-58, 167-221) behind
SpanningRecordSerializer's 4-byte big-endian length (RT/io/network/api/serialization/SpanningRecordSerializer.java:
76-98).  The fixture (tests/golden/make_wire_fixture.py) is an event-time timer the reference's heap backend wrote
into win-op-migration-test-reduce-event-time-flink1.4-snapshot: TimeWindow [0, 3000) as two big-endian longs and
its timestamp 2999 — the encodings of a fired row's window fields and of its element timestamp."""
import json
import os
import struct

import numpy as np

from oracle import oracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))
F3 = [("long", "key"), ("long", "skip"), ("int", "value")]


def test_reference_bytes_pin_the_long_encoding():
    fx = json.load(open(os.path.join(HERE, "golden", "wire_fixture.json")))
    entry = bytes.fromhex(fx["timer_entry_hex"])
    row = np.zeros(1, dtype=orc.ROW_DTYPE)
    row["key"], row["start"], row["end"] = 1, fx["start"], fx["end"]
    el = orc.wire_encode(row, [("long", "start"), ("long", "end")])
    # length 25, tag 0 (record with timestamp), timestamp = maxTimestamp, then Tuple2<Long, Long>(start, end)
    assert el[:5] == struct.pack(">IB", 25, 0)
    assert el[5:13] == entry[21:29]   # the timer's timestamp: BE i64 2999
    assert el[13:21] == entry[5:13]   # TimeWindow.start: BE i64 0
    assert el[21:29] == entry[13:21]  # TimeWindow.end: BE i64 3000
    # the key: StringValue.writeString("key1") = length + 1 as a varint, then the chars
    assert entry[:5] == bytes([5]) + b"key1"


def test_element_layouts_by_hand():
    # StreamElementSerializer.serialize, element by element
    w = orc.WireStream(F3)
    w.record([7, -1, -5], ts=1000)
    w.record([8, 2, 3])
    w.watermark(999)
    w.status(0)
    w.latency(5, 1, 2, 3)
    b = w.bytes()
    exp = (struct.pack(">IBqqqi", 1 + 8 + 20, 0, 1000, 7, -1, -5) + struct.pack(">IBqqi", 1 + 20, 1, 8, 2, 3)
           + struct.pack(">IBq", 9, 2, 999) + struct.pack(">IBi", 5, 4, 0) + struct.pack(">IBqqqi", 29, 3, 5, 1, 2, 3))
    assert b == exp
    (k, t, v), st, rc = orc.wire_decode(b, F3)
    assert rc == 0
    assert list(k) == [7, 8] and list(v) == [-5, 3] and list(t) == [1000, -(1 << 63)]
    assert (st["watermarks"], st["statuses"], st["latency_markers"], st["watermark"], st["status"]) == (1, 1, 1, 999, 0)
    assert st["consumed"] == len(b)


def test_every_field_kind_round_trips():
    fields = [("byte", "skip"), ("short", "key"), ("boolean", "skip"), ("float", "value"), ("double", "skip"),
              ("int", "skip"), ("long", "skip")]
    f = np.float32(-1.25)
    w = orc.WireStream(fields)
    w.record([-3, -300, 1, struct.unpack("<q", struct.pack("<d", float(f)))[0],
              struct.unpack("<q", struct.pack("<d", 2.5))[0], -7, 1 << 40], ts=5)
    (k, t, v), st, rc = orc.wire_decode(w.bytes(), fields)
    assert rc == 0 and k[0] == -300 and t[0] == 5
    assert struct.unpack("<d", struct.pack("<q", int(v[0])))[0] == -1.25  # Float widened to double


def test_partial_trailing_element_and_corrupt_tags():
    w = orc.WireStream(F3)
    for i in range(5):
        w.record([i, 0, i], ts=i)
    b = w.bytes()
    for cut in (1, 3, 4, 10, 29):
        (k, t, v), st, rc = orc.wire_decode(b[:-cut], F3)
        assert rc == 0 and len(k) == 4 and st["consumed"] == 4 * 33
    bad = bytearray(b)
    bad[33 + 4] = 9  # the second element's tag
    (k, _, _), st, rc = orc.wire_decode(bytes(bad), F3)
    assert rc == -1 and st["bad_tag"] == 9 and len(k) == 1 and st["consumed"] == 33
    other = struct.pack(">IBq", 9, 0, 1)  # a record element of another layout
    _, st, rc = orc.wire_decode(b + other, F3)
    assert rc == -1 and st["bad_tag"] == -2


def test_encode_rows_and_decode_them_back():
    rng = np.random.default_rng(3)
    rows = np.zeros(50, dtype=orc.ROW_DTYPE)
    rows["key"] = rng.integers(-1000, 1000, 50)
    rows["start"] = rng.integers(0, 1 << 40, 50)
    rows["end"] = rows["start"] + 1000
    rows["count"] = rng.integers(1, 100, 50)
    rows["sum"] = rng.integers(-(1 << 40), 1 << 40, 50)
    out = [("long", "key"), ("long", "end"), ("long", "count"), ("long", "sum")]
    b = orc.wire_encode(rows, out)
    back = [("long", "key"), ("long", "skip"), ("long", "skip"), ("long", "value")]
    (k, t, v), st, rc = orc.wire_decode(b, back)
    assert rc == 0 and list(k) == list(rows["key"]) and list(v) == list(rows["sum"])
    assert list(t) == list(rows["end"] - 1)  # window.maxTimestamp()


# ---- String fields (StringSerializer -> StringValue.writeString / readString, StringValue.java:745-817)
S2 = [("string", "key"), ("int", "value")]  # WindowWordCount's Tuple2<String, Integer>


def test_string_value_pinned_by_reference_bytes():
    # the heap backend wrote the key "key1" with StringSerializer: StringValue.writeString's bytes
    from flink_amd.keygroups import string_hash_code, string_key_id
    fx = json.load(open(os.path.join(HERE, "golden", "wire_fixture.json")))
    sv = bytes.fromhex(fx["timer_entry_hex"])[:5]
    assert orc.write_string("key1") == sv
    el = struct.pack(">IBq", 1 + 8 + len(sv) + 4, 0, 2999) + sv + struct.pack(">i", 3)
    (k, kh, t, v), st, rc = orc.wire_decode_keyed(el, S2)
    assert rc == 0 and st["records"] == 1 and st["consumed"] == len(el)
    assert (int(kh[0]), int(k[0]), int(t[0]), int(v[0])) == (string_hash_code("key1"), string_key_id("key1"), 2999, 3)
    assert orc.string_key_id("key1") == string_key_id("key1")


def test_string_fields_varints_and_nulls():
    from flink_amd.keygroups import string_hash_code, string_key_id
    # chars of one, two and three varint bytes, the empty string, a length needing a two-byte varint
    words = ["a", "wörd", "日本語", "", "x" * 130, "€uro"]
    assert orc.write_string("x" * 130)[:2] == bytes([131 & 0x7f | 0x80, 131 >> 7])
    assert orc.write_string("日")[1:] == bytes([0xE5 & 0x7f | 0x80, (0x65E5 >> 7) & 0x7f | 0x80, 0x65E5 >> 14])
    fields = [("long", "skip"), ("string", "key"), ("string", "skip"), ("int", "value")]
    w = orc.WireStream(fields)
    for i, s in enumerate(words):
        w.record_str([i, s, None if i % 2 else "skipped", i * 10], ts=i if i % 3 else None)
        w.watermark(100 + i)
    (k, kh, t, v), st, rc = orc.wire_decode_keyed(w.bytes(), fields)
    assert rc == 0 and st["records"] == len(words) and st["watermarks"] == len(words)
    assert list(kh) == [string_hash_code(s) for s in words]
    assert list(k) == [string_key_id(s) for s in words]
    assert list(v) == [i * 10 for i in range(len(words))]
    # a String key needs the hash column; a null key is a corrupt element
    (_, _, _), _, rc = orc.wire_decode(w.bytes(), fields)
    assert rc == -3
    bad = orc.WireStream(fields)
    bad.record_str([1, "ok", "x", 1], ts=1)
    bad.record_str([2, None, "x", 2], ts=2)
    _, st, rc = orc.wire_decode_keyed(bad.bytes(), fields)
    assert rc == -1 and st["bad_tag"] == -4 and st["records"] == 1
    # an element whose length prefix disagrees with its String fields
    short = struct.pack(">IBq", 9 + 4, 0, 5) + orc.write_string("abcdef")[:4]
    _, st, rc = orc.wire_decode_keyed(short, [("string", "key")])
    assert rc == -1 and st["bad_tag"] == -2
