"""f1: the heap backend's snapshot format (flink_amd/heapstate.py), pinned by the reference's own migration
fixtures (flink-streaming-java/src/test/resources/win-op-migration-test-*-flink1.{3,4}-snapshot, written by
WindowOperatorMigrationTest.java's writeReducingEventTimeWindowsSnapshot / writeApplyEventTimeWindowsSnapshot and
restored by testRestoreReducingEventTimeWindows :381-433 / testRestoreApplyEventTimeWindows :497-548).  The files
are kept as data under tests/golden/heap/; the reader walks them without deserializing any Java object."""
import os

import pytest

from flink_amd import heapstate as H

HEAP = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "heap")
TUP = H.TupleSer(H.StringSer(), H.IntSer())
EXPECTED_TIMERS = {("key1", (0, 3000), 2999), ("key2", (0, 3000), 2999), ("key2", (3000, 6000), 5999)}


def load(name, version):
    with open(os.path.join(HEAP, f"win-op-migration-test-{name}-flink{version}-snapshot"), "rb") as f:
        return f.read()


def serializers(name):
    return {"window-contents": (H.TimeWindowSer(), H.StringSer(), TUP if name == "reduce-event-time" else H.ListSer(TUP))}


@pytest.mark.parametrize("version", ["1.3", "1.4"])
@pytest.mark.parametrize("name", ["reduce-event-time", "apply-event-time"])
def test_reads_migration_fixture(name, version):
    snap = H.read_operator_snapshot(load(name, version))
    assert snap["raw_operator"] is None and snap["managed_operator"] is None
    (mk,), (rk,) = snap["managed_keyed"], snap["raw_keyed"]
    assert list(mk.key_groups()) == [0] and list(rk.key_groups()) == [0]  # the harness' one key group
    meta, groups = H.read_heap_keyed_state(mk, serializers(name))
    assert meta["version"] == (3 if version == "1.3" else 4)
    assert meta["states"] == [("REDUCING" if name == "reduce-event-time" else "LIST", "window-contents")]
    got = sorted(groups[0]["window-contents"], key=lambda m: (m[0], m[1]))
    if name == "reduce-event-time":  # the reduced tuples: testRestoreReducingEventTimeWindows' expected sums
        assert got == [((0, 3000), "key1", ("key1", 3)), ((0, 3000), "key2", ("key2", 3)),
                       ((3000, 6000), "key2", ("key2", 2))]
    else:  # the window contents: (key, 1) elements
        assert got == [((0, 3000), "key1", [("key1", 1)] * 3), ((0, 3000), "key2", [("key2", 1)] * 3),
                       ((3000, 6000), "key2", [("key2", 1)] * 2)]
    timers = H.read_timers(rk, H.StringSer(), H.TimeWindowSer())
    assert H.event_timers(timers) == EXPECTED_TIMERS
    assert timers[0]["window-timers"][1] == []  # no processing-time timers


@pytest.mark.parametrize("version", ["1.3", "1.4"])
@pytest.mark.parametrize("name", ["reduce-event-time", "apply-event-time"])
def test_writes_key_group_sections_byte_exact(name, version):
    # the writer reproduces the heap backend's key-group section (HeapKeyedStateBackend.java:375-381) byte for byte
    data = load(name, version)
    mk = H.read_operator_snapshot(data)["managed_keyed"][0]
    meta, groups = H.read_heap_keyed_state(mk, serializers(name))
    sec = H.write_key_group_section(0, [(0, "window-contents", groups[0]["window-contents"])], serializers(name))
    assert sec == mk.data[mk.offsets[0]:]
    stream, offsets = H.write_keyed_state_stream(mk.data[:meta["header_end"]], [sec])
    assert stream == mk.data and offsets == mk.offsets


def test_string_value_codec():
    # StringValue.writeString: length + 1 as a varint, chars as varints (StringValue.java:789-817)
    w = H.DataOutput()
    for s in ("key1", "", None, "é中" * 50):
        H.StringSer().write(w, s)
    r = H.DataInput(w.getvalue())
    assert [H.StringSer().read(r) for _ in range(4)] == ["key1", "", None, "é中" * 50]
    w = H.DataOutput()
    H.StringSer().write(w, "key1")
    assert w.getvalue() == b"\x05key1"


def test_bridges_round_trip():
    mk = H.read_operator_snapshot(load("reduce-event-time", "1.4"))["managed_keyed"][0]
    _, groups = H.read_heap_keyed_state(mk, serializers("reduce-event-time"))
    ids = {"key1": 1, "key2": 2}
    names = {v: k for k, v in ids.items()}
    rows, pt = H.reduce_rows_from_heap(groups[0]["window-contents"], EXPECTED_TIMERS, ids.__getitem__, 1)
    assert all(r["timer"] == 1 for r in rows)
    back = H.heap_from_reduce_rows(rows, names.__getitem__, pt, 1)
    assert sorted(back) == sorted(groups[0]["window-contents"])
    mk = H.read_operator_snapshot(load("apply-event-time", "1.4"))["managed_keyed"][0]
    _, groups = H.read_heap_keyed_state(mk, serializers("apply-event-time"))
    lists, elems = H.list_state_from_heap(groups[0]["window-contents"], EXPECTED_TIMERS, ids.__getitem__,
                                          lambda v: v[1])
    assert [r["n_elems"] for r in lists] == [2, 3, 3] and len(elems) == 8
    back = H.heap_from_list_state(lists, elems, names.__getitem__, lambda e: None)
    assert [len(m[2]) for m in back] == [2, 3, 3]


def _rewrite(data, name, version, shuffle_seed):
    """every byte of a savepoint file from its content: the mappings and timers (shuffled, then put in the heap's
    iteration order), the host's opaque serializer blocks and handle names"""
    import random
    snap = H.read_operator_snapshot(data)
    mk, rk = snap["managed_keyed"][0], snap["raw_keyed"][0]
    meta, groups = H.read_heap_keyed_state(mk, serializers(name))
    tmeta = {}
    timers = H.read_timers(rk, H.StringSer(), H.TimeWindowSer(), meta=tmeta)
    rnd = random.Random(shuffle_seed)
    mappings = list(groups[0]["window-contents"])
    ev = list(timers[0]["window-timers"][0])
    rnd.shuffle(mappings)
    rnd.shuffle(ev)
    return H.write_savepoint_key_group_0(meta, tmeta[0], mappings, ev, serializers(name), snap["chain_index"],
                                         mk.name, rk.name, table="nested_maps" if version == "1.3" else "copy_on_write")


@pytest.mark.parametrize("version", ["1.3", "1.4"])
@pytest.mark.parametrize("name", ["reduce-event-time", "apply-event-time"])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_writes_savepoint_byte_exact(name, version, seed):
    # snapshot direction (HeapKeyedStateBackend.snapshot, HeapKeyedStateBackend.java:366-383, + the timer services,
    # InternalTimeServiceManager.java:114-118): the serialization proxy header, the key-group section in the heap
    # table's iteration order (1.3: NestedMapsStateTable, 1.4: CopyOnWriteStateTable), the timer section in the
    # HashSet's order, both KeyGroupsStateHandles and the operator snapshot file equal the reference's file
    data = load(name, version)
    assert _rewrite(data, name, version, seed) == data


def test_java_iteration_orders():
    # HashSet: capacity 16 until 13 elements, then 32; buckets by (h ^ h >>> 16) & (cap - 1), insertion order inside
    assert H.hash_set_order([17, 1, 33, 2], lambda x: x) == [17, 1, 33, 2]  # all of 17, 1, 33 in bucket 1 (cap 16)
    assert H.hash_set_order(list(range(13))[::-1], lambda x: x) == list(range(13))  # cap 32 past 12 elements
    assert H.hash_set_order([0x10000, 1], lambda x: x) == [0x10000, 1]  # 0x10000 spreads to bucket 1 too
    # CopyOnWriteStateTable: chains newest first
    same = [(("ns"), "a", 1), (("ns"), "b", 2)]
    assert H.state_table_order(same, lambda k: 7, lambda n: 0) == same[::-1]
    # putEntry doubles when size() > threshold BEFORE adding (CopyOnWriteStateTable.java:486-490): 769 mappings stay
    # at capacity 1024 (threshold 768), the 770th is added to a doubled table
    for m, cap in ((769, 1024), (770, 2048)):
        maps = [("ns", i, i) for i in range(m)]
        b = [H.bit_mix(i ^ 0) & (cap - 1) for i in range(m)]
        want = [maps[i] for i in sorted(range(m), key=lambda i: (b[i], -i))]
        assert H.state_table_order(maps, lambda k: k, lambda n: 0) == want, m
    assert H.long_to_int_with_bit_mixing(0) == 0


def test_trigger_counts_carry_into_list_state():
    counts = H.trigger_counts_from_heap([((0, 3000), "key1", 2), ((3000, 6000), "key2", 1)])
    assert counts == {("key1", (0, 3000)): 2, ("key2", (3000, 6000)): 1}
    lists, _ = H.list_state_from_heap([((0, 3000), "key1", [1, 2]), ((0, 3000), "key2", [3])], set(),
                                      {"key1": 1, "key2": 2}.__getitem__, lambda v: v, trigger_counts=counts)
    assert [r["trigger_count"] for r in lists] == [2, 0]
