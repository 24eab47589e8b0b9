"""f1 on the GPU: the reference's own savepoints (WindowOperatorMigrationTest's win-op-migration-test-*-snapshot
fixtures, tests/golden/heap/) restored into the GPU operators, which then fire what the reference's restore tests
expect (testRestoreReducingEventTimeWindows, WindowOperatorMigrationTest.java:381-433; testRestoreApplyEventTime
Windows, :497-548), and the GPU state snapshotted back into the heap backend's key-group format."""
import os

import numpy as np
import pytest

from flink_amd import FirstElementReduce, TumblingEventTimeWindows
from flink_amd import heapstate as H
from flink_amd.keygroups import string_hash_code

pytestmark = pytest.mark.gpu

HEAP = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "heap")
TUP = H.TupleSer(H.StringSer(), H.IntSer())
IDS = {"key1": 1, "key2": 2}
NAMES = {v: k for k, v in IDS.items()}
# (epoch, (key, sum), timestamp): watermarks 2999, 3999, 4999, 5999 (:416-429, :531-544)
EXPECTED = sorted([(0, ("key1", 3), 2999), (0, ("key2", 3), 2999), (3, ("key2", 2), 5999)])


def _restored(name, version):
    with open(os.path.join(HEAP, f"win-op-migration-test-{name}-flink{version}-snapshot"), "rb") as f:
        snap = H.read_operator_snapshot(f.read())
    val = TUP if name == "reduce-event-time" else H.ListSer(TUP)
    _, groups = H.read_heap_keyed_state(snap["managed_keyed"][0], {"window-contents": (H.TimeWindowSer(),
                                                                                       H.StringSer(), val)})
    timers = H.event_timers(H.read_timers(snap["raw_keyed"][0], H.StringSer(), H.TimeWindowSer()))
    return groups[0]["window-contents"], timers


@pytest.mark.parametrize("version", ["1.3", "1.4"])
def test_gpu_restores_reducing_window_savepoint(version):
    from flink_amd.operator import STATE_DTYPE, GpuWindowOperator
    mappings, timers = _restored("reduce-event-time", version)
    rows, passthrough = H.reduce_rows_from_heap(mappings, timers, IDS.__getitem__, 1)
    # the harness' operator: one key group (maxParallelism 1), String keys hashed by the host
    op = GpuWindowOperator(TumblingEventTimeWindows.of(3000), FirstElementReduce("int"), key_type="hashed",
                           max_parallelism=1)
    arr = np.zeros(len(rows), dtype=STATE_DTYPE)
    for i, r in enumerate(rows):
        for f in STATE_DTYPE.names:
            arr[i][f] = r[f]
    op.restore_key_group(0, arr)
    # snapshot before firing: the same mappings in the heap format, section bytes included
    back = H.heap_from_reduce_rows(op.snapshot_key_group(0), NAMES.__getitem__, passthrough, 1)
    assert sorted(back) == sorted(mappings)
    ser = {"window-contents": (H.TimeWindowSer(), H.StringSer(), TUP)}
    sec = H.write_key_group_section(0, [(0, "window-contents", back)], ser)
    assert sorted(H.read_key_group_section(H.DataInput(sec), 0, ["window-contents"], ser)["window-contents"]) \
        == sorted(mappings)
    out = []
    for wm in (2999, 3999, 4999, 5999):
        for r in op.process_watermark(wm):
            e = list(passthrough[int(r["max"])])
            e[1] = int(r["sum"])
            out.append((int(r["epoch"]), tuple(e), int(r["end"]) - 1))
    assert sorted(out) == EXPECTED
    # later elements are numbered after the restored ordinals
    op.process(np.array([1]), np.array([7000]), np.array([5]), key_hash=np.array([string_hash_code("key1")]))
    r = op.process_watermark(8999)
    assert len(r) == 1 and int(r["max"][0]) == len(rows)
    op.close()


@pytest.mark.parametrize("version", ["1.3", "1.4"])
def test_gpu_restores_list_window_savepoint(version):
    from flink_amd.listwindow import GpuListWindowOperator
    mappings, timers = _restored("apply-event-time", version)
    lists, elems = H.list_state_from_heap(mappings, timers, IDS.__getitem__, lambda v: v[1])
    op = GpuListWindowOperator(TumblingEventTimeWindows.of(3000), value_type="int", key_type="hashed",
                               max_parallelism=1,
                               window_function=lambda k, w, el: (NAMES[k], int(el["val"].sum())))
    la = np.zeros(len(lists), dtype=[(f, "<i8") for f in ("key", "start", "end", "trigger_count", "timer", "n_elems")])
    for i, r in enumerate(lists):
        for f in la.dtype.names:
            la[i][f] = r[f]
    ea = np.array(elems, dtype=[("ts", "<i8"), ("val", "<i8"), ("ordinal", "<i8")])
    op.restore_key_group(0, la, ea)
    sl, se = op.snapshot_key_group(0)
    back = H.heap_from_list_state(sl, se, NAMES.__getitem__, lambda e: None)
    assert sorted((m[0], m[1], len(m[2])) for m in back) == sorted((m[0], m[1], len(m[2])) for m in mappings)
    assert op.stats()["keyed_state_entries"] == 3 and op.stats()["event_time_timers"] == 3
    for wm in (2999, 3999, 4999, 5999):
        op.watermark(wm)
    got = sorted((e, out, int(r["end"]) - 1) for (e, out), r in zip(op.outputs(), op.rows()))
    assert got == EXPECTED
    op.close()


def _fixture_meta(name, version):
    with open(os.path.join(HEAP, f"win-op-migration-test-{name}-flink{version}-snapshot"), "rb") as f:
        data = f.read()
    snap = H.read_operator_snapshot(data)
    val = TUP if name == "reduce-event-time" else H.ListSer(TUP)
    ser = {"window-contents": (H.TimeWindowSer(), H.StringSer(), val)}
    meta, _ = H.read_heap_keyed_state(snap["managed_keyed"][0], ser)
    tmeta = {}
    H.read_timers(snap["raw_keyed"][0], H.StringSer(), H.TimeWindowSer(), meta=tmeta)
    return data, snap, meta, tmeta[0], ser


@pytest.mark.parametrize("version", ["1.3", "1.4"])
@pytest.mark.parametrize("name", ["reduce-event-time", "apply-event-time"])
def test_gpu_state_writes_reference_savepoint(name, version):
    """Snapshot direction: the reference's savepoint restored into the GPU operator, then the GPU's own snapshot
    (fw_snapshot_key_group / fw_list_snapshot_key_group rows and their trigger-timer flags) written back through the
    heap backend's format -- serialization proxy, key-group section in the heap table's order, timer section, both
    KeyGroupsStateHandles -- is byte-for-byte the reference's file (HeapKeyedStateBackend.java:366-383,
    InternalTimeServiceManager.java:114-118, InternalTimerServiceSerializationProxy.java:92-106)."""
    data, snap, meta, tmeta, ser = _fixture_meta(name, version)
    mappings, timers = _restored(name, version)
    if name == "reduce-event-time":
        from flink_amd.operator import STATE_DTYPE, GpuWindowOperator
        rows, passthrough = H.reduce_rows_from_heap(mappings, timers, IDS.__getitem__, 1)
        op = GpuWindowOperator(TumblingEventTimeWindows.of(3000), FirstElementReduce("int"), key_type="hashed",
                               max_parallelism=1)
        arr = np.zeros(len(rows), dtype=STATE_DTYPE)
        for i, r in enumerate(rows):
            for f in STATE_DTYPE.names:
                arr[i][f] = r[f]
        op.restore_key_group(0, arr)
        snap_rows = op.snapshot_key_group(0)
        back = H.heap_from_reduce_rows(snap_rows, NAMES.__getitem__, passthrough, 1)
        gpu_timers = H.rows_to_timers(snap_rows, NAMES.__getitem__)
    else:
        from flink_amd.listwindow import GpuListWindowOperator
        lists, elems = H.list_state_from_heap(mappings, timers, IDS.__getitem__, lambda v: v[1])
        op = GpuListWindowOperator(TumblingEventTimeWindows.of(3000), value_type="int", key_type="hashed",
                                   max_parallelism=1)
        la = np.zeros(len(lists), dtype=[(f, "<i8") for f in ("key", "start", "end", "trigger_count", "timer",
                                                              "n_elems")])
        for i, r in enumerate(lists):
            for f in la.dtype.names:
                la[i][f] = r[f]
        op.restore_key_group(0, la, np.array(elems, dtype=[("ts", "<i8"), ("val", "<i8"), ("ordinal", "<i8")]))
        sl, se = op.snapshot_key_group(0)
        back, k = [], 0
        for r in sl:  # the list's elements in list order: (key, value) tuples
            key, n = NAMES[int(r["key"])], int(r["n_elems"])
            back.append(((int(r["start"]), int(r["end"])), key, [(key, int(e["val"])) for e in se[k:k + n]]))
            k += n
        gpu_timers = H.rows_to_timers(sl, NAMES.__getitem__)
    op.close()
    assert set(gpu_timers) == timers
    out = H.write_savepoint_key_group_0(meta, tmeta, back, gpu_timers, ser, snap["chain_index"],
                                        snap["managed_keyed"][0].name, snap["raw_keyed"][0].name,
                                        table="nested_maps" if version == "1.3" else "copy_on_write")
    assert out == data


def test_gpu_list_restore_keeps_count_trigger_counts():
    """A CountTrigger window's partial count lives in its "count" ReducingState (CountTrigger.java:41-55): restored
    with it (trigger_counts_from_heap), a window holding 2 elements under CountTrigger.of(3) fires at its next
    element, as the reference's would; restored without it, it waits for 3 more."""
    from flink_amd import CountTrigger
    from flink_amd.listwindow import GpuListWindowOperator
    mappings = [((0, 3000), "key1", [("key1", 4), ("key1", 5)])]
    fired = []
    for counts in (H.trigger_counts_from_heap([((0, 3000), "key1", 2)]), None):
        lists, elems = H.list_state_from_heap(mappings, set(), IDS.__getitem__, lambda v: v[1], trigger_counts=counts)
        op = GpuListWindowOperator(TumblingEventTimeWindows.of(3000), trigger=CountTrigger.of(3), value_type="int",
                                   key_type="hashed", max_parallelism=1)
        la = np.zeros(len(lists), dtype=[(f, "<i8") for f in ("key", "start", "end", "trigger_count", "timer",
                                                              "n_elems")])
        for i, r in enumerate(lists):
            for f in la.dtype.names:
                la[i][f] = r[f]
        op.restore_key_group(0, la, np.array(elems, dtype=[("ts", "<i8"), ("val", "<i8"), ("ordinal", "<i8")]))
        op.process(np.array([1]), np.array([100]), np.array([6]), key_hash=np.array([string_hash_code("key1")]))
        fired.append(len(op.rows()))
        op.close()
    assert fired == [1, 0]
