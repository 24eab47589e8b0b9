"""GpuListWindowOperator: the window-contents (ListState) paths on one MI355X — WindowedStream.apply / process
with an Iterable window function, and the EvictingWindowOperator (f4; include/flink_window.h fw_list_*):

  WindowOperator(assigner, ..., ListStateDescriptor("window-contents"), InternalIterableWindowFunction, trigger,
                 allowedLateness, lateDataOutputTag)             (WindowOperator.java:179-212, WindowedStream.java:1080-1123)
  EvictingWindowOperator(..., trigger, evictor, ...)            (EvictingWindowOperator.java:76-98)
  processElement -> process_batch, processWatermark -> process_watermark   (EvictingWindowOperator.java:102-286)

Every firing yields a row (key, window, count, the built-in reduce sum / min / max over the contents, the first
element's arrival ordinal) and, with emit_contents, its elements in list order, on which `window_function(key,
window, elements)` — the host's Iterable function — is applied.  All state lives in HBM and every call goes through
libflinkwin.so; there is no CPU implementation.
"""
import ctypes

import numpy as np

from . import _native as N
from .keygroups import KeyGroupRange
from .operator import _KEY_KINDS, _is_torch
from .windowing import VALUE_TYPES, CountTrigger, EventTimeTrigger, Evictor, Trigger, WindowAssigner

LIST_ROW_FIELDS = ("key", "start", "end", "count", "sum", "min", "max", "first", "elem_off")
LIST_ROW_DTYPE = np.dtype([(f, "<i8") for f in LIST_ROW_FIELDS] + [("epoch", "<i8")])
ELEM_DTYPE = np.dtype([("ts", "<i8"), ("val", "<i8"), ("ordinal", "<i8")])
SIDE_DTYPE = np.dtype([("key", "<i8"), ("ts", "<i8"), ("val", "<i8"), ("epoch", "<i8")])
LIST_STATE_DTYPE = np.dtype([(f, "<i8") for f in ("key", "start", "end", "trigger_count", "timer", "n_elems")])


class GpuListWindowOperator:
    def __init__(self, assigner: WindowAssigner, trigger: Trigger = None, evictor: Evictor = None,
                 allowed_lateness=0, side_output=False, value_type="long", key_type="long", max_parallelism=128,
                 key_group_range: KeyGroupRange = None, emit_contents=True, window_function=None, device=0,
                 expected_elements=0, max_batch=0):
        trigger = trigger or EventTimeTrigger.create()
        nested = getattr(trigger, "nested", trigger)
        if not isinstance(nested, (EventTimeTrigger, CountTrigger)):
            raise ValueError("triggers: EventTimeTrigger, CountTrigger, or PurgingTrigger of either")
        if allowed_lateness < 0:
            raise ValueError("The allowed lateness cannot be negative.")
        kgr = key_group_range or KeyGroupRange(0, max_parallelism - 1)
        c = N.FwListConfig()
        cfg = assigner.config()
        c.assigner = cfg["assigner"]
        c.size, c.slide, c.offset = cfg.get("size", 0), cfg.get("slide", 0), cfg.get("offset", 0)
        if "gap" in cfg:  # EventTimeSessionWindows: the session gap (the merging branch, EvictingWindowOperator:110-170)
            c.size = cfg["gap"]
        c.value_type = VALUE_TYPES[value_type]
        c.key_kind = _KEY_KINDS[key_type]
        c.trigger = N.FW_TRIGGER_COUNT if isinstance(nested, CountTrigger) else N.FW_TRIGGER_EVENT_TIME
        c.trigger_count = nested.count if isinstance(nested, CountTrigger) else 0
        c.purging = int(trigger.purging)
        ev = evictor or Evictor()
        c.evictor, c.evict_after = ev.kind, int(ev.evict_after)
        c.evict_count, c.delta_threshold = int(getattr(ev, "arg", 0)), float(getattr(ev, "threshold", 0.0))
        c.side_output = int(side_output)
        c.emit_contents = int(emit_contents)
        c.max_parallelism = max_parallelism
        c.key_group_start, c.key_group_end = kgr.start_key_group, kgr.end_key_group
        c.device = device
        c.allowed_lateness = allowed_lateness
        c.expected_elements, c.max_batch = expected_elements, max_batch
        self.assigner, self.trigger, self.evictor = assigner, trigger, evictor
        self.value_type, self.key_group_range = value_type, kgr
        self.emit_contents, self.window_function = bool(emit_contents), window_function
        self.side_output_enabled = bool(side_output)
        self._cfg = c
        self._h = ctypes.c_void_p()
        L = N.lib()
        rc = L.fw_list_create(ctypes.byref(c), ctypes.byref(self._h))
        if rc != N.FW_OK:
            msg = L.fw_list_last_error(self._h).decode() if self._h else "fw_list_create failed"
            L.fw_list_destroy(self._h)
            self._h = None
            raise N.NativeError(rc, msg)
        self.epoch = 0
        self._rows, self._elems, self._side, self._outputs = [], [], [], []

    def close(self):
        if getattr(self, "_h", None):
            N.lib().fw_list_destroy(self._h)
            self._h = None

    dispose = close

    def __del__(self):
        self.close()

    def _check(self, rc):
        if rc != N.FW_OK:
            raise N.NativeError(rc, N.lib().fw_list_last_error(self._h).decode())

    # ------------------------------------------------------------------ processElement
    def process_batch(self, keys, timestamps, values, key_hash=None):
        """processElement for every record of the batch, in order; rows fired meanwhile (count triggers, late
        firings) are kept for the next drain."""
        L = N.lib()
        fl = self.value_type in ("double", "float")
        if _is_torch(keys):
            import torch
            n = keys.numel()
            want = torch.float64 if fl else torch.int64
            for t in (keys, timestamps, values) + ((key_hash,) if key_hash is not None else ()):
                if not t.is_cuda or not t.is_contiguous() or t.numel() != n:
                    raise ValueError("device columns must be contiguous CUDA tensors of equal length")
            if keys.dtype != torch.int64 or timestamps.dtype != torch.int64 or values.dtype != want:
                raise ValueError(f"keys / timestamps must be int64 and values {want}")
            torch.cuda.current_stream(keys.device).synchronize()  # the push reads the columns on its own stream
            rc = L.fw_list_push_batch_device(self._h, keys.data_ptr(), timestamps.data_ptr(), values.data_ptr(),
                                             key_hash.data_ptr() if key_hash is not None else None, n)
        else:
            keys = np.ascontiguousarray(keys, dtype=np.int64)
            timestamps = np.ascontiguousarray(timestamps, dtype=np.int64)
            values = np.ascontiguousarray(values, dtype=np.float64 if fl else np.int64)
            kh = None
            if key_hash is not None:
                key_hash = np.ascontiguousarray(key_hash, dtype=np.int32)
                kh = key_hash.ctypes.data
            if not (len(keys) == len(timestamps) == len(values)):
                raise ValueError("columns must have equal length")
            rc = L.fw_list_push_batch(self._h, keys.ctypes.data, timestamps.ctypes.data, values.ctypes.data, kh,
                                      len(keys))
        self._check(rc)

    processElements = process_batch

    # ------------------------------------------------------------------ processWatermark
    def advance_watermark(self, wm):
        n = ctypes.c_int64()
        self._check(N.lib().fw_list_advance_watermark(self._h, int(wm), ctypes.byref(n)))
        self.epoch += 1
        return n.value

    def drain(self, epoch=-1):
        """(rows LIST_ROW_DTYPE, elements ELEM_DTYPE) pending, cleared from HBM; elem_off indexes the elements."""
        L = N.lib()
        nr, ne, ns = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        self._check(L.fw_list_pending(self._h, ctypes.byref(nr), ctypes.byref(ne), ctypes.byref(ns)))
        cols = {f: np.zeros(nr.value, dtype=np.int64) for f in LIST_ROW_FIELDS}
        ecols = {f: np.zeros(ne.value, dtype=np.int64) for f in ("ts", "val", "ordinal")}
        rows = N.FwListRows(**{f: cols[f].ctypes.data for f in LIST_ROW_FIELDS})
        elems = N.FwListElems(**{f: ecols[f].ctypes.data for f in ecols})
        gr, ge = ctypes.c_int64(), ctypes.c_int64()
        self._check(L.fw_list_drain(self._h, ctypes.byref(rows), nr.value, ctypes.byref(elems), ne.value,
                                    ctypes.byref(gr), ctypes.byref(ge)))
        out = np.zeros(gr.value, dtype=LIST_ROW_DTYPE)
        for f in LIST_ROW_FIELDS:
            out[f] = cols[f][:gr.value]
        out["epoch"] = epoch
        el = np.zeros(ge.value, dtype=ELEM_DTYPE)
        for f in ecols:
            el[f] = ecols[f][:ge.value]
        return out, el

    def pending(self):
        """(rows, elements, side rows) pending in HBM"""
        nr, ne, ns = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        self._check(N.lib().fw_list_pending(self._h, ctypes.byref(nr), ctypes.byref(ne), ctypes.byref(ns)))
        return nr.value, ne.value, ns.value

    def clear_pending(self):
        """a discarding sink: the pending rows and elements are dropped in HBM"""
        self._check(N.lib().fw_list_clear_pending(self._h))

    def drain_side(self, epoch=-1):
        L = N.lib()
        ns = ctypes.c_int64()
        self._check(L.fw_list_pending(self._h, None, None, ctypes.byref(ns)))
        k, t, v = (np.zeros(ns.value, dtype=np.int64) for _ in range(3))
        dst = N.FwSideRows(key=k.ctypes.data, ts=t.ctypes.data, val=v.ctypes.data)
        got = ctypes.c_int64()
        self._check(L.fw_list_drain_side(self._h, ctypes.byref(dst), ns.value, ctypes.byref(got)))
        out = np.zeros(got.value, dtype=SIDE_DTYPE)
        out["key"], out["ts"], out["val"], out["epoch"] = k[:got.value], t[:got.value], v[:got.value], epoch
        return out

    def _collect(self, epoch):
        rows, el = self.drain(epoch)
        if len(rows):
            off = sum(len(e) for e in self._elems)
            rows["elem_off"] += off
            self._rows.append(rows)
            self._elems.append(el)
            if self.window_function is not None:
                for r in rows:
                    contents = el[r["elem_off"] - off:r["elem_off"] - off + r["count"]] if self.emit_contents else None
                    self._outputs.append((int(r["epoch"]), self.window_function(int(r["key"]), (int(r["start"]),
                                                                                               int(r["end"])), contents)))
        if self.side_output_enabled:
            self._side.append(self.drain_side(epoch))
        return rows

    def process_watermark(self, wm):
        """processWatermark: the rows fired since the previous watermark (element firings, then this watermark's
        timers)."""
        self.advance_watermark(wm)
        return self._collect(self.epoch - 1)

    processWatermark = process_watermark

    # ------------------------------------------------------------------ harness-style interface
    def process(self, keys, ts, vals, key_hash=None):
        self.process_batch(keys, ts, vals, key_hash)
        self._collect(self.epoch)

    def watermark(self, wm):
        self.process_watermark(wm)

    def rows(self):
        return np.concatenate(self._rows) if self._rows else np.zeros(0, dtype=LIST_ROW_DTYPE)

    def elems(self):
        return np.concatenate(self._elems) if self._elems else np.zeros(0, dtype=ELEM_DTYPE)

    def contents(self):
        """[(row, elements)] of every firing so far, in drain order"""
        e = self.elems()
        return [(r, e[r["elem_off"]:r["elem_off"] + r["count"]]) for r in self.rows()]

    def outputs(self):
        """[(epoch, window_function result)] of every firing so far"""
        return list(self._outputs)

    def side_rows(self):
        return np.concatenate(self._side) if self._side else np.zeros(0, dtype=SIDE_DTYPE)

    # ------------------------------------------------------------------ snapshot / restore per key group
    def snapshot_key_group(self, kg):
        """(lists LIST_STATE_DTYPE, elements ELEM_DTYPE concatenated in list order) of key group kg."""
        L = N.lib()
        nl, ne = ctypes.c_int64(), ctypes.c_int64()
        self._check(L.fw_list_snapshot_key_group(self._h, int(kg), None, 0, 0, ctypes.byref(nl), ctypes.byref(ne)))
        lc = {f: np.zeros(nl.value, dtype=np.int64) for f in LIST_STATE_DTYPE.names}
        ec = {f: np.zeros(ne.value, dtype=np.int64) for f in ("ts", "val", "ordinal")}
        st = N.FwListState(**{f: lc[f].ctypes.data for f in lc}, **{f: ec[f].ctypes.data for f in ec})
        self._check(L.fw_list_snapshot_key_group(self._h, int(kg), ctypes.byref(st), nl.value, ne.value,
                                                 ctypes.byref(nl), ctypes.byref(ne)))
        lists = np.zeros(nl.value, dtype=LIST_STATE_DTYPE)
        for f in lc:
            lists[f] = lc[f]
        el = np.zeros(ne.value, dtype=ELEM_DTYPE)
        for f in ec:
            el[f] = ec[f]
        return lists, el

    def snapshot_state(self):
        return {kg: self.snapshot_key_group(kg) for kg in self.key_group_range}

    def restore_key_group(self, kg, lists, elems):
        lists = np.ascontiguousarray(lists, dtype=LIST_STATE_DTYPE)
        elems = np.ascontiguousarray(elems, dtype=ELEM_DTYPE)
        lc = {f: np.ascontiguousarray(lists[f]) for f in LIST_STATE_DTYPE.names}
        ec = {f: np.ascontiguousarray(elems[f]) for f in ELEM_DTYPE.names}
        st = N.FwListState(**{f: lc[f].ctypes.data for f in lc}, **{f: ec[f].ctypes.data for f in ec})
        self._check(N.lib().fw_list_restore_key_group(self._h, int(kg), ctypes.byref(st), len(lists), len(elems)))

    def initialize_state(self, snapshot):
        for kg, (lists, elems) in snapshot.items():
            if kg in self.key_group_range and len(lists):
                self.restore_key_group(kg, lists, elems)

    snapshotState, initializeState = snapshot_state, initialize_state

    # ------------------------------------------------------------------ metrics
    def stats(self):
        s = N.FwStats()
        self._check(N.lib().fw_list_get_stats(self._h, ctypes.byref(s)))
        return {f: getattr(s, f) for f, _ in N.FwStats._fields_}

    @property
    def late_dropped(self):
        return self.stats()["late_records_dropped"]

    numLateRecordsDropped = late_dropped

    @property
    def num_keyed_state_entries(self):
        return self.stats()["keyed_state_entries"]

    @property
    def num_event_time_timers(self):
        return self.stats()["event_time_timers"]
