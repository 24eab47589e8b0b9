"""GpuWindowOperator: the drop-in for WindowOperator + heap keyed state backend + event-time timer
service on one MI355X.  Mirrors the reference operator's interface in batch form:

  WindowOperator(windowAssigner, ..., stateDesc, windowFunction, trigger, allowedLateness, lateDataOutputTag)
      (flink-streaming-java/.../runtime/operators/windowing/WindowOperator.java:179-212)
  processElement(StreamRecord)   -> process_batch(keys, timestamps, values)    (:291-421)
  processWatermark(Watermark)    -> process_watermark(wm) -> fired rows         (AbstractStreamOperator.java:735-740)
  numLateRecordsDropped, numKeyedStateEntries, numEventTimeTimers               (WindowOperator.java:138-140;
                                                                                 KeyedOneInputStreamOperatorTestHarness:71-81)

Inputs are either numpy arrays (host; copied to HBM by the library) or torch tensors already on the
GPU (consumed in place).  Every call goes through libflinkwin.so; there is no CPU implementation.
"""
import ctypes

import numpy as np

from . import _native as N
from .keygroups import KeyGroupRange
from .windowing import CountSumMinMax, EventTimeTrigger, Trigger, WindowAssigner

ROW_FIELDS = ("key", "start", "end", "count", "sum", "min", "max")
ROW_DTYPE = np.dtype([(f, "<i8") for f in ROW_FIELDS] + [("epoch", "<i8")])
STATE_FIELDS = ("key", "start", "end", "count", "sum", "min", "max", "timer")
STATE_DTYPE = np.dtype([(f, "<i8") for f in STATE_FIELDS])
SIDE_DTYPE = np.dtype([("key", "<i8"), ("ts", "<i8"), ("val", "<i8"), ("epoch", "<i8")])

_KEY_KINDS = {"long": N.FW_KEY_LONG, "int": N.FW_KEY_INT, "hashed": N.FW_KEY_HASHED}


def _is_torch(x):
    return type(x).__module__.startswith("torch")


class Partials(tuple):
    """The six partial-accumulator columns (key, start, cnt, sum, min, max) of one combine_extract, with `config`,
    the producing combiner's configuration tag that push_partials hands back to fw_push_partials_device."""
    config = 0


class GpuWindowOperator:
    def __init__(self, assigner: WindowAssigner, aggregate=CountSumMinMax(), trigger: Trigger = None,
                 allowed_lateness=0, side_output=False, key_type="long", max_parallelism=128,
                 key_group_range: KeyGroupRange = None, device=0, expected_entries=0, max_batch=0,
                 sub_partitions=0, async_input=True):
        trigger = trigger or EventTimeTrigger.create()
        if not isinstance(getattr(trigger, "nested", trigger), EventTimeTrigger):
            raise ValueError("GpuWindowOperator takes EventTimeTrigger or PurgingTrigger.of(EventTimeTrigger); "
                             "count triggers run on GpuListWindowOperator")
        if allowed_lateness < 0:
            raise ValueError("The allowed lateness cannot be negative.")
        kgr = key_group_range or KeyGroupRange(0, max_parallelism - 1)
        c = N.FwConfig()
        for k, v in assigner.config().items():
            setattr(c, k, v)
        c.value_type = aggregate.native()
        c.hll_precision = aggregate.hll_precision()
        td = aggregate.tdigest()
        if td is not None:
            c.tdigest_compression = td.compression
            c.tdigest_export = int(td.export)
            c.tdigest_quantiles = (ctypes.c_double * 3)(*td.quantiles)
        c.aggregate = aggregate.aggregate_kind()
        if c.aggregate == N.FW_AGG_ROW:  # the Table API's group-window accumulator (RowAggregate)
            c.row_columns = len(aggregate.column_types)
            c.row_aggregates = len(aggregate.aggregates)
            for j, t in enumerate(aggregate.type_codes()[:8]):
                c.row_column_type[j] = t
            for q, w in enumerate(aggregate.spec_words()[:16]):
                c.row_aggregate[q] = w
        c.key_kind = _KEY_KINDS[key_type]
        c.purging = int(trigger.purging)
        c.side_output = int(side_output)
        c.max_parallelism = max_parallelism
        c.key_group_start = kgr.start_key_group
        c.key_group_end = kgr.end_key_group
        c.device = device
        c.sub_partitions = sub_partitions
        c.allowed_lateness = allowed_lateness
        c.expected_entries = expected_entries
        c.max_batch = max_batch
        self.assigner, self.aggregate, self.trigger = assigner, aggregate, trigger
        self.allowed_lateness = allowed_lateness
        self.side_output_enabled = bool(side_output)
        self.key_group_range = kgr
        self.max_parallelism = max_parallelism
        self.device = device
        self._cfg = c
        self._h = ctypes.c_void_p()
        L = N.lib()
        rc = L.fw_create(ctypes.byref(c), ctypes.byref(self._h))
        if rc != N.FW_OK:
            msg = L.fw_last_error(self._h).decode() if self._h else "fw_create failed"
            L.fw_destroy(self._h)
            self._h = None
            raise N.NativeError(rc, msg)
        if async_input:  # device batches are partitioned beside the previous batch's aggregation (fw_set_async_input)
            N.check(L.fw_set_async_input(self._h, 1), self._h)
        self._inflight = None  # device columns of a push the library may still be reading
        self.epoch = 0  # watermarks processed so far
        self._rows = []
        self._side = []
        self._rowres = []

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "_h", None):
            N.lib().fw_destroy(self._h)  # waits for the stream
            self._h = None
        self._inflight = None

    dispose = close

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def stream(self):
        return N.lib().fw_stream(self._h)

    def _torch_stream(self, device):
        """The library's HIP stream as a torch stream object (for stream-ordered handoffs)."""
        s = getattr(self, "_tstream", None)
        if s is None:
            import torch
            s = self._tstream = torch.cuda.ExternalStream(self.stream, device=device)
        return s

    def set_async_input(self, enable=True):
        """fw_set_async_input: a device batch's partitioning kernels run on the library's input stream, beside
        the previous batch's aggregation (the columns' producer is ordered before that stream by process_batch)."""
        N.check(N.lib().fw_set_async_input(self._h, 1 if enable else 0), self._h)
        self._istream = None

    def _input_stream(self, device):
        """The stream fw_push_batch_device reads its columns on (fw_input_stream), as a torch stream object."""
        s = getattr(self, "_istream", None)
        if s is None:
            import torch
            s = self._istream = torch.cuda.ExternalStream(N.lib().fw_input_stream(self._h), device=device)
        return s

    # ------------------------------------------------------------------ processElement
    def process_batch(self, keys, timestamps, values, key_hash=None):
        """Hands a micro-batch (all records between two watermarks, or a part of them) to the GPU."""
        L = N.lib()
        if _is_torch(keys):
            import torch
            n = keys.numel()
            for t in (keys, timestamps, values) + ((key_hash,) if key_hash is not None else ()):
                if not t.is_cuda or not t.is_contiguous() or t.numel() != n:
                    raise ValueError("device columns must be contiguous CUDA tensors of equal length")
            if keys.dtype != torch.int64 or timestamps.dtype != torch.int64:
                raise ValueError("keys and timestamps must be int64")
            # fw_push_batch_device reads 8 bytes per value: a narrower column would be read out of bounds,
            # and a float64 / int64 mix would be reinterpreted as bits
            want = torch.float64 if self.aggregate.value_type in ("double", "float") else torch.int64
            if values.dtype != want:
                raise ValueError(f"values must be {want} for a {self.aggregate.value_type!r} aggregate, got {values.dtype}")
            if key_hash is not None and key_hash.dtype != torch.int32:
                raise ValueError("key_hash must be int32 (Java hashCode)")
            # stream-ordered handoff: the library's input stream waits for the producer's writes.  The push
            # is asynchronous; the columns are referenced until the next push has settled it.
            self._input_stream(keys.device).wait_stream(torch.cuda.current_stream(keys.device))
            rc = L.fw_push_batch_device(self._h, keys.data_ptr(), timestamps.data_ptr(), values.data_ptr(),
                                        key_hash.data_ptr() if key_hash is not None else None, n)
            self._inflight = (keys, timestamps, values, key_hash)
        else:
            keys = np.ascontiguousarray(keys, dtype=np.int64)
            timestamps = np.ascontiguousarray(timestamps, dtype=np.int64)
            values = np.asarray(values)
            values = np.ascontiguousarray(values, dtype=np.float64 if self.aggregate.value_type in ("double", "float")
                                          else np.int64)
            kh = None
            if key_hash is not None:
                key_hash = np.ascontiguousarray(key_hash, dtype=np.int32)
                kh = key_hash.ctypes.data
            n = len(keys)
            if len(timestamps) != n or len(values) != n:
                raise ValueError("columns must have equal length")
            rc = L.fw_push_batch(self._h, keys.ctypes.data, timestamps.ctypes.data, values.ctypes.data, kh, n)
        N.check(rc, self._h)

    processElements = process_batch

    def process_rows(self, keys, timestamps, cols, nulls=None, key_hash=None):
        """RowAggregate: a micro-batch of the Table API's input rows -- keys, timestamps, the value columns (a
        sequence of columns, or one [columns, n] array / tensor; int64 values, or float64 for "double" / "float"
        columns) and an optional NULL mask per record (uint8, bit j = column j is NULL)."""
        L = N.lib()
        nc = len(self.aggregate.column_types)
        if _is_torch(keys):
            import torch
            n = keys.numel()
            mat = cols if _is_torch(cols) else torch.stack([c.view(torch.int64) if c.dtype == torch.float64 else c
                                                            for c in cols])
            if mat.dtype == torch.float64:
                mat = mat.view(torch.int64)
            mat = mat.contiguous()
            if mat.shape != (nc, n) or mat.dtype != torch.int64 or not mat.is_cuda:
                raise ValueError(f"cols must be {nc} int64 / float64 CUDA columns of {n} values")
            if nulls is not None and (nulls.dtype != torch.uint8 or nulls.numel() != n or not nulls.is_cuda):
                raise ValueError("nulls must be a uint8 CUDA tensor, one mask per record")
            for t in (keys, timestamps) + ((key_hash,) if key_hash is not None else ()):
                if not t.is_cuda or not t.is_contiguous() or t.numel() != n:
                    raise ValueError("device columns must be contiguous CUDA tensors of equal length")
            self._input_stream(keys.device).wait_stream(torch.cuda.current_stream(keys.device))
            rc = L.fw_push_row_batch_device(self._h, keys.data_ptr(), timestamps.data_ptr(), mat.data_ptr(),
                                            nulls.data_ptr() if nulls is not None else None,
                                            key_hash.data_ptr() if key_hash is not None else None, n)
            self._inflight = (keys, timestamps, mat, nulls, key_hash)
        else:
            keys = np.ascontiguousarray(keys, dtype=np.int64)
            timestamps = np.ascontiguousarray(timestamps, dtype=np.int64)
            n = len(keys)
            mat = np.ascontiguousarray(np.stack([np.asarray(c).view(np.int64) if np.asarray(c).dtype == np.float64
                                                 else np.asarray(c, dtype=np.int64) for c in cols])
                                       if not isinstance(cols, np.ndarray) or cols.ndim != 2 else cols.view(np.int64)
                                       if cols.dtype == np.float64 else cols.astype(np.int64))
            if mat.shape != (nc, n) or len(timestamps) != n:
                raise ValueError(f"cols must be {nc} columns of {n} values")
            nm = None
            if nulls is not None:
                nulls = np.ascontiguousarray(nulls, dtype=np.uint8)
                nm = nulls.ctypes.data
            kh = None
            if key_hash is not None:
                key_hash = np.ascontiguousarray(key_hash, dtype=np.int32)
                kh = key_hash.ctypes.data
            rc = L.fw_push_row_batch(self._h, keys.ctypes.data, timestamps.ctypes.data, mat.ctypes.data, nm, kh, n)
        N.check(rc, self._h)

    def drain_row_results(self):
        """RowAggregate: the pending rows' aggregate values (int64 [rows, aggregates]: integers, or f64 bits for
        floating results) and NULL masks (uint32 [rows]), in row order.  Call before the rows are drained."""
        L = N.lib()
        n_rows = ctypes.c_int64()
        N.check(L.fw_pending(self._h, ctypes.byref(n_rows), None), self._h)
        n, ns = n_rows.value, len(self.aggregate.aggregates)
        vals = np.zeros((n, ns), dtype=np.int64)
        nm = np.zeros(n, dtype=np.uint32)
        got = ctypes.c_int64()
        N.check(L.fw_drain_row_results(self._h, vals.ctypes.data, nm.ctypes.data, n, ctypes.byref(got)), self._h)
        return vals[:got.value], nm[:got.value]

    # ------------------------------------------------------------------ pre-shuffle combining
    def combine_extract(self, world=1):
        """fw_combine_extract_device on this handle used as a combiner: drains its state into partial accumulators
        (six int64 device columns key, start, cnt, sum, min, max in key-group order) and returns them with the
        number of partials for each of `world` destination subtasks.  The columns are views of buffers the
        handle reuses: consume them before the next call."""
        import torch
        L = N.lib()
        dev = torch.device("cuda", self.device)
        counts = (ctypes.c_int64 * world)()
        n = ctypes.c_int64()
        while True:
            bufs = getattr(self, "_pbuf", None)
            cap = bufs[0].numel() if bufs else 0
            out = N.FwPartials(*(t.data_ptr() for t in bufs)) if bufs else N.FwPartials()
            rc = L.fw_combine_extract_device(self._h, world, ctypes.byref(out), cap, counts, ctypes.byref(n))
            if rc == N.FW_ERR_CAPACITY and n.value > cap:
                cap = max(n.value, 2 * cap)
                self._pbuf = [torch.empty(cap, dtype=torch.int64, device=dev) for _ in range(6)]
                continue
            N.check(rc, self._h)
            break
        if n.value == 0:
            cols = Partials(torch.empty(0, dtype=torch.int64, device=dev) for _ in range(6))
        else:
            cols = Partials(t[:n.value] for t in self._pbuf)
        cols.config = out.config
        return cols, list(counts)

    def combine_extract_hll(self, world=1):
        """HyperLogLog combining (fw_combine_extract_hll_device + fw_combine_hll_registers_device): drains this
        combiner into partial rows (six int64 columns; a row's sum = how many non-zero registers it carries) in
        key-group order and their registers (uint32 index << 8 | rank, in row order).  Returns (cols, counts,
        regs, reg_counts): per destination subtask its rows and its registers, each one contiguous slice.  The
        columns are views of buffers the handle reuses: consume them before the next call."""
        import torch
        L = N.lib()
        dev = torch.device("cuda", self.device)
        counts = (ctypes.c_int64 * world)()
        rcounts = (ctypes.c_int64 * world)()
        n, nr = ctypes.c_int64(), ctypes.c_int64()
        while True:
            bufs = getattr(self, "_pbuf", None)
            cap = bufs[0].numel() if bufs else 0
            out = N.FwPartials(*(t.data_ptr() for t in bufs)) if bufs else N.FwPartials()
            rc = L.fw_combine_extract_hll_device(self._h, world, ctypes.byref(out), cap, counts, rcounts,
                                                 ctypes.byref(n), ctypes.byref(nr))
            if rc == N.FW_ERR_CAPACITY and n.value > cap:
                self._pbuf = [torch.empty(max(n.value, 2 * cap), dtype=torch.int64, device=dev) for _ in range(6)]
                continue
            N.check(rc, self._h)
            break
        rb = getattr(self, "_rbuf", None)
        if rb is None or rb.numel() < max(nr.value, 1):
            self._rbuf = rb = torch.empty(max(nr.value, 2 * (rb.numel() if rb is not None else 0), 1),
                                          dtype=torch.int32, device=dev)
        N.check(L.fw_combine_hll_registers_device(self._h, ctypes.byref(out), n.value, rb.data_ptr(), rb.numel()),
                self._h)
        cols = Partials((t[:n.value] for t in self._pbuf) if n.value else
                        (torch.empty(0, dtype=torch.int64, device=dev) for _ in range(6)))
        cols.config = out.config
        return cols, list(counts), rb[:nr.value], list(rcounts)

    def push_hll_partials(self, key, start, cnt, sum_, min_, max_, regs, config):
        """fw_push_hll_partials_device: merges HyperLogLog partial rows (from combine_extract_hll of a combiner with
        this operator's configuration) and raises their registers (`regs`: the rows' register lists in row order,
        int32 / uint32 bits)."""
        import torch
        cols = (key, start, cnt, sum_, min_, max_)
        n = key.numel()
        for t in cols:
            if not t.is_cuda or not t.is_contiguous() or t.numel() != n or t.dtype != torch.int64:
                raise ValueError("partials must be contiguous int64 CUDA tensors of equal length")
        if not regs.is_cuda or not regs.is_contiguous() or regs.dtype != torch.int32:
            raise ValueError("registers must be a contiguous int32 CUDA tensor")
        if n == 0:
            return
        self._torch_stream(key.device).wait_stream(torch.cuda.current_stream(key.device))
        p = N.FwPartials(*(t.data_ptr() for t in cols), config)
        N.check(N.lib().fw_push_hll_partials_device(self._h, ctypes.byref(p), n, regs.data_ptr() if regs.numel() else None,
                                                    regs.numel()), self._h)
        self._inflight = cols + (regs,)

    def push_partials(self, key, start, cnt, sum_, min_, max_, config):
        """fw_push_partials_device: merges partial accumulators (from combine_extract of a combiner with the same
        configuration; `config` = that extraction's Partials.config tag, checked against this handle's own) of this
        subtask's KeyGroupRange; late ones are dropped and counted with their records."""
        import torch
        cols = (key, start, cnt, sum_, min_, max_)
        n = key.numel()
        for t in cols:
            if not t.is_cuda or not t.is_contiguous() or t.numel() != n or t.dtype != torch.int64:
                raise ValueError("partials must be contiguous int64 CUDA tensors of equal length")
        if n == 0:
            return
        self._torch_stream(key.device).wait_stream(torch.cuda.current_stream(key.device))
        p = N.FwPartials(*(t.data_ptr() for t in cols), config)
        N.check(N.lib().fw_push_partials_device(self._h, ctypes.byref(p), n), self._h)
        self._inflight = cols

    # ------------------------------------------------------------------ processWatermark
    def advance_watermark(self, wm, wait=True):
        """Fires due windows; returns the number of rows pending in HBM (not copied).  With
        wait=False the firing is only queued and None is returned (errors surface at the next call)."""
        if not wait:
            N.check(N.lib().fw_advance_watermark(self._h, int(wm), None), self._h)
            self.epoch += 1
            return None
        n = ctypes.c_int64()
        N.check(N.lib().fw_advance_watermark(self._h, int(wm), ctypes.byref(n)), self._h)
        self._inflight = None
        self.epoch += 1
        return n.value

    def process_watermark(self, wm):
        """processWatermark: returns every row emitted since the previous watermark (late firings
        during process_batch, then the timer firings of this watermark) as a structured array."""
        self.advance_watermark(wm)
        rows = self.drain_rows(self.epoch - 1)
        if self.side_output_enabled:
            self._side.append(self.drain_side(self.epoch - 1))
        return rows

    processWatermark = process_watermark

    def drain_rows(self, epoch=-1):
        L = N.lib()
        n_rows = ctypes.c_int64()
        N.check(L.fw_pending(self._h, ctypes.byref(n_rows), None), self._h)
        out = np.zeros(n_rows.value, dtype=ROW_DTYPE)
        cols = {f: np.zeros(n_rows.value, dtype=np.int64) for f in ROW_FIELDS}
        dst = N.FwRows(**{f: cols[f].ctypes.data for f in ROW_FIELDS})
        got = ctypes.c_int64()
        N.check(L.fw_drain_rows(self._h, ctypes.byref(dst), n_rows.value, ctypes.byref(got)), self._h)
        for f in ROW_FIELDS:
            out[f] = cols[f][:got.value]
        out["epoch"] = epoch
        return out

    def drain_rows_torch(self, fields=ROW_FIELDS):
        """fw_drain_rows into fresh int64 tensors on this operator's GPU (HBM to HBM, no host copy): {field: tensor}
        for the requested row fields; the pending rows are cleared."""
        import torch
        L = N.lib()
        n_rows = ctypes.c_int64()
        N.check(L.fw_pending(self._h, ctypes.byref(n_rows), None), self._h)
        dev = torch.device("cuda", self.device)
        cols = {f: torch.empty(max(n_rows.value, 1), dtype=torch.int64, device=dev) for f in fields}
        # the output blocks come from torch's allocator on the current stream, and the library writes them on its
        # own stream: it must not start before the current stream's pending work on a recycled block is done
        self._torch_stream(dev).wait_stream(torch.cuda.current_stream(dev))
        dst = N.FwRows(**{f: cols[f].data_ptr() for f in fields})
        got = ctypes.c_int64()
        N.check(L.fw_drain_rows(self._h, ctypes.byref(dst), n_rows.value, ctypes.byref(got)), self._h)
        # and the current stream's readers of the rows come after the library's copies (fw_drain_rows also waits)
        torch.cuda.current_stream(dev).wait_stream(self._torch_stream(dev))
        return {f: t[:got.value] for f, t in cols.items()}

    def drain_digests(self):
        """TDigest(export=True): the centroids of the pending rows, as a list of (sums f64[], weights i64[])
        in row order.  Call before the rows are drained (process_watermark drains them: use
        advance_watermark, then drain_digests, then drain_rows)."""
        L = N.lib()
        n_rows = ctypes.c_int64()
        N.check(L.fw_pending(self._h, ctypes.byref(n_rows), None), self._h)
        nb = self.aggregate.compression // 2
        n = n_rows.value
        cnt = np.zeros(n, dtype=np.int64)
        sums = np.zeros(n * nb, dtype=np.float64)
        ws = np.zeros(n * nb, dtype=np.int64)
        got = ctypes.c_int64()
        N.check(L.fw_drain_digests(self._h, cnt.ctypes.data, sums.ctypes.data, ws.ctypes.data, n,
                                   ctypes.byref(got)), self._h)
        return [(sums[i * nb:i * nb + cnt[i]].copy(), ws[i * nb:i * nb + cnt[i]].copy()) for i in range(got.value)]

    def drain_side(self, epoch=-1):
        L = N.lib()
        n_side = ctypes.c_int64()
        N.check(L.fw_pending(self._h, None, ctypes.byref(n_side)), self._h)
        k, t, v = (np.zeros(n_side.value, dtype=np.int64) for _ in range(3))
        dst = N.FwSideRows(key=k.ctypes.data, ts=t.ctypes.data, val=v.ctypes.data)
        got = ctypes.c_int64()
        N.check(L.fw_drain_side(self._h, ctypes.byref(dst), n_side.value, ctypes.byref(got)), self._h)
        out = np.zeros(got.value, dtype=SIDE_DTYPE)
        out["key"], out["ts"], out["val"], out["epoch"] = k[:got.value], t[:got.value], v[:got.value], epoch
        return out

    def rows_device(self):
        """Device view of the pending rows: (dict of column -> raw device pointer, n)."""
        view = N.FwRows()
        n = ctypes.c_int64()
        N.check(N.lib().fw_rows_device(self._h, ctypes.byref(view), ctypes.byref(n)), self._h)
        return {f: getattr(view, f) for f in ROW_FIELDS}, n.value

    def clear_pending(self):
        N.check(N.lib().fw_clear_pending(self._h), self._h)

    def synchronize(self):
        N.check(N.lib().fw_synchronize(self._h), self._h)
        self._inflight = None

    # ------------------------------------------------------------------ harness-style interface
    # (the shape of OneInputStreamOperatorTestHarness used by tests/kat_util.replay)
    def process(self, keys, ts, vals, key_hash=None):
        # processElement raises at once in the reference: wait for the batch and surface its errors
        self.process_batch(keys, ts, vals, key_hash)
        self.synchronize()
        if self.assigner.kind == N.FW_COUNT:  # count windows fire while the elements are processed
            self._rows.append(self.drain_rows(self.epoch))

    def watermark(self, wm):
        if self.aggregate.aggregate_kind() == N.FW_AGG_ROW:  # the rows' aggregate values before the rows go
            self.advance_watermark(wm)
            self._rowres.append(self.drain_row_results())
            self._rows.append(self.drain_rows(self.epoch - 1))
            return
        self._rows.append(self.process_watermark(wm))

    def process_row_batch(self, keys, ts, cols, nulls=None, key_hash=None):
        """Harness form of process_rows: the batch is processed (and its errors raised) before return."""
        self.process_rows(keys, ts, cols, nulls, key_hash)
        self.synchronize()

    def rows(self):
        return np.concatenate(self._rows) if self._rows else np.zeros(0, dtype=ROW_DTYPE)

    def row_results(self):
        """RowAggregate, harness form: (values, NULL masks) of every row rows() returns, in the same order."""
        ns = len(self.aggregate.aggregates)
        if not self._rowres:
            return np.zeros((0, ns), dtype=np.int64), np.zeros(0, dtype=np.uint32)
        return np.concatenate([v for v, _ in self._rowres]), np.concatenate([m for _, m in self._rowres])

    def side_rows(self):
        return np.concatenate(self._side) if self._side else np.zeros(0, dtype=SIDE_DTYPE)

    # ------------------------------------------------------------------ snapshot / restore
    # AbstractStreamOperator.snapshotState writes keyed state per key group
    # (HeapKeyedStateBackend.java:289-399, per-key-group offsets :370-381; timers via
    # InternalTimeServiceManager.snapshotStateForKeyGroup :114); a restore may hand the key groups
    # to operators with a different KeyGroupRange (rescaling).
    def state_dtype(self):
        """Row type of this operator's snapshots: STATE_DTYPE, plus `acc` (the accumulator block, fw_state_block_bytes
        bytes: HyperLogLog registers / the t-digest's centroids) for the HyperLogLog and t-digest aggregates."""
        bb = N.lib().fw_state_block_bytes(self._h)
        return STATE_DTYPE if bb == 0 else np.dtype(STATE_DTYPE.descr + [("acc", "u1", (bb,))])

    def snapshot_key_group(self, kg):
        """Live (key, window) accumulators of key group kg as a state_dtype() array (no order)."""
        L = N.lib()
        bb = L.fw_state_block_bytes(self._h)
        n = ctypes.c_int64()
        N.check(L.fw_snapshot_key_group_blocks(self._h, int(kg), None, None, 0, ctypes.byref(n)), self._h)
        cols = {f: np.zeros(n.value, dtype=np.int64) for f in STATE_FIELDS}
        acc = np.zeros((n.value, max(bb, 1)), dtype=np.uint8)
        dst = N.FwStateRows(**{f: cols[f].ctypes.data for f in STATE_FIELDS})
        got = ctypes.c_int64()
        N.check(L.fw_snapshot_key_group_blocks(self._h, int(kg), ctypes.byref(dst), acc.ctypes.data if bb else None,
                                               n.value, ctypes.byref(got)), self._h)
        out = np.zeros(got.value, dtype=self.state_dtype())
        for f in STATE_FIELDS:
            out[f] = cols[f][:got.value]
        if bb:
            out["acc"] = acc[:got.value]
        return out

    def snapshot_state(self):
        """{key group: state_dtype() rows} for every key group of this operator's KeyGroupRange."""
        return {kg: self.snapshot_key_group(kg) for kg in self.key_group_range}

    def restore_key_group(self, kg, rows):
        L = N.lib()
        bb = L.fw_state_block_bytes(self._h)
        rows = np.ascontiguousarray(rows)
        if bb and (rows.dtype.names is None or "acc" not in rows.dtype.names or rows.dtype["acc"].shape != (bb,)):
            raise ValueError(f"rows of this aggregate carry `acc` blocks of {bb} bytes (state_dtype())")
        cols = {f: np.ascontiguousarray(rows[f], dtype=np.int64) for f in STATE_FIELDS}
        acc = np.ascontiguousarray(rows["acc"], dtype=np.uint8) if bb else None
        src = N.FwStateRows(**{f: cols[f].ctypes.data for f in STATE_FIELDS})
        N.check(L.fw_restore_key_group_blocks(self._h, int(kg), ctypes.byref(src),
                                              acc.ctypes.data if bb and len(rows) else None, len(rows)), self._h)

    def initialize_state(self, snapshot):
        """Restores the key groups of `snapshot` ({kg: rows}) that this operator owns; others are skipped,
        as a subtask reads only the key groups of its own KeyGroupRange."""
        for kg, rows in snapshot.items():
            if kg in self.key_group_range and len(rows):
                self.restore_key_group(kg, rows)

    snapshotState, initializeState = snapshot_state, initialize_state

    # ------------------------------------------------------------------ metrics
    def stats(self):
        s = N.FwStats()
        N.check(N.lib().fw_get_stats(self._h, ctypes.byref(s)), self._h)
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
