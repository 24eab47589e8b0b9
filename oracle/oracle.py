"""ctypes wrapper over oracle/_build/liboracle.so — the CPU restatement of Flink's WindowOperator.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, never by the product package flink_amd/.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

TUMBLING, SLIDING, SESSION = 0, 1, 2
VAL_I64, VAL_I32, VAL_F64, VAL_I16, VAL_I8, VAL_F32 = 0, 1, 2, 3, 4, 5
_ASSIGNERS = {"tumbling": TUMBLING, "sliding": SLIDING, "session": SESSION}
_VALTYPES = {"i64": VAL_I64, "i32": VAL_I32, "f64": VAL_F64, "i16": VAL_I16, "i8": VAL_I8, "f32": VAL_F32}


class OracleCfg(ctypes.Structure):
    _fields_ = [("assigner", ctypes.c_int32), ("value_type", ctypes.c_int32), ("size", ctypes.c_int64),
                ("slide", ctypes.c_int64), ("offset", ctypes.c_int64), ("gap", ctypes.c_int64),
                ("lateness", ctypes.c_int64), ("purging", ctypes.c_int32), ("side_output", ctypes.c_int32),
                ("aggregate", ctypes.c_int32), ("hll_p", ctypes.c_int32), ("td_delta", ctypes.c_int32),
                ("td_pad", ctypes.c_int32), ("td_q", ctypes.c_double * 3), ("row_nc", ctypes.c_int32),
                ("row_ns", ctypes.c_int32), ("row_type", ctypes.c_int32 * 8), ("row_spec", ctypes.c_int32 * 16)]


ROW_DTYPE = np.dtype([("key", "<i8"), ("start", "<i8"), ("end", "<i8"), ("count", "<i8"), ("sum", "<i8"),
                      ("min", "<i8"), ("max", "<i8"), ("epoch", "<i8")])
SIDE_DTYPE = np.dtype([("key", "<i8"), ("ts", "<i8"), ("val", "<i8"), ("epoch", "<i8")])

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        I64P = ctypes.POINTER(ctypes.c_int64)
        I32P = ctypes.POINTER(ctypes.c_int32)
        L.oracle_create.restype = P
        L.oracle_create.argtypes = [ctypes.POINTER(OracleCfg)]
        L.oracle_destroy.argtypes = [P]
        L.oracle_process.argtypes = [P, I64P, I64P, I64P, ctypes.c_int64]
        L.oracle_watermark.argtypes = [P, ctypes.c_int64]
        for f in ("oracle_num_rows", "oracle_num_side_rows", "oracle_late_dropped", "oracle_num_state_entries",
                  "oracle_num_timers", "oracle_current_watermark"):
            getattr(L, f).restype = ctypes.c_int64
            getattr(L, f).argtypes = [P]
        L.oracle_get_rows.argtypes = [P, P]
        L.oracle_get_side_rows.argtypes = [P, P]
        L.oracle_clear_rows.argtypes = [P]
        L.oracle_long_hash.restype = ctypes.c_int32
        L.oracle_long_hash.argtypes = [ctypes.c_int64]
        L.oracle_murmur_hash.restype = ctypes.c_int32
        L.oracle_murmur_hash.argtypes = [ctypes.c_int32]
        L.oracle_key_group.restype = ctypes.c_int32
        L.oracle_key_group.argtypes = [ctypes.c_int32, ctypes.c_int32]
        L.oracle_operator_index.restype = ctypes.c_int32
        L.oracle_operator_index.argtypes = [ctypes.c_int32] * 3
        L.oracle_key_group_range.argtypes = [ctypes.c_int32] * 3 + [I32P, I32P]
        L.oracle_key_groups_long.argtypes = [I64P, ctypes.c_int64, ctypes.c_int32, I32P]
        L.oracle_window_start.restype = ctypes.c_int64
        L.oracle_window_start.argtypes = [ctypes.c_int64] * 3
        L.oracle_string_hash.restype = ctypes.c_int32
        L.oracle_string_hash.argtypes = [ctypes.c_char_p, ctypes.c_int64]
        L.oracle_run_parallel.restype = ctypes.c_int64
        L.oracle_run_parallel.argtypes = [ctypes.POINTER(OracleCfg), I64P, I64P, I64P, ctypes.c_int64, ctypes.c_int64,
                                          I64P, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, I64P]
        L.oracle_count_create.restype = P
        L.oracle_count_create.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]
        L.oracle_count_destroy.argtypes = [P]
        L.oracle_count_process.argtypes = [P, I64P, I64P, ctypes.c_int64]
        L.oracle_count_num_rows.restype = ctypes.c_int64
        L.oracle_count_num_rows.argtypes = [P]
        L.oracle_count_get_rows.argtypes = [P, P]
        L.oracle_row_digest.restype = ctypes.c_int64
        L.oracle_row_digest.argtypes = [P, ctypes.c_int64, P, P, ctypes.c_int64]
        L.oracle_process_rows.argtypes = [P, I64P, I64P, I64P, P, ctypes.c_int64]
        L.oracle_row_results.restype = ctypes.c_int32
        L.oracle_row_results.argtypes = [P, ctypes.c_int64, I64P, ctypes.POINTER(ctypes.c_uint32)]
        _lib = L
    return _lib


def _i64p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


AGG_COUNT_SUM_MIN_MAX, AGG_HLL, AGG_FIRST, AGG_MINBY, AGG_MAXBY, AGG_FIRST_MAX, AGG_TDIGEST, AGG_ROW = range(8)
ROW_FNS = {"count_star": 0, "count": 1, "sum": 2, "min": 3, "max": 4, "avg": 5}


def make_cfg(assigner="tumbling", size=0, slide=0, offset=0, gap=0, lateness=0, purging=False, side_output=False,
             value_type="i64", hll_p=0, first=False, by=None, tdigest=0, quantiles=(0.5, 0.95, 0.99), row=None):
    """hll_p > 0 selects the HyperLogLog AggregateFunction with 2^hll_p registers; first=True the
    first-element reduce of sum(pos)/min(pos) (max = arrival ordinal of the window's first element;
    window_oracle.h); tdigest = delta > 0 the t-digest of an f64 value column with rows carrying
    `quantiles`."""
    agg = (AGG_HLL if hll_p else AGG_TDIGEST if tdigest else AGG_FIRST_MAX if first == "max" else AGG_FIRST if first
           else {"min": AGG_MINBY, "max": AGG_MAXBY}[by] if by else AGG_COUNT_SUM_MIN_MAX)
    if tdigest:
        value_type = "f64"
    c = OracleCfg(_ASSIGNERS[assigner], _VALTYPES[value_type], size, slide, offset, gap, lateness, int(purging),
                  int(side_output), agg, int(hll_p), int(tdigest), 0, (ctypes.c_double * 3)(*quantiles))
    if row is not None:  # OR_AGG_ROW: row = (column types, [(fn, column), ...]) (window_oracle.h)
        types, specs = row
        c.aggregate = AGG_ROW
        c.row_nc, c.row_ns = len(types), len(specs)
        for j, t in enumerate(types):
            c.row_type[j] = _VALTYPES[t]
        for q, (fn, col) in enumerate(specs):
            c.row_spec[q] = (ROW_FNS[fn] << 8) | col
    return c


class OracleError(RuntimeError):
    def __init__(self, code):
        super().__init__(f"oracle error {code}")
        self.code = code


class WindowOperatorOracle:
    """Element-by-element WindowOperator restatement (see window_oracle.h)."""

    def __init__(self, **cfg):
        self.cfg = make_cfg(**cfg)
        self._h = lib().oracle_create(ctypes.byref(self.cfg))

    def close(self):
        if self._h:
            lib().oracle_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def process(self, keys, ts, vals):
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        vals = np.ascontiguousarray(vals)
        if vals.dtype == np.float64:
            vals = vals.view(np.int64)
        vals = np.ascontiguousarray(vals, dtype=np.int64)
        rc = lib().oracle_process(self._h, _i64p(keys), _i64p(ts), _i64p(vals), len(keys))
        if rc != 0:
            raise OracleError(rc)

    def watermark(self, wm):
        rc = lib().oracle_watermark(self._h, int(wm))
        if rc != 0:
            raise OracleError(rc)

    def rows(self):
        n = lib().oracle_num_rows(self._h)
        out = np.zeros(n, dtype=ROW_DTYPE)
        if n:
            lib().oracle_get_rows(self._h, out.ctypes.data)
        return out

    def clear_rows(self):
        lib().oracle_clear_rows(self._h)

    def process_rows(self, keys, ts, cols, nulls=None):
        """OR_AGG_ROW: cols = [column j values] (i64, or f64 viewed as bits), nulls = uint8 mask per record."""
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        mat = np.ascontiguousarray(np.stack([np.asarray(c).view(np.int64) if np.asarray(c).dtype == np.float64
                                             else np.asarray(c, dtype=np.int64) for c in cols]))
        nm = None if nulls is None else np.ascontiguousarray(nulls, dtype=np.uint8)
        rc = lib().oracle_process_rows(self._h, _i64p(keys), _i64p(ts), _i64p(mat),
                                       None if nm is None else nm.ctypes.data, len(keys))
        if rc != 0:
            raise OracleError(rc)

    def row_results(self):
        """OR_AGG_ROW: (values int64[rows, nspec], null mask uint32[rows]) of every emitted row, in row order."""
        n, ns = lib().oracle_num_rows(self._h), self.cfg.row_ns
        vals = np.zeros((n, ns), dtype=np.int64)
        nm = np.zeros(n, dtype=np.uint32)
        for r in range(n):
            m = ctypes.c_uint32()
            lib().oracle_row_results(self._h, r, vals[r].ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), ctypes.byref(m))
            nm[r] = m.value
        return vals, nm

    def digest(self, row):
        """t-digest centroids (sum f64[], weight i64[]) of emitted row `row`."""
        n = lib().oracle_row_digest(self._h, row, None, None, 0)
        s, w = np.zeros(max(n, 0)), np.zeros(max(n, 0), dtype=np.int64)
        if n > 0:
            lib().oracle_row_digest(self._h, row, s.ctypes.data, w.ctypes.data, n)
        return s, w

    def side_rows(self):
        n = lib().oracle_num_side_rows(self._h)
        out = np.zeros(n, dtype=SIDE_DTYPE)
        if n:
            lib().oracle_get_side_rows(self._h, out.ctypes.data)
        return out

    @property
    def late_dropped(self):
        return lib().oracle_late_dropped(self._h)

    @property
    def num_state_entries(self):
        return lib().oracle_num_state_entries(self._h)

    @property
    def num_timers(self):
        return lib().oracle_num_timers(self._h)


class CountWindowOracle:
    """a14: countWindow(size, slide).sum(pos) — GlobalWindows + CountTrigger + CountEvictor (evict before the
    window function, or after it with evict_after=True); see window_oracle.h.  Rows have max = the arrival
    ordinal of the first reduced element (flink_amd.windowing.first_element_results rebuilds the tuples)."""

    def __init__(self, size, slide, evict_after=False, value_type="i32"):
        self._h = lib().oracle_count_create(size, slide, int(evict_after), _VALTYPES[value_type])
        if not self._h:
            raise ValueError("count window size and slide must be positive")

    def close(self):
        if self._h:
            lib().oracle_count_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def process(self, keys, vals):
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        vals = np.ascontiguousarray(vals, dtype=np.int64)
        lib().oracle_count_process(self._h, _i64p(keys), _i64p(vals), len(keys))

    def rows(self):
        n = lib().oracle_count_num_rows(self._h)
        out = np.zeros(n, dtype=ROW_DTYPE)
        if n:
            lib().oracle_count_get_rows(self._h, out.ctypes.data)
        return out


# ---- f4: window-contents (ListState) operators (list_oracle.h) -----------------------------------------
LIST_TRIGGERS = {"event_time": 0, "count": 1}
LIST_EVICTORS = {"none": 0, "count": 1, "time": 2, "delta": 3}
_LIST_ASSIGNERS = {"tumbling": TUMBLING, "sliding": SLIDING, "global": 3, "session": SESSION}


class OracleListCfg(ctypes.Structure):
    _fields_ = [("assigner", ctypes.c_int32), ("value_type", ctypes.c_int32), ("size", ctypes.c_int64),
                ("slide", ctypes.c_int64), ("offset", ctypes.c_int64), ("lateness", ctypes.c_int64),
                ("trigger", ctypes.c_int32), ("purging", ctypes.c_int32), ("trigger_count", ctypes.c_int64),
                ("evictor", ctypes.c_int32), ("evict_after", ctypes.c_int32), ("evict_count", ctypes.c_int64),
                ("delta_threshold", ctypes.c_double), ("side_output", ctypes.c_int32), ("pad", ctypes.c_int32)]


LIST_ROW_DTYPE = np.dtype([("key", "<i8"), ("start", "<i8"), ("end", "<i8"), ("count", "<i8"), ("sum", "<i8"),
                           ("min", "<i8"), ("max", "<i8"), ("first", "<i8"), ("elem_off", "<i8"), ("epoch", "<i8")])
LIST_ELEM_DTYPE = np.dtype([("ts", "<i8"), ("val", "<i8"), ("ord", "<i8")])


def _list_lib():
    L = lib()
    if not getattr(L, "_list_ready", False):
        P = ctypes.c_void_p
        I64P = ctypes.POINTER(ctypes.c_int64)
        L.oracle_list_create.restype = P
        L.oracle_list_create.argtypes = [ctypes.POINTER(OracleListCfg)]
        L.oracle_list_destroy.argtypes = [P]
        L.oracle_list_process.argtypes = [P, I64P, I64P, I64P, ctypes.c_int64]
        L.oracle_list_watermark.argtypes = [P, ctypes.c_int64]
        for f in ("oracle_list_num_rows", "oracle_list_num_elems", "oracle_list_num_side_rows",
                  "oracle_list_late_dropped", "oracle_list_num_state_entries", "oracle_list_num_timers"):
            getattr(L, f).restype = ctypes.c_int64
            getattr(L, f).argtypes = [P]
        L.oracle_list_get_rows.argtypes = [P, P]
        L.oracle_list_get_elems.argtypes = [P, P]
        L.oracle_list_get_side_rows.argtypes = [P, I64P, I64P, I64P, I64P]
        L._list_ready = True
    return L


def make_list_cfg(assigner="tumbling", size=0, slide=0, offset=0, lateness=0, trigger="event_time", trigger_count=0,
                  purging=False, evictor="none", evict_after=False, evict_arg=0, threshold=0.0, side_output=False,
                  value_type="i64", gap=0):
    if assigner == "session":  # (list_oracle.h: the gap travels in `size`)
        size = gap
    return OracleListCfg(_LIST_ASSIGNERS[assigner], _VALTYPES[value_type], size, slide, offset, lateness,
                         LIST_TRIGGERS[trigger], int(purging), trigger_count, LIST_EVICTORS[evictor], int(evict_after),
                         evict_arg, float(threshold), int(side_output), 0)


class ListWindowOracle:
    """EvictingWindowOperator / WindowOperator over ListState with an Iterable window function (list_oracle.h):
    rows (key, window, count, sum, min, max, first ordinal, offset of the contents, epoch) and the contents of
    every firing."""

    def __init__(self, **cfg):
        self.cfg = make_list_cfg(**cfg)
        self._h = _list_lib().oracle_list_create(ctypes.byref(self.cfg))
        if not self._h:
            raise ValueError("invalid list window configuration")

    def close(self):
        if self._h:
            _list_lib().oracle_list_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def process(self, keys, ts, vals):
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        vals = np.ascontiguousarray(vals)
        if vals.dtype == np.float64:
            vals = vals.view(np.int64)
        vals = np.ascontiguousarray(vals, dtype=np.int64)
        rc = _list_lib().oracle_list_process(self._h, _i64p(keys), _i64p(ts), _i64p(vals), len(keys))
        if rc != 0:
            raise OracleError(rc)

    def watermark(self, wm):
        _list_lib().oracle_list_watermark(self._h, int(wm))

    def rows(self):
        n = _list_lib().oracle_list_num_rows(self._h)
        out = np.zeros(n, dtype=LIST_ROW_DTYPE)
        if n:
            _list_lib().oracle_list_get_rows(self._h, out.ctypes.data)
        return out

    def elems(self):
        n = _list_lib().oracle_list_num_elems(self._h)
        out = np.zeros(n, dtype=LIST_ELEM_DTYPE)
        if n:
            _list_lib().oracle_list_get_elems(self._h, out.ctypes.data)
        return out

    def contents(self):
        """[(row, elements)] in emission order"""
        r, e = self.rows(), self.elems()
        return [(x, e[x["elem_off"]:x["elem_off"] + x["count"]]) for x in r]

    def side_rows(self):
        n = _list_lib().oracle_list_num_side_rows(self._h)
        cols = [np.zeros(n, dtype=np.int64) for _ in range(4)]
        if n:
            _list_lib().oracle_list_get_side_rows(self._h, *[_i64p(c) for c in cols])
        return cols

    @property
    def late_dropped(self):
        return _list_lib().oracle_list_late_dropped(self._h)

    @property
    def num_state_entries(self):
        return _list_lib().oracle_list_num_state_entries(self._h)

    @property
    def num_timers(self):
        return _list_lib().oracle_list_num_timers(self._h)


def key_groups_long(keys, max_par):
    keys = np.ascontiguousarray(keys, dtype=np.int64)
    out = np.zeros(len(keys), dtype=np.int32)
    lib().oracle_key_groups_long(_i64p(keys), len(keys), max_par, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return out


def run_parallel(cfg, keys, ts, vals, batch, wms, max_par, threads):
    c = make_cfg(**cfg)
    late = np.zeros(1, dtype=np.int64)
    wms = np.ascontiguousarray(wms, dtype=np.int64)
    keys = np.ascontiguousarray(keys, dtype=np.int64)
    ts = np.ascontiguousarray(ts, dtype=np.int64)
    vals = np.ascontiguousarray(vals)
    if vals.dtype == np.float64:
        vals = vals.view(np.int64)
    rows = lib().oracle_run_parallel(ctypes.byref(c), _i64p(keys), _i64p(ts), _i64p(vals), len(keys), batch,
                                     _i64p(wms), len(wms), max_par, threads, _i64p(late))
    return rows, int(late[0])


# ---- f2: the wire format (wire_oracle.h) -------------------------------------------------------------
WIRE_KINDS = {"long": 0, "int": 1, "double": 2, "short": 3, "byte": 4, "float": 5, "boolean": 6, "string": 7}
WIRE_ROLES = {"skip": 0, "key": 1, "value": 2, "start": 3, "end": 4, "count": 5, "sum": 6, "min": 7, "max": 8}


class OracleWireLayout(ctypes.Structure):
    _fields_ = [("nfields", ctypes.c_int32), ("kind", ctypes.c_int32 * 8), ("role", ctypes.c_int32 * 8)]


class OracleWireStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in ("records", "watermarks", "latency_markers", "statuses", "consumed",
                                               "watermark")] + [("status", ctypes.c_int32), ("bad_tag", ctypes.c_int32)]


_wire_ready = False


def _wire_lib():
    global _wire_ready
    L = lib()
    if not _wire_ready:
        P, U8 = ctypes.c_void_p, ctypes.c_void_p
        L.oracle_wire_decode.restype = ctypes.c_int
        L.oracle_wire_decode.argtypes = [U8, ctypes.c_int64, ctypes.POINTER(OracleWireLayout), P, P, P, ctypes.c_int64,
                                         ctypes.POINTER(OracleWireStats)]
        L.oracle_wire_decode_keyed.restype = ctypes.c_int
        L.oracle_wire_decode_keyed.argtypes = [U8, ctypes.c_int64, ctypes.POINTER(OracleWireLayout), P, P, P, P,
                                               ctypes.c_int64, ctypes.POINTER(OracleWireStats)]
        L.oracle_string_key_id.restype = ctypes.c_int64
        L.oracle_string_key_id.argtypes = [P, ctypes.c_int64]
        L.oracle_wire_encode.restype = ctypes.c_int64
        L.oracle_wire_encode.argtypes = [ctypes.POINTER(OracleWireLayout), P, ctypes.c_int64, ctypes.c_int32, U8,
                                         ctypes.c_int64]
        L.oracle_wire_put_record.restype = ctypes.c_int64
        L.oracle_wire_put_record.argtypes = [ctypes.POINTER(OracleWireLayout), ctypes.c_int32, ctypes.c_int64, P, U8]
        L.oracle_wire_put_watermark.restype = ctypes.c_int64
        L.oracle_wire_put_watermark.argtypes = [ctypes.c_int64, U8]
        L.oracle_wire_put_status.restype = ctypes.c_int64
        L.oracle_wire_put_status.argtypes = [ctypes.c_int32, U8]
        L.oracle_wire_put_latency.restype = ctypes.c_int64
        L.oracle_wire_put_latency.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, U8]
        _wire_ready = True
    return L


def wire_layout(fields):
    L = OracleWireLayout()
    L.nfields = len(fields)
    for i, (k, r) in enumerate(fields):
        L.kind[i] = WIRE_KINDS[k]
        L.role[i] = WIRE_ROLES[r]
    return L


class WireStream:
    """Builds a channel's bytes element by element (the reference serializers' output)."""

    def __init__(self, fields):
        self.fields = fields
        self._L = wire_layout(fields)
        self._parts = []

    def record(self, values, ts=None):
        buf = (ctypes.c_uint8 * 64)()
        v = np.ascontiguousarray(values, dtype=np.int64)
        n = _wire_lib().oracle_wire_put_record(ctypes.byref(self._L), int(ts is not None), 0 if ts is None else int(ts),
                                               v.ctypes.data, ctypes.addressof(buf))
        self._parts.append(bytes(buf[:n]))

    def record_str(self, values, ts=None):
        """A record whose layout may hold String fields (values: str or None for those, ints otherwise), written
        here in Python: StreamElementSerializer's tag / timestamp, TupleSerializer's fields in order, a String
        through StringValue.writeString (StringValue.java:789-817)."""
        import struct
        body = bytearray()
        for (kind, _), x in zip(self.fields, values):
            if kind == "string":
                body += write_string(x)
            else:
                fmt = {"long": ">q", "double": ">q", "int": ">i", "float": ">I", "short": ">h", "byte": ">b",
                       "boolean": ">B"}[kind]
                if kind == "float":  # the value is double bits: Float.floatToIntBits((float) d)
                    d = struct.unpack("<d", struct.pack("<q", int(x)))[0]
                    x = struct.unpack(">I", struct.pack(">f", d))[0]
                body += struct.pack(fmt, int(x))
        head = struct.pack(">Bq", 0, int(ts)) if ts is not None else struct.pack(">B", 1)
        self._parts.append(struct.pack(">I", len(head) + len(body)) + head + bytes(body))

    def watermark(self, wm):
        buf = (ctypes.c_uint8 * 16)()
        n = _wire_lib().oracle_wire_put_watermark(int(wm), ctypes.addressof(buf))
        self._parts.append(bytes(buf[:n]))

    def status(self, s):
        buf = (ctypes.c_uint8 * 16)()
        n = _wire_lib().oracle_wire_put_status(int(s), ctypes.addressof(buf))
        self._parts.append(bytes(buf[:n]))

    def latency(self, marked, lo, hi, subtask):
        buf = (ctypes.c_uint8 * 40)()
        n = _wire_lib().oracle_wire_put_latency(int(marked), int(lo), int(hi), int(subtask), ctypes.addressof(buf))
        self._parts.append(bytes(buf[:n]))

    def raw(self, b):
        self._parts.append(bytes(b))

    def bytes(self):
        return b"".join(self._parts)


def wire_decode(data, fields, cap=None):
    """-> (key, ts, val) int64 arrays, stats dict, rc (0 ok, -1 corrupt, -2 capacity)."""
    b = np.frombuffer(bytes(data), dtype=np.uint8)
    cap = len(b) // 10 + 1 if cap is None else cap
    key, ts, val = (np.zeros(max(1, cap), dtype=np.int64) for _ in range(3))
    st = OracleWireStats()
    L = wire_layout(fields)
    rc = _wire_lib().oracle_wire_decode(b.ctypes.data if len(b) else None, len(b), ctypes.byref(L), key.ctypes.data,
                                        ts.ctypes.data, val.ctypes.data, cap, ctypes.byref(st))
    r = st.records
    return (key[:r], ts[:r], val[:r]), {f: getattr(st, f) for f, _ in OracleWireStats._fields_}, rc


def write_string(s):
    """StringValue.writeString (StringValue.java:789-817): length + 1 as a base-128 varint (low group first, 0 for
    null), then every UTF-16 char as a base-128 varint."""
    out = bytearray()
    if s is None:
        return bytes([0])
    enc = s.encode("utf-16-le")
    units = [int.from_bytes(enc[i:i + 2], "little") for i in range(0, len(enc), 2)]
    n = len(units) + 1
    while n >= 0x80:
        out.append((n | 0x80) & 0xff)
        n >>= 7
    out.append(n)
    for c in units:
        while c >= 0x80:
            out.append((c | 0x80) & 0xff)
            c >>= 7
        out.append(c)
    return bytes(out)


def string_key_id(s):
    """The key column's identity of a String key (oracle_string_key_id)."""
    u = np.frombuffer(s.encode("utf-16-le"), dtype=np.uint16).copy()
    return int(_wire_lib().oracle_string_key_id(u.ctypes.data if len(u) else None, len(u)))


def wire_decode_keyed(data, fields, cap=None):
    """-> (key, key_hash, ts, val) arrays, stats dict, rc (0 ok, -1 corrupt, -2 capacity)."""
    b = np.frombuffer(bytes(data), dtype=np.uint8)
    cap = len(b) // 6 + 1 if cap is None else cap
    key, ts, val = (np.zeros(max(1, cap), dtype=np.int64) for _ in range(3))
    kh = np.zeros(max(1, cap), dtype=np.int32)
    st = OracleWireStats()
    L = wire_layout(fields)
    rc = _wire_lib().oracle_wire_decode_keyed(b.ctypes.data if len(b) else None, len(b), ctypes.byref(L),
                                              key.ctypes.data, kh.ctypes.data, ts.ctypes.data, val.ctypes.data, cap,
                                              ctypes.byref(st))
    r = st.records
    return (key[:r], kh[:r], ts[:r], val[:r]), {f: getattr(st, f) for f, _ in OracleWireStats._fields_}, rc


def wire_encode(rows, fields, f64=False):
    rows = np.ascontiguousarray(rows, dtype=ROW_DTYPE)
    L = wire_layout(fields)
    size = 13 + sum({"long": 8, "double": 8, "int": 4, "float": 4, "short": 2, "byte": 1, "boolean": 1}[k]
                    for k, _ in fields)
    out = np.zeros(max(1, len(rows) * size), dtype=np.uint8)
    n = _wire_lib().oracle_wire_encode(ctypes.byref(L), rows.ctypes.data, len(rows), int(f64), out.ctypes.data,
                                       len(out))
    assert n >= 0
    return out[:n].tobytes()
