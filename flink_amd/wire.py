"""f2: Flink's wire format for one channel <-> device columns (fw_wire_*, include/flink_window.h).

The bytes a channel carries are SpanningRecordSerializer's length-prefixed StreamElements
(flink-runtime/.../io/network/api/serialization/SpanningRecordSerializer.java:76-98;
flink-streaming-java/.../runtime/streamrecord/StreamElementSerializer.java:54-58, 167-221): records with or
without a timestamp, watermarks, latency markers and stream statuses.  WireCodec.decode turns a device byte stream
into the key / timestamp / value columns GpuWindowOperator.process_batch takes (plus the last watermark for
process_watermark), without a per-record JVM step; WireCodec.encode turns fired rows into elements of the
operator's output channel (timestamp = the window's maxTimestamp).

Layouts name the value type's fields: Tuple fields in order (TupleSerializer, no null mask) or one bare field,
each a Java type and a role, e.g. Tuple3<Long, Long, Integer> keyed by field 0 summing field 2:
    WireLayout([("long", "key"), ("long", "skip"), ("int", "value")])
or WindowWordCount's Tuple2<String, Integer> (StringValue.writeString's varint encoding):
    WireLayout([("string", "key"), ("int", "value")])
whose decode also returns the key_hash column (String.hashCode); the key column holds the word's 64-bit id
(keygroups.string_key_id), and the pair goes to a GpuWindowOperator with key_type="hashed".

Key identity of String keys.  The operator keys its state by the 64-bit id (FNV-1a over the UTF-16 units, then
fmix64), not by the string: two distinct strings with the same id would share their windows' state.  Routing stays
exact (key groups come from String.hashCode, carried beside the id).  For k distinct keys the chance of any such
collision is about k^2 / 2^65 (1e6 keys: 3e-8; 1e8 keys: 3e-4).  The host that owns the strings maps each fired
row's id back to its string and can detect a collision there (two strings of one id), so a job whose key space is
large enough for that risk to matter should do so; this library cannot, as it never holds the strings.
"""
import ctypes

from . import _native as N

_KINDS = {"long": N.FW_WIRE_LONG, "int": N.FW_WIRE_INT, "double": N.FW_WIRE_DOUBLE, "short": N.FW_WIRE_SHORT,
          "byte": N.FW_WIRE_BYTE, "float": N.FW_WIRE_FLOAT, "boolean": N.FW_WIRE_BOOL, "string": N.FW_WIRE_STRING}
_ROLES = {"skip": N.FW_ROLE_SKIP, "key": N.FW_ROLE_KEY, "value": N.FW_ROLE_VALUE, "start": N.FW_ROLE_START,
          "end": N.FW_ROLE_END, "count": N.FW_ROLE_COUNT, "sum": N.FW_ROLE_SUM, "min": N.FW_ROLE_MIN,
          "max": N.FW_ROLE_MAX}


class WireLayout:
    def __init__(self, fields):
        if not 1 <= len(fields) <= 8:
            raise ValueError("a layout has 1 to 8 fields")
        self.fields = [(k.lower(), r.lower()) for k, r in fields]
        for k, r in self.fields:
            if k not in _KINDS or r not in _ROLES:
                raise ValueError(f"unknown field kind / role: {k!r} / {r!r}")

    def native(self):
        L = N.FwWireLayout()
        L.nfields = len(self.fields)
        for i, (k, r) in enumerate(self.fields):
            L.kind[i] = _KINDS[k]
            L.role[i] = _ROLES[r]
        return L


class WireCodec:
    def __init__(self, layout: WireLayout, max_bytes, device=0):
        self.layout = layout
        self.device = device
        self._h = ctypes.c_void_p()
        L = N.lib()
        rc = L.fw_wire_create(ctypes.byref(layout.native()), int(max_bytes), device, ctypes.byref(self._h))
        if rc != N.FW_OK:
            msg = L.fw_wire_last_error(self._h).decode() if self._h else "fw_wire_create failed"
            L.fw_wire_destroy(self._h)
            self._h = None
            raise N.NativeError(rc, msg)

    def close(self):
        if getattr(self, "_h", None):
            N.lib().fw_wire_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def _check(self, rc):
        if rc != N.FW_OK:
            raise N.NativeError(rc, N.lib().fw_wire_last_error(self._h).decode())

    def string_key(self):
        return any(k == "string" and r == "key" for k, r in self.layout.fields)

    def decode(self, data, cap=None):
        """data: a CUDA uint8 tensor.  Returns (key, ts, val) int64 CUDA tensors (val holds double bits for Double /
        Float value fields), plus the int32 key_hash column when the key is a String, and the stats dict (records,
        watermarks, latency_markers, statuses, consumed, watermark, status)."""
        import torch
        n = data.numel()
        cap = n // (5 + self.value_bytes()) + 1 if cap is None else cap  # the smallest record element
        dev = data.device
        key, ts, val = (torch.empty(cap, dtype=torch.int64, device=dev) for _ in range(3))
        kh = torch.empty(cap, dtype=torch.int32, device=dev) if self.string_key() else None
        st = N.FwWireStats()
        torch.cuda.current_stream(dev).synchronize()  # the codec's stream reads the bytes
        self._check(N.lib().fw_wire_decode_keyed_device(self._h, data.data_ptr(), n, key.data_ptr(),
                                                        kh.data_ptr() if kh is not None else None, ts.data_ptr(),
                                                        val.data_ptr(), cap, ctypes.byref(st)))
        r = st.records
        cols = (key[:r], ts[:r], val[:r]) + ((kh[:r],) if kh is not None else ())
        return cols, {f: getattr(st, f) for f, _ in N.FwWireStats._fields_ if f != "pad"}

    def value_bytes(self):
        """The value's bytes (a String field counts its shortest form, one byte)."""
        return sum({"long": 8, "double": 8, "int": 4, "float": 4, "short": 2, "byte": 1, "boolean": 1, "string": 1}[k]
                   for k, _ in self.layout.fields)

    def encode(self, rows_view, n, f64=False):
        """rows_view: the device row pointers of GpuWindowOperator.rows_device() (a dict or an FwRows); returns a
        CUDA uint8 tensor of n elements."""
        import torch
        if isinstance(rows_view, dict):
            rows_view = N.FwRows(**{f: rows_view[f] for f in ("key", "start", "end", "count", "sum", "min", "max")})
        size = 13 + self.value_bytes()
        out = torch.empty(max(1, n * size), dtype=torch.uint8, device=torch.device("cuda", self.device))
        written = ctypes.c_int64()
        self._check(N.lib().fw_wire_encode_device(self._h, ctypes.byref(rows_view), n, int(f64), out.data_ptr(),
                                                  out.numel(), ctypes.byref(written)))
        return out[:written.value]
