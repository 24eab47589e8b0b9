"""ctypes binding of include/flink_window.h (libflinkwin.so, built for gfx950 by
flink_amd/csrc/Makefile).  There is no fallback: if the library is missing the import fails."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# FW_LIB selects a diagnostic build variant (tools/variants.sh); the product build is _lib/libflinkwin.so
LIB_PATH = os.environ.get("FW_LIB") or os.path.join(_HERE, "_lib", "libflinkwin.so")
CSRC = os.path.join(_HERE, "csrc")

FW_OK = 0
FW_ERR_ARG = -1
FW_ERR_HIP = -2
FW_ERR_NO_TIMESTAMP = -3
FW_ERR_KEY_GROUP = -4
FW_ERR_CAPACITY = -5
FW_ERR_UNSUPPORTED = -6
FW_ERR_STATE = -7

FW_TUMBLING, FW_SLIDING, FW_SESSION, FW_COUNT = 0, 1, 2, 3
FW_VAL_I64, FW_VAL_I32, FW_VAL_F64, FW_VAL_I16, FW_VAL_I8, FW_VAL_F32 = 0, 1, 2, 3, 4, 5
FW_KEY_LONG, FW_KEY_INT, FW_KEY_HASHED = 0, 1, 2
FW_AGG_COUNT_SUM_MIN_MAX, FW_AGG_HLL, FW_AGG_FIRST, FW_AGG_MINBY, FW_AGG_MAXBY, FW_AGG_FIRST_MAX = 0, 1, 2, 3, 4, 5
FW_AGG_TDIGEST = 6
FW_AGG_ROW = 7
FW_ROW_COUNT_STAR, FW_ROW_COUNT, FW_ROW_SUM, FW_ROW_MIN, FW_ROW_MAX, FW_ROW_AVG = 0, 1, 2, 3, 4, 5
FW_NUM_KERNELS = 7
FW_PROFILE_KINDS = 0x100  # fw_profile(op, FW_PROFILE_KINDS | 1 << kind): time only those kinds

I64P = ctypes.POINTER(ctypes.c_int64)
I32P = ctypes.POINTER(ctypes.c_int32)
VP = ctypes.c_void_p


class FwConfig(ctypes.Structure):
    _fields_ = [("assigner", ctypes.c_int32), ("value_type", ctypes.c_int32), ("key_kind", ctypes.c_int32),
                ("purging", ctypes.c_int32), ("side_output", ctypes.c_int32), ("max_parallelism", ctypes.c_int32),
                ("key_group_start", ctypes.c_int32), ("key_group_end", ctypes.c_int32), ("device", ctypes.c_int32),
                ("sub_partitions", ctypes.c_int32), ("size", ctypes.c_int64), ("slide", ctypes.c_int64),
                ("offset", ctypes.c_int64), ("gap", ctypes.c_int64), ("allowed_lateness", ctypes.c_int64),
                ("expected_entries", ctypes.c_int64), ("max_batch", ctypes.c_int64),
                ("aggregate", ctypes.c_int32), ("hll_precision", ctypes.c_int32),
                ("tdigest_compression", ctypes.c_int32), ("tdigest_export", ctypes.c_int32),
                ("tdigest_quantiles", ctypes.c_double * 3), ("count_evict_after", ctypes.c_int32),
                ("pad0", ctypes.c_int32), ("row_columns", ctypes.c_int32), ("row_aggregates", ctypes.c_int32),
                ("row_column_type", ctypes.c_int32 * 8), ("row_aggregate", ctypes.c_int32 * 16)]


class FwRows(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("key", "start", "end", "count", "sum", "min", "max")]


class FwPartials(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("key", "start", "cnt", "sum", "min", "max")] + [("config", ctypes.c_uint64)]


class FwSideRows(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("key", "ts", "val")]


class FwStateRows(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("key", "start", "end", "count", "sum", "min", "max", "timer")]


class FwStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in (
        "records_in", "late_records_dropped", "keyed_state_entries", "event_time_timers", "current_watermark",
        "fired_rows_total", "pending_rows", "pending_side_rows", "table_capacity", "table_grows",
        "slow_path_records", "state_merges", "digest_centroids_fired", "single_pass_batches",
        "single_pass_redone", "narrow_pass_batches", "narrow_pass_redone", "push_resumptions")]


FW_WIRE_LONG, FW_WIRE_INT, FW_WIRE_DOUBLE, FW_WIRE_SHORT, FW_WIRE_BYTE, FW_WIRE_FLOAT, FW_WIRE_BOOL, FW_WIRE_STRING = range(8)
(FW_ROLE_SKIP, FW_ROLE_KEY, FW_ROLE_VALUE, FW_ROLE_START, FW_ROLE_END, FW_ROLE_COUNT, FW_ROLE_SUM, FW_ROLE_MIN,
 FW_ROLE_MAX) = range(9)


class FwCommStats(ctypes.Structure):
    _fields_ = [("world", ctypes.c_int32), ("rank", ctypes.c_int32)] + [(n, ctypes.c_int64) for n in (
        "batches", "items_sent", "items_received", "bytes_sent", "bytes_received", "recv_reallocs", "recv_capacity")]


class FwExchangePlan(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in ("send_total", "recv_total", "items_sent", "items_received",
                                               "recv_bound")]


class FwWireLayout(ctypes.Structure):
    _fields_ = [("nfields", ctypes.c_int32), ("kind", ctypes.c_int32 * 8), ("role", ctypes.c_int32 * 8)]


class FwWireStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in ("records", "watermarks", "latency_markers", "statuses", "consumed",
                                               "watermark")] + [("status", ctypes.c_int32), ("pad", ctypes.c_int32)]


FW_GLOBAL = 4
FW_TRIGGER_EVENT_TIME, FW_TRIGGER_COUNT = 0, 1
FW_EVICT_NONE, FW_EVICT_COUNT, FW_EVICT_TIME, FW_EVICT_DELTA = 0, 1, 2, 3


class FwListConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "assigner", "value_type", "key_kind", "trigger", "purging", "evictor", "evict_after", "side_output",
        "emit_contents", "max_parallelism", "key_group_start", "key_group_end", "device", "pad0")] + \
        [(n, ctypes.c_int64) for n in ("size", "slide", "offset", "allowed_lateness", "trigger_count",
                                       "evict_count")] + \
        [("delta_threshold", ctypes.c_double), ("expected_elements", ctypes.c_int64), ("max_batch", ctypes.c_int64)]


class FwListRows(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("key", "start", "end", "count", "sum", "min", "max", "first",
                                               "elem_off")]


class FwListElems(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("ts", "val", "ordinal")]


class FwListState(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("key", "start", "end", "trigger_count", "timer", "n_elems", "ts", "val",
                                               "ordinal")]


# every exported symbol with its ctypes signature (restype, argtypes); mirrors include/flink_window.h
SIGNATURES = {
    "fw_create": (ctypes.c_int, [ctypes.POINTER(FwConfig), ctypes.POINTER(VP)]),
    "fw_destroy": (None, [VP]),
    "fw_last_error": (ctypes.c_char_p, [VP]),
    "fw_push_batch": (ctypes.c_int, [VP, VP, VP, VP, VP, ctypes.c_int64]),
    "fw_push_batch_device": (ctypes.c_int, [VP, VP, VP, VP, VP, ctypes.c_int64]),
    "fw_advance_watermark": (ctypes.c_int, [VP, ctypes.c_int64, I64P]),
    "fw_pending": (ctypes.c_int, [VP, I64P, I64P]),
    "fw_drain_rows": (ctypes.c_int, [VP, ctypes.POINTER(FwRows), ctypes.c_int64, I64P]),
    "fw_drain_side": (ctypes.c_int, [VP, ctypes.POINTER(FwSideRows), ctypes.c_int64, I64P]),
    "fw_rows_device": (ctypes.c_int, [VP, ctypes.POINTER(FwRows), I64P]),
    "fw_clear_pending": (ctypes.c_int, [VP]),
    "fw_drain_digests": (ctypes.c_int, [VP, VP, VP, VP, ctypes.c_int64, I64P]),
    "fw_push_row_batch": (ctypes.c_int, [VP, VP, VP, VP, VP, VP, ctypes.c_int64]),
    "fw_push_row_batch_device": (ctypes.c_int, [VP, VP, VP, VP, VP, VP, ctypes.c_int64]),
    "fw_drain_row_results": (ctypes.c_int, [VP, VP, VP, ctypes.c_int64, I64P]),
    "fw_get_stats": (ctypes.c_int, [VP, ctypes.POINTER(FwStats)]),
    "fw_synchronize": (ctypes.c_int, [VP]),
    "fw_profile": (ctypes.c_int, [VP, ctypes.c_int]),
    "fw_profile_read": (ctypes.c_int, [VP, ctypes.POINTER(ctypes.c_double), I64P, ctypes.c_int]),
    "fw_kernel_name": (ctypes.c_char_p, [ctypes.c_int]),
    "fw_stream": (VP, [VP]),
    "fw_set_async_input": (ctypes.c_int, [VP, ctypes.c_int]),
    "fw_input_stream": (VP, [VP]),
    "fw_combine_extract_device": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.POINTER(FwPartials), ctypes.c_int64, I64P,
                                                 I64P]),
    "fw_push_partials_device": (ctypes.c_int, [VP, ctypes.POINTER(FwPartials), ctypes.c_int64]),
    "fw_combine_extract_hll_device": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.POINTER(FwPartials), ctypes.c_int64,
                                                     I64P, I64P, I64P, I64P]),
    "fw_combine_hll_registers_device": (ctypes.c_int, [VP, ctypes.POINTER(FwPartials), ctypes.c_int64, VP,
                                                       ctypes.c_int64]),
    "fw_push_hll_partials_device": (ctypes.c_int, [VP, ctypes.POINTER(FwPartials), ctypes.c_int64, VP, ctypes.c_int64]),
    "fw_keyby_combine_push_device": (ctypes.c_int, [VP, VP, VP, VP, VP, VP, ctypes.c_int64, ctypes.c_int64, I64P]),
    "fw_snapshot_key_group": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.POINTER(FwStateRows), ctypes.c_int64, I64P]),
    "fw_restore_key_group": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.POINTER(FwStateRows), ctypes.c_int64]),
    "fw_state_block_bytes": (ctypes.c_int64, [VP]),
    "fw_snapshot_key_group_blocks": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.POINTER(FwStateRows), VP,
                                                    ctypes.c_int64, I64P]),
    "fw_restore_key_group_blocks": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.POINTER(FwStateRows), VP,
                                                   ctypes.c_int64]),
    "fw_key_groups_device": (ctypes.c_int, [VP, VP, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, VP, VP]),
    "fw_route_device": (ctypes.c_int, [VP, VP, VP, VP, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                                       ctypes.c_int32, VP, VP, VP, VP, VP, VP, ctypes.c_int64, VP]),
    "fw_route_scratch_bytes": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32]),
    "fw_comm_unique_id": (ctypes.c_int, [VP]),
    "fw_comm_init": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(VP)]),
    "fw_comm_destroy": (None, [VP]),
    "fw_keyby_push_device": (ctypes.c_int, [VP, VP, VP, VP, VP, VP, ctypes.c_int64, ctypes.c_int64, I64P]),
    "fw_comm_get_stats": (ctypes.c_int, [VP, ctypes.POINTER(FwCommStats)]),
    "fw_exchange_plan": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, I64P, I64P, I64P,
                                        ctypes.POINTER(FwExchangePlan)]),
    "fw_wire_create": (ctypes.c_int, [ctypes.POINTER(FwWireLayout), ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(VP)]),
    "fw_wire_destroy": (None, [VP]),
    "fw_wire_last_error": (ctypes.c_char_p, [VP]),
    "fw_wire_decode_device": (ctypes.c_int, [VP, VP, ctypes.c_int64, VP, VP, VP, ctypes.c_int64,
                                             ctypes.POINTER(FwWireStats)]),
    "fw_wire_decode_keyed_device": (ctypes.c_int, [VP, VP, ctypes.c_int64, VP, VP, VP, VP, ctypes.c_int64,
                                             ctypes.POINTER(FwWireStats)]),
    "fw_wire_encode_device": (ctypes.c_int, [VP, ctypes.POINTER(FwRows), ctypes.c_int64, ctypes.c_int32, VP,
                                             ctypes.c_int64, I64P]),
    "fw_list_create": (ctypes.c_int, [ctypes.POINTER(FwListConfig), ctypes.POINTER(VP)]),
    "fw_list_destroy": (None, [VP]),
    "fw_list_last_error": (ctypes.c_char_p, [VP]),
    "fw_list_push_batch": (ctypes.c_int, [VP, VP, VP, VP, VP, ctypes.c_int64]),
    "fw_list_push_batch_device": (ctypes.c_int, [VP, VP, VP, VP, VP, ctypes.c_int64]),
    "fw_list_advance_watermark": (ctypes.c_int, [VP, ctypes.c_int64, I64P]),
    "fw_list_pending": (ctypes.c_int, [VP, I64P, I64P, I64P]),
    "fw_list_drain": (ctypes.c_int, [VP, ctypes.POINTER(FwListRows), ctypes.c_int64, ctypes.POINTER(FwListElems),
                                     ctypes.c_int64, I64P, I64P]),
    "fw_list_clear_pending": (ctypes.c_int, [VP]),
    "fw_list_drain_side": (ctypes.c_int, [VP, ctypes.POINTER(FwSideRows), ctypes.c_int64, I64P]),
    "fw_list_get_stats": (ctypes.c_int, [VP, ctypes.POINTER(FwStats)]),
    "fw_list_snapshot_key_group": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.POINTER(FwListState), ctypes.c_int64,
                                                  ctypes.c_int64, I64P, I64P]),
    "fw_list_restore_key_group": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.POINTER(FwListState), ctypes.c_int64,
                                                 ctypes.c_int64]),
    "fw_generate_device": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, VP,
                                          ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, VP, VP, VP, VP, VP]),
}

_lib = None


class NativeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def lib():
    """Load libflinkwin.so.  Raises if it was not built — the GPU path has no CPU fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make -C {CSRC}` "
                              "(or __graft_entry__.build()); flink_amd has no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, handle=None):
    if rc != FW_OK:
        msg = lib().fw_last_error(handle).decode() if handle else "error"
        raise NativeError(rc, msg)
    return rc
