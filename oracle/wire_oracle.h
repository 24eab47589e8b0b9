/* wire_oracle.h — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py's cpu_baseline may use it; the product
 * path never does).  A sequential CPU restatement of Flink's wire format for one input channel, the checker of
 * fw_wire_decode_device / fw_wire_encode_device (include/flink_window.h, f2).
 *
 *   SpanningRecordSerializer.addRecord (flink-runtime/src/main/java/org/apache/flink/runtime/io/network/api/
 *     serialization/SpanningRecordSerializer.java:76-98): a 4-byte big-endian length, then the element's bytes.
 *   StreamElementSerializer.serialize / deserialize (flink-streaming-java/src/main/java/org/apache/flink/
 *     streaming/runtime/streamrecord/StreamElementSerializer.java:54-58, 167-221): tag 0 = record with
 *     timestamp (BE i64), 1 = record without, 2 = watermark (BE i64), 3 = latency marker (BE i64 marked time,
 *     BE i64 lower / upper operator id, BE i32 subtask index), 4 = stream status (BE i32); otherwise
 *     IOException("Corrupt stream, found tag: " + tag).
 *   TupleSerializer.serialize (flink-java/src/main/java/org/apache/flink/api/java/typeutils/runtime/
 *     TupleSerializer.java): the fields in order, no null mask; LongSerializer / IntSerializer / ShortSerializer
 *     / ByteSerializer / BooleanSerializer / DoubleSerializer / FloatSerializer (flink-core/.../common/typeutils/
 *     base/{Long,Int,...}Serializer.java): DataOutputView's big-endian writeLong / writeInt / writeShort / writeByte /
 *     writeBoolean, writeDouble = writeLong(Double.doubleToLongBits), writeFloat = writeInt(floatToIntBits).
 *   StringSerializer -> StringValue.writeString / readString (flink-core/src/main/java/org/apache/flink/types/
 *     StringValue.java:745-830): length + 1 as a little-endian base-128 varint (0 = null), then each UTF-16 char
 *     as a base-128 varint (chars < 0x80 one byte); readString keeps the low 16 bits of a decoded char.  A String
 *     key's hash is String.hashCode (31 h + c over the chars, int wrap) and its identity in the key column is the
 *     build's 64-bit id of the chars (string_key_id below, also flink_amd/keygroups.py); a null key is an error
 *     (KeySelector.getKey of a null field fails in KeyGroupStreamPartitioner).
 *   StreamRecord.getTimestamp of a record without timestamp = Long.MIN_VALUE (StreamRecord.java:91-100).
 *   WindowOperator.emitWindowContents: the row's timestamp is the window's maxTimestamp = end - 1.
 * Pinned by the big-endian TimeWindow / timer longs inside the reference's own win-op-migration snapshot
 * (tests/golden/wire_fixture.json) and by round trips. */
#pragma once
#include <stdint.h>
#include "window_oracle.h"

#ifdef __cplusplus
extern "C" {
#endif
enum { OR_WIRE_LONG = 0, OR_WIRE_INT = 1, OR_WIRE_DOUBLE = 2, OR_WIRE_SHORT = 3, OR_WIRE_BYTE = 4, OR_WIRE_FLOAT = 5,
       OR_WIRE_BOOL = 6, OR_WIRE_STRING = 7 };
enum { OR_ROLE_SKIP = 0, OR_ROLE_KEY = 1, OR_ROLE_VALUE = 2, OR_ROLE_START = 3, OR_ROLE_END = 4, OR_ROLE_COUNT = 5,
       OR_ROLE_SUM = 6, OR_ROLE_MIN = 7, OR_ROLE_MAX = 8 };
typedef struct {
  int32_t nfields;
  int32_t kind[8];
  int32_t role[8];
} oracle_wire_layout;
typedef struct {
  int64_t records, watermarks, latency_markers, statuses;
  int64_t consumed;
  int64_t watermark;
  int32_t status;
  int32_t bad_tag;  /* the corrupt tag (or -2 for an element that does not fit the layout, -4 for a null String
                       key), when decode returns -1 */
} oracle_wire_stats;
/* 0 = ok, -1 = corrupt stream (stats->bad_tag), -2 = more records than cap, -3 = a String key without key_hash */
int oracle_wire_decode(const uint8_t* bytes, int64_t n, const oracle_wire_layout* layout, int64_t* key, int64_t* ts,
                       int64_t* val, int64_t cap, oracle_wire_stats* stats);
/* the same with the key's hash column (String.hashCode of a String key, else 0); key_hash may be NULL unless the
 * key field is a String */
int oracle_wire_decode_keyed(const uint8_t* bytes, int64_t n, const oracle_wire_layout* layout, int64_t* key,
                             int32_t* key_hash, int64_t* ts, int64_t* val, int64_t cap, oracle_wire_stats* stats);
/* the key column's identity of a String key: FNV-1a 64 over the UTF-16 chars, then fmix64 of it ^ the length */
int64_t oracle_string_key_id(const uint16_t* chars, int64_t n);
/* rows -> elements (tag 0, ts = end - 1, the fields the roles name); returns the bytes written, -1 if cap is short */
int64_t oracle_wire_encode(const oracle_wire_layout* layout, const oracle_row* rows, int64_t n, int32_t f64,
                           uint8_t* out, int64_t cap);
/* helpers for building test streams: one element of each kind; return the bytes written */
int64_t oracle_wire_put_record(const oracle_wire_layout* layout, int32_t with_ts, int64_t ts, const int64_t* fields,
                               uint8_t* out);
int64_t oracle_wire_put_watermark(int64_t wm, uint8_t* out);
int64_t oracle_wire_put_status(int32_t status, uint8_t* out);
int64_t oracle_wire_put_latency(int64_t marked, int64_t id_lo, int64_t id_hi, int32_t subtask, uint8_t* out);
#ifdef __cplusplus
}
#endif
