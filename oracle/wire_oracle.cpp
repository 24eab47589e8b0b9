// wire_oracle.cpp — TEST INFRASTRUCTURE ONLY: see wire_oracle.h (Flink wire format, sequential restatement).
#include "wire_oracle.h"

#include <cstring>

namespace {

int field_bytes(int32_t kind) {
  switch (kind) {
    case OR_WIRE_LONG:
    case OR_WIRE_DOUBLE: return 8;
    case OR_WIRE_INT:
    case OR_WIRE_FLOAT: return 4;
    case OR_WIRE_SHORT: return 2;
    case OR_WIRE_BYTE:
    case OR_WIRE_BOOL: return 1;
  }
  return -1;
}
int value_bytes(const oracle_wire_layout* L) {  // (fixed-size fields only)
  int f = 0;
  for (int i = 0; i < L->nfields; i++) f += field_bytes(L->kind[i]);
  return f;
}
bool has_string(const oracle_wire_layout* L) {
  for (int i = 0; i < L->nfields; i++)
    if (L->kind[i] == OR_WIRE_STRING) return true;
  return false;
}
uint64_t fmix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}
// StringValue.readString (StringValue.java:745-786): one base-128 varint, low group first; -1 past `end`
int64_t read_varint(const uint8_t* p, const uint8_t* end, uint32_t* out) {
  const uint8_t* q = p;
  if (q >= end) return -1;
  uint32_t v = *q++;
  if (v >= 0x80) {
    int shift = 7;
    uint32_t curr;
    v &= 0x7f;
    for (;;) {
      if (q >= end) return -1;
      curr = *q++;
      if (curr < 0x80) break;
      v |= (curr & 0x7f) << shift;
      shift += 7;
    }
    v |= curr << shift;
  }
  *out = v;
  return q - p;
}
// a String field at p: its bytes (-1 if it runs past end); *is_null, and for a non-null one its hashCode and id
int64_t read_string(const uint8_t* p, const uint8_t* end, bool* is_null, int32_t* hash, int64_t* id) {
  uint32_t len;
  int64_t at = read_varint(p, end, &len);
  if (at < 0) return -1;
  *is_null = len == 0;
  if (len == 0) return at;
  len -= 1;
  uint32_t h = 0;
  uint64_t f = 0xcbf29ce484222325ull;
  for (uint32_t i = 0; i < len; i++) {
    uint32_t c;
    const int64_t k = read_varint(p + at, end, &c);
    if (k < 0) return -1;
    at += k;
    const uint16_t ch = (uint16_t)c;  // (char) c
    h = 31u * h + ch;                 // String.hashCode
    f = (f ^ ch) * 0x100000001b3ull;
  }
  *hash = (int32_t)h;
  *id = (int64_t)fmix64(f ^ (uint64_t)len);
  return at;
}
// DataInputView.readLong / readInt / readShort: big-endian
uint64_t get_be(const uint8_t* p, int nb) {
  uint64_t v = 0;
  for (int i = 0; i < nb; i++) v = (v << 8) | p[i];
  return v;
}
void put_be(uint8_t* p, uint64_t v, int nb) {
  for (int i = nb - 1; i >= 0; i--) {
    p[i] = (uint8_t)(v & 0xff);
    v >>= 8;
  }
}
// a field read back as the operator's 64-bit column value: integers sign-extended (Boolean 0 / 1), Double as its
// bits, Float widened to double (Float.intBitsToFloat, then the float's exact double)
int64_t field_value(int32_t kind, const uint8_t* p) {
  switch (kind) {
    case OR_WIRE_LONG:
    case OR_WIRE_DOUBLE: return (int64_t)get_be(p, 8);
    case OR_WIRE_INT: return (int64_t)(int32_t)(uint32_t)get_be(p, 4);
    case OR_WIRE_SHORT: return (int64_t)(int16_t)(uint16_t)get_be(p, 2);
    case OR_WIRE_BYTE: return (int64_t)(int8_t)p[0];
    case OR_WIRE_BOOL: return p[0] != 0;
    case OR_WIRE_FLOAT: {
      const uint32_t b = (uint32_t)get_be(p, 4);
      float f;
      std::memcpy(&f, &b, 4);
      const double d = (double)f;
      int64_t r;
      std::memcpy(&r, &d, 8);
      return r;
    }
  }
  return 0;
}
void put_field(int32_t kind, uint8_t* p, int64_t v) {
  switch (kind) {
    case OR_WIRE_LONG:
    case OR_WIRE_DOUBLE: put_be(p, (uint64_t)v, 8); break;
    case OR_WIRE_INT: put_be(p, (uint32_t)v, 4); break;
    case OR_WIRE_SHORT: put_be(p, (uint16_t)v, 2); break;
    case OR_WIRE_BYTE:
    case OR_WIRE_BOOL: p[0] = (uint8_t)v; break;
    case OR_WIRE_FLOAT: {  // the value is double bits: Float.floatToIntBits((float) d)
      double d;
      std::memcpy(&d, &v, 8);
      const float f = (float)d;
      uint32_t b;
      std::memcpy(&b, &f, 4);
      put_be(p, b, 4);
      break;
    }
  }
}

}  // namespace

extern "C" {

int oracle_wire_decode(const uint8_t* b, int64_t n, const oracle_wire_layout* L, int64_t* key, int64_t* ts,
                       int64_t* val, int64_t cap, oracle_wire_stats* st) {
  return oracle_wire_decode_keyed(b, n, L, key, nullptr, ts, val, cap, st);
}

int64_t oracle_string_key_id(const uint16_t* chars, int64_t n) {
  uint64_t f = 0xcbf29ce484222325ull;
  for (int64_t i = 0; i < n; i++) f = (f ^ chars[i]) * 0x100000001b3ull;
  return (int64_t)fmix64(f ^ (uint64_t)n);
}

int oracle_wire_decode_keyed(const uint8_t* b, int64_t n, const oracle_wire_layout* L, int64_t* key, int32_t* kh,
                             int64_t* ts, int64_t* val, int64_t cap, oracle_wire_stats* st) {
  std::memset(st, 0, sizeof *st);
  st->watermark = INT64_MIN;
  st->status = 0;  // StreamStatus.ACTIVE when the stream carried none
  for (int i = 0; i < L->nfields; i++)
    if (L->kind[i] == OR_WIRE_STRING && L->role[i] == OR_ROLE_KEY && !kh) return -3;
  const int F = value_bytes(L);
  const bool strings = has_string(L);
  int64_t pos = 0;
  while (pos + 4 <= n) {
    const int64_t len = (int64_t)get_be(b + pos, 4);
    if (pos + 4 + len > n) break;  // a partial element: the next call's
    const uint8_t* e = b + pos + 4;
    const int tag = len > 0 ? (int8_t)e[0] : -3;  // readByte
    int64_t want = tag == 0 ? 9 + F : tag == 1 ? 1 + F : tag == 2 ? 9 : tag == 3 ? 29 : tag == 4 ? 5 : -1;
    if (want < 0) {
      st->bad_tag = tag;
      st->consumed = pos;
      return -1;
    }
    int64_t k = 0, v = 0;
    int32_t h = 0;
    bool null_key = false;
    if (tag <= 1) {  // the value's fields (a String's length is only known by reading it)
      const uint8_t* f = e + 1 + (tag == 0 ? 8 : 0);
      const uint8_t* end = e + len;
      int64_t at = 0;
      bool ok = true;
      for (int i = 0; i < L->nfields && ok; i++) {
        if (L->kind[i] == OR_WIRE_STRING) {
          bool is_null = false;
          int32_t sh = 0;
          int64_t sid = 0;
          const int64_t m = read_string(f + at, end, &is_null, &sh, &sid);
          if (m < 0) {
            ok = false;
            break;
          }
          if (L->role[i] == OR_ROLE_KEY) {
            null_key = is_null;
            k = sid;
            h = sh;
          }
          at += m;
        } else {
          if (f + at + field_bytes(L->kind[i]) > end) {
            ok = false;
            break;
          }
          if (L->role[i] == OR_ROLE_KEY) k = field_value(L->kind[i], f + at);
          if (L->role[i] == OR_ROLE_VALUE) v = field_value(L->kind[i], f + at);
          at += field_bytes(L->kind[i]);
        }
      }
      if (strings) want = ok ? (f - e) + at : -1;
    }
    if (len != want) {  // an element of another layout
      st->bad_tag = -2;
      st->consumed = pos;
      return -1;
    }
    if (null_key) {
      st->bad_tag = -4;
      st->consumed = pos;
      return -1;
    }
    if (tag <= 1) {
      if (st->records >= cap) return -2;
      const int64_t r = st->records++;
      ts[r] = tag == 0 ? (int64_t)get_be(e + 1, 8) : INT64_MIN;
      key[r] = k;
      val[r] = v;
      if (kh) kh[r] = h;
    } else if (tag == 2) {
      st->watermarks++;
      st->watermark = (int64_t)get_be(e + 1, 8);
    } else if (tag == 3) {
      st->latency_markers++;
    } else {
      st->statuses++;
      st->status = (int32_t)get_be(e + 1, 4);
    }
    pos += 4 + len;
  }
  st->consumed = pos;
  return 0;
}

int64_t oracle_wire_encode(const oracle_wire_layout* L, const oracle_row* rows, int64_t n, int32_t f64, uint8_t* out,
                           int64_t cap) {
  const int F = value_bytes(L);
  const int64_t S = 4 + 9 + F;
  if (n * S > cap) return -1;
  for (int64_t r = 0; r < n; r++) {
    uint8_t* p = out + r * S;
    put_be(p, (uint64_t)(9 + F), 4);
    p[4] = 0;
    // window.maxTimestamp(): TimeWindow end - 1 (TimeWindow.java:83-85); GlobalWindow Long.MAX_VALUE
    // (GlobalWindow.java:45-46, count-window rows carry end = Long.MAX_VALUE)
    put_be(p + 5, (uint64_t)(rows[r].end == INT64_MAX ? rows[r].end : rows[r].end - 1), 8);
    uint8_t* f = p + 13;
    for (int i = 0; i < L->nfields; i++) {
      const oracle_row& w = rows[r];
      const int role = L->role[i];
      int64_t v = role == OR_ROLE_KEY ? w.key : role == OR_ROLE_START ? w.start : role == OR_ROLE_END ? w.end
                : role == OR_ROLE_COUNT ? w.count : role == OR_ROLE_SUM ? w.sum : role == OR_ROLE_MIN ? w.min
                : role == OR_ROLE_MAX ? w.max : 0;
      const bool dbl_field = L->kind[i] == OR_WIRE_DOUBLE || L->kind[i] == OR_WIRE_FLOAT;
      const bool dbl_value = f64 && (role == OR_ROLE_SUM || role == OR_ROLE_MIN || role == OR_ROLE_MAX);
      if (dbl_field && !dbl_value) {  // an integer row field written as a Double / Float field
        const double d = (double)v;
        std::memcpy(&v, &d, 8);
      } else if (!dbl_field && dbl_value) {  // a double row field written as an integer field: Java's (long) cast
        double d;
        std::memcpy(&d, &v, 8);
        v = d != d ? 0 : d >= 9.2233720368547758e18 ? INT64_MAX : d <= -9.2233720368547758e18 ? INT64_MIN : (int64_t)d;
      }
      put_field(L->kind[i], f, v);
      f += field_bytes(L->kind[i]);
    }
  }
  return n * S;
}

int64_t oracle_wire_put_record(const oracle_wire_layout* L, int32_t with_ts, int64_t ts, const int64_t* fields,
                               uint8_t* out) {
  const int F = value_bytes(L);
  const int64_t len = (with_ts ? 9 : 1) + F;
  put_be(out, (uint64_t)len, 4);
  out[4] = with_ts ? 0 : 1;
  uint8_t* f = out + 5;
  if (with_ts) {
    put_be(f, (uint64_t)ts, 8);
    f += 8;
  }
  for (int i = 0; i < L->nfields; i++) {
    put_field(L->kind[i], f, fields[i]);
    f += field_bytes(L->kind[i]);
  }
  return 4 + len;
}
int64_t oracle_wire_put_watermark(int64_t wm, uint8_t* out) {
  put_be(out, 9, 4);
  out[4] = 2;
  put_be(out + 5, (uint64_t)wm, 8);
  return 13;
}
int64_t oracle_wire_put_status(int32_t status, uint8_t* out) {
  put_be(out, 5, 4);
  out[4] = 4;
  put_be(out + 5, (uint32_t)status, 4);
  return 9;
}
int64_t oracle_wire_put_latency(int64_t marked, int64_t id_lo, int64_t id_hi, int32_t subtask, uint8_t* out) {
  put_be(out, 29, 4);
  out[4] = 3;
  put_be(out + 5, (uint64_t)marked, 8);
  put_be(out + 13, (uint64_t)id_lo, 8);
  put_be(out + 21, (uint64_t)id_hi, 8);
  put_be(out + 29, (uint32_t)subtask, 4);
  return 33;
}

}  // extern "C"
