// fw_wire.hip — f2: Flink's wire format for one input / output channel <-> device columns (include/flink_window.h).
//
// Decode.  A channel's bytes are 4-byte big-endian lengths each followed by a StreamElement
// (SpanningRecordSerializer.java:76-98, StreamElementSerializer.java:54-58,167-221).  Element boundaries depend on
// every earlier length, so the stream is cut into WCH-byte chunks and each chunk is parsed speculatively by one
// wave, lane e starting at the chunk's byte e: an element is at most WE = 64 bytes with its prefix, so the first
// element that starts in a chunk starts in its first 64 bytes.  Each (chunk, e) yields where the walk leaves the
// chunk (the offset into the next one, or END / BAD) and how many records it passed.  These transfer functions
// are composed 64 at a time up to one function for the whole stream, applied to entry 0 and pushed back down to
// every chunk (log64 levels), which gives every chunk its true first element.  A scan of the chunks' record
// counts places each chunk's records; one wave per chunk then walks its elements once more and writes them.
// Encode.  One thread per fired row writes one fixed-size element.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/flink_window.h"
#include "fw_internal.h"

namespace {

constexpr int WCH = 2048;  // chunk bytes
constexpr int WE = 64;     // possible first-element offsets per chunk = the largest element with its prefix
constexpr uint8_t X_END = 0xFE, X_BAD = 0xFF;  // the walk ended with the stream / met an element that cannot be
constexpr int WMAX_ELEMS = WCH / 5 + 2;         // elements starting in one chunk, at most (the smallest is 9 B)

struct WireL {
  int32_t nf, F;  // fields, value bytes (of the fixed-size fields)
  int32_t vs;     // the layout has String fields: a record's value length is found by reading them
  int32_t kind[FW_WIRE_MAX_FIELDS], role[FW_WIRE_MAX_FIELDS], off[FW_WIRE_MAX_FIELDS];
};

__host__ __device__ inline int field_bytes(int32_t kind) {
  return kind == FW_WIRE_LONG || kind == FW_WIRE_DOUBLE ? 8 : kind == FW_WIRE_INT || kind == FW_WIRE_FLOAT ? 4
       : kind == FW_WIRE_SHORT ? 2 : kind == FW_WIRE_BYTE || kind == FW_WIRE_BOOL ? 1 : -1;
}
__device__ inline uint64_t ld_be(const uint8_t* p, int nb) {
  uint64_t v = 0;
  for (int i = 0; i < nb; i++) v = (v << 8) | p[i];
  return v;
}
__device__ inline void st_be(uint8_t* p, uint64_t v, int nb) {
  for (int i = nb - 1; i >= 0; i--) {
    p[i] = (uint8_t)(v & 0xffu);
    v >>= 8;
  }
}
// StreamElementSerializer's element length for a tag under layout L, -1 for an unknown tag
__device__ inline int64_t want_len(const WireL& L, int tag) {
  return tag == 0 ? 9 + L.F : tag == 1 ? 1 + L.F : tag == 2 ? 9 : tag == 3 ? 29 : tag == 4 ? 5 : -1;
}
__device__ inline uint64_t wfmix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}
// StringValue.readString's base-128 varint (StringValue.java:745-786), low group first: its bytes, -1 past end
__device__ inline int wire_varint(const uint8_t* p, const uint8_t* end, uint32_t* out) {
  uint32_t v = 0;
  int shift = 0;
  for (int k = 0; p + k < end && k < 5; k++) {
    const uint32_t c = p[k];
    v |= (c & 0x7fu) << shift;
    if (c < 0x80u) {
      *out = v;
      return k + 1;
    }
    shift += 7;
  }
  return -1;
}
// a String field at p (StringValue.readString): its bytes, -1 if it runs past end; for a non-null one
// String.hashCode and the key column's id (FNV-1a 64 over the UTF-16 chars, fmix64 of it ^ the length:
// oracle_string_key_id)
__device__ inline int wire_string(const uint8_t* p, const uint8_t* end, bool* is_null, int32_t* hash, int64_t* id) {
  uint32_t len;
  int at = wire_varint(p, end, &len);
  if (at < 0) return -1;
  *is_null = len == 0;
  if (len == 0) return at;
  len -= 1;
  uint32_t h = 0;
  uint64_t f = 0xcbf29ce484222325ull;
  for (uint32_t i = 0; i < len; i++) {
    uint32_t c;
    const int k = wire_varint(p + at, end, &c);
    if (k < 0) return -1;
    at += k;
    const uint32_t ch = c & 0xffffu;  // (char) c
    h = 31u * h + ch;
    f = (f ^ ch) * 0x100000001b3ull;
  }
  *hash = (int32_t)h;
  *id = (int64_t)wfmix64(f ^ (uint64_t)len);
  return at;
}
// a record's value fields from p (the byte after the tag / timestamp) up to end: their bytes (-1 if they do not
// fit, or a String key is null), the key, its hash and the value
__device__ inline int64_t wire_fields(const WireL& L, const uint8_t* p, const uint8_t* end, int64_t* key, int32_t* kh,
                                      int64_t* val);
// the element at pos: its size with the prefix (> 0), -1 if the stream ends inside it (the next call's), 0 if it
// cannot be an element of this layout (an unknown tag, a length other than its tag's, a record whose String fields
// do not end where it does or whose String key is null, a String record longer than WE); *tag = its tag
__device__ inline int elem_at(const uint8_t* b, int64_t n, int64_t pos, const WireL& L, int* tag) {
  if (pos + 4 > n) return -1;
  const int64_t len = (int64_t)ld_be(b + pos, 4);
  if (pos + 4 + len > n) return -1;
  *tag = len > 0 ? (int)(int8_t)b[pos + 4] : -3;  // DataInputView.readByte of an empty element: EOF
  if (L.vs && (*tag == 0 || *tag == 1)) {
    if (4 + len > WE) return 0;
    const uint8_t* e = b + pos + 4;
    int64_t k, v;
    int32_t h;
    const int64_t head = *tag == 0 ? 9 : 1;
    const int64_t m = len >= head ? wire_fields(L, e + head, e + len, &k, &h, &v) : -1;
    return m >= 0 && head + m == len ? (int)(4 + len) : 0;
  }
  const int64_t w = want_len(L, *tag);
  return (w < 0 || len != w) ? 0 : (int)(4 + len);
}
// a field as the operator's 64-bit column: integers sign-extended, Double as its bits, Float widened to double bits
__device__ inline int64_t field_value(int32_t kind, const uint8_t* p) {
  switch (kind) {
    case FW_WIRE_LONG:
    case FW_WIRE_DOUBLE: return (int64_t)ld_be(p, 8);
    case FW_WIRE_INT: return (int64_t)(int32_t)(uint32_t)ld_be(p, 4);
    case FW_WIRE_SHORT: return (int64_t)(int16_t)(uint16_t)ld_be(p, 2);
    case FW_WIRE_BYTE: return (int64_t)(int8_t)p[0];
    case FW_WIRE_BOOL: return p[0] != 0;
    case FW_WIRE_FLOAT: return __double_as_longlong((double)__int_as_float((int)(uint32_t)ld_be(p, 4)));
  }
  return 0;
}

__device__ inline int64_t wire_fields(const WireL& L, const uint8_t* p, const uint8_t* end, int64_t* key, int32_t* kh,
                                      int64_t* val) {
  int64_t at = 0;
  *key = 0;
  *kh = 0;
  *val = 0;
  for (int f = 0; f < L.nf; f++) {
    if (L.kind[f] == FW_WIRE_STRING) {
      bool is_null = false;
      int32_t h = 0;
      int64_t id = 0;
      const int m = wire_string(p + at, end, &is_null, &h, &id);
      if (m < 0) return -1;
      if (L.role[f] == FW_ROLE_KEY) {
        if (is_null) return -1;  // a null key
        *key = id;
        *kh = h;
      }
      at += m;
    } else {
      const int fb = field_bytes(L.kind[f]);
      if (p + at + fb > end) return -1;
      if (L.role[f] == FW_ROLE_KEY) *key = field_value(L.kind[f], p + at);
      if (L.role[f] == FW_ROLE_VALUE) *val = field_value(L.kind[f], p + at);
      at += fb;
    }
  }
  return at;
}

// ---- speculation: per (chunk, first-element offset e) the exit into the next chunk and the records passed
__global__ __launch_bounds__(WE) void k_wire_spec(const uint8_t* __restrict__ b, int64_t n, int64_t nchunks, WireL L,
                                                 uint8_t* __restrict__ xt, uint32_t* __restrict__ ct) {
  const int64_t c = blockIdx.x;
  const int e = threadIdx.x;
  const int64_t cs = c * WCH, ce = cs + WCH;
  int64_t pos = cs + e;
  uint32_t cnt = 0;
  uint8_t x = 0;
  bool done = false;
  while (!done && pos < ce) {
    int tag = 0;
    const int sz = pos >= n ? -1 : elem_at(b, n, pos, L, &tag);
    if (sz < 0) {
      x = X_END;
      done = true;
    } else if (sz == 0) {
      x = X_BAD;
      done = true;
    } else {
      cnt += tag <= 1;
      pos += sz;
    }
  }
  if (!done) x = (uint8_t)(pos - ce);
  xt[c * WE + e] = x;
  ct[c * WE + e] = cnt;
}
// ---- composition: groups of 64 children -> one transfer function per group (one lane per entry)
__global__ __launch_bounds__(WE) void k_wire_up(const uint8_t* __restrict__ cx, const uint32_t* __restrict__ cc,
                                               int64_t nchild, uint8_t* __restrict__ gx, uint32_t* __restrict__ gc) {
  const int64_t g = blockIdx.x;
  uint32_t e = threadIdx.x, tot = 0;
  uint8_t x = 0;
  bool done = false;
  for (int64_t j = g * WE; j < min(nchild, (g + 1) * WE) && !done; j++) {
    const uint8_t y = cx[j * WE + e];
    tot += cc[j * WE + e];
    if (y >= X_END) {
      x = y;
      done = true;
    } else {
      e = y;
    }
  }
  if (!done) x = (uint8_t)e;
  gx[g * WE + threadIdx.x] = x;
  gc[g * WE + threadIdx.x] = tot;
}
// ---- and back down: a group's entry -> its children's entries, in order (one thread per group)
__global__ void k_wire_down(const uint8_t* __restrict__ cx, int64_t nchild, const uint8_t* __restrict__ gentry,
                            int64_t ngroups, uint8_t* __restrict__ centry) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngroups) return;
  uint8_t e = gentry[g];
  for (int64_t j = g * WE; j < min(nchild, (g + 1) * WE); j++) {
    centry[j] = e;
    if (e < X_END) e = cx[j * WE + e];
  }
}
// records of each chunk from its true first element (for the scan of output positions)
__global__ void k_wire_counts(const uint8_t* __restrict__ entry, const uint32_t* __restrict__ ct, int64_t nchunks,
                              uint32_t* __restrict__ cnt) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchunks) return;
  cnt[c] = entry[c] < X_END ? ct[c * WE + entry[c]] : 0u;
}
struct WireOut {
  int64_t *key, *ts, *val;
  int32_t* kh;              // the key's hash (String.hashCode of a String key), or nullptr
  int64_t* chunk_wm;        // per chunk: its last watermark, or INT64_MIN
  int64_t* chunk_status;    // per chunk: its last stream status, or INT64_MIN
  unsigned long long* acc;  // [0] watermarks, [1] latency markers, [2] statuses, [3] consumed (min over END walks),
                            // [4] first corrupt element (min), [5] its tag + 8
};
// ---- emission: one wave per chunk walks its elements from the true entry (lane 0), then all lanes write them
__global__ __launch_bounds__(WE) void k_wire_emit(const uint8_t* __restrict__ b, int64_t n, int64_t nchunks, WireL L,
                                                 const uint8_t* __restrict__ entry, const uint32_t* __restrict__ offs,
                                                 WireOut o) {
  const int64_t c = blockIdx.x;
  const int64_t cs = c * WCH, ce = cs + WCH;
  __shared__ uint16_t rel[WMAX_ELEMS];
  __shared__ int8_t tg[WMAX_ELEMS];
  __shared__ uint16_t rank[WMAX_ELEMS];
  __shared__ int ne;
  if (threadIdx.x == 0) {
    int k = 0, r = 0, wms = 0, lats = 0, sts = 0;
    int64_t wm = INT64_MIN, status = INT64_MIN;
    if (entry[c] < X_END) {
      int64_t pos = cs + entry[c];
      while (pos < ce) {
        int tag = 0;
        const int sz = pos >= n ? -1 : elem_at(b, n, pos, L, &tag);
        if (sz < 0) {  // the stream (or its complete elements) end here
          atomicMin(&o.acc[3], (unsigned long long)min(pos, n));
          break;
        }
        if (sz == 0) {  // IOException("Corrupt stream, found tag: " + tag)
          atomicMin(&o.acc[4], (unsigned long long)pos);
          break;
        }
        rel[k] = (uint16_t)(pos - cs);
        tg[k] = (int8_t)tag;
        rank[k] = (uint16_t)r;
        if (tag <= 1) r++;
        if (tag == 2) {
          wms++;
          wm = (int64_t)ld_be(b + pos + 5, 8);
        } else if (tag == 3) {
          lats++;
        } else if (tag == 4) {
          sts++;
          status = (int64_t)(int32_t)(uint32_t)ld_be(b + pos + 5, 4);
        }
        k++;
        pos += sz;
      }
    }
    ne = k;
    o.chunk_wm[c] = wm;
    o.chunk_status[c] = status;
    if (wms) atomicAdd(&o.acc[0], (unsigned long long)wms);
    if (lats) atomicAdd(&o.acc[1], (unsigned long long)lats);
    if (sts) atomicAdd(&o.acc[2], (unsigned long long)sts);
  }
  __syncthreads();
  const uint32_t base = offs[c];
  for (int i = threadIdx.x; i < ne; i += WE) {
    if (tg[i] > 1) continue;
    const uint8_t* p = b + cs + rel[i] + 5;
    const int64_t r = (int64_t)base + rank[i];
    int64_t t = INT64_MIN;  // StreamRecord.getTimestamp without a timestamp
    if (tg[i] == 0) {
      t = (int64_t)ld_be(p, 8);
      p += 8;
    }
    int64_t k = 0, v = 0;
    int32_t h = 0;
    if (L.vs) {  // (elem_at checked the fields)
      (void)wire_fields(L, p, b + n, &k, &h, &v);
    } else {
      for (int f = 0; f < L.nf; f++) {
        if (L.role[f] == FW_ROLE_KEY) k = field_value(L.kind[f], p + L.off[f]);
        if (L.role[f] == FW_ROLE_VALUE) v = field_value(L.kind[f], p + L.off[f]);
      }
    }
    o.key[r] = k;
    o.ts[r] = t;
    o.val[r] = v;
    if (o.kh) o.kh[r] = h;
  }
}
// the last watermark / status over the chunks (one workgroup), the tag of the first corrupt element
__global__ __launch_bounds__(1024) void k_wire_final(const uint8_t* __restrict__ b, int64_t nchunks, WireOut o,
                                                    int64_t* __restrict__ last) {
  __shared__ long long cw, cs_;
  if (threadIdx.x == 0) {
    cw = -1;
    cs_ = -1;
  }
  __syncthreads();
  for (int64_t c = threadIdx.x; c < nchunks; c += blockDim.x) {
    if (o.chunk_wm[c] != INT64_MIN) atomicMax(&cw, (long long)c);
    if (o.chunk_status[c] != INT64_MIN) atomicMax(&cs_, (long long)c);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    last[0] = cw >= 0 ? o.chunk_wm[cw] : INT64_MIN;
    last[1] = cs_ >= 0 ? o.chunk_status[cs_] : 0;  // StreamStatus.ACTIVE when the stream carried none
    const unsigned long long bad = o.acc[4];
    int64_t tag = 0;
    if (bad != ~0ull) {  // (an empty element has no tag byte: DataInputView.readByte at its end)
      const uint32_t len = ((uint32_t)b[bad] << 24) | ((uint32_t)b[bad + 1] << 16) | ((uint32_t)b[bad + 2] << 8) | b[bad + 3];
      tag = len > 0 ? (int64_t)(int8_t)b[bad + 4] : -3;
    }
    last[2] = tag;
  }
}
// ---- encode: row r -> one element (tag 0, ts = end - 1, the layout's fields)
__global__ void k_wire_encode(DevRows rows, int64_t n, WireL L, int32_t f64, uint8_t* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int64_t S = 13 + L.F;
  uint8_t* p = out + r * S;
  st_be(p, (uint64_t)(9 + L.F), 4);
  p[4] = 0;
  // window.maxTimestamp(): end - 1 for a TimeWindow (TimeWindow.java:83-85), Long.MAX_VALUE for the GlobalWindow
  // of a count window (GlobalWindow.java:45-46; its rows carry end = Long.MAX_VALUE)
  const int64_t end = rows.end[r];
  st_be(p + 5, (uint64_t)(end == INT64_MAX ? end : end - 1), 8);
  for (int f = 0; f < L.nf; f++) {
    const int role = L.role[f];
    int64_t v = role == FW_ROLE_KEY ? rows.key[r] : role == FW_ROLE_START ? rows.start[r]
              : role == FW_ROLE_END ? rows.end[r] : role == FW_ROLE_COUNT ? rows.cnt[r]
              : role == FW_ROLE_SUM ? rows.sum[r] : role == FW_ROLE_MIN ? rows.mn[r] : rows.mx[r];
    const bool dbl_field = L.kind[f] == FW_WIRE_DOUBLE || L.kind[f] == FW_WIRE_FLOAT;
    const bool dbl_value = f64 && (role == FW_ROLE_SUM || role == FW_ROLE_MIN || role == FW_ROLE_MAX);
    if (dbl_field && !dbl_value) {
      v = __double_as_longlong((double)v);
    } else if (!dbl_field && dbl_value) {  // Java's (long) cast of a double
      const double d = __longlong_as_double(v);
      v = d != d ? 0 : d >= 9.2233720368547758e18 ? INT64_MAX : d <= -9.2233720368547758e18 ? INT64_MIN : (int64_t)d;
    }
    uint8_t* q = p + 13 + L.off[f];
    switch (L.kind[f]) {
      case FW_WIRE_LONG:
      case FW_WIRE_DOUBLE: st_be(q, (uint64_t)v, 8); break;
      case FW_WIRE_INT: st_be(q, (uint32_t)v, 4); break;
      case FW_WIRE_SHORT: st_be(q, (uint16_t)v, 2); break;
      case FW_WIRE_BYTE:
      case FW_WIRE_BOOL: q[0] = (uint8_t)v; break;
      case FW_WIRE_FLOAT: st_be(q, (uint32_t)__float_as_int((float)__longlong_as_double(v)), 4); break;
    }
  }
}

}  // namespace

struct fw_wire {
  fw_wire_layout layout{};
  WireL dl{};
  int32_t device = 0;
  int64_t max_bytes = 0, max_chunks = 0;
  hipStream_t stream = nullptr;
  std::string err;
  std::vector<int64_t> level_n;          // chunks, groups, groups of groups, ... (last = 1)
  std::vector<uint8_t*> lx;              // transfer-function exits per level
  std::vector<uint32_t*> lc;             // record counts per level
  std::vector<uint8_t*> lentry;          // entries per level
  uint32_t *cnt = nullptr, *scan_tmp = nullptr;
  int64_t* chunk_wm = nullptr;
  int64_t* chunk_status = nullptr;
  unsigned long long* acc = nullptr;
  int64_t* last = nullptr;
  int64_t* h_tot = nullptr;  // pinned: records, then acc[0..5], last[0..2]
};

namespace {
int wire_err(fw_wire* w, int code, const std::string& m) {
  if (w) w->err = m;
  return code;
}
#define WIRE_HIP(w, x)                                                                   \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) return wire_err(w, FW_ERR_HIP, std::string("HIP: ") + hipGetErrorString(e_)); \
  } while (0)
}  // namespace

extern "C" {

int fw_wire_create(const fw_wire_layout* layout, int64_t max_bytes, int32_t device, fw_wire** out) {
  if (!layout || !out || max_bytes <= 0) return FW_ERR_ARG;
  *out = nullptr;
  fw_wire* w = new fw_wire();
  w->layout = *layout;
  WireL& L = w->dl;
  L.nf = layout->nfields;
  if (L.nf < 1 || L.nf > FW_WIRE_MAX_FIELDS) {
    w->err = "a layout has 1 to 8 fields";
    *out = w;
    return FW_ERR_ARG;
  }
  int keys = 0, vals = 0;
  for (int f = 0; f < L.nf; f++) {
    L.kind[f] = layout->kind[f];
    L.role[f] = layout->role[f];
    const bool str = L.kind[f] == FW_WIRE_STRING;
    const int fb = str ? 0 : field_bytes(L.kind[f]);
    if (fb < 0 || L.role[f] < FW_ROLE_SKIP || L.role[f] > FW_ROLE_MAX) {
      w->err = "unknown field kind or role";
      *out = w;
      return FW_ERR_ARG;
    }
    if (str && L.role[f] != FW_ROLE_KEY && L.role[f] != FW_ROLE_SKIP) {
      w->err = "a String field is a key or skipped";
      *out = w;
      return FW_ERR_ARG;
    }
    L.vs |= str;
    L.off[f] = L.F;
    L.F += fb;
    keys += L.role[f] == FW_ROLE_KEY;
    vals += L.role[f] == FW_ROLE_VALUE;
  }
  if (keys > 1 || vals > 1) {
    w->err = "at most one key and one value field";
    *out = w;
    return FW_ERR_ARG;
  }
  w->device = device;
  w->max_bytes = max_bytes;
  *out = w;
  WIRE_HIP(w, hipSetDevice(device));
  WIRE_HIP(w, hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking));
  const int64_t nc = (max_bytes + WCH - 1) / WCH;
  w->max_chunks = nc;
  for (int64_t m = nc;; m = (m + WE - 1) / WE) {
    w->level_n.push_back(m);
    if (m == 1) break;
  }
  for (int64_t m : w->level_n) {
    uint8_t *x = nullptr, *en = nullptr;
    uint32_t* c = nullptr;
    WIRE_HIP(w, hipMalloc(&x, (size_t)m * WE));
    WIRE_HIP(w, hipMalloc(&c, (size_t)m * WE * sizeof(uint32_t)));
    WIRE_HIP(w, hipMalloc(&en, (size_t)m));
    w->lx.push_back(x);
    w->lc.push_back(c);
    w->lentry.push_back(en);
  }
  WIRE_HIP(w, hipMalloc(&w->cnt, (size_t)(nc + 1) * sizeof(uint32_t)));
  WIRE_HIP(w, hipMalloc(&w->scan_tmp, (size_t)((nc + 1) / 4096 + 2) * sizeof(uint32_t)));
  WIRE_HIP(w, hipMalloc(&w->chunk_wm, (size_t)nc * sizeof(int64_t)));
  WIRE_HIP(w, hipMalloc(&w->chunk_status, (size_t)nc * sizeof(int64_t)));
  WIRE_HIP(w, hipMalloc(&w->acc, 6 * sizeof(unsigned long long)));
  WIRE_HIP(w, hipMalloc(&w->last, 3 * sizeof(int64_t)));
  WIRE_HIP(w, hipHostMalloc(&w->h_tot, 16 * sizeof(int64_t)));
  return FW_OK;
}

void fw_wire_destroy(fw_wire* w) {
  if (!w) return;
  (void)hipSetDevice(w->device);
  if (w->stream) (void)hipStreamSynchronize(w->stream);
  for (auto* p : w->lx) (void)hipFree(p);
  for (auto* p : w->lc) (void)hipFree(p);
  for (auto* p : w->lentry) (void)hipFree(p);
  (void)hipFree(w->cnt);
  (void)hipFree(w->scan_tmp);
  (void)hipFree(w->chunk_wm);
  (void)hipFree(w->chunk_status);
  (void)hipFree(w->acc);
  (void)hipFree(w->last);
  if (w->h_tot) (void)hipHostFree(w->h_tot);
  if (w->stream) (void)hipStreamDestroy(w->stream);
  delete w;
}

const char* fw_wire_last_error(const fw_wire* w) { return w ? w->err.c_str() : "null codec"; }

int fw_wire_decode_device(fw_wire* w, const uint8_t* bytes, int64_t nbytes, int64_t* key, int64_t* ts, int64_t* val,
                          int64_t cap, fw_wire_stats* stats) {
  return fw_wire_decode_keyed_device(w, bytes, nbytes, key, nullptr, ts, val, cap, stats);
}

int fw_wire_decode_keyed_device(fw_wire* w, const uint8_t* bytes, int64_t nbytes, int64_t* key, int32_t* key_hash,
                                int64_t* ts, int64_t* val, int64_t cap, fw_wire_stats* stats) {
  if (!w || !stats || (nbytes > 0 && !bytes) || nbytes < 0) return FW_ERR_ARG;
  if (nbytes > w->max_bytes) return wire_err(w, FW_ERR_ARG, "stream longer than the codec's max_bytes");
  if (13 + w->dl.F > WE) return wire_err(w, FW_ERR_ARG, "decoded elements are at most 64 bytes (fields <= 51 bytes)");
  for (int f = 0; f < w->dl.nf; f++)
    if (w->dl.kind[f] == FW_WIRE_STRING && w->dl.role[f] == FW_ROLE_KEY && !key_hash)
      return wire_err(w, FW_ERR_ARG, "a String key needs the key_hash column (fw_wire_decode_keyed_device)");
  std::memset(stats, 0, sizeof *stats);
  stats->watermark = INT64_MIN;
  if (nbytes == 0) return FW_OK;
  WIRE_HIP(w, hipSetDevice(w->device));
  hipStream_t s = w->stream;
  const int64_t nc = (nbytes + WCH - 1) / WCH;
  // the levels of this stream: chunks, then groups of 64, ... up to one
  std::vector<int64_t> ln;
  for (int64_t m = nc;; m = (m + WE - 1) / WE) {
    ln.push_back(m);
    if (m == 1) break;
  }
  hipLaunchKernelGGL(k_wire_spec, dim3((unsigned)nc), dim3(WE), 0, s, bytes, nbytes, nc, w->dl, w->lx[0], w->lc[0]);
  for (size_t l = 1; l < ln.size(); l++)
    hipLaunchKernelGGL(k_wire_up, dim3((unsigned)ln[l]), dim3(WE), 0, s, w->lx[l - 1], w->lc[l - 1], ln[l - 1],
                       w->lx[l], w->lc[l]);
  // the whole stream starts at its byte 0; push the entries down
  WIRE_HIP(w, hipMemsetAsync(w->lentry[ln.size() - 1], 0, 1, s));
  for (size_t l = ln.size() - 1; l > 0; l--)
    hipLaunchKernelGGL(k_wire_down, dim3((unsigned)((ln[l] + 255) / 256)), dim3(256), 0, s, w->lx[l - 1], ln[l - 1],
                       w->lentry[l], ln[l], w->lentry[l - 1]);
  hipLaunchKernelGGL(k_wire_counts, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s, w->lentry[0], w->lc[0], nc,
                     w->cnt);
  WIRE_HIP(w, hipMemsetAsync(w->cnt + nc, 0, sizeof(uint32_t), s));
  fwdev::launch_scan(w->cnt, nc + 1, w->scan_tmp, s);  // cnt[nc] = the records
  WIRE_HIP(w, hipMemcpyAsync(w->h_tot, w->cnt + nc, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  WIRE_HIP(w, hipStreamSynchronize(s));
  const int64_t records = (int64_t)*reinterpret_cast<uint32_t*>(w->h_tot);
  if (records > cap) return wire_err(w, FW_ERR_STATE, "the stream holds " + std::to_string(records) +
                                                          " records, more than the output's capacity");
  unsigned long long init[6] = {0, 0, 0, (unsigned long long)nbytes, ~0ull, 0};
  WIRE_HIP(w, hipMemcpyAsync(w->acc, init, sizeof init, hipMemcpyHostToDevice, s));
  WireOut o{key, ts, val, key_hash, w->chunk_wm, w->chunk_status, w->acc};
  hipLaunchKernelGGL(k_wire_emit, dim3((unsigned)nc), dim3(WE), 0, s, bytes, nbytes, nc, w->dl, w->lentry[0], w->cnt, o);
  hipLaunchKernelGGL(k_wire_final, dim3(1), dim3(1024), 0, s, bytes, nc, o, w->last);
  WIRE_HIP(w, hipMemcpyAsync(w->h_tot + 1, w->acc, 6 * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  WIRE_HIP(w, hipMemcpyAsync(w->h_tot + 7, w->last, 3 * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  WIRE_HIP(w, hipGetLastError());
  WIRE_HIP(w, hipStreamSynchronize(s));
  const int64_t* h = w->h_tot;
  const uint64_t bad = (uint64_t)h[5];
  stats->records = records;
  stats->watermarks = h[1];
  stats->latency_markers = h[2];
  stats->statuses = h[3];
  stats->consumed = h[4];
  stats->watermark = h[7];
  stats->status = (int32_t)h[8];
  if (bad != ~0ull) {  // the reference's deserializer throws at the first element it cannot read
    stats->consumed = (int64_t)bad;
    const int64_t tag = h[9];
    const bool known = tag >= 0 && tag <= 4;
    return wire_err(w, FW_ERR_STATE,
                    known ? std::string("Corrupt stream: an element whose length does not match the layout") +
                                (w->dl.vs ? " (or a null String key, or a String record longer than 64 bytes)" : "") +
                                " at byte " + std::to_string(bad)
                          : "Corrupt stream, found tag: " + std::to_string(tag));
  }
  return FW_OK;
}

int fw_wire_encode_device(fw_wire* w, const fw_rows* rows, int64_t n, int32_t f64, uint8_t* out, int64_t cap,
                          int64_t* written) {
  if (!w || !rows || !written || n < 0) return FW_ERR_ARG;
  for (int f = 0; f < w->dl.nf; f++)
    if (w->dl.role[f] == FW_ROLE_VALUE) return wire_err(w, FW_ERR_ARG, "an output layout names row fields, not VALUE");
  if (w->dl.vs) return wire_err(w, FW_ERR_ARG, "String fields are decoded only (rows carry the key's 64-bit id)");
  const int64_t S = 13 + w->dl.F;
  *written = 0;
  if (n * S > cap) return wire_err(w, FW_ERR_STATE, "output buffer too small");
  if (n == 0) return FW_OK;
  WIRE_HIP(w, hipSetDevice(w->device));
  DevRows r{};
  r.key = rows->key;
  r.start = rows->start;
  r.end = rows->end;
  r.cnt = rows->count;
  r.sum = rows->sum;
  r.mn = rows->min;
  r.mx = rows->max;
  hipLaunchKernelGGL(k_wire_encode, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, w->stream, r, n, w->dl, f64, out);
  WIRE_HIP(w, hipGetLastError());
  WIRE_HIP(w, hipStreamSynchronize(w->stream));
  *written = n * S;
  return FW_OK;
}

}  // extern "C"
