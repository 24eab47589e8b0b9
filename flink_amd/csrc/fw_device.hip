// fw_device.hip — HIP kernels (gfx950) of the MI355X keyed event-time window operator.
//
// Per micro-batch (fw_push_*), with the watermark wm constant over the batch:
//   k_classify_hist   — KeyGroupRangeAssignment murmur hash -> state partition, window assignment
//                       and lateness class of every record; per-tile partition histogram.
//   k_scan_*          — exclusive scan of the (partition, tile) histogram.
//   k_scatter         — records of the order-independent class ("normal": every window of the
//                       record ends after wm) scattered into per-partition runs as whole 32-byte
//                       sectors; fully late records to the side output / late counter.
//   k_scatter_ordered — records that need arrival order (late firing, partially late, sessions)
//                       compacted in order into the ordered list (tiles without any exit at once).
//   k_aggregate       — one workgroup per state partition: pre-aggregation of the partition's
//                       (key, window) accumulators in a bucketized, fingerprint-tagged LDS hash
//                       table (64-bit LDS atomics), flushed into the partition's HBM region with
//                       plain read-modify-write (the region is owned by exactly one workgroup, so
//                       no global atomics on the data).
//   k_slow            — ordered replay of the ordered list, one thread per key, element by element
//                       exactly as WindowOperator.processElement (WindowOperator.java:291-421),
//                       including MergingWindowSet.addWindow for sessions.
// Per watermark (fw_advance_watermark):
//   k_fire            — HeapInternalTimerService.advanceWatermark as a scan/compaction: every region
//                       whose earliest timer is <= wm emits its fired windows and is rebuilt, without
//                       the cleaned-up entries, into the region's other buffer.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <rocprim/device/device_radix_sort.hpp>

#include "../../include/flink_window.h"
#include "fw_internal.h"

namespace {

constexpr int64_t LMAX = INT64_MAX;
constexpr int64_t LMIN = INT64_MIN;
typedef long long i64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ Java arithmetic, key hashing
#include "fw_jmath.h"
// fmix64 is a bijection: its inverse (multiplicative inverses of the two constants mod 2^64)
__device__ __forceinline__ uint64_t fmix64_inv(uint64_t x) {
  x ^= x >> 33;
  x *= 0x9cb4b2f8129337dbull;
  x ^= x >> 33;
  x *= 0x4f74430c22a54005ull;
  x ^= x >> 33;
  return x;
}
constexpr uint64_t SUB_SALT = 0x5851F42D4C957F2Dull;
// state partition of a key inside the handle's KeyGroupRange, -1 when outside it
__device__ __forceinline__ int32_t partition_of(const DevCfg& c, int64_t key, int32_t h) {
  int32_t local = key_group(h, c.max_par) - c.kg0;
  if ((uint32_t)local >= (uint32_t)c.n_kg) return -1;
  uint32_t sub = c.log_s ? (uint32_t)(fmix64((uint64_t)key ^ SUB_SALT) >> (64 - c.log_s)) : 0u;
  return (local << c.log_s) | (int32_t)sub;
}
// unsigned n / d for an invariant d via its reciprocal (m, l) from make_div_inv (Granlund and
// Montgomery, "Division by invariant integers using multiplication", Fig. 4.1): exact for every n
__device__ __forceinline__ uint64_t div_inv(uint64_t n, uint64_t m, int32_t l) {
  if (l == 0) return n;  // d == 1
  const uint64_t t1 = __umul64hi(m, n);
  return (t1 + ((n - t1) >> 1)) >> (l - 1);
}
// Java's truncating `t % d` for d > 0 (sign of the dividend), through the reciprocal
__device__ __forceinline__ int64_t jrem(int64_t t, int64_t d, uint64_t m, int32_t l) {
  const uint64_t u = t < 0 ? (uint64_t)0 - (uint64_t)t : (uint64_t)t;  // |t|, also for Long.MIN_VALUE
  const uint64_t r = u - div_inv(u, m, l) * (uint64_t)d;
  return t < 0 ? -(int64_t)r : (int64_t)r;
}
// TimeWindow.getWindowStartWithOffset (TimeWindow.java:254-256), Java overflow semantics
__device__ __forceinline__ int64_t wstart(int64_t ts, int64_t off, int64_t size, uint64_t m, int32_t l) {
  int64_t t = jadd(jsub(ts, off), size);
  return jsub(ts, jrem(t, size, m, l));
}
// WindowOperator.cleanupTime (WindowOperator.java:637-644) of window [., end)
__device__ __forceinline__ int64_t cleanup_of(int64_t end, int64_t lateness) {
  int64_t mx = jsub(end, 1);
  int64_t c = jadd(mx, lateness);
  return c >= mx ? c : LMAX;
}
// ---- compact records (CRec, DevCfg::compact)
// window delta of a one-window record's window start, or -1 when it has no compact form
__device__ __forceinline__ int64_t compact_delta(const DevCfg& c, int64_t start) {
  const uint64_t diff = (uint64_t)start - (uint64_t)c.cbase;
  const uint64_t d = div_inv(diff, c.mag_slide, c.l_slide);
  return d < (1ull << c.log_s) ? (int64_t)d : -1;
}
__device__ __forceinline__ int64_t compact_encode(const DevCfg& c, int64_t key, int64_t d) {
  const int sh = 64 - c.log_s;
  return (int64_t)((fmix64((uint64_t)key ^ SUB_SALT) & ((1ull << sh) - 1)) | ((uint64_t)d << sh));
}
// the key and window start of a compact record of partition p
__device__ __forceinline__ void compact_decode(const DevCfg& c, int32_t p, int64_t kw, int64_t* key, int64_t* start) {
  const int sh = 64 - c.log_s;
  const uint64_t sub = (uint64_t)(p & ((1 << c.log_s) - 1));
  const uint64_t h = ((uint64_t)kw & ((1ull << sh) - 1)) | (sub << sh);
  *key = (int64_t)(fmix64_inv(h) ^ SUB_SALT);
  *start = (int64_t)((uint64_t)c.cbase + ((uint64_t)kw >> sh) * (uint64_t)c.slide);
}
// ---- narrow records (DevCfg::narrow; dense single-pass batches): 8 bytes, {key << 35 | (d - ndn0) << 32 | (u32)value}
// for a key in [-2^28, 2^28), a window delta d (compact_delta) in [ndn0, ndn0 + 8) and an int32 value.  The
// aggregate widens a narrow record back to its CRec in registers (narrow_to_crec), so its LDS table and the region
// entries are those of the compact form.
constexpr int NW_DBITS = 3;
__device__ __forceinline__ bool narrow_encode(const DevCfg& c, int64_t key, int64_t d, int64_t v, uint64_t* w) {
  const int64_t dn = d - c.ndn0;
  if ((uint64_t)dn >= (1ull << NW_DBITS) || key < -(1ll << 28) || key >= (1ll << 28) || v != (int64_t)(int32_t)v)
    return false;
  *w = ((uint64_t)key << 35) | ((uint64_t)dn << 32) | (uint64_t)(uint32_t)v;
  return true;
}
__device__ __forceinline__ i64x2 narrow_to_crec(const DevCfg& c, uint64_t w) {
  const int64_t key = (int64_t)w >> 35;
  const int64_t d = (int64_t)((w >> 32) & ((1u << NW_DBITS) - 1)) + c.ndn0;
  return i64x2{compact_encode(c, key, d), (int64_t)(int32_t)(uint32_t)w};
}

// earliest pending timer of an entry: trigger timer at maxTimestamp if registered, else GC timer
__device__ __forceinline__ int64_t timer_of(const Entry& e, int64_t lateness) {
  return (e.meta & FW_TIMER) ? jsub(e.end, 1) : cleanup_of(e.end, lateness);
}
// end of the state entry that starts at `start`: the window's, or the pane's when sliding windows are
// kept as panes (DevCfg::panes)
__device__ __forceinline__ int64_t wend(const DevCfg& c, int64_t start) {
  return jadd(start, c.panes ? c.slide : c.size);
}
// ---- HyperLogLog (FW_AGG_HLL; the definition is restated in oracle/window_oracle.h)
__device__ __forceinline__ uint64_t pool_block_of(const Entry& e) { return (uint64_t)e.meta >> 1; }
// earliest pending timer of an entry; a pane's is its meta (the next window end it belongs to)
__device__ __forceinline__ int64_t entry_timer(const DevCfg& c, const Entry& e) {
  return c.panes ? e.meta : timer_of(e, c.lateness);
}

// Double.compare order as a signed 64-bit key (canonical NaN, Double.doubleToLongBits)
__device__ __forceinline__ int64_t f64_sortable(int64_t bits) {
  if ((bits & 0x7ff0000000000000ll) == 0x7ff0000000000000ll && (bits & 0x000fffffffffffffll)) bits = 0x7ff8000000000000ll;
  return bits >= 0 ? bits : (bits ^ 0x7fffffffffffffffll);
}
__device__ __forceinline__ int64_t f64_unsortable(int64_t s) { return s >= 0 ? s : (s ^ 0x7fffffffffffffffll); }

// ------------------------------------------------------------------ record classes
enum { CLS_NORMAL = 0, CLS_SLOW = 1, CLS_LATE = 2, CLS_SKIP = 3, CLS_BADTS = 4 };

// Windows of a record, newest first (SlidingEventTimeWindows.java:71-75 loop order).
__device__ __forceinline__ int num_windows(const DevCfg& c, int64_t ts, int64_t* last_start) {
  if (c.assigner == FW_TUMBLING) {
    *last_start = wstart(ts, c.offset, c.size, c.mag_size, c.l_size);
    return 1;
  }
  int64_t last = wstart(ts, c.offset, c.slide, c.mag_slide, c.l_slide);
  *last_start = last;
  int k = 0;
  const int64_t lo = jsub(ts, c.size);
  for (int64_t s = last; s > lo && k <= c.wpr; s = jsub(s, c.slide)) k++;
  return k;
}

// sessions: is `key` in the batch's taint set (keys with an ordered-path record in the batch)?
__device__ __forceinline__ uint32_t taint_slot0(const DevCfg& c, int64_t key) {
  return (uint32_t)(fmix64((uint64_t)key ^ 0x2545F4914F6CDD1Dull)) & c.taint_mask;
}
__device__ __forceinline__ bool taint_has(const DevCfg& c, int64_t key) {
  for (uint32_t i = 0, s = taint_slot0(c, key); i <= c.taint_mask; i++, s = (s + 1) & c.taint_mask) {
    if (c.taint_state[s] != c.taint_epoch) return false;
    if (c.taint_key[s] == (uint64_t)key) return true;
  }
  return false;
}
// a session element that may fire, merge into a fired window or be dropped: it needs arrival order
__device__ __forceinline__ bool session_ordered(const DevCfg& c, int64_t wm, int64_t ts) {
  return ts == LMIN || jsub(jadd(ts, c.gap), 1) <= wm;
}

// class of a record against watermark wm; for CLS_NORMAL also its windows (newest start, count).
// taint: the batch's Status.taint_any (sessions only).
__device__ __forceinline__ int classify(const DevCfg& c, int64_t wm, int64_t ts, int64_t* last_out = nullptr,
                                        int* k_out = nullptr, int64_t key = 0, int taint = 0) {
  if (c.assigner == FW_SESSION) {
    // A session element whose window [ts, ts + gap) ends after wm is added without firing, and every
    // merge it takes part in ends after wm too, so such elements commute (MergingWindowSet.addWindow
    // builds the connected components of the in-flight windows in any order): they take the parallel
    // path unless their key also has an element that needs arrival order in this batch.
    if (session_ordered(c, wm, ts)) return CLS_SLOW;
    if (taint == 2 || (taint == 1 && taint_has(c, key))) return CLS_SLOW;
    if (last_out) {
      *last_out = ts;
      *k_out = 1;
    }
    return CLS_NORMAL;
  }
  if (ts == LMIN) return CLS_BADTS;  // TumblingEventTimeWindows.java:69-71
  if (c.panes) {
    // allowedLateness 0: a window whose maxTimestamp <= wm has fired (or had no contents) and is never
    // evaluated again, so adding the element to its pane adds it to exactly the windows that are not
    // late (WindowOperator.java:379-407); only when the newest window is late is the element dropped
    const int64_t last = wstart(ts, c.offset, c.slide, c.mag_slide, c.l_slide);
    if (last_out) {
      *last_out = last;
      *k_out = 1;
    }
    if (cleanup_of(jadd(last, c.size), 0) > wm) return CLS_NORMAL;
    return ts <= wm ? CLS_LATE : CLS_SKIP;
  }
  int64_t last;
  int k = num_windows(c, ts, &last);
  if (last_out) {
    *last_out = last;
    *k_out = k;
  }
  if (k == 0) return jadd(ts, c.lateness) <= wm ? CLS_LATE : CLS_SKIP;
  const int64_t newest_end = jadd(last, c.size);
  const int64_t oldest_end = jadd(jsub(last, (int64_t)(k - 1) * c.slide), c.size);
  if (jsub(oldest_end, 1) > wm) return CLS_NORMAL;  // every window: maxTimestamp > wm
  if (cleanup_of(newest_end, c.lateness) <= wm)     // every window late (isWindowLate)
    return jadd(ts, c.lateness) <= wm ? CLS_LATE : CLS_SKIP;  // isElementLate
  if (c.agg == FW_AGG_TDIGEST && c.lateness == 0) {
    // t-digest (allowed lateness 0): the element goes into its windows that are not late -- the newest ones,
    // maxTimestamp > wm -- and none of them fires on it (WindowOperator.java:379-407), so it needs no arrival
    // order: the parallel path takes it with those windows only
    int kk = 1;
    while (kk < k && jsub(jadd(jsub(last, (int64_t)kk * c.slide), c.size), 1) > wm) kk++;
    if (k_out) *k_out = kk;
    return CLS_NORMAL;
  }
  return CLS_SLOW;
}

// slot hash of (key, window): low 32 bits pick the slot, bits 40..63 are the state-word fingerprint.
// Sessions hash the key only, so every in-flight session of a key sits on one probe chain.
__device__ __forceinline__ uint64_t slot_hash(const DevCfg& c, int64_t key, int64_t start) {
  uint64_t h = (uint64_t)key * 0x9E3779B97F4A7C15ull;
  if (c.assigner != FW_SESSION) h ^= fmix64((uint64_t)start + 0x632BE59BD9B4E019ull);
  return fmix64(h);
}
__device__ __forceinline__ uint32_t tag_of(uint64_t h) { return (uint32_t)(h >> 40) << 8; }
__device__ __forceinline__ uint32_t live_word(uint64_t h) { return SLOT_LIVE | tag_of(h); }

// a[j] for a runtime j without demoting the register array to scratch (select chain)
template <int N>
__device__ __forceinline__ int64_t pick(const int64_t (&a)[N], int j) {
  int64_t r = a[0];
#pragma unroll
  for (int q = 1; q < N; q++) r = j == q ? a[q] : r;
  return r;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
  const uint32_t lane = __lane_id();
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

__device__ __forceinline__ uint32_t ld_state(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// A region's state words at workgroup scope, for code in which one workgroup owns the region for the whole launch (the
// session flush): agent-scope accesses are kept coherent across the XCDs' L2s, so each one travels past the L2 (a
// round trip to the fabric per probe); these stay in the CU's L1 / the XCD's L2.  The next kernel sees the words
// through the launch boundary, as it sees the entries written with plain stores.
__device__ __forceinline__ uint32_t ld_state_wg(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t cas_state_wg(uint32_t* p, uint32_t expect, uint32_t v) {
  __hip_atomic_compare_exchange_strong(p, &expect, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return expect;
}
__device__ __forceinline__ void st_state_wg(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ------------------------------------------------------------------ output
// FW_AGG_FIRST / MINBY / MAXBY carry the records' arrival ordinals
__host__ __device__ __forceinline__ bool agg_ordinal(const DevCfg& c) {
  return c.agg >= FW_AGG_FIRST && c.agg <= FW_AGG_FIRST_MAX;
}
// MINBY / MAXBY (ComparableAggregator.java:72-94 with first = true): the entry's mn holds the selected
// element's field as a key whose minimum it is (Double.compare order for f64, ~ for maxBy) and mx its full
// arrival ordinal; a pair (key, ordinal) replaces it when it is lexicographically smaller (a strictly
// smaller field, or an equal field of an earlier element)
__device__ __forceinline__ int64_t by_key(int agg, int vtype, int64_t v) {
  const int64_t k = vtype == FW_VAL_F64 ? f64_sortable(v) : v;
  return agg == FW_AGG_MAXBY ? ~k : k;
}
__device__ __forceinline__ bool by_less(int64_t k, int64_t o, int64_t k2, int64_t o2) {
  return k < k2 || (k == k2 && o < o2);
}
// MINBY / MAXBY row: the selected field and the selected element's ordinal
__device__ __forceinline__ void by_row(int agg, int vtype, const Entry& e, int64_t* field, int64_t* ord) {
  const int64_t k = agg == FW_AGG_MAXBY ? ~e.mn : e.mn;
  *field = vtype == FW_VAL_F64 ? f64_unsortable(k) : k;
  *ord = e.mx;
}
__device__ __forceinline__ bool agg_first(int agg) { return agg == FW_AGG_FIRST || agg == FW_AGG_FIRST_MAX; }
__device__ __forceinline__ bool agg_by(int agg) { return agg == FW_AGG_MINBY || agg == FW_AGG_MAXBY; }
// the value the entry's mn lane takes for one record (sv: the field, f64 in sortable form): FIRST_MAX keeps
// ~field so the min is the max (MINBY / MAXBY update mn and mx together: by_less)
__device__ __forceinline__ int64_t mn_in(int agg, int64_t sv) { return agg == FW_AGG_FIRST_MAX ? ~sv : sv; }
// row / snapshot columns of an entry's mn and mx (MINBY / MAXBY: by_row)
__device__ __forceinline__ int64_t mn_out(const DevCfg& c, int64_t mn) {
  const int64_t s = c.agg == FW_AGG_FIRST_MAX ? ~mn : mn;
  return c.vtype == FW_VAL_F64 ? f64_unsortable(s) : s;
}
__device__ __forceinline__ int64_t mx_out(const DevCfg& c, int64_t mx) {
  return agg_first(c.agg) ? ~mx : c.vtype == FW_VAL_F64 ? f64_unsortable(mx) : mx;
}
// the sum in the field's type: Integer / Short / Byte sums wrap to their width (SumFunction.java:56-107), a Float
// field's sum is rounded to float (its double bits)
__device__ __forceinline__ int64_t sum_out(const DevCfg& c, int64_t s) {
  if (c.vtype == FW_VAL_F64) return c.f32 ? __double_as_longlong((double)(float)__longlong_as_double(s)) : s;
  return c.sum_bits == 32 ? (int64_t)(int32_t)s : c.sum_bits == 16 ? (int64_t)(int16_t)s
       : c.sum_bits == 8 ? (int64_t)(int8_t)s : s;
}
__device__ __forceinline__ void write_row(const DevCfg& c, const DevRows& out, unsigned long long pos, const Entry& e) {
  out.key[pos] = e.key;
  out.start[pos] = e.start;
  out.end[pos] = e.end;
  out.cnt[pos] = e.cnt;
  out.sum[pos] = sum_out(c, e.sum);
  out.mn[pos] = mn_out(c, e.mn);
  out.mx[pos] = mx_out(c, e.mx);
  if (agg_by(c.agg)) by_row(c.agg, c.vtype, e, &out.mn[pos], &out.mx[pos]);
}
// single-lane emission (ordered path)
__device__ __forceinline__ void emit_one(const DevCfg& c, const DevRows& out, Status* st, const Entry& e) {
  unsigned long long pos = atomicAdd(&st->out_rows, 1ull);
  if ((int64_t)pos < out.cap)
    write_row(c, out, pos, e);
  else
    atomicOr(&st->flags, FW_STATUS_OUT_FULL);
}
__device__ __forceinline__ void side_one(const DevSide& sd, Status* st, int64_t k, int64_t t, int64_t v) {
  unsigned long long pos = atomicAdd(&st->side_rows, 1ull);
  if ((int64_t)pos < sd.cap) {
    sd.key[pos] = k;
    sd.ts[pos] = t;
    sd.val[pos] = v;
  } else {
    atomicOr(&st->flags, FW_STATUS_SIDE_FULL);
  }
}

// accumulate one value (AggregateFunction.add of the built-in count/sum/min/max)
// (FW_AGG_FIRST: mx takes ~ordinal `fo` of the record, so the max keeps the first element's ordinal)
__device__ __forceinline__ void acc_add(const DevCfg& c, Entry& e, int64_t v, int64_t fo) {
  if (c.agg == FW_AGG_HLL || c.agg == FW_AGG_ROW) {  // the block is the accumulator; the row keeps the count
    e.cnt += 1;                                       // (as lds_acc's LDS_CNT_ONLY)
    return;
  }
  if (agg_by(c.agg)) {
    const int64_t k = by_key(c.agg, c.vtype, v);
    if (e.cnt == 0 || by_less(k, fo, e.mn, e.mx)) {
      e.mn = k;
      e.mx = fo;
    }
  }
  e.cnt += 1;
  int64_t sv = v;
  if (c.vtype == FW_VAL_F64) {
    double s = __longlong_as_double(e.sum) + __longlong_as_double(v);
    e.sum = __double_as_longlong(s);
    sv = f64_sortable(v);
  } else {
    e.sum = jadd(e.sum, v);
  }
  if (agg_by(c.agg)) return;
  const int64_t nv = mn_in(c.agg, sv);
  e.mn = nv < e.mn ? nv : e.mn;
  const int64_t xv = agg_ordinal(c) ? ~fo : sv;
  e.mx = xv > e.mx ? xv : e.mx;
}
// AggregateFunction.merge
__device__ __forceinline__ void acc_merge(const DevCfg& c, Entry& a, const Entry& b) {
  if (b.cnt == 0) return;
  if (agg_by(c.agg)) {  // the lexicographically smaller (key, ordinal) of the two
    if (a.cnt == 0 || by_less(b.mn, b.mx, a.mn, a.mx)) {
      a.mn = b.mn;
      a.mx = b.mx;
    }
    a.cnt += b.cnt;
    a.sum = c.vtype == FW_VAL_F64 ? __double_as_longlong(__longlong_as_double(a.sum) + __longlong_as_double(b.sum))
                                  : jadd(a.sum, b.sum);
    return;
  }
  a.cnt += b.cnt;
  if (c.vtype == FW_VAL_F64)
    a.sum = __double_as_longlong(__longlong_as_double(a.sum) + __longlong_as_double(b.sum));
  else
    a.sum = jadd(a.sum, b.sum);
  a.mn = b.mn < a.mn ? b.mn : a.mn;
  a.mx = b.mx > a.mx ? b.mx : a.mx;
}
__device__ __forceinline__ void acc_clear(Entry& e) {
  e.cnt = 0;
  e.sum = 0;
  e.mn = LMAX;
  e.mx = LMIN;
}

// ------------------------------------------------------------------ HBM regions
struct Region {
  Entry* ent;
  uint32_t* state;
  uint32_t mask;
};
__device__ __forceinline__ Region region_of(const DevCfg& c, const DevTable& tb, int32_t p, int which) {
  const int64_t base = (int64_t)p << c.log_r;
  Region r;
  r.ent = tb.ent[which] + base;
  r.state = tb.state[which] + base;
  r.mask = (1u << c.log_r) - 1u;
  return r;
}
// find the live slot of (key, start, end), -1 if absent (linear probing up to the first EMPTY).
// The fingerprint in the state word skips foreign slots without touching their entries.
// (from slot h & mask on, for the state word `want`)
// (OWN: the caller's workgroup owns the region for the launch -- the state words at workgroup scope, ld_state_wg)
template <bool OWN = false>
__device__ __forceinline__ int32_t region_find(const Region& r, uint64_t h, int64_t key, int64_t start, int64_t end,
                                               uint32_t want) {
  for (uint32_t i = 0; i < r.mask; i++) {
    const uint32_t s = ((uint32_t)h + i) & r.mask;
    const uint32_t st = OWN ? ld_state_wg(r.state + s) : ld_state(r.state + s);
    if (st == SLOT_EMPTY) return -1;
    if (st == want) {
      const Entry& e = r.ent[s];
      if (e.key == key && e.start == start && e.end == end) return (int32_t)s;
    }
  }
  return -1;
}
template <bool OWN = false>
__device__ __forceinline__ int32_t region_find(const Region& r, uint64_t h, int64_t key, int64_t start, int64_t end) {
  const uint32_t want = live_word(h);
  for (uint32_t i = 0; i <= r.mask; i++) {
    const uint32_t s = ((uint32_t)h + i) & r.mask;
    const uint32_t st = OWN ? ld_state_wg(r.state + s) : ld_state(r.state + s);
    if (st == SLOT_EMPTY) return -1;
    if (st == want) {
      const Entry& e = r.ent[s];
      if (e.key == key && e.start == start && e.end == end) return (int32_t)s;
    }
  }
  return -1;
}
// claim the first EMPTY slot of the probe sequence (state -> `word`), -1 if the region is full
template <bool OWN = false>
__device__ __forceinline__ int32_t region_claim(const Region& r, uint64_t h, uint32_t word) {
  for (uint32_t i = 0; i <= r.mask; i++) {
    const uint32_t s = ((uint32_t)h + i) & r.mask;
    if ((OWN ? ld_state_wg(r.state + s) : ld_state(r.state + s)) != SLOT_EMPTY) continue;
    if ((OWN ? cas_state_wg(r.state + s, SLOT_EMPTY, word) : atomicCAS(r.state + s, SLOT_EMPTY, word)) == SLOT_EMPTY)
      return (int32_t)s;
  }
  return -1;
}

// ============================================================================== kernels

// ---- K0 (sessions): the batch's taint set.  Keys with an element that needs arrival order
// (session_ordered) go into an open-addressing set whose slots are stamped with the batch's epoch, so
// the set is never cleared between batches.  Status.taint_any = 1 when some key was inserted, 2 when
// the set overflowed (then every record of the batch takes the ordered path).
constexpr uint32_t TAINT_BUSY = 0x80000000u;
constexpr int TAINT_MAX_PROBES = 64;
__device__ __forceinline__ bool taint_insert(const DevCfg& c, int64_t key) {
  uint32_t s = taint_slot0(c, key);
  for (int probes = 0; probes < TAINT_MAX_PROBES;) {
    // (relaxed agent-scope loads and write-through publication, as cnt_slot: no L1 invalidation per probe)
    const uint32_t cur = __hip_atomic_load(&c.taint_state[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_signal_fence(__ATOMIC_ACQUIRE);
    if (cur == c.taint_epoch) {
      if (__hip_atomic_load(&c.taint_key[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint64_t)key) return true;
      s = (s + 1) & c.taint_mask;
      probes++;
      continue;
    }
    if (cur == (c.taint_epoch | TAINT_BUSY)) continue;  // being published by another lane: re-read
    if (atomicCAS(&c.taint_state[s], cur, c.taint_epoch | TAINT_BUSY) == cur) {
      __hip_atomic_store(&c.taint_key[s], (uint64_t)key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&c.taint_state[s], c.taint_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return true;
    }
  }
  return false;
}
__global__ __launch_bounds__(256) void k_taint(DevCfg c, int64_t wm, const int64_t* __restrict__ key,
                                               const int64_t* __restrict__ ts, int64_t n, Status* st) {
  int any = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (!session_ordered(c, wm, ts[i])) continue;
    any = max(any, taint_insert(c, key[i]) ? 1 : 2);
  }
  if (any) atomicMax(&st->taint_any, any);
}

// ---- streaming input of the classify / scatter tiles.  A round covers blockDim.x * FW_RPT records;
// lane `tid` holds the pairs (j = 0 .. FW_RPT/2-1) of records rec_index(b, j, e) = b + 2(j*blockDim + tid) + e,
// loaded as one 16-byte load per column and pair when the columns are 16-byte aligned (DevCfg::vec_in).
__device__ __forceinline__ int64_t rec_index(int64_t b, int j, int e) {
  return b + 2 * ((int64_t)j * blockDim.x + threadIdx.x) + e;
}
template <int NP, bool VAL>
__device__ __forceinline__ void load_records(const DevCfg& c, const int64_t* __restrict__ key, const int64_t* __restrict__ ts,
                                             const int64_t* __restrict__ val, const int32_t* __restrict__ kh, int64_t b,
                                             int64_t end, int64_t (&k)[2 * NP], int64_t (&t)[2 * NP], int64_t (&v)[2 * NP],
                                             int32_t (&h)[2 * NP]) {
  const bool hashed = c.key_kind == FW_KEY_HASHED;
#pragma unroll
  for (int j = 0; j < NP; j++) {  // all loads in flight before any use
    const int64_t i = rec_index(b, j, 0);
    if (c.vec_in && i + 1 < end) {
      const i64x2 kk = *reinterpret_cast<const i64x2*>(key + i);
      const i64x2 tt = *reinterpret_cast<const i64x2*>(ts + i);
      k[2 * j] = kk.x, k[2 * j + 1] = kk.y;
      t[2 * j] = tt.x, t[2 * j + 1] = tt.y;
      if (VAL) {
        const i64x2 vv = *reinterpret_cast<const i64x2*>(val + i);
        v[2 * j] = vv.x, v[2 * j + 1] = vv.y;
      }
      if (hashed) {
        const int2 hh = *reinterpret_cast<const int2*>(kh + i);
        h[2 * j] = hh.x, h[2 * j + 1] = hh.y;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 2; e++) {
        const bool in = i + e < end;
        k[2 * j + e] = in ? key[i + e] : 0;
        t[2 * j + e] = in ? ts[i + e] : 0;
        if (VAL) v[2 * j + e] = in ? val[i + e] : 0;
        if (hashed) h[2 * j + e] = in ? kh[i + e] : 0;
      }
    }
  }
}
// tile of a classify / scatter workgroup: with FW_XCD_TILES, blocks b, b+8, b+16, ... (one XCD) take
// consecutive tiles, so the partition runs of neighbouring tiles meet in one L2
__device__ __forceinline__ int32_t tile_of_block(int32_t T) {
  const int32_t b = blockIdx.x;
  if (!FW_XCD_TILES) return b;
  const int32_t per = T >> 3, rem = T & 7, g = b & 7;
  return g * per + min(g, rem) + (b >> 3);
}

// The streaming kernels are instantiated for the common shapes too: Long keys with tumbling windows, and Long
// keys with panes.  The configuration is then known to the compiler (the generic instantiation's branches for
// other assigners, key kinds and session taint drop out of the per-record loop).
enum { M_GEN = 0, M_TUMB = 1, M_PANE = 2 };
template <int MODE>
__device__ __forceinline__ void specialize(DevCfg& c) {
  if constexpr (MODE == M_TUMB) {
    c.assigner = FW_TUMBLING;
    c.panes = 0;
    c.wpr = 1;
    c.key_kind = FW_KEY_LONG;
  } else if constexpr (MODE == M_PANE) {
    c.assigner = FW_SLIDING;
    c.panes = 1;
    c.key_kind = FW_KEY_LONG;
  }
}
__host__ __forceinline__ int stream_mode(const DevCfg& c) {
  if (c.key_kind != FW_KEY_LONG) return M_GEN;
  if (c.assigner == FW_TUMBLING) return M_TUMB;
  return c.panes ? M_PANE : M_GEN;
}

// single-pass scatter (k_scatter_rsv): its slots behind the P run lengths, rsv[P + x]
enum { RSV_OVER = 0, RSV_KG = 1, RSV_TS = 2, RSV_LATE = 4 };  // RSV_LATE: 64-bit (FW_RSV_WORDS in all)

// ---- K1: classify + partition histogram.  hist is (P+1) x T, partition-major; row P counts
// the records of each tile that go to the ordered path (scanned with the partitions), row P+1
// keeps that count unscanned for k_scatter_ordered.
template <int MODE>
__global__ __launch_bounds__(FW_TILE_THREADS) void k_classify_hist(DevCfg c, int64_t wm, const int64_t* __restrict__ key,
                                                                   const int64_t* __restrict__ ts,
                                                                   const int32_t* __restrict__ kh, int64_t n, int32_t T,
                                                                   uint32_t* __restrict__ hist, Status* st,
                                                                   const uint32_t* __restrict__ rsv) {
  specialize<MODE>(c);
  if (rsv && !rsv[c.P + RSV_OVER]) {  // the single pass took the batch: its counts go to the status once
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      if (rsv[c.P + RSV_KG]) atomicAdd(&st->kg_errors, (int)rsv[c.P + RSV_KG]);
      if (rsv[c.P + RSV_TS]) atomicAdd(&st->ts_errors, (int)rsv[c.P + RSV_TS]);
      const unsigned long long late = *reinterpret_cast<const unsigned long long*>(rsv + c.P + RSV_LATE);
      if (late) atomicAdd(&st->late_dropped, late);
    }
    return;
  }
  if (rsv && blockIdx.x == 0 && threadIdx.x == 0) {
    if (rsv[c.P + FW_RSV_NARROW])
      atomicAdd(&st->narrow_misses, 1);
    else
      atomicAdd(&st->rsv_fallbacks, 1);
  }
  extern __shared__ uint32_t lh[];
  for (int i = threadIdx.x; i <= c.P; i += blockDim.x) lh[i] = 0;
  __syncthreads();
  const int32_t tile = blockIdx.x;
  const int64_t base = (int64_t)tile * FW_TILE;
  const int64_t end = min(n, base + (int64_t)FW_TILE);
  int bad_kg = 0, bad_ts = 0, wide = 0;
  unsigned slow = 0;
  const int taint = c.assigner == FW_SESSION ? st->taint_any : 0;
  for (int64_t b = base; b < end; b += (int64_t)blockDim.x * FW_RPT) {
    int64_t k[FW_RPT], t[FW_RPT], v[FW_RPT];
    int32_t h[FW_RPT];
    load_records<FW_RPT / 2, false>(c, key, ts, nullptr, kh, b, end, k, t, v, h);
#pragma unroll
    for (int j = 0; j < FW_RPT; j++) {
      const int64_t i = rec_index(b, j >> 1, j & 1);
      if (i >= end) continue;
      const int32_t p = partition_of(c, k[j], c.key_kind == FW_KEY_HASHED ? h[j] : key_hash_of(c.key_kind, k[j], kh, i));
      if (p < 0) {
        bad_kg++;
        continue;
      }
      int64_t last = 0;
      int nw = 0;
      const int cls = classify(c, wm, t[j], &last, &nw, k[j], taint);
      if (cls == CLS_NORMAL) {
        atomicAdd(&lh[p], 1u);
        if (c.compact && compact_delta(c, last) < 0) wide = 1;
      } else if (cls == CLS_SLOW)
        slow++;
      else if (cls == CLS_BADTS)
        bad_ts++;
    }
  }
  if (slow) atomicAdd(&lh[c.P], slow);
  __syncthreads();
  for (int i = threadIdx.x; i <= c.P; i += blockDim.x) hist[(int64_t)i * T + tile] = lh[i];
  if (threadIdx.x == 0) hist[(int64_t)(c.P + 1) * T + tile] = lh[c.P];
  if (bad_kg) atomicAdd(&st->kg_errors, bad_kg);
  if (bad_ts) atomicAdd(&st->ts_errors, bad_ts);
  if (wide) atomicOr(c.wide, 1);
}

// ---- generic in-place exclusive scan of uint32 (block = 1024 threads x 4 elements)
constexpr int SCAN_T = 1024, SCAN_E = 4, SCAN_B = SCAN_T * SCAN_E;

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sw, uint32_t* total) {
  const int lane = __lane_id(), wid = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sw[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = 0;
    const int nw = blockDim.x >> 6;
    for (int w = 0; w < nw; w++) {
      uint32_t t = sw[w];
      sw[w] = run;
      run += t;
    }
    sw[nw] = run;
  }
  __syncthreads();
  *total = sw[blockDim.x >> 6];
  uint32_t r = sw[wid] + x - v;
  __syncthreads();
  return r;
}

// (gate: a flag the scan runs behind, nullptr = always)
__global__ __launch_bounds__(SCAN_T) void k_scan_blocks(uint32_t* data, int64_t m, uint32_t* sums, const uint32_t* gate) {
  if (gate && !*gate) return;
  __shared__ uint32_t sw[SCAN_T / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * SCAN_B + (int64_t)threadIdx.x * SCAN_E;
  uint32_t v[SCAN_E];
  uint32_t local = 0;
#pragma unroll
  for (int e = 0; e < SCAN_E; e++) {
    v[e] = base + e < m ? data[base + e] : 0u;
    local += v[e];
  }
  uint32_t total;
  uint32_t off = block_excl_scan(local, sw, &total);
#pragma unroll
  for (int e = 0; e < SCAN_E; e++) {
    if (base + e < m) data[base + e] = off;
    off += v[e];
  }
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}
__global__ __launch_bounds__(SCAN_T) void k_scan_top(uint32_t* sums, int64_t nb, const uint32_t* gate) {
  if (gate && !*gate) return;
  __shared__ uint32_t sw[SCAN_T / 64 + 1];
  uint32_t carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += SCAN_T) {
    const int64_t i = b0 + threadIdx.x;
    uint32_t v = i < nb ? sums[i] : 0u, total;
    uint32_t off = block_excl_scan(v, sw, &total);
    if (i < nb) sums[i] = off + carry;
    carry += total;
  }
}
__global__ __launch_bounds__(SCAN_T) void k_scan_add(uint32_t* data, int64_t m, const uint32_t* sums, const uint32_t* gate) {
  if (gate && !*gate) return;
  const uint32_t add = sums[blockIdx.x];
  const int64_t base = (int64_t)blockIdx.x * SCAN_B;
  for (int e = threadIdx.x; e < SCAN_B; e += SCAN_T)
    if (base + e < m) data[base + e] += add;
}

// the gated scan of a single-pass fallback in one workgroup: one launch when the gate is closed (the common case: the
// batch went through the single pass), a slower scan when it is open (a batch the single pass could not take, rare:
// three in a row turn the single pass off)
__global__ __launch_bounds__(SCAN_T) void k_scan_gated(uint32_t* data, int64_t m, const uint32_t* gate) {
  if (!*gate) return;
  __shared__ uint32_t sw[SCAN_T / 64 + 1];
  uint32_t carry = 0;
  for (int64_t b0 = 0; b0 < m; b0 += SCAN_B) {
    const int64_t base = b0 + (int64_t)threadIdx.x * SCAN_E;
    uint32_t v[SCAN_E];
    uint32_t local = 0;
#pragma unroll
    for (int e = 0; e < SCAN_E; e++) {
      v[e] = base + e < m ? data[base + e] : 0u;
      local += v[e];
    }
    uint32_t total;
    uint32_t off = block_excl_scan(local, sw, &total) + carry;
#pragma unroll
    for (int e = 0; e < SCAN_E; e++) {
      if (base + e < m) data[base + e] = off;
      off += v[e];
    }
    carry += total;
    __syncthreads();  // (sw is reused by the next chunk's scan)
  }
}

// Store a 32-byte record per lane as whole sectors written by lane pairs: lanes 2i and 2i+1 first
// write lane 2i's record (16 B each, contiguous), then lane 2i+1's.  The halves and positions are
// swapped between the pair with DPP (quad_perm [1,0,3,2]); a wave's store then addresses 32 sectors
// instead of 64 scattered 16-byte halves.  Every lane of the wave must reach this call.
__device__ __forceinline__ uint32_t dpp_swap1(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ int64_t dpp_swap1(int64_t x) {
  const uint32_t lo = dpp_swap1((uint32_t)(uint64_t)x), hi = dpp_swap1((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ void store_pair(PRec* part, bool valid, uint32_t pos, i64x2 a, i64x2 b) {
  const bool odd = __lane_id() & 1;
  const i64x2 send = odd ? a : b;
  const i64x2 recv = {dpp_swap1((int64_t)send.x), dpp_swap1((int64_t)send.y)};
  const uint32_t ppos = dpp_swap1(pos);
  const bool pval = dpp_swap1((uint32_t)valid) != 0;
  // the even lane's record: the even lane writes its first half, the odd lane its second half
  if (odd ? pval : valid) reinterpret_cast<i64x2*>(part + (odd ? ppos : pos))[odd] = odd ? recv : a;
  // the odd lane's record
  if (odd ? valid : pval) reinterpret_cast<i64x2*>(part + (odd ? pos : ppos))[odd] = odd ? b : recv;
}

// ---- K2: scatter.  Normal records -> their partition's run (any order inside the run), one
// 32-byte sector per record; late records -> side output / counter.
// (the body of one tile: base = P words of LDS for the runs' next free slots)
__device__ __forceinline__ void scatter_direct(const DevCfg& c, int64_t wm, const int64_t* __restrict__ key,
                                               const int64_t* __restrict__ ts, const int64_t* __restrict__ val,
                                               const int32_t* __restrict__ kh, int64_t n, int32_t T,
                                               const uint32_t* __restrict__ offs, PRec* __restrict__ part, DevSide side,
                                               Status* st, uint32_t* base, int32_t tile) {
  for (int i = threadIdx.x; i < c.P; i += blockDim.x) base[i] = offs[(int64_t)i * T + tile];
  __syncthreads();
  const int64_t tbase = (int64_t)tile * FW_TILE;
  const int64_t tend = min(n, tbase + (int64_t)FW_TILE);
  unsigned long long late = 0;
  const int taint = c.assigner == FW_SESSION ? st->taint_any : 0;
  const bool cmp = c.compact && !*c.wide;  // (uniform: every classify workgroup has finished)
  for (int64_t b = tbase; b < tend; b += (int64_t)blockDim.x * FW_RPT) {
    int64_t k[FW_RPT], t[FW_RPT], v[FW_RPT];
    int32_t hh[FW_RPT];
    load_records<FW_RPT / 2, true>(c, key, ts, val, kh, b, tend, k, t, v, hh);
#pragma unroll
    for (int j = 0; j < FW_RPT; j++) {
      const int64_t i = rec_index(b, j >> 1, j & 1);
      bool norm = false;
      uint32_t pos = 0;
      int64_t last = 0;
      int nwin = 0;
      if (i < tend) {
        const int32_t h = c.key_kind == FW_KEY_HASHED ? hh[j] : key_hash_of(c.key_kind, k[j], kh, i);
        const int32_t p = partition_of(c, k[j], h);
        if (p >= 0) {
          const int cls = classify(c, wm, t[j], &last, &nwin, k[j], taint);
          if (cls == CLS_NORMAL) {
            pos = atomicAdd(&base[p], 1u);
            norm = true;
          } else if (cls == CLS_LATE) {
            if (c.side_output)
              side_one(side, st, k[j], t[j], v[j]);
            else
              late++;
          }
        }
      }
      if (c.diag & (DIAG_SCATTER_NO_STORE | DIAG_SCATTER_LINEAR | DIAG_SCATTER_SINGLE | DIAG_SCATTER_HALF |
                    DIAG_SCATTER_NT)) {
        if (c.diag & DIAG_SCATTER_NO_STORE) {
          asm volatile("" ::"v"(pos), "v"(k[j]), "v"(last), "v"(v[j]));
          continue;
        }
        if (c.diag & DIAG_SCATTER_LINEAR) pos = (uint32_t)i;
        if ((c.diag & DIAG_SCATTER_HALF) && norm) {  // 16 B per record (timing of a compact record)
          i64x2* dst = reinterpret_cast<i64x2*>(part) + pos;
          if (c.diag & DIAG_SCATTER_NT)
            __builtin_nontemporal_store(i64x2{k[j] ^ last, v[j]}, dst);
          else
            *dst = i64x2{k[j] ^ last, v[j]};
          continue;
        }
        if ((c.diag & DIAG_SCATTER_NT) && norm) {
          i64x2* dst = reinterpret_cast<i64x2*>(part + pos);
          __builtin_nontemporal_store(i64x2{k[j], last}, dst);
          __builtin_nontemporal_store(i64x2{v[j], (long long)nwin}, dst + 1);
          continue;
        }
        if (norm) {
          i64x2* dst = reinterpret_cast<i64x2*>(part + pos);
          dst[0] = i64x2{k[j], last};
          dst[1] = i64x2{v[j], (long long)nwin};
        }
        continue;
      }
      if (cmp) {  // CRec: one 16-byte store
        if (norm) reinterpret_cast<i64x2*>(part)[pos] = i64x2{compact_encode(c, k[j], compact_delta(c, last)), v[j]};
        continue;
      }
      // ordinal aggregates: the record's index in the batch rides above the window count (nwin < 2^16); the
      // aggregate adds the batch's ordinal base (DevCfg::ord_base), so ordinals are exact to 2^63
      const int64_t nwf = agg_ordinal(c) ? (i << 16) | nwin : (int64_t)nwin;
      store_pair(part, norm, pos, i64x2{k[j], last}, i64x2{v[j], (long long)nwf});
    }
  }
  if (late) atomicAdd(&st->late_dropped, late);
}
template <int MODE>
__global__ __launch_bounds__(FW_TILE_THREADS, FW_SCATTER_WAVES) void k_scatter(DevCfg c, int64_t wm, const int64_t* __restrict__ key,
                                                             const int64_t* __restrict__ ts,
                                                             const int64_t* __restrict__ val,
                                                             const int32_t* __restrict__ kh, int64_t n, int32_t T,
                                                             const uint32_t* __restrict__ offs, PRec* __restrict__ part,
                                                             DevSide side, Status* st) {
  specialize<MODE>(c);
  extern __shared__ uint32_t base[];  // P: next free slot of each partition's run for this tile
  scatter_direct(c, wm, key, ts, val, kh, n, T, offs, part, side, st, base, tile_of_block(T));
}

// ---- K2, staged form (compact batches, P <= 2048).  The scattered 16-byte stores of k_scatter land as partial
// lines all over the partition runs (2x the written bytes at 4096 partitions, profiles/traffic_r02_c2.json).  Here a
// tile goes through in rounds of RR records: each round's compact records are sorted by partition in LDS and every
// partition's piece is written as one contiguous run (consecutive lanes, consecutive addresses) behind the pieces of
// the earlier rounds.  Same layout as k_scatter (partition-major runs at the scan offsets, any order inside a run).
// A batch without compact records goes through k_scatter's body.
//
// RSV (dense regions, single pass): no histogram and no scan before it.  Partition p's run is [p * rcap, p * rcap +
// rsv[p]) and a round reserves its piece of every partition with one global atomic on rsv[p].  A record without a
// compact form or a run longer than rcap sets rsv[P] (RSV_OVER): then the batch goes through classify, scan and the
// offset scatter after all (those kernels are gated on rsv[P] and return at once without it).  The error and late
// counts wait in rsv until the gated classify adds them to the status (RSV_* slots), so a redone batch counts once.
template <int MODE, int RR, bool RSV, bool NW = false>
__device__ __forceinline__ void scatter_staged_body(DevCfg c, int64_t wm, const int64_t* __restrict__ key,
                                                    const int64_t* __restrict__ ts, const int64_t* __restrict__ val,
                                                    const int32_t* __restrict__ kh, int64_t n, int32_t T,
                                                    const uint32_t* __restrict__ offs, PRec* __restrict__ part,
                                                    DevSide side, Status* st, uint32_t* rsv, int64_t rcap) {
  specialize<MODE>(c);
  extern __shared__ __attribute__((aligned(16))) uint8_t sraw[];
  // RR: the round's records sorted by partition (NW: narrow 8-byte records)
  i64x2* stg = reinterpret_cast<i64x2*>(sraw);
  uint64_t* stg8 = reinterpret_cast<uint64_t*>(sraw);
  uint16_t* sp = reinterpret_cast<uint16_t*>(sraw + (size_t)RR * (NW ? 8 : 16));  // RR: their partitions
  uint32_t* gb = reinterpret_cast<uint32_t*>(sp + RR);   // P: next free slot of each partition's run
  uint32_t* cs = gb + c.P;                               // P + 1: the round's counts, then their starts in stg
  uint32_t* wsum = cs + c.P + 1;                         // block scan
  const int32_t tile = tile_of_block(T);
  if constexpr (!RSV) {
    const bool cmp = c.compact && !*c.wide;  // (uniform: every classify workgroup has finished)
    if (!cmp) {
      scatter_direct(c, wm, key, ts, val, kh, n, T, offs, part, side, st, gb, tile);
      return;
    }
    for (int i = threadIdx.x; i < c.P; i += FW_TILE_THREADS) gb[i] = offs[(int64_t)i * T + tile];
  }
  const int64_t tbase = (int64_t)tile * FW_TILE;
  const int64_t tend = min(n, tbase + (int64_t)FW_TILE);
  unsigned long long late = 0;
  int bad_kg = 0, bad_ts = 0, over = 0, nmiss = 0;
  constexpr int RPT = RR / FW_TILE_THREADS;
  const int ppt = (c.P + FW_TILE_THREADS - 1) / FW_TILE_THREADS;
  i64x2* out = reinterpret_cast<i64x2*>(part);
  uint64_t* out8 = reinterpret_cast<uint64_t*>(part);
  for (int64_t b = tbase; b < tend; b += RR) {
    for (int i = threadIdx.x; i <= c.P; i += FW_TILE_THREADS) cs[i] = 0;
    __syncthreads();
    // (two halves of RPT / 2 records: each half's loads in flight together, fewer registers than all at once)
    uint32_t rk[RPT];
    uint32_t pj[RPT];
    int64_t w[RPT], v[RPT];
#pragma unroll
    for (int hf = 0; hf < 2; hf++) {
      constexpr int H = RPT / 2;
      const int64_t bh = b + (int64_t)hf * H * FW_TILE_THREADS;
      int64_t k[H], t[H], vh[H];
      int32_t hh[H];
      load_records<H / 2, true>(c, key, ts, val, kh, bh, tend, k, t, vh, hh);
#pragma unroll
      for (int j = 0; j < H; j++) {
        const int jj = hf * H + j;
        const int64_t i = rec_index(bh, j >> 1, j & 1);
        pj[jj] = 0xffffffffu;
        v[jj] = vh[j];
        if (i >= tend) continue;
        const int32_t h = c.key_kind == FW_KEY_HASHED ? hh[j] : key_hash_of(c.key_kind, k[j], kh, i);
        const int32_t p = partition_of(c, k[j], h);
        if (p < 0) {
          bad_kg++;
          continue;
        }
        int64_t last = 0;
        int nwin = 0;
        const int cls = classify(c, wm, t[j], &last, &nwin, k[j], 0);
        if (cls == CLS_NORMAL) {
          const int64_t d = compact_delta(c, last);
          if (RSV && d < 0) {  // no compact form: the batch takes the offset path
            over = 1;
            continue;
          }
          if constexpr (NW) {
            uint64_t nw;
            if (!narrow_encode(c, k[j], d, vh[j], &nw)) {  // no narrow form: the offset path, with CRecs
              over = 1;
              nmiss = 1;
              continue;
            }
            w[jj] = (int64_t)nw;
          } else {
            w[jj] = compact_encode(c, k[j], d);
          }
          rk[jj] = atomicAdd(&cs[p], 1u);
          pj[jj] = (uint32_t)p;
        } else if (cls == CLS_LATE) {
          if (!RSV && c.side_output)
            side_one(side, st, k[j], t[j], vh[j]);
          else
            late++;
        } else if (cls == CLS_BADTS) {
          bad_ts++;
        }
      }
    }
    __syncthreads();
    // exclusive scan of the round's counts (ppt partitions per thread), cs[P] = the round's records
    constexpr int CQ = ((RSV ? FW_GMAX_P : FW_STAGED_MAX_P) + FW_TILE_THREADS - 1) / FW_TILE_THREADS;
    uint32_t cq[CQ], sum = 0;
#pragma unroll
    for (int q = 0; q < CQ; q++) {
      const int pp = threadIdx.x * ppt + q;
      cq[q] = q < ppt && pp < c.P ? cs[pp] : 0u;
      sum += cq[q];
    }
    uint32_t total;
    uint32_t e = block_excl_scan(sum, wsum, &total);
#pragma unroll
    for (int q = 0; q < CQ; q++) {
      const int pp = threadIdx.x * ppt + q;
      if (q < ppt && pp < c.P) cs[pp] = e;
      e += cq[q];
    }
    if (threadIdx.x == 0) cs[c.P] = total;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RPT; j++) {
      if (pj[j] == 0xffffffffu) continue;
      const uint32_t pos = cs[pj[j]] + rk[j];
      if constexpr (NW)
        stg8[pos] = (uint64_t)w[j];
      else
        stg[pos] = i64x2{w[j], v[j]};
      sp[pos] = (uint16_t)pj[j];
    }
    if constexpr (RSV) {  // this round's piece of every partition it has records for
      for (int i = threadIdx.x; i < c.P; i += FW_TILE_THREADS) {
        const uint32_t m = cs[i + 1] - cs[i];
        if (m == 0) continue;
        const uint32_t g = atomicAdd(&rsv[i], m);
        if ((int64_t)g + m > rcap) {
          over = 1;
          gb[i] = 0xffffffffu;
        } else {
          gb[i] = (uint32_t)((int64_t)i * rcap + g);
        }
      }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < total; i += FW_TILE_THREADS) {
      const uint32_t pp = sp[i];
      if (RSV && gb[pp] == 0xffffffffu) continue;
      if constexpr (NW)
        out8[gb[pp] + (i - cs[pp])] = stg8[i];
      else
        out[gb[pp] + (i - cs[pp])] = stg[i];
    }
    __syncthreads();
    if constexpr (!RSV) {
      for (int i = threadIdx.x; i < c.P; i += FW_TILE_THREADS) gb[i] += cs[i + 1] - cs[i];
      __syncthreads();
    }
  }
  if constexpr (RSV) {
    if (over) rsv[c.P + RSV_OVER] = 1;
    if (NW && nmiss) rsv[c.P + FW_RSV_NARROW] = 1;
    if (bad_kg) atomicAdd(&rsv[c.P + RSV_KG], (uint32_t)bad_kg);
    if (bad_ts) atomicAdd(&rsv[c.P + RSV_TS], (uint32_t)bad_ts);
    if (late) atomicAdd(reinterpret_cast<unsigned long long*>(rsv + c.P + RSV_LATE), late);
  } else if (late) {
    atomicAdd(&st->late_dropped, late);
  }
}
// the offset form (gate: the single pass's RSV_OVER word, the batch comes here only when it is set; nullptr = always)
template <int MODE, int RR>
__global__ __launch_bounds__(FW_TILE_THREADS) void k_scatter_staged(DevCfg c, int64_t wm, const int64_t* __restrict__ key,
                                                                   const int64_t* __restrict__ ts,
                                                                   const int64_t* __restrict__ val,
                                                                   const int32_t* __restrict__ kh, int64_t n, int32_t T,
                                                                   const uint32_t* __restrict__ offs,
                                                                   PRec* __restrict__ part, DevSide side, Status* st,
                                                                   const uint32_t* __restrict__ gate) {
  if (gate && !gate[0]) return;  // (the batch went through the single pass)
  scatter_staged_body<MODE, RR, false>(c, wm, key, ts, val, kh, n, T, offs, part, side, st, nullptr, 0);
}
// the single pass (tumbling windows, dense regions); NW: narrow records, rcap in 8-byte records
template <int RR, bool NW>
__global__ __launch_bounds__(FW_TILE_THREADS) void k_scatter_rsv(DevCfg c, int64_t wm, const int64_t* __restrict__ key,
                                                                const int64_t* __restrict__ ts,
                                                                const int64_t* __restrict__ val,
                                                                const int32_t* __restrict__ kh, int64_t n, int32_t T,
                                                                PRec* __restrict__ part, uint32_t* rsv, int64_t rcap) {
  scatter_staged_body<M_TUMB, RR, true, NW>(c, wm, key, ts, val, kh, n, T, nullptr, part, DevSide{}, nullptr, rsv, rcap);
}

// ---- K2b: ordered compaction of the ordered-path records of a tile (skipped by tiles that have none).
// srow: the scanned ordered-path counts per tile, then the raw counts.  G: a gathered batch (tiles of
// FW_GTILE; a normal record without a compact form takes the ordered path, as k_stage decided)
template <bool G>
__global__ __launch_bounds__(FW_TILE_THREADS) void k_scatter_ordered(DevCfg c, int64_t wm, const int64_t* __restrict__ key,
                                                                     const int64_t* __restrict__ ts,
                                                                     const int64_t* __restrict__ val,
                                                                     const int32_t* __restrict__ kh, int64_t n,
                                                                     int32_t T, const uint32_t* __restrict__ srow,
                                                                     int64_t* __restrict__ sk, int64_t* __restrict__ stt,
                                                                     int64_t* __restrict__ sv, int32_t* __restrict__ skh, const Status* st) {
  const uint32_t* tile_slow = srow + T;
  if (tile_slow[blockIdx.x] == 0) return;
  const int taint = c.assigner == FW_SESSION ? st->taint_any : 0;
  __shared__ uint32_t wtot[FW_TILE_THREADS / 64];
  const uint32_t slow_base = srow[blockIdx.x] - srow[0];
  constexpr int64_t TL = G ? FW_GTILE : FW_TILE;
  const int64_t tbase = (int64_t)blockIdx.x * TL;
  const int64_t tend = min(n, tbase + TL);
  const int lane = __lane_id(), wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t running = 0;
  for (int64_t j = tbase; j < tend; j += blockDim.x) {
    const int64_t i = j + threadIdx.x;
    int cls = CLS_SKIP;
    int32_t p = -1, h = 0;
    int64_t k = 0, t = 0, v = 0;
    if (i < tend) {
      k = key[i];
      t = ts[i];
      v = val[i];
      h = key_hash_of(c.key_kind, k, kh, i);
      p = partition_of(c, k, h);
      if (p >= 0) {
        int64_t last = 0;
        int nw = 0;
        cls = classify(c, wm, t, &last, &nw, k, taint);
        if (G && cls == CLS_NORMAL && compact_delta(c, last) < 0) cls = CLS_SLOW;
      }
    }
    const bool is_slow = cls == CLS_SLOW;
    const uint64_t ball = __ballot(is_slow);
    if (lane == 0) wtot[wid] = (uint32_t)__popcll(ball);
    __syncthreads();
    uint32_t woff = 0, tot = 0;
    for (int w = 0; w < nw; w++) {
      const uint32_t x = wtot[w];
      woff += w < wid ? x : 0u;
      tot += x;
    }
    if (is_slow) {
      const uint32_t pos = slow_base + running + woff + (uint32_t)__popcll(ball & lanemask_lt());
      sk[pos] = k;
      stt[pos] = t;
      sv[pos] = v;
      skh[pos] = h;
      if (agg_ordinal(c)) c.slow_ord[pos] = c.ord_base + i;
    }
    running += tot;
    __syncthreads();
  }
}

// ---- K2 (gathered batches): classify + tile-local partition sort.  A workgroup takes one tile of FW_GTILE
// records (8 per thread, in registers), ranks each normal record in its partition with an LDS counter, scans
// the counters into the tile's partition runs, places the records' compact form (CRec) in LDS at their run
// slots and writes the sorted tile back with whole-line stores.  rt[tile][p] = run start | count << 16 (the
// aggregate gathers partition p's runs from every tile); srow[tile] = srow[T8 + tile] = the tile's
// ordered-path records, among them the normal records without a compact form (their window is out of the
// batch's compact range).  Late records go to the side output / late counter here.
template <int MODE>
__global__ __launch_bounds__(FW_TILE_THREADS) void k_stage(DevCfg c, int64_t wm, const int64_t* __restrict__ key,
                                                           const int64_t* __restrict__ ts, const int64_t* __restrict__ val,
                                                           const int32_t* __restrict__ kh, int64_t n, int32_t T8,
                                                           i64x2* __restrict__ part, uint32_t* __restrict__ rt,
                                                           uint32_t* __restrict__ srow, DevSide side, Status* st) {
  specialize<MODE>(c);
  constexpr int R = FW_GTILE / FW_TILE_THREADS;  // records per thread (even: pairs)
  extern __shared__ __align__(16) uint8_t lds_raw[];
  i64x2* stg = reinterpret_cast<i64x2*>(lds_raw);                         // FW_GTILE records
  uint32_t* cnt = reinterpret_cast<uint32_t*>(stg + FW_GTILE);            // P run counters, then run starts
  __shared__ uint32_t wsum[FW_TILE_THREADS / 64 + 1];
  __shared__ uint32_t slow_s;
  for (int i = threadIdx.x; i < c.P; i += FW_TILE_THREADS) cnt[i] = 0;
  if (threadIdx.x == 0) slow_s = 0;
  __syncthreads();
  const int32_t tile = blockIdx.x;
  const int64_t tbase = (int64_t)tile * FW_GTILE;
  const int64_t tend = min(n, tbase + (int64_t)FW_GTILE);
  int64_t k[R], t[R], v[R];
  int32_t hh[R];
  load_records<R / 2, true>(c, key, ts, val, kh, tbase, tend, k, t, v, hh);
  uint32_t pr[R];  // partition << 16 | rank, or ~0u
  int64_t kw[R];
  unsigned slow = 0, bad_kg = 0, bad_ts = 0;
  unsigned long long late = 0;
#pragma unroll
  for (int j = 0; j < R; j++) {
    pr[j] = ~0u;
    kw[j] = 0;
    const int64_t i = rec_index(tbase, j >> 1, j & 1);
    if (i >= tend) continue;
    const int32_t h = c.key_kind == FW_KEY_HASHED ? hh[j] : key_hash_of(c.key_kind, k[j], kh, i);
    const int32_t p = partition_of(c, k[j], h);
    if (p < 0) {
      bad_kg++;
      continue;
    }
    int64_t last = 0;
    int nw = 0;
    const int cls = classify(c, wm, t[j], &last, &nw, k[j], 0);
    if (cls == CLS_NORMAL) {
      const int64_t d = compact_delta(c, last);
      if (d < 0) {
        slow++;  // no compact form: the ordered path takes it (k_scatter_ordered<true> decides the same)
      } else {
        kw[j] = compact_encode(c, k[j], d);
        pr[j] = ((uint32_t)p << 16) | atomicAdd(&cnt[p], 1u);
      }
    } else if (cls == CLS_SLOW) {
      slow++;
    } else if (cls == CLS_LATE) {
      if (c.side_output)
        side_one(side, st, k[j], t[j], v[j]);
      else
        late++;
    } else if (cls == CLS_BADTS) {
      bad_ts++;
    }
  }
  if (slow) atomicAdd(&slow_s, slow);
  __syncthreads();
  // exclusive scan of the run counters (P <= FW_GMAX_P: at most 2 per thread), in place into run starts
  constexpr int PPT = FW_GMAX_P / FW_TILE_THREADS;
  uint32_t a[PPT], tot = 0;
#pragma unroll
  for (int q = 0; q < PPT; q++) {
    const int pp = threadIdx.x * PPT + q;
    a[q] = pp < c.P ? cnt[pp] : 0u;
    tot += a[q];
  }
  uint32_t total;
  uint32_t ex = block_excl_scan(tot, wsum, &total);
#pragma unroll
  for (int q = 0; q < PPT; q++) {
    const int pp = threadIdx.x * PPT + q;
    if (pp < c.P) {
      cnt[pp] = ex;
      rt[(int64_t)tile * c.P + pp] = ex | (a[q] << 16);
    }
    ex += a[q];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < R; j++)
    if (pr[j] != ~0u) stg[cnt[pr[j] >> 16] + (pr[j] & 0xffffu)] = i64x2{kw[j], v[j]};
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < total; i += FW_TILE_THREADS) part[tbase + i] = stg[i];
  if (threadIdx.x == 0) {
    srow[tile] = slow_s;
    srow[T8 + tile] = slow_s;
  }
  if (late) atomicAdd(&st->late_dropped, late);
  if (bad_kg) atomicAdd(&st->kg_errors, (int)bad_kg);
  if (bad_ts) atomicAdd(&st->ts_errors, (int)bad_ts);
}
// the runs table [T8][P] -> [P][T8] through 64 x 64 LDS tiles; tot[p] += the runs' counts (the partitions'
// record counts, scanned afterwards into their virtual offsets)
__global__ __launch_bounds__(1024) void k_rt_transpose(const uint32_t* __restrict__ rt, uint32_t* __restrict__ rt_t,
                                                        int32_t T8, int32_t P, uint32_t* __restrict__ tot) {
  __shared__ uint32_t sq[64][65];
  const int32_t t0 = blockIdx.x * 64, p0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 16
  for (int r = ty; r < 64; r += 16) {
    const int32_t t = t0 + r, p = p0 + tx;
    sq[r][tx] = (t < T8 && p < P) ? rt[(int64_t)t * P + p] : 0u;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 16) {
    const int32_t p = p0 + r, t = t0 + tx;
    const uint32_t w = sq[tx][r];
    if (p < P && t < T8) rt_t[(int64_t)p * T8 + t] = w;
    uint32_t c = w >> 16;  // the row's counts over these 64 tiles
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (tx == 0 && p < P && c) atomicAdd(&tot[p], c);
  }
}

// A gathered batch's partition (k_stage): its records are runs in every tile.  The workgroup keeps the
// partition's row of the runs table in LDS: pre[t] = records of the partition in tiles < t, s0[t] = the run's
// start inside tile t; base = the partition's virtual offset (record indices are base + 0 .. base + count - 1).
struct GatherRuns {
  const uint32_t* pre;
  const uint16_t* s0;
  int32_t nt;
  int64_t base;
};
// the last tile t in [lo, hi] with pre[t] <= r
__device__ __forceinline__ int32_t gather_tile(const GatherRuns& g, uint32_t r, int32_t lo, int32_t hi) {
  while (lo < hi) {
    const int32_t mid = (lo + hi + 1) >> 1;
    if (g.pre[mid] <= r) lo = mid; else hi = mid - 1;
  }
  return lo;
}
// the CRec index of record i: the tile whose run holds it (the last t with pre[t] <= i - base), then the slot.
// A wave's lanes hold consecutive records: the wave first finds the tile of its first record (every lane reads
// the same LDS words), then each lane searches the next 64 tiles (runs average FW_GTILE / P records)
__device__ __forceinline__ int64_t gather_index(const GatherRuns& g, int64_t i) {
  const uint32_t r = (uint32_t)(i - g.base);
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)r);
  const int32_t t0 = gather_tile(g, r0 < r ? r0 : r, 0, g.nt - 1);
  int32_t lo = t0, hi = min(t0 + 63, g.nt - 1);
  if (g.pre[hi] <= r) {
    lo = hi;
    hi = g.nt - 1;
  }
  const int32_t t = gather_tile(g, r, lo, hi);
  return (int64_t)t * FW_GTILE + g.s0[t] + (r - g.pre[t]);
}
// ---- K2c (gathered batches): plan and regroup.  k_gplan (one workgroup): the partitions' counts -> their
// virtual offsets (exclusive scan, total at P), the regroup's chunks per partition (FW_REGROUP_CHUNK records
// each, at least one) -> cbase (exclusive scan, total at P), and the ordered-path row's scan (srow).
__global__ __launch_bounds__(FW_TILE_THREADS) void k_gplan(uint32_t* __restrict__ voffs, uint32_t* __restrict__ cbase,
                                                           int32_t P, uint32_t* __restrict__ srow, int32_t t8) {
  __shared__ uint32_t sw[FW_TILE_THREADS / 64 + 1];
  constexpr int PPT = FW_GMAX_P / FW_TILE_THREADS;
  static_assert(FW_GMAX_T <= FW_GMAX_P, "one scan width");
  uint32_t a[PPT], ch[PPT], sa = 0, sc = 0, ss[PPT], s_tot = 0;
#pragma unroll
  for (int q = 0; q < PPT; q++) {
    const int i = threadIdx.x * PPT + q;
    a[q] = i < P ? voffs[i] : 0u;
    ch[q] = i < P ? max(1u, (a[q] + FW_REGROUP_CHUNK - 1) / FW_REGROUP_CHUNK) : 0u;
    ss[q] = i < t8 ? srow[i] : 0u;
    sa += a[q];
    sc += ch[q];
    s_tot += ss[q];
  }
  uint32_t ta, tc, ts;
  uint32_t ea = block_excl_scan(sa, sw, &ta);
  uint32_t ec = block_excl_scan(sc, sw, &tc);
  uint32_t es = block_excl_scan(s_tot, sw, &ts);
#pragma unroll
  for (int q = 0; q < PPT; q++) {
    const int i = threadIdx.x * PPT + q;
    if (i < P) {
      voffs[i] = ea;
      cbase[i] = ec;
    }
    if (i < t8) srow[i] = es;
    ea += a[q];
    ec += ch[q];
    es += ss[q];
  }
  if (threadIdx.x == 0) {
    voffs[P] = ta;
    cbase[P] = tc;
  }
}
// One workgroup per chunk of a partition: copies the chunk's records out of the tiles' runs into the
// partition's contiguous run at its virtual offset (the partition-major layout every aggregate reads).
// Consecutive chunks (so consecutive partitions) run on one XCD (blocks b, b + 8, ... take consecutive
// ones): their runs sit side by side in each tile, so the gathered lines are read once through that L2.
__global__ __launch_bounds__(FW_REGROUP_THREADS) void k_regroup(const i64x2* __restrict__ src, i64x2* __restrict__ dst,
                                                               const uint32_t* __restrict__ rt_t, int32_t t8,
                                                               const uint32_t* __restrict__ voffs,
                                                               const uint32_t* __restrict__ cbase, int32_t P) {
  __shared__ uint32_t pre[FW_GMAX_T];
  __shared__ uint16_t s0[FW_GMAX_T];
  __shared__ uint32_t sw[FW_REGROUP_THREADS / 64 + 1];
  const uint32_t vb = (gridDim.x & 7) == 0 ? (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  if (vb >= cbase[P]) return;
  int32_t lo = 0, hi = P - 1;  // the last partition whose first chunk <= vb
  while (lo < hi) {
    const int32_t mid = (lo + hi + 1) >> 1;
    if (cbase[mid] <= vb) lo = mid; else hi = mid - 1;
  }
  const int32_t p = lo;
  const uint32_t total = voffs[p + 1] - voffs[p];
  const uint32_t cb = (vb - cbase[p]) * FW_REGROUP_CHUNK, ce = min(total, cb + FW_REGROUP_CHUNK);
  const uint32_t* row = rt_t + (int64_t)p * t8;
  constexpr int TPT = FW_GMAX_T / FW_REGROUP_THREADS;
  uint32_t cnt[TPT], tot = 0;
#pragma unroll
  for (int q = 0; q < TPT; q++) {
    const int t = threadIdx.x * TPT + q;
    const uint32_t w = t < t8 ? row[t] : 0u;
    if (t < t8) s0[t] = (uint16_t)(w & 0xffffu);
    cnt[q] = w >> 16;
    tot += cnt[q];
  }
  uint32_t all;
  uint32_t e = block_excl_scan(tot, sw, &all);
#pragma unroll
  for (int q = 0; q < TPT; q++) {
    const int t = threadIdx.x * TPT + q;
    if (t < t8) pre[t] = e;
    e += cnt[q];
  }
  __syncthreads();
  const GatherRuns g{pre, s0, t8, 0};
  i64x2* out = dst + voffs[p];
  constexpr int RR = 4;
  for (uint32_t b = cb; b < ce; b += FW_REGROUP_THREADS * RR) {
    i64x2 r[RR];
#pragma unroll
    for (int j = 0; j < RR; j++) {
      const uint32_t i = b + j * FW_REGROUP_THREADS + threadIdx.x;
      if (i < ce) r[j] = src[gather_index(g, i)];
    }
#pragma unroll
    for (int j = 0; j < RR; j++) {
      const uint32_t i = b + j * FW_REGROUP_THREADS + threadIdx.x;
      if (i < ce) out[i] = r[j];
    }
  }
}

// ---- K3: per-partition LDS pre-aggregation + flush into the HBM region.
// LDS table: FW_LDS_SLOTS slots in buckets of 4.  tag[] holds 0 = empty, 1 = being claimed, or a
// fingerprint >= 2 of (key, window); one ds_read_b128 checks a whole bucket, so a lookup is one
// LDS read for almost every record and the wave does not wait on a long probe tail.
constexpr int LDS_BUCKETS = FW_LDS_SLOTS / 4;
struct AggLds {
  uint32_t tag[FW_LDS_SLOTS];
  uint32_t cnt[FW_LDS_SLOTS];  // per LDS epoch: at most one batch of one partition, < 2^32
  i64x2 kv[FW_LDS_SLOTS];      // {key, window start}: one ds_read_b128 per comparison
  int64_t mn[FW_LDS_SLOTS];
  int64_t mx[FW_LDS_SLOTS];
  int64_t sum[FW_LDS_SLOTS];
  int32_t slot[FW_LDS_SLOTS];  // flush: the window's slot in the region, -1 if new
  int fill;
  int anyfail;
  int spill;   // split partition: deltas this chunk wrote
  int last;    // split partition: this workgroup finished the partition's last chunk
  int nnew;    // flush: windows of this LDS epoch not yet in the region
  int live;    // occupied slots of the region
  unsigned long long flushed;
  int64_t min_timer;
  int hl_lo, hl_take, hl_idx;  // block pool: this flush's accumulator blocks (free-stack slice, then pool tail)
  long long hl_bump;
  const int64_t* byv;          // MINBY / MAXBY: the batch's value column (DevCfg::by_val)
  int64_t byb;                 // MINBY / MAXBY: the batch's ordinal base
};
enum : uint32_t { LT_EMPTY = 0, LT_BUSY = 1 };

// LDS slot hash of (key, window start): 32-bit multiplies only (full-rate VALU), independent of
// the fmix64 bits that chose the partition.  Low bits pick the bucket, the rest is the fingerprint.
__device__ __forceinline__ uint32_t lds_hash(int64_t key, int64_t start) {
  const uint64_t uk = (uint64_t)key, us = (uint64_t)start;
  uint32_t h = (uint32_t)uk * 0x9E3779B1u ^ (uint32_t)(uk >> 32) * 0x85EBCA77u ^
               ((uint32_t)us ^ (uint32_t)(us >> 32)) * 0xC2B2AE3Du;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return h;
}
__device__ __forceinline__ uint32_t lds_fp(uint32_t h) { return (h >> 8) | 2u; }  // >= 2, never EMPTY/BUSY

// accumulate one value into LDS slot `target` with no-return LDS atomics (nothing waits on the LDS)
// (first = FW_AGG_FIRST: the max lane takes ~fo, fo = the record's arrival ordinal)
// MINBY / MAXBY in LDS: the slot's mx holds the batch index of the element it selects (-1: none yet), whose
// field is read back from the batch's value column (DevCfg::by_val, copied per push); an element replaces it
// with one 64-bit CAS when (its key, its index) is lexicographically smaller (lock-free: a failed CAS
// re-reads the winner and compares again).  The flush turns the index into (key, full ordinal).
__device__ __forceinline__ void lds_by(AggLds& L, int target, int agg, int vtype, int64_t key, int64_t idx) {
  int64_t cur = __hip_atomic_load(&L.mx[target], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (true) {
    if (cur >= 0 && !by_less(key, idx, by_key(agg, vtype, L.byv[cur]), cur)) return;
    const int64_t prev = atomicCAS((unsigned long long*)&L.mx[target], (unsigned long long)cur, (unsigned long long)idx);
    if (prev == cur) return;
    cur = prev;
  }
}
// first == LDS_CNT_ONLY: the count alone (HyperLogLog: its rows are the registers' estimate, the entry's count the
// only accumulator field they show)
constexpr int LDS_CNT_ONLY = -1;
__device__ __forceinline__ void lds_acc(AggLds& L, int target, int vtype, int64_t v, int64_t fo, int first) {
  if (first == LDS_CNT_ONLY) {
    atomicAdd(&L.cnt[target], 1u);
    return;
  }
  if (agg_by(first)) {
    atomicAdd(&L.cnt[target], 1u);
    lds_by(L, target, first, vtype, by_key(first, vtype, v), fo - L.byb);
    if (vtype == FW_VAL_F64)
      atomicAdd((double*)&L.sum[target], __longlong_as_double(v));
    else
      atomicAdd((unsigned long long*)&L.sum[target], (unsigned long long)v);
    return;
  }
  atomicAdd(&L.cnt[target], 1u);
  // min / max only fall / rise, so a read that the value does not pass needs no atomic
  const int64_t sv = vtype == FW_VAL_F64 ? f64_sortable(v) : v;
  const int64_t a = first ? mn_in(first, sv) : sv, b = first ? ~fo : sv;
  if (vtype == FW_VAL_F64)
    atomicAdd((double*)&L.sum[target], __longlong_as_double(v));
  else
    atomicAdd((unsigned long long*)&L.sum[target], (unsigned long long)v);
  if (a < *(volatile int64_t*)&L.mn[target]) atomicMin((long long*)&L.mn[target], (long long)a);
  if (b > *(volatile int64_t*)&L.mx[target]) atomicMax((long long*)&L.mx[target], (long long)b);
}

// take one of the FW_LDS_FILL_LIMIT slot tickets before claiming a slot: concurrent claims then
// cannot fill the table past the limit, so every probe chain ends at an EMPTY slot
__device__ __forceinline__ bool lds_reserve(AggLds& L) {
  if (__hip_atomic_load(&L.fill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= FW_LDS_FILL_LIMIT) return false;
  if (atomicAdd(&L.fill, 1) < FW_LDS_FILL_LIMIT) return true;
  atomicSub(&L.fill, 1);
  return false;
}

// merge a delta (an accumulator in Entry form) into LDS slot `target` (AggregateFunction.merge)
__device__ __forceinline__ void lds_acc_delta(AggLds& L, int target, int vtype, const Entry& d, int agg) {
  if (agg_by(agg)) {  // a chunk's delta of the same batch: (key, full ordinal)
    atomicAdd(&L.cnt[target], (uint32_t)d.cnt);
    lds_by(L, target, agg, vtype, d.mn, d.mx - L.byb);
    if (vtype == FW_VAL_F64)
      atomicAdd((double*)&L.sum[target], __longlong_as_double(d.sum));
    else
      atomicAdd((unsigned long long*)&L.sum[target], (unsigned long long)d.sum);
    return;
  }
  atomicAdd(&L.cnt[target], (uint32_t)d.cnt);
  if (vtype == FW_VAL_F64)
    atomicAdd((double*)&L.sum[target], __longlong_as_double(d.sum));
  else
    atomicAdd((unsigned long long*)&L.sum[target], (unsigned long long)d.sum);
  atomicMin((long long*)&L.mn[target], (long long)d.mn);
  atomicMax((long long*)&L.mx[target], (long long)d.mx);
}

// find or claim the LDS slot of (key, window start); -1 when the table is at its fill limit
// (the caller flushes and retries).  A lane that claims a slot publishes it inside the same loop
// iteration (CAS EMPTY -> BUSY, write the key, store the fingerprint), so lanes of its own wave that
// wait on the BUSY tag see the fingerprint on their next iteration.  LDS operations of one wave
// complete in order, so a reader that sees the fingerprint reads the key written before it.
__device__ __forceinline__ int lds_slot(AggLds& L, int64_t key, int64_t start) {
  const uint32_t h = lds_hash(key, start), fp = lds_fp(h);
  uint32_t b = h & (LDS_BUCKETS - 1);
  int target = -1;
  for (int guard = 0; guard < 4 * LDS_BUCKETS;) {
    asm volatile("" ::: "memory");  // re-read the bucket every iteration (it may be claimed meanwhile)
    const u32x4 t4 = *reinterpret_cast<const u32x4*>(&L.tag[b * 4]);
    // branch-free scan of the bucket: one fingerprint candidate (the first; a second candidate with
    // the same fingerprint is looked at on the next iteration), the first EMPTY slot, any BUSY slot
    const int cand = t4.x == fp ? 0 : t4.y == fp ? 1 : t4.z == fp ? 2 : t4.w == fp ? 3 : -1;
    const int empty = t4.x == LT_EMPTY ? 0 : t4.y == LT_EMPTY ? 1 : t4.z == LT_EMPTY ? 2 : t4.w == LT_EMPTY ? 3 : -1;
    const bool busy = t4.x == LT_BUSY || t4.y == LT_BUSY || t4.z == LT_BUSY || t4.w == LT_BUSY;
    if (cand >= 0) {
      asm volatile("" ::: "memory");
      const i64x2 kv = L.kv[b * 4 + cand];
      if (kv.x == key && kv.y == start) {
        target = (int)b * 4 + cand;
        break;
      }
      // fingerprint collision: compare the bucket's other candidates one by one
      bool found = false;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t tq = q == 0 ? t4.x : q == 1 ? t4.y : q == 2 ? t4.z : t4.w;
        if (q > cand && tq == fp && !found) {
          const i64x2 kq = L.kv[b * 4 + q];
          if (kq.x == key && kq.y == start) {
            target = (int)b * 4 + q;
            found = true;
          }
        }
      }
      if (found) break;
    }
    if (busy) {  // a slot of this bucket is being published: re-read it
      guard++;
      continue;
    }
    if (empty >= 0) {
      if (!lds_reserve(L)) return -1;  // table full: flush first
      const int s = (int)b * 4 + empty;
      if (atomicCAS(&L.tag[s], LT_EMPTY, LT_BUSY) == LT_EMPTY) {
        L.kv[s] = i64x2{key, start};
        L.cnt[s] = 0;
        L.sum[s] = 0;
        L.mn[s] = LMAX;
        L.mx[s] = LMIN;
        __hip_atomic_store(&L.tag[s], fp, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        target = s;
        break;
      }
      atomicSub(&L.fill, 1);
      continue;  // lost the claim race: re-read the bucket
    }
    b = (b + 1) & (LDS_BUCKETS - 1);  // bucket full without a match
    guard++;
  }
  return target;
}
__device__ __forceinline__ bool lds_upsert(AggLds& L, int vtype, int64_t key, int64_t start, int64_t v,
                                           int diag = 0, int64_t fo = 0, int first = 0) {
  const int target = lds_slot(L, key, start);
  if (target < 0) return false;
  if (diag & DIAG_AGG_NO_ACCUM) return true;
  lds_acc(L, target, vtype, v, fo, first);
  return true;
}

// lds_acc (count / sum / min / max) of the lanes with ok set, each into its slot tg: when the whole wave runs and
// every such lane takes the same slot (a hot key's session), the wave sums its values first and one lane does the
// atomics -- sixty-four lanes' atomics on one LDS address otherwise serialise.  (A Double sum's order is not the
// arrival order either way; integer sums are exact.)
__device__ __forceinline__ void lds_acc_wave(AggLds& L, int tg, int vtype, int64_t v, bool ok, int first = 0) {
  const uint64_t okm = __ballot(ok);
  if ((first == 0 || first == LDS_CNT_ONLY) && __ballot(1) == ~0ull && __popcll(okm) >= 8) {
    const int lead = __ffsll((unsigned long long)okm) - 1;
    const int t0 = __shfl(tg, lead, 64);
    if (__ballot(ok && tg == t0) == okm) {
      if (first == LDS_CNT_ONLY) {  // (HyperLogLog: the registers are the accumulator, the slot keeps the count)
        if (__lane_id() == lead) atomicAdd(&L.cnt[t0], (uint32_t)__popcll(okm));
        return;
      }
      const bool f64 = vtype == FW_VAL_F64;
      const int64_t key = f64 ? f64_sortable(v) : v;
      int64_t mn = ok ? key : LMAX, mx = ok ? key : LMIN;
      double ds = ok && f64 ? __longlong_as_double(v) : 0.0;
      unsigned long long is = ok && !f64 ? (unsigned long long)v : 0ull;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, (int64_t)__shfl_xor((long long)mn, o, 64));
        mx = max(mx, (int64_t)__shfl_xor((long long)mx, o, 64));
        if (f64)
          ds += __shfl_xor(ds, o, 64);
        else
          is += (unsigned long long)__shfl_xor((long long)is, o, 64);
      }
      if (__lane_id() == lead) {
        atomicAdd(&L.cnt[t0], (uint32_t)__popcll(okm));
        if (f64)
          atomicAdd((double*)&L.sum[t0], ds);
        else
          atomicAdd((unsigned long long*)&L.sum[t0], is);
        if (mn < *(volatile int64_t*)&L.mn[t0]) atomicMin((long long*)&L.mn[t0], (long long)mn);
        if (mx > *(volatile int64_t*)&L.mx[t0]) atomicMax((long long*)&L.mx[t0], (long long)mx);
      }
      return;
    }
  }
  if (ok) lds_acc(L, tg, vtype, v, 0, first);
}
// One-window records (tumbling, panes), RPT per thread: every record's (key, window) is first looked up in
// its home bucket with all RPT lookups in flight together (tag bucket, then the candidate's key), and the
// hits accumulate at once; the rest (new windows, fingerprint collisions, buckets being claimed) go through
// lds_slot one by one.  dm: bit j = record j is accumulated (or absent); false when the table is full (the
// caller flushes and calls again with the same dm).
template <int RPT>
__device__ __forceinline__ bool lds_upsert_batch(AggLds& L, int vtype, const int64_t (&k)[RPT], const int64_t (&s)[RPT],
                                                 const int64_t (&v)[RPT], const int64_t (&o)[RPT], int first,
                                                 uint32_t& dm) {
  uint32_t b[RPT], fp[RPT];
  u32x4 t4[RPT];
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    const uint32_t h = lds_hash(k[j], s[j]);
    fp[j] = lds_fp(h);
    b[j] = h & (LDS_BUCKETS - 1);
    if (!(dm >> j & 1)) t4[j] = *reinterpret_cast<const u32x4*>(&L.tag[b[j] * 4]);
  }
  int cand[RPT];
  i64x2 kv[RPT];
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    cand[j] = -1;
    if (dm >> j & 1) continue;
    const u32x4 t = t4[j];
    cand[j] = t.x == fp[j] ? 0 : t.y == fp[j] ? 1 : t.z == fp[j] ? 2 : t.w == fp[j] ? 3 : -1;
    if (cand[j] >= 0) kv[j] = L.kv[b[j] * 4 + cand[j]];
  }
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    if (cand[j] < 0 || kv[j].x != k[j] || kv[j].y != s[j]) continue;
    lds_acc(L, (int)b[j] * 4 + cand[j], vtype, v[j], o[j], first);
    dm |= 1u << j;
  }
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    if (dm >> j & 1) continue;
    const int target = lds_slot(L, k[j], s[j]);
    if (target < 0) return false;
    lds_acc(L, target, vtype, v[j], o[j], first);
    dm |= 1u << j;
  }
  return true;
}

// the LDS delta of slot h as a region entry
__device__ __forceinline__ Entry lds_delta(const DevCfg& c, const AggLds& L, int h) {
  const i64x2 kv = L.kv[h];
  Entry d;
  d.key = kv.x;
  d.start = kv.y;
  d.end = wend(c, kv.y);
  d.cnt = (int64_t)L.cnt[h];
  d.sum = L.sum[h];
  d.mn = L.mn[h];
  d.mx = L.mx[h];
  if (agg_by(c.agg)) {  // the selected element: its key and full ordinal
    d.mn = by_key(c.agg, c.vtype, L.byv[d.mx]);
    d.mx += L.byb;
  }
  // a new pane belongs to the windows that end after the watermark, from its first window on
  d.meta = c.panes ? max(jsub(d.end, 1), c.nt_floor) : (int64_t)FW_TIMER;  // (+ HLL block: agg_flush)
  return d;
}

// merge every LDS window into the partition's HBM region, then reset the LDS table.
// Phase A locates each window in the region (read-only: its probe chain) and counts the new ones;
// if the region cannot take them within its load limit the flush changes nothing and returns false
// (the kernel suspends and resumes after the table grows).  Phase B then updates the found entries
// in place (plain read-modify-write: the workgroup owns the region) and claims EMPTY slots for the
// new ones.  (A front-to-back sweep of the region instead of probe chains measured slower at C2:
// its dependent loads per thread are longer than a probe chain at a region's load.)
// DIAG_AGG_TIMING clocks of the tumbling/sliding flush (thread 0): [0] flushes, [1] phase A, [2] phase B, [3] tail
__device__ unsigned long long g_flt[4];
__device__ __forceinline__ bool agg_flush(const DevCfg& c, AggLds& L, const Region& r, Status* st) {
  __syncthreads();
  const bool timing = FW_AGG_TIMING_BUILD && (c.diag & DIAG_AGG_TIMING);
  const unsigned long long tf0 = timing ? __builtin_amdgcn_s_memtime() : 0;
  if (c.diag & DIAG_AGG_NO_FLUSH) {
    for (int h = threadIdx.x; h < FW_LDS_SLOTS; h += blockDim.x) L.tag[h] = LT_EMPTY;
    if (threadIdx.x == 0) L.fill = 0;
    __syncthreads();
    return true;
  }
  // Phase A.  Each thread locates its FS LDS windows with every home slot's state word and entry
  // identity (key, start, end) loaded together, so the common cases at a region's load (the home slot
  // holds the window, or is EMPTY) cost one round trip for all of them; longer probe chains continue one
  // slot at a time.  (Phase B re-reads the entries it merges into from the L2.)
  constexpr int FS = FW_LDS_SLOTS / FW_AGG_THREADS;
  int nnew = 0;
  bool lv[FS];
  uint32_t hw[FS];
  i64x2 hks[FS];
  int64_t hend[FS];
#pragma unroll
  for (int q = 0; q < FS; q++) {
    const int h = threadIdx.x + q * FW_AGG_THREADS;
    lv[q] = L.tag[h] >= 2;
    if (lv[q]) {
      const i64x2 kv = L.kv[h];
      const uint32_t home = (uint32_t)slot_hash(c, kv.x, kv.y) & r.mask;
      hw[q] = ld_state_wg(r.state + home);
      hks[q] = *reinterpret_cast<const i64x2*>(&r.ent[home].key);
      hend[q] = r.ent[home].end;
    }
  }
#pragma unroll
  for (int q = 0; q < FS; q++) {
    if (!lv[q]) continue;
    const int h = threadIdx.x + q * FW_AGG_THREADS;
    const i64x2 kv = L.kv[h];
    const uint64_t hs = slot_hash(c, kv.x, kv.y);
    const int64_t we = wend(c, kv.y);
    int32_t slot = -1;
    if (hw[q] == live_word(hs) && hks[q].x == kv.x && hks[q].y == kv.y && hend[q] == we)
      slot = (int32_t)((uint32_t)hs & r.mask);
    else if (hw[q] != SLOT_EMPTY)  // the rest of the probe chain
      slot = region_find<true>(r, hs + 1, kv.x, kv.y, we, live_word(hs));
    L.slot[h] = slot;
    nnew += slot < 0;
  }
  if (nnew) atomicAdd(&L.nnew, nnew);
  __syncthreads();
  const unsigned long long tf1 = timing ? __builtin_amdgcn_s_memtime() : 0;
  const int32_t need = L.live + L.nnew;
  if (need > region_limit(c.log_r)) {
    if (threadIdx.x == 0) atomicMax(&st->need_live, need);
    return false;
  }
  if (c.pool_bytes) {  // one reservation of accumulator blocks for every new window of the flush
    if (threadIdx.x == 0) {
      const int k = L.nnew;
      int take = 0, lo = 0;
      long long bump = 0;
      if (k) {
        // pop k from the free stack (nothing is pushed while the aggregate runs); what the stack
        // lacks comes from the pool's tail
        const int t = atomicSub(&c.pool_ctr[0], k);
        take = max(0, min(t, k));
        lo = t - take;
        if (take < k) {
          atomicAdd(&c.pool_ctr[0], k - take);
          bump = atomicAdd(&c.pool_ctr[1], k - take);
          if (bump + (k - take) > c.pool_blocks) atomicOr(&st->flags, FW_STATUS_POOL);
        }
      }
      L.hl_lo = lo;
      L.hl_take = take;
      L.hl_bump = bump;
      L.hl_idx = 0;
    }
    __syncthreads();
  }
  int64_t mt = LMAX;
  unsigned long long nflush = 0;
  int lost = 0;
#pragma unroll
  for (int q = 0; q < FS; q++) {
    if (!lv[q]) continue;
    const int h = threadIdx.x + q * FW_AGG_THREADS;
    const Entry d = lds_delta(c, L, h);
    nflush++;
    mt = min(mt, c.panes ? d.meta : jsub(d.end, 1));
    const int32_t slot = L.slot[h];
    if (slot >= 0) {
      Entry cur = r.ent[slot];
      acc_merge(c, cur, d);
      if (c.panes)
        cur.meta = min(cur.meta, d.meta);
      else
        cur.meta |= FW_TIMER;
      r.ent[slot] = cur;
    } else {
      const uint64_t hs = slot_hash(c, d.key, d.start);
      const int32_t ns = region_claim<true>(r, hs, live_word(hs));
      if (ns >= 0) {
        Entry n = d;
        if (c.pool_bytes) {
          const int i = atomicAdd(&L.hl_idx, 1);
          int64_t blk = i < L.hl_take ? (int64_t)c.pool_free[L.hl_lo + i] : L.hl_bump + (i - L.hl_take);
          if (blk >= c.pool_blocks) blk = 0;  // pool exhausted: flagged above, the push fails
          n.meta |= blk << 1;
          if (c.agg == FW_AGG_TDIGEST)  // an empty digest
            *reinterpret_cast<TdHead*>(c.pool + (uint64_t)blk * (uint64_t)c.pool_bytes) = TdHead{0, 0, 0};
        }
        r.ent[ns] = n;
      } else {
        lost++;  // cannot happen below the load limit
      }
    }
  }
  if (lost) atomicOr(&st->flags, FW_STATUS_STATE_LOST);
  if (mt != LMAX) atomicMin((long long*)&L.min_timer, (long long)mt);
  if (nflush) atomicAdd(&L.flushed, nflush);
  __syncthreads();
  const unsigned long long tf2 = timing ? __builtin_amdgcn_s_memtime() : 0;
  for (int h = threadIdx.x; h < FW_LDS_SLOTS; h += blockDim.x) L.tag[h] = LT_EMPTY;
  if (threadIdx.x == 0) {
    L.fill = 0;
    L.live = need;
    L.nnew = 0;
  }
  __syncthreads();
  if (timing && threadIdx.x == 0) {
    atomicAdd(&g_flt[0], 1ull);
    atomicAdd(&g_flt[1], tf1 - tf0);
    atomicAdd(&g_flt[2], tf2 - tf1);
    atomicAdd(&g_flt[3], __builtin_amdgcn_s_memtime() - tf2);
  }
  return true;
}

// ---- sessions on the parallel path (EventTimeSessionWindows + MergingWindowSet.addWindow).
// Only in-time elements of untainted keys get here (classify), so nothing fires and no merge result
// is late: a key's in-flight sessions after the batch are the connected components
// (TimeWindow.intersects) of its sessions before the batch and the batch's element windows
// [ts, ts + gap), whatever the order of the elements, each with the merged accumulator of its parts.
// LDS: a slot holds one interval [start, end) of a key (the hull of the element windows that joined
// it, which is always connected) and its accumulator; `end` lives in the separate array E.  An element
// joins a slot of its key whose interval intersects its window and widens it with LDS min/max, or
// claims a new slot.  Slots of one key that come to overlap are joined by the flush.
__device__ __forceinline__ int lds_session_slot(AggLds& L, int64_t* E, int64_t key, int64_t ws, int64_t we) {
  const uint32_t h = lds_hash(key, 0), fp = lds_fp(h);
  uint32_t b = h & (LDS_BUCKETS - 1);
  int target = -1;
  for (int guard = 0; guard < 4 * LDS_BUCKETS;) {
    asm volatile("" ::: "memory");  // re-read the bucket every iteration (it may be claimed meanwhile)
    const u32x4 t4 = *reinterpret_cast<const u32x4*>(&L.tag[b * 4]);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t tq = q == 0 ? t4.x : q == 1 ? t4.y : q == 2 ? t4.z : t4.w;
      if (target < 0 && tq == fp) {
        const int s = (int)b * 4 + q;
        const i64x2 kv = L.kv[s];
        if (kv.x == key && kv.y <= we && E[s] >= ws) target = s;  // TimeWindow.intersects
      }
    }
    if (target >= 0) break;
    const int empty = t4.x == LT_EMPTY ? 0 : t4.y == LT_EMPTY ? 1 : t4.z == LT_EMPTY ? 2 : t4.w == LT_EMPTY ? 3 : -1;
    const bool busy = t4.x == LT_BUSY || t4.y == LT_BUSY || t4.z == LT_BUSY || t4.w == LT_BUSY;
    if (busy) {
      guard++;
      continue;
    }
    if (empty >= 0) {
      if (!lds_reserve(L)) return -1;
      const int s = (int)b * 4 + empty;
      if (atomicCAS(&L.tag[s], LT_EMPTY, LT_BUSY) == LT_EMPTY) {
        L.kv[s] = i64x2{key, ws};
        E[s] = we;
        L.cnt[s] = 0;
        L.sum[s] = 0;
        L.mn[s] = LMAX;
        L.mx[s] = LMIN;
        __hip_atomic_store(&L.tag[s], fp, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        target = s;
        break;
      }
      atomicSub(&L.fill, 1);
      continue;
    }
    b = (b + 1) & (LDS_BUCKETS - 1);
    guard++;
  }
  if (target < 0) return -1;
  // TimeWindow.cover: an interval only widens, so a read that already covers [ws, we) needs no atomic (a hot key's
  // elements mostly fall inside its session)
  long long* st = reinterpret_cast<long long*>(&L.kv[target]) + 1;
  if (*(volatile long long*)st > (long long)ws) atomicMin(st, (long long)ws);
  if (*(volatile int64_t*)&E[target] < we) atomicMax((long long*)&E[target], (long long)we);
  return target;
}
__device__ __forceinline__ bool lds_session_upsert(AggLds& L, int64_t* E, int vtype, int64_t key, int64_t ws,
                                                   int64_t we, int64_t v, int64_t fo = 0, int first = 0) {
  const int target = lds_session_slot(L, E, key, ws, we);
  if (target < 0) return false;
  lds_acc(L, target, vtype, v, fo, first);
  return true;
}

// one accumulator block for a window the ordered path or the session flush creates (the protocol of agg_flush's reservation, k = 1)
__device__ __forceinline__ uint64_t pool_alloc_one(const DevCfg& c, Status* st) {
  const int t = atomicSub(&c.pool_ctr[0], 1);
  if (t >= 1) return (uint64_t)c.pool_free[t - 1];
  atomicAdd(&c.pool_ctr[0], 1);
  const long long bump = atomicAdd(&c.pool_ctr[1], 1);
  if (bump + 1 > c.pool_blocks) {
    atomicOr(&st->flags, FW_STATUS_POOL);
    return 0;
  }
  return (uint64_t)bump;
}
// AggregateFunction.merge of two HyperLogLog accumulators (register max, AbstractHeapMergingState.mergeNamespaces,
// AbstractHeapMergingState.java:67-93): src's marked chunks are raised into dst bytewise (dst's chunks marked), src is
// left zeroed and goes on the deferred free list.  One thread; the caller owns both blocks (the key's entries).
__device__ __forceinline__ uint32_t max_u8x4(uint32_t a, uint32_t b) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 32; k += 8) r |= max((a >> k) & 0xffu, (b >> k) & 0xffu) << k;
  return r;
}
__device__ void hll_merge_blocks(const DevCfg& c, uint64_t dst, uint64_t src) {
  const int p = c.hll_p;
  uint8_t* bs = c.pool + src * (uint64_t)c.pool_bytes;
  uint8_t* bd = c.pool + dst * (uint64_t)c.pool_bytes;
  uint32_t* ms = reinterpret_cast<uint32_t*>(bs);
  uint32_t* md = reinterpret_cast<uint32_t*>(bd);
  uint4* qs = reinterpret_cast<uint4*>(bs + hll_hdr_bytes(p));
  uint4* qd = reinterpret_cast<uint4*>(bd + hll_hdr_bytes(p));
  const int32_t nq = (int32_t)(((int64_t)1 << p) / 16), nw = (nq + 31) / 32;
  for (int32_t w = 0; w < nw; w++) {
    const uint32_t word0 = ms[w];
    uint32_t word = word0;
    while (word) {
      const int b = __ffs(word) - 1;
      word &= word - 1;
      const uint4 a = qs[w * 32 + b], d = qd[w * 32 + b];
      qd[w * 32 + b] = make_uint4(max_u8x4(a.x, d.x), max_u8x4(a.y, d.y), max_u8x4(a.z, d.z), max_u8x4(a.w, d.w));
      qs[w * 32 + b] = make_uint4(0, 0, 0, 0);
    }
    if (word0) {
      md[w] |= word0;
      ms[w] = 0u;
    }
  }
  __threadfence();  // (zeroed before its id can be handed out)
  c.pool_defer[atomicAdd(&c.pool_ctr[2], 1)] = (uint32_t)src;
}
__device__ void row_merge_blocks(const DevCfg& c, uint64_t dst, uint64_t src);
// AggregateFunction.merge of two accumulator blocks as sessions merge: HyperLogLog raises dst to the register max
// now; a t-digest logs the pair, and the push's compression merges the centroid lists (launch_tdigest)
__device__ __forceinline__ void pool_merge_blocks(const DevCfg& c, uint64_t dst, uint64_t src) {
  if (c.agg == FW_AGG_HLL) {
    hll_merge_blocks(c, dst, src);
  } else if (c.agg == FW_AGG_ROW) {
    row_merge_blocks(c, dst, src);
  } else if (c.agg == FW_AGG_TDIGEST) {
    const int i = atomicAdd(c.td_mctr, 1);
    c.td_mdst[i] = (uint32_t)dst;
    c.td_msrc[i] = (uint32_t)src;
  }
}

// ---- Table API group-window aggregates (FW_AGG_ROW; the definition is oracle/window_oracle.h's OR_AGG_ROW, after
// flink-table .../functions/aggfunctions/{Count,Sum,Min,Max,Avg}AggFunction.scala).  A window's block is one RowAcc
// per value column (fw_internal.h), zero = empty; every update is an atomic (the records of a window may be added by
// several workgroups: the per-record update kernel, the ordered path).
constexpr uint64_t ROW_SIGN = 0x8000000000000000ull;
__device__ __forceinline__ RowAcc* row_acc(const DevCfg& c, uint64_t blk) {
  return reinterpret_cast<RowAcc*>(c.pool + blk * (uint64_t)c.pool_bytes);
}
__device__ __forceinline__ bool row_float(const DevCfg& c, int j) {
  return c.row_ts[j] == FW_VAL_F64 || c.row_ts[j] == FW_VAL_F32;
}
// a value's order key (Double.compare order for a floating column, Scala's Ordering.Double / Float), and the min /
// max encodings whose identity is 0 under an unsigned max: max = key ^ sign, min = ~(key ^ sign)
__device__ __forceinline__ int64_t row_key(const DevCfg& c, int j, int64_t v) { return row_float(c, j) ? f64_sortable(v) : v; }
__device__ __forceinline__ uint64_t row_enc_max(int64_t k) { return (uint64_t)k ^ ROW_SIGN; }
__device__ __forceinline__ uint64_t row_enc_min(int64_t k) { return ~((uint64_t)k ^ ROW_SIGN); }
__device__ __forceinline__ int64_t row_dec_max(uint64_t e) { return (int64_t)(e ^ ROW_SIGN); }
__device__ __forceinline__ int64_t row_dec_min(uint64_t e) { return (int64_t)(~e ^ ROW_SIGN); }
// the exact 128-bit integral sum: the low word's carry out goes to the high word with the addend's sign extension
__device__ __forceinline__ void row_add128(RowAcc& a, unsigned long long lo, long long hi) {
  const unsigned long long old = atomicAdd(&a.lo, lo);
  const long long h = hi + (old + lo < old ? 1ll : 0ll);
  if (h) atomicAdd(reinterpret_cast<unsigned long long*>(&a.hi), (unsigned long long)h);
}
// AggregateFunction.add of record i (its index in the push) into block blk: every aggregate of every non-null column
__device__ void row_add(const DevCfg& c, uint64_t blk, int64_t i) {
  RowAcc* acc = row_acc(c, blk);
  const uint32_t nm = c.row_nulls ? (uint32_t)c.row_nulls[i] : 0u;
  for (int j = 0; j < c.row_nc; j++) {
    if ((nm >> j) & 1u) continue;
    const int64_t v = c.row_cols[(int64_t)j * c.row_stride + i];
    RowAcc& a = acc[j];
    atomicAdd(&a.nn, 1ull);
    if (row_float(c, j))
      atomicAdd(reinterpret_cast<double*>(&a.lo), __longlong_as_double(v));
    else
      row_add128(a, (unsigned long long)v, v < 0 ? -1ll : 0ll);
    const int64_t k = row_key(c, j, v);
    const uint64_t em = row_enc_min(k), ex = row_enc_max(k);
    if (em > a.mn) atomicMax(&a.mn, em);  // (a stale read is below the current value: skipping is exact)
    if (ex > a.mx) atomicMax(&a.mx, ex);
  }
}
__device__ __forceinline__ void row_clear(const DevCfg& c, uint64_t blk) {
  RowAcc* a = row_acc(c, blk);
  for (int j = 0; j < c.row_nc; j++) a[j] = RowAcc{0, 0, 0, 0, 0};
}
// AggregateFunction.merge of block src into dst (sessions, AbstractHeapMergingState.mergeNamespaces): counts and sums
// add, min / max take the extremes; src is zeroed and goes on the deferred free list.  One thread.
__device__ void row_merge_blocks(const DevCfg& c, uint64_t dst, uint64_t src) {
  RowAcc* d = row_acc(c, dst);
  RowAcc* sa = row_acc(c, src);
  for (int j = 0; j < c.row_nc; j++) {
    const RowAcc o = sa[j];
    if (o.nn) {
      atomicAdd(&d[j].nn, o.nn);
      if (row_float(c, j))
        atomicAdd(reinterpret_cast<double*>(&d[j].lo), __longlong_as_double((long long)o.lo));
      else
        row_add128(d[j], o.lo, o.hi);
      atomicMax(&d[j].mn, o.mn);
      atomicMax(&d[j].mx, o.mx);
    }
    sa[j] = RowAcc{0, 0, 0, 0, 0};
  }
  __threadfence();  // (zeroed before its id can be handed out)
  c.pool_defer[atomicAdd(&c.pool_ctr[2], 1)] = (uint32_t)src;
}
// |x| / d of a 128-bit two's-complement x (d >= 1), truncated toward zero: BigInteger.divide (AvgAggFunction
// .scala:160-166); the quotient of an average fits 64 bits
__device__ int64_t row_div128(unsigned long long lo, long long hi, unsigned long long d) {
  const bool neg = hi < 0;
  unsigned long long ul = lo, uh = (unsigned long long)hi;
  if (neg) {  // negate
    ul = ~ul + 1ull;
    uh = ~uh + (ul == 0ull ? 1ull : 0ull);
  }
  unsigned long long q = 0, r = uh % d;  // (uh / d is 0 for an average's magnitude)
  for (int b = 63; b >= 0; b--) {
    const bool top = (r >> 63) != 0;
    r = (r << 1) | ((ul >> b) & 1ull);
    if (top || r >= d) {
      r -= d;
      q |= 1ull << b;
    }
  }
  return neg ? -(int64_t)q : (int64_t)q;
}
__device__ __forceinline__ int64_t row_narrow(int t, int64_t v) {
  return t == FW_VAL_I32 ? (int64_t)(int32_t)v : t == FW_VAL_I16 ? (int64_t)(int16_t)v
       : t == FW_VAL_I8 ? (int64_t)(int8_t)v : v;
}
// getValue of aggregate s (oracle/window_oracle.cpp row_value): the value or NULL
__device__ int64_t row_value(const DevCfg& c, const RowAcc* acc, int64_t cnt, int s, bool* null) {
  const int fn = c.row_ts[8 + s] >> 8, j = c.row_ts[8 + s] & 0xff;
  *null = false;
  if (fn == FW_ROW_COUNT_STAR) return cnt;
  const RowAcc a = acc[j];
  if (fn == FW_ROW_COUNT) return (int64_t)a.nn;
  if (a.nn == 0) {
    *null = true;
    return 0;
  }
  const int t = c.row_ts[j];
  const double ds = __longlong_as_double((long long)a.lo);
  switch (fn) {
    case FW_ROW_SUM:
      if (t == FW_VAL_F32) return __double_as_longlong((double)(float)ds);
      return t == FW_VAL_F64 ? (int64_t)a.lo : row_narrow(t, (int64_t)a.lo);
    case FW_ROW_MIN: {
      const int64_t k = row_dec_min(a.mn);
      return row_float(c, j) ? f64_unsortable(k) : k;
    }
    case FW_ROW_MAX: {
      const int64_t k = row_dec_max(a.mx);
      return row_float(c, j) ? f64_unsortable(k) : k;
    }
    default:  // FW_ROW_AVG
      if (t == FW_VAL_F64) return __double_as_longlong(ds / (double)a.nn);
      if (t == FW_VAL_F32) return __double_as_longlong((double)(float)(ds / (double)a.nn));
      if (t == FW_VAL_I64) return row_div128(a.lo, a.hi, a.nn);
      return row_narrow(t, (int64_t)a.lo / (int64_t)a.nn);  // the Long sum / count (Java division), narrowed
  }
}
// a fired row's aggregates into the export buffer (out.dig: the NULL mask, then row_ns values); the block is freed
// when the window goes (rel: 1 + its free-stack slot, as td_finish)
__device__ void row_finish(const DevCfg& c, const DevRows& out, uint64_t row, int64_t stack_base) {
  const uint64_t tag = (uint64_t)out.sum[row];
  const uint64_t blk = tag & 0xffffffffull;
  const int64_t rel = (int64_t)(tag >> 32);
  const RowAcc* a = row_acc(c, blk);
  int64_t* d = out.dig + row * (1 + (int64_t)c.row_ns);
  uint32_t nm = 0;
  for (int q = 0; q < c.row_ns; q++) {
    bool nl;
    d[1 + q] = row_value(c, a, out.cnt[row], q, &nl);
    if (nl) nm |= 1u << q;
  }
  d[0] = (int64_t)nm;
  out.sum[row] = out.mn[row] = out.mx[row] = 0;
  if (rel) {
    row_clear(c, blk);
    __threadfence();
    c.pool_free[stack_base + rel - 1] = (uint32_t)blk;
  }
}
// a new window's accumulator block (an empty t-digest, or HyperLogLog's zero registers)
__device__ __forceinline__ uint64_t pool_new_block(const DevCfg& c, Status* st) {
  const uint64_t blk = pool_alloc_one(c, st);
  if (c.agg == FW_AGG_TDIGEST) *reinterpret_cast<TdHead*>(c.pool + blk * (uint64_t)c.pool_bytes) = TdHead{0, 0, 0};
  return blk;
}
// MergingWindowSet.addWindow (MergingWindowSet.java:156-225) of a session delta d (an interval with
// its accumulator) into the key's in-flight sessions of region r: d's connected component becomes one
// session (merge function + mergeNamespaces, WindowOperator.java:308-339,
// AbstractHeapMergingState.java:67-93; EventTimeTrigger.onMerge/onElement register maxTimestamp,
// which is after the watermark).  A key's in-flight sessions are pairwise disjoint and non-touching (any
// two that intersected were merged), so d's component is exactly the sessions that intersect d: one walk
// of the key's probe chain merges them into the first one met, whatever their number (no cap on a key's
// in-flight sessions).  Only the thread that owns d.key touches the key's entries; new slots are published
// BUSY -> LIVE because other threads walk the same probe chains.
// Returns the region slots newly taken; *timer = maxTimestamp of the resulting session.
// DIAG_AGG_TIMING clocks of the session flush (thread 0): [0] flushes, [1] linking, [2] adding, [3] tail
__device__ unsigned long long g_sess[4];
// The key's entries lie on its probe chain from its home slot up to the chain's first EMPTY slot, and no slot
// becomes EMPTY during the launch: an EMPTY home slot means the key has no session in the region.  So the home
// slot is claimed first, at once -- the usual case, a key's first session of the batch, takes one round trip.
// Returns the claimed home slot, or -1.
__device__ __forceinline__ int32_t session_claim_home(const DevCfg& c, const Region& r, int64_t key) {
  const uint32_t home = (uint32_t)slot_hash(c, key, 0) & r.mask;
  return cas_state_wg(r.state + home, SLOT_EMPTY, SLOT_BUSY) == SLOT_EMPTY ? (int32_t)home : -1;
}
// pre: the result of session_claim_home for d.key when the caller tried it (-1: the home is taken), -2 if not
__device__ __forceinline__ int session_add(const DevCfg& c, const Region& r, const Entry& d, int64_t* timer, Status* st,
                                           int32_t pre = -2) {
  const uint64_t h = slot_hash(c, d.key, 0);
  const uint32_t want = live_word(h);
  int32_t target = -1;
  Entry m;
  int32_t ns = pre == -2 ? session_claim_home(c, r, d.key) : pre;
  // otherwise the probe chain is read SW state words at a time, all in flight together (slots of other keys
  // claimed meanwhile by other threads do not matter here); only the key's candidates' entries are then read
  constexpr int SW = 16;
  bool end_seen = ns >= 0;
  uint32_t first_empty = 0;  // (the chain's first EMPTY slot when the scan ends there: where a claim starts)
  for (uint32_t i0 = 0; i0 <= r.mask && !end_seen; i0 += SW) {
    uint32_t w[SW];
#pragma unroll
    for (int u = 0; u < SW; u++) w[u] = ld_state_wg(r.state + (((uint32_t)h + i0 + u) & r.mask));
    uint32_t cand = 0;
#pragma unroll
    for (int u = 0; u < SW; u++) {
      if (end_seen) continue;
      if (w[u] == SLOT_EMPTY) {
        end_seen = true;
        first_empty = i0 + u;
      } else if (w[u] == want) {
        cand |= 1u << u;
      }
    }
    if (cand) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    while (cand) {
      // up to four candidates' (key, start, end) in flight together; only an intersecting one's entry is read whole
      constexpr int CQ = 4;
      uint32_t cs[CQ];
      i64x2 ckv[CQ];
      int64_t cend[CQ];
      int nc = 0;
#pragma unroll
      for (int q = 0; q < CQ; q++) {
        if (!cand) continue;
        const int u = __builtin_ctz(cand);
        cand &= cand - 1;
        cs[q] = ((uint32_t)h + i0 + u) & r.mask;
        ckv[q] = *reinterpret_cast<const i64x2*>(&r.ent[cs[q]].key);
        cend[q] = r.ent[cs[q]].end;
        nc = q + 1;
      }
#pragma unroll
      for (int q = 0; q < CQ; q++) {
      if (q >= nc) continue;
      const uint32_t s = cs[q];
      if (ckv[q].x != d.key || !(d.start <= cend[q] && d.end >= ckv[q].y)) continue;  // TimeWindow.intersects
      const Entry e = r.ent[s];
      if (target < 0) {
        target = (int32_t)s;
        m = e;
        continue;
      }
      acc_merge(c, m, e);
      if (c.pool_bytes) pool_merge_blocks(c, pool_block_of(m), pool_block_of(e));
      m.start = min(m.start, e.start);
      m.end = max(m.end, e.end);
      // the slot stays occupied (live counts occupied slots) until k_fire rebuilds the region
      st_state_wg(r.state + s, SLOT_DEAD);
      }
    }
  }
  if (target < 0) {  // a new session
    *timer = jsub(d.end, 1);
    if (ns < 0) ns = region_claim<true>(r, h + first_empty, SLOT_BUSY);
    if (ns < 0) {  // cannot happen below the load limit (checked by the flush)
      atomicOr(&st->flags, FW_STATUS_STATE_LOST);
      return 0;
    }
    Entry nd = d;
    if (c.pool_bytes) nd.meta |= (int64_t)(pool_new_block(c, st) << 1);  // (filled after the aggregate)
    r.ent[ns] = nd;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    st_state_wg(r.state + ns, want);
    return 1;
  }
  acc_merge(c, m, d);
  m.start = min(m.start, d.start);  // TimeWindow.cover
  m.end = max(m.end, d.end);
  m.meta = c.pool_bytes ? (m.meta | FW_TIMER) : FW_TIMER;  // (the block id stays above the timer bit)
  *timer = jsub(m.end, 1);
  r.ent[target] = m;
  return 0;
}

// A key without sessions in the region (its home slot just claimed by the flush) whose LDS intervals (the chain from
// `first` through L.slot) are pairwise disjoint: each interval is a new session.  The home slot takes the first, the
// next EMPTY slots of the key's probe chain the others -- their claims in flight together -- and all are published
// behind one fence (instead of a scan, a claim and a fence per interval).  Returns false, having done nothing, when
// two of the intervals intersect or there are more than 8.  The region slot of each interval is kept in its L.cnt.
template <class Delta>
__device__ bool session_fresh_chain(const DevCfg& c, const Region& r, AggLds& L, const int64_t* E, int first,
                                    int32_t home, Status* st, int& nnew, int64_t& mt, unsigned long long& nflush,
                                    Delta delta) {
  constexpr int CH = 8;
  auto next = [&](int j) { return (L.slot[j] & 0xffff) - 1; };
  int n = 0;
  for (int a = first; a >= 0; a = next(a)) {
    if (++n > CH) return false;
    const int64_t as = L.kv[a].y, ae = E[a];
    int m = n;
    for (int b = next(a); b >= 0 && m < CH; b = next(b), m++)
      if (as <= E[b] && ae >= L.kv[b].y) return false;  // TimeWindow.intersects
  }
  const uint32_t want = live_word(slot_hash(c, L.kv[first].x, 0));
  auto place = [&](int j, int32_t s) {
    Entry nd = delta(j);
    if (c.pool_bytes) nd.meta |= (int64_t)(pool_new_block(c, st) << 1);  // (filled after the aggregate)
    r.ent[s] = nd;
    L.cnt[j] = (uint32_t)s;
    mt = min(mt, jsub(nd.end, 1));
  };
  place(first, home);
  int j = next(first);
  constexpr int SW = 16;
  // the claims keep the key's entries before its chain's first EMPTY slot: a chunk's EMPTY slots are taken in order,
  // and when a claim loses a race the chunk is read again before any slot past it is taken
  for (uint32_t i0 = 1; j >= 0 && i0 <= r.mask;) {
    uint32_t w[SW];
#pragma unroll
    for (int u = 0; u < SW; u++) w[u] = ld_state_wg(r.state + (((uint32_t)home + i0 + u) & r.mask));
    int want_n = 0;
    for (int b = j; b >= 0; b = next(b)) want_n++;
    uint32_t take = 0;
    int k = 0;
#pragma unroll
    for (int u = 0; u < SW; u++)
      if (w[u] == SLOT_EMPTY && k < want_n && i0 + u <= r.mask) {
        take |= 1u << u;
        k++;
      }
    uint32_t got = 0;
#pragma unroll
    for (int u = 0; u < SW; u++)
      if ((take >> u) & 1u)
        if (cas_state_wg(r.state + (((uint32_t)home + i0 + u) & r.mask), SLOT_EMPTY, SLOT_BUSY) == SLOT_EMPTY) got |= 1u << u;
    const bool lost = got != take;
    while (got && j >= 0) {
      const int u = __builtin_ctz(got);
      got &= got - 1;
      place(j, (int32_t)(((uint32_t)home + i0 + u) & r.mask));
      j = next(j);
    }
    if (!lost) i0 += SW;
  }
  if (j >= 0) atomicOr(&st->flags, FW_STATUS_STATE_LOST);  // cannot happen below the load limit
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  for (int a = first; a >= 0; a = next(a)) {
    if (a == j) break;  // (the unplaced rest, after a lost claim)
    st_state_wg(r.state + L.cnt[a], want);
    nnew++;
    nflush++;
  }
  return true;
}

// flush of the session LDS table.  Every LDS slot takes at most one new region slot, so the load limit
// is checked up front (live + fill), before anything changes.  A key's slots lie in the buckets from
// its home bucket to the first one with an EMPTY slot (a bucket fills front to back and is passed only
// when full).  Pass 1 lists each key's slots on its first slot, which owns the key (L.slot: next slot + 1);
// pass 2 lets every owner add its key's slots one per step, so the lanes of a wave call session_add
// together instead of one after another.
__device__ __forceinline__ bool agg_flush_session(const DevCfg& c, AggLds& L, const int64_t* E, const Region& r,
                                                  Status* st) {
  __syncthreads();
  const bool timing = FW_AGG_TIMING_BUILD && (c.diag & DIAG_AGG_TIMING);
  const unsigned long long ts0 = timing ? __builtin_amdgcn_s_memtime() : 0;
  if (c.diag & DIAG_AGG_NO_FLUSH) {
    for (int h = threadIdx.x; h < FW_LDS_SLOTS; h += blockDim.x) L.tag[h] = LT_EMPTY;
    if (threadIdx.x == 0) L.fill = 0;
    __syncthreads();
    return true;
  }
  const int32_t need = L.live + L.fill;
  if (need > region_limit(c.log_r)) {
    if (threadIdx.x == 0) atomicMax(&st->need_live, need);
    return false;
  }
  // pass 1: every slot finds its key's owner (the key's first slot from its home bucket) and, unless it is the owner,
  // puts itself on the owner's list (L.slot: next + 1, 0 = the end).  The order of a key's slots on the list does not
  // matter: its intervals' merges commute.
  // The owners go on a dense list (s_own), so that the adds spread one owner per lane before any lane takes two.
  constexpr int FQ = (FW_LDS_SLOTS + FW_AGG_THREADS - 1) / FW_AGG_THREADS;
  __shared__ uint16_t s_own[FW_LDS_SLOTS];
  __shared__ int s_nown;
  for (int h = threadIdx.x; h < FW_LDS_SLOTS; h += blockDim.x) L.slot[h] = 0;
  if (threadIdx.x == 0) s_nown = 0;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < FQ; q++) {
    const int h = threadIdx.x + q * (int)blockDim.x;
    if (h >= FW_LDS_SLOTS || L.tag[h] < 2) continue;
    const int64_t key = L.kv[h].x;
    const uint32_t hk = lds_hash(key, 0), fp = lds_fp(hk);
    int owner = h;
    bool found = false;
    for (uint32_t i = 0, b = hk & (LDS_BUCKETS - 1); i < LDS_BUCKETS && !found; i++, b = (b + 1) & (LDS_BUCKETS - 1)) {
      const u32x4 t4 = *reinterpret_cast<const u32x4*>(&L.tag[b * 4]);
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const uint32_t t = u == 0 ? t4.x : u == 1 ? t4.y : u == 2 ? t4.z : t4.w;
        if (!found && t == fp && L.kv[b * 4 + u].x == key) {
          owner = (int)b * 4 + u;
          found = true;
        }
      }
    }
    if (owner == h)
      s_own[atomicAdd(&s_nown, 1)] = (uint16_t)h;
    else
      L.slot[h] = atomicExch(&L.slot[owner], h + 1);
  }
  __syncthreads();
  const int nown = s_nown;
  const unsigned long long ts1 = timing ? __builtin_amdgcn_s_memtime() : 0;
  int nnew = 0;
  int64_t mt = LMAX;
  unsigned long long nflush = 0;
  auto delta = [&](int j) {
    const i64x2 kv = L.kv[j];
    Entry d;
    d.key = kv.x;
    d.start = kv.y;
    d.end = E[j];
    d.cnt = (int64_t)L.cnt[j];
    d.sum = L.sum[j];
    d.mn = L.mn[j];
    d.mx = L.mx[j];
    if (agg_by(c.agg)) {  // the selected element: its key and full ordinal
      d.mn = by_key(c.agg, c.vtype, L.byv[d.mx]);
      d.mx += L.byb;
    }
    d.meta = FW_TIMER;
    return d;
  };
  // this thread's owner slots: their home slots claimed together (the claims in flight at once); a claimed key
  // with one interval is a new session, written and published with one fence for all of them
  int32_t pre[FQ];
  bool pub[FQ];
  int oh[FQ];  // this thread's owners' slots
#pragma unroll
  for (int q = 0; q < FQ; q++) {
    const int oi = threadIdx.x + q * (int)blockDim.x;
    oh[q] = oi < nown ? (int)s_own[oi] : -1;
    pre[q] = oh[q] >= 0 ? session_claim_home(c, r, L.kv[oh[q]].x) : -3;
  }
  bool anypub = false;
#pragma unroll
  for (int q = 0; q < FQ; q++) {
    const int h = oh[q];
    pub[q] = pre[q] >= 0 && (L.slot[h] & 0xffff) == 0;
    if (!pub[q]) continue;
    Entry nd = delta(h);
    if (c.pool_bytes) nd.meta |= (int64_t)(pool_new_block(c, st) << 1);  // (filled after the aggregate)
    r.ent[pre[q]] = nd;
    mt = min(mt, jsub(nd.end, 1));
    nnew++;
    nflush++;
    anypub = true;
  }
  if (anypub) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
#pragma unroll
  for (int q = 0; q < FQ; q++) {
    if (pub[q])
      st_state_wg(r.state + pre[q], live_word(slot_hash(c, L.kv[oh[q]].x, 0)));
  }
#pragma unroll
  for (int q = 0; q < FQ; q++) {
    if (pre[q] == -3 || pub[q]) continue;
    int j = oh[q];
    int32_t pq = pre[q];
#ifndef FW_SESS_FRESH
#define FW_SESS_FRESH 1
#endif
    if (FW_SESS_FRESH && pq >= 0 && session_fresh_chain(c, r, L, E, j, pq, st, nnew, mt, nflush, delta)) continue;
    while (j >= 0) {
      int64_t tm;
      nnew += session_add(c, r, delta(j), &tm, st, pq);
      pq = -1;  // (the key has a session now: its home slot is taken)
      mt = min(mt, tm);
      nflush++;
      j = (L.slot[j] & 0xffff) - 1;
#ifdef FW_SESS_DIAG_ONE
      if (FW_SESS_DIAG_ONE == 1) j = -1;
#endif
    }
  }
  const unsigned long long ts2 = timing ? __builtin_amdgcn_s_memtime() : 0;
  if (nnew) atomicAdd(&L.nnew, nnew);
  if (mt != LMAX) atomicMin((long long*)&L.min_timer, (long long)mt);
  if (nflush) atomicAdd(&L.flushed, nflush);
  __syncthreads();
  for (int h = threadIdx.x; h < FW_LDS_SLOTS; h += blockDim.x) L.tag[h] = LT_EMPTY;
  if (threadIdx.x == 0) {
    L.fill = 0;
    L.live += L.nnew;
    L.nnew = 0;
  }
  __syncthreads();
  if (timing && threadIdx.x == 0) {
    atomicAdd(&g_sess[0], 1ull);
    atomicAdd(&g_sess[1], ts1 - ts0);
    atomicAdd(&g_sess[2], ts2 - ts1);
    atomicAdd(&g_sess[3], __builtin_amdgcn_s_memtime() - ts2);
  }
  return true;
}

template <bool SESS>
__device__ __forceinline__ bool agg_flush_any(const DevCfg& c, AggLds& L, const int64_t* E, const Region& r,
                                              Status* st) {
  if constexpr (SESS)
    return agg_flush_session(c, L, E, r, st);
  else
    return agg_flush(c, L, r, st);
}

// write back what the workgroup learnt about its region (on completion and on suspension)
__device__ __forceinline__ void agg_publish(const DevCfg& c, AggLds& L, DevTable& tb, int32_t p, Status* st) {
  tb.live[p] = L.live;
  if (L.min_timer < tb.next_timer[p]) tb.next_timer[p] = L.min_timer;
  if (L.flushed) atomicAdd(&st->merged, L.flushed);
  if (L.live > (1 << c.log_r) / 2) st->need_grow = 1;
}

// ---- split partitions (hot keys, see AggHot).  Chunks per partition, for the scan that maps
// workgroups to (partition, chunk); a resumed launch keeps the plan of the launch it resumes.
__global__ void k_chunk_plan(DevCfg c, const uint32_t* __restrict__ offs, int32_t T, AggHot hot) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p > c.P) return;
  if (p == c.P) {
    hot.chunk_base[p] = 0;
    return;
  }
  const int64_t len = (int64_t)offs[(int64_t)(p + 1) * T] - offs[(int64_t)p * T];
  hot.chunk_base[p] = len > c.agg_chunk ? (uint32_t)((len + c.agg_chunk - 1) / c.agg_chunk) : 1u;
  hot.pdone[p] = 0;
}

// write the LDS entries of a chunk as deltas (Entry form, accumulators as in the LDS) and empty the table
template <bool SESS>
__device__ __forceinline__ void agg_spill(const DevCfg& c, AggLds& L, const int64_t* E, Entry* out) {
  __syncthreads();
  for (int h = threadIdx.x; h < FW_LDS_SLOTS; h += blockDim.x) {
    if (L.tag[h] < 2) continue;
    Entry d = lds_delta(c, L, h);
    if constexpr (SESS) d.end = E[h];
    out[atomicAdd(&L.spill, 1)] = d;
  }
  __syncthreads();
  for (int h = threadIdx.x; h < FW_LDS_SLOTS; h += blockDim.x) L.tag[h] = LT_EMPTY;
  if (threadIdx.x == 0) L.fill = 0;
  __syncthreads();
}

// One chunk of a split partition.  Phase 1 (every chunk): pre-aggregate the chunk's records, spilling
// the LDS table as deltas whenever it fills (no region access, so no suspension).  The workgroup that
// finishes the partition's last chunk (release/acquire through pdone) runs phase 2: it merges every
// chunk's deltas into the region with the LDS table and the usual flush, which may suspend; a resumed
// launch continues phase 2 in the partition's chunk-0 workgroup (prog.rb = delta round, prog.tp = delta
// of the round per thread).
// the LDS copy of partition p's row of the runs table (every thread of the workgroup calls it)
__device__ __forceinline__ void gather_prologue(const uint32_t* __restrict__ row, int32_t nt, uint32_t* pre,
                                                uint16_t* s0, uint32_t* sw) {
  constexpr int TPT = FW_GMAX_T / FW_AGG_THREADS;
  uint32_t cnt[TPT], tot = 0;
#pragma unroll
  for (int q = 0; q < TPT; q++) {
    const int t = threadIdx.x * TPT + q;
    const uint32_t w = t < nt ? row[t] : 0u;
    if (t < nt) s0[t] = (uint16_t)(w & 0xffffu);
    cnt[q] = w >> 16;
    tot += cnt[q];
  }
  uint32_t total;
  uint32_t e = block_excl_scan(tot, sw, &total);
#pragma unroll
  for (int q = 0; q < TPT; q++) {
    const int t = threadIdx.x * TPT + q;
    if (t < nt) pre[t] = e;
    e += cnt[q];
  }
  __syncthreads();
}
// record i of a partition run: the raw 32 bytes of a PRec, or the 16 bytes of a CRec (cmp), loaded as
// 16-byte halves, then unpacked once every record of the round is in flight
__device__ __forceinline__ void load_prec_raw(bool cmp, const PRec* part, int64_t i, bool in, i64x2& a, i64x2& b,
                                              const GatherRuns* g = nullptr) {
  a = i64x2{0, 0};
  b = i64x2{0, 0};
  if (!in) return;
  if (g) {
    a = reinterpret_cast<const i64x2*>(part)[gather_index(*g, i)];
    return;
  }
  if (cmp) {
    a = reinterpret_cast<const i64x2*>(part)[i];
  } else {
    const i64x2* src = reinterpret_cast<const i64x2*>(part + i);
    a = src[0];
    b = src[1];
  }
}
// key, newest window start, value, window count and (FIRST) arrival ordinal of a record of partition p
template <bool FIRST>
__device__ __forceinline__ void unpack_prec(const DevCfg& c, bool cmp, int32_t p, const i64x2& a, const i64x2& b,
                                            int64_t& k, int64_t& t, int64_t& v, int& nw, int64_t& o) {
  if (cmp) {
    compact_decode(c, p, a.x, &k, &t);
    v = a.y;
    nw = 1;
    o = 0;
    return;
  }
  k = a.x;
  t = a.y;
  v = b.x;
  nw = FIRST ? (int)(b.y & 0xffff) : (int)b.y;
  o = FIRST ? c.ord_base + (int64_t)((uint64_t)b.y >> 16) : 0;
}

// LM: the run's record form, 0 = PRec, 1 = CRec, 2 = gathered CRec (GatherRuns).  Two register sets alternate
// without copies (copying the set in flight would wait for its loads), and the loads are branch-free, from an index
// clamped into the run (a load under a branch is waited for at once).
template <int RPT, bool SESS, bool FIRST, int LM>
__device__ __forceinline__ void agg_walk_lm(const DevCfg& c, AggLds& L, int64_t* E, const PRec* __restrict__ part,
                                            int32_t p, int64_t end, int64_t RS, int64_t& myrb, uint32_t& dm,
                                            const GatherRuns* g) {
  if (myrb >= end) return;
  auto load = [&](i64x2 (&a)[RPT], i64x2 (&b)[RPT], int64_t r0) {
#pragma unroll
    for (int j = 0; j < RPT; j++) {
      const int64_t i = r0 + (int64_t)j * blockDim.x + threadIdx.x;
      if constexpr (LM == 2) {
        load_prec_raw(true, part, i, i < end, a[j], b[j], g);
      } else {
        const int64_t ic = i < end ? i : end - 1;
        if constexpr (LM == 1) {
          a[j] = reinterpret_cast<const i64x2*>(part)[ic];
          b[j] = i64x2{0, 0};
        } else {
          const i64x2* src = reinterpret_cast<const i64x2*>(part + ic);
          a[j] = src[0];
          b[j] = src[1];
        }
      }
    }
  };
  // one round's records into the LDS table; false (dm = the round's done mask, L.anyfail set) when it is full
  auto round = [&](const i64x2 (&ca)[RPT], const i64x2 (&cb)[RPT], int64_t r0) -> bool {
    int64_t k[RPT], t[RPT], v[RPT], o[RPT];
    int nw[RPT];
#pragma unroll
    for (int j = 0; j < RPT; j++) unpack_prec<FIRST>(c, LM != 0, p, ca[j], cb[j], k[j], t[j], v[j], nw[j], o[j]);
    uint32_t m = dm;
#pragma unroll
    for (int j = 0; j < RPT; j++)
      if (r0 + (int64_t)j * blockDim.x + threadIdx.x >= end) m |= 1u << j;
    bool up = true;
    if (c.diag & DIAG_AGG_NO_LDS) {
#pragma unroll
      for (int j = 0; j < RPT; j++) asm volatile("" ::"v"(k[j]), "v"(t[j]), "v"(v[j]), "v"(o[j]));
    } else if constexpr (SESS) {
#pragma unroll
      for (int j = 0; j < RPT; j++) {
        const bool act = up && !(m >> j & 1);
        const int tg = act ? lds_session_slot(L, E, k[j], t[j], jadd(t[j], c.gap)) : -1;
        if (act && tg < 0) up = false;
        if constexpr (FIRST) {
          if (tg >= 0) lds_acc(L, tg, c.vtype, v[j], o[j], c.agg);
        } else {
          lds_acc_wave(L, tg, c.vtype, v[j], tg >= 0);  // (every lane of the wave takes part)
        }
        if (tg >= 0) m |= 1u << j;
      }
    } else {
      up = lds_upsert_batch<RPT>(L, c.vtype, k, t, v, o,
                                 FIRST ? c.agg : (c.agg == FW_AGG_HLL || c.agg == FW_AGG_ROW) ? LDS_CNT_ONLY : 0, m);
    }
    if (!up) {
      dm = m;
      __hip_atomic_store(&L.anyfail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return up;
  };
  i64x2 ca[RPT], cb[RPT], na[RPT], nb[RPT];
  load(ca, cb, myrb);
  for (;;) {
    load(na, nb, myrb + RS);
    if (!round(ca, cb, myrb)) break;
    dm = 0;
    myrb += RS;
    if (myrb >= end) break;
    load(ca, cb, myrb + RS);
    if (!round(na, nb, myrb)) break;
    dm = 0;
    myrb += RS;
    if (myrb >= end) break;
  }
}
// The free-running record walk of a one-window (or session) partition run [.., end): this thread's rounds from
// myrb on (dm: the done mask of its first round), with the next round's records in flight while the current
// ones are upserted, until its rounds are done or its upsert found the LDS table full (L.anyfail; the failing
// round and mask stay in myrb / dm; the other waves go on until they finish or fail too).  The caller meets the
// other waves at a barrier, flushes or spills the table when L.anyfail is set, and calls again.
template <int RPT, bool SESS, bool FIRST>
__device__ __forceinline__ void agg_walk(const DevCfg& c, AggLds& L, int64_t* E, const PRec* __restrict__ part, bool cmp,
                                         int32_t p, int64_t end, int64_t RS, int64_t& myrb, uint32_t& dm,
                                         const GatherRuns* g) {
  if (g)
    agg_walk_lm<RPT, SESS, FIRST, 2>(c, L, E, part, p, end, RS, myrb, dm, g);
  else if (cmp)
    agg_walk_lm<RPT, SESS, FIRST, 1>(c, L, E, part, p, end, RS, myrb, dm, g);
  else
    agg_walk_lm<RPT, SESS, FIRST, 0>(c, L, E, part, p, end, RS, myrb, dm, g);
}

template <int RPT, bool SESS, bool FIRST>
__device__ __forceinline__ void agg_split(const DevCfg& c, AggLds& L, int64_t* E, const PRec* __restrict__ part, int64_t begin,
                          int64_t end, int32_t p, int32_t ch, int32_t nch, DevTable& tb, const AggProg& prog,
                          int resume, const AggHot& hot, Status* st, const GatherRuns* g) {
  const int32_t c0 = (int32_t)hot.chunk_base[p];
  if (resume && (ch != 0 || prog.done[p])) return;
  const bool cmp = g || (c.compact && !*c.wide);
  for (int h = threadIdx.x; h < FW_LDS_SLOTS; h += blockDim.x) L.tag[h] = LT_EMPTY;
  if (threadIdx.x == 0) {
    L.fill = 0;
    L.anyfail = 0;
    L.spill = 0;
    L.byv = c.by_val;
    L.byb = c.ord_base;
    L.last = 0;
  }
  __syncthreads();
  if (!resume) {
    const int64_t cb = begin + (int64_t)ch * c.agg_chunk, ce = min(end, cb + (int64_t)c.agg_chunk);
    int64_t myrb = cb;
    uint32_t dm = 0;
    for (;;) {  // free-running waves (agg_walk); the table is spilled as deltas whenever it fills
      agg_walk<RPT, SESS, FIRST>(c, L, E, part, cmp, p, ce, (int64_t)blockDim.x * RPT, myrb, dm, g);
      __syncthreads();
      const int need = L.anyfail;
      __syncthreads();
      if (!need) break;
      agg_spill<SESS>(c, L, E, hot.delta + cb);
      if (threadIdx.x == 0) L.anyfail = 0;
      __syncthreads();
    }
    agg_spill<SESS>(c, L, E, hot.delta + cb);
    if (threadIdx.x == 0) hot.nd[c0 + ch] = L.spill;
    __threadfence();  // release this chunk's deltas to the workgroup that merges them
    __syncthreads();
    if (threadIdx.x == 0) L.last = atomicAdd(&hot.pdone[p], 1u) == (uint32_t)(nch - 1);
    __syncthreads();
    if (!L.last) return;
    __threadfence();  // acquire the other chunks' deltas
  }
  // phase 2: merge the deltas of every chunk into the region
  int64_t srb = begin;
  int srj = 0;
  if (resume) {
    srb = prog.rb[p];
    srj = (int)(prog.tp[(int64_t)p * FW_AGG_THREADS + threadIdx.x] & 0xffu);
  }
  if (threadIdx.x == 0) {
    L.anyfail = 0;
    L.nnew = 0;
    L.byv = c.by_val;
    L.byb = c.ord_base;
    L.live = tb.live[p];
    L.flushed = 0;
    L.min_timer = LMAX;
  }
  __syncthreads();
  const Region r = region_of(c, tb, p, tb.cur[p]);
  bool ok = true, first = true;
  for (int32_t j = (int32_t)((srb - begin) / c.agg_chunk); j < nch && ok; j++) {
    const int64_t db = begin + (int64_t)j * c.agg_chunk, de = db + hot.nd[c0 + j];
    for (int64_t rb = max(db, srb); rb < de && ok; rb += (int64_t)blockDim.x * RPT) {
      Entry d[RPT];
#pragma unroll
      for (int q = 0; q < RPT; q++) {
        const int64_t i = rb + (int64_t)q * blockDim.x + threadIdx.x;
        if (i < de) d[q] = hot.delta[i];
      }
      int rj = first ? srj : 0;
      first = false;
      for (;;) {
        bool failed = false;
#pragma unroll
        for (int q = 0; q < RPT; q++) {
          if (failed || q < rj || rb + (int64_t)q * blockDim.x + threadIdx.x >= de) continue;
          int tg;
          if constexpr (SESS)
            tg = lds_session_slot(L, E, d[q].key, d[q].start, d[q].end);
          else
            tg = lds_slot(L, d[q].key, d[q].start);
          if (tg < 0) {
            failed = true;
            rj = q;
          } else {
            lds_acc_delta(L, tg, c.vtype, d[q], c.agg);
          }
        }
        if (failed)
          L.anyfail = 1;
        else
          rj = RPT;
        __syncthreads();
        const int need = L.anyfail;
        __syncthreads();
        if (!need) break;
        if (!agg_flush_any<SESS>(c, L, E, r, st)) {
          ok = false;
          break;
        }
        srb = rb;
        srj = rj;
        if (threadIdx.x == 0) L.anyfail = 0;
        __syncthreads();
      }
    }
  }
  if (ok) ok = agg_flush_any<SESS>(c, L, E, r, st);
  if (!ok) {
    prog.tp[(int64_t)p * FW_AGG_THREADS + threadIdx.x] = (uint32_t)srj;
    if (threadIdx.x == 0) {
      prog.rb[p] = srb;
      prog.done[p] = 0;
      atomicOr(&st->suspended, (int)FW_SUSP_AGG);
    }
  } else if (threadIdx.x == 0) {
    prog.done[p] = 1;
  }
  if (threadIdx.x == 0) agg_publish(c, L, tb, p, st);
}

// DIAG_AGG_TIMING: per-workgroup phase clocks (s_memtime), summed over the launch and printed by the
// last workgroup to finish: [0] record loop, [1] flushes, [2] whole workgroup, [3] finished workgroups
__device__ unsigned long long g_aggt[4];
__device__ unsigned long long g_occ[3];  // running, sum of running at starts, max running
__device__ unsigned long long g_loop[3];  // thread 0's record loop: load wait, LDS upsert, barriers
// POOL: the aggregate keeps a pool block per window (HLL, t-digest); without it the instantiation is
// compiled for count/sum/min/max (or the ordinal aggregates) alone, which keeps the pool's code out of its
// registers
// GATHER: a gathered batch (k_stage): offs = the partitions' virtual offsets (T = 1), rt_t = the runs table
// [P][t8]; consecutive partitions run on one XCD (blocks b, b + 8, ... take consecutive ones), so the runs that
// sit side by side in every tile are read through one L2.
template <int RPT, bool SESS, bool FIRST, bool POOL, bool GATHER = false>
__global__ __launch_bounds__(FW_AGG_THREADS, GATHER ? FW_GATHER_WAVES : SESS ? FW_SESS_WAVES : FW_AGG_WAVES) void k_aggregate(DevCfg c, int64_t wm, const PRec* __restrict__ part,
                                                              const uint32_t* __restrict__ offs, int32_t T, DevTable tb,
                                                              AggProg prog, int resume, Status* st, AggHot hot,
                                                              const uint32_t* __restrict__ rt_t, int32_t t8) {
  if constexpr (!POOL) {
    c.pool_bytes = 0;
    if (!FIRST) c.agg = FW_AGG_COUNT_SUM_MIN_MAX;
  }
  __shared__ AggLds L;
  __shared__ int64_t sess_end[SESS ? FW_LDS_SLOTS : 1];  // sessions: interval end of each LDS slot
  __shared__ uint32_t g_pre[GATHER ? FW_GMAX_T : 1];
  __shared__ uint16_t g_s0[GATHER ? FW_GMAX_T : 1];
  __shared__ uint32_t g_sw[GATHER ? FW_AGG_THREADS / 64 + 1 : 1];
  const int32_t vb = GATHER && (gridDim.x & 7) == 0 ? (int32_t)((blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3))
                                                    : (int32_t)blockIdx.x;
  int32_t p = vb;
  int32_t nch = 1, ch = 0;
  if (hot.chunk_base) {  // workgroup -> (partition, chunk): last partition whose first chunk <= vb
    if ((uint32_t)vb >= hot.chunk_base[c.P]) return;
    int32_t lo = 0, hi = c.P - 1;
    while (lo < hi) {
      const int32_t mid = (lo + hi + 1) >> 1;
      if (hot.chunk_base[mid] <= (uint32_t)vb)
        lo = mid;
      else
        hi = mid - 1;
    }
    p = lo;
    nch = (int32_t)(hot.chunk_base[p + 1] - hot.chunk_base[p]);
    ch = (int32_t)(vb - hot.chunk_base[p]);
  } else if (p >= c.P) {
    return;
  }
  GatherRuns gr{g_pre, g_s0, t8, 0};
  if constexpr (GATHER) {
    gr.base = offs[p];
    gather_prologue(rt_t + (int64_t)p * t8, t8, g_pre, g_s0, g_sw);
  }
  const GatherRuns* g = GATHER ? &gr : nullptr;
  if (nch > 1) {
    const int64_t b0 = offs[(int64_t)p * T], e0 = offs[(int64_t)(p + 1) * T];
    agg_split<RPT, SESS, FIRST>(c, L, sess_end, part, b0, e0, p, ch, nch, tb, prog, resume, hot, st, g);
    return;
  }
  if (resume && prog.done[p]) return;
  const bool cmp = GATHER || (c.compact && !*c.wide);
  const int64_t begin = offs[(int64_t)p * T], end = offs[(int64_t)(p + 1) * T];
  if (begin == end) {
    if (threadIdx.x == 0) prog.done[p] = 1;
    return;
  }
  // resume point: round start srb and this thread's (record, window) inside that round; it moves
  // forward after every flush that succeeds
  int64_t srb = begin;
  int srj = 0, srwi = 0;
  if (resume) {
    srb = prog.rb[p];
    const uint32_t tp = prog.tp[(int64_t)p * FW_AGG_THREADS + threadIdx.x];
    srj = (int)(tp & 0xffu);
    srwi = (int)(tp >> 8);
  }
  for (int h = threadIdx.x; h < FW_LDS_SLOTS; h += blockDim.x) L.tag[h] = LT_EMPTY;
  if (threadIdx.x == 0) {
    L.fill = 0;
    L.anyfail = 0;
    L.nnew = 0;
    L.byv = c.by_val;
    L.byb = c.ord_base;
    L.live = tb.live[p];
    L.flushed = 0;
    L.min_timer = LMAX;
  }
  __syncthreads();
  const Region r = region_of(c, tb, p, tb.cur[p]);
  bool ok = true, first = true;
  const bool onewin = c.wpr == 1 || c.panes;
  const bool timing = FW_AGG_TIMING_BUILD && (c.diag & DIAG_AGG_TIMING);
  unsigned long long tw0 = timing ? __builtin_amdgcn_s_memtime() : 0, tflush = 0;
  if (timing && threadIdx.x == 0) {  // concurrency: workgroups running when this one starts
    const unsigned long long run = atomicAdd(&g_occ[0], 1ull) + 1;
    atomicAdd(&g_occ[1], run);
    atomicMax(&g_occ[2], run);
  }
  unsigned long long t_ld = 0, t_up = 0, t_bar = 0, ts_a = 0;
  if (SESS || onewin) {
    // One window per record (tumbling, panes, session elements): the waves run free.  Each thread walks its rounds with the
    // next round's records in flight while it upserts the current ones, and meets the others at a barrier
    // only when some lane's upsert found the LDS table full (L.anyfail) or every wave is done; a full table
    // is flushed there and every thread continues from its own (round, done mask).  A suspension keeps each
    // thread's (round, mask) as of the last flush that succeeded (prog.tp: mask | round << 8).
    const int64_t RS = (int64_t)blockDim.x * RPT;
    int64_t myrb = resume ? begin + (int64_t)srwi * RS : begin;
    uint32_t dm = resume ? (uint32_t)srj : 0u;
    int64_t ck_rb = myrb;
    uint32_t ck_dm = dm;
    for (;;) {
      agg_walk<RPT, SESS, FIRST>(c, L, sess_end, part, cmp, p, end, RS, myrb, dm, g);
      __syncthreads();
      const int need = L.anyfail;
      __syncthreads();
      if (!need) break;  // every wave has walked all of its rounds
      if (!agg_flush_any<SESS>(c, L, sess_end, r, st)) {
        ok = false;
        break;
      }
      ck_rb = myrb;
      ck_dm = dm;
      if (threadIdx.x == 0) L.anyfail = 0;
      __syncthreads();
    }
    srb = begin;
    srj = (int)ck_dm;
    srwi = (int)((ck_rb - begin) / RS);
  } else
  for (int64_t rb = srb; rb < end && ok; rb += (int64_t)blockDim.x * RPT) {
    int64_t k[RPT], t[RPT], v[RPT], o[RPT];
    int nw[RPT];
    if (timing) ts_a = __builtin_amdgcn_s_memtime();
    {
      i64x2 ra[RPT], rbb[RPT];
#pragma unroll
      for (int j = 0; j < RPT; j++) {  // all loads in flight before any use
        const int64_t i = rb + (int64_t)j * blockDim.x + threadIdx.x;
        load_prec_raw(cmp, part, i, i < end, ra[j], rbb[j], g);
      }
      if (timing) {
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long x = __builtin_amdgcn_s_memtime();
        t_ld += x - ts_a;
        ts_a = x;
      }
      // t = newest window start (assigned by k_scatter); o = FW_AGG_FIRST: arrival ordinal
#pragma unroll
      for (int j = 0; j < RPT; j++) unpack_prec<FIRST>(c, cmp, p, ra[j], rbb[j], k[j], t[j], v[j], nw[j], o[j]);
    }
    if (c.diag & DIAG_AGG_NO_LDS) {
#pragma unroll
      for (int j = 0; j < RPT; j++) asm volatile("" ::"v"(k[j]), "v"(t[j]), "v"(v[j]), "v"(nw[j]));
      continue;
    }
    // progress (record rj, window rwi) survives a flush-and-retry when the LDS table fills up;
    // the record loop is unrolled so the register arrays are only indexed by constants
    int rj = first ? srj : 0, rwi = first ? srwi : 0;
    first = false;
    for (;;) {
      bool failed = false;
#pragma unroll
      for (int j = 0; j < RPT; j++) {
        if (failed || j < rj || rb + (int64_t)j * blockDim.x + threadIdx.x >= end) continue;
        for (int wi = j == rj ? rwi : 0; wi < nw[j]; wi++) {
          bool in;
          if constexpr (SESS)
            in = lds_session_upsert(L, sess_end, c.vtype, k[j], t[j], jadd(t[j], c.gap), v[j], o[j], FIRST ? c.agg : 0);
          else
            in = lds_upsert(L, c.vtype, k[j], jsub(t[j], (int64_t)wi * c.slide), v[j], c.diag, o[j],
                            FIRST ? c.agg : (c.agg == FW_AGG_HLL || c.agg == FW_AGG_ROW) ? LDS_CNT_ONLY : 0);
          if (!in) {
            failed = true;
            rj = j;
            rwi = wi;
            break;
          }
        }
      }
      if (failed)
        L.anyfail = 1;
      else
        rj = RPT;  // all done: a retry pass after another thread's flush skips every record
      if (timing) {
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long x = __builtin_amdgcn_s_memtime();
        t_up += x - ts_a;
        ts_a = x;
      }
      __syncthreads();
      const int need = L.anyfail;
      __syncthreads();
      if (timing) {
        const unsigned long long x = __builtin_amdgcn_s_memtime();
        t_bar += x - ts_a;
        ts_a = x;
      }
      if (!need) break;
      const unsigned long long tf0 = timing ? __builtin_amdgcn_s_memtime() : 0;
      const bool fl = agg_flush_any<SESS>(c, L, sess_end, r, st);
      if (timing) tflush += __builtin_amdgcn_s_memtime() - tf0;
      if (!fl) {
        ok = false;
        break;
      }
      srb = rb;
      srj = rj;
      srwi = rwi;
      if (threadIdx.x == 0) L.anyfail = 0;
      __syncthreads();
    }
  }
  const unsigned long long tl = timing ? __builtin_amdgcn_s_memtime() : 0;
  if (ok) ok = agg_flush_any<SESS>(c, L, sess_end, r, st);
  if (timing && threadIdx.x == 0) {
    const unsigned long long te = __builtin_amdgcn_s_memtime();
    atomicAdd(&g_aggt[0], tl - tw0 - tflush);
    atomicAdd(&g_aggt[1], tflush + (te - tl));
    atomicAdd(&g_aggt[2], te - tw0);
    atomicSub(&g_occ[0], 1ull);
    atomicAdd(&g_loop[0], t_ld);
    atomicAdd(&g_loop[1], t_up);
    atomicAdd(&g_loop[2], t_bar);
    if (atomicAdd(&g_aggt[3], 1ull) == (unsigned long long)c.P - 1) {  // (counts unsplit partitions only)
      __threadfence();
      const double n = (double)gridDim.x;
      printf("agg timing: per WG loop %.0f flush %.0f total %.0f clocks (%d WGs); running at start avg %.1f max %llu\n",
             g_aggt[0] / n, g_aggt[1] / n, g_aggt[2] / n, (int)gridDim.x, (double)g_occ[1] / (double)c.P, g_occ[2]);
      printf("loop (thread 0, per WG): load %.0f upsert %.0f barriers %.0f clocks\n", g_loop[0] / (double)c.P,
             g_loop[1] / (double)c.P, g_loop[2] / (double)c.P);
      g_occ[1] = g_occ[2] = 0;
      g_loop[0] = g_loop[1] = g_loop[2] = 0;
      if (SESS)
        printf("session flush (thread 0, per flush): %llu flushes, link %.0f, add %.0f, tail %.0f clocks\n",
               g_sess[0], (double)g_sess[1] / (g_sess[0] + 1), (double)g_sess[2] / (g_sess[0] + 1),
               (double)g_sess[3] / (g_sess[0] + 1));
      else
        printf("flush (thread 0, per flush): %llu flushes, phase A %.0f, phase B %.0f, tail %.0f clocks\n",
               g_flt[0], (double)g_flt[1] / (g_flt[0] + 1), (double)g_flt[2] / (g_flt[0] + 1),
               (double)g_flt[3] / (g_flt[0] + 1));
      g_flt[0] = g_flt[1] = g_flt[2] = g_flt[3] = 0;

      g_aggt[0] = g_aggt[1] = g_aggt[2] = g_aggt[3] = 0;
      g_sess[0] = g_sess[1] = g_sess[2] = g_sess[3] = 0;
    }
  }
  if (!ok) {  // suspend: everything up to the last successful flush is in the region
    prog.tp[(int64_t)p * FW_AGG_THREADS + threadIdx.x] = (uint32_t)srj | ((uint32_t)srwi << 8);
    if (threadIdx.x == 0) {
      prog.rb[p] = srb;
      prog.done[p] = 0;
      atomicOr(&st->suspended, (int)FW_SUSP_AGG);
    }
  } else if (threadIdx.x == 0) {
    prog.done[p] = 1;
  }
  if (threadIdx.x == 0) agg_publish(c, L, tb, p, st);
}

// ---- K_slow: ordered replay (one workgroup; one thread per key inside each chunk)
constexpr int SLOW_CHUNK = FW_SLOW_THREADS;

struct SlowCtx {
  DevCfg c;
  int64_t wm;
  DevTable tb;
  DevRows out;
  DevSide side;
  Status* st;
};

__device__ __forceinline__ void note_timer(const SlowCtx& x, int32_t p, const Entry& e) {
  atomicMin((long long*)&x.tb.next_timer[p], (long long)timer_of(e, x.c.lateness));
}
__device__ __forceinline__ void kill_slot(const SlowCtx& x, const Region& r, int32_t p, int32_t s) {
  // the slot stays occupied (tb.live counts occupied slots) until the region is rebuilt by k_fire
  __hip_atomic_store(r.state + s, SLOT_DEAD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// new entry: claim BUSY, write, publish LIVE with the fingerprint (readers never see a torn entry)
__device__ __forceinline__ int32_t new_slot(const SlowCtx& x, const Region& r, int32_t p, uint64_t h, const Entry& e) {
  const int32_t s = region_claim<true>(r, h, SLOT_BUSY);  // (k_slow: one workgroup)
  if (s < 0) {  // cannot happen: k_slow checked the region's room for the chunk
    atomicOr(&x.st->flags, FW_STATUS_STATE_LOST);
    return -1;
  }
  r.ent[s] = e;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __hip_atomic_store(r.state + s, live_word(h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int live = atomicAdd(&x.tb.live[p], 1) + 1;
  if (live > (1 << x.c.log_r) / 2) x.st->need_grow = 1;
  return s;
}

__device__ void hll_clear(const DevCfg& c, uint64_t blk);
__device__ void hll_estimate(const DevCfg& c, uint64_t blk, double* est, int64_t* zeros_out, int64_t* lo_out);
// HyperLogLog add of one item into block blk (k_hll_update's raise: CAS on the register's word while larger, the
// chunk marked when the register leaves zero)
__device__ __forceinline__ void hll_raise(const DevCfg& c, uint64_t blk, int64_t item) {
  const int p = c.hll_p;
  const uint64_t h = fmix64((uint64_t)item);
  const uint32_t j = (uint32_t)(h >> (64 - p));
  const uint32_t rank = (uint32_t)__clzll((long long)((h << p) | (1ull << (p - 1)))) + 1u;
  uint8_t* base = c.pool + blk * (uint64_t)c.pool_bytes;
  uint32_t* w = reinterpret_cast<uint32_t*>(base + hll_hdr_bytes(p) + (j & ~3u));
  const int sh = (int)(j & 3) * 8;
  uint32_t o = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (((o >> sh) & 0xffu) < rank) {
    const uint32_t nw = (o & ~(0xffu << sh)) | (rank << sh);
    if (__hip_atomic_compare_exchange_strong(w, &o, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
      if (((o >> sh) & 0xffu) == 0u) {
        const uint32_t ch = j >> 4;
        atomicOr(reinterpret_cast<uint32_t*>(base) + (ch >> 5), 1u << (ch & 31u));
      }
      break;
    }
  }
}

__device__ void td_late_row(const SlowCtx& x, const Entry& en, int32_t head);
__device__ void td_late_row_session(const SlowCtx& x, const Entry& en, int32_t head);
__device__ void td_purge(const DevCfg& c, uint32_t g, uint64_t blk);
constexpr int32_t TD_DROPPED = -3;  // td_olink of a value purged from the push's compression (td_purge)
// a window's chain of the push's values (t-digest under allowed lateness) is kept in Double.compare order of the
// values: link l (element l / wpr) goes before the first link of a larger value
__device__ __forceinline__ uint64_t td_key(int64_t bits);
__device__ __forceinline__ void td_chain_insert(const DevCfg& c, int32_t* head, int32_t l, int64_t v) {
  const uint64_t kx = td_key(v);
  int32_t* at = head;
  while (*at >= 0 && td_key(c.td_ovv[*at / c.wpr]) < kx) at = &c.td_olink[*at];
  c.td_olink[l] = *at;
  *at = l;
}

// WindowOperator.processElement, non-merging branch (WindowOperator.java:371-407)
__device__ void replay_time_windows(const SlowCtx& x, int32_t p, int64_t k, int64_t t, int64_t v, int64_t fo, bool* skipped) {
  const DevCfg& c = x.c;
  const Region r = region_of(c, x.tb, p, x.tb.cur[p]);
  int64_t last;
  const int nwin = num_windows(c, t, &last);
  // t-digest (allowed lateness): the element joins the push's compression of its non-late windows (the newest nl)
  const bool td = c.agg == FW_AGG_TDIGEST && c.td_olast;
  int32_t oj = -1, nl = 0;
  for (int wi = 0; wi < nwin; wi++) {
    const int64_t s = jsub(last, (int64_t)wi * c.slide);
    const int64_t e = jadd(s, c.size);
    if (cleanup_of(e, c.lateness) <= x.wm) continue;  // isWindowLate
    *skipped = false;
    const uint64_t h = slot_hash(c, k, s);
    int32_t slot = region_find<true>(r, h, k, s, e);
    if (slot < 0) {
      Entry ne;
      ne.key = k;
      ne.start = s;
      ne.end = e;
      acc_clear(ne);
      ne.meta = c.pool_bytes ? (int64_t)(pool_new_block(c, x.st) << 1) : 0;
      slot = new_slot(x, r, p, h, ne);
      if (slot < 0) continue;
    }
    Entry en = r.ent[slot];
    acc_add(c, en, v, fo);
    if (c.agg == FW_AGG_HLL) hll_raise(c, pool_block_of(en), v);  // (k_hll_update takes the partitioned records)
    if (c.agg == FW_AGG_ROW) row_add(c, pool_block_of(en), v);   // (v: the record's index in the push)
    int32_t head = -1;
    if (td) {  // the window's chain of this push's values: this element on top
      if (oj < 0) {
        oj = atomicAdd(c.td_ovctr, 1);
        c.td_ovk[oj] = k;
        c.td_ovt[oj] = last;
        c.td_ovv[oj] = v;
        c.td_ovp[oj] = p;
      }
      const uint32_t g = ((uint32_t)p << c.log_r) | (uint32_t)slot;
      td_chain_insert(c, &c.td_olast[g], oj * c.wpr + wi, v);
      head = c.td_olast[g];
      nl = wi + 1;
    }
    bool keep = true;
    if (jsub(e, 1) <= x.wm) {  // EventTimeTrigger.onElement -> FIRE (WindowOperator.java:395-401)
      if (td) {  // getResult over the centroids and the push's values so far (the window stays)
        td_late_row(x, en, head);
      } else if (c.agg == FW_AGG_HLL) {  // getResult from the window's registers (the window stays unless purged)
        Entry fr = en;
        double est;
        hll_estimate(c, pool_block_of(en), &est, &fr.mn, &fr.mx);
        fr.sum = __double_as_longlong(est);
        emit_one(c, x.out, x.st, fr);
      } else {
        emit_one(c, x.out, x.st, en);
      }
      if (c.purging) keep = false;  // FIRE_AND_PURGE
    } else {
      en.meta |= FW_TIMER;  // registerEventTimeTimer(maxTimestamp)
    }
    if (!keep && (c.agg == FW_AGG_HLL || td)) {
      // the purged window keeps its slot and emptied block as empty state (cnt 0: nothing fires from it, and its GC
      // timer frees the block in k_fire): this kernel pops blocks for new windows, and a push beside those pops could
      // hand out a block before its slot on the free stack is written.  (t-digest: the push's chains and items
      // refer to the slot, and its values so far leave the push's compression)
      if (td)
        td_purge(c, ((uint32_t)p << c.log_r) | (uint32_t)slot, pool_block_of(en));
      else
        hll_clear(c, pool_block_of(en));
      acc_clear(en);
      en.meta &= ~(int64_t)FW_TIMER;
      keep = true;
    }
    if (keep) {
      r.ent[slot] = en;
      note_timer(x, p, en);
    } else {
      kill_slot(x, r, p, slot);
    }
  }
  if (oj >= 0) c.td_ovn[oj] = nl;
}

// t-digest sessions under allowed lateness: session e (slot se) merged into m (slot sm) -- e's chain of the push's
// values joined into m's (both sorted: a linear merge), and e's block with the blocks merged into it put on the list
// of blocks merged into m's block (td_late_row_session takes their union)
__device__ void td_session_join(const DevCfg& c, int32_t p, int32_t sm, int32_t se, const Entry& m, const Entry& e) {
  const uint32_t gm = ((uint32_t)p << c.log_r) | (uint32_t)sm, ge = ((uint32_t)p << c.log_r) | (uint32_t)se;
  int32_t a = c.td_olast[gm], b = c.td_olast[ge];
  int32_t out = -1;
  int32_t* tail = &out;
  while (a >= 0 && b >= 0) {
    if (td_key(c.td_ovv[a]) <= td_key(c.td_ovv[b])) {
      *tail = a;
      tail = &c.td_olink[a];
      a = c.td_olink[a];
    } else {
      *tail = b;
      tail = &c.td_olink[b];
      b = c.td_olink[b];
    }
  }
  *tail = a >= 0 ? a : b;
  c.td_olast[gm] = out;
  c.td_olast[ge] = -1;
  const int32_t dst = (int32_t)pool_block_of(m), src = (int32_t)pool_block_of(e);
  int32_t t = src;
  c.td_bnext[src] = c.td_bhead[src];
  while (c.td_bnext[t] >= 0) t = c.td_bnext[t];
  c.td_bnext[t] = c.td_bhead[dst];
  c.td_bhead[dst] = src;
  c.td_bhead[src] = -1;
}

// WindowOperator.processElement, merging branch (WindowOperator.java:297-370) with
// MergingWindowSet.addWindow (MergingWindowSet.java:150-225) over the key's in-flight sessions.
__device__ void replay_session(const SlowCtx& x, int32_t p, int64_t k, int64_t t, int64_t v, int64_t fo, bool* skipped) {
  const DevCfg& c = x.c;
  const Region r = region_of(c, x.tb, p, x.tb.cur[p]);
  const uint64_t h = slot_hash(c, k, 0);
  const uint32_t want = live_word(h);
  const int64_t ws = t, we = jadd(t, c.gap);  // EventTimeSessionWindows.assignWindows
  // TimeWindow.mergeWindows: in-flight windows are pairwise disjoint and non-touching, so the new window's
  // connected component is the windows that intersect it.  Every live entry of the key sits on its probe
  // chain: one walk finds the component (its first slot, its size, its hull), a second merges it.
  int32_t first = -1, n_in = 0;
  int64_t cs = ws, ce = we;
  for (uint32_t i = 0; i <= r.mask; i++) {
    const uint32_t s = ((uint32_t)h + i) & r.mask;
    const uint32_t stt = ld_state_wg(r.state + s);
    if (stt == SLOT_EMPTY) break;
    if (stt != want) continue;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const Entry& e = r.ent[s];
    if (e.key != k || !(ws <= e.end && we >= e.start)) continue;  // TimeWindow.intersects
    if (first < 0) first = (int32_t)s;
    n_in++;
    cs = min(cs, e.start);
    ce = max(ce, e.end);
  }
  int32_t actual = -1;
  bool fresh = false;
  if (first < 0) {
    Entry ne;
    ne.key = k;
    ne.start = ws;
    ne.end = we;
    acc_clear(ne);
    ne.meta = c.pool_bytes ? (int64_t)(pool_new_block(c, x.st) << 1) : 0;
    actual = new_slot(x, r, p, h, ne);
    if (actual < 0) return;
    fresh = true;
  } else {
    const Entry& f = r.ent[first];
    const bool contained = n_in == 1 && f.start == cs && f.end == ce;
    actual = first;
    if (!contained) {
      // merge function (WindowOperator.java:308-339)
      if (jadd(jsub(ce, 1), c.lateness) <= x.wm) {
        atomicOr(&x.st->flags, FW_STATUS_MERGE_LATE);
        return;
      }
      Entry m = f;
      for (uint32_t i = 0; i <= r.mask; i++) {
        const uint32_t s = ((uint32_t)h + i) & r.mask;
        const uint32_t stt = ld_state_wg(r.state + s);
        if (stt == SLOT_EMPTY) break;
        if (stt != want || (int32_t)s == first) continue;
        const Entry& e = r.ent[s];
        if (e.key != k || !(ws <= e.end && we >= e.start)) continue;
        acc_merge(c, m, e);  // mergeNamespaces
        if (c.pool_bytes) pool_merge_blocks(c, pool_block_of(m), pool_block_of(e));
        if (c.agg == FW_AGG_TDIGEST && c.td_olast) td_session_join(c, p, first, (int32_t)s, m, e);
        kill_slot(x, r, p, (int32_t)s);
      }
      m.start = cs;
      m.end = ce;
      // EventTimeTrigger.onMerge registers maxTimestamp unconditionally (the block id stays above the timer bit)
      m.meta = c.pool_bytes ? (m.meta | FW_TIMER) : FW_TIMER;
      r.ent[actual] = m;
    }
  }
  Entry en = r.ent[actual];
  if (cleanup_of(en.end, c.lateness) <= x.wm) {  // isWindowLate(actualWindow) -> retireWindow
    if (fresh) {
      if (c.pool_bytes) {  // its (untouched) block on the deferred list
        __threadfence();
        c.pool_defer[atomicAdd(&c.pool_ctr[2], 1)] = (uint32_t)pool_block_of(en);
      }
      kill_slot(x, r, p, actual);
    }
    return;
  }
  *skipped = false;
  acc_add(c, en, v, fo);
  if (c.agg == FW_AGG_HLL) hll_raise(c, pool_block_of(en), v);  // (k_hll_update takes the partitioned records)
  if (c.agg == FW_AGG_ROW) row_add(c, pool_block_of(en), v);   // (v: the record's index in the push)
  if (c.agg == FW_AGG_TDIGEST) {  // the value joins the push's compression
    const int j = atomicAdd(c.td_ovctr, 1);
    c.td_ovk[j] = k;
    c.td_ovt[j] = t;
    c.td_ovv[j] = v;
    c.td_ovp[j] = p;
    // (allowed lateness: and the session's sorted chain of the push's values, for its late firings)
    if (c.td_olast) td_chain_insert(c, &c.td_olast[((uint32_t)p << c.log_r) | (uint32_t)actual], j, v);
  }
  if (jsub(en.end, 1) <= x.wm) {
    if (c.agg == FW_AGG_TDIGEST && c.td_olast) {  // getResult over the session's digest and values so far
      td_late_row_session(x, en, c.td_olast[((uint32_t)p << c.log_r) | (uint32_t)actual]);
    } else if (c.agg == FW_AGG_HLL) {  // getResult from the session's registers (it stays in flight)
      Entry fr = en;
      double est;
      hll_estimate(c, pool_block_of(en), &est, &fr.mn, &fr.mx);
      fr.sum = __double_as_longlong(est);
      emit_one(c, x.out, x.st, fr);
    } else {
      emit_one(c, x.out, x.st, en);
    }
    if (c.purging) {  // FIRE_AND_PURGE clears the contents; the window stays in flight
      acc_clear(en);
      if (c.agg == FW_AGG_HLL) hll_clear(c, pool_block_of(en));
      if (c.agg == FW_AGG_TDIGEST && c.td_olast)
        td_purge(c, ((uint32_t)p << c.log_r) | (uint32_t)actual, pool_block_of(en));
    }
  } else {
    en.meta |= FW_TIMER;
  }
  r.ent[actual] = en;
  note_timer(x, p, en);
}

__global__ __launch_bounds__(FW_SLOW_THREADS) void k_slow(DevCfg c, int64_t wm, const uint32_t* __restrict__ srow,
                                                          int32_t T, const int64_t* __restrict__ sk,
                                                          const int64_t* __restrict__ stt,
                                                          const int64_t* __restrict__ sv,
                                                          const int32_t* __restrict__ skh, DevTable tb, DevRows out,
                                                          DevSide side, Status* st, int resume) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;  // resumed later
  // list length: the ordered-path offset of the last tile plus that tile's own count
  const int64_t n = (int64_t)(srow[T - 1] - srow[0]) + srow[T + T - 1];
  const int64_t first = resume ? st->slow_resume : 0;
  if (first >= n) return;
  __shared__ int64_t ck[SLOW_CHUNK];
  __shared__ int32_t ci[SLOW_CHUNK], cp[SLOW_CHUNK], cd[SLOW_CHUNK];
  __shared__ int bad;
  SlowCtx x{c, wm, tb, out, side, st};
  unsigned long long late = 0;
  const int tid = threadIdx.x;
  const int64_t row_bound = c.assigner == FW_SESSION ? 1 : c.wpr;  // fired rows per record, at most
  int64_t b0 = first;
  for (; b0 < n; b0 += SLOW_CHUNK) {
    const int m = (int)min((int64_t)SLOW_CHUNK, n - b0);
    if (tid == 0) bad = 0;
    if (tid < m) {
      const int64_t i = b0 + tid;
      ck[tid] = sk[i];
      cp[tid] = partition_of(c, ck[tid], skh[i]);
      int64_t last;
      cd[tid] = c.assigner == FW_SESSION ? 1 : num_windows(c, stt[i], &last);  // new windows, at most
      ci[tid] = tid;
    } else {
      ck[tid] = LMAX;
      cp[tid] = INT32_MAX;
      cd[tid] = 0;
      ci[tid] = INT32_MAX;
    }
    __syncthreads();
    // bitonic sort by (partition, key, arrival index): a key's records stay in arrival order and a
    // partition's records are contiguous, so its demand on the region is one segmented sum
    for (int kk = 2; kk <= SLOW_CHUNK; kk <<= 1) {
      for (int jj = kk >> 1; jj > 0; jj >>= 1) {
        const int o = tid ^ jj;
        if (o > tid) {
          const bool up = (tid & kk) == 0;
          const int32_t pa = cp[tid], pb = cp[o];
          const int64_t a = ck[tid], b = ck[o];
          const int32_t ia = ci[tid], ib = ci[o];
          const bool gt = pa > pb || (pa == pb && (a > b || (a == b && ia > ib)));
          if (gt == up) {
            cp[tid] = pb;
            cp[o] = pa;
            ck[tid] = b;
            ck[o] = a;
            ci[tid] = ib;
            ci[o] = ia;
            const int32_t da = cd[tid];
            cd[tid] = cd[o];
            cd[o] = da;
          }
        }
        __syncthreads();
      }
    }
    // capacity: every region the chunk touches must take its new windows within the load limit,
    // and the fired-row buffer must take every row the chunk may fire; otherwise suspend here
    if (tid < m && (tid == 0 || cp[tid - 1] != cp[tid])) {
      int64_t demand = 0;
      for (int j = tid; j < m && cp[j] == cp[tid]; j++) demand += cd[j];
      const int64_t want = (int64_t)tb.live[cp[tid]] + demand;
      if (want > region_limit(c.log_r)) {
        bad = 1;
        atomicMax(&st->need_live, (int32_t)min(want, (int64_t)INT32_MAX));
      }
    }
    if (tid == 0) {
      const int64_t want = (int64_t)__hip_atomic_load(&st->out_rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) +
                           (int64_t)m * row_bound;
      if (want > out.slow_limit) {
        bad = 1;
        atomicMax((long long*)&st->need_out, (long long)want);
      }
    }
    __syncthreads();
    if (bad) break;
    if (tid < m && (tid == 0 || ck[tid - 1] != ck[tid] || cp[tid - 1] != cp[tid])) {
      for (int j = tid; j < m && ck[j] == ck[tid] && cp[j] == cp[tid]; j++) {
        const int64_t i = b0 + ci[j];
        const int64_t k = sk[i], t = stt[i], v = sv[i];
        const int64_t fo = agg_ordinal(c) ? c.slow_ord[i] : 0;
        const int32_t p = cp[j];
        bool skipped = true;
        if (c.assigner == FW_SESSION)
          replay_session(x, p, k, t, v, fo, &skipped);
        else
          replay_time_windows(x, p, k, t, v, fo, &skipped);
        if (skipped && jadd(t, c.lateness) <= wm) {  // isSkippedElement && isElementLate
          if (c.side_output)
            side_one(side, st, k, t, v);
          else
            late++;
        }
      }
    }
    __syncthreads();
  }
  if (late) atomicAdd(&st->late_dropped, late);
  if (tid == 0) {
    atomicAdd(&st->slow_total, (unsigned long long)(min(b0, n) - first));
    if (b0 < n) {
      st->slow_resume = b0;
      atomicOr(&st->suspended, (int)FW_SUSP_SLOW);
    }
  }
}

// a fired row's block handed to the finish (out.mx for HyperLogLog, bit 63 of out.sum for t-digest) when the window
// fired with FIRE_AND_PURGE and stays in flight (a session): the block is emptied after its row is read, and kept
constexpr int64_t HLL_ZERO_KEEP = -2;
constexpr uint64_t TD_PURGE_TAG = 1ull << 63;
// a fired HLL row from its marked chunks' sums (lo, hi: sum_j 2^(65-p-M[j]) over them, 128 bits; zeros; touched
// chunks): the unmarked chunks are 16 zero registers each, 2^rmax apiece (rmax <= 61: the product fits 128 bits)
__device__ void hll_row_out(const DevCfg& c, const DevRows& out, uint64_t row, uint64_t lo, uint64_t hi, uint32_t zeros,
                            uint32_t touched, bool release, int64_t stack_slot, uint64_t blk) {
  const int p = c.hll_p, rmax = 65 - p;
  const int64_t m = (int64_t)1 << p;
  const int32_t nq = (int32_t)(m / 16);
  const uint64_t un = (uint64_t)(nq - (int32_t)touched) * 16u;
  const uint64_t ulo = un << rmax, uhi = rmax ? un >> (64 - rmax) : 0ull;
  const uint64_t t = lo + ulo;
  hi = hi + uhi + (t < lo ? 1ull : 0ull);
  lo = t;
  zeros += (uint32_t)un;
  const double sd = (double)hi * 18446744073709551616.0 + (double)lo;
  const double md = (double)m;
  const double alpha = m == 16 ? 0.673 : m == 32 ? 0.697 : m == 64 ? 0.709 : 0.7213 / (1.0 + 1.079 / md);
  const double raw = (alpha * md * md) * ldexp(1.0, rmax) / sd;
  const double est = (raw <= 2.5 * md && zeros > 0) ? md * log(md / (double)zeros) : raw;
  out.sum[row] = __double_as_longlong(est);
  out.mn[row] = (int64_t)zeros;
  out.mx[row] = (int64_t)lo;
  if (release) c.pool_free[stack_slot] = (uint32_t)blk;  // zeroed before the next kernel can hand it out
}
// ---- K_fire: watermark.  Regions with next_timer <= wm emit and are rebuilt into the other buffer.
// Pass 1 decides every slot, re-inserts the survivors into the other buffer and counts the fired
// rows; one reservation per workgroup in the output; pass 2 re-decides and writes the rows.
// one wave per fired row: estimate from the row's register block (out.mn holds its id), then zero the
// block and push it on the free stack.  S = sum_j 2^(65-p-M[j]) exactly, in 128 bits.  Only the chunks the
// block's bitmap marks are read (and zeroed): every register of an unmarked chunk is zero.
// stack_slot < 0: the window stays (FIRE without purge under allowed lateness): the block is read, not zeroed or freed;
// HLL_ZERO_KEEP: a session fired with FIRE_AND_PURGE stays in flight: the block is read and zeroed, not freed.
// A block with at most 64 marked chunks (a window of few distinct items: most windows of a Zipf stream's tail keys)
// takes two round trips: the bitmap (a word per lane), then every marked chunk at once, one per lane, from the
// chunk ids the wave lays out in its LDS scratch `ids` (64 words); a fuller block walks its bitmap 256 chunks a pass.
__device__ void hll_finish(const DevCfg& c, const DevRows& out, uint64_t row, int64_t stack_slot, uint32_t* ids) {
  const bool release = stack_slot >= 0;
  const bool zero = release || stack_slot == HLL_ZERO_KEEP;
  const int lane = __lane_id();
  const int p = c.hll_p, rmax = 65 - p;
  const int64_t m = (int64_t)1 << p;
  const uint64_t blk = (uint64_t)out.mn[row];
  uint8_t* base = c.pool + blk * (uint64_t)c.pool_bytes;
  uint32_t* bits = reinterpret_cast<uint32_t*>(base);
  uint4* q = reinterpret_cast<uint4*>(base + hll_hdr_bytes(p));
  const int32_t nq = (int32_t)(m / 16);  // 16-byte chunks
  const int32_t nw = (nq + 31) / 32;     // bitmap words
  uint64_t s = 0, sh = 0;
  uint32_t zeros = 0, touched = 0;
  constexpr int U = 4;  // word pairs per pass: up to 4 chunk loads in flight per lane
  uint32_t myw = lane < nw ? bits[lane] : 0u;  // the bitmap, one word per lane (64 words = 2^15 registers at a time)
  int32_t w_start = 0;
  if (nw <= 64) {
    const uint32_t cnt = (uint32_t)__popc(myw);
    uint32_t x = cnt;  // inclusive prefix of the marked chunks over the lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
      if (lane >= o) x += y;
    }
    const uint32_t tot = (uint32_t)__shfl((int)x, 63, 64);
    if (tot <= 64) {
      uint32_t k = x - cnt, word = myw;
      while (word) {
        const int b = __ffs(word) - 1;
        word &= word - 1;
        ids[k++] = (uint32_t)(lane * 32 + b);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if ((uint32_t)lane < tot) {
        const uint32_t j = ids[lane];
        const uint4 v = q[j];
        touched = 1;
        const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int kk = 0; kk < 4; kk++)
#pragma unroll
          for (int b = 0; b < 4; b++) {
            const uint32_t r = (ws[kk] >> (8 * b)) & 0xffu;
            const uint64_t t = s + (1ull << (rmax - (int)r));
            sh += t < s;
            s = t;
            zeros += r == 0;
          }
        if (zero) q[j] = make_uint4(0, 0, 0, 0);
      }
      __builtin_amdgcn_wave_barrier();  // (ids is the wave's next row's)
      w_start = nw;                     // every marked chunk is read
    }
  }
  for (int32_t w0 = w_start; w0 < nw; w0 += 2 * U) {
    if ((w0 & 63) == 0 && w0 > 0) myw = w0 + lane < nw ? bits[w0 + lane] : 0u;
    uint4 v[U];
    bool on[U];
    int32_t jj[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int32_t w = w0 + 2 * u + (lane >> 5);
      const uint32_t word = (uint32_t)__shfl((int)myw, (w & 63), 64);
      jj[u] = w * 32 + (lane & 31);
      on[u] = jj[u] < nq && ((word >> (lane & 31)) & 1u);
      v[u] = on[u] ? q[jj[u]] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (!on[u]) continue;
      touched++;
      const uint32_t ws[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int k = 0; k < 4; k++)
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const uint32_t r = (ws[k] >> (8 * b)) & 0xffu;
          const uint64_t t = s + (1ull << (rmax - (int)r));
          sh += t < s;  // 16 terms of up to 2^61 per chunk overflow 64 bits at small p
          s = t;
          zeros += r == 0;
        }
      if (zero) q[jj[u]] = make_uint4(0, 0, 0, 0);
    }
  }
  if (zero)
    for (int32_t w = lane; w < nw; w += 64) bits[w] = 0u;
  uint64_t hi = sh, lo = s;
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t lo2 = __shfl_xor(lo, o, 64), hi2 = __shfl_xor(hi, o, 64);
    const uint64_t t = lo + lo2;
    hi = hi + hi2 + (t < lo ? 1ull : 0ull);
    lo = t;
    zeros += __shfl_xor(zeros, o, 64);
    touched += __shfl_xor(touched, o, 64);
  }
  if (lane == 0) hll_row_out(c, out, row, lo, hi, zeros, touched, release, stack_slot, blk);
}
// four rows a wave, sixteen lanes each (p <= 14: at most 32 bitmap words, two per lane): a row with at most 16 marked
// chunks (most windows of a Zipf stream's tail keys) is read in two round trips by its sixteen lanes, four rows in
// flight; a fuller one is finished by the whole wave afterwards (hll_finish).  rows: the wave's four rows r,
// r + stride, ...; ri: their free-stack slots (out.mx, read before any of them is overwritten)
__device__ void hll_finish4(const DevCfg& c, const DevRows& out, uint64_t r, uint64_t stride, uint64_t end, int hl_sb,
                            uint32_t* ids) {
  const int lane = __lane_id(), g = lane >> 4, gl = lane & 15;
  const int p = c.hll_p, rmax = 65 - p;
  const int32_t nq = (int32_t)(((int64_t)1 << p) / 16), nw = (nq + 31) / 32;
  const uint64_t row = r + (uint64_t)g * stride;
  const bool valid = row < end;
  const int64_t ri = valid ? out.mx[row] : -1;
  const bool release = ri >= 0, zero = release || ri == HLL_ZERO_KEEP;
  const int64_t slot = release ? hl_sb + ri : ri;
  const uint64_t blk = valid ? (uint64_t)out.mn[row] : 0;
  uint8_t* base = c.pool + blk * (uint64_t)c.pool_bytes;
  uint32_t* bits = reinterpret_cast<uint32_t*>(base);
  uint4* q = reinterpret_cast<uint4*>(base + hll_hdr_bytes(p));
  const uint32_t w0 = valid && gl < nw ? bits[gl] : 0u, w1 = valid && gl + 16 < nw ? bits[gl + 16] : 0u;
  const uint32_t cnt = (uint32_t)(__popc(w0) + __popc(w1));
  uint32_t x = cnt;  // inclusive prefix over the row's sixteen lanes
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o, 16);
    if (gl >= o) x += y;
  }
  const uint32_t tot = (uint32_t)__shfl((int)x, 15, 16);
  const bool small = valid && tot <= 16;
  uint64_t s = 0, sh = 0;
  uint32_t zeros = 0, touched = 0;
  if (small) {
    uint32_t k = x - cnt;
    uint32_t word = w0;
    while (word) {
      const int b = __ffs(word) - 1;
      word &= word - 1;
      ids[g * 16 + k++] = (uint32_t)(gl * 32 + b);
    }
    word = w1;
    while (word) {
      const int b = __ffs(word) - 1;
      word &= word - 1;
      ids[g * 16 + k++] = (uint32_t)((gl + 16) * 32 + b);
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  if (small && (uint32_t)gl < tot) {
    const uint32_t j = ids[g * 16 + gl];
    const uint4 v = q[j];
    touched = 1;
    const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int kk = 0; kk < 4; kk++)
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const uint32_t rr = (ws[kk] >> (8 * b)) & 0xffu;
        const uint64_t t = s + (1ull << (rmax - (int)rr));
        sh += t < s;
        s = t;
        zeros += rr == 0;
      }
    if (zero) q[j] = make_uint4(0, 0, 0, 0);
  }
  if (small && zero) {
    if (gl < nw) bits[gl] = 0u;
    if (gl + 16 < nw) bits[gl + 16] = 0u;
  }
  uint64_t hi = sh, lo = s;
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) {  // (within the row's sixteen lanes)
    const uint64_t lo2 = __shfl_xor(lo, o, 16), hi2 = __shfl_xor(hi, o, 16);
    const uint64_t t = lo + lo2;
    hi = hi + hi2 + (t < lo ? 1ull : 0ull);
    lo = t;
    zeros += __shfl_xor(zeros, o, 16);
    touched += __shfl_xor(touched, o, 16);
  }
  if (small && gl == 0) hll_row_out(c, out, row, lo, hi, zeros, touched, release, slot, blk);
  __builtin_amdgcn_wave_barrier();  // (ids is the full-wave finishes' and the next rows')
  // the fuller rows, one after another by the whole wave
  const uint64_t full = __ballot(valid && !small && gl == 0);
#pragma unroll
  for (int gg = 0; gg < 4; gg++) {
    if (!((full >> (gg * 16)) & 1ull)) continue;
    const uint64_t rw = r + (uint64_t)gg * stride;
    const int64_t sl = __shfl(slot, gg * 16, 64);
    const uint64_t bk = __shfl(blk, gg * 16, 64);
    (void)bk;
    hll_finish(c, out, rw, sl, ids);
  }
}
// the same estimate by one thread, the block kept (a late firing of the ordered path under allowed lateness)
__device__ void hll_estimate(const DevCfg& c, uint64_t blk, double* est, int64_t* zeros_out, int64_t* lo_out) {
  const int p = c.hll_p, rmax = 65 - p;
  const int64_t m = (int64_t)1 << p;
  const uint8_t* base = c.pool + blk * (uint64_t)c.pool_bytes;
  const uint32_t* bits = reinterpret_cast<const uint32_t*>(base);
  const uint4* q = reinterpret_cast<const uint4*>(base + hll_hdr_bytes(p));
  const int32_t nq = (int32_t)(m / 16);
  uint64_t lo = 0, hi = 0;
  uint32_t zeros = 0, touched = 0;
  for (int32_t jq = 0; jq < nq; jq++) {
    if (!((bits[jq >> 5] >> (jq & 31)) & 1u)) continue;
    touched++;
    const uint4 v = q[jq];
    const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
    for (int k = 0; k < 4; k++)
      for (int b = 0; b < 4; b++) {
        const uint32_t r = (ws[k] >> (8 * b)) & 0xffu;
        const uint64_t t = lo + (1ull << (rmax - (int)r));
        hi += t < lo;
        lo = t;
        zeros += r == 0;
      }
  }
  const uint64_t un = (uint64_t)(nq - (int32_t)touched) * 16u;
  const uint64_t ulo = un << rmax, uhi = rmax ? un >> (64 - rmax) : 0ull;
  const uint64_t t = lo + ulo;
  hi = hi + uhi + (t < lo ? 1ull : 0ull);
  lo = t;
  zeros += (uint32_t)un;
  const double sd = (double)hi * 18446744073709551616.0 + (double)lo;
  const double md = (double)m;
  const double alpha = m == 16 ? 0.673 : m == 32 ? 0.697 : m == 64 ? 0.709 : 0.7213 / (1.0 + 1.079 / md);
  const double raw = (alpha * md * md) * ldexp(1.0, rmax) / sd;
  *est = (raw <= 2.5 * md && zeros > 0) ? md * log(md / (double)zeros) : raw;
  *zeros_out = (int64_t)zeros;
  *lo_out = (int64_t)lo;
}
// one thread: zero a register block's marked chunks and its bitmap (a window collected without a row)
__device__ void hll_clear(const DevCfg& c, uint64_t blk) {
  uint8_t* base = c.pool + blk * (uint64_t)c.pool_bytes;
  uint32_t* bits = reinterpret_cast<uint32_t*>(base);
  uint4* q = reinterpret_cast<uint4*>(base + hll_hdr_bytes(c.hll_p));
  const int32_t nq = (int32_t)(((int64_t)1 << c.hll_p) / 16), nw = (nq + 31) / 32;
  for (int32_t w = 0; w < nw; w++) {
    uint32_t word = bits[w];
    while (word) {
      const int b = __ffs(word) - 1;
      word &= word - 1;
      q[w * 32 + b] = make_uint4(0, 0, 0, 0);
    }
    bits[w] = 0u;
  }
}

// fold each partitioned record's item into the registers of its (key, window): M[j] = max(M[j], rank).
// One workgroup per FW_HLL_CHUNK records; a record's partition is found from the scan offsets.  Byte
// registers are raised with a CAS on their 32-bit word, only when the rank is larger (max is idempotent,
// so a resumed push may run this again over the whole batch).
#ifndef FW_HLL_CHUNK_N
#define FW_HLL_CHUNK_N 4096
#endif
constexpr int FW_HLL_CHUNK = FW_HLL_CHUNK_N;
#ifndef FW_HLL_MARK
#define FW_HLL_MARK 3  // chunk marks skipped: 1 = when the mark's word (read through L1) has it, 2 = when another
                       // register of the raised word is non-zero (its raise marks, or marked, the chunk)
#endif
#ifndef FW_HLL_BLIND
#define FW_HLL_BLIND 256
#endif
#ifndef FW_HLL_WAVES
#define FW_HLL_WAVES 1
#endif
// SLIDE: records of sliding windows (PRec, nwin windows each); tumbling records carry one window (no window loop)
template <bool SLIDE>
__global__ __launch_bounds__(256, FW_HLL_WAVES) void k_hll_update(DevCfg c, const PRec* __restrict__ part,
                                                    const uint32_t* __restrict__ offs, int32_t T, DevTable tb,
                                                    Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int64_t total = offs[(int64_t)c.P * T];
  const int64_t i0 = (int64_t)blockIdx.x * FW_HLL_CHUNK;
  if (i0 >= total) return;
  __shared__ int32_t p0_s;
  if (threadIdx.x == 0) {  // partition of the chunk's first record: last p with offs[p*T] <= i0
    int32_t lo = 0, hi = c.P - 1;
    while (lo < hi) {
      const int32_t mid = (lo + hi + 1) >> 1;
      if ((int64_t)offs[(int64_t)mid * T] <= i0)
        lo = mid;
      else
        hi = mid - 1;
    }
    p0_s = lo;
  }
  __syncthreads();
  const int p = c.hll_p;
  const bool cmp = c.compact && !*c.wide;
  const int64_t i1 = min(total, i0 + (int64_t)FW_HLL_CHUNK);
  const int64_t hdr = hll_hdr_bytes(p);
  // HU records per thread in flight: the record, its home slot's state word and entry identity, the entry's
  // block id and the register word are each loaded for all of them before any is used (the common case at a
  // region's load is a home-slot hit; a miss walks the rest of its probe chain on its own)
  constexpr int HU = 4;
  int32_t pp = p0_s;
  // sliding windows (fan-out): a record raises the same register in each of its nwin windows, newest first
  // (SlidingEventTimeWindows.java:67-81); the windows are walked one per pass of this loop
  for (int64_t ib = i0 + threadIdx.x; ib < i1; ib += (int64_t)blockDim.x * HU) {
   int32_t nw_max = 1;
   for (int32_t wi = 0; wi < (SLIDE ? nw_max : 1); wi++) {
    int64_t key[HU], last[HU], val[HU];
    int32_t part_of_rec[HU];
    bool in[HU];
    int32_t pp_w = pp;
#pragma unroll
    for (int u = 0; u < HU; u++) {
      const int64_t i = ib + (int64_t)u * blockDim.x;
      in[u] = i < i1;
      key[u] = last[u] = val[u] = 0;
      part_of_rec[u] = pp_w;
      if (!in[u]) continue;
      while ((int64_t)offs[(int64_t)(pp_w + 1) * T] <= i) pp_w++;
      part_of_rec[u] = pp_w;
      if (cmp) {
        const i64x2 r = reinterpret_cast<const i64x2*>(part)[i];
        compact_decode(c, pp_w, r.x, &key[u], &last[u]);
        val[u] = r.y;
      } else {
        const PRec rec = part[i];
        key[u] = rec.key;
        last[u] = rec.last;
        if constexpr (SLIDE) {
          const int32_t nw = (int32_t)(rec.nwin & 0xffff);
          nw_max = max(nw_max, nw);
          in[u] = wi < nw;
          last[u] = jsub(rec.last, (int64_t)wi * c.slide);
        }
        val[u] = rec.val;
      }
    }
    uint32_t hw[HU];
    i64x2 hk[HU];
    int64_t hend[HU], hmeta[HU], hcnt[HU];
    uint64_t hs[HU];
    Region rg[HU];
#pragma unroll
    for (int u = 0; u < HU; u++) {
      rg[u] = region_of(c, tb, part_of_rec[u], tb.cur[part_of_rec[u]]);
      hs[u] = slot_hash(c, key[u], last[u]);
      hw[u] = 0;
      if (!in[u]) continue;
      const uint32_t home = (uint32_t)hs[u] & rg[u].mask;
#ifdef FW_HLL_NOLOOKUP
      continue;
#endif
      hw[u] = rg[u].state[home];  // (the table is read-only here: a plain, L1-cacheable read)
      hk[u] = *reinterpret_cast<const i64x2*>(&rg[u].ent[home].key);
      hend[u] = rg[u].ent[home].end;
      hmeta[u] = rg[u].ent[home].meta;
      hcnt[u] = rg[u].ent[home].cnt;
    }
    uint64_t blk[HU];
    bool blind[HU];
#pragma unroll
    for (int u = 0; u < HU; u++) {
      blk[u] = 0;
      blind[u] = false;
      if (!in[u]) continue;
#ifdef FW_HLL_NOLOOKUP  // (timing ablation only: the block from a hash, results wrong)
      blk[u] = fmix64((uint64_t)key[u] ^ (uint64_t)last[u]) % (uint64_t)c.pool_blocks;
      continue;
#endif
      const int64_t we = wend(c, last[u]);
      if (hw[u] == live_word(hs[u]) && hk[u].x == key[u] && hk[u].y == last[u] && hend[u] == we) {
        blk[u] = (uint64_t)hmeta[u] >> 1;
        blind[u] = hcnt[u] <= FW_HLL_BLIND;
      } else {
        const int32_t slot = hw[u] == SLOT_EMPTY ? -1 : region_find(rg[u], hs[u] + 1, key[u], last[u], we, live_word(hs[u]));
        if (slot < 0) {
          atomicOr(&st->flags, FW_STATUS_STATE_LOST);  // the aggregate stored every record's window
          in[u] = false;
          continue;
        }
        blk[u] = pool_block_of(rg[u].ent[slot]);
        blind[u] = rg[u].ent[slot].cnt <= FW_HLL_BLIND;
      }
    }
    uint32_t* w[HU];
    uint32_t old[HU], rank[HU], jj[HU];
#pragma unroll
    for (int u = 0; u < HU; u++) {
      const uint64_t h = fmix64((uint64_t)val[u]);
      jj[u] = (uint32_t)(h >> (64 - p));
      rank[u] = (uint32_t)__clzll((long long)((h << p) | (1ull << (p - 1)))) + 1u;
      w[u] = reinterpret_cast<uint32_t*>(c.pool + blk[u] * (uint64_t)c.pool_bytes + hdr + (jj[u] & ~3u));
      // a plain (L1-cacheable) read: registers only grow, so a stale copy is never above the register and
      // costs at most a CAS that returns the current word (a hot digest's block stays in the CU's L1).  A window
      // of few items (its count, after this batch, at most FW_HLL_BLIND) skips the read: its word is most likely
      // still zero, and a CAS that finds it otherwise returns it
      old[u] = in[u] && !blind[u] ? *w[u] : 0u;
    }
    // every raise's CAS in flight at once; one that lost to another record's raise of the same word retries alone
    uint32_t got[HU], nwv[HU];
    bool need[HU];
#pragma unroll
    for (int u = 0; u < HU; u++) {
      const int sh = (int)(jj[u] & 3) * 8;
      need[u] = in[u] && ((old[u] >> sh) & 0xffu) < rank[u];
#if defined(FW_HLL_ABL) && (FW_HLL_ABL & 2)  // (timing ablation only: registers read, never raised)
      need[u] = false;
#endif
      nwv[u] = (old[u] & ~(0xffu << sh)) | (rank[u] << sh);
      got[u] = need[u] ? atomicCAS(w[u], old[u], nwv[u]) : old[u];
    }
#pragma unroll
    for (int u = 0; u < HU; u++) {
      if (!need[u]) continue;
      const int sh = (int)(jj[u] & 3) * 8;
      uint32_t o = got[u], prev = old[u];
      bool done = o == old[u];
      while (!done && ((o >> sh) & 0xffu) < rank[u]) {
        const uint32_t nw = (o & ~(0xffu << sh)) | (rank[u] << sh);
        prev = o;
        done = __hip_atomic_compare_exchange_strong(w[u], &o, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
      }
      // this record took the register out of zero: mark its chunk for the fire, unless another register of the
      // word is non-zero (its raise marks, or marked, the chunk) or the mark's word (read through L1) has it (a
      // stale unmarked copy costs one redundant atomic; a mark is never cleared meanwhile)
#if defined(FW_HLL_ABL) && (FW_HLL_ABL & 1)  // (timing ablation only: no chunk marks)
      done = false;
#endif
      if (done && ((prev >> sh) & 0xffu) == 0u) {
        const uint32_t ch = jj[u] >> 4;
        uint32_t* mw = reinterpret_cast<uint32_t*>(c.pool + blk[u] * (uint64_t)c.pool_bytes) + (ch >> 5);
        bool mark = true;
        if (FW_HLL_MARK & 2) mark = (prev & ~(0xffu << sh)) == 0u;
        if ((FW_HLL_MARK & 1) && mark) mark = !((*mw >> (ch & 31u)) & 1u);
        if (mark) atomicOr(mw, 1u << (ch & 31u));
      }
    }
    if (wi + 1 == nw_max) pp = pp_w;
   }
  }
}

// the same for session windows: a record's window [ts, ts + gap) lies, after the aggregate's merges, inside exactly
// one of its key's in-flight sessions (MergingWindowSet keeps them pairwise disjoint), found on the key's probe chain
// (sessions hash the key only); its item raises that session's registers.  HU records' chain heads in flight.
__global__ __launch_bounds__(256) void k_hll_update_sessions(DevCfg c, const PRec* __restrict__ part,
                                                             const uint32_t* __restrict__ offs, int32_t T, DevTable tb,
                                                             Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int64_t total = offs[(int64_t)c.P * T];
  const int64_t i0 = (int64_t)blockIdx.x * FW_HLL_CHUNK;
  if (i0 >= total) return;
  __shared__ int32_t p0_s;
  if (threadIdx.x == 0) {  // partition of the chunk's first record: last p with offs[p*T] <= i0
    int32_t lo = 0, hi = c.P - 1;
    while (lo < hi) {
      const int32_t mid = (lo + hi + 1) >> 1;
      if ((int64_t)offs[(int64_t)mid * T] <= i0)
        lo = mid;
      else
        hi = mid - 1;
    }
    p0_s = lo;
  }
  __syncthreads();
  const bool cmp = c.compact && !*c.wide;
  const int64_t i1 = min(total, i0 + (int64_t)FW_HLL_CHUNK);
  int32_t pp = p0_s;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    while ((int64_t)offs[(int64_t)(pp + 1) * T] <= i) pp++;
    int64_t key, ts, val;
    if (cmp) {
      const i64x2 r = reinterpret_cast<const i64x2*>(part)[i];
      compact_decode(c, pp, r.x, &key, &ts);
      val = r.y;
    } else {
      const PRec rec = part[i];
      key = rec.key;
      ts = rec.last;
      val = rec.val;
    }
    const int64_t te = jadd(ts, c.gap);
    const Region r = region_of(c, tb, pp, tb.cur[pp]);
    const uint64_t h = slot_hash(c, key, 0);
    const uint32_t want = live_word(h);
    int64_t blk = -1;
    for (uint32_t k = 0; k <= r.mask; k++) {
      const uint32_t s = ((uint32_t)h + k) & r.mask;
      const uint32_t w = r.state[s];  // (the table is read-only here)
      if (w == SLOT_EMPTY) break;
      if (w != want) continue;
      const Entry& e = r.ent[s];
      if (e.key == key && e.start <= ts && te <= e.end) {
        blk = (int64_t)pool_block_of(e);
        break;
      }
    }
    if (blk < 0) {
      atomicOr(&st->flags, FW_STATUS_STATE_LOST);  // the aggregate stored every record's session
      continue;
    }
    hll_raise(c, (uint64_t)blk, val);
  }
}
// the blocks session merges freed (zeroed, on the deferred list) onto the free stack: before a firing, when nothing
// pops (one workgroup)
__global__ __launch_bounds__(256) void k_pool_release(DevCfg c) {
  const int32_t n = c.pool_ctr[2];
  if (n <= 0) return;
  __shared__ int32_t base_s;
  if (threadIdx.x == 0) base_s = atomicAdd(&c.pool_ctr[0], n);
  __syncthreads();
  for (int32_t i = threadIdx.x; i < n; i += blockDim.x) c.pool_free[base_s + i] = c.pool_defer[i];
  __syncthreads();
  if (threadIdx.x == 0) c.pool_ctr[2] = 0;
}


// FW_AGG_ROW: after the aggregate created every record's window (or merged its session) and counted it, each
// partitioned record adds its columns (read by its batch index, the record's value) into its window's block
// (row_add).  The adds are not idempotent: the kernel runs only when the aggregate did not suspend (a resumed push
// launches it once more, after the resumed aggregate).  One workgroup per FW_HLL_CHUNK records, a record's partition
// from the scan offsets.  MODE 0: one window per record (tumbling), 1: sliding fan-out (PRec, nwin windows, newest
// first), 2: sessions (the in-flight session of the key that contains [ts, ts + gap), sessions hash the key only).
__device__ __forceinline__ int32_t session_containing(const Region& r, const DevCfg& c, int64_t key, int64_t ts);
template <int MODE>
__global__ __launch_bounds__(256) void k_row_update(DevCfg c, const PRec* __restrict__ part,
                                                   const uint32_t* __restrict__ offs, int32_t T, DevTable tb,
                                                   Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int64_t total = offs[(int64_t)c.P * T];
  const int64_t i0 = (int64_t)blockIdx.x * FW_HLL_CHUNK;
  if (i0 >= total) return;
  __shared__ int32_t p0_s;
  if (threadIdx.x == 0) {  // partition of the chunk's first record: last p with offs[p*T] <= i0
    int32_t lo = 0, hi = c.P - 1;
    while (lo < hi) {
      const int32_t mid = (lo + hi + 1) >> 1;
      if ((int64_t)offs[(int64_t)mid * T] <= i0)
        lo = mid;
      else
        hi = mid - 1;
    }
    p0_s = lo;
  }
  __syncthreads();
  const bool cmp = c.compact && !*c.wide;
  const int64_t i1 = min(total, i0 + (int64_t)FW_HLL_CHUNK);
  int32_t pp = p0_s;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    while ((int64_t)offs[(int64_t)(pp + 1) * T] <= i) pp++;
    int64_t key, last, idx;
    int32_t nw = 1;
    if (cmp) {
      const i64x2 r = reinterpret_cast<const i64x2*>(part)[i];
      compact_decode(c, pp, r.x, &key, &last);
      idx = r.y;
    } else {
      const PRec rec = part[i];
      key = rec.key;
      last = rec.last;
      idx = rec.val;
      nw = (int32_t)(rec.nwin & 0xffff);
    }
    const Region r = region_of(c, tb, pp, tb.cur[pp]);
    if constexpr (MODE == 2) {
      const int32_t slot = session_containing(r, c, key, last);
      if (slot < 0) {
        atomicOr(&st->flags, FW_STATUS_STATE_LOST);  // the aggregate stored every record's session
        continue;
      }
      row_add(c, pool_block_of(r.ent[slot]), idx);
    } else {
      for (int32_t wi = 0; wi < (MODE == 1 ? nw : 1); wi++) {
        const int64_t ws = jsub(last, (int64_t)wi * c.slide);
        const int64_t we = wend(c, ws);
        const int32_t slot = region_find(r, slot_hash(c, key, ws), key, ws, we);
        if (slot < 0) {
          atomicOr(&st->flags, FW_STATUS_STATE_LOST);
          continue;
        }
        row_add(c, pool_block_of(r.ent[slot]), idx);
      }
    }
  }
}

// ---- t-digest (FW_AGG_TDIGEST).  The definition is oracle/window_oracle.h's OR_AGG_TDIGEST, restated here
// operation for operation in IEEE double without contraction (the library is built with -ffp-contract=off),
// so a digest is bit-exact with the oracle's.  Per push, after the aggregate created the entries and their
// blocks: every record's (entry slot, value) pair is sorted (rocPRIM radix sort by value, then stably by
// slot), so the batch values of one digest form one run in Double.compare order.  Each digest then merges
// its run with its centroids into the other half of its block, in one of three tiers by size:
//   serial  (<= FW_TD_T1 values + centroids): one thread walks the merged sequence;
//   wave    (<= FW_TD_T3): one wave — each lane places 64 values at a time (its bucket from its merged
//           position: binary searches over the old centroids in LDS), then per bucket the wave sums the
//           bucket's values 64 at a time as butterfly trees and folds the old centroids' sums;
//   large   (> FW_TD_T3, the hottest keys): the placement runs over the whole grid and one wave per
//           (digest, bucket) forms the bucket's centroid.
// All three produce the definition's sums: per bucket, the old centroids' sums left to right, the new values
// in blocks of 64 from the bucket's first value, each block a perfect binary tree over 64 slots, the block
// sums left to right.
constexpr int TD_NB_MAX = 250;  // delta <= 500
__device__ __forceinline__ uint64_t td_key(int64_t bits) { return (uint64_t)f64_sortable(bits) ^ 0x8000000000000000ull; }
__device__ __forceinline__ double td_val(uint64_t key) {
  return __longlong_as_double(f64_unsortable((int64_t)(key ^ 0x8000000000000000ull)));
}
__device__ __forceinline__ uint64_t td_mean_key(double sum, int64_t w) {
  return td_key(__double_as_longlong(sum / (double)w));
}
__device__ __forceinline__ TdHead* td_head(const DevCfg& c, uint64_t blk) {
  return reinterpret_cast<TdHead*>(c.pool + blk * (uint64_t)c.pool_bytes);
}
__device__ __forceinline__ TdCent* td_half(const DevCfg& c, uint64_t blk, int h) {
  return reinterpret_cast<TdCent*>(c.pool + blk * (uint64_t)c.pool_bytes + sizeof(TdHead)) + (int64_t)h * c.td_nb;
}
// bucket of an item's midpoint: the largest b < nb with W * qb[b] <= mid
// (qb: the quantile bounds, staged in LDS by the kernels: td_stage_qb)
__device__ __forceinline__ int td_bucket(const DevCfg& c, const double* qb, double W, double mid) {
  int lo = 0, hi = c.td_nb - 1;
  while (lo < hi) {
    const int m = (lo + hi + 1) >> 1;
    if (W * qb[m] <= mid)
      lo = m;
    else
      hi = m - 1;
  }
  return lo;
}
// the workgroup's copy of the quantile bounds (every thread of the workgroup calls it)
__device__ __forceinline__ void td_stage_qb(const DevCfg& c, double* s_qb) {
  for (int b = threadIdx.x; b < c.td_nb; b += blockDim.x) s_qb[b] = c.td_qb[b];
  __syncthreads();
}
__device__ __forceinline__ int64_t td_weight(const TdCent* ce, int32_t j) { return ce[j].cum - (j ? ce[j - 1].cum : 0); }
// a left-to-right fold of partial sums (`any` = something folded yet)
__device__ __forceinline__ void td_fold(double& s, bool& any, double x) {
  s = any ? s + x : x;
  any = true;
}
// one thread's tree sum of a block of up to 64 values (a binary counter of complete subtrees)
struct TdTree {
  double st[7];
  uint32_t cnt;
  __device__ void push(double x) {
    double v = x;
    bool placed = false;
#pragma unroll
    for (int l = 0; l < 7; l++) {
      if (placed) continue;
      if ((cnt >> l) & 1u) {
        v = st[l] + v;
      } else {
        st[l] = v;
        placed = true;
      }
    }
    cnt++;
  }
  // the block's sum, the subtrees joined from the smallest (rightmost) up
  __device__ double finish() const {
    double t = 0.0;
    bool any = false;
#pragma unroll
    for (int l = 0; l < 7; l++) {
      if (!((cnt >> l) & 1u)) continue;
      t = any ? st[l] + t : st[l];
      any = true;
    }
    return t;
  }
};
// the wave's tree sum of the 64 lanes' values in lane order (lanes without a value contribute nothing)
__device__ __forceinline__ double td_wave_tree(double x, bool has) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double ox = __shfl_xor(x, o, 64);
    const bool oh = __shfl_xor((int)has, o, 64) != 0;
    if (has && oh)
      x = x + ox;  // left + right (the upper lane adds right + left: the same IEEE sum)
    else if (oh)
      x = ox;
    has = has || oh;
  }
  return x;
}
// the wave's S_new of a bucket: its sorted values v[ns, ne) in blocks of 64, tree sums folded left to right
#ifndef FW_TD_SUM_U
#define FW_TD_SUM_U 8
#endif
__device__ double td_wave_new_sum(const uint64_t* __restrict__ v, int64_t ns, int64_t ne) {
  // FW_TD_SUM_U full blocks a round, the next round's loads in flight while this one's trees are summed (a hot
  // bucket of a large digest holds tens of thousands of values: one wave walks them)
  constexpr int U = FW_TD_SUM_U;
  constexpr int64_t RW = (int64_t)U * 64;
  const int lane = __lane_id();
  double s = 0.0;
  bool any = false;
  int64_t b0 = ns;
  const int64_t full = ns + (ne - ns) / RW * RW;
  if (b0 < full) {
    double xa[U], xb[U];
    // (branch-free loads: past the last full round a round reloads the last one)
    auto ld = [&](double (&x)[U], int64_t base) {
      const int64_t bb = min(base, full - RW);
#pragma unroll
      for (int u = 0; u < U; u++) x[u] = td_val(v[bb + u * 64 + lane]);
    };
    ld(xa, b0);
    for (;;) {
      ld(xb, b0 + RW);
#pragma unroll
      for (int u = 0; u < U; u++) td_fold(s, any, td_wave_tree(xa[u], true));
      b0 += RW;
      if (b0 >= full) break;
      ld(xa, b0 + RW);
#pragma unroll
      for (int u = 0; u < U; u++) td_fold(s, any, td_wave_tree(xb[u], true));
      b0 += RW;
      if (b0 >= full) break;
    }
  }
  for (; b0 < ne; b0 += 64) {
    const bool has = b0 + lane < ne;
    const double x = has ? td_val(v[b0 + lane]) : 0.0;
    td_fold(s, any, td_wave_tree(x, has));
  }
  return s;
}

// serial merge of nn sorted value keys, taken in order from next(), with the no centroids `old` into `out`
// (window_oracle.cpp td_compress)
template <class Next>
__device__ int32_t td_merge_run(const DevCfg& c, const double* qb, Next next, int64_t nn, const TdCent* __restrict__ old,
                                int32_t no, TdCent* __restrict__ out, int64_t W) {
  const double Wd = (double)W;
  int64_t i = 0, cw = 0, gw = 0, cum_out = 0, prev_old = 0;
  int32_t j = 0, k = 0;
  uint64_t mk = no ? td_mean_key(old[0].sum, old[0].cum) : 0;
  uint64_t nk = nn ? next() : 0;  // the next new value's key
  double so = 0.0, sn = 0.0;
  bool any_o = false, any_n = false;
  TdTree tr;
  tr.cnt = 0;
  int b = 0, cur = -1;
  auto emit = [&]() {
    if (tr.cnt) td_fold(sn, any_n, tr.finish());
    cum_out += gw;
    out[k++] = TdCent{any_o && any_n ? so + sn : any_o ? so : sn, cum_out};
    gw = 0;
    any_o = any_n = false;
    tr.cnt = 0;
  };
  while (i < nn || j < no) {
    const bool take_new = j == no || (i < nn && nk <= mk);
    double x;
    int64_t w;
    if (take_new) {
      x = td_val(nk);
      w = 1;
      i++;
      if (i < nn) nk = next();
    } else {
      x = old[j].sum;
      w = old[j].cum - prev_old;
      prev_old = old[j].cum;
      j++;
      if (j < no) mk = td_mean_key(old[j].sum, old[j].cum - prev_old);
    }
    const double mid = (double)cw + (double)w * 0.5;
    while (b + 1 < c.td_nb && Wd * qb[b + 1] <= mid) b++;
    if (b != cur && gw > 0) emit();
    cur = b;
    if (take_new) {
      tr.push(x);
      if (tr.cnt == 64) {
        td_fold(sn, any_n, tr.finish());
        tr.cnt = 0;
      }
    } else {
      td_fold(so, any_o, x);
    }
    gw += w;
    cw += w;
  }
  if (gw > 0) emit();
  return k;
}
// the same over the sorted run v[beg, beg + nn)
__device__ int32_t td_merge_serial(const DevCfg& c, const double* qb, const uint64_t* __restrict__ v, int64_t beg,
                                   int64_t nn, const TdCent* __restrict__ old, int32_t no, TdCent* __restrict__ out,
                                   int64_t W) {
  const uint64_t* p = v + beg;
  return td_merge_run(c, qb, [&]() { return *p++; }, nn, old, no, out, W);
}

// td_merge_serial for the serial tier (k_td_small): the same merge, with the run's value keys and the old centroids
// read TD_BN / TD_BO at a time into registers.  Element by element, every step of the merge waited for its own load
// (the next key decides which stream the step takes); a block's loads are in flight together.
#ifndef FW_TD_BN
#define FW_TD_BN 8
#endif
#ifndef FW_TD_BO
#define FW_TD_BO 4
#endif
constexpr int TD_BN = FW_TD_BN, TD_BO = FW_TD_BO;
static_assert((TD_BN & (TD_BN - 1)) == 0 && (TD_BO & (TD_BO - 1)) == 0, "blocks of a power of two");
__device__ int32_t td_merge_serial_blk(const DevCfg& c, const double* qb, const uint64_t* __restrict__ v, int64_t beg,
                                       int64_t nn, const TdCent* __restrict__ old, int32_t no, TdCent* __restrict__ out,
                                       int64_t W) {
  const uint64_t* __restrict__ pv = v + beg;
  uint64_t nbk[TD_BN];
  double osb[TD_BO];
  int64_t ocb[TD_BO];
  auto fill_n = [&](int64_t i0) {
#pragma unroll
    for (int u = 0; u < TD_BN; u++) nbk[u] = i0 + u < nn ? pv[i0 + u] : 0ull;
  };
  auto fill_o = [&](int32_t j0) {
#pragma unroll
    for (int u = 0; u < TD_BO; u++) {
      osb[u] = 0.0;
      ocb[u] = 0;
      if (j0 + u < no) {
        const TdCent t = old[j0 + u];
        osb[u] = t.sum;
        ocb[u] = t.cum;
      }
    }
  };
  // element i of the current block (selects, not an indexed register array)
  auto pick_n = [&](int64_t i) {
    const int s = (int)(i & (TD_BN - 1));
    uint64_t x = nbk[0];
#pragma unroll
    for (int u = 1; u < TD_BN; u++) x = s == u ? nbk[u] : x;
    return x;
  };
  auto pick_o = [&](int32_t j, double& sum, int64_t& cum) {
    const int s = j & (TD_BO - 1);
    sum = osb[0];
    cum = ocb[0];
#pragma unroll
    for (int u = 1; u < TD_BO; u++) {
      sum = s == u ? osb[u] : sum;
      cum = s == u ? ocb[u] : cum;
    }
  };
  const double Wd = (double)W;
  int64_t i = 0, cw = 0, gw = 0, cum_out = 0, prev_old = 0;
  int32_t j = 0, k = 0;
  if (nn) fill_n(0);
  if (no) fill_o(0);
  double osum = 0.0;
  int64_t ocum = 0;
  if (no) pick_o(0, osum, ocum);
  uint64_t mk = no ? td_mean_key(osum, ocum) : 0;
  uint64_t nk = nn ? pick_n(0) : 0;  // the next new value's key
  double so = 0.0, sn = 0.0;
  bool any_o = false, any_n = false;
  TdTree tr;
  tr.cnt = 0;
  int b = 0, cur = -1;
  auto emit = [&]() {
    if (tr.cnt) td_fold(sn, any_n, tr.finish());
    cum_out += gw;
    out[k++] = TdCent{any_o && any_n ? so + sn : any_o ? so : sn, cum_out};
    gw = 0;
    any_o = any_n = false;
    tr.cnt = 0;
  };
  while (i < nn || j < no) {
    const bool take_new = j == no || (i < nn && nk <= mk);
    double x;
    int64_t w;
    if (take_new) {
      x = td_val(nk);
      w = 1;
      i++;
      if (i < nn) {
        if ((i & (TD_BN - 1)) == 0) fill_n(i);
        nk = pick_n(i);
      }
    } else {
      x = osum;
      w = ocum - prev_old;
      prev_old = ocum;
      j++;
      if (j < no) {
        if ((j & (TD_BO - 1)) == 0) fill_o(j);
        pick_o(j, osum, ocum);
        mk = td_mean_key(osum, ocum - prev_old);
      }
    }
    const double mid = (double)cw + (double)w * 0.5;
    while (b + 1 < c.td_nb && Wd * qb[b + 1] <= mid) b++;
    if (b != cur && gw > 0) emit();
    cur = b;
    if (take_new) {
      tr.push(x);
      if (tr.cnt == 64) {
        td_fold(sn, any_n, tr.finish());
        tr.cnt = 0;
      }
    } else {
      td_fold(so, any_o, x);
    }
    gw += w;
    cw += w;
  }
  if (gw > 0) emit();
  return k;
}

// piecewise-linear quantile through (0, min), (centre_i, mean_i) ..., (W, max) (window_oracle.cpp td_quantile)
__device__ double td_quantile(const TdCent* ce, int32_t n, int64_t W, double mn, double mx, double qv) {
  if (n == 0) return __longlong_as_double(0x7ff8000000000000ll);
  const double Wd = (double)W;
  const double x = qv * Wd;
  double x0 = 0.0, y0 = mn;
  int64_t before = 0;
  for (int32_t i = 0; i < n; i++) {
    const int64_t w = ce[i].cum - before;
    const double t = (double)before + (double)w * 0.5;
    const double m = ce[i].sum / (double)w;
    if (t >= x) return y0 + (m - y0) * ((x - x0) / (t - x0));
    x0 = t;
    y0 = m;
    before = ce[i].cum;
  }
  return y0 + (mx - y0) * ((x - x0) / (Wd - x0));
}

// the union of digests' centroids u[0, m) held as (sum, weight): ordered by (mean key, weight, sum key) -- an
// insertion sort (oracle td_union) -- and the weights made cumulative
__device__ void td_union_sort(TdCent* u, int32_t m) {
  for (int32_t a = 1; a < m; a++) {
    const TdCent x = u[a];
    const uint64_t xm = td_mean_key(x.sum, x.cum), xs = td_key(__double_as_longlong(x.sum));
    int32_t b = a - 1;
    while (b >= 0) {
      const uint64_t ym = td_mean_key(u[b].sum, u[b].cum);
      const bool after = ym > xm || (ym == xm && (u[b].cum > x.cum ||
                                                  (u[b].cum == x.cum && td_key(__double_as_longlong(u[b].sum)) > xs)));
      if (!after) break;
      u[b + 1] = u[b];
      b--;
    }
    u[b + 1] = x;
  }
  int64_t cum = 0;
  for (int32_t a = 0; a < m; a++) {
    cum += u[a].cum;
    u[a].cum = cum;
  }
}

// a late firing's row: the quantiles of the scratch digest cp[0, n) of weight wt (and the digest, when exported)
__device__ void td_late_emit(const SlowCtx& x, const Entry& en, const TdCent* cp, int32_t n, int64_t wt) {
  const DevCfg& c = x.c;
  const unsigned long long pos = atomicAdd(&x.st->out_rows, 1ull);
  if ((int64_t)pos >= x.out.cap) {
    atomicOr(&x.st->flags, FW_STATUS_OUT_FULL);
    return;
  }
  write_row(c, x.out, pos, en);
  const double mn = __longlong_as_double(x.out.mn[pos]), mx = __longlong_as_double(x.out.mx[pos]);
  x.out.sum[pos] = __double_as_longlong(td_quantile(cp, n, wt, mn, mx, c.td_quant[0]));
  x.out.mn[pos] = __double_as_longlong(td_quantile(cp, n, wt, mn, mx, c.td_quant[1]));
  x.out.mx[pos] = __double_as_longlong(td_quantile(cp, n, wt, mn, mx, c.td_quant[2]));
  if (x.out.dig) {
    int64_t* d = x.out.dig + pos * (1 + 2 * (int64_t)c.td_nb);
    d[0] = n;
    for (int32_t k = 0; k < n; k++) {
      d[1 + 2 * k] = __double_as_longlong(cp[k].sum);
      d[2 + 2 * k] = td_weight(cp, k);
    }
  }
  atomicAdd(&x.st->td_cent, (unsigned long long)n);
}

// FIRE_AND_PURGE of a t-digest window in the ordered path (allowed lateness; WindowOperator.java:403-405
// windowState.clear() after a FIRE_AND_PURGE): the state goes -- the block's centroids, those of the blocks merged into
// it during the push (a session: their union is then empty, td_late_row_session and k_td_mbuild), and the values the
// push added to it so far, whose items leave the push's compression (TD_DROPPED: k_td_group and k_td_relink skip them).
// The slot and block stay as empty state (cnt 0) until the window's cleanup time.
__device__ void td_purge(const DevCfg& c, uint32_t g, uint64_t blk) {
  for (int32_t l = c.td_olast[g]; l >= 0;) {
    const int32_t nx = c.td_olink[l];
    c.td_olink[l] = TD_DROPPED;
    l = nx;
  }
  c.td_olast[g] = -1;
  TdHead* h = td_head(c, blk);
  *h = TdHead{h->cur, 0, 0};
  if (c.td_bhead)
    for (int32_t b = c.td_bhead[blk]; b >= 0; b = c.td_bnext[b]) {
      TdHead* hb = td_head(c, (uint64_t)b);
      *hb = TdHead{hb->cur, 0, 0};
    }
}

// a session's late firing (allowed lateness): as td_late_row, over the session's digest -- its block's centroids and
// those of the blocks merged into it during the push (td_bhead chain: their union, as td_union, in the thread's
// td_lateu scratch) -- compressed with the values the push added to it so far (its sorted chain from `head`, merged
// sessions' chains joined in)
__device__ void td_late_row_session(const SlowCtx& x, const Entry& en, int32_t head) {
  const DevCfg& c = x.c;
  int64_t L = 0;
  for (int32_t l = head; l >= 0; l = c.td_olink[l]) L++;
  const uint64_t blk = pool_block_of(en);
  const TdHead h = *td_head(c, blk);
  const TdCent* old = td_half(c, blk, h.cur);
  int32_t no = h.n;
  int64_t wold = h.w;
  if (c.td_bhead[blk] >= 0) {  // merged digests: their union
    TdCent* u = c.td_lateu + (int64_t)threadIdx.x * c.td_lateu_cap;
    int32_t m = 0;
    wold = 0;
    bool over = false;
    for (int32_t b = (int32_t)blk; b >= 0 && !over; b = b == (int32_t)blk ? c.td_bhead[blk] : c.td_bnext[b]) {
      const TdHead hb = *td_head(c, (uint64_t)b);
      const TdCent* ce = td_half(c, (uint64_t)b, hb.cur);
      if (m + hb.n > c.td_lateu_cap) {
        over = true;
        break;
      }
      for (int32_t q = 0; q < hb.n; q++) u[m++] = TdCent{ce[q].sum, td_weight(ce, q)};
      wold += hb.w;
    }
    if (over) {
      atomicOr(&x.st->flags, FW_STATUS_TD_UNION);
      return;
    }
    td_union_sort(u, m);
    old = u;
    no = m;
  }
  TdCent* cp = c.td_late + (int64_t)threadIdx.x * c.td_nb;
  int32_t at = head;
  auto next = [&]() -> uint64_t {
    const uint64_t key = td_key(c.td_ovv[at]);
    at = c.td_olink[at];
    return key;
  };
  const int32_t n = td_merge_run(c, c.td_qb, next, L, old, no, cp, wold + L);
  td_late_emit(x, en, cp, n, wold + L);
}

// getResult of a window that fires on an element of the ordered path (allowed lateness) while the push's values
// are still buffered: as window_oracle.cpp emit, a copy of the digest -- its centroids compressed with the window's
// values of this push so far, the sorted chain from `head` -- gives the quantiles (one thread of k_slow; the copy
// goes to the thread's td_late scratch).
__device__ void td_late_row(const SlowCtx& x, const Entry& en, int32_t head) {
  const DevCfg& c = x.c;
  int64_t L = 0;
  for (int32_t l = head; l >= 0; l = c.td_olink[l]) L++;
  const uint64_t blk = pool_block_of(en);
  const TdHead h = *td_head(c, blk);
  const TdCent* old = td_half(c, blk, h.cur);
  TdCent* cp = c.td_late + (int64_t)threadIdx.x * c.td_nb;
  int32_t at = head;
  auto next = [&]() -> uint64_t {  // (the chain is in value order: td_chain_insert)
    const uint64_t key = td_key(c.td_ovv[at / c.wpr]);
    at = c.td_olink[at];
    return key;
  };
  const int64_t wt = h.w + L;
  const int32_t n = td_merge_run(c, c.td_qb, next, L, old, h.n, cp, wt);
  td_late_emit(x, en, cp, n, wt);
}

// getResult of a fired row (one thread): out.sum holds the block id and above it 1 + the block's free-stack slot
// past `stack_base` if its window goes (k_fire) and TD_PURGE_TAG if it stays emptied, out.min / out.max the min /
// max; returns the digest's centroid count
__device__ int32_t td_finish(const DevCfg& c, const DevRows& out, uint64_t row, int64_t stack_base) {
  const uint64_t tag = (uint64_t)out.sum[row];
  const uint64_t blk = tag & 0xffffffffull;
  const int64_t rel = (int64_t)((tag & ~TD_PURGE_TAG) >> 32);
  const TdHead h = *td_head(c, blk);
  const TdCent* ce = td_half(c, blk, h.cur);
  const double mn = __longlong_as_double(out.mn[row]), mx = __longlong_as_double(out.mx[row]);
  const double q0 = td_quantile(ce, h.n, h.w, mn, mx, c.td_quant[0]);
  const double q1 = td_quantile(ce, h.n, h.w, mn, mx, c.td_quant[1]);
  const double q2 = td_quantile(ce, h.n, h.w, mn, mx, c.td_quant[2]);
  if (out.dig) {
    int64_t* d = out.dig + row * (1 + 2 * (int64_t)c.td_nb);
    d[0] = h.n;
    for (int32_t k = 0; k < h.n; k++) {
      d[1 + 2 * k] = __double_as_longlong(ce[k].sum);
      d[2 + 2 * k] = td_weight(ce, k);
    }
  }
  out.sum[row] = __double_as_longlong(q0);
  out.mn[row] = __double_as_longlong(q1);
  out.mx[row] = __double_as_longlong(q2);
  if (rel) c.pool_free[stack_base + rel - 1] = (uint32_t)blk;
  if (tag & TD_PURGE_TAG) *td_head(c, blk) = TdHead{h.cur, 0, 0};  // FIRE_AND_PURGE: the session stays, empty
  return h.n;
}

// the slot of key's in-flight session that contains [ts, ts + gap) (sessions hash the key only: one probe chain),
// -1 if none
__device__ __forceinline__ int32_t session_containing(const Region& r, const DevCfg& c, int64_t key, int64_t ts) {
  const uint64_t h = slot_hash(c, key, 0);
  const uint32_t want = live_word(h);
  const int64_t te = jadd(ts, c.gap);
  for (uint32_t k = 0; k <= r.mask; k++) {
    const uint32_t s = ((uint32_t)h + k) & r.mask;
    const uint32_t w = r.state[s];
    if (w == SLOT_EMPTY) return -1;
    if (w != want) continue;
    const Entry& e = r.ent[s];
    if (e.key == key && e.start <= ts && te <= e.end) return (int32_t)s;
  }
  return -1;
}
// ---- t-digest: the batch's values grouped by digest and sorted within each digest (launch_tdigest).  The tiers want
// every touched digest's values of the push as one run in Double.compare order: v[0] from tbeg[i] for the digest
// tslot[i], gsort the digest of every position.  The batch is already grouped by state partition, so instead of a
// whole-batch LSD radix sort (8 passes over 12-byte pairs):
//   k_td_group   every item's digest (the region lookup) and value key; a workgroup's items counted per digest in an
//                LDS table, then one global add per (workgroup, digest) on dcnt[digest] gives the workgroup's place in
//                the digest's run (the first add lists the digest as touched); every item keeps (digest, rank)
//   runs         a scan over the touched digests' counts: the runs' starts (tbeg), written back into dcnt
//   k_td_place   every item to its place in its digest's run (v[1], gsort)
//   sorts        runs of <= 16 values by 16 lanes, of <= 64 by a wave (bitonic networks over the lanes), of
//                <= TD_SORT_MAX by a workgroup in LDS; longer runs (the hot keys) are split first by MSD passes on
//                their highest differing key bits into bins of about TD_SORT_MAX / 2 values (two levels), whatever is
//                still longer by a workgroup's bitonic network in global memory (a fallback)
// Every comparison is on the full 64-bit key: equal keys are equal values, so no tie fix-up is needed.
constexpr int TD_GCHUNK = 4096;     // items per k_td_group workgroup (a digest's rank among them: 12 bits)
constexpr int TD_GTHREADS = 1024;   // (its 64-KB table: two workgroups, 32 waves per CU for the region lookups)
constexpr int TD_GHASH_LOG = 13;
constexpr int TD_GHASH = 1 << TD_GHASH_LOG;  // its LDS table of digests (at most TD_GCHUNK of them)
constexpr uint32_t TD_GEMPTY = 0xffffffffu;
constexpr int TD_SORT_MAX = 4096;   // values a workgroup sorts in LDS
constexpr int TD_TILE_PT = 16;      // MSD tile: values per thread
constexpr int TD_TILE = 256 * TD_TILE_PT;
constexpr int TD_MSD_BINS = 4096;  // per run: its sample sort's buckets (at most 2 * 2047 + 1)
constexpr uint32_t TD_RUN_V1 = 0x80000000u;  // TdRun.len: the run's values are in v[1]

// the digest's LDS slot in the workgroup's table, and this item's rank among the workgroup's items of the digest
__device__ __forceinline__ uint32_t td_group_rank(uint32_t* hk, uint32_t* hc, uint32_t g) {
  uint32_t h = (g * 0x9E3779B1u) >> (32 - TD_GHASH_LOG);
  while (true) {
    const uint32_t cur = __hip_atomic_load(&hk[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (cur == g) break;
    if (cur == TD_GEMPTY) {
      const uint32_t prev = atomicCAS(&hk[h], TD_GEMPTY, g);
      if (prev == TD_GEMPTY || prev == g) break;
    }
    h = (h + 1) & (TD_GHASH - 1);
  }
  // a hot digest's items (a Zipf stream's head keys fill whole chunks): the lanes of the wave that share the
  // first active lane's digest take their ranks from one LDS add
  const uint64_t act = __ballot(1);
  const int lead = __ffsll((long long)act) - 1;
  const uint32_t hl = (uint32_t)__shfl((int)h, lead, 64);
  const uint64_t peers = __ballot(h == hl);
  uint32_t rank;
  if (h == hl) {
    uint32_t base = 0;
    if ((int)__lane_id() == lead) base = atomicAdd(&hc[h], (uint32_t)__popcll(peers));
    base = (uint32_t)__shfl((int)base, lead, 64);
    rank = base + (uint32_t)__popcll(peers & lanemask_lt());
  } else {
    rank = atomicAdd(&hc[h], 1u);
  }
  return (h << 12) | rank;
}
#ifndef FW_TDG_U
#define FW_TDG_U 4  // k_td_group's one-window form: items per thread with their lookups in flight together
#endif
// FAST: one window per record (tumbling), no session, no lateness (no values beyond the batch's records): a
// thread's FW_TDG_U items go through the lookup together -- records, then home slots, then the entries -- as
// k_hll_update does, instead of one dependent chain of loads per item
template <bool FAST>
__global__ __launch_bounds__(TD_GTHREADS) void k_td_group(DevCfg c, const PRec* __restrict__ part, const uint32_t* __restrict__ offs,
                                                  int32_t T, int64_t n, int32_t rchunk, DevTable tb, uint32_t none,
                                                  TdBuf td, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  __shared__ uint32_t hk[TD_GHASH], hc[TD_GHASH];
  __shared__ int32_t p0_s;
  const int64_t total = offs[(int64_t)c.P * T];
  const int64_t i0 = (int64_t)blockIdx.x * rchunk;
  const int64_t i1 = min(n, i0 + (int64_t)rchunk);
  const int W = c.assigner == FW_SLIDING ? c.wpr : 1;
  for (int h = threadIdx.x; h < TD_GHASH; h += blockDim.x) {
    hk[h] = TD_GEMPTY;
    hc[h] = 0u;
  }
  if (threadIdx.x == 0) {  // partition of the chunk's first record: last p with offs[p*T] <= i0
    int32_t lo = 0, hi = c.P - 1;
    while (lo < hi) {
      const int32_t mid = (lo + hi + 1) >> 1;
      if ((int64_t)offs[(int64_t)mid * T] <= i0)
        lo = mid;
      else
        hi = mid - 1;
    }
    p0_s = lo;
  }
  __syncthreads();
  const bool cmp = c.compact && !*c.wide;
  const bool sess = c.assigner == FW_SESSION;
  const int64_t nov = c.td_ovctr ? (int64_t)*c.td_ovctr : 0;
  uint32_t* __restrict__ gs0 = td.gs[0];
  uint32_t* __restrict__ gs1 = td.gs[1];
  int32_t pp = p0_s;
  if constexpr (FAST) {
    constexpr int GU = FW_TDG_U;
    const int64_t iend = min(i1, total);
    for (int64_t ib = i0 + threadIdx.x; ib < i1; ib += (int64_t)blockDim.x * GU) {
      int64_t key[GU], last[GU], val[GU];
      int32_t rp[GU];
      bool in[GU];
#pragma unroll
      for (int u = 0; u < GU; u++) {
        const int64_t i = ib + (int64_t)u * blockDim.x;
        in[u] = i < iend;
        rp[u] = pp;
        key[u] = last[u] = val[u] = 0;
        if (!in[u]) continue;
        while ((int64_t)offs[(int64_t)(pp + 1) * T] <= i) pp++;
        rp[u] = pp;
        if (cmp) {
          const i64x2 r = reinterpret_cast<const i64x2*>(part)[i];
          key[u] = r.x;  // (the compact word: decoded below, once every load is in flight)
          val[u] = r.y;
        } else {
          const PRec rec = part[i];
          key[u] = rec.key;
          last[u] = rec.last;
          val[u] = rec.val;
        }
      }
      uint64_t hs[GU];
      uint32_t hw[GU];
      i64x2 hk2[GU];
      int64_t hend[GU], hmeta[GU];
      Region rg[GU];
#pragma unroll
      for (int u = 0; u < GU; u++) {
        if (cmp && in[u]) compact_decode(c, rp[u], key[u], &key[u], &last[u]);
        rg[u] = region_of(c, tb, rp[u], tb.cur[rp[u]]);
        hs[u] = slot_hash(c, key[u], last[u]);
        hw[u] = SLOT_EMPTY;
        if (!in[u]) continue;
        const uint32_t home = (uint32_t)hs[u] & rg[u].mask;
        hw[u] = rg[u].state[home];  // (the table is read-only here: plain reads)
        hk2[u] = *reinterpret_cast<const i64x2*>(&rg[u].ent[home].key);
        hend[u] = rg[u].ent[home].end;
        hmeta[u] = rg[u].ent[home].meta;
      }
#pragma unroll
      for (int u = 0; u < GU; u++) {
        const int64_t i = ib + (int64_t)u * blockDim.x;
        if (!in[u]) {
          if (i < i1) gs0[i] = none;
          continue;
        }
        const int64_t we = wend(c, last[u]);
        int32_t slot;
        uint64_t blk;
        const uint32_t home = (uint32_t)hs[u] & rg[u].mask;
        if (hw[u] == live_word(hs[u]) && hk2[u].x == key[u] && hk2[u].y == last[u] && hend[u] == we) {
          slot = (int32_t)home;
          blk = (uint64_t)hmeta[u] >> 1;
        } else {
          slot = hw[u] == SLOT_EMPTY ? -1 : region_find(rg[u], hs[u], key[u], last[u], we);
          blk = slot < 0 ? 0 : pool_block_of(rg[u].ent[slot]);
        }
        if (slot < 0) {
          atomicOr(&st->flags, FW_STATUS_STATE_LOST);  // the aggregate stored every record's window
          gs0[i] = none;
          continue;
        }
        const uint32_t g = ((uint32_t)rp[u] << c.log_r) | (uint32_t)slot;
        if (td.binv[blk] != g) td.binv[blk] = g;
        td.v[0][i] = td_key(val[u]);
        gs0[i] = g;
        gs1[i] = td_group_rank(hk, hc, g);
      }
    }
  } else
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    int nw = 0;
    if (i < total + nov) {
      PRec rec;
      int32_t rp;
      if (i < total) {
        while ((int64_t)offs[(int64_t)(pp + 1) * T] <= i) pp++;
        rp = pp;
        if (cmp) {
          const i64x2 r = reinterpret_cast<const i64x2*>(part)[i];
          compact_decode(c, pp, r.x, &rec.key, &rec.last);
          rec.val = r.y;
          rec.nwin = 1;
        } else {
          rec = part[i];
        }
      } else {
        const int64_t j = i - total;
        rec.key = c.td_ovk[j];
        rec.last = c.td_ovt[j];
        rec.val = c.td_ovv[j];
        rec.nwin = c.td_ovn ? c.td_ovn[j] : 1;
        rp = c.td_ovp[j];
      }
      nw = W == 1 ? 1 : (int)(rec.nwin & 0xffff);
      const Region r = region_of(c, tb, rp, tb.cur[rp]);
      const uint64_t k = td_key(rec.val);
      for (int wi = 0; wi < nw; wi++) {
        const int64_t o = i * W + wi;
        if (i >= total && c.td_olink && c.td_olink[(i - total) * c.wpr + wi] == TD_DROPPED) {  // purged (td_purge)
          gs0[o] = none;
          continue;
        }
        const int64_t s = jsub(rec.last, (int64_t)wi * c.slide);
        const int32_t slot = sess ? session_containing(r, c, rec.key, rec.last) :
                                    region_find(r, slot_hash(c, rec.key, s), rec.key, s, wend(c, s));
        if (slot < 0) {
          atomicOr(&st->flags, FW_STATUS_STATE_LOST);  // the aggregate stored every record's window
          gs0[o] = none;
          continue;
        }
        const uint32_t g = ((uint32_t)rp << c.log_r) | (uint32_t)slot;
        const uint64_t blk = pool_block_of(r.ent[slot]);
        if (td.binv[blk] != g) td.binv[blk] = g;
        td.v[0][o] = k;
        gs0[o] = g;
        gs1[o] = td_group_rank(hk, hc, g);
      }
    }
    for (int wi = nw; wi < W; wi++) gs0[i * W + wi] = none;
  }
  __syncthreads();
  // per digest of the workgroup one global add (all of a thread's in flight together); the digest's first workgroup
  // (the add returned 0) lists it as touched, with one list reservation per workgroup
  constexpr int HU = TD_GHASH / TD_GTHREADS;
  uint32_t base[HU];
  uint32_t firsts = 0;
#pragma unroll
  for (int u = 0; u < HU; u++) {
    const int h = u * TD_GTHREADS + (int)threadIdx.x;
    const uint32_t g = hk[h];
    base[u] = g != TD_GEMPTY ? atomicAdd(&td.dcnt[g], hc[h]) : 1u;
  }
#pragma unroll
  for (int u = 0; u < HU; u++) firsts += base[u] == 0u;
  __shared__ uint32_t sw[TD_GTHREADS / 64 + 1];
  __shared__ uint32_t lbase_s;
  uint32_t ftotal;
  uint32_t fpos = block_excl_scan(firsts, sw, &ftotal);
  if (threadIdx.x == 0) lbase_s = ftotal ? (uint32_t)atomicAdd(&td.ctr[0], (int)ftotal) : 0u;
  __syncthreads();
  fpos += lbase_s;
#pragma unroll
  for (int u = 0; u < HU; u++) {
    const int h = u * TD_GTHREADS + (int)threadIdx.x;
    if (base[u] == 0u) td.tslot[fpos++] = hk[h];
    hc[h] = base[u];
  }
  __syncthreads();
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x)  // (the items this thread wrote)
    for (int wi = 0; wi < W; wi++) {
      const int64_t o = i * W + wi;
      if (gs0[o] == none) continue;
      const uint32_t x = gs1[o];
      gs1[o] = hc[x >> 12] + (x & 4095u);
    }
}
// The serial tier takes one digest per thread, and a wave lasts as long as its longest merge: the touched digests go
// to it longest first, by classes of their batch run's length (1, 2, 3-4, ..., 65+; a digest's old centroids grow with
// its key's frequency as its values do, and every window of the push is at the same point of its span).
// lctr[TD_LC_CNT + k]: the class's digests, lctr[TD_LC_CUR + k]: its placement cursor; the order is td.gs[1]
// (free once k_td_place has read the ranks).
constexpr int TD_NCLS = 8;
constexpr int TD_LC_CNT = 5, TD_LC_CUR = TD_LC_CNT + TD_NCLS, TD_LC_WORDS = TD_LC_CUR + TD_NCLS;
static_assert(TD_LC_WORDS == FW_TD_LC_WORDS, "TdBuf::lctr's allocation");
__device__ __forceinline__ int td_len_class(uint32_t len) {
  return len <= 1 ? 0 : min(TD_NCLS - 1, 32 - __clz((int)(len - 1)));
}
// a wave's count of its lanes' class k items (every lane gets the counts of all TD_NCLS classes: c[k])
__device__ __forceinline__ void td_class_ballots(bool valid, int k, uint64_t (&m)[TD_NCLS]) {
#pragma unroll
  for (int q = 0; q < TD_NCLS; q++) m[q] = __ballot(valid && k == q);
}
// the touched digests' counts (tbeg[nt] = 0), scanned in place by the device-sized scan below, and counted by length
// class (per wave by ballots, one LDS add per wave and class, one global add per workgroup)
__global__ __launch_bounds__(256) void k_td_counts(TdBuf td, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  __shared__ int32_t ccnt[TD_NCLS];
  if (threadIdx.x < TD_NCLS) ccnt[threadIdx.x] = 0;
  __syncthreads();
  const int32_t nt = td.ctr[0];
  int32_t wc[TD_NCLS] = {};
  for (int32_t i0 = blockIdx.x * blockDim.x; i0 <= nt; i0 += gridDim.x * blockDim.x) {  // (whole waves iterate)
    const int32_t i = i0 + threadIdx.x;
    const uint32_t len = i < nt ? td.dcnt[td.tslot[i]] : 0u;
    if (i <= nt) td.tbeg[i] = len;
    uint64_t m[TD_NCLS];
    td_class_ballots(i < nt, td_len_class(len), m);
#pragma unroll
    for (int q = 0; q < TD_NCLS; q++) wc[q] += __popcll(m[q]);
  }
  if (__lane_id() == 0)
#pragma unroll
    for (int q = 0; q < TD_NCLS; q++)
      if (wc[q]) atomicAdd(&ccnt[q], wc[q]);
  __syncthreads();
  if (threadIdx.x < TD_NCLS && ccnt[threadIdx.x]) atomicAdd(&td.lctr[TD_LC_CNT + threadIdx.x], ccnt[threadIdx.x]);
}
// k_scan_* over data[0 .. *mdev] (the length read on the device)
__global__ __launch_bounds__(SCAN_T) void k_scan_blocks_d(uint32_t* data, const int32_t* mdev, uint32_t* sums) {
  const int64_t m = (int64_t)*mdev + 1;
  if ((int64_t)blockIdx.x * SCAN_B >= m) return;
  __shared__ uint32_t sw[SCAN_T / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * SCAN_B + (int64_t)threadIdx.x * SCAN_E;
  uint32_t v[SCAN_E];
  uint32_t local = 0;
#pragma unroll
  for (int e = 0; e < SCAN_E; e++) {
    v[e] = base + e < m ? data[base + e] : 0u;
    local += v[e];
  }
  uint32_t total;
  uint32_t off = block_excl_scan(local, sw, &total);
#pragma unroll
  for (int e = 0; e < SCAN_E; e++) {
    if (base + e < m) data[base + e] = off;
    off += v[e];
  }
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}
__global__ __launch_bounds__(SCAN_T) void k_scan_top_d(uint32_t* sums, const int32_t* mdev) {
  const int64_t nb = ((int64_t)*mdev + 1 + SCAN_B - 1) / SCAN_B;
  __shared__ uint32_t sw[SCAN_T / 64 + 1];
  uint32_t carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += SCAN_T) {
    const int64_t i = b0 + threadIdx.x;
    uint32_t v = i < nb ? sums[i] : 0u, total;
    uint32_t off = block_excl_scan(v, sw, &total);
    if (i < nb) sums[i] = off + carry;
    carry += total;
  }
}
__global__ __launch_bounds__(SCAN_T) void k_scan_add_d(uint32_t* data, const int32_t* mdev, const uint32_t* sums) {
  const int64_t m = (int64_t)*mdev + 1;
  const int64_t base = (int64_t)blockIdx.x * SCAN_B;
  if (base >= m) return;
  const uint32_t add = sums[blockIdx.x];
  for (int e = threadIdx.x; e < SCAN_B; e += SCAN_T)
    if (base + e < m) data[base + e] += add;
}
// a wave's appends to a run list: one reservation per wave (the lanes with `want`)
__device__ __forceinline__ void td_list_put(TdRun* list, int32_t* ctr, bool want, TdRun r) {
  const uint64_t m = __ballot(want);
  if (!m) return;
  const int lead = __ffsll((long long)m) - 1;
  int base = 0;
  if ((int)__lane_id() == lead) base = atomicAdd(ctr, __popcll(m));
  base = __shfl(base, lead, 64);
  if (want) list[base + __popcll(m & lanemask_lt())] = r;
}
// the runs' starts into dcnt (read by k_td_place), and the long runs listed for the LDS sort / the MSD passes
__global__ __launch_bounds__(256) void k_td_starts(TdBuf td, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int32_t nt = td.ctr[0];
  for (int32_t i0 = blockIdx.x * blockDim.x; i0 < nt; i0 += gridDim.x * blockDim.x) {  // (whole waves iterate)
    const int32_t i = i0 + threadIdx.x;
    uint32_t beg = 0, len = 0;
    if (i < nt) {
      beg = td.tbeg[i];
      len = td.tbeg[i + 1] - beg;
      td.dcnt[td.tslot[i]] = beg;
    }
    td_list_put(td.brun[0], &td.lctr[1], len > TD_SORT_MAX, TdRun{beg, len | TD_RUN_V1});
    td_list_put(td.lrun, &td.lctr[0], len > 64 && len <= TD_SORT_MAX, TdRun{beg, len | TD_RUN_V1});
  }
}
// the touched digests in class order, longest class first, into td.gs[1]: a workgroup takes TD_PERM_CH of them
// (TD_PERM_PT a thread), counts them per wave and class, reserves each class's share with one global add, and places
// them in wave order
constexpr int TD_PERM_PT = 16, TD_PERM_CH = 256 * TD_PERM_PT;
__global__ __launch_bounds__(256) void k_td_perm(TdBuf td, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  __shared__ int32_t wcnt[4][TD_NCLS], wb[4][TD_NCLS];
  const int32_t nt = td.ctr[0];
  const int32_t c0 = blockIdx.x * TD_PERM_CH;
  if (c0 >= nt) return;
  const int wv = threadIdx.x >> 6, lane = __lane_id();
  int cls[TD_PERM_PT];
  int32_t run[TD_NCLS] = {};
#pragma unroll
  for (int j = 0; j < TD_PERM_PT; j++) {
    const int32_t i = c0 + j * 256 + (int32_t)threadIdx.x;
    cls[j] = i < nt ? td_len_class(td.tbeg[i + 1] - td.tbeg[i]) : 0;
    uint64_t m[TD_NCLS];
    td_class_ballots(i < nt, cls[j], m);
#pragma unroll
    for (int q = 0; q < TD_NCLS; q++) run[q] += __popcll(m[q]);
  }
  if (lane < TD_NCLS) {
    int32_t x = run[0];
#pragma unroll
    for (int q = 1; q < TD_NCLS; q++) x = lane == q ? run[q] : x;
    wcnt[wv][lane] = x;
  }
  __syncthreads();
  if (threadIdx.x < TD_NCLS) {
    const int k = (int)threadIdx.x;
    int32_t base = 0;  // the longer classes' digests come first
    for (int q = TD_NCLS - 1; q > k; q--) base += td.lctr[TD_LC_CNT + q];
    const int32_t tot = wcnt[0][k] + wcnt[1][k] + wcnt[2][k] + wcnt[3][k];
    int32_t at = base + (tot ? atomicAdd(&td.lctr[TD_LC_CUR + k], tot) : 0);
    for (int w = 0; w < 4; w++) {
      wb[w][k] = at;
      at += wcnt[w][k];
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < TD_NCLS; q++) run[q] = 0;
#pragma unroll
  for (int j = 0; j < TD_PERM_PT; j++) {
    const int32_t i = c0 + j * 256 + (int32_t)threadIdx.x;
    uint64_t m[TD_NCLS];
    td_class_ballots(i < nt, cls[j], m);
    int32_t pos = 0;
#pragma unroll
    for (int q = 0; q < TD_NCLS; q++) {
      if (cls[j] == q) pos = wb[wv][q] + run[q] + __popcll(m[q] & lanemask_lt());
      run[q] += __popcll(m[q]);
    }
    if (i < nt) td.gs[1][pos] = (uint32_t)i;
  }
}
// every item to its run (v[1]) and its digest to gsort; positions past the runs get `none`
__global__ __launch_bounds__(256) void k_td_place(TdBuf td, int64_t n, uint32_t none, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int64_t placed = td.tbeg[td.ctr[0]];
  for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < n; o += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t g = td.gs[0][o];
    if (g != none) {
      const uint32_t pos = td.dcnt[g] + td.gs[1][o];
      td.v[1][pos] = td.v[0][o];
      td.gsort[pos] = g;
    }
    if (o >= placed) td.gsort[o] = none;
  }
}
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t x, int m, int w) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x, m, w), hi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), m, w);
  return ((uint64_t)hi << 32) | lo;
}
// the runs of <= 16 (G = 16: four runs a wave) or 17..64 values (G = 64) sorted by a bitonic network over G lanes
// (the "flip" form: every compare-exchange puts the smaller key at the lower index, so the lanes past the run hold
// the largest key and stay there)
template <int G>
__global__ __launch_bounds__(256) void k_td_sort_lanes(TdBuf td, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int lane = (int)(threadIdx.x & (G - 1));
  const int64_t groups = ((int64_t)gridDim.x * blockDim.x) / G;
  // only the runs of this length: their length classes' stretch of k_td_perm's order (classes 0-4: <= 16 values,
  // 5-6: 17 .. 64; longer classes first)
  int32_t lo = 0, hi = 0;
  for (int k = TD_NCLS - 1; k >= 0; k--) {
    const int32_t cnt = td.lctr[TD_LC_CNT + k];
    if (G == 16 ? k >= 5 : k >= 7) lo += cnt;
    if (G == 16 ? true : k >= 5) hi += cnt;
  }
  for (int64_t pos = lo + ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G; pos < hi; pos += groups) {
    const int32_t d = (int32_t)td.gs[1][pos];
    const uint32_t beg = td.tbeg[d], len = td.tbeg[d + 1] - beg;
    uint64_t x = (uint32_t)lane < len ? td.v[1][beg + lane] : ~0ull;
#pragma unroll
    for (int k = 2; k <= G; k <<= 1) {
      {
        const uint64_t y = shfl_xor_u64(x, k - 1, G);
        x = (lane & (k >> 1)) ? max(x, y) : min(x, y);
      }
#pragma unroll
      for (int j = k >> 2; j > 0; j >>= 1) {
        const uint64_t y = shfl_xor_u64(x, j, G);
        x = (lane & j) ? max(x, y) : min(x, y);
      }
    }
    if ((uint32_t)lane < len) td.v[0][beg + lane] = x;
  }
}
// bitonic network ("flip" form) over keys a[0 .. len) in LDS, by the workgroup; positions >= len are +infinity
__device__ void td_bitonic_lds(uint64_t* a, uint32_t len) {
  uint32_t n2 = 1;
  while (n2 < len) n2 <<= 1;
  for (uint32_t k = 2; k <= n2; k <<= 1) {
    const uint32_t hk = k >> 1;
    for (uint32_t t = threadIdx.x; t < (n2 >> 1); t += blockDim.x) {
      const uint32_t i = (t & ~(hk - 1)) * 2 + (t & (hk - 1)), p = i ^ (k - 1);
      if (p < len) {
        const uint64_t x = a[i], y = a[p];
        if (x > y) {
          a[i] = y;
          a[p] = x;
        }
      }
    }
    __syncthreads();
    for (uint32_t j = k >> 2; j > 0; j >>= 1) {
      for (uint32_t t = threadIdx.x; t < (n2 >> 1); t += blockDim.x) {
        const uint32_t i = (t & ~(j - 1)) * 2 + (t & (j - 1)), p = i + j;
        if (p < len) {
          const uint64_t x = a[i], y = a[p];
          if (x > y) {
            a[i] = y;
            a[p] = x;
          }
        }
      }
      __syncthreads();
    }
  }
}
// the same network with the first stages in registers: thread t holds keys [t E, t E + E) of the n2 = 256 E padded
// positions, so every stage whose partner distance is below E (the flip stages of blocks up to E, and the low
// half-cleaners) runs on its registers; only the longer stages go through the LDS (by the workgroup's 256 threads)
template <int E>
__device__ __forceinline__ void td_cswap(uint64_t& a, uint64_t& b) {
  const uint64_t x = min(a, b), y = max(a, b);
  a = x;
  b = y;
}
template <int E>
__device__ void td_bitonic_reg(uint64_t* a, uint32_t len) {
  constexpr uint32_t n2 = 256u * E;
  const uint32_t t0 = threadIdx.x * E;
  uint64_t x[E];
#pragma unroll
  for (int e = 0; e < E; e++) x[e] = t0 + e < len ? a[t0 + e] : ~0ull;
  for (uint32_t k = 2; k <= n2; k <<= 1) {
    if (k > (uint32_t)E) {  // the flip stage and the half-cleaners of distance >= E through the LDS
#pragma unroll
      for (int e = 0; e < E; e++) a[t0 + e] = x[e];
      __syncthreads();
      const uint32_t hk = k >> 1;
      for (uint32_t t = threadIdx.x; t < (n2 >> 1); t += blockDim.x) {
        const uint32_t i = (t & ~(hk - 1)) * 2 + (t & (hk - 1)), p = i ^ (k - 1);
        const uint64_t u = a[i], v = a[p];
        if (u > v) {
          a[i] = v;
          a[p] = u;
        }
      }
      __syncthreads();
      for (uint32_t j = k >> 2; j >= (uint32_t)E; j >>= 1) {
        for (uint32_t t = threadIdx.x; t < (n2 >> 1); t += blockDim.x) {
          const uint32_t i = (t & ~(j - 1)) * 2 + (t & (j - 1)), p = i + j;
          const uint64_t u = a[i], v = a[p];
          if (u > v) {
            a[i] = v;
            a[p] = u;
          }
        }
        __syncthreads();
      }
#pragma unroll
      for (int e = 0; e < E; e++) x[e] = a[t0 + e];
      __syncthreads();
    } else {  // the flip stage of a block inside the thread's keys
#pragma unroll
      for (int e = 0; e < E; e++) {
        const int p = e ^ (int)(k - 1);
        if (e < p) td_cswap<E>(x[e], x[p]);
      }
    }
#pragma unroll
    for (int j = E >> 1; j > 0; j >>= 1) {  // the half-cleaners of distance < E (those below k / 2)
      if ((uint32_t)j > (k >> 2)) continue;
#pragma unroll
      for (int e = 0; e < E; e++) {
        const int p = e ^ j;
        if (e < p) td_cswap<E>(x[e], x[p]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; e++) a[t0 + e] = x[e];
  __syncthreads();
}
// The same network with the stages inside a wave on shuffles: thread t holds keys [t E, t E + E), so a wave holds 64 E
// consecutive positions; a stage whose partner distance is below E runs on the thread's registers, below 64 E on
// cross-lane shuffles (no barrier), and only the longer ones (the last two levels of a 256-thread workgroup's sort)
// through the LDS.
template <int E, int NT>
__device__ __forceinline__ void td_lds_stages(uint64_t* a, uint64_t (&x)[E], uint32_t k, bool flip, uint32_t jlo) {
  constexpr uint32_t n2 = (uint32_t)NT * E;
  const uint32_t t0 = threadIdx.x * E;
#pragma unroll
  for (int e = 0; e < E; e++) a[t0 + e] = x[e];
  __syncthreads();
  if (flip) {
    const uint32_t hk = k >> 1;
    for (uint32_t t = threadIdx.x; t < (n2 >> 1); t += blockDim.x) {
      const uint32_t i = (t & ~(hk - 1)) * 2 + (t & (hk - 1)), p = i ^ (k - 1);
      const uint64_t u = a[i], v = a[p];
      if (u > v) {
        a[i] = v;
        a[p] = u;
      }
    }
    __syncthreads();
  }
  for (uint32_t j = flip ? k >> 2 : k; j >= jlo && j > 0; j >>= 1) {
    for (uint32_t t = threadIdx.x; t < (n2 >> 1); t += blockDim.x) {
      const uint32_t i = (t & ~(j - 1)) * 2 + (t & (j - 1)), p = i + j;
      const uint64_t u = a[i], v = a[p];
      if (u > v) {
        a[i] = v;
        a[p] = u;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int e = 0; e < E; e++) x[e] = a[t0 + e];
  __syncthreads();
}
template <int E, int NT = 256>
__device__ void td_bitonic_wave(uint64_t* a, uint32_t len) {  // (NT: the workgroup's threads)
  constexpr uint32_t n2 = (uint32_t)NT * E, WSPAN = 64u * E;
  constexpr int LE = E == 1 ? 0 : E == 2 ? 1 : E == 4 ? 2 : E == 8 ? 3 : 4;
  static_assert((1 << LE) == E, "E: 1, 2, 4, 8 or 16");
  const uint32_t t0 = threadIdx.x * E;
  const int lane = __lane_id();
  uint64_t x[E];
#pragma unroll
  for (int e = 0; e < E; e++) x[e] = t0 + e < len ? a[t0 + e] : ~0ull;
#pragma unroll  // (every stage's distances constants)
  for (uint32_t k = 2; k <= n2; k <<= 1) {
    uint32_t j = k >> 2;  // the first half-cleaner after the flip stage
    if (k <= (uint32_t)E) {  // the flip stage of a block inside the thread's keys
#pragma unroll
      for (int e = 0; e < E; e++) {
        const int p = e ^ (int)(k - 1);
        if (e < p) td_cswap<E>(x[e], x[p]);
      }
    } else if (k <= WSPAN) {  // ... inside the wave: the partner of key e is key E-1-e of lane ^ ((k-1) >> LE)
      const int lm = (int)((k - 1) >> LE);
      const bool lower = (lane & (int)((k >> 1) >> LE)) == 0;
      uint64_t y[E];
#pragma unroll
      for (int e = 0; e < E; e++) y[E - 1 - e] = shfl_xor_u64(x[e], lm, 64);
#pragma unroll
      for (int e = 0; e < E; e++) x[e] = lower ? min(x[e], y[e]) : max(x[e], y[e]);
    } else {  // across waves: the flip stage and the half-cleaners of distance >= 64 E through the LDS
      td_lds_stages<E, NT>(a, x, k, true, WSPAN);
      j = WSPAN >> 1;
    }
#pragma unroll
    for (; j >= (uint32_t)E && j > 0; j >>= 1) {  // half-cleaners on shuffles: the partner is lane ^ (j >> LE)
      const int lm = (int)(j >> LE);
      const bool lower = (lane & lm) == 0;
#pragma unroll
      for (int e = 0; e < E; e++) {
        const uint64_t y = shfl_xor_u64(x[e], lm, 64);
        x[e] = lower ? min(x[e], y) : max(x[e], y);
      }
    }
#pragma unroll
    for (int jj = E >> 1; jj > 0; jj >>= 1) {  // the half-cleaners of distance < E (those below k / 2)
      if ((uint32_t)jj > (k >> 2)) continue;
#pragma unroll
      for (int e = 0; e < E; e++) {
        const int p = e ^ jj;
        if (e < p) td_cswap<E>(x[e], x[p]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; e++) a[t0 + e] = x[e];
  __syncthreads();
}
// the runs of 65 .. TD_SORT_MAX values (digests, and the MSD passes' bins): one workgroup each, in LDS, into v[0]
__global__ __launch_bounds__(256) void k_td_sort_lds(TdBuf td, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  __shared__ uint64_t a[TD_SORT_MAX];
  const int32_t nw = td.lctr[0];
  for (int32_t w = blockIdx.x; w < nw; w += gridDim.x) {
    const TdRun r = td.lrun[w];
    const uint32_t len = r.len & ~TD_RUN_V1;
    const uint64_t* __restrict__ src = (r.len & TD_RUN_V1) ? td.v[1] : td.v[0];
    for (uint32_t i = threadIdx.x; i < len; i += blockDim.x) a[i] = src[r.beg + i];
    __syncthreads();
#ifndef FW_TD_LDS_SORT
    if (len > 2048)
      td_bitonic_wave<16>(a, len);
    else if (len > 1024)
      td_bitonic_wave<8>(a, len);
    else if (len > 512)
      td_bitonic_wave<4>(a, len);
    else if (len > 256)
      td_bitonic_wave<2>(a, len);
    else
      td_bitonic_wave<1>(a, len);
#else
    if (len > 2048)
      td_bitonic_reg<16>(a, len);
    else if (len > 1024)
      td_bitonic_reg<8>(a, len);
    else if (len > 512)
      td_bitonic_reg<4>(a, len);
    else if (len > 256)
      td_bitonic_reg<2>(a, len);
    else
      td_bitonic_lds(a, len);
#endif
    for (uint32_t i = threadIdx.x; i < len; i += blockDim.x) td.v[0][r.beg + i] = a[i];
    __syncthreads();
  }
}
// ---- sample-sort passes over the runs longer than TD_SORT_MAX (level L: brun[L]; buckets of more than TD_SORT_MAX
// values go to brun[L + 1], brun[2] being the fallback).  A run's splitters are every (S / (ns + 1))-th key of a sorted
// sample of S <= TD_SAMPLE of its keys (ns + 1 = the run's length / (TD_SORT_MAX / 2), rounded up to a power of two,
// at most TD_MAX_SPL + 1); key x goes to bucket 2 lb + 1 when it equals splitter lb = lower_bound(x) -- a bucket of
// equal keys, already sorted, written to v[0] at once -- else to bucket 2 lb (strictly between two splitters).  The
// splitters are keys of the run, so every strict bucket is shorter than the run: each level makes progress whatever
// the distribution (heavy ties included).
constexpr int TD_SAMPLE = 8192;
constexpr int TD_MAX_SPL = 2047;
constexpr int TD_BUCKETS = 2 * TD_MAX_SPL + 1;
__device__ __forceinline__ int32_t td_tile_run(const TdMsd* msd, int32_t nl, uint32_t t) {
  int32_t lo = 0, hi = nl - 1;  // the last run whose first tile is <= t
  while (lo < hi) {
    const int32_t mid = (lo + hi + 1) >> 1;
    if (msd[mid].toff <= t)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}
__device__ __forceinline__ uint32_t td_bucket(const uint64_t* spl, uint32_t ns, uint64_t x) {
  uint32_t lo = 0, hi = ns;  // lower_bound: the first splitter >= x
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (spl[mid] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return 2 * lo + (lo < ns && spl[lo] == x ? 1u : 0u);
}
__global__ __launch_bounds__(256) void k_td_msd_prep(TdBuf td, int L, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int64_t nl = td.lctr[1 + L];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nl * TD_MSD_BINS;
       i += (int64_t)gridDim.x * blockDim.x)
    td.hist[i] = 0u;
}
// the runs' first tiles (one workgroup), and the level's tile count in lctr[4]
__global__ __launch_bounds__(1024) void k_td_msd_plan(TdBuf td, int L, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  __shared__ uint32_t sw[1024 / 64 + 1];
  const int32_t nl = td.lctr[1 + L];
  uint32_t carry = 0;
  for (int32_t j0 = 0; j0 < nl; j0 += blockDim.x) {
    const int32_t j = j0 + threadIdx.x;
    const uint32_t nt = j < nl ? ((td.brun[L][j].len & ~TD_RUN_V1) + TD_TILE - 1) / TD_TILE : 0u;
    uint32_t total;
    const uint32_t off = block_excl_scan(nt, sw, &total);
    if (j < nl) td.msd[j].toff = carry + off;
    carry += total;
    __syncthreads();
  }
  if (threadIdx.x == 0) td.lctr[4] = (int32_t)carry;
}
// one workgroup per run: a sorted sample of its keys, its splitters (td.spl, msd.nsp)
__global__ __launch_bounds__(1024) void k_td_msd_sample(TdBuf td, int L, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  __shared__ uint64_t a[TD_SAMPLE];
  const int32_t nl = td.lctr[1 + L];
  for (int32_t j = blockIdx.x; j < nl; j += gridDim.x) {
    const TdRun r = td.brun[L][j];
    const uint32_t len = r.len & ~TD_RUN_V1;
    const uint64_t* __restrict__ src = (r.len & TD_RUN_V1) ? td.v[1] : td.v[0];
    const uint32_t S = min((uint32_t)TD_SAMPLE, len);
    for (uint32_t i = threadIdx.x; i < S; i += blockDim.x) a[i] = src[r.beg + (uint32_t)(((uint64_t)i * len) / S)];
    __syncthreads();
    td_bitonic_wave<TD_SAMPLE / 1024, 1024>(a, S);
    uint32_t nb = 2;  // buckets between splitters: ~TD_SORT_MAX / 2 values each
    while (nb < TD_MAX_SPL + 1 && (uint64_t)nb * (TD_SORT_MAX / 2) < len) nb <<= 1;
    const uint32_t ns = nb - 1;
    for (uint32_t b = threadIdx.x; b < ns; b += blockDim.x)
      td.spl[(int64_t)j * TD_MAX_SPL + b] = a[(uint32_t)(((uint64_t)(b + 1) * S) / nb)];
    if (threadIdx.x == 0) td.msd[j].nsp = ns;
    __syncthreads();
  }
}
// one tile's keys (TD_TILE_PT per thread; past the run: ~0), and the run's splitters into LDS
__device__ __forceinline__ void td_tile_load(const TdBuf& td, const TdRun& r, uint32_t t0, uint64_t (&x)[TD_TILE_PT],
                                             uint32_t* lo_out, uint32_t* hi_out) {
  const uint32_t len = r.len & ~TD_RUN_V1;
  const uint64_t* __restrict__ src = (r.len & TD_RUN_V1) ? td.v[1] : td.v[0];
  const uint32_t lo = t0 * TD_TILE, hi = min(len, lo + TD_TILE);
#pragma unroll
  for (int u = 0; u < TD_TILE_PT; u++) {
    const uint32_t q = lo + u * 256 + threadIdx.x;
    x[u] = q < hi ? src[r.beg + q] : ~0ull;
  }
  *lo_out = lo;
  *hi_out = hi;
}
__global__ __launch_bounds__(256) void k_td_msd_hist(TdBuf td, int L, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int32_t nl = td.lctr[1 + L];
  const uint32_t ntile = (uint32_t)td.lctr[4];
  __shared__ uint32_t hs[TD_BUCKETS];
  __shared__ uint64_t spl[TD_MAX_SPL];
  for (uint32_t t = blockIdx.x; t < ntile; t += gridDim.x) {
    const int32_t j = td_tile_run(td.msd, nl, t);
    const TdRun r = td.brun[L][j];
    const TdMsd m = td.msd[j];
    const uint32_t ns = m.nsp, nb = 2 * ns + 1;
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) hs[b] = 0u;
    for (uint32_t b = threadIdx.x; b < ns; b += blockDim.x) spl[b] = td.spl[(int64_t)j * TD_MAX_SPL + b];
    uint64_t x[TD_TILE_PT];
    uint32_t lo, hi;
    td_tile_load(td, r, t - m.toff, x, &lo, &hi);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < TD_TILE_PT; u++) {
      const uint32_t q = lo + u * 256 + threadIdx.x;
      if (q < hi) atomicAdd(&hs[td_bucket(spl, ns, x[u])], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x)
      if (hs[b]) atomicAdd(&td.hist[(int64_t)j * TD_MSD_BINS + b], hs[b]);
    __syncthreads();
  }
}
// one workgroup per run: its buckets' starts (the cursors k_td_msd_scatter advances), and its strict buckets listed
// as runs of the next step -- the LDS sort (<= TD_SORT_MAX values) or the next level
__global__ __launch_bounds__(256) void k_td_msd_scan(TdBuf td, int L, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  __shared__ uint32_t sw[256 / 64 + 1];
  const int32_t nl = td.lctr[1 + L];
  for (int32_t j = blockIdx.x; j < nl; j += gridDim.x) {
    const TdRun r = td.brun[L][j];
    const uint32_t dst = (r.len & TD_RUN_V1) ? 0u : TD_RUN_V1;  // the strict buckets land in the other buffer
    const uint32_t nb = 2 * td.msd[j].nsp + 1;
    uint32_t* h = td.hist + (int64_t)j * TD_MSD_BINS;
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += blockDim.x) {
      const uint32_t b = b0 + threadIdx.x;
      const uint32_t cnt = b < nb ? h[b] : 0u;
      uint32_t total;
      const uint32_t off = block_excl_scan(cnt, sw, &total) + carry;
      if (b < nb) h[b] = off;
      const bool strict = b < nb && !(b & 1u);
      td_list_put(td.brun[L + 1], &td.lctr[2 + L], strict && cnt > TD_SORT_MAX, TdRun{r.beg + off, cnt | dst});
      // (a single value is sorted; it moves to v[0] through the LDS sort when it landed in v[1])
      td_list_put(td.lrun, &td.lctr[0], strict && cnt <= TD_SORT_MAX && (cnt > 1 || (cnt == 1 && dst)),
                  TdRun{r.beg + off, cnt | dst});
      carry += total;
      __syncthreads();
    }
  }
}
__global__ __launch_bounds__(256) void k_td_msd_scatter(TdBuf td, int L, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int32_t nl = td.lctr[1 + L];
  const uint32_t ntile = (uint32_t)td.lctr[4];
  __shared__ uint32_t hs[TD_BUCKETS];
  __shared__ uint64_t spl[TD_MAX_SPL];
  for (uint32_t t = blockIdx.x; t < ntile; t += gridDim.x) {
    const int32_t j = td_tile_run(td.msd, nl, t);
    const TdRun r = td.brun[L][j];
    const TdMsd m = td.msd[j];
    const uint32_t ns = m.nsp, nb = 2 * ns + 1;
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) hs[b] = 0u;
    for (uint32_t b = threadIdx.x; b < ns; b += blockDim.x) spl[b] = td.spl[(int64_t)j * TD_MAX_SPL + b];
    uint64_t x[TD_TILE_PT];
    uint32_t lo, hi;
    td_tile_load(td, r, t - m.toff, x, &lo, &hi);
    __syncthreads();
    uint32_t bk[TD_TILE_PT], rk[TD_TILE_PT];
#pragma unroll
    for (int u = 0; u < TD_TILE_PT; u++) {
      const uint32_t q = lo + u * 256 + threadIdx.x;
      bk[u] = q < hi ? td_bucket(spl, ns, x[u]) : 0u;
      rk[u] = q < hi ? atomicAdd(&hs[bk[u]], 1u) : 0u;
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x)
      if (hs[b]) hs[b] = atomicAdd(&td.hist[(int64_t)j * TD_MSD_BINS + b], hs[b]);
    __syncthreads();
    uint64_t* __restrict__ dst = (r.len & TD_RUN_V1) ? td.v[0] : td.v[1];
#pragma unroll
    for (int u = 0; u < TD_TILE_PT; u++) {
      const uint32_t q = lo + u * 256 + threadIdx.x;
      if (q < hi) ((bk[u] & 1u) ? td.v[0] : dst)[r.beg + hs[bk[u]] + rk[u]] = x[u];  // (equal keys: final)
    }
    __syncthreads();
  }
}
// the fallback: runs still longer than TD_SORT_MAX after two MSD levels (keys crowded into a few bits' range), one
// workgroup each, a bitonic network in global memory (in place), then into v[0]
__global__ __launch_bounds__(256) void k_td_sort_global(TdBuf td, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int32_t nw = td.lctr[3];
  for (int32_t w = blockIdx.x; w < nw; w += gridDim.x) {
    const TdRun r = td.brun[2][w];
    const uint32_t len = r.len & ~TD_RUN_V1;
    uint64_t* a = ((r.len & TD_RUN_V1) ? td.v[1] : td.v[0]) + r.beg;
    uint32_t n2 = 1;
    while (n2 < len) n2 <<= 1;
    for (uint32_t k = 2; k <= n2; k <<= 1) {
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        for (uint32_t t = threadIdx.x; t < (n2 >> 1); t += blockDim.x) {
          const uint32_t i = (t & ~(j - 1)) * 2 + (t & (j - 1));
          const uint32_t p = j == (k >> 1) ? (i ^ (k - 1)) : i + j;
          if (p < len) {
            const uint64_t x = a[i], y = a[p];
            if (x > y) {
              a[i] = y;
              a[p] = x;
            }
          }
        }
        __threadfence_block();
        __syncthreads();
      }
    }
    if (r.len & TD_RUN_V1)
      for (uint32_t i = threadIdx.x; i < len; i += blockDim.x) td.v[0][r.beg + i] = a[i];
    __syncthreads();
  }
}
// after the tiers: the touched digests' counters back to zero (whatever ran: k_td_group lists what it counted)
__global__ __launch_bounds__(256) void k_td_reset(TdBuf td) {
  const int32_t nt = td.ctr[0];
  for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nt; i += gridDim.x * blockDim.x) td.dcnt[td.tslot[i]] = 0u;
}

// ---- t-digest session merges (DevCfg::td_mdst / td_msrc, logged by the session flush and the ordered replay):
// AggregateFunction.merge of digests = the union of their centroids, compressed with the batch's values
// (oracle/window_oracle.cpp td_union).  A merge chain (a block merged into one that is merged further) ends at one
// final target per merged session; its union of old centroids is built once, and the tiers read it instead of the
// target's live half.
__global__ void k_td_mlink(DevCfg c, TdBuf td) {
  const int32_t nl = *c.td_mctr;
  for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += gridDim.x * blockDim.x)
    td.fwd[c.td_msrc[i]] = c.td_mdst[i];
}
__device__ __forceinline__ uint32_t td_final_target(const TdBuf& td, uint32_t b) {
  while (td.fwd[b] != ~0u) b = td.fwd[b];
  return b;
}
__global__ void k_td_mlist(DevCfg c, TdBuf td) {
  const int32_t nl = *c.td_mctr;
  for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += gridDim.x * blockDim.x) {
    const uint32_t t = td_final_target(td, c.td_mdst[i]);
    const int32_t prev = atomicExch(&td.mhead[t], i);
    td.mnext[i] = prev < 0 ? -2 : prev;  // -2: the list's last entry (the first in), which builds the union
  }
}
__global__ void k_td_mbuild(DevCfg c, DevTable tb, TdBuf td, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int32_t nl = *c.td_mctr;
  for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += gridDim.x * blockDim.x) {
    if (td.mnext[i] != -2) continue;
    const uint32_t t = td_final_target(td, c.td_mdst[i]);
    // the target's slot, which k_td_group wrote when one of the push's values went to it -- none may have (the
    // merged session fired with FIRE_AND_PURGE afterwards: td_purge emptied every digest of the union and dropped
    // the values), and then binv is a stale slot: the union (empty) is not needed, only the sources' release
    const uint32_t g = td.binv[t];
    bool own = (int64_t)g < td.lidx_slots;
    if (own) {
      const int32_t p = (int32_t)(g >> c.log_r);
      const Region r = region_of(c, tb, p, tb.cur[p]);
      const uint32_t sl = g & r.mask;
      own = st_kind(r.state[sl]) == SLOT_LIVE && pool_block_of(r.ent[sl]) == (uint64_t)t;
    }
    if (!own) {
      for (int32_t j = td.mhead[t]; j >= 0; j = td.mnext[j]) {
        c.pool_defer[atomicAdd(&c.pool_ctr[2], 1)] = c.td_msrc[j];
        if (td.mnext[j] == -2) break;
      }
      continue;
    }
    // the target's centroids and every merged block's (weights for now), then freed sources
    int32_t m = 0;
    const TdHead ht = *td_head(c, t);
    m += ht.n;
    for (int32_t j = td.mhead[t]; j >= 0; j = td.mnext[j]) {
      m += td_head(c, c.td_msrc[j])->n;
      if (td.mnext[j] == -2) break;
    }
    const unsigned long long off = atomicAdd(&td.uctr[0], (unsigned long long)m);
    TdCent* u = td.uni + off;
    int32_t k = 0;
    int64_t wold = 0;
    auto take = [&](uint64_t b) {
      const TdHead h = *td_head(c, b);
      const TdCent* ce = td_half(c, b, h.cur);
      for (int32_t q = 0; q < h.n; q++) u[k++] = TdCent{ce[q].sum, td_weight(ce, q)};
      wold += h.w;
    };
    take(t);
    for (int32_t j = td.mhead[t]; j >= 0; j = td.mnext[j]) {
      take(c.td_msrc[j]);
      c.pool_defer[atomicAdd(&c.pool_ctr[2], 1)] = c.td_msrc[j];  // (a t-digest block needs no zeroing)
      if (td.mnext[j] == -2) break;
    }
    td_union_sort(u, m);
    const int32_t ov = (int32_t)atomicAdd(&td.uctr[1], 1ull);
    td.ovr[ov] = TdOverride{u, m, g, wold};
    td.mover[g] = ov;
  }
}
// after the tiers: the push's merge bookkeeping back to empty
__global__ void k_td_mclear(DevCfg c, TdBuf td) {
  const int32_t nl = *c.td_mctr;
  for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += gridDim.x * blockDim.x) {
    td.fwd[c.td_msrc[i]] = ~0u;
    td.mhead[c.td_msrc[i]] = -1;
    td.mhead[c.td_mdst[i]] = -1;
  }
  const int32_t no = (int32_t)td.uctr[1];
  for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < no; i += gridDim.x * blockDim.x) td.mover[td.ovr[i].slot] = -1;
}

// each touched digest: merged serially here, or queued for the wave or the grid-wide merge
__global__ __launch_bounds__(256) void k_td_small(DevCfg c, DevTable tb, TdBuf td, const uint64_t* __restrict__ v, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  __shared__ double s_qb[TD_NB_MAX];
  td_stage_qb(c, s_qb);
  const int32_t nt = td.ctr[0];
  const uint32_t mask = (1u << c.log_r) - 1u;
  for (int32_t idx0 = blockIdx.x * blockDim.x; idx0 < nt; idx0 += gridDim.x * blockDim.x) {
    const int32_t pos = idx0 + (int32_t)threadIdx.x;
#ifdef FW_TD_NOPERM
    const int32_t idx = pos;
#else
    const int32_t idx = pos < nt ? (int32_t)td.gs[1][pos] : pos;  // (longest first: k_td_perm)
#endif
    bool mid = false;
    if (pos < nt) {
      const uint32_t g = td.tslot[idx];
      const int64_t beg = td.tbeg[idx];
      const int32_t p = (int32_t)(g >> c.log_r);
      const Region r = region_of(c, tb, p, tb.cur[p]);
      const Entry& e = r.ent[g & mask];
      const uint64_t blk = pool_block_of(e);
      TdHead* hp = td_head(c, blk);
      const TdHead h = *hp;
      const TdCent* old = td_half(c, blk, h.cur);
      int32_t no = h.n;
      int64_t hw = h.w;
      if (td.mover) {  // a merged session's digest: the union of the merged digests' centroids (k_td_mbuild)
        const int32_t ov = td.mover[g];
        if (ov >= 0) {
          const TdOverride o = td.ovr[ov];
          old = o.old;
          no = o.no;
          hw = o.wold;
        }
      }
      const int64_t W = e.cnt, nn = W - hw;
      TdCent* out = td_half(c, blk, h.cur ^ 1);
      td.lidx[g] = -1;
      if (nn + no <= FW_TD_T1) {
#ifdef FW_TD_SMALL_OLD
        const int32_t k = td_merge_serial(c, c.td_qb, v, beg, nn, old, no, out, W);
#else
        const int32_t k = td_merge_serial_blk(c, s_qb, v, beg, nn, old, no, out, W);
#endif
        *hp = TdHead{h.cur ^ 1, k, W};
      } else if (nn + no <= FW_TD_T3) {
        mid = true;
      } else {
        const int32_t L = atomicAdd(&td.ctr[1], 1);
        if (L >= td.max_large) {  // cannot happen: max_large bounds the digests with > FW_TD_T3 - td_nb values
          atomicOr(&st->flags, FW_STATUS_STATE_LOST);
        } else {
          td.lidx[g] = L;
          td.large[L] = TdLarge{beg, nn, W, no, h.cur ^ 1, old, out, hp};
          for (int b = 0; b < c.td_nb; b++) {
            td.nstart[(int64_t)L * c.td_nb + b] = -1;
            td.ostart[(int64_t)L * c.td_nb + b] = -1;
          }
        }
      }
    }
    // wave-aggregated reservation of the wave-tier list
    const uint64_t m = __ballot(mid);
    if (m) {
      int base = 0;
      const int leader = __ffsll((long long)m) - 1;
      if ((int)__lane_id() == leader) base = atomicAdd(&td.ctr[2], __popcll(m));
      base = __shfl(base, leader, 64);
      if (mid) td.mid[base + __popcll(m & lanemask_lt())] = (uint32_t)idx;
    }
  }
}

// placement of one value: the old centroids whose mean is below it precede it (a value goes before an equal
// mean); keys/cum: the old centroids' mean keys and cumulative weights
__device__ __forceinline__ int td_bucket_new(const DevCfg& c, const double* qb, const uint64_t* keys, const int64_t* cum,
                                             int32_t no, double W, int64_t r, uint64_t vkey) {
  int32_t lo = 0, hi = no;  // first old centroid whose mean key >= vkey
  while (lo < hi) {
    const int32_t m = (lo + hi) >> 1;
    if (keys[m] < vkey)
      lo = m + 1;
    else
      hi = m;
  }
  const int64_t cw = r + (lo ? cum[lo - 1] : 0);
  return td_bucket(c, qb, W, (double)cw + 0.5);
}
// placement of old centroid j: the values <= its mean precede it (binary search in the digest's sorted run)
__device__ __forceinline__ int td_bucket_old(const DevCfg& c, const double* qb, const uint64_t* __restrict__ v,
                                             int64_t beg, int64_t nn, uint64_t mk, int64_t cum_before, int64_t w,
                                             double W) {
  int64_t lo = 0, hi = nn;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (v[beg + m] <= mk)
      lo = m + 1;
    else
      hi = m;
  }
  return td_bucket(c, qb, W, (double)(lo + cum_before) + (double)w * 0.5);
}

// the wave tier: one wave per digest (its old centroids and bucket starts in LDS).  LDS per wave (dynamic,
// td_wave_lds_bytes): the old centroids' mean keys (then their sums), cumulative weights, each bucket's first
// value / first old centroid / where its runs end / its first block, and the tree sums of the batch values'
// blocks (a digest's nn <= FW_TD_T3 values form at most FW_TD_T3 / 64 + nb blocks)
constexpr int TD_WAVES = 4;
__host__ __device__ constexpr int td_wave_blocks(int nb) { return FW_TD_T3 / 64 + nb + 1; }
__host__ __device__ constexpr size_t td_wave_lds_wave(int nb) {
  return (8 * (size_t)(4 * nb + 1 + td_wave_blocks(nb)) + 4 * (size_t)(3 * nb + 1) + 7) & ~(size_t)7;
}
size_t td_wave_lds_bytes(int nb) { return TD_WAVES * td_wave_lds_wave(nb); }
__global__ __launch_bounds__(64 * TD_WAVES) void k_td_wave(DevCfg c, DevTable tb, TdBuf td, const uint64_t* __restrict__ v,
                                                           Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  extern __shared__ __align__(8) uint8_t td_lds[];
  __shared__ double s_qb[TD_NB_MAX];
  td_stage_qb(c, s_qb);
  const int wv = threadIdx.x >> 6, lane = __lane_id();
  const int nb = c.td_nb;
  uint8_t* base = td_lds + (size_t)wv * td_wave_lds_wave(nb);
  uint64_t* keys = reinterpret_cast<uint64_t*>(base);                 // [nb]; the old sums after the placement
  double* osum = reinterpret_cast<double*>(base);
  int64_t* cum = reinterpret_cast<int64_t*>(base) + nb;               // [nb]
  int64_t* ns = cum + nb;                                             // [nb + 1] first value of each bucket (-1: none)
  int64_t* s_en = ns + nb + 1;                                        // [nb] where each bucket's runs end
  double* bsum = reinterpret_cast<double*>(s_en + nb);                // [td_wave_blocks(nb)]
  int32_t* os = reinterpret_cast<int32_t*>(bsum + td_wave_blocks(nb));  // [nb + 1] first old centroid (-1: none)
  int32_t* s_eo = os + nb + 1;                                        // [nb]
  int32_t* bst = s_eo + nb;                                           // [nb] first block of each bucket
  const int32_t nmid = td.ctr[2];
  const uint32_t mask = (1u << c.log_r) - 1u;
  for (int32_t q = blockIdx.x * TD_WAVES + wv; q < nmid; q += gridDim.x * TD_WAVES) {
    TdLarge d;
    {
      const uint32_t idx = td.mid[q];
      const uint32_t g = td.tslot[idx];
      const int32_t p = (int32_t)(g >> c.log_r);
      const Region r = region_of(c, tb, p, tb.cur[p]);
      const Entry& e = r.ent[g & mask];
      const uint64_t blk = pool_block_of(e);
      TdHead* hp = td_head(c, blk);
      const TdHead h = *hp;
      d = TdLarge{td.tbeg[idx], e.cnt - h.w, e.cnt, h.n, h.cur ^ 1, td_half(c, blk, h.cur), td_half(c, blk, h.cur ^ 1), hp};
      if (td.mover) {  // a merged session's digest (k_td_mbuild)
        const int32_t ov = td.mover[g];
        if (ov >= 0) {
          const TdOverride o = td.ovr[ov];
          d.old = o.old;
          d.no = o.no;
          d.nn = e.cnt - o.wold;
        }
      }
    }
    const double W = (double)d.W;
    double my_osum[4];  // this lane's old sums (j = lane + 64 u), staged into LDS once the keys are no longer read
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int32_t j = lane + 64 * u;
      if (j < d.no) {
        const TdCent cj = d.old[j];
        const int64_t w = cj.cum - (j ? d.old[j - 1].cum : 0);
        keys[j] = td_mean_key(cj.sum, w);
        cum[j] = cj.cum;
        my_osum[u] = cj.sum;
      }
    }
    for (int b = lane; b < nb; b += 64) {
      ns[b] = -1;
      os[b] = -1;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    // place the values, 64 at a time; a bucket starts where a value's bucket differs from its predecessor's
    int carry = -1;
    for (int64_t i0 = 0; i0 < d.nn; i0 += 64) {
      const int64_t i = i0 + lane;
      int b = -1;
      if (i < d.nn) b = td_bucket_new(c, s_qb, keys, cum, d.no, W, i, v[d.beg + i]);
      int prev = __shfl_up(b, 1, 64);
      if (lane == 0) prev = carry;
      if (i < d.nn && prev != b) ns[b] = d.beg + i;
      carry = __shfl(b, 63, 64);
    }
    carry = -1;
    for (int32_t j0 = 0; j0 < d.no; j0 += 64) {
      const int32_t j = j0 + lane;
      int b = -1;
      if (j < d.no) b = td_bucket_old(c, s_qb, v, d.beg, d.nn, keys[j], j ? cum[j - 1] : 0, td_weight(d.old, j), W);
      int prev = __shfl_up(b, 1, 64);
      if (lane == 0) prev = carry;
      if (j < d.no && prev != b) os[b] = j;
      carry = __shfl(b, 63, 64);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
    for (int u = 0; u < 4; u++)
      if (lane + 64 * u < d.no) osum[lane + 64 * u] = my_osum[u];  // (the keys are read no more)
    // the end of every bucket's runs = the start of the next bucket that has one (the starts grow with the
    // bucket): an exclusive suffix minimum over the buckets, 64 at a time from the last chunk down
    {
      int64_t carry_n = d.beg + d.nn;
      int32_t carry_o = d.no;
      for (int b0 = ((nb - 1) >> 6) << 6; b0 >= 0; b0 -= 64) {
        const int b = b0 + lane;
        int64_t xn = b < nb && ns[b] >= 0 ? ns[b] : INT64_MAX;
        int32_t xo = b < nb && os[b] >= 0 ? os[b] : INT32_MAX;
        for (int o = 1; o < 64; o <<= 1) {  // inclusive suffix minimum over lanes >= lane
          const int64_t yn = __shfl_down(xn, o, 64);
          const int32_t yo = __shfl_down(xo, o, 64);
          if (lane + o < 64) {
            xn = min(xn, yn);
            xo = min(xo, yo);
          }
        }
        int64_t en = __shfl_down(xn, 1, 64);
        int32_t eo = __shfl_down(xo, 1, 64);
        if (lane == 63) {
          en = INT64_MAX;
          eo = INT32_MAX;
        }
        if (b < nb) {
          s_en[b] = min(en, carry_n);
          s_eo[b] = min(eo, carry_o);
        }
        carry_n = min(carry_n, __shfl(xn, 0, 64));
        carry_o = min(carry_o, __shfl(xo, 0, 64));
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // each bucket's blocks of 64 new values (from its first value): bst = exclusive prefix of the block counts
    int32_t nblocks = 0;
    for (int b0 = 0; b0 < nb; b0 += 64) {
      const int b = b0 + lane;
      int32_t cnt = 0;
      if (b < nb && ns[b] >= 0) cnt = (int32_t)((s_en[b] - ns[b] + 63) >> 6);
      int32_t x = cnt;
      for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (b < nb) bst[b] = nblocks + x - cnt;
      nblocks += __shfl(x, 63, 64);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // every block's tree sum, four blocks' values in flight (the same trees as td_wave_new_sum's)
    {
      int bk = 0;  // bucket of block k (blocks are in bucket order)
      for (int32_t k0 = 0; k0 < nblocks; k0 += 4) {
        double x[4];
        bool has[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int32_t k = k0 + u;
          has[u] = false;
          x[u] = 0.0;
          if (k < nblocks) {
            // (blocks are in bucket order; a bucket without new values owns none)
            while (ns[bk] < 0 || k >= bst[bk] + (int32_t)((s_en[bk] - ns[bk] + 63) >> 6)) bk++;
            const int64_t start = ns[bk] + (int64_t)(k - bst[bk]) * 64;
            has[u] = start + lane < s_en[bk];
            if (has[u]) x[u] = td_val(v[start + lane]);
          }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
          if (k0 + u >= nblocks) break;
          const double t = td_wave_tree(x[u], has[u]);
          if (lane == 0) bsum[k0 + u] = t;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // buckets in order, a lane per bucket: each non-empty one is a centroid
    int32_t kbase = 0;
    int64_t cbase = 0;
    for (int b0 = 0; b0 < nb; b0 += 64) {
      const int b = b0 + lane;
      const bool live = b < nb && (ns[b] >= 0 || os[b] >= 0);
      double sum = 0.0;
      int64_t w = 0;
      if (live) {
        const int64_t sn = ns[b];
        const int32_t so = os[b];
        const int64_t end_n = s_en[b];
        const int32_t end_o = s_eo[b];
        const int64_t a_n = sn >= 0 ? sn : end_n;
        const int32_t a_o = so >= 0 ? so : end_o;
        double s_new = 0.0, s_old = 0.0;
        bool any_n = false, any_o = false;
        if (sn >= 0) {
          const int32_t k1 = bst[b] + (int32_t)((end_n - sn + 63) >> 6);
          for (int32_t k = bst[b]; k < k1; k++) td_fold(s_new, any_n, bsum[k]);
        }
        for (int32_t j = a_o; j < end_o; j++) td_fold(s_old, any_o, osum[j]);
        sum = any_o && any_n ? s_old + s_new : any_o ? s_old : s_new;
        w = (end_n - a_n) + (end_o > a_o ? cum[end_o - 1] - (a_o ? cum[a_o - 1] : 0) : 0);
      }
      const uint64_t m = __ballot(live);
      int64_t x = w;  // inclusive prefix of the weights
      for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (live) d.out[kbase + __popcll(m & lanemask_lt())] = TdCent{sum, cbase + x};
      kbase += __popcll(m);
      cbase += __shfl(x, 63, 64);
    }
    if (lane == 0) *d.head = TdHead{d.pad, kbase, d.W};
    __builtin_amdgcn_wave_barrier();
  }
}

// the large tier: placement of every value of a large digest over the whole grid
#ifndef FW_TD_ITEMS_PT
#define FW_TD_ITEMS_PT 8
#endif
static_assert(FW_TD_ITEMS_PT % 4 == 0, "k_td_large_items: whole 16-byte loads");
// A thread takes FW_TD_ITEMS_PT consecutive sorted positions: inside one digest its items' old-centroid places only
// grow (the search resumes from the last one), and an item's predecessor is usually the thread's previous item, whose
// bucket is known
__global__ __launch_bounds__(256) void k_td_large_items(DevCfg c, int64_t n, const uint32_t* __restrict__ gs,
                                                        const uint64_t* __restrict__ v, uint32_t none, TdBuf td, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || td.ctr[1] == 0) return;
  __shared__ double s_qb[TD_NB_MAX];
  td_stage_qb(c, s_qb);
  constexpr int IT = FW_TD_ITEMS_PT;
  const int64_t nch = (n + IT - 1) / IT;
  for (int64_t ch = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; ch < nch; ch += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i0 = ch * IT;
    // the chunk's digests and values with whole-chunk vector loads (a lane's IT items are consecutive, so per-item
    // loads would stride a wave's lanes IT items apart and fetch every line IT times)
    uint32_t gq[IT];
    uint64_t vq[IT];
    const bool whole = i0 + IT <= n;
    if (whole) {
#pragma unroll
      for (int q = 0; q < IT; q += 4) {
        const uint4 x = *reinterpret_cast<const uint4*>(gs + i0 + q);
        gq[q] = x.x, gq[q + 1] = x.y, gq[q + 2] = x.z, gq[q + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < IT; q++) gq[q] = i0 + q < n ? gs[i0 + q] : none;
    }
    bool anyl = false;
    int32_t lq[IT];
#pragma unroll
    for (int q = 0; q < IT; q++) {
      lq[q] = gq[q] == none ? -1 : td.lidx[gq[q]];
      anyl |= lq[q] >= 0;
    }
    if (!anyl) continue;
    if (whole) {
#pragma unroll
      for (int q = 0; q < IT; q += 2) {
        const i64x2 x = *reinterpret_cast<const i64x2*>(v + i0 + q);
        vq[q] = (uint64_t)x.x, vq[q + 1] = (uint64_t)x.y;
      }
    } else {
#pragma unroll
      for (int q = 0; q < IT; q++) vq[q] = i0 + q < n ? v[i0 + q] : 0ull;
    }
    uint32_t pg = none;  // the previous item's digest (none: no previous item of a large digest)
    int pb = 0;
    int32_t plo = 0;
    TdLarge d{};
    const uint64_t* keys = nullptr;
    double W = 0.0;
#pragma unroll
    for (int k = 0; k < IT; k++) {
      const int64_t i = i0 + k;
      const uint32_t g = gq[k];
      const int32_t L = lq[k];
      if (i >= n || L < 0) {
        pg = none;
        continue;
      }
      const bool same = g == pg;
      if (!same) {
        d = td.large[L];
        keys = td.okey + (int64_t)L * c.td_nb;
        W = (double)d.W;
        plo = 0;
      }
      const int64_t r = i - d.beg;
      int32_t lo = plo, hi = d.no;  // (sorted values: the place of this one is at or after the previous one's)
      const uint64_t vk = vq[k];
      while (lo < hi) {
        const int32_t m = (lo + hi) >> 1;
        if (keys[m] < vk)
          lo = m + 1;
        else
          hi = m;
      }
      const int b = td_bucket(c, s_qb, W, (double)(r + (lo ? d.old[lo - 1].cum : 0)) + 0.5);
      bool start = r == 0;
      if (!start && same) {
        start = pb != b;
      } else if (!start) {
        const uint64_t pk = v[i - 1];
        int32_t lo2 = 0, hi2 = lo;  // the predecessor's place is at most this value's
        while (lo2 < hi2) {
          const int32_t m = (lo2 + hi2) >> 1;
          if (keys[m] < pk)
            lo2 = m + 1;
          else
            hi2 = m;
        }
        start = td_bucket(c, s_qb, W, (double)(r - 1 + (lo2 ? d.old[lo2 - 1].cum : 0)) + 0.5) != b;
      }
      if (start) td.nstart[(int64_t)L * c.td_nb + b] = (int32_t)i;
      pg = g;
      pb = b;
      plo = lo;
    }
  }
}
// the old centroids of the large digests (one wave per digest): their mean keys, buckets and bucket starts
__global__ __launch_bounds__(256) void k_td_large_old(DevCfg c, const uint64_t* __restrict__ v, TdBuf td, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  __shared__ double s_qb[TD_NB_MAX];
  td_stage_qb(c, s_qb);
  const int32_t nl = td.ctr[1];
  const int lane = __lane_id();
  for (int32_t L = (int32_t)((blockIdx.x * blockDim.x + threadIdx.x) >> 6); L < nl; L += (gridDim.x * blockDim.x) >> 6) {
    const TdLarge d = td.large[L];
    int carry = -1;
    for (int32_t j0 = 0; j0 < d.no; j0 += 64) {
      const int32_t j = j0 + lane;
      int b = -1;
      if (j < d.no) {
        const int64_t w = td_weight(d.old, j);
        const uint64_t mk = td_mean_key(d.old[j].sum, w);
        td.okey[(int64_t)L * c.td_nb + j] = mk;
        b = td_bucket_old(c, s_qb, v, d.beg, d.nn, mk, j ? d.old[j - 1].cum : 0, w, (double)d.W);
      }
      int prev = __shfl_up(b, 1, 64);
      if (lane == 0) prev = carry;
      if (j < d.no && prev != b) td.ostart[(int64_t)L * c.td_nb + b] = j;
      carry = __shfl(b, 63, 64);
    }
  }
}
// one wave per (large digest, bucket): the bucket's centroid; out[b] = {sum, weight} (weight 0: empty)
__global__ __launch_bounds__(256) void k_td_large_groups(DevCfg c, const uint64_t* __restrict__ v, TdBuf td, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int nb = c.td_nb;
  const int64_t units = (int64_t)td.ctr[1] * nb;
  const int lane = __lane_id();
  for (int64_t u = (int64_t)((blockIdx.x * blockDim.x + threadIdx.x) >> 6); u < units; u += (gridDim.x * blockDim.x) >> 6) {
    const int32_t L = (int32_t)(u / nb);
    const int b = (int)(u - (int64_t)L * nb);
    const TdLarge d = td.large[L];
    const int32_t* ns_row = td.nstart + (int64_t)L * nb;
    const int32_t* os_row = td.ostart + (int64_t)L * nb;
    int64_t a_n = ns_row[b];
    int32_t a_o = os_row[b];
    if (a_n < 0 && a_o < 0) {
      if (lane == 0) d.out[b] = TdCent{0.0, 0};
      continue;
    }
    // ends: the next bucket that starts anything, else the ends of the runs
    int64_t end_n = d.beg + d.nn;
    int32_t end_o = d.no;
    bool fn = false, fo = false;
    for (int b0 = b + 1; b0 < nb && !(fn && fo); b0 += 64) {
      const int bb = b0 + lane;
      const uint64_t mn = __ballot(bb < nb && ns_row[bb] >= 0), mo = __ballot(bb < nb && os_row[bb] >= 0);
      if (mn && !fn) {
        end_n = ns_row[b0 + __ffsll((long long)mn) - 1];
        fn = true;
      }
      if (mo && !fo) {
        end_o = os_row[b0 + __ffsll((long long)mo) - 1];
        fo = true;
      }
    }
    if (a_n < 0) a_n = end_n;
    if (a_o < 0) a_o = end_o;
    double s_new = 0.0, s_old = 0.0;
    bool any_o = false;
    const bool any_n = end_n > a_n;
    if (any_n) s_new = td_wave_new_sum(v, a_n, end_n);
    for (int32_t j = a_o; j < end_o; j++) td_fold(s_old, any_o, d.old[j].sum);
    const int64_t w = (end_n - a_n) + (end_o > a_o ? d.old[end_o - 1].cum - (a_o ? d.old[a_o - 1].cum : 0) : 0);
    if (lane == 0) d.out[b] = TdCent{any_o && any_n ? s_old + s_new : any_o ? s_old : s_new, w};
  }
}
// compaction of a large digest's buckets into its centroids (in place, in order), then the head
__global__ __launch_bounds__(64) void k_td_large_compact(DevCfg c, TdBuf td, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int32_t nl = td.ctr[1];
  for (int32_t L = blockIdx.x * blockDim.x + threadIdx.x; L < nl; L += gridDim.x * blockDim.x) {
    const TdLarge d = td.large[L];
    int32_t k = 0;
    int64_t cum = 0;
    for (int b = 0; b < c.td_nb; b++) {
      const TdCent g = d.out[b];
      if (g.cum == 0) continue;
      cum += g.cum;
      d.out[k++] = TdCent{g.sum, cum};
    }
    *d.head = TdHead{d.pad, k, d.W};
  }
}

// ---- count windows (FW_COUNT): KeyedStream.countWindow(size, slide) = GlobalWindows + CountTrigger.of(slide) +
// CountEvictor.of(size) (KeyedStream.java:383-397).  EvictingWindowOperator.processElement appends the element to
// the key's list and CountTrigger.onElement fires every slide-th element of the key (CountTrigger.java:47-55);
// the fire evicts all but the last `size` (CountEvictor.java:63-78) and reduces them in arrival order
// (EvictingWindowOperator.java:334-366).  With CountEvictor.of(size, true) the eviction follows the function,
// so the fired list is the last size + slide elements once it is that long: the window length wl.
// On the GPU: every record gets its key's slot, the batch is sorted stably by slot, so a key's records form one run in arrival order, the record at rank r of its run is the
// key's element number seq = count + r + 1; it fires when seq % slide == 0 over the elements seq - w + 1 .. seq
// (w = min(wl, seq)), read from the run and from the key's ring of its last wl - 1 earlier elements.
__device__ __forceinline__ int32_t cnt_slot(const DevCount& cw, int64_t key, Status* st) {
  uint32_t s = (uint32_t)fmix64((uint64_t)key ^ 0x3C6EF372FE94F82Bull) & cw.cap_mask;
  for (uint32_t probes = 0; probes <= cw.cap_mask;) {
    // relaxed agent-scope (L2) loads: an acquire here would invalidate the CU's L1 on every record; the publisher
    // below stores the key and slot write-through and waits for them before it stores the state
    const uint32_t cur = __hip_atomic_load(&cw.mstate[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_signal_fence(__ATOMIC_ACQUIRE);  // (the compiler keeps the key loads behind it)
    if (cur == 2) {
      if (__hip_atomic_load(&cw.mkey[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == key) {
        const uint32_t slot = __hip_atomic_load(&cw.mslot[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (slot >= (uint32_t)cw.max_keys) break;  // a key refused earlier stays refused
        return (int32_t)slot;
      }
      s = (s + 1) & cw.cap_mask;
      probes++;
      continue;
    }
    if (cur == 1) continue;  // being published by another lane: re-read
    if (atomicCAS(&cw.mstate[s], 0u, 1u) == 0u) {
      const int32_t slot = atomicAdd(cw.nslots, 1);
      __hip_atomic_store(&cw.mkey[s], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&cw.mslot[s], (uint32_t)slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&cw.mstate[s], 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (slot >= cw.max_keys) {
        atomicOr(&st->flags, FW_STATUS_STATE_LOST);
        return -1;
      }
      return slot;
    }
  }
  atomicOr(&st->flags, FW_STATUS_STATE_LOST);
  return -1;
}
__global__ __launch_bounds__(256) void k_cnt_slots(DevCount cw, const int64_t* __restrict__ key, int64_t n,
                                                   uint32_t none, Status* st) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t slot = cnt_slot(cw, key[i], st);
    cw.sk[0][i] = slot < 0 ? none : (uint32_t)slot;
    cw.sv[0][i] = (uint32_t)i;
  }
}
__global__ __launch_bounds__(256) void k_cnt_bounds(DevCount cw, const uint32_t* __restrict__ sk, int64_t n,
                                                    uint32_t none) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t g = sk[i];
    if (g == none) continue;
    if (i == 0 || sk[i - 1] != g) cw.sbeg[g] = (int32_t)i;
    if (i == n - 1 || sk[i + 1] != g) cw.send[g] = (int32_t)(i + 1);
  }
}
// the reduce of one fire: SumAggregator over the window's elements in arrival order (integer sums wrap, so their
// order does not matter; Double sums add left to right, Float sums round each partial sum to float)
// the batch's values in sorted order (each run's elements side by side for the fire), as two 32-bit halves in the
// sort's spare buffers: one gather per record instead of one per element of every window that reads it
__global__ __launch_bounds__(256) void k_cnt_gather(const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv,
                                                    const int64_t* __restrict__ val, int64_t n, uint32_t none,
                                                    uint32_t* __restrict__ vlo, uint32_t* __restrict__ vhi) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (sk[i] == none) continue;
    const uint64_t v = (uint64_t)val[sv[i]];
    vlo[i] = (uint32_t)v;
    vhi[i] = (uint32_t)(v >> 32);
  }
}
// one workgroup per chunk of CF_CHUNK sorted records: a counting pass, one reservation of the chunk's rows (a single
// output counter took one contended atomic per wave before), then the rows at their offsets
constexpr int CF_CHUNK = 4096;
__device__ __forceinline__ bool cnt_fires(const DevCount& cw, const uint32_t* __restrict__ sk, int64_t i, int64_t n,
                                          uint32_t none) {
  if (i >= n || sk[i] == none) return false;
  const uint32_t g = sk[i];
  return (cw.cnt[g] + (i - cw.sbeg[g]) + 1) % cw.slide == 0;
}
__global__ __launch_bounds__(256) void k_cnt_fire(DevCfg c, DevCount cw, const uint32_t* __restrict__ sk,
                                                  const uint32_t* __restrict__ sv, const int64_t* __restrict__ key,
                                                  const uint32_t* __restrict__ vlo, const uint32_t* __restrict__ vhi,
                                                  int64_t n, uint32_t none, DevRows out, Status* st) {
  __shared__ uint32_t sw[256 / 64 + 1];
  __shared__ unsigned long long base_s;
  const int64_t ring = cw.wl - 1;
  constexpr int PER = CF_CHUNK / 256;
  for (int64_t c0 = (int64_t)blockIdx.x * CF_CHUNK; c0 < n; c0 += (int64_t)gridDim.x * CF_CHUNK) {
    uint32_t nf = 0;
#pragma unroll 4
    for (int k = 0; k < PER; k++) nf += cnt_fires(cw, sk, c0 + k * 256 + threadIdx.x, n, none) ? 1u : 0u;
    uint32_t total;
    unsigned long long pos = block_excl_scan(nf, sw, &total);
    if (threadIdx.x == 0) base_s = total ? atomicAdd(&st->out_rows, (unsigned long long)total) : 0ull;
    __syncthreads();
    pos += base_s;
    for (int k = 0; k < PER && nf; k++) {
      const int64_t i = c0 + k * 256 + threadIdx.x;
      if (!cnt_fires(cw, sk, i, n, none)) continue;
      nf--;
      Entry e;
      const uint32_t g = sk[i];
      const int64_t r = i - cw.sbeg[g], before = cw.cnt[g], seq = before + r + 1;
      const int64_t w = min(cw.wl, seq);
      e.key = key[sv[i]];
      e.start = LMIN;
      e.end = LMAX;
      e.cnt = w;
      double ds = 0.0, dm = 0.0;
      int64_t is = 0, im = LMAX;
      for (int64_t q = seq - w + 1; q <= seq; q++) {  // oldest first
        int64_t v, o;
        if (q > before) {
          const int64_t j = i - (seq - q);
          v = (int64_t)(((uint64_t)vhi[j] << 32) | vlo[j]);
          o = q == seq - w + 1 ? c.ord_base + (int64_t)sv[j] : 0;
        } else {
          const int64_t at = (int64_t)g * ring + (q - 1) % ring;
          v = cw.ring_v[at];
          o = cw.ring_o[at];
        }
        if (q == seq - w + 1) e.mx = o;  // the window's first element
        if (c.vtype == FW_VAL_F64) {
          const double d = __longlong_as_double(v);
          ds = q == seq - w + 1 ? d : c.f32 ? (double)((float)ds + (float)d) : ds + d;
          if (q == seq - w + 1 || f64_sortable(v) < f64_sortable(__double_as_longlong(dm))) dm = d;
        } else {
          is = jadd(is, v);
          im = min(im, v);
        }
      }
      if (c.vtype == FW_VAL_F64) {
        e.sum = __double_as_longlong(ds);
        e.mn = __double_as_longlong(dm);
        if ((e.mn & 0x7ff0000000000000ll) == 0x7ff0000000000000ll && (e.mn & 0x000fffffffffffffll))
          e.mn = 0x7ff8000000000000ll;  // Double.doubleToLongBits: canonical NaN
      } else {
        e.sum = sum_out(c, is);
        e.mn = im;
      }
      if ((int64_t)pos < out.cap) {
        out.key[pos] = e.key;
        out.start[pos] = e.start;
        out.end[pos] = e.end;
        out.cnt[pos] = e.cnt;
        out.sum[pos] = e.sum;
        out.mn[pos] = e.mn;
        out.mx[pos] = e.mx;
      } else {
        atomicOr(&st->flags, FW_STATUS_OUT_FULL);
      }
      pos++;
    }
    __syncthreads();  // (base_s is rewritten by the next chunk)
  }
}
// after every fire of the batch read them: the key's ring takes its last wl - 1 elements, its count the run's length
__global__ __launch_bounds__(256) void k_cnt_update(DevCfg c, DevCount cw, const uint32_t* __restrict__ sk,
                                                    const uint32_t* __restrict__ sv, const int64_t* __restrict__ val,
                                                    int64_t n, uint32_t none) {
  const int64_t ring = cw.wl - 1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t g = sk[i];
    if (g == none) continue;
    const int64_t b0 = cw.sbeg[g], len = cw.send[g] - b0, r = i - b0, before = cw.cnt[g];
    if (ring > 0 && r >= len - ring) {
      const int64_t at = (int64_t)g * ring + (before + r) % ring;  // element number before + r + 1
      cw.ring_v[at] = val[sv[i]];
      cw.ring_o[at] = c.ord_base + (int64_t)sv[i];
    }
  }
}
// then the counts (a kernel of their own: the ring update read them)
__global__ __launch_bounds__(256) void k_cnt_count(DevCount cw, const uint32_t* __restrict__ sk, int64_t n, uint32_t none) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t g = sk[i];
    if (g == none || (i + 1 < n && sk[i + 1] == g)) continue;  // the last record of the key's run
    cw.cnt[g] += cw.send[g] - cw.sbeg[g];
  }
}

struct FireDecision {
  bool fire, keep;
};
__device__ __forceinline__ FireDecision fire_decide(const DevCfg& c, int64_t wm, Entry& e, Entry& fe) {
  FireDecision d{false, true};
  if ((e.meta & FW_TIMER) && jsub(e.end, 1) <= wm) {  // trigger timer fires (EventTimeTrigger.onEventTime)
    e.meta &= ~(int64_t)FW_TIMER;
    fe = e;
    d.fire = e.cnt > 0;                                 // contents != null (WindowOperator.java:452-459)
    if (c.purging) {                                    // FIRE_AND_PURGE
      if (c.assigner == FW_SESSION)
        acc_clear(e);                                   // the session stays in the MergingWindowSet
      else
        d.keep = false;
    }
  }
  const int64_t cl = cleanup_of(e.end, c.lateness);
  if (cl != LMAX && cl <= wm) d.keep = false;  // GC timer: clearAllState (WindowOperator.java:461-463)
  return d;
}

// POOL: instantiated for the accumulator-block aggregates (HLL, t-digest: their rows are finished here from the
// blocks) apart from the plain ones, whose scan keeps FIRE_U slots per thread in flight
template <bool POOL>
__global__ __launch_bounds__(FW_FIRE_THREADS, POOL ? 5 : 1) void k_fire(DevCfg c, int64_t wm, DevTable tb, DevRows out,
                                                                       Status* st) {
  if constexpr (!POOL) c.pool_bytes = 0;
  const int32_t p = blockIdx.x;
  // a suspended push has not finished updating the state: the host resumes it and fires again
  if (tb.next_timer[p] > wm || __hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  __shared__ int live_s;
  __shared__ long long next_s;
  __shared__ uint32_t sw[FW_FIRE_THREADS / 64 + 1];
  __shared__ unsigned long long base_s;
  const int X = tb.cur[p], Y = X ^ 1;
  const Region rx = region_of(c, tb, p, X), ry = region_of(c, tb, p, Y);
  const uint32_t R = rx.mask + 1;
  for (uint32_t s = threadIdx.x; s < R; s += blockDim.x) ry.state[s] = SLOT_EMPTY;
  if (threadIdx.x == 0) {
    live_s = 0;
    next_s = LMAX;
  }
  __syncthreads();
  int live = 0;
  uint32_t nfire = 0;
  int64_t nt = LMAX;
  // FIRE_U slots per thread per step: their state words, then their live entries, are loaded before any is used
  // (one slot at a time left the scan waiting on each load in turn)
  constexpr int FIRE_U = POOL ? 1 : 4;  // (the pool rows' one-wave-per-row finish wants the occupancy more)
  // (the next step's state words are loaded with this step's entries: one round trip per step)
  uint32_t wn[FIRE_U];
#pragma unroll
  for (int u = 0; u < FIRE_U; u++) {
    const uint32_t s = u * blockDim.x + threadIdx.x;
    wn[u] = s < R ? ld_state_wg(rx.state + s) : (uint32_t)SLOT_EMPTY;
  }
  for (uint32_t s0 = 0; s0 < R; s0 += blockDim.x * FIRE_U) {
    uint32_t w[FIRE_U];
#pragma unroll
    for (int u = 0; u < FIRE_U; u++) w[u] = wn[u];
    Entry eu[FIRE_U];
#pragma unroll
    for (int u = 0; u < FIRE_U; u++)
      if (st_kind(w[u]) == SLOT_LIVE) eu[u] = rx.ent[s0 + u * blockDim.x + threadIdx.x];
#pragma unroll
    for (int u = 0; u < FIRE_U; u++) {
      const uint32_t s = s0 + blockDim.x * FIRE_U + u * blockDim.x + threadIdx.x;
      wn[u] = s < R ? ld_state_wg(rx.state + s) : (uint32_t)SLOT_EMPTY;
    }
#pragma unroll
    for (int u = 0; u < FIRE_U; u++) {
      if (st_kind(w[u]) != SLOT_LIVE) continue;
      Entry e = eu[u], fe;
      const FireDecision d = fire_decide(c, wm, e, fe);
      nfire += d.fire;
      if (!d.keep && !d.fire && c.pool_bytes) {  // GC without a row: free its block here (HLL: zeroed)
        const uint64_t blk = pool_block_of(e);
        if (c.agg == FW_AGG_HLL || c.agg == FW_AGG_ROW) {
          if (c.agg == FW_AGG_HLL)
            hll_clear(c, blk);
          else
            row_clear(c, blk);
          __threadfence();
        }
        c.pool_free[atomicAdd(&c.pool_ctr[0], 1)] = (uint32_t)blk;
      }
      if (!d.keep) continue;
      const uint64_t h = slot_hash(c, e.key, e.start);
      const int32_t dst = region_claim<true>(ry, h, live_word(h));
      if (dst >= 0) {
        ry.ent[dst] = e;
        live++;
        nt = min(nt, timer_of(e, c.lateness));
      } else {
        atomicOr(&st->flags, FW_STATUS_STATE_LOST);  // cannot happen: the survivors fit the region they came from
      }
    }
  }
  uint32_t total;
  uint32_t pos0 = block_excl_scan(nfire, sw, &total);
  if (threadIdx.x == 0) base_s = total ? atomicAdd(&st->out_rows, (unsigned long long)total) : 0ull;
  if (live) atomicAdd(&live_s, live);
  if (nt != LMAX) atomicMin(&next_s, (long long)nt);
  __syncthreads();
  __shared__ int nrel_s;  // HLL rows whose window goes (their blocks are freed by the finish)
  if (threadIdx.x == 0) nrel_s = 0;
  __syncthreads();
  if (nfire) {
    unsigned long long pos = base_s + pos0;
    // (the next step's state words are loaded with this step's entries: one round trip per step)
    uint32_t wn[FIRE_U];
#pragma unroll
    for (int u = 0; u < FIRE_U; u++) {
      const uint32_t s = u * blockDim.x + threadIdx.x;
      wn[u] = s < R ? ld_state_wg(rx.state + s) : (uint32_t)SLOT_EMPTY;
    }
    for (uint32_t s0 = 0; s0 < R; s0 += blockDim.x * FIRE_U) {
      uint32_t w[FIRE_U];
#pragma unroll
      for (int u = 0; u < FIRE_U; u++) w[u] = wn[u];
      Entry eu[FIRE_U];
#pragma unroll
      for (int u = 0; u < FIRE_U; u++)
        if (st_kind(w[u]) == SLOT_LIVE) eu[u] = rx.ent[s0 + u * blockDim.x + threadIdx.x];
#pragma unroll
      for (int u = 0; u < FIRE_U; u++) {
        const uint32_t s = s0 + blockDim.x * FIRE_U + u * blockDim.x + threadIdx.x;
        wn[u] = s < R ? ld_state_wg(rx.state + s) : (uint32_t)SLOT_EMPTY;
      }
#pragma unroll
      for (int u = 0; u < FIRE_U; u++) {
        if (st_kind(w[u]) != SLOT_LIVE) continue;
        Entry e = eu[u], fe;
        const FireDecision d2 = fire_decide(c, wm, e, fe);
        if (!d2.fire) continue;
        if ((int64_t)pos < out.cap) {
          write_row(c, out, pos, fe);
          // a session that fires with FIRE_AND_PURGE stays in flight with its state cleared (fire_decide): its
          // block is emptied after the row is read, and kept
          const bool purge = d2.keep && c.purging;
          if (c.agg == FW_AGG_HLL) {  // read back by hll_finish: the block, and its free-stack slot when it goes
            out.mn[pos] = (int64_t)pool_block_of(fe);
            out.mx[pos] = d2.keep ? (purge ? HLL_ZERO_KEEP : -1) : (int64_t)atomicAdd(&nrel_s, 1);
          }
          if (c.agg == FW_AGG_TDIGEST || c.agg == FW_AGG_ROW)  // read back by td_finish / row_finish: the block,
            out.sum[pos] = (int64_t)(pool_block_of(fe) |       // above it 1 + its free-stack slot, bit 63 a purge
                                     (d2.keep ? 0ull : (uint64_t)(atomicAdd(&nrel_s, 1) + 1) << 32) |
                                     (purge && c.agg == FW_AGG_TDIGEST ? TD_PURGE_TAG : 0ull));
        } else {
          atomicOr(&st->flags, FW_STATUS_OUT_FULL);
        }
        pos++;
      }
    }
  }
  if (c.pool_bytes && total) {
    __shared__ int hl_sb;
    __syncthreads();  // (nrel_s complete)
    __threadfence_block();
    // free-stack slots for this workgroup's released blocks (the rows whose window goes)
    if (threadIdx.x == 0) hl_sb = atomicAdd(&c.pool_ctr[0], nrel_s);
    __syncthreads();
    const uint64_t end = min((unsigned long long)out.cap, base_s + total);
    if (c.agg == FW_AGG_HLL) {
      __shared__ uint32_t hl_ids[FW_FIRE_THREADS];  // 64 chunk ids per wave (hll_finish)
      const uint64_t nwv = blockDim.x >> 6;
      if (c.hll_p <= 14) {  // (at most 32 bitmap words: four rows a wave)
        for (uint64_t r = base_s + (threadIdx.x >> 6); r < end; r += 4 * nwv)
          hll_finish4(c, out, r, nwv, end, hl_sb, hl_ids + (threadIdx.x & ~63u));
      } else {
        for (uint64_t r = base_s + (threadIdx.x >> 6); r < end; r += nwv) {
          const int64_t ri = out.mx[r];  // (every lane reads it before lane 0 overwrites it)
          hll_finish(c, out, r, ri < 0 ? ri : hl_sb + ri, hl_ids + (threadIdx.x & ~63u));
        }
      }
    } else if (c.agg == FW_AGG_ROW) {
      for (uint64_t r = base_s + threadIdx.x; r < end; r += blockDim.x) row_finish(c, out, r, hl_sb);
    } else {
      __shared__ unsigned long long cent_s;
      if (threadIdx.x == 0) cent_s = 0;
      __syncthreads();
      unsigned long long cent = 0;
      for (uint64_t r = base_s + threadIdx.x; r < end; r += blockDim.x)
        cent += td_finish(c, out, r, hl_sb);
      if (cent) atomicAdd(&cent_s, cent);
      __syncthreads();
      if (threadIdx.x == 0 && cent_s) atomicAdd(&st->td_cent, cent_s);
    }
  }
  if (threadIdx.x == 0) {
    if (total) atomicAdd(&st->fired_total, (unsigned long long)total);
    tb.cur[p] = (uint8_t)Y;
    tb.live[p] = live_s;
    tb.next_timer[p] = next_s;
  }
}

// ---- K_fire for sliding windows kept as panes (DevCfg::panes).  A window [s, s + size) of a key is
// the AggregateFunction.merge of the key's panes p in [s, s + size - slide]; its contents are non-null
// (WindowOperator.java:452-459) iff one of those panes exists.  A pane's pending windows are those
// whose maxTimestamp E lies in [max(meta, pane_floor), p + size - 1]: meta excludes the windows that
// were already late when the pane was created, pane_floor the ones formed by earlier watermarks.
// For each pending E <= wm in increasing order (EventTimeTrigger fires in timer order; the operator's
// output order per watermark is not part of the contract, TestHarnessUtil.java:70-108), the region's
// panes of E are merged per key in an LDS table and emitted as rows; when a region holds more keys
// than the table, E is formed in slices of the key-hash space.  Panes whose last window has been
// formed are dead (GC timer at maxTimestamp, allowedLateness 0): they are tombstoned in place and the
// region is compacted into the other buffer once tombstones pass R/8.  A slice whose rows do not fit
// the output suspends the launch at (E, slice); the host grows the buffer and fires again.
#ifndef FW_PF_U
#define FW_PF_U 4
#endif
#ifndef FW_PF_ABL
#define FW_PF_ABL 0
#endif
#ifndef FW_PF_THREADS
#define FW_PF_THREADS 1024
#endif
#ifndef FW_PF_SLOTS_LOG2
#define FW_PF_SLOTS_LOG2 11
#endif
constexpr int PF_THREADS = FW_PF_THREADS;
constexpr int PF_SLOTS = 1 << FW_PF_SLOTS_LOG2;
constexpr int PF_LIMIT = PF_SLOTS * 3 / 4;
constexpr int PF_U = FW_PF_U;  // region slots per thread in flight in the pane scan
struct PaneLds {
  uint32_t tag[PF_SLOTS];  // 0 empty, 1 being claimed, 2 full
  uint32_t sel[PF_SLOTS];  // minBy / maxBy: region slot of the pane holding the window's selected element
  int64_t key[PF_SLOTS];
  unsigned long long cnt[PF_SLOTS];
  int64_t sum[PF_SLOTS], mn[PF_SLOTS], mx[PF_SLOTS];
  int fill, over, wpos, dead, susp;
  long long enext, ntmin;
  unsigned long long base;
};
__device__ __forceinline__ uint32_t pf_hash(int64_t key) { return (uint32_t)(fmix64((uint64_t)key ^ 0x243F6A8885A308D3ull) >> 32); }

// (pane: the entry's region slot; ent: the region's entries, read back by a minBy / maxBy selection)
__device__ __forceinline__ bool pf_upsert(const DevCfg& c, PaneLds& L, const Entry& e, uint32_t h, uint32_t pane,
                                          const Entry* __restrict__ ent) {
  uint32_t s = (h * 0x9E3779B1u) >> (32 - FW_PF_SLOTS_LOG2);
  for (int i = 0, spin = 0; i < PF_SLOTS;) {
    if (++spin > (1 << 24)) return false;  // a slot never published: cannot happen; the pass reports overflow
    const uint32_t t = __hip_atomic_load(&L.tag[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (t == 2) {
      if (L.key[s] == e.key) break;
      s = (s + 1) & (PF_SLOTS - 1);
      i++;
      continue;
    }
    if (t == 1) continue;  // being published by a lane of this loop iteration
    if (__hip_atomic_load(&L.fill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= PF_LIMIT) return false;
    if (atomicAdd(&L.fill, 1) >= PF_LIMIT) {
      atomicSub(&L.fill, 1);
      return false;
    }
    if (atomicCAS(&L.tag[s], 0u, 1u) == 0u) {
      L.key[s] = e.key;
      L.cnt[s] = 0;
      L.sum[s] = 0;
      L.mn[s] = LMAX;
      L.mx[s] = LMIN;
      L.sel[s] = 0xffffffffu;
      __hip_atomic_store(&L.tag[s], 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      break;
    }
    atomicSub(&L.fill, 1);  // lost the claim: re-read the slot
  }
  atomicAdd(&L.cnt[s], (unsigned long long)e.cnt);
  if (c.vtype == FW_VAL_F64)
    atomicAdd((double*)&L.sum[s], __longlong_as_double(e.sum));
  else
    atomicAdd((unsigned long long*)&L.sum[s], (unsigned long long)e.sum);
  if (agg_by(c.agg)) {
    // minBy / maxBy (ComparableAggregator.java:72-94, first = true): the window's element is the lexicographically
    // smallest (key, ordinal) over its panes (a pane's entry holds its own), which is not two independent min / max;
    // the slot keeps the region slot of the pane holding it, replaced by CAS while this pane's pair is smaller
    uint32_t cur = __hip_atomic_load(&L.sel[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (;;) {
      if (cur != 0xffffffffu) {
        const i64x2 b = *reinterpret_cast<const i64x2*>(&ent[cur].mn);  // {mn, mx} of the current choice
        if (!by_less(e.mn, e.mx, b.x, b.y)) break;
      }
      const uint32_t old = atomicCAS(&L.sel[s], cur, pane);
      if (old == cur) break;
      cur = old;
    }
    return true;
  }
  atomicMin((long long*)&L.mn[s], (long long)e.mn);
  atomicMax((long long*)&L.mx[s], (long long)e.mx);
  return true;
}

__global__ __launch_bounds__(PF_THREADS) void k_fire_panes(DevCfg c, int64_t wm, DevTable tb, DevRows out, Status* st) {
  const int32_t p = blockIdx.x;
  // LMAX = no pending window (also when wm is Long.MAX_VALUE, the end-of-input watermark)
  if (tb.next_timer[p] > wm || tb.next_timer[p] == LMAX ||
      __hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    return;
  __shared__ PaneLds L;
  const int tid = threadIdx.x;
  const int X = tb.cur[p];
  const Region rx = region_of(c, tb, p, X);
  const uint32_t R = rx.mask + 1;
  const int64_t floor0 = tb.pane_floor[p];
  const bool resumed = tb.fire_e[p] != LMIN;
  int64_t E = resumed ? tb.fire_e[p] : tb.next_timer[p];
  uint64_t lo = resumed ? tb.fire_lo[p] : 0ull;
  uint64_t width = 1ull << 32;
  int64_t ntmin = LMAX;
  int dead = 0;
  for (;;) {
    for (int h = tid; h < PF_SLOTS; h += PF_THREADS) L.tag[h] = 0;
    if (tid == 0) {
      L.fill = 0;
      L.over = 0;
      L.wpos = 0;
      L.dead = 0;
      L.enext = LMAX;
      L.ntmin = LMAX;
    }
    __syncthreads();
    // otherwise: a last pass that only gathers tombstones and the next timer
    const bool forming = E <= wm && E != LMAX;
    int64_t en = LMAX, nt = LMAX;
    int dd = 0;
    bool over = false;
    // PF_U slots per thread per step: their state words, then their live entries, are loaded before
    // any is used, so each thread keeps PF_U loads in flight (one at a time left the scan latency-bound)
    // (the next step's state words are loaded with this step's entries: one round trip per step)
    uint32_t wn[PF_U];
#pragma unroll
    for (int u = 0; u < PF_U; u++) {
      const uint32_t s = u * PF_THREADS + tid;
      wn[u] = s < R ? ld_state_wg(rx.state + s) : (uint32_t)SLOT_EMPTY;
    }
    for (uint32_t s0 = 0; s0 < R; s0 += PF_THREADS * PF_U) {
      uint32_t w[PF_U];
#pragma unroll
      for (int u = 0; u < PF_U; u++) w[u] = wn[u];
      Entry eu[PF_U];
#pragma unroll
      for (int u = 0; u < PF_U; u++)
        if (st_kind(w[u]) == SLOT_LIVE) eu[u] = rx.ent[s0 + u * PF_THREADS + tid];
#pragma unroll
      for (int u = 0; u < PF_U; u++) {
        const uint32_t s = s0 + (uint32_t)(PF_THREADS * PF_U) + u * PF_THREADS + tid;
        wn[u] = s < R ? ld_state_wg(rx.state + s) : (uint32_t)SLOT_EMPTY;
      }
#pragma unroll
      for (int u = 0; u < PF_U; u++) {
      const uint32_t s = s0 + u * PF_THREADS + tid;
      if (st_kind(w[u]) != SLOT_LIVE) {
        dd += st_kind(w[u]) == SLOT_DEAD;
        continue;
      }
      const Entry& e = eu[u];
      const int64_t last_end = jsub(jadd(e.start, c.size), 1);  // maxTimestamp of the pane's last window
      const int64_t lo_e = max(e.meta, floor0);
      if (lo_e > last_end) {  // every window formed by an earlier watermark: GC
        __hip_atomic_store(rx.state + s, (uint32_t)SLOT_DEAD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dd++;
        continue;
      }
      const int64_t hi_e = min(wm, last_end);
      if (last_end > wm) nt = min(nt, max(lo_e, c.nt_floor));  // survives this watermark
      if (!forming) continue;
      if (lo_e <= E && E <= hi_e) {
        const uint32_t h = pf_hash(e.key);
#if FW_PF_ABL & 1  // (timing ablation only: no window formed)
        asm volatile("" ::"v"(h), "v"(e.cnt), "v"(e.sum));
#else
        if (!over && (uint64_t)h >= lo && (uint64_t)h < lo + width && !pf_upsert(c, L, e, h, s, rx.ent)) over = true;
#endif
      }
      const int64_t cand = max(lo_e, E + c.slide);
      if (E < LMAX - c.slide && cand <= hi_e) en = min(en, cand);
      }
    }
    if (over) L.over = 1;
    if (en != LMAX) atomicMin(&L.enext, (long long)en);
    if (nt != LMAX) atomicMin(&L.ntmin, (long long)nt);
    if (dd) atomicAdd(&L.dead, dd);
    __syncthreads();
    dead = L.dead;
    ntmin = L.ntmin;
    const int ov = L.over;
    const uint32_t n = (uint32_t)L.fill;
    const int64_t enext = L.enext;
    __syncthreads();  // every thread has read the pass's results before thread 0 writes L again
    if (!forming) break;
    if (ov) {
      if (width == 1) {  // cannot happen: one hash value never holds PF_LIMIT keys of one region
        if (tid == 0) atomicOr(&st->flags, FW_STATUS_STATE_LOST);
        return;
      }
      width >>= 1;
      continue;
    }
    if (tid == 0) {
      bool ok = true;
      unsigned long long cur = __hip_atomic_load(&st->out_rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      while (n) {
        if ((int64_t)(cur + n) > out.cap) {
          ok = false;
          break;
        }
        if (__hip_atomic_compare_exchange_strong(&st->out_rows, &cur, cur + n, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
          break;
      }
      L.base = cur;
      if (!ok) {  // suspend at (E, lo): the host grows the output and fires again
        tb.fire_e[p] = E;
        tb.fire_lo[p] = lo;
        atomicMax((long long*)&st->need_out, (long long)(cur + n));
        atomicOr(&st->suspended, (int)FW_SUSP_FIRE);
      }
      L.susp = ok ? 0 : 1;
    }
    __syncthreads();
    if (L.susp) return;
    if (n) {
      const int64_t ws = jsub(jadd(E, 1), c.size);
      for (int h = tid; h < PF_SLOTS; h += PF_THREADS) {
        if (L.tag[h] != 2) continue;
        Entry r;
        r.key = L.key[h];
        r.start = ws;
        r.end = jadd(E, 1);
        r.cnt = (int64_t)L.cnt[h];
        r.sum = L.sum[h];
        r.mn = L.mn[h];
        r.mx = L.mx[h];
        if (agg_by(c.agg)) {  // the selected element's (key, ordinal), from its pane
          const uint32_t ps = L.sel[h];
          r.mn = rx.ent[ps].mn;
          r.mx = rx.ent[ps].mx;
        }
        write_row(c, out, L.base + (unsigned long long)atomicAdd(&L.wpos, 1), r);
      }
      if (tid == 0) atomicAdd(&st->fired_total, (unsigned long long)n);
    }
    __syncthreads();  // the rows are read out of L before the next pass clears it
    lo += width;
    if (lo >= (1ull << 32)) {
      lo = 0;
      width = 1ull << 32;
      E = enext;
      if (E > wm || E == LMAX) break;  // this pass saw every slot: its tombstone count and next timer are final
    }
  }
  // every pending window <= wm is formed
  if (dead * 8 > (int)R) {  // compact: re-insert the live panes into the other buffer
    const Region ry = region_of(c, tb, p, X ^ 1);
    for (uint32_t s = tid; s < R; s += PF_THREADS) ry.state[s] = SLOT_EMPTY;
    __syncthreads();
    int live = 0;
    for (uint32_t s = tid; s < R; s += PF_THREADS) {
      if (st_kind(ld_state_wg(rx.state + s)) != SLOT_LIVE) continue;
      const Entry e = rx.ent[s];
      const uint64_t h = slot_hash(c, e.key, e.start);
      const int32_t d = region_claim<true>(ry, h, live_word(h));
      if (d >= 0) {
        ry.ent[d] = e;
        live++;
      } else {
        atomicOr(&st->flags, FW_STATUS_STATE_LOST);
      }
    }
    if (tid == 0) L.wpos = 0;
    __syncthreads();
    if (live) atomicAdd(&L.wpos, live);
    __syncthreads();
    if (tid == 0) {
      tb.cur[p] = (uint8_t)(X ^ 1);
      tb.live[p] = L.wpos;
    }
  }
  if (tid == 0) {
    tb.pane_floor[p] = max(floor0, c.nt_floor);
    tb.next_timer[p] = ntmin;
    tb.fire_e[p] = LMIN;
  }
}

// ---- table growth: re-insert every live entry of the old table into the new one (buffer 0);
// DEAD slots are dropped, so the region's occupied count becomes its live count
__global__ __launch_bounds__(FW_FIRE_THREADS) void k_rehash(DevCfg oc, DevTable ot, DevCfg nc, DevTable nt) {
  __shared__ int live_s;
  const int32_t p = blockIdx.x;
  const Region ro = region_of(oc, ot, p, ot.cur[p]);
  const Region rn = region_of(nc, nt, p, 0);
  const uint32_t R = ro.mask + 1;
  if (threadIdx.x == 0) live_s = 0;
  __syncthreads();
  int live = 0;
  for (uint32_t s = threadIdx.x; s < R; s += blockDim.x) {
    if (st_kind(ld_state(ro.state + s)) != SLOT_LIVE) continue;
    const Entry e = ro.ent[s];
    // the new region is larger than the old one, so a slot is always found
    const uint64_t h = slot_hash(nc, e.key, e.start);
    const int32_t d = region_claim(rn, h, live_word(h));
    if (d >= 0) {
      rn.ent[d] = e;
      live++;
    }
  }
  if (live) atomicAdd(&live_s, live);
  __syncthreads();
  if (threadIdx.x == 0) {
    nt.cur[p] = 0;
    nt.live[p] = live_s;
    nt.next_timer[p] = ot.next_timer[p];
  }
}

__global__ void k_reset_regions(DevCfg c, DevTable tb) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= c.P) return;
  tb.cur[p] = 0;
  tb.live[p] = 0;
  tb.next_timer[p] = LMAX;
  tb.fire_e[p] = LMIN;
  tb.fire_lo[p] = 0;
  tb.pane_floor[p] = LMIN;
  tb.passes[p] = 0;
}

// ---- keyed-state snapshot of one key group (HeapKeyedStateBackend.snapshot writes per key group,
// HeapKeyedStateBackend.java:370-381): one workgroup per partition of the key group; each compacts
// its region's live entries into the output columns behind one atomic reservation.
__global__ __launch_bounds__(FW_FIRE_THREADS) void k_snapshot(DevCfg c, DevTable tb, int32_t p0, StateCols out,
                                                             unsigned long long* count) {
  __shared__ uint32_t sw[FW_FIRE_THREADS / 64 + 1];
  __shared__ unsigned long long base_s;
  const int32_t p = p0 + blockIdx.x;
  const Region r = region_of(c, tb, p, tb.cur[p]);
  // (dense regions: the live prefix, no state words)
  const uint32_t R = c.dense ? (uint32_t)tb.live[p] : r.mask + 1;
  // one pass per block of the region: count, reserve, write
  for (uint32_t s0 = 0; s0 < R; s0 += blockDim.x) {
    const uint32_t s = s0 + threadIdx.x;
    bool live = s < R && (c.dense || st_kind(ld_state(r.state + s)) == SLOT_LIVE);
    if (live && c.panes && max(r.ent[s].meta, tb.pane_floor[p]) > jsub(jadd(r.ent[s].start, c.size), 1))
      live = false;  // a pane whose windows have all been formed (GC'd at the next watermark)
    uint32_t total;
    const uint32_t pos = block_excl_scan(live ? 1u : 0u, sw, &total);
    if (threadIdx.x == 0) base_s = total ? atomicAdd(count, (unsigned long long)total) : 0ull;
    __syncthreads();
    if (live) {
      const Entry e = r.ent[s];
      const unsigned long long o = base_s + pos;
      out.key[o] = e.key;
      out.start[o] = e.start;
      out.end[o] = e.end;
      out.cnt[o] = e.cnt;
      out.sum[o] = sum_out(c, e.sum);
      out.mn[o] = mn_out(c, e.mn);
      out.mx[o] = mx_out(c, e.mx);
      if (agg_by(c.agg)) by_row(c.agg, c.vtype, e, &out.mn[o], &out.mx[o]);
      // a pane's timer: the maxTimestamp of its next window to form
      out.timer[o] = c.panes ? max(e.meta, tb.pane_floor[p]) : (e.meta & FW_TIMER) ? 1 : 0;
      if (out.blk) out.blk[o] = (int64_t)pool_block_of(e);  // exported by k_block_export
    }
    __syncthreads();
  }
}

// ---- accumulator blocks of the pool aggregates in their snapshot form (flink_window.h, fw_state_block_bytes).
// One wave per row.  HyperLogLog: the 2^p registers (an unmarked chunk is all zero, so they are copied whole);
// t-digest: n, then (sum bits, weight) of the live half's centroids, zero-padded.
__global__ __launch_bounds__(256) void k_block_export(DevCfg c, const int64_t* __restrict__ blk, int64_t n,
                                                      uint8_t* __restrict__ acc) {
  const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = __lane_id();
  if (row >= n) return;
  const uint64_t b = (uint64_t)blk[row];
  if (c.agg == FW_AGG_HLL) {
    const int32_t nq = (int32_t)(((int64_t)1 << c.hll_p) / 16);
    const uint4* q = reinterpret_cast<const uint4*>(c.pool + b * (uint64_t)c.pool_bytes + hll_hdr_bytes(c.hll_p));
    uint4* d = reinterpret_cast<uint4*>(acc + row * (int64_t)nq * 16);
    for (int32_t j = lane; j < nq; j += 64) d[j] = q[j];
  } else if (c.agg == FW_AGG_ROW) {  // per column: count, sum lo, sum hi, min, max (the column's values; 0 if empty)
    const RowAcc* a = row_acc(c, b);
    int64_t* d = reinterpret_cast<int64_t*>(acc) + row * 5 * (int64_t)c.row_nc;
    for (int32_t j = lane; j < c.row_nc; j += 64) {
      const RowAcc x = a[j];
      const bool f = row_float(c, j);
      d[5 * j] = (int64_t)x.nn;
      d[5 * j + 1] = (int64_t)x.lo;
      d[5 * j + 2] = f ? 0 : x.hi;
      d[5 * j + 3] = !x.nn ? 0 : f ? f64_unsortable(row_dec_min(x.mn)) : row_dec_min(x.mn);
      d[5 * j + 4] = !x.nn ? 0 : f ? f64_unsortable(row_dec_max(x.mx)) : row_dec_max(x.mx);
    }
  } else {
    const TdHead h = *td_head(c, b);
    const TdCent* ce = td_half(c, b, h.cur);
    const int32_t nw = 1 + 2 * c.td_nb;
    int64_t* d = reinterpret_cast<int64_t*>(acc) + row * (int64_t)nw;
    for (int32_t j = lane; j < nw; j += 64) {
      const int32_t k = (j - 1) >> 1;
      d[j] = j == 0 ? (int64_t)h.n : k >= h.n ? 0 : (j & 1) ? __double_as_longlong(ce[k].sum) : td_weight(ce, k);
    }
  }
}
__device__ __forceinline__ uint32_t bytes_max(uint32_t a, uint32_t b) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 32; k += 8) r |= max((a >> k) & 0xffu, (b >> k) & 0xffu) << k;
  return r;
}
// a digest restores only with at most delta/2 centroids of weight >= 1 (registers: any bytes)
__device__ bool acc_valid(const DevCfg& c, const uint8_t* src) {
  if (c.agg == FW_AGG_HLL) return true;
  if (c.agg == FW_AGG_ROW) {  // counts >= 0
    const int64_t* s = reinterpret_cast<const int64_t*>(src);
    for (int j = 0; j < c.row_nc; j++)
      if (s[5 * j] < 0) return false;
    return true;
  }
  const int64_t* s = reinterpret_cast<const int64_t*>(src);
  if (s[0] < 0 || s[0] > c.td_nb) return false;
  for (int32_t k = 0; k < (int32_t)s[0]; k++)
    if (s[2 + 2 * k] < 1) return false;
  return true;
}
// one thread: a row's accumulator into block b (merge: HyperLogLog register max into a live block)
__device__ void block_import(const DevCfg& c, uint64_t b, const uint8_t* src, bool merge) {
  uint8_t* base = c.pool + b * (uint64_t)c.pool_bytes;
  if (c.agg == FW_AGG_ROW) {  // (merge: AggregateFunction.merge into the live block)
    RowAcc* a = row_acc(c, b);
    const int64_t* s = reinterpret_cast<const int64_t*>(src);
    for (int j = 0; j < c.row_nc; j++) {
      if (!merge) a[j] = RowAcc{0, 0, 0, 0, 0};
      if (s[5 * j] <= 0) continue;
      const bool f = row_float(c, j);
      atomicAdd(&a[j].nn, (unsigned long long)s[5 * j]);
      if (f)
        atomicAdd(reinterpret_cast<double*>(&a[j].lo), __longlong_as_double(s[5 * j + 1]));
      else
        row_add128(a[j], (unsigned long long)s[5 * j + 1], s[5 * j + 2]);
      atomicMax(&a[j].mn, row_enc_min(row_key(c, j, s[5 * j + 3])));
      atomicMax(&a[j].mx, row_enc_max(row_key(c, j, s[5 * j + 4])));
    }
    return;
  }
  if (c.agg == FW_AGG_HLL) {
    const int32_t nq = (int32_t)(((int64_t)1 << c.hll_p) / 16), nw = (nq + 31) / 32;
    uint32_t* bits = reinterpret_cast<uint32_t*>(base);
    uint4* q = reinterpret_cast<uint4*>(base + hll_hdr_bytes(c.hll_p));
    const uint4* s = reinterpret_cast<const uint4*>(src);
    for (int32_t w = 0; w < nw; w++) {
      uint32_t word = merge ? bits[w] : 0u;
      for (int32_t j = w * 32; j < min(nq, w * 32 + 32); j++) {
        uint4 v = s[j];
        if (merge) {
          const uint4 o = q[j];
          v.x = bytes_max(v.x, o.x);
          v.y = bytes_max(v.y, o.y);
          v.z = bytes_max(v.z, o.z);
          v.w = bytes_max(v.w, o.w);
        }
        q[j] = v;
        if (v.x | v.y | v.z | v.w) word |= 1u << (j & 31);
      }
      bits[w] = word;
    }
    return;
  }
  const int64_t* s = reinterpret_cast<const int64_t*>(src);
  const int32_t nc = (int32_t)s[0];
  TdCent* ce = td_half(c, b, 0);
  int64_t cum = 0;
  for (int32_t k = 0; k < nc; k++) {
    cum += s[2 + 2 * k];
    ce[k] = TdCent{__longlong_as_double(s[1 + 2 * k]), cum};
  }
  *td_head(c, b) = TdHead{0, nc, cum};
}
// free-stack blocks and fresh blocks for a restore (the host took them off the counters)
__global__ void k_pool_take(DevCfg c, int32_t h, int32_t take, int64_t bump, int64_t n, int64_t* ids) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ids[i] = i < take ? (int64_t)c.pool_free[h - take + i] : bump + (i - take);
}
// blocks a restore did not use, back on the free stack (untouched: still zero for HyperLogLog)
__global__ void k_pool_give(DevCfg c, const int64_t* ids, int64_t n, int32_t h) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) c.pool_free[h + i] = (uint32_t)ids[i];
}

// partition of a restored row of key group kg (the caller vouches for hashed keys); -1 when a
// Long/Integer key does not belong to kg
__device__ __forceinline__ int32_t restore_partition(const DevCfg& c, int32_t kg, int64_t key) {
  if (c.key_kind != FW_KEY_HASHED && key_group(key_hash_of(c.key_kind, key, nullptr, 0), c.max_par) != kg) return -1;
  const uint32_t sub = c.log_s ? (uint32_t)(fmix64((uint64_t)key ^ 0x5851F42D4C957F2Dull) >> (64 - c.log_s)) : 0u;
  return ((kg - c.kg0) << c.log_s) | (int32_t)sub;
}

// demand of a restore per partition (to grow the table before inserting) and key-group errors
__global__ void k_restore_count(DevCfg c, int32_t kg, StateCols in, int64_t n, int32_t* demand, Status* st) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t p = restore_partition(c, kg, in.key[i]);
  if (p < 0)
    atomicAdd(&st->kg_errors, 1);
  else
    atomicAdd(&demand[p], 1);
}

// insert (or merge) restored rows; the table has room for all of them (k_restore_count + growth)
__global__ void k_restore(DevCfg c, int32_t kg, StateCols in, int64_t n, DevTable tb, Status* st,
                          const int32_t* round_of, int32_t round) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (round_of && round_of[i] != round)) return;
  const int32_t p = restore_partition(c, kg, in.key[i]);
  if (p < 0) return;
  Entry d;
  d.key = in.key[i];
  d.start = in.start[i];
  d.end = in.end[i];
  d.cnt = in.cnt[i];
  d.sum = in.sum[i];
  d.mn = c.vtype == FW_VAL_F64 ? f64_sortable(in.mn[i]) : in.mn[i];
  if (c.agg == FW_AGG_FIRST_MAX) d.mn = ~d.mn;
  d.mx = agg_first(c.agg) ? ~in.mx[i] : c.vtype == FW_VAL_F64 ? f64_sortable(in.mx[i]) : in.mx[i];
  if (agg_by(c.agg)) {  // (the selected field, its ordinal)
    d.mn = by_key(c.agg, c.vtype, in.mn[i]);
    d.mx = in.mx[i];
  }
  d.meta = c.panes ? in.timer[i] : in.timer[i] ? FW_TIMER : 0;
  const Region r = region_of(c, tb, p, tb.cur[p]);
  const uint64_t h = slot_hash(c, d.key, c.assigner == FW_SESSION ? 0 : d.start);
  const int32_t found = region_find(r, h, d.key, d.start, d.end);
  const uint8_t* acc = in.acc ? in.acc + i * in.acc_bytes : nullptr;
  if (found >= 0) {  // the window is already there (restored earlier, or an earlier round): AggregateFunction.merge
    Entry& x = r.ent[found];
    Entry cur = x;
    if (c.pool_bytes) {  // register max / the Table aggregates' merge into its block; a digest is not re-compressed here
      if (c.agg != FW_AGG_HLL && c.agg != FW_AGG_ROW) {
        atomicAdd(&st->acc_refused, 1);
        return;
      }
      block_import(c, pool_block_of(cur), acc, true);
    }
    acc_merge(c, cur, d);
    cur.meta = c.panes ? min(cur.meta, d.meta) : (cur.meta | d.meta);
    x = cur;
    atomicMin((long long*)&tb.next_timer[p], (long long)entry_timer(c, cur));
    return;
  }
  if (c.pool_bytes) {
    if (!acc_valid(c, acc)) {
      atomicAdd(&st->acc_refused, 1);
      return;
    }
    const uint64_t b = (uint64_t)in.blk[atomicAdd(in.used, 1)];
    block_import(c, b, acc, false);
    d.meta |= (int64_t)(b << 1);
  }
  const int32_t s = region_claim(r, h, SLOT_BUSY);
  if (s < 0) {
    atomicOr(&st->flags, FW_STATUS_STATE_LOST);
    return;
  }
  r.ent[s] = d;
  __threadfence();
  __hip_atomic_store(r.state + s, live_word(h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  atomicAdd(&tb.live[p], 1);
  atomicMin((long long*)&tb.next_timer[p], (long long)entry_timer(c, d));
}


// ============================================================== pre-shuffle combining
// A combiner operator (full KeyGroupRange, watermark never advanced) aggregates a subtask's batch before the keyBy
// exchange; its table is then drained into partial accumulators in key-group order, so each destination's share
// is one contiguous slice (KeyGroupRangeAssignment.computeOperatorIndexForKeyGroup, :115-117), and the receiving
// operator merges them (AggregateFunction.merge, AggregateFunction.java:160) as its own aggregate would have
// added the records.  Decomposable count/sum/min/max on tumbling windows without allowed lateness only: a late
// partial is dropped with all of its records (with lateness 0 a record of a late window is itself late,
// WindowOperator.java:402-418), and no record fires on arrival.
__global__ void k_live_u32(DevTable tb, int32_t P, uint32_t* offs) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p <= P) offs[p] = p < P ? (uint32_t)tb.live[p] : 0u;
}
// one workgroup per partition: its live entries at offs[p] in slot order, then the region emptied
__global__ __launch_bounds__(FW_FIRE_THREADS) void k_extract(DevCfg c, DevTable tb, const uint32_t* __restrict__ offs,
                                                            PartialCols out) {
  __shared__ uint32_t sw[FW_FIRE_THREADS / 64 + 1];
  __shared__ uint32_t run_s;
  const int32_t p = blockIdx.x;
  const Region r = region_of(c, tb, p, tb.cur[p]);
  const uint32_t R = c.dense ? (uint32_t)tb.live[p] : r.mask + 1;  // (dense regions: the live prefix)
  if (threadIdx.x == 0) run_s = 0;
  __syncthreads();
  for (uint32_t s0 = 0; s0 < R; s0 += blockDim.x) {
    const uint32_t s = s0 + threadIdx.x;
    const bool live = s < R && (c.dense || st_kind(ld_state(r.state + s)) == SLOT_LIVE);
    uint32_t total;
    const uint32_t pos = block_excl_scan(live ? 1u : 0u, sw, &total);
    if (live) {
      const Entry e = r.ent[s];
      const uint64_t o = (uint64_t)offs[p] + run_s + pos;
      out.key[o] = e.key;
      out.start[o] = e.start;
      out.cnt[o] = e.cnt;
      out.sum[o] = e.sum;
      out.mn[o] = c.agg == FW_AGG_HLL ? (int64_t)pool_block_of(e) : e.mn;  // (HLL: k_hll_extract reads it)
      out.mx[o] = e.mx;
    }
    if (s < R && !c.dense) r.state[s] = SLOT_EMPTY;
    __syncthreads();
    if (threadIdx.x == 0) run_s += total;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    tb.live[p] = 0;
    tb.next_timer[p] = LMAX;
  }
}
// the receiver: partials of its KeyGroupRange into partition runs (k_classify_hist counted them with the window
// start as the timestamp); late partials are dropped and counted with their records
__global__ __launch_bounds__(FW_TILE_THREADS) void k_pscatter(DevCfg c, int64_t wm, PartialCols in, int64_t n, int32_t T,
                                                             const uint32_t* __restrict__ offs,
                                                             PartialRec* __restrict__ part, Status* st) {
  extern __shared__ uint32_t base[];
  const int32_t tile = blockIdx.x;
  for (int i = threadIdx.x; i < c.P; i += blockDim.x) base[i] = offs[(int64_t)i * T + tile];
  __syncthreads();
  const int64_t tbase = (int64_t)tile * FW_TILE, tend = min(n, tbase + (int64_t)FW_TILE);
  unsigned long long late = 0, recs = 0;
  for (int64_t i = tbase + threadIdx.x; i < tend; i += blockDim.x) {
    const int64_t key = in.key[i], start = in.start[i];
    const int32_t p = partition_of(c, key, key_hash_of(c.key_kind, key, nullptr, i));
    if (p < 0) continue;  // counted by k_classify_hist
    recs += (unsigned long long)in.cnt[i];
    int64_t last = 0;
    int nw = 0;
    const int cls = classify(c, wm, start, &last, &nw);
    if (cls == CLS_NORMAL) {
      const uint32_t pos = atomicAdd(&base[p], 1u);
      part[pos] = PartialRec{key, start, in.cnt[i], in.sum[i], in.mn[i], in.mx[i]};
    } else if (cls == CLS_LATE) {
      late += (unsigned long long)in.cnt[i];
    }
  }
  if (late) atomicAdd(&st->late_dropped, late);
  if (recs) atomicAdd(&st->partial_records, recs);
}
// one workgroup per partition: its partials merged in the LDS table and flushed into the region (agg_flush);
// a flush the region cannot take suspends the launch, and the resumed one restarts from the last flush that
// succeeded (prog.rb = its round, prog.tp = whether the thread's partial of that round was in it)
__global__ __launch_bounds__(FW_AGG_THREADS) void k_pmerge(DevCfg c, const PartialRec* __restrict__ part,
                                                          const uint32_t* __restrict__ offs, int32_t T, DevTable tb,
                                                          AggProg prog, int resume, Status* st) {
  if (c.agg != FW_AGG_HLL) {  // (HLL partials: their counts merge here, new windows take blocks; registers follow)
    c.pool_bytes = 0;
    c.agg = FW_AGG_COUNT_SUM_MIN_MAX;
  }
  __shared__ AggLds L;
  const int32_t p = blockIdx.x;
  if (p >= c.P || (resume && prog.done[p])) return;
  const int64_t begin = offs[(int64_t)p * T], end = offs[(int64_t)(p + 1) * T];
  if (begin == end) {
    if (threadIdx.x == 0) prog.done[p] = 1;
    return;
  }
  int64_t ck_rb = resume ? (int64_t)prog.rb[p] : begin;
  bool ck_done = resume ? prog.tp[(int64_t)p * FW_AGG_THREADS + threadIdx.x] != 0 : false;
  for (int h = threadIdx.x; h < FW_LDS_SLOTS; h += blockDim.x) L.tag[h] = LT_EMPTY;
  if (threadIdx.x == 0) {
    L.fill = 0;
    L.anyfail = 0;
    L.nnew = 0;
    L.live = tb.live[p];
    L.flushed = 0;
    L.min_timer = LMAX;
  }
  __syncthreads();
  const Region r = region_of(c, tb, p, tb.cur[p]);
  bool ok = true;
  for (int64_t rb = ck_rb; rb < end && ok; rb += blockDim.x) {
    const int64_t i = rb + threadIdx.x;
    bool done = i >= end || (rb == ck_rb && ck_done);
    PartialRec d{};
    if (!done) d = part[i];
    for (;;) {
      if (!done) {
        const int tg = lds_slot(L, d.key, d.start);
        if (tg >= 0) {
          atomicAdd(&L.cnt[tg], (uint32_t)d.cnt);
          // (HLL: the count only, as LDS_CNT_ONLY in the record path; a partial's sum column is its register count,
          // which is not part of the accumulator, so snapshots of combined and uncombined windows agree)
          if (c.agg != FW_AGG_HLL) {
            if (c.vtype == FW_VAL_F64)
              atomicAdd((double*)&L.sum[tg], __longlong_as_double(d.sum));
            else
              atomicAdd((unsigned long long*)&L.sum[tg], (unsigned long long)d.sum);
            atomicMin((long long*)&L.mn[tg], (long long)d.mn);
            atomicMax((long long*)&L.mx[tg], (long long)d.mx);
          }
          done = true;
        } else {
          L.anyfail = 1;
        }
      }
      __syncthreads();
      const int need = L.anyfail;
      __syncthreads();
      if (!need) break;
      if (!agg_flush(c, L, r, st)) {
        ok = false;
        break;
      }
      ck_rb = rb;
      ck_done = done;
      if (threadIdx.x == 0) L.anyfail = 0;
      __syncthreads();
    }
  }
  if (ok) ok = agg_flush(c, L, r, st);
  if (!ok) {
    prog.tp[(int64_t)p * FW_AGG_THREADS + threadIdx.x] = ck_done ? 1u : 0u;
    if (threadIdx.x == 0) {
      prog.rb[p] = ck_rb;
      prog.done[p] = 0;
      atomicOr(&st->suspended, (int)FW_SUSP_AGG);
    }
  } else if (threadIdx.x == 0) {
    prog.done[p] = 1;
  }
  if (threadIdx.x == 0) agg_publish(c, L, tb, p, st);
}

// ---- HyperLogLog partials (pre-shuffle combining): a combined window crosses the exchange as its
// partial row (key, start, count; sum = how many of its registers are non-zero) and those registers as u32
// (index << 8 | rank), in partial order.  The receiver merges the counts like any partial (k_pmerge creates the
// windows and their blocks) and raises the registers into the blocks: AggregateFunction.merge = register max
// (AggregateFunction.java:160), so the result equals pushing the records themselves.
__device__ __forceinline__ void hll_raise_jr(const DevCfg& c, uint64_t blk, uint32_t j, uint32_t rank) {
  uint8_t* base = c.pool + blk * (uint64_t)c.pool_bytes;
  uint32_t* w = reinterpret_cast<uint32_t*>(base + hll_hdr_bytes(c.hll_p) + (j & ~3u));
  const int sh = (int)(j & 3) * 8;
  uint32_t o = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (((o >> sh) & 0xffu) < rank) {
    const uint32_t nw = (o & ~(0xffu << sh)) | (rank << sh);
    if (__hip_atomic_compare_exchange_strong(w, &o, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
      if (((o >> sh) & 0xffu) == 0u) {
        const uint32_t ch = j >> 4;
        atomicOr(reinterpret_cast<uint32_t*>(base) + (ch >> 5), 1u << (ch & 31u));
      }
      break;
    }
  }
}
// combiner side (the block id is in mn, k_extract).  A thread per partial; a partial of more than HLL_WAVE_CNT
// records (a hot key's window: up to 2^p registers) is taken by its whole wave afterwards, lane l over the block's
// bitmap words l, l + 64, ... (a word covers 32 chunks of 16 registers).  Pass 1 counts the non-zero registers;
// pass 2 writes them at the scanned offsets in index order, then zeroes and frees the block (the combiner is
// emptied).
constexpr int64_t HLL_WAVE_CNT = 256;
__device__ __forceinline__ uint32_t hll_nz16(const uint4 v) {
  const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
  uint32_t k = 0;
#pragma unroll
  for (int u = 0; u < 4; u++)
#pragma unroll
    for (int y = 0; y < 32; y += 8) k += ((ws[u] >> y) & 0xffu) != 0u;
  return k;
}
// the non-zero registers of block blk's bitmap words w0, w0 + ws, ... (ws = 1: one thread, 64: a wave's lane)
__device__ __forceinline__ uint32_t hll_count_words(const DevCfg& c, uint64_t blk, int32_t w0, int32_t ws) {
  const uint8_t* base = c.pool + blk * (uint64_t)c.pool_bytes;
  const uint32_t* bits = reinterpret_cast<const uint32_t*>(base);
  const uint4* q = reinterpret_cast<const uint4*>(base + hll_hdr_bytes(c.hll_p));
  const int32_t nw = (int32_t)((((int64_t)1 << c.hll_p) / 16 + 31) / 32);
  uint32_t k = 0;
  for (int32_t w = w0; w < nw; w += ws) {
    uint32_t word = bits[w];
    while (word) {
      const int b = __ffs(word) - 1;
      word &= word - 1;
      k += hll_nz16(q[w * 32 + b]);
    }
  }
  return k;
}
// writes word w's registers from position o on, zeroes its chunks and the word; returns the new position
__device__ __forceinline__ uint64_t hll_take_word(const DevCfg& c, uint64_t blk, int32_t w, uint64_t o,
                                                  uint32_t* __restrict__ regs) {
  uint8_t* base = c.pool + blk * (uint64_t)c.pool_bytes;
  uint32_t* bits = reinterpret_cast<uint32_t*>(base);
  uint4* q = reinterpret_cast<uint4*>(base + hll_hdr_bytes(c.hll_p));
  uint32_t word = bits[w];
  if (!word) return o;
  while (word) {
    const int b = __ffs(word) - 1;
    word &= word - 1;
    const int32_t ch = w * 32 + b;
    const uint4 v = q[ch];
    const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int u = 0; u < 4; u++)
#pragma unroll
      for (int y = 0; y < 4; y++) {
        const uint32_t rank = (ws[u] >> (8 * y)) & 0xffu;
        if (rank) regs[o++] = ((uint32_t)(ch * 16 + u * 4 + y) << 8) | rank;
      }
    q[ch] = make_uint4(0, 0, 0, 0);
  }
  bits[w] = 0u;
  return o;
}
__global__ __launch_bounds__(256) void k_hll_extract_counts(DevCfg c, PartialCols out, int64_t n,
                                                            uint32_t* __restrict__ cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = __lane_id();
  const bool in = i < n;
  const bool big = in && out.cnt[i] > HLL_WAVE_CNT;
  const uint64_t blk = in ? (uint64_t)out.mn[i] : 0;
  if (in && !big) {
    const uint32_t k = hll_count_words(c, blk, 0, 1);
    out.sum[i] = (int64_t)k;
    cnt[i] = k;
  }
  uint64_t m = __ballot(big);
  while (m) {
    const int src = __ffsll((long long)m) - 1;
    m &= m - 1;
    const uint64_t b = (uint64_t)__shfl((long long)blk, src, 64);
    uint32_t k = hll_count_words(c, b, lane, 64);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) k += (uint32_t)__shfl_xor((int)k, o, 64);
    if (lane == src) {
      out.sum[i] = (int64_t)k;
      cnt[i] = k;
    }
  }
}
__global__ __launch_bounds__(256) void k_hll_extract_regs(DevCfg c, PartialCols out, int64_t n,
                                                          const uint32_t* __restrict__ off, uint32_t* __restrict__ regs) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = __lane_id();
  const bool in = i < n;
  const bool big = in && out.cnt[i] > HLL_WAVE_CNT;
  const uint64_t blk = in ? (uint64_t)out.mn[i] : 0;
  const int32_t nw = (int32_t)((((int64_t)1 << c.hll_p) / 16 + 31) / 32);
  if (in && !big) {
    uint64_t o = off[i];
    for (int32_t w = 0; w < nw; w++) o = hll_take_word(c, blk, w, o, regs);
  }
  uint64_t m = __ballot(big);
  while (m) {
    const int src = __ffsll((long long)m) - 1;
    m &= m - 1;
    const uint64_t b = (uint64_t)__shfl((long long)blk, src, 64);
    uint64_t o0 = (uint64_t)__shfl((long long)(in ? off[i] : 0), src, 64);
    for (int32_t w0 = 0; w0 < nw; w0 += 64) {
      const int32_t w = w0 + lane;
      const uint32_t mine = w < nw ? hll_count_words(c, b, w, nw) : 0u;  // (this word only)
      uint32_t x = mine;  // inclusive prefix over the lanes (words in order)
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
        if (lane >= o) x += y;
      }
      if (w < nw) (void)hll_take_word(c, b, w, o0 + x - mine, regs);
      o0 += (uint64_t)__shfl((int)x, 63, 64);
    }
  }
  if (in) {
    out.mn[i] = LMAX;  // (the partial's min / max are not value statistics for HLL)
    __threadfence();
    c.pool_free[atomicAdd(&c.pool_ctr[0], 1)] = (uint32_t)blk;
  }
}
// receiver: each partial's registers raised into its window's block (a late or foreign partial was dropped and
// counted by the scatter); regs of partial i start at off[i]
// (a thread per partial; one with more than 64 registers is raised by its whole wave afterwards)
__global__ __launch_bounds__(256) void k_hll_push_regs(DevCfg c, int64_t wm, PartialCols in, int64_t n,
                                                       const uint32_t* __restrict__ regs,
                                                       const uint32_t* __restrict__ off, DevTable tb, Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;  // rerun when resumed
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = __lane_id();
  int64_t blk = -1;
  uint64_t b0 = 0, b1 = 0;
  if (i < n) {
    const int64_t key = in.key[i], start = in.start[i];
    const int32_t p = partition_of(c, key, key_hash_of(c.key_kind, key, nullptr, i));
    if (p >= 0 && classify(c, wm, start) == CLS_NORMAL) {
      const Region r = region_of(c, tb, p, tb.cur[p]);
      const int32_t slot = region_find(r, slot_hash(c, key, start), key, start, wend(c, start));
      if (slot < 0)
        atomicOr(&st->flags, FW_STATUS_STATE_LOST);  // k_pmerge stored every partial's window
      else
        blk = (int64_t)pool_block_of(r.ent[slot]);
      b0 = off[i];
      b1 = b0 + (uint64_t)in.sum[i];
    }
  }
  const bool big = blk >= 0 && b1 - b0 > 64;
  if (blk >= 0 && !big)
    for (uint64_t k = b0; k < b1; k++) hll_raise_jr(c, (uint64_t)blk, regs[k] >> 8, regs[k] & 0xffu);
  uint64_t m = __ballot(big);
  while (m) {
    const int src = __ffsll((long long)m) - 1;
    m &= m - 1;
    const uint64_t b = (uint64_t)__shfl((long long)blk, src, 64);
    const uint64_t s0 = (uint64_t)__shfl((long long)b0, src, 64), s1 = (uint64_t)__shfl((long long)b1, src, 64);
    for (uint64_t k = s0 + lane; k < s1; k += 64) hll_raise_jr(c, b, regs[k] >> 8, regs[k] & 0xffu);
  }
}

// out3 = {live entries, event-time timers}
__global__ __launch_bounds__(FW_FIRE_THREADS) void k_table_stats(DevCfg c, DevTable tb, unsigned long long* out3) {
  const int32_t p = blockIdx.x;
  const Region r = region_of(c, tb, p, tb.cur[p]);
  unsigned long long live = 0, timers = 0;
  const uint32_t lim = c.dense ? (uint32_t)tb.live[p] : r.mask + 1;  // (dense regions: the live prefix)
  for (uint32_t s = threadIdx.x; s < lim; s += blockDim.x) {
    if (!c.dense && st_kind(ld_state(r.state + s)) != SLOT_LIVE) continue;
    const Entry& e = r.ent[s];
    if (c.panes) {  // one pending timer per pane (its next window end); formed-out panes are garbage
      if (max(e.meta, tb.pane_floor[p]) > jsub(jadd(e.start, c.size), 1)) continue;
      live++;
      timers++;
      continue;
    }
    live++;
    const int64_t mx = jsub(e.end, 1), cl = cleanup_of(e.end, c.lateness);
    if (e.meta & FW_TIMER) timers++;
    if (cl != LMAX && !((e.meta & FW_TIMER) && cl == mx)) timers++;
  }
  if (live) atomicAdd(&out3[0], live);
  if (timers) atomicAdd(&out3[1], timers);
}

// ============================================================== dense tumbling regions (DevCfg::dense)
// Tumbling windows with the count/sum/min/max accumulator and allowed lateness 0 (BASELINE configs[1]; the state
// op replaced is HeapAggregatingState.add over CopyOnWriteStateTable.transform, CopyOnWriteStateTable.java:449-495).
// Every record of a batch lands in a window that ends after the watermark, and a window is removed when it fires, so
// a region's live entries are few and nearly all of them are touched by every batch.  A region therefore keeps its
// entries densely in slots [0, live) of its current buffer (no state words, no probing in HBM):
//   k_dt_aggregate  loads the region's entries into an LDS hash table, adds the batch's records (or merges partial
//                   accumulators: combining, restore), and writes every group densely into the region's other buffer
//                   (whole 64-byte entries, coalesced); a region is committed (buffer flipped) only when all of its
//                   groups are written, so a suspended launch resumes by redoing the regions not yet committed;
//   k_dt_fire       streams the due regions' entries: windows with maxTimestamp <= wm are emitted
//                   (WindowOperator.onEventTime, :424-469), the rest are copied into the other buffer.
// A region whose entries and new groups exceed the LDS table is done in 2^b passes, each over the (key, window)s
// whose hash has prefix k: every pass reads the region and the records again and keeps its share.
enum { DT_RECS = 0, DT_PARTS = 1 };
enum { DT_OK = 0, DT_OVER = 1, DT_WIDE = 2 };  // an attempt's outcome (dt_attempt)
// The LDS table has two layouts.  The compact one (DtLdsK) keys a slot by the 64-bit CRec word of (key, window)
// (compact_encode: fmix64 of the key with the window delta in its top log_s bits, unique inside a region): a lookup
// reads one word, a claim is one 64-bit CAS (the accumulators are initialised when the table is cleared).  The wide
// one (DtLds: {key, window start} behind a fingerprint tag, the protocol of lds_slot) takes what has no compact form
// (a wide batch, partials, entries far from the watermark).
constexpr int DT_LIMIT = FW_DT_SLOTS * 13 / 16;  // claims stop here, so every probe chain ends at an EMPTY slot
constexpr int DT_BUCKETS = FW_DT_SLOTS / 4;
static_assert(FW_DT_SLOTS % 4 == 0, "FW_DT_SLOTS: buckets of 4");
struct DtLds {
  uint32_t tag[FW_DT_SLOTS];  // LT_EMPTY, LT_BUSY or a fingerprint >= 2 of (key, window start)
  i64x2 kv[FW_DT_SLOTS];      // {key, window start}
  unsigned long long cnt[FW_DT_SLOTS];
  int64_t sum[FW_DT_SLOTS], mn[FW_DT_SLOTS], mx[FW_DT_SLOTS];
};
constexpr int DK_SLOTS = (int)(sizeof(DtLds) / 36 / 16 * 16);  // 36 bytes a slot
#ifndef FW_DK_FILL16
#define FW_DK_FILL16 15  // claims stop at this many 16ths of the compact table (buckets of 4 keep probes short)
#endif
constexpr int DK_LIMIT = DK_SLOTS * FW_DK_FILL16 / 16;
constexpr unsigned long long DK_EMPTY = ~0ull;  // (a record or entry whose word is this takes the wide table)
#ifndef FW_DK_BW
#define FW_DK_BW 4  // slots per bucket of the compact table (4: a 32-byte read per probe, 2: one 16-byte read)
#endif
constexpr int DK_BW = FW_DK_BW;
constexpr int DK_BUCKETS = DK_SLOTS / DK_BW;  // a word's home is a bucket of DK_BW slots
// A compact slot's count is the 32-bit count of the region's window so far (an entry whose count would not fit sends
// its region to the wide table); min and max sit side by side, read together before either is raised.
struct DtLdsK {
  i64x2 mm[DK_SLOTS];  // {min, max}
  alignas(16) unsigned long long kw[DK_SLOTS];
  int64_t sum[DK_SLOTS];
  uint32_t cnt[DK_SLOTS];
};
union DtTab {
  DtLds w;
  DtLdsK k;
};
struct DtMisc {
  int fill, over, nout, capover, widefb;
  long long ntmin, out;
};
__device__ __forceinline__ uint32_t dt_bucket(uint32_t h) { return (uint32_t)(((uint64_t)h * DT_BUCKETS) >> 32); }
// first slot of the word's home bucket
__device__ __forceinline__ uint32_t dk_home(unsigned long long kw) {
  uint32_t h = (uint32_t)(kw >> 32) * 0x9E3779B1u ^ (uint32_t)kw;
  h ^= h >> 15;
  return (uint32_t)(((uint64_t)h * DK_BUCKETS) >> 32) * (uint32_t)DK_BW;
}
// the DK_BW words of the bucket at slot s0
__device__ __forceinline__ void dk_read4(const DtLdsK& K, uint32_t s0, unsigned long long (&g)[DK_BW]) {
#pragma unroll
  for (int q = 0; q < DK_BW; q += 2) {
    const i64x2 a = *reinterpret_cast<const i64x2*>(&K.kw[s0 + q]);
    g[q] = (unsigned long long)a.x, g[q + 1] = (unsigned long long)a.y;
  }
}
// the hash pass of (key, window): prefix of a hash independent of the LDS slot's
__device__ __forceinline__ int dt_pass(const DevCfg& c, int64_t key, int64_t start, int hb) {
  return hb ? (int)((uint32_t)(slot_hash(c, key, start) >> 32) >> (32 - hb)) : 0;
}
// one claim ticket below the table's fill limit
__device__ __forceinline__ bool dt_ticket(DtMisc& M, int limit) {
  if (__hip_atomic_load(&M.fill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= limit) return false;
  if (atomicAdd(&M.fill, 1) < limit) return true;
  atomicSub(&M.fill, 1);
  return false;
}
// wide table: find or claim the slot of (key, start); -1 at the fill limit (the protocol of lds_slot)
__device__ __forceinline__ int dt_slot(DtLds& L, DtMisc& M, int64_t key, int64_t start, uint32_t h) {
  const uint32_t fp = lds_fp(h);
  uint32_t b = dt_bucket(h);
  for (int guard = 0; guard < 4 * DT_BUCKETS;) {
    asm volatile("" ::: "memory");
    const u32x4 t4 = *reinterpret_cast<const u32x4*>(&L.tag[b * 4]);
    int found = -1;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t tq = q == 0 ? t4.x : q == 1 ? t4.y : q == 2 ? t4.z : t4.w;
      if (found < 0 && tq == fp) {
        asm volatile("" ::: "memory");
        const i64x2 kq = L.kv[b * 4 + q];
        if (kq.x == key && kq.y == start) found = (int)b * 4 + q;
      }
    }
    if (found >= 0) return found;
    const int empty = t4.x == LT_EMPTY ? 0 : t4.y == LT_EMPTY ? 1 : t4.z == LT_EMPTY ? 2 : t4.w == LT_EMPTY ? 3 : -1;
    const bool busy = t4.x == LT_BUSY || t4.y == LT_BUSY || t4.z == LT_BUSY || t4.w == LT_BUSY;
    if (busy) {  // a slot of this bucket is being published: re-read it
      guard++;
      continue;
    }
    if (empty >= 0) {
      if (!dt_ticket(M, DT_LIMIT)) return -1;
      const int s = (int)b * 4 + empty;
      if (atomicCAS(&L.tag[s], LT_EMPTY, LT_BUSY) == LT_EMPTY) {
        L.kv[s] = i64x2{key, start};
        L.cnt[s] = 0;
        L.sum[s] = 0;
        L.mn[s] = LMAX;
        L.mx[s] = LMIN;
        __hip_atomic_store(&L.tag[s], fp, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        return s;
      }
      atomicSub(&M.fill, 1);
      continue;  // lost the claim race: re-read the bucket
    }
    b = b + 1 == (uint32_t)DT_BUCKETS ? 0u : b + 1;  // bucket full without a match
    guard++;
  }
  return -1;
}
// compact table: find or claim the slot of word kw from the bucket at slot s0 on; -1 at the fill limit.  A word is
// claimed in the first EMPTY slot of the first bucket that has one (buckets in probe order, slots in bucket order), and
// a slot never empties while the table is in use, so a lookup that meets a bucket with an EMPTY slot and no match
// knows the word is absent; a lost claim race re-reads the bucket.
__device__ __forceinline__ int dk_slot(DtLdsK& K, DtMisc& M, unsigned long long kw, uint32_t s0) {
  for (int guard = 0; guard < 2 * DK_BUCKETS;) {
    asm volatile("" ::: "memory");
    unsigned long long g[DK_BW];
    dk_read4(K, s0, g);
    int e = -1;
#pragma unroll
    for (int q = DK_BW - 1; q >= 0; q--) {
      if (g[q] == kw) return (int)s0 + q;
      if (g[q] == DK_EMPTY) e = q;
    }
    if (e >= 0) {
      if (!dt_ticket(M, DK_LIMIT)) return -1;
      const unsigned long long o = atomicCAS(&K.kw[s0 + e], DK_EMPTY, kw);
      if (o == DK_EMPTY) return (int)s0 + e;  // claimed (the accumulators were initialised with the table)
      atomicSub(&M.fill, 1);
      if (o == kw) return (int)s0 + e;
      continue;
    }
    s0 = s0 + DK_BW == (uint32_t)DK_SLOTS ? 0u : s0 + DK_BW;
    guard++;
  }
  return -1;
}
// AggregateFunction.add of one element (the value in the table's representation: f64 min/max sortable), and
// AggregateFunction.merge of an accumulator in that representation, into slot s of either layout
template <class L>
__device__ __forceinline__ void dt_add(L& T, int s, int vtype, int64_t v) {
  atomicAdd(&T.cnt[s], 1ull);
  int64_t sv = v;
  if (vtype == FW_VAL_F64) {
    atomicAdd((double*)&T.sum[s], __longlong_as_double(v));
    sv = f64_sortable(v);
  } else {
    atomicAdd((unsigned long long*)&T.sum[s], (unsigned long long)v);
  }
  atomicMin((long long*)&T.mn[s], (long long)sv);
  atomicMax((long long*)&T.mx[s], (long long)sv);
}
// the compact table: the count as a 32-bit add, min / max raised only when the element passes them (a stale read
// can only be above the minimum / below the maximum, so skipping is exact; LDS atomics are the record loop's cost)
__device__ __forceinline__ void dt_add(DtLdsK& T, int s, int vtype, int64_t v) {
  atomicAdd(&T.cnt[s], 1u);
  int64_t sv = v;
  if (vtype == FW_VAL_F64) {
    atomicAdd((double*)&T.sum[s], __longlong_as_double(v));
    sv = f64_sortable(v);
  } else {
    atomicAdd((unsigned long long*)&T.sum[s], (unsigned long long)v);
  }
  const i64x2 m = T.mm[s];
  long long* mp = reinterpret_cast<long long*>(&T.mm[s]);
  if (sv < m.x) atomicMin(mp, (long long)sv);
  if (sv > m.y) atomicMax(mp + 1, (long long)sv);
}
__device__ __forceinline__ void dt_merge(DtLdsK& T, int s, int vtype, int64_t cnt, int64_t sum, int64_t mn, int64_t mx) {
  atomicAdd(&T.cnt[s], (uint32_t)cnt);
  if (vtype == FW_VAL_F64)
    atomicAdd((double*)&T.sum[s], __longlong_as_double(sum));
  else
    atomicAdd((unsigned long long*)&T.sum[s], (unsigned long long)sum);
  long long* mp = reinterpret_cast<long long*>(&T.mm[s]);
  atomicMin(mp, (long long)mn);
  atomicMax(mp + 1, (long long)mx);
}
template <class L>
__device__ __forceinline__ void dt_merge(L& T, int s, int vtype, int64_t cnt, int64_t sum, int64_t mn, int64_t mx) {
  atomicAdd(&T.cnt[s], (unsigned long long)cnt);
  if (vtype == FW_VAL_F64)
    atomicAdd((double*)&T.sum[s], __longlong_as_double(sum));
  else
    atomicAdd((unsigned long long*)&T.sum[s], (unsigned long long)sum);
  atomicMin((long long*)&T.mn[s], (long long)mn);
  atomicMax((long long*)&T.mx[s], (long long)mx);
}
// RPT elements into the wide table: home buckets and candidates looked up together, the rest one by one
// (lds_upsert_batch's shape); dm: bit j = element j done or absent.  false when the table is full.
template <int RPT>
__device__ __forceinline__ bool dt_add_batch(DtLds& L, DtMisc& M, int vtype, const int64_t (&k)[RPT],
                                             const int64_t (&s)[RPT], const int64_t (&v)[RPT], uint32_t dm) {
  uint32_t hh[RPT], b[RPT], fp[RPT];
  u32x4 t4[RPT];
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    hh[j] = lds_hash(k[j], s[j]);
    fp[j] = lds_fp(hh[j]);
    b[j] = dt_bucket(hh[j]);
    if (!(dm >> j & 1)) t4[j] = *reinterpret_cast<const u32x4*>(&L.tag[b[j] * 4]);
  }
  int cand[RPT];
  i64x2 kv[RPT];
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    cand[j] = -1;
    if (dm >> j & 1) continue;
    const u32x4 t = t4[j];
    cand[j] = t.x == fp[j] ? 0 : t.y == fp[j] ? 1 : t.z == fp[j] ? 2 : t.w == fp[j] ? 3 : -1;
    if (cand[j] >= 0) kv[j] = L.kv[b[j] * 4 + cand[j]];
  }
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    if (cand[j] < 0 || kv[j].x != k[j] || kv[j].y != s[j]) continue;
    dt_add(L, (int)b[j] * 4 + cand[j], vtype, v[j]);
    dm |= 1u << j;
  }
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    if (dm >> j & 1) continue;
    const int t = dt_slot(L, M, k[j], s[j], hh[j]);
    if (t < 0) return false;
    dt_add(L, t, vtype, v[j]);
  }
  return true;
}
// the same for compact words: every home slot read together, then claims / probes one by one
template <int RPT>
__device__ __forceinline__ bool dk_add_batch(DtLdsK& K, DtMisc& M, int vtype, const unsigned long long (&w)[RPT],
                                             const int64_t (&v)[RPT], uint32_t dm) {
  uint32_t s[RPT];
  unsigned long long g[RPT][DK_BW];
  // every home bucket read before any is used (plain reads: a word, once claimed, never changes, and a stale EMPTY
  // only sends the element to dk_slot, which re-reads)
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    s[j] = dk_home(w[j]);
    dk_read4(K, s[j], g[j]);
  }
  uint32_t miss = 0;
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    if (dm >> j & 1) continue;
    int q = -1;
#pragma unroll
    for (int b = DK_BW - 1; b >= 0; b--)
      if (g[j][b] == w[j]) q = b;
    if (q >= 0)
      dt_add(K, (int)s[j] + q, vtype, v[j]);
    else
      miss |= 1u << j;
  }
  if (miss) {
#pragma unroll
    for (int j = 0; j < RPT; j++) {
      if (!(miss >> j & 1)) continue;
      const int t = dk_slot(K, M, w[j], s[j]);
      if (t < 0) return false;
      dt_add(K, t, vtype, v[j]);
    }
  }
  return true;
}

#ifndef FW_DT_TIMING
#define FW_DT_TIMING 0  // 1: per-phase clocks of the compact launch, printed by its last workgroup (diagnostics)
#endif
__device__ unsigned long long g_dtt[6];
// One attempt at a region: 2^hb passes over the (key, window)s by hash prefix; each clears the table, loads the
// region's entries of the pass, adds the records of the pass and writes the pass's groups densely into dst
// behind the earlier passes' (M.out).  KW: the compact table (every record is a CRec; an entry or record without a
// compact word makes the attempt DT_WIDE).  DT_OVER: some pass did not fit the table.  NAR: a launch whose every
// record is narrow (nar then always holds), with the ring of raw pairs below and no other record path
template <int SRC, bool KW, bool NAR>
__device__ __forceinline__ int dt_attempt(const DevCfg& c, DtTab& U, DtMisc& M, int32_t p, const Entry* __restrict__ src,
                                          int32_t live, Entry* __restrict__ dst, int64_t R, const void* __restrict__ in,
                                          int64_t begin, int64_t end, bool cmp, int hb, bool nar) {
  constexpr int NS = KW ? DK_SLOTS : FW_DT_SLOTS;
  const PRec* __restrict__ part = reinterpret_cast<const PRec*>(in);
  const PartialRec* __restrict__ pin = reinterpret_cast<const PartialRec*>(in);
  const int lane = __lane_id();
  if (threadIdx.x == 0) {
    M.out = 0;
    M.ntmin = LMAX;
    M.capover = 0;
    M.widefb = 0;
  }
  // compact records: each pass's first round of records is loaded before the table is cleared and the region's
  // entries are read, so its latency overlaps theirs (two register sets, alternating without copies: round r is
  // added while round r + 1 loads; branch-free loads from an index clamped into the run)
  constexpr int RPT = FW_DT_RPT;
  constexpr int64_t RS = (int64_t)FW_DT_THREADS * RPT;
  const i64x2* __restrict__ crec = reinterpret_cast<const i64x2*>(in);
  const uint64_t* __restrict__ nrec = reinterpret_cast<const uint64_t*>(in);
  // record j of this thread in the round at r0: CRecs lane-strided; narrow records (nar) in lane pairs, so a lane
  // reads its two with one 16-byte load (the run starts at an even record: p * 2 rcap)
  auto ridx = [&](int64_t r0, int j) -> int64_t {
    return nar ? r0 + (int64_t)(j & ~1) * FW_DT_THREADS + 2 * (int64_t)threadIdx.x + (j & 1)
               : r0 + (int64_t)j * FW_DT_THREADS + threadIdx.x;
  };
  auto load = [&](i64x2 (&d)[RPT], int64_t r0) {
    if (nar) {
      static_assert(RPT % 2 == 0, "narrow records are loaded in pairs");
#pragma unroll
      for (int j = 0; j < RPT; j += 2) {
        int64_t i = r0 + (int64_t)j * FW_DT_THREADS + 2 * (int64_t)threadIdx.x;
        if (i >= end) i = (end - 1) & ~(int64_t)1;
        const i64x2 q = *reinterpret_cast<const i64x2*>(nrec + i);
        d[j] = narrow_to_crec(c, (uint64_t)q.x);
        d[j + 1] = narrow_to_crec(c, (uint64_t)q.y);
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < RPT; j++) {
      const int64_t i = r0 + (int64_t)j * FW_DT_THREADS + threadIdx.x;
      d[j] = crec[i < end ? i : end - 1];
    }
  };
  // narrow records in the compact table: ND rounds in flight as raw pairs (a raw pair is 4 registers, a widened
  // record 4 per record), widened only when their round is added -- a widening at the load would wait for it there
  constexpr int ND = FW_DT_NDEPTH;
  static_assert(RPT % 2 == 0, "narrow records are loaded in pairs");
  auto load_raw = [&](i64x2 (&q)[RPT / 2], int64_t r0) {
#pragma unroll
    for (int j = 0; j < RPT; j += 2) {
      int64_t i = r0 + (int64_t)j * FW_DT_THREADS + 2 * (int64_t)threadIdx.x;
      if (i >= end) i = (end - 1) & ~(int64_t)1;
      q[j / 2] = *reinterpret_cast<const i64x2*>(nrec + i);
    }
  };
  constexpr bool ring = KW && SRC == DT_RECS && NAR && ND > 0;
  i64x2 ra[RPT], rn[RPT], rq[ND > 0 ? ND : 1][RPT / 2];
  for (int k = 0; k < (1 << hb); k++) {
    if constexpr (ring) {  // (the other rounds after the entries: their registers would spill beside the entries')
      load_raw(rq[0], begin);
    } else if constexpr (KW && SRC == DT_RECS) {
      load(ra, begin);
    }
    if constexpr (KW) {
      for (int h = threadIdx.x; h < DK_SLOTS; h += FW_DT_THREADS) {
        U.k.kw[h] = DK_EMPTY;
        U.k.cnt[h] = 0u;
        U.k.sum[h] = 0;
        U.k.mm[h] = i64x2{LMAX, LMIN};
      }
    } else {
      for (int h = threadIdx.x; h < FW_DT_SLOTS; h += FW_DT_THREADS) U.w.tag[h] = LT_EMPTY;
    }
    if (threadIdx.x == 0) {
      M.fill = 0;
      M.over = 0;
      M.nout = 0;
    }
    const unsigned long long ta = FW_DT_TIMING ? __builtin_amdgcn_s_memtime() : 0;
    __syncthreads();
    // the region's entries of pass k (two per thread in flight)
    for (int32_t i0 = 0; i0 < live; i0 += 2 * FW_DT_THREADS) {
      Entry e[2];
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const int32_t i = i0 + u * FW_DT_THREADS + (int32_t)threadIdx.x;
        if (i < live) e[u] = src[i];
      }
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const int32_t i = i0 + u * FW_DT_THREADS + (int32_t)threadIdx.x;
        if (i >= live || (hb && dt_pass(c, e[u].key, e[u].start, hb) != k)) continue;
        int s;
        if constexpr (KW) {
          const int64_t d = compact_delta(c, e[u].start);
          const unsigned long long w = d < 0 ? DK_EMPTY : (unsigned long long)compact_encode(c, e[u].key, d);
          // (a window's count must stay below 2^32 with this batch's records added: else the wide table)
          if (w == DK_EMPTY || (uint64_t)e[u].cnt + (uint64_t)(end - begin) > 0xffffffffull) {
            M.widefb = 1;
            break;
          }
          s = dk_slot(U.k, M, w, dk_home(w));
          if (s < 0) {
            M.over = 1;
            break;
          }
          dt_merge(U.k, s, c.vtype, e[u].cnt, e[u].sum, e[u].mn, e[u].mx);
        } else {
          s = dt_slot(U.w, M, e[u].key, e[u].start, lds_hash(e[u].key, e[u].start));
          if (s < 0) {
            M.over = 1;
            break;
          }
          dt_merge(U.w, s, c.vtype, e[u].cnt, e[u].sum, e[u].mn, e[u].mx);
        }
      }
    }
    __syncthreads();
    const unsigned long long tb1 = FW_DT_TIMING ? __builtin_amdgcn_s_memtime() : 0;
    if (M.widefb) return DT_WIDE;
    if (!M.over) {
      if constexpr (SRC == DT_RECS) {
        // the batch's records, the next round's in flight while the current ones are added (a load under a branch
        // is waited for at once)
        if constexpr (KW) {
          auto add_round = [&](const i64x2 (&cur)[RPT], int64_t r0) -> int {  // 0 done, 1 table full, 2 EMPTY word
            unsigned long long ww[RPT];
            int64_t vv[RPT];
            uint32_t dm = 0;
            bool bad = false;
#pragma unroll
            for (int j = 0; j < RPT; j++) {
              ww[j] = (unsigned long long)cur[j].x;
              vv[j] = cur[j].y;
              const int64_t i = ridx(r0, j);
              if (i >= end) {
                dm |= 1u << j;
                continue;
              }
              bad |= ww[j] == DK_EMPTY;
              if (hb) {
                int64_t kk, tt;
                compact_decode(c, p, cur[j].x, &kk, &tt);
                if (dt_pass(c, kk, tt, hb) != k) dm |= 1u << j;
              }
            }
            if (bad) return 2;
            return dk_add_batch<RPT>(U.k, M, c.vtype, ww, vv, dm) ? 0 : 1;
          };
          int res = 0;  // (ra / rq: loaded at the top of the pass)
          if constexpr (ring) {
#pragma unroll
            for (int d = 1; d < ND; d++) load_raw(rq[d], begin + (int64_t)d * RS);
            // round r0 + d RS sits in rq[d]; once widened, rq[d] takes the round ND rounds later (the ring's slot is
            // fixed by the unrolled d, so no register moves wait on a load)
            for (int64_t r0 = begin; r0 < end && !res; r0 += ND * RS) {
#pragma unroll
              for (int d = 0; d < ND; d++) {
                const int64_t rr = r0 + (int64_t)d * RS;
                if (rr < end && !res) {
                  i64x2 cur[RPT];
#pragma unroll
                  for (int j = 0; j < RPT; j += 2) {
                    cur[j] = narrow_to_crec(c, (uint64_t)rq[d][j / 2].x);
                    cur[j + 1] = narrow_to_crec(c, (uint64_t)rq[d][j / 2].y);
                  }
                  if (rr + ND * RS < end) load_raw(rq[d], rr + ND * RS);
                  res = add_round(cur, rr);
                }
              }
            }
          } else {
            for (int64_t r0 = begin; r0 < end; r0 += 2 * RS) {
              load(rn, r0 + RS);
              if ((res = add_round(ra, r0))) break;
              if (r0 + RS >= end) break;
              load(ra, r0 + 2 * RS);
              if ((res = add_round(rn, r0 + RS))) break;
            }
          }
          if (res == 2)  // a word equal to the EMPTY marker: the wide table takes the region
            M.widefb = 1;
          else if (res == 1)
            M.over = 1;
        } else {
          i64x2 ca[RPT], cb[RPT];
          // (narrow records: widened to their CRec on load, then read as a compact batch)
          auto ld = [&](int64_t i, i64x2& a, i64x2& b) {
            if (nar) {
              a = i < end ? narrow_to_crec(c, nrec[i]) : i64x2{0, 0};
              b = i64x2{0, 0};
            } else {
              load_prec_raw(cmp, part, i, i < end, a, b);
            }
          };
          const bool cm = cmp || nar;
#pragma unroll
          for (int j = 0; j < RPT; j++) ld(begin + (int64_t)j * FW_DT_THREADS + threadIdx.x, ca[j], cb[j]);
          for (int64_t rb = begin; rb < end; rb += RS) {
            i64x2 na[RPT], nb[RPT];
#pragma unroll
            for (int j = 0; j < RPT; j++) ld(rb + RS + (int64_t)j * FW_DT_THREADS + threadIdx.x, na[j], nb[j]);
            uint32_t dm = 0;
            int64_t kk[RPT], tt[RPT], vv[RPT];
#pragma unroll
            for (int j = 0; j < RPT; j++) {
              int64_t o;
              int nw;
              unpack_prec<false>(c, cm, p, ca[j], cb[j], kk[j], tt[j], vv[j], nw, o);
              const int64_t i = rb + (int64_t)j * FW_DT_THREADS + threadIdx.x;
              if (i >= end || (hb && dt_pass(c, kk[j], tt[j], hb) != k)) dm |= 1u << j;
            }
            if (!dt_add_batch<RPT>(U.w, M, c.vtype, kk, tt, vv, dm)) {
              M.over = 1;
              break;
            }
#pragma unroll
            for (int j = 0; j < RPT; j++) {
              ca[j] = na[j];
              cb[j] = nb[j];
            }
          }
        }
      } else {
        for (int64_t i0 = begin; i0 < end; i0 += 2 * FW_DT_THREADS) {
          if (__hip_atomic_load(&M.over, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
          PartialRec d[2];
#pragma unroll
          for (int u = 0; u < 2; u++) {
            const int64_t i = i0 + u * FW_DT_THREADS + threadIdx.x;
            if (i < end) d[u] = pin[i];
          }
          bool full = false;
#pragma unroll
          for (int u = 0; u < 2; u++) {
            const int64_t i = i0 + u * FW_DT_THREADS + threadIdx.x;
            if (full || i >= end || (hb && dt_pass(c, d[u].key, d[u].start, hb) != k)) continue;
            const int s = dt_slot(U.w, M, d[u].key, d[u].start, lds_hash(d[u].key, d[u].start));
            if (s < 0) {
              full = true;
              continue;
            }
            dt_merge(U.w, s, c.vtype, d[u].cnt, d[u].sum, d[u].mn, d[u].mx);
          }
          if (full) {
            M.over = 1;
            break;
          }
        }
      }
    }
    __syncthreads();
    const unsigned long long tc = FW_DT_TIMING ? __builtin_amdgcn_s_memtime() : 0;
    if (M.widefb) return DT_WIDE;
    if (M.over) return DT_OVER;
    // the pass's groups, densely behind the earlier passes' (a wave reserves its lanes' positions at once)
    const long long ob = M.out;
    long long nt = LMAX;
    for (int h0 = 0; h0 < NS; h0 += FW_DT_THREADS) {
      const int h = h0 + (int)threadIdx.x;
      bool g;
      if constexpr (KW)
        g = h < NS && U.k.kw[h] != DK_EMPTY;
      else
        g = h < NS && U.w.tag[h] >= 2;
      const uint64_t m = __ballot(g);
      int wb = 0;
      if (lane == 0 && m) wb = atomicAdd(&M.nout, __popcll(m));
      wb = __shfl(wb, 0, 64);
      if (g) {
        const int64_t pos = ob + wb + __popcll(m & lanemask_lt());
        Entry e;
        if constexpr (KW) {
          compact_decode(c, p, (int64_t)U.k.kw[h], &e.key, &e.start);
          e.cnt = (int64_t)U.k.cnt[h];
          e.sum = U.k.sum[h];
          const i64x2 m = U.k.mm[h];
          e.mn = m.x;
          e.mx = m.y;
        } else {
          const i64x2 kv = U.w.kv[h];
          e.key = kv.x;
          e.start = kv.y;
          e.cnt = (int64_t)U.w.cnt[h];
          e.sum = U.w.sum[h];
          e.mn = U.w.mn[h];
          e.mx = U.w.mx[h];
        }
        e.end = jadd(e.start, c.size);
        e.meta = FW_TIMER;  // EventTimeTrigger's timer at maxTimestamp (= the GC timer with lateness 0)
        if (pos < R)
          dst[pos] = e;
        else
          M.capover = 1;
        nt = min(nt, (long long)jsub(e.end, 1));
      }
    }
    if (nt != LMAX) atomicMin(&M.ntmin, nt);
    __syncthreads();
    if (threadIdx.x == 0) M.out += M.nout;
    if (FW_DT_TIMING && KW && threadIdx.x == 0) {
      atomicAdd(&g_dtt[1], tb1 - ta);
      atomicAdd(&g_dtt[2], tc - tb1);
      atomicAdd(&g_dtt[3], __builtin_amdgcn_s_memtime() - tc);
    }
    __syncthreads();
  }
  return DT_OK;
}

// One workgroup per region.  SRC = DT_RECS: the batch's records (CRec / PRec runs of k_scatter); DT_PARTS: partial
// accumulators (PartialRec runs of k_pscatter or of a restore).  KW: the compact table, for the regions of a compact
// batch; a region it cannot take (an entry without a compact word) is left for the wide launch that follows it
// (two kernels, so each keeps its own registers).  A region is committed (its buffer flipped) only when every group
// was written.  NAR: a single-pass batch of narrow records (launch_aggregate's first launch of one); a batch the single
// pass could not take (rsv[P + RSV_OVER]) suspends it, and the resumed launch (NAR false) reads the offset form.
template <int SRC, bool KW, bool NAR = false>
__global__ __launch_bounds__(FW_DT_THREADS) void k_dt_aggregate(DevCfg c, const void* __restrict__ in,
                                                                const uint32_t* __restrict__ offs, int32_t T, DevTable tb,
                                                                AggProg prog, int resume, Status* st,
                                                                const uint32_t* __restrict__ rsv, int64_t rcap) {
  __shared__ DtTab U;
  __shared__ DtMisc M;
  const int32_t p = blockIdx.x;
  if (p >= c.P || (resume && prog.done[p])) return;
  // the partition's run: at the scan offsets, or where the single-pass scatter reserved it (launch_scatter_rsv)
  const bool single = rsv && !rsv[c.P + RSV_OVER];
  if (NAR && !single) {
    if (threadIdx.x == 0) {
      prog.done[p] = 0;
      atomicOr(&st->suspended, (int)FW_SUSP_AGG);
    }
    return;
  }
  const bool nar = NAR || (single && c.narrow);  // (narrow: runs of 8-byte records, twice rcap of them per partition)
  const int64_t begin = single ? (int64_t)p * (nar ? 2 * rcap : rcap) : (int64_t)offs[(int64_t)p * T];
  const int64_t end = single ? begin + rsv[p] : (int64_t)offs[(int64_t)(p + 1) * T];
  if (begin == end) {  // nothing for this region: it stays as it is
    if (threadIdx.x == 0) prog.done[p] = 1;
    return;
  }
  const bool cmp = SRC == DT_RECS && c.compact && !*c.wide;
  // a batch without compact words: the wide launch takes it.  That launch runs only in a resumed sequence (a
  // region the compact table cannot take is rare: a record far from the watermark), so the first launch suspends
  // the push and the host resumes it with both launches
  if (KW && (!cmp || (c.diag & DIAG_DT_WIDE))) {
    if (threadIdx.x == 0) {
      prog.done[p] = 0;
      if (!resume) atomicOr(&st->suspended, (int)FW_SUSP_AGG);
    }
    return;
  }
  const unsigned long long t0 = FW_DT_TIMING ? __builtin_amdgcn_s_memtime() : 0;
  const int X = tb.cur[p], Y = X ^ 1;
  const int64_t base = (int64_t)p << c.log_r, R = (int64_t)1 << c.log_r;
  const Entry* __restrict__ src = tb.ent[X] + base;
  Entry* __restrict__ dst = tb.ent[Y] + base;
  const int32_t live = tb.live[p];
  int hb = tb.passes[p];
  bool lost = false, wide = false;
  for (;;) {
    const int r = dt_attempt<SRC, KW, NAR>(c, U, M, p, src, live, dst, R, in, begin, end, cmp, hb, nar);
    __syncthreads();
    if (r == DT_OK) break;
    if (r == DT_WIDE) {  // (KW only)
      wide = true;
      break;
    }
    if (++hb > 24) {  // more groups with one hash prefix than 2^24 passes can split: cannot happen
      lost = true;
      break;
    }
  }
  if (threadIdx.x == 0) {
    // the passes a region needs follow its groups down again: a batch that straddles a window end doubles them until
    // the old window fires, and a region kept at 2^b passes would read its records 2^b times for every later batch
    int keep = min(hb, 24);
#ifndef FW_DT_NO_DECAY
    if (!wide && !lost && !M.capover && keep > 0 &&
        M.out < ((long long)(KW ? DK_LIMIT : DT_LIMIT) * 3 / 4 << (keep - 1)))
      keep--;
#endif
    tb.passes[p] = (uint8_t)keep;
    if (wide) {
      prog.done[p] = 0;
      if (!resume) atomicOr(&st->suspended, (int)FW_SUSP_AGG);
    } else if (lost) {
      atomicOr(&st->flags, FW_STATUS_STATE_LOST);
      prog.done[p] = 1;
    } else if (M.capover) {  // the region's buffers are too small: nothing committed, the host grows them and resumes
      atomicMax(&st->need_live, (int)min(M.out, (long long)INT32_MAX));
      prog.done[p] = 0;
      atomicOr(&st->suspended, (int)FW_SUSP_AGG);
    } else {
      tb.cur[p] = (uint8_t)Y;
      tb.live[p] = (int32_t)M.out;
      tb.next_timer[p] = M.ntmin;
      prog.done[p] = 1;
      atomicAdd(&st->merged, (unsigned long long)M.out);
      if (M.out > (3 * R) / 4) st->need_grow = 1;
    }
    if (FW_DT_TIMING && KW) {
      atomicAdd(&g_dtt[0], __builtin_amdgcn_s_memtime() - t0);
      if (atomicAdd(&g_dtt[5], 1ull) == (unsigned long long)gridDim.x - 1) {
        const double nb = (double)gridDim.x;
        printf("dt timing per WG: total %.0f clear+load %.0f records %.0f writeback %.0f clocks\n", g_dtt[0] / nb,
               g_dtt[1] / nb, g_dtt[2] / nb, g_dtt[3] / nb);
        for (int i = 0; i < 6; i++) g_dtt[i] = 0;
      }
    }
  }
}

// per watermark: the due regions' windows with maxTimestamp <= wm fire (FIRE / FIRE_AND_PURGE and the GC timer
// coincide with lateness 0); the other entries are copied densely into the region's other buffer.  A workgroup
// first counts its region's rows (the entries' end / count sector only), reserves them with one atomic on the
// fired-row counter (per-wave reservations on that one address serialised the whole grid), then writes rows and
// survivors.
constexpr int DT_FIRE_U = 4;
__global__ __launch_bounds__(FW_FIRE_THREADS) void k_dt_fire(DevCfg c, int64_t wm, DevTable tb, DevRows out, Status* st) {
  const int32_t p = blockIdx.x;
  // a suspended push has not finished updating the state: the host resumes it and fires again
  if (tb.next_timer[p] > wm || __hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  __shared__ int surv_s, rows_s;
  __shared__ long long nt_s;
  __shared__ unsigned long long base_s;
  if (threadIdx.x == 0) {
    surv_s = 0;
    rows_s = 0;
    nt_s = LMAX;
  }
  __syncthreads();
  const int X = tb.cur[p], Y = X ^ 1;
  const int64_t base = (int64_t)p << c.log_r;
  const Entry* __restrict__ src = tb.ent[X] + base;
  Entry* __restrict__ dst = tb.ent[Y] + base;
  const int32_t live = tb.live[p];
  const int lane = __lane_id();
  // 1. the region's rows: windows with maxTimestamp <= wm and contents (WindowOperator.java:452-459)
  int mine = 0;
  for (int32_t i0 = 0; i0 < live; i0 += FW_FIRE_THREADS * DT_FIRE_U) {
    i64x2 ec[DT_FIRE_U];  // {end, cnt}
#pragma unroll
    for (int u = 0; u < DT_FIRE_U; u++) {
      const int32_t i = i0 + u * FW_FIRE_THREADS + (int32_t)threadIdx.x;
      ec[u] = reinterpret_cast<const i64x2*>(src + (i < live ? i : live - 1))[1];
    }
#pragma unroll
    for (int u = 0; u < DT_FIRE_U; u++) {
      const int32_t i = i0 + u * FW_FIRE_THREADS + (int32_t)threadIdx.x;
      mine += i < live && jsub(ec[u].x, 1) <= wm && ec[u].y > 0;
    }
  }
  mine += __shfl_xor(mine, 1, 64);
  mine += __shfl_xor(mine, 2, 64);
  mine += __shfl_xor(mine, 4, 64);
  mine += __shfl_xor(mine, 8, 64);
  mine += __shfl_xor(mine, 16, 64);
  mine += __shfl_xor(mine, 32, 64);
  if (lane == 0 && mine) atomicAdd(&rows_s, mine);
  __syncthreads();
  if (threadIdx.x == 0) {
    base_s = rows_s ? atomicAdd(&st->out_rows, (unsigned long long)rows_s) : 0ull;
    if (rows_s) atomicAdd(&st->fired_total, (unsigned long long)rows_s);
    rows_s = 0;
  }
  __syncthreads();
  const unsigned long long rbase = base_s;
  // 2. rows at the reserved range, survivors densely into the other buffer
  long long nt = LMAX;
  for (int32_t i0 = 0; i0 < live; i0 += FW_FIRE_THREADS * DT_FIRE_U) {
    Entry e[DT_FIRE_U];
#pragma unroll
    for (int u = 0; u < DT_FIRE_U; u++) {
      const int32_t i = i0 + u * FW_FIRE_THREADS + (int32_t)threadIdx.x;
      e[u] = src[i < live ? i : live - 1];
    }
#pragma unroll
    for (int u = 0; u < DT_FIRE_U; u++) {
      const int32_t i = i0 + u * FW_FIRE_THREADS + (int32_t)threadIdx.x;
      const bool valid = i < live;
      const bool due = valid && jsub(e[u].end, 1) <= wm;
      const bool row = due && e[u].cnt > 0;
      const bool keep = valid && !due;
      const uint64_t rm = __ballot(row), km = __ballot(keep);
      int rb = 0, sb = 0;
      if (lane == 0) {
        if (rm) rb = atomicAdd(&rows_s, __popcll(rm));
        if (km) sb = atomicAdd(&surv_s, __popcll(km));
      }
      rb = __shfl(rb, 0, 64);
      sb = __shfl(sb, 0, 64);
      if (row) {
        const unsigned long long pos = rbase + (unsigned long long)(rb + __popcll(rm & lanemask_lt()));
        if ((int64_t)pos < out.cap)
          write_row(c, out, pos, e[u]);
        else
          atomicOr(&st->flags, FW_STATUS_OUT_FULL);
      }
      if (keep) {
        dst[sb + __popcll(km & lanemask_lt())] = e[u];
        nt = min(nt, (long long)jsub(e[u].end, 1));
      }
    }
  }
  if (nt != LMAX) atomicMin(&nt_s, nt);
  __syncthreads();
  if (threadIdx.x == 0) {
    tb.cur[p] = (uint8_t)Y;
    tb.live[p] = surv_s;
    tb.next_timer[p] = nt_s;
  }
}

// table growth of dense regions: the live prefix of each region into buffer 0 of the larger table
__global__ __launch_bounds__(FW_FIRE_THREADS) void k_dt_rehash(DevCfg oc, DevTable ot, DevCfg nc, DevTable nt) {
  const int32_t p = blockIdx.x;
  const Entry* src = ot.ent[ot.cur[p]] + ((int64_t)p << oc.log_r);
  Entry* dst = nt.ent[0] + ((int64_t)p << nc.log_r);
  const int32_t live = ot.live[p];
  for (int32_t i = threadIdx.x; i < live; i += blockDim.x) dst[i] = src[i];
  if (threadIdx.x == 0) {
    nt.cur[p] = 0;
    nt.live[p] = live;
    nt.next_timer[p] = ot.next_timer[p];
  }
}

// restore into dense regions: every row of key group kg as a partial accumulator in the table's representation
// (k_restore's conversion), its partition in rp (-1 and a key-group error when a Long / Integer key is not in kg)
__global__ void k_dt_rows_prep(DevCfg c, int32_t kg, StateCols in, int64_t n, int32_t* rp, PartialRec* tmp, Status* st) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t p = restore_partition(c, kg, in.key[i]);
  rp[i] = p;
  if (p < 0) {
    atomicAdd(&st->kg_errors, 1);
    return;
  }
  PartialRec d;
  d.key = in.key[i];
  d.start = in.start[i];
  d.cnt = in.cnt[i];
  d.sum = in.sum[i];
  d.mn = c.vtype == FW_VAL_F64 ? f64_sortable(in.mn[i]) : in.mn[i];
  d.mx = c.vtype == FW_VAL_F64 ? f64_sortable(in.mx[i]) : in.mx[i];
  tmp[i] = d;
}
__global__ __launch_bounds__(FW_TILE_THREADS) void k_dt_rows_hist(int32_t P, const int32_t* __restrict__ rp, int64_t n,
                                                                  int32_t T, uint32_t* __restrict__ hist) {
  extern __shared__ uint32_t lh[];
  for (int i = threadIdx.x; i <= P; i += blockDim.x) lh[i] = 0;
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * FW_TILE, e = min(n, b + (int64_t)FW_TILE);
  for (int64_t i = b + threadIdx.x; i < e; i += blockDim.x)
    if (rp[i] >= 0) atomicAdd(&lh[rp[i]], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i <= P; i += blockDim.x) hist[(int64_t)i * T + blockIdx.x] = i < P ? lh[i] : 0u;
}
__global__ __launch_bounds__(FW_TILE_THREADS) void k_dt_rows_scatter(int32_t P, const int32_t* __restrict__ rp,
                                                                     const PartialRec* __restrict__ tmp, int64_t n, int32_t T,
                                                                     const uint32_t* __restrict__ offs,
                                                                     PartialRec* __restrict__ part) {
  extern __shared__ uint32_t base[];
  for (int i = threadIdx.x; i < P; i += blockDim.x) base[i] = offs[(int64_t)i * T + blockIdx.x];
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * FW_TILE, e = min(n, b + (int64_t)FW_TILE);
  for (int64_t i = b + threadIdx.x; i < e; i += blockDim.x)
    if (rp[i] >= 0) part[atomicAdd(&base[rp[i]], 1u)] = tmp[i];
}

// ---- keyBy routing: key groups and stable grouping by destination operator index
__global__ void k_key_groups(const int64_t* key, const int32_t* kh, int32_t kind, int64_t n, int32_t max_par,
                             int32_t* kg) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    kg[i] = key_group(key_hash_of(kind, key[i], kh, i), max_par);
}

__device__ __forceinline__ int32_t dest_of(const int64_t* key, const int32_t* kh, int32_t kind, int64_t i,
                                           int32_t max_par, int32_t par) {
  // KeyGroupRangeAssignment.computeOperatorIndexForKeyGroup (KeyGroupRangeAssignment.java:115-117)
  return key_group(key_hash_of(kind, key[i], kh, i), max_par) * par / max_par;
}

__global__ __launch_bounds__(FW_TILE_THREADS) void k_route_hist(const int64_t* key, const int32_t* kh, int32_t kind,
                                                                int64_t n, int32_t max_par, int32_t par, int32_t T,
                                                                uint32_t* hist) {
  extern __shared__ uint32_t lh[];
  for (int i = threadIdx.x; i < par; i += blockDim.x) lh[i] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * FW_TILE, end = min(n, base + (int64_t)FW_TILE);
  for (int64_t i = base + threadIdx.x; i < end; i += blockDim.x) atomicAdd(&lh[dest_of(key, kh, kind, i, max_par, par)], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < par; i += blockDim.x) hist[(int64_t)i * T + blockIdx.x] = lh[i];
}

__global__ __launch_bounds__(FW_TILE_THREADS) void k_route_scatter(const int64_t* key, const int64_t* ts,
                                                                   const int64_t* val, const int32_t* kh, int32_t kind,
                                                                   int64_t n, int32_t max_par, int32_t par, int32_t T,
                                                                   const uint32_t* offs, int64_t* ko, int64_t* to,
                                                                   int64_t* vo, int32_t* ho) {
  extern __shared__ uint32_t sm[];
  const int nw = blockDim.x >> 6;
  uint32_t* run = sm;            // par
  uint32_t* wc = sm + par;       // nw * par
  for (int d = threadIdx.x; d < par; d += blockDim.x) run[d] = offs[(int64_t)d * T + blockIdx.x];
  __syncthreads();
  const int lane = __lane_id(), wid = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * FW_TILE, end = min(n, base + (int64_t)FW_TILE);
  for (int64_t j = base; j < end; j += blockDim.x) {
    const int64_t i = j + threadIdx.x;
    const int32_t d = i < end ? dest_of(key, kh, kind, i, max_par, par) : -1;
    uint32_t rank = 0;
    for (int q = 0; q < par; q++) {
      const uint64_t b = __ballot(d == q);
      if (d == q) rank = (uint32_t)__popcll(b & lanemask_lt());
      if (lane == 0) wc[wid * par + q] = (uint32_t)__popcll(b);
    }
    __syncthreads();
    if (d >= 0) {
      uint32_t pos = run[d] + rank;
      for (int w = 0; w < wid; w++) pos += wc[w * par + d];
      ko[pos] = key[i];
      to[pos] = ts[i];
      vo[pos] = val[i];
      ho[pos] = key_hash_of(kind, key[i], kh, i);
    }
    __syncthreads();
    for (int q = threadIdx.x; q < par; q += blockDim.x) {
      uint32_t t = 0;
      for (int w = 0; w < nw; w++) t += wc[w * par + q];
      run[q] += t;
    }
    __syncthreads();
  }
}
__global__ void k_route_counts(const uint32_t* offs, int32_t par, int32_t T, int64_t n, int64_t* counts) {
  const int d = threadIdx.x;
  if (d >= par) return;
  const int64_t b = offs[(int64_t)d * T];
  const int64_t e = d + 1 < par ? (int64_t)offs[(int64_t)(d + 1) * T] : n;
  counts[d] = e - b;
}

// ---- synthetic source (splitmix64 counter-based; see fw_generate_device)
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ __launch_bounds__(256) void k_generate(uint64_t seed, int64_t first, int64_t n, int64_t num_keys,
                                                  const double* cdf, int64_t ts_base, int64_t rate, int64_t jitter,
                                                  int64_t* key, int64_t* ts, int64_t* val, int64_t* max_ts) {
  int64_t mx = LMIN;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t i = (uint64_t)(first + j);
    const uint64_t r0 = splitmix64(seed ^ (4 * i)), r1 = splitmix64(seed ^ (4 * i + 1)),
                   r2 = splitmix64(seed ^ (4 * i + 2));
    int64_t k;
    if (cdf) {
      const double u = (double)(r0 >> 11) * (1.0 / 9007199254740992.0);
      int64_t lo = 0, hi = num_keys;  // first index with cdf[idx] > u
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (cdf[mid] > u)
          hi = mid;
        else
          lo = mid + 1;
      }
      k = lo < num_keys ? lo : num_keys - 1;
    } else {
      k = (int64_t)(r0 % (uint64_t)num_keys);
    }
    const int64_t t = ts_base + (int64_t)((i * 1000ull) / (uint64_t)rate) - (jitter > 0 ? (int64_t)(r2 % (uint64_t)jitter) : 0);
    key[j] = k;
    ts[j] = t;
    val[j] = (int64_t)(int32_t)(uint32_t)r1;
    mx = t > mx ? t : mx;
  }
  if (max_ts) {
    for (int o = 32; o > 0; o >>= 1) {
      const int64_t y = __shfl_xor(mx, o, 64);
      mx = y > mx ? y : mx;
    }
    if (__lane_id() == 0 && mx != LMIN) atomicMax((long long*)max_ts, (long long)mx);
  }
}

}  // namespace

// ============================================================================== launchers
namespace fwdev {

thread_local ExtTiming g_ext{};  // per host thread: operators timed from different threads do not share it
// a kind's main kernel: with the dispatch's own start / stop events when fw_profile asked for them (g_ext)
#define FW_LAUNCH_MAIN(kern, grid, block, lds, s, ...)                                                        \
  do {                                                                                                     \
    if (g_ext.a && !g_ext.used) {                                                                          \
      hipExtLaunchKernelGGL(kern, grid, block, lds, s, g_ext.a, g_ext.b, 0, __VA_ARGS__);                  \
      g_ext.used = true;                                                                                   \
    } else {                                                                                               \
      hipLaunchKernelGGL(kern, grid, block, lds, s, __VA_ARGS__);                                          \
    }                                                                                                      \
  } while (0)

static inline int32_t ntiles(int64_t n) { return (int32_t)((n + FW_TILE - 1) / FW_TILE); }

void launch_classify_hist(const DevCfg& c, int64_t wm, const int64_t* key, const int64_t* ts, const int32_t* kh,
                          int64_t n, int32_t T, uint32_t* hist, Status* st, hipStream_t s, const uint32_t* rsv) {
  const size_t lds = (c.P + 1) * sizeof(uint32_t);
  switch (stream_mode(c)) {
    case M_TUMB:
      hipLaunchKernelGGL(k_classify_hist<M_TUMB>, dim3(T), dim3(FW_TILE_THREADS), lds, s, c, wm, key, ts, kh, n, T, hist, st, rsv);
      break;
    case M_PANE:
      hipLaunchKernelGGL(k_classify_hist<M_PANE>, dim3(T), dim3(FW_TILE_THREADS), lds, s, c, wm, key, ts, kh, n, T, hist, st, rsv);
      break;
    default:
      hipLaunchKernelGGL(k_classify_hist<M_GEN>, dim3(T), dim3(FW_TILE_THREADS), lds, s, c, wm, key, ts, kh, n, T, hist, st, rsv);
  }
}

// a scratch set's single-pass words back to zero once its aggregate has read them (unless the push suspended: its
// resumption reads them again, and the host zeroes them after it settles)
__global__ void k_rsv_reset(uint32_t* rsv, int32_t words, const Status* st) {
  if (__hip_atomic_load(&st->suspended, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < words; i += gridDim.x * blockDim.x) rsv[i] = 0u;
}
void launch_rsv_reset(uint32_t* rsv, int32_t words, const Status* st, hipStream_t s) {
  hipLaunchKernelGGL(k_rsv_reset, dim3((unsigned)std::min(64, (words + 255) / 256)), dim3(256), 0, s, rsv, words, st);
}
void launch_scan(uint32_t* data, int64_t m, uint32_t* scratch, hipStream_t s, const uint32_t* gate) {
  if (gate) {
    hipLaunchKernelGGL(k_scan_gated, dim3(1), dim3(SCAN_T), 0, s, data, m, gate);
    return;
  }
  const int64_t nb = (m + SCAN_B - 1) / SCAN_B;
  hipLaunchKernelGGL(k_scan_blocks, dim3((unsigned)nb), dim3(SCAN_T), 0, s, data, m, scratch, gate);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_T), 0, s, scratch, nb, gate);
  hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nb), dim3(SCAN_T), 0, s, data, m, (const uint32_t*)scratch, gate);
}

void launch_taint(const DevCfg& c, int64_t wm, const int64_t* key, const int64_t* ts, int64_t n, Status* st,
                  hipStream_t s) {
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 2048);
  if (blocks > 0) hipLaunchKernelGGL(k_taint, dim3((unsigned)blocks), dim3(256), 0, s, c, wm, key, ts, n, st);
}

void launch_scatter(const DevCfg& c, int64_t wm, const int64_t* key, const int64_t* ts, const int64_t* val,
                    const int32_t* kh, int64_t n, int32_t T, uint32_t* offs, PRec* part, int64_t* sk, int64_t* stt,
                    int64_t* sv, int32_t* skh, DevSide side, Status* st, hipStream_t s, const uint32_t* gate) {
  const size_t lds = (size_t)c.P * sizeof(uint32_t);
  const uint32_t* o = offs;
  static const bool no_staged = getenv("FW_NO_STAGED") && atoi(getenv("FW_NO_STAGED"));
  if (c.compact && c.P <= (gate ? FW_GMAX_P : FW_STAGED_MAX_P) && stream_mode(c) != M_GEN && (!no_staged || gate)) {
    // staged: rounds of 8192 records up to 1024 partitions, 4096 up to 4096 (the LDS); C3's 4096 partitions: the
    // step 1.567 -> 1.531 ms against the plain offset scatter
    const bool big = c.P <= 1024;
    const int rr = big ? 8192 : 4096;
    const size_t sl = (size_t)rr * (sizeof(i64x2) + sizeof(uint16_t)) + (2 * (size_t)c.P + 1) * sizeof(uint32_t) +
                      (FW_TILE_THREADS / 64 + 1) * sizeof(uint32_t);
    static bool attr = false;
    if (!attr) {  // LDS beyond 64 KB
      (void)hipFuncSetAttribute((const void*)k_scatter_staged<M_TUMB, 8192>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)k_scatter_staged<M_TUMB, 4096>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)k_scatter_staged<M_PANE, 8192>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)k_scatter_staged<M_PANE, 4096>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    const bool tumb = stream_mode(c) == M_TUMB;
    if (tumb && big)
      hipLaunchKernelGGL((k_scatter_staged<M_TUMB, 8192>), dim3(T), dim3(FW_TILE_THREADS), sl, s, c, wm, key, ts, val, kh, n,
                         T, o, part, side, st, gate);
    else if (tumb)
      hipLaunchKernelGGL((k_scatter_staged<M_TUMB, 4096>), dim3(T), dim3(FW_TILE_THREADS), sl, s, c, wm, key, ts, val, kh, n,
                         T, o, part, side, st, gate);
    else if (big)
      hipLaunchKernelGGL((k_scatter_staged<M_PANE, 8192>), dim3(T), dim3(FW_TILE_THREADS), sl, s, c, wm, key, ts, val, kh, n,
                         T, o, part, side, st, gate);
    else
      hipLaunchKernelGGL((k_scatter_staged<M_PANE, 4096>), dim3(T), dim3(FW_TILE_THREADS), sl, s, c, wm, key, ts, val, kh, n,
                         T, o, part, side, st, gate);
  } else
  switch (stream_mode(c)) {
    case M_TUMB:
      hipLaunchKernelGGL(k_scatter<M_TUMB>, dim3(T), dim3(FW_TILE_THREADS), lds, s, c, wm, key, ts, val, kh, n, T, o, part,
                         side, st);
      break;
    case M_PANE:
      hipLaunchKernelGGL(k_scatter<M_PANE>, dim3(T), dim3(FW_TILE_THREADS), lds, s, c, wm, key, ts, val, kh, n, T, o, part,
                         side, st);
      break;
    default:
      hipLaunchKernelGGL(k_scatter<M_GEN>, dim3(T), dim3(FW_TILE_THREADS), lds, s, c, wm, key, ts, val, kh, n, T, o, part,
                         side, st);
  }
  if (!c.dense)  // (dense configurations never have a record that needs arrival order)
    hipLaunchKernelGGL(k_scatter_ordered<false>, dim3(T), dim3(FW_TILE_THREADS), 0, s, c, wm, key, ts, val, kh, n, T,
                       (const uint32_t*)(offs + (int64_t)c.P * T), sk, stt, sv, skh, (const Status*)st);
}

bool rsv_eligible(const DevCfg& c) {
  static const bool off = getenv("FW_NO_RSV") && atoi(getenv("FW_NO_RSV"));
  return !off && c.dense && c.compact && !c.side_output && c.P <= FW_GMAX_P && stream_mode(c) == M_TUMB;
}
void launch_scatter_rsv(const DevCfg& c, int64_t wm, const int64_t* key, const int64_t* ts, const int64_t* val,
                        const int32_t* kh, int64_t n, int32_t T, PRec* part, uint32_t* rsv, int64_t rcap, hipStream_t s) {
  const bool big = c.P <= 1024;
  const int rr = big ? 8192 : 4096;
  const size_t sl = (size_t)rr * ((c.narrow ? 8 : sizeof(i64x2)) + sizeof(uint16_t)) +
                    (2 * (size_t)c.P + 1) * sizeof(uint32_t) + (FW_TILE_THREADS / 64 + 1) * sizeof(uint32_t);
  static bool attr = false;
  if (!attr) {  // LDS beyond 64 KB
    for (const void* f : {(const void*)k_scatter_rsv<8192, false>, (const void*)k_scatter_rsv<4096, false>,
                          (const void*)k_scatter_rsv<8192, true>, (const void*)k_scatter_rsv<4096, true>})
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  // (narrow: a partition's run holds twice as many 8-byte records in the same bytes)
  if (c.narrow && big)
    FW_LAUNCH_MAIN((k_scatter_rsv<8192, true>), dim3(T), dim3(FW_TILE_THREADS), sl, s, c, wm, key, ts, val, kh, n, T,
                   part, rsv, 2 * rcap);
  else if (c.narrow)
    FW_LAUNCH_MAIN((k_scatter_rsv<4096, true>), dim3(T), dim3(FW_TILE_THREADS), sl, s, c, wm, key, ts, val, kh, n, T,
                   part, rsv, 2 * rcap);
  else if (big)
    FW_LAUNCH_MAIN((k_scatter_rsv<8192, false>), dim3(T), dim3(FW_TILE_THREADS), sl, s, c, wm, key, ts, val, kh, n, T,
                   part, rsv, rcap);
  else
    FW_LAUNCH_MAIN((k_scatter_rsv<4096, false>), dim3(T), dim3(FW_TILE_THREADS), sl, s, c, wm, key, ts, val, kh, n, T,
                   part, rsv, rcap);
}

// panes: maxTimestamp of the earliest window ending after wm (windows [s, s + size), s = offset mod slide)
int64_t pane_nt_floor(const DevCfg& c, int64_t wm) {
  if (!c.panes) return 0;
  const __int128 x = (__int128)wm - c.size + 2;  // first start s with s + size - 1 > wm
  __int128 r = ((__int128)c.offset - x) % c.slide;
  if (r < 0) r += c.slide;
  const __int128 e = x + r + c.size - 1;
  return e > (__int128)LMAX ? LMAX : e < (__int128)LMIN ? LMIN : (int64_t)e;
}

void launch_aggregate(const DevCfg& c0, int64_t wm, const PRec* part, const uint32_t* offs, int32_t T, DevTable tb,
                      AggProg prog, int resume, const AggHot* hot, int64_t n, Status* st, hipStream_t s,
                      const uint32_t* rt_t, int32_t t8, const uint32_t* rsv, int64_t rcap) {
  DevCfg c = c0;
  c.nt_floor = pane_nt_floor(c, wm);
  AggHot h{};
  unsigned grid = (unsigned)c.P;
  if (hot) {  // at most n / agg_chunk chunks beyond one per partition
    h = *hot;
    grid += (unsigned)((n + c.agg_chunk - 1) / c.agg_chunk);
    if (!resume) {
      hipLaunchKernelGGL(k_chunk_plan, dim3((c.P + 1 + 255) / 256), dim3(256), 0, s, c, offs, T, h);
      launch_scan(h.chunk_base, (int64_t)c.P + 1, h.scan_tmp, s);
    }
  }
  if (c.dense) {  // the compact table; in a resumed sequence the wide launch takes the regions it left
    if (!resume && rsv && c.narrow && FW_DT_NDEPTH > 0)  // (its own kernel: the ring's registers)
      FW_LAUNCH_MAIN((k_dt_aggregate<DT_RECS, true, true>), dim3(c.P), dim3(FW_DT_THREADS), 0, s, c, (const void*)part, offs,
                     T, tb, prog, resume, st, rsv, rcap);
    else
      FW_LAUNCH_MAIN((k_dt_aggregate<DT_RECS, true>), dim3(c.P), dim3(FW_DT_THREADS), 0, s, c, (const void*)part, offs, T,
                     tb, prog, resume, st, rsv, rcap);
    if (resume)
      hipLaunchKernelGGL((k_dt_aggregate<DT_RECS, false>), dim3(c.P), dim3(FW_DT_THREADS), 0, s, c, (const void*)part,
                         offs, T, tb, prog, 1, st, rsv, rcap);
    return;
  }
  const dim3 b(FW_AGG_THREADS);
  if (rt_t) {  // gathered: count/sum/min/max of compact records (gather_mode)
    grid = (grid + 7) & ~7u;  // whole groups of 8 for the XCD mapping (the extra workgroups return)
    hipLaunchKernelGGL((k_aggregate<FW_AGG_RPT, false, false, false, true>), dim3(grid), b, 0, s, c, wm, part, offs, T,
                       tb, prog, resume, st, h, rt_t, t8);
    return;
  }
  const uint32_t* nr = nullptr;
  const bool first = agg_ordinal(c), pool = c.pool_bytes != 0;
  if (c.assigner == FW_SESSION && first)
    hipLaunchKernelGGL((k_aggregate<FW_AGG_RPT, true, true, false>), dim3(grid), b, 0, s, c, wm, part, offs, T, tb, prog,
                       resume, st, h, nr, 0);
  else if (c.assigner == FW_SESSION && pool)
    hipLaunchKernelGGL((k_aggregate<FW_SESS_RPT, true, false, true>), dim3(grid), b, 0, s, c, wm, part, offs, T, tb, prog,
                       resume, st, h, nr, 0);
  else if (c.assigner == FW_SESSION)
    hipLaunchKernelGGL((k_aggregate<FW_SESS_RPT, true, false, false>), dim3(grid), b, 0, s, c, wm, part, offs, T, tb,
                       prog, resume, st, h, nr, 0);
  else if (first)
    hipLaunchKernelGGL((k_aggregate<FW_AGG_RPT, false, true, false>), dim3(grid), b, 0, s, c, wm, part, offs, T, tb,
                       prog, resume, st, h, nr, 0);
  else if (pool)
    hipLaunchKernelGGL((k_aggregate<FW_POOL_RPT, false, false, true>), dim3(grid), b, 0, s, c, wm, part, offs, T, tb,
                       prog, resume, st, h, nr, 0);
  else
    hipLaunchKernelGGL((k_aggregate<FW_PLAIN_RPT, false, false, false>), dim3(grid), b, 0, s, c, wm, part, offs, T, tb,
                       prog, resume, st, h, nr, 0);
}

int gather_mode(const DevCfg& c, int64_t n) {
  // opt-in (FW_GATHER=1): at C2 it measured even with the partition-major scatter (0.90 vs 0.895 ms per step;
  // k_stage 185 us + regroup ~150 us against classify + scan + scatter 0.41 ms), see DESIGN.md
  static const bool on = getenv("FW_GATHER") && atoi(getenv("FW_GATHER"));
  return on && c.compact && c.agg != FW_AGG_ROW && c.assigner != FW_SESSION && (c.assigner == FW_TUMBLING || c.panes) &&
         c.P <= FW_GMAX_P && n <= (int64_t)FW_GMAX_T * FW_GTILE;
}

void launch_stage(const DevCfg& c, int64_t wm, const int64_t* key, const int64_t* ts, const int64_t* val,
                  const int32_t* kh, int64_t n, PRec* part, int64_t mb, uint32_t* rt, uint32_t* rt_t, uint32_t* voffs,
                  uint32_t* srow, uint32_t* scan_tmp, int64_t* sk, int64_t* stt, int64_t* sv, int32_t* skh, DevSide side,
                  Status* st, hipStream_t s) {
  const int32_t t8 = (int32_t)((n + FW_GTILE - 1) / FW_GTILE);
  const size_t lds = (size_t)FW_GTILE * sizeof(i64x2) + (size_t)c.P * sizeof(uint32_t);
  static bool attr = false;
  if (!attr) {  // LDS beyond 64 KB
    (void)hipFuncSetAttribute((const void*)k_stage<M_TUMB>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)k_stage<M_PANE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)k_stage<M_GEN>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  // the tiles go to the second half of the record buffer (PRec-sized: 2 CRecs per record), the regrouped
  // partition runs to the first
  i64x2* out = reinterpret_cast<i64x2*>(part) + mb;
  switch (stream_mode(c)) {
    case M_TUMB:
      hipLaunchKernelGGL(k_stage<M_TUMB>, dim3(t8), dim3(FW_TILE_THREADS), lds, s, c, wm, key, ts, val, kh, n, t8, out, rt,
                         srow, side, st);
      break;
    case M_PANE:
      hipLaunchKernelGGL(k_stage<M_PANE>, dim3(t8), dim3(FW_TILE_THREADS), lds, s, c, wm, key, ts, val, kh, n, t8, out, rt,
                         srow, side, st);
      break;
    default:
      hipLaunchKernelGGL(k_stage<M_GEN>, dim3(t8), dim3(FW_TILE_THREADS), lds, s, c, wm, key, ts, val, kh, n, t8, out, rt,
                         srow, side, st);
  }
  // voffs: the partitions' counts (k_rt_transpose), then their virtual offsets and the regroup's chunks (k_gplan);
  // the regroup's chunk bases go to cbase (P + 1)
  uint32_t* cbase = scan_tmp;
  (void)hipMemsetAsync(voffs, 0, ((size_t)c.P + 1) * sizeof(uint32_t), s);
  hipLaunchKernelGGL(k_rt_transpose, dim3((t8 + 63) / 64, (c.P + 63) / 64), dim3(1024), 0, s, rt, rt_t, t8, c.P, voffs);
  hipLaunchKernelGGL(k_gplan, dim3(1), dim3(FW_TILE_THREADS), 0, s, voffs, cbase, c.P, srow, t8);
  hipLaunchKernelGGL(k_scatter_ordered<true>, dim3(t8), dim3(FW_TILE_THREADS), 0, s, c, wm, key, ts, val, kh, n, t8,
                     (const uint32_t*)srow, sk, stt, sv, skh, (const Status*)st);
  const unsigned grid = (unsigned)((c.P + (n + FW_REGROUP_CHUNK - 1) / FW_REGROUP_CHUNK + 7) & ~7ll);
  hipLaunchKernelGGL(k_regroup, dim3(grid), dim3(FW_REGROUP_THREADS), 0, s, (const i64x2*)out,
                     reinterpret_cast<i64x2*>(part), (const uint32_t*)rt_t, t8, (const uint32_t*)voffs,
                     (const uint32_t*)cbase, c.P);
}

void launch_hll_update(const DevCfg& c, const PRec* part, const uint32_t* offs, int32_t T, int64_t n, DevTable tb,
                       Status* st, hipStream_t s) {
  if (n <= 0) return;
  const dim3 grid((unsigned)((n + FW_HLL_CHUNK - 1) / FW_HLL_CHUNK));
  if (c.assigner == FW_SESSION)
    hipLaunchKernelGGL(k_hll_update_sessions, grid, dim3(256), 0, s, c, part, offs, T, tb, st);
  else if (c.assigner == FW_SLIDING)
    hipLaunchKernelGGL(k_hll_update<true>, grid, dim3(256), 0, s, c, part, offs, T, tb, st);
  else
    hipLaunchKernelGGL(k_hll_update<false>, grid, dim3(256), 0, s, c, part, offs, T, tb, st);
}

void launch_row_update(const DevCfg& c, const PRec* part, const uint32_t* offs, int32_t T, int64_t n, DevTable tb,
                       Status* st, hipStream_t s) {
  if (n <= 0) return;
  const dim3 grid((unsigned)((n + FW_HLL_CHUNK - 1) / FW_HLL_CHUNK));
  if (c.assigner == FW_SESSION)
    hipLaunchKernelGGL(k_row_update<2>, grid, dim3(256), 0, s, c, part, offs, T, tb, st);
  else if (c.assigner == FW_SLIDING)
    hipLaunchKernelGGL(k_row_update<1>, grid, dim3(256), 0, s, c, part, offs, T, tb, st);
  else
    hipLaunchKernelGGL(k_row_update<0>, grid, dim3(256), 0, s, c, part, offs, T, tb, st);
}

void launch_slow(const DevCfg& c, int64_t wm, const uint32_t* srow, int32_t T, const int64_t* sk, const int64_t* stt,
                 const int64_t* sv, const int32_t* skh, DevTable tb, DevRows out, DevSide side, Status* st, int resume,
                 hipStream_t s) {
  hipLaunchKernelGGL(k_slow, dim3(1), dim3(FW_SLOW_THREADS), 0, s, c, wm, srow, T, sk, stt, sv, skh, tb, out, side,
                     st, resume);
}

void launch_fire(const DevCfg& c0, int64_t wm, DevTable tb, DevRows out, Status* st, hipStream_t s) {
  DevCfg c = c0;
  c.nt_floor = pane_nt_floor(c, wm);
  if (c.panes) {
    hipLaunchKernelGGL(k_fire_panes, dim3(c.P), dim3(PF_THREADS), 0, s, c, wm, tb, out, st);
    return;
  }
  if (c.dense) {
    hipLaunchKernelGGL(k_dt_fire, dim3(c.P), dim3(FW_FIRE_THREADS), 0, s, c, wm, tb, out, st);
    return;
  }
  if (c.pool_bytes && c.assigner == FW_SESSION)  // blocks freed by session merges go back first
    hipLaunchKernelGGL(k_pool_release, dim3(1), dim3(256), 0, s, c);
  if (c.pool_bytes)
    hipLaunchKernelGGL(k_fire<true>, dim3(c.P), dim3(FW_FIRE_THREADS), 0, s, c, wm, tb, out, st);
  else
    hipLaunchKernelGGL(k_fire<false>, dim3(c.P), dim3(FW_FIRE_THREADS), 0, s, c, wm, tb, out, st);
}

size_t count_sort_bytes(int64_t n) {
  size_t a = 0;
  rocprim::double_buffer<uint32_t> ks(nullptr, nullptr), vs(nullptr, nullptr);
  (void)rocprim::radix_sort_pairs(nullptr, a, ks, vs, (size_t)n, 0, 32);
  return a;
}
void launch_count(const DevCfg& c, DevCount& cw, const int64_t* key, const int64_t* val, int64_t n, DevRows out,
                  Status* st, hipStream_t s) {
  if (n <= 0) return;
  const uint32_t none = (uint32_t)cw.max_keys;
  unsigned bits = 1;
  while (((int64_t)1 << bits) <= cw.max_keys) bits++;
  const unsigned grid = (unsigned)std::min<int64_t>(8192, (n + 255) / 256);
  hipLaunchKernelGGL(k_cnt_slots, dim3(grid), dim3(256), 0, s, cw, key, n, none, st);
  rocprim::double_buffer<uint32_t> ks(cw.sk[0], cw.sk[1]), vs(cw.sv[0], cw.sv[1]);
  size_t bytes = cw.tmp_bytes;
  (void)rocprim::radix_sort_pairs(cw.tmp, bytes, ks, vs, (size_t)n, 0, bits, s);  // stable: arrival order per key
  const uint32_t* sk = ks.current();
  const uint32_t* sv = vs.current();
  hipLaunchKernelGGL(k_cnt_bounds, dim3(grid), dim3(256), 0, s, cw, sk, n, none);
  uint32_t* vlo = ks.alternate();  // (the sort's spare halves)
  uint32_t* vhi = vs.alternate();
  hipLaunchKernelGGL(k_cnt_gather, dim3(grid), dim3(256), 0, s, sk, sv, val, n, none, vlo, vhi);
  hipLaunchKernelGGL(k_cnt_fire, dim3((unsigned)std::min<int64_t>(8192, (n + CF_CHUNK - 1) / CF_CHUNK)), dim3(256), 0, s,
                     c, cw, sk, sv, key, vlo, vhi, n, none, out, st);
  hipLaunchKernelGGL(k_cnt_update, dim3(grid), dim3(256), 0, s, c, cw, sk, sv, val, n, none);
  hipLaunchKernelGGL(k_cnt_count, dim3(grid), dim3(256), 0, s, cw, sk, n, none);
}
// t-digest under allowed lateness: the push's late-firing chains rebuilt after the table grew mid-push (settle
// resumes the ordered path over moved slots).  A chain's order does not matter (td_late_row selects in value order).
__global__ void k_td_relink(DevCfg c, DevTable tb) {
  const int64_t nov = *c.td_ovctr;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nov; j += (int64_t)gridDim.x * blockDim.x) {
    const int32_t p = c.td_ovp[j];
    const Region r = region_of(c, tb, p, tb.cur[p]);
    const int64_t k = c.td_ovk[j], last = c.td_ovt[j];
    if (c.assigner == FW_SESSION) {  // (the session that holds the element now: merged sessions' values included)
      if (c.td_olink[j] == TD_DROPPED) continue;  // (purged: in no chain)
      const int32_t slot = session_containing(r, c, k, last);
      c.td_olink[j] = slot < 0 ? -1 : atomicExch(&c.td_olast[((uint32_t)p << c.log_r) | (uint32_t)slot], (int32_t)j);
      continue;
    }
    for (int wi = 0; wi < c.td_ovn[j]; wi++) {
      const int64_t s = jsub(last, (int64_t)wi * c.slide);
      const int32_t slot = region_find(r, slot_hash(c, k, s), k, s, wend(c, s));
      const int32_t l = (int32_t)j * c.wpr + wi;
      if (c.td_olink[l] == TD_DROPPED) continue;
      c.td_olink[l] = slot < 0 ? -1 : atomicExch(&c.td_olast[((uint32_t)p << c.log_r) | (uint32_t)slot], l);
    }
  }
}
// ... then each chain back in value order (an insertion sort of the list)
__global__ void k_td_resort(DevCfg c, int64_t slots) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < slots; g += (int64_t)gridDim.x * blockDim.x) {
    int32_t l = c.td_olast[g];
    if (l < 0) continue;
    int32_t sorted = -1;
    while (l >= 0) {
      const int32_t nx = c.td_olink[l];
      td_chain_insert(c, &sorted, l, c.td_ovv[l / c.wpr]);
      l = nx;
    }
    c.td_olast[g] = sorted;
  }
}
void launch_td_relink(const DevCfg& c, DevTable tb, hipStream_t s) {
  hipLaunchKernelGGL(k_td_relink, dim3(256), dim3(256), 0, s, c, tb);
  hipLaunchKernelGGL(k_td_resort, dim3(1024), dim3(256), 0, s, c, (int64_t)c.P << c.log_r);
}
void launch_tdigest(const DevCfg& c, const PRec* part, const uint32_t* offs, int32_t T, int64_t n, DevTable tb,
                    TdBuf& td, Status* st, hipStream_t s) {
  if (n <= 0) return;
  const uint32_t none = (uint32_t)td.lidx_slots;  // no slot has this id (slots are 0 .. table slots - 1)
  const int64_t nrec = n;
  const int W = c.assigner == FW_SLIDING ? c.wpr : 1;
  n *= W;  // the items: one per (record, window)
  (void)hipMemsetAsync(td.ctr, 0, 3 * sizeof(int32_t), s);
  (void)hipMemsetAsync(td.lctr, 0, TD_LC_WORDS * sizeof(int32_t), s);
  const int32_t rchunk = std::max(1, TD_GCHUNK / W);  // (records per grouping workgroup: at most TD_GCHUNK items)
#ifndef FW_TDG_OFF
  const bool fast = c.assigner != FW_SLIDING && c.assigner != FW_SESSION && !c.td_ovctr;
#else
  const bool fast = false;
#endif
  hipLaunchKernelGGL((fast ? k_td_group<true> : k_td_group<false>), dim3((unsigned)((nrec + rchunk - 1) / rchunk)),
                     dim3(TD_GTHREADS), 0, s, c, part, offs, T, nrec, rchunk, tb, none, td, st);
  if (c.assigner == FW_SESSION) {  // the push's session merges: each merged digest's union of old centroids
    hipLaunchKernelGGL(k_td_mlink, dim3(64), dim3(256), 0, s, c, td);
    hipLaunchKernelGGL(k_td_mlist, dim3(64), dim3(256), 0, s, c, td);
    hipLaunchKernelGGL(k_td_mbuild, dim3(64), dim3(256), 0, s, c, tb, td, st);
  }
  // the digests' runs: their counts scanned (tbeg[0 .. nt], nt read on the device; td.mid is the scan's scratch:
  // the wave tier lists its digests there later), the items placed
  const unsigned grid = (unsigned)std::min<int64_t>(8192, (n + 255) / 256);
  hipLaunchKernelGGL(k_td_counts, dim3(grid), dim3(256), 0, s, td, st);
  const unsigned nb = (unsigned)((n + 1 + SCAN_B - 1) / SCAN_B);
  hipLaunchKernelGGL(k_scan_blocks_d, dim3(nb), dim3(SCAN_T), 0, s, td.tbeg, (const int32_t*)td.ctr, td.mid);
  hipLaunchKernelGGL(k_scan_top_d, dim3(1), dim3(SCAN_T), 0, s, td.mid, (const int32_t*)td.ctr);
  hipLaunchKernelGGL(k_scan_add_d, dim3(nb), dim3(SCAN_T), 0, s, td.tbeg, (const int32_t*)td.ctr, (const uint32_t*)td.mid);
  hipLaunchKernelGGL(k_td_starts, dim3(grid), dim3(256), 0, s, td, st);
  hipLaunchKernelGGL(k_td_place, dim3(grid), dim3(256), 0, s, td, n, none, st);
  hipLaunchKernelGGL(k_td_perm, dim3((unsigned)((n + TD_PERM_CH - 1) / TD_PERM_CH)), dim3(256), 0, s, td, st);  // (gs[1]:
  // after the place)
  // each run sorted: by lanes, by MSD passes (two levels) and the fallback, then in LDS (into v[0])
  hipLaunchKernelGGL(k_td_sort_lanes<16>, dim3(4096), dim3(256), 0, s, td, st);
  hipLaunchKernelGGL(k_td_sort_lanes<64>, dim3(4096), dim3(256), 0, s, td, st);
  for (int L = 0; L < 2; L++) {
    hipLaunchKernelGGL(k_td_msd_prep, dim3(1024), dim3(256), 0, s, td, L, st);
    hipLaunchKernelGGL(k_td_msd_plan, dim3(1), dim3(1024), 0, s, td, L, st);
    hipLaunchKernelGGL(k_td_msd_sample, dim3(512), dim3(1024), 0, s, td, L, st);
    hipLaunchKernelGGL(k_td_msd_hist, dim3(2048), dim3(256), 0, s, td, L, st);
    hipLaunchKernelGGL(k_td_msd_scan, dim3(1024), dim3(256), 0, s, td, L, st);
    hipLaunchKernelGGL(k_td_msd_scatter, dim3(2048), dim3(256), 0, s, td, L, st);
  }
  hipLaunchKernelGGL(k_td_sort_global, dim3(256), dim3(256), 0, s, td, st);
  hipLaunchKernelGGL(k_td_sort_lds, dim3(4096), dim3(256), 0, s, td, st);
  // the merge by size tier (the digests' old centroids and their sorted values)
  const uint64_t* vsorted = td.v[0];
  hipLaunchKernelGGL(k_td_small, dim3(grid), dim3(256), 0, s, c, tb, td, vsorted, st);
  hipLaunchKernelGGL(k_td_wave, dim3(2048), dim3(64 * TD_WAVES), td_wave_lds_bytes(c.td_nb), s, c, tb, td, vsorted, st);
  hipLaunchKernelGGL(k_td_large_old, dim3(64), dim3(256), 0, s, c, vsorted, td, st);  // (the mean keys: first)
  hipLaunchKernelGGL(k_td_large_items, dim3(grid), dim3(256), 0, s, c, n, (const uint32_t*)td.gsort, vsorted, none, td, st);
  hipLaunchKernelGGL(k_td_large_groups, dim3(2048), dim3(256), 0, s, c, vsorted, td, st);
  hipLaunchKernelGGL(k_td_large_compact, dim3(64), dim3(64), 0, s, c, td, st);
  if (c.assigner == FW_SESSION) hipLaunchKernelGGL(k_td_mclear, dim3(64), dim3(256), 0, s, c, td);
  hipLaunchKernelGGL(k_td_reset, dim3(grid), dim3(256), 0, s, td);
}
void launch_rehash(const DevCfg& oc, DevTable ot, const DevCfg& nc, DevTable nt, hipStream_t s) {
  if (oc.dense)
    hipLaunchKernelGGL(k_dt_rehash, dim3(oc.P), dim3(FW_FIRE_THREADS), 0, s, oc, ot, nc, nt);
  else
    hipLaunchKernelGGL(k_rehash, dim3(oc.P), dim3(FW_FIRE_THREADS), 0, s, oc, ot, nc, nt);
}


void launch_snapshot(const DevCfg& c, DevTable tb, int32_t p0, int32_t np, StateCols out, unsigned long long* count,
                     hipStream_t s) {
  hipLaunchKernelGGL(k_snapshot, dim3(np), dim3(FW_FIRE_THREADS), 0, s, c, tb, p0, out, count);
}
void launch_block_export(const DevCfg& c, const int64_t* blk, int64_t n, uint8_t* acc, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_block_export, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, c, blk, n, acc);
}
void launch_pool_take(const DevCfg& c, int32_t h, int32_t take, int64_t bump, int64_t n, int64_t* ids, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_pool_take, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c, h, take, bump, n, ids);
}
void launch_pool_give(const DevCfg& c, const int64_t* ids, int64_t n, int32_t h, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_pool_give, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c, ids, n, h);
}
void launch_restore(const DevCfg& c, int32_t kg, StateCols in, int64_t n, int32_t* demand, DevTable tb, Status* st,
                    const int32_t* round_of, int32_t rounds, hipStream_t s) {
  const unsigned blocks = (unsigned)((n + 255) / 256);
  if (!blocks) return;
  if (demand) {
    hipLaunchKernelGGL(k_restore_count, dim3(blocks), dim3(256), 0, s, c, kg, in, n, demand, st);
    return;
  }
  // rows restoring the same (key, window) twice go in different rounds, so each round inserts a window at
  // most once and later rounds merge into it (one launch per round, stream-ordered)
  for (int32_t r = 0; r < std::max(1, rounds); r++)
    hipLaunchKernelGGL(k_restore, dim3(blocks), dim3(256), 0, s, c, kg, in, n, tb, st, round_of, r);
}

void launch_live_offsets(const DevCfg& c, DevTable tb, uint32_t* offs, uint32_t* scratch, hipStream_t s) {
  hipLaunchKernelGGL(k_live_u32, dim3((unsigned)((c.P + 256) / 256)), dim3(256), 0, s, tb, c.P, offs);
  launch_scan(offs, (int64_t)c.P + 1, scratch, s);
}
void launch_extract(const DevCfg& c, DevTable tb, const uint32_t* offs, PartialCols out, hipStream_t s) {
  hipLaunchKernelGGL(k_extract, dim3(c.P), dim3(FW_FIRE_THREADS), 0, s, c, tb, offs, out);
}
void launch_hll_extract_counts(const DevCfg& c, PartialCols out, int64_t n, uint32_t* cnt, uint32_t* scan_tmp,
                               hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_hll_extract_counts, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c, out, n, cnt);
  (void)hipMemsetAsync(cnt + n, 0, sizeof(uint32_t), s);
  launch_scan(cnt, n + 1, scan_tmp, s);  // in place: offsets, cnt[n] = total
}
void launch_hll_extract_regs(const DevCfg& c, PartialCols out, int64_t n, const uint32_t* off, uint32_t* regs,
                             hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_hll_extract_regs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c, out, n, off, regs);
}
__global__ void k_hll_reg_counts(PartialCols in, int64_t n, uint32_t* __restrict__ off) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= n) off[i] = i < n ? (uint32_t)in.sum[i] : 0u;
}
void launch_hll_reg_offsets(PartialCols in, int64_t n, uint32_t* off, uint32_t* scan_tmp, hipStream_t s) {
  hipLaunchKernelGGL(k_hll_reg_counts, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, s, in, n, off);
  launch_scan(off, n + 1, scan_tmp, s);  // off[i] = partial i's first register, off[n] = their total
}
void launch_hll_push_regs(const DevCfg& c, int64_t wm, PartialCols in, int64_t n, const uint32_t* regs,
                          const uint32_t* off, DevTable tb, Status* st, hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL(k_hll_push_regs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c, wm, in, n, regs, off, tb, st);
}
void launch_pscatter(const DevCfg& c, int64_t wm, PartialCols in, int64_t n, int32_t T, uint32_t* offs, PartialRec* part,
                     Status* st, hipStream_t s) {
  if (T > 0)
    hipLaunchKernelGGL(k_pscatter, dim3(T), dim3(FW_TILE_THREADS), (size_t)c.P * sizeof(uint32_t), s, c, wm, in, n, T,
                       (const uint32_t*)offs, part, st);
}
void launch_pmerge(const DevCfg& c, const PartialRec* part, const uint32_t* offs, int32_t T, DevTable tb, AggProg prog,
                   int resume, Status* st, hipStream_t s) {
  if (c.dense)
    hipLaunchKernelGGL((k_dt_aggregate<DT_PARTS, false>), dim3(c.P), dim3(FW_DT_THREADS), 0, s, c, (const void*)part, offs,
                       T, tb, prog, resume, st, (const uint32_t*)nullptr, (int64_t)0);
  else
    hipLaunchKernelGGL(k_pmerge, dim3(c.P), dim3(FW_AGG_THREADS), 0, s, c, part, offs, T, tb, prog, resume, st);
}
void launch_dt_restore_runs(const DevCfg& c, int32_t kg, StateCols in, int64_t n, int32_t* rp, uint32_t* hist,
                            uint32_t* scan_tmp, PartialRec* tmp, PartialRec* part, Status* st, hipStream_t s) {
  if (n <= 0) return;
  const int32_t T = ntiles(n);
  hipLaunchKernelGGL(k_dt_rows_prep, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c, kg, in, n, rp, tmp, st);
  hipLaunchKernelGGL(k_dt_rows_hist, dim3(T), dim3(FW_TILE_THREADS), (size_t)(c.P + 1) * sizeof(uint32_t), s, c.P,
                     (const int32_t*)rp, n, T, hist);
  launch_scan(hist, (int64_t)(c.P + 1) * T, scan_tmp, s);
  hipLaunchKernelGGL(k_dt_rows_scatter, dim3(T), dim3(FW_TILE_THREADS), (size_t)c.P * sizeof(uint32_t), s, c.P,
                     (const int32_t*)rp, (const PartialRec*)tmp, n, T, (const uint32_t*)hist, part);
}
void launch_table_stats(const DevCfg& c, DevTable tb, unsigned long long* out3, hipStream_t s) {
  hipLaunchKernelGGL(k_table_stats, dim3(c.P), dim3(FW_FIRE_THREADS), 0, s, c, tb, out3);
}

void launch_reset_regions(const DevCfg& c, DevTable tb, hipStream_t s) {
  hipLaunchKernelGGL(k_reset_regions, dim3((c.P + 255) / 256), dim3(256), 0, s, c, tb);
}

void launch_key_groups(const int64_t* key, const int32_t* kh, int32_t kind, int64_t n, int32_t max_par, int32_t* kg,
                       hipStream_t s) {
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  if (blocks > 0) hipLaunchKernelGGL(k_key_groups, dim3((unsigned)blocks), dim3(256), 0, s, key, kh, kind, n, max_par, kg);
}

void launch_route(const int64_t* key, const int64_t* ts, const int64_t* val, const int32_t* kh, int32_t kind,
                  int64_t n, int32_t max_par, int32_t par, int64_t* ko, int64_t* to, int64_t* vo, int32_t* ho,
                  int64_t* counts, uint32_t* scratch, hipStream_t s) {
  const int32_t T = ntiles(n);
  const int64_t m = (int64_t)par * T;
  uint32_t* hist = scratch;
  uint32_t* scan_tmp = scratch + m;
  if (T > 0) {
    hipLaunchKernelGGL(k_route_hist, dim3(T), dim3(FW_TILE_THREADS), par * sizeof(uint32_t), s, key, kh, kind, n,
                       max_par, par, T, hist);
    launch_scan(hist, m, scan_tmp, s);
    const size_t lds = (size_t)par * (1 + FW_TILE_THREADS / 64) * sizeof(uint32_t);
    hipLaunchKernelGGL(k_route_scatter, dim3(T), dim3(FW_TILE_THREADS), lds, s, key, ts, val, kh, kind, n, max_par, par,
                       T, (const uint32_t*)hist, ko, to, vo, ho);
    hipLaunchKernelGGL(k_route_counts, dim3(1), dim3(std::max(64, ((par + 63) / 64) * 64)), 0, s, (const uint32_t*)hist,
                       par, T, n, counts);
  } else {
    (void)hipMemsetAsync(counts, 0, par * sizeof(int64_t), s);
  }
}

void launch_generate(uint64_t seed, int64_t first, int64_t n, int64_t num_keys, const double* cdf, int64_t ts_base,
                     int64_t rate, int64_t jitter, int64_t* key, int64_t* ts, int64_t* val, int64_t* max_ts,
                     hipStream_t s) {
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
  if (blocks > 0)
    hipLaunchKernelGGL(k_generate, dim3((unsigned)blocks), dim3(256), 0, s, seed, first, n, num_keys, cdf, ts_base, rate,
                       jitter, key, ts, val, max_ts);
}

}  // namespace fwdev
