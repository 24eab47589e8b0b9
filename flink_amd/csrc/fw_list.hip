// fw_list.hip — f4: the window-contents (ListState) operator of the C-ABI (fw_list_*, include/flink_window.h):
// WindowedStream.apply / process with an Iterable window function and the EvictingWindowOperator
// (paths relative to /root/reference/flink-streaming-java/src/main/java/org/apache/flink/streaming/):
//   runtime/operators/windowing/EvictingWindowOperator.java:102-239 processElement, :241-286 onEventTime,
//   :334-366 emitWindowContents; WindowOperator.java:291-469 (no evictor), :576-651 lateness and cleanup;
//   api/windowing/triggers/{EventTimeTrigger.java:37-73, CountTrigger.java:47-70, PurgingTrigger.java:45-59};
//   api/windowing/evictors/{CountEvictor.java:50-78, TimeEvictor.java:54-104, DeltaEvictor.java:59-80}.
//
// HBM layout (one handle = one subtask on one GPU):
//   groups   an open-addressing map (key, window start) -> group id (the slot), per group its key group, the
//            CountTrigger count and flags {trigger timer registered, touched by the current push, due to fire,
//            due to be cleaned up}: the (key, window) namespaces of "window-contents" and the trigger state;
//   log      the elements of every list as SoA columns {ts, value, arrival ordinal, group id} in arrival
//            order; an evicted, purged or cleaned-up element gets group id -1.  A list is the group's live
//            elements in log order.  Dead elements are dropped by a stable compaction (with a map rebuild)
//            once they outnumber the live ones.
// A push appends its records' (record, window) entries to the log (one scan for the offsets, one pass for
// the map lookups / inserts); only when elements can fire while being processed (CountTrigger, or an
// EventTimeTrigger window whose maxTimestamp is already <= the watermark: allowed lateness) are the touched
// groups' lists gathered (a stable radix sort of their log positions by group) and walked in order, one
// thread per list, exactly as processElement's trigger / evictor / emit sequence.  A watermark marks the
// groups whose trigger timer (maxTimestamp) or cleanup timer is due, walks the lists of the firing ones the
// same way, and drops the cleaned-up ones.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <string>
#include <vector>

#include "../../include/flink_window.h"

namespace {

constexpr int64_t LMAX = INT64_MAX;
constexpr int64_t LMIN = INT64_MIN;
#include "fw_jmath.h"

#ifndef FW_LIST_ROOM
#define FW_LIST_ROOM (int64_t(1) << 28)  // elements a walk may size its output for up front
#endif
enum : uint32_t { GF_TIMER = 1u, GF_TOUCH = 2u, GF_FIRE = 4u, GF_CLEAN = 8u };
enum : uint32_t { LF_NO_TS = 1u, LF_KEY_GROUP = 2u, LF_MAP_FULL = 4u, LF_ELEMS = 8u, LF_MERGE_LATE = 16u, LF_MERGE_WIDE = 32u };
constexpr uint32_t G_EMPTY = 0u, G_BUSY = 1u, G_LIVE = 2u, G_TOMB = 3u;

struct LCfg {
  int32_t assigner, vt, key_kind, trigger, purging, evictor, evict_after, side_output, emit, max_par, kg0, nkg;
  int64_t size, slide, offset, lateness, trig_n, ev_n;
  double thr;
};

struct LCounters {
  unsigned long long rows, elems, side, late, dead, live_groups, tombs, nfire, nclean, count;
  unsigned int flags, need_seq;
  long long next_due;  // no group's trigger or cleanup timer is earlier: a watermark below it has nothing to do
};

struct alignas(32) GSlot {
  uint32_t st;    // G_EMPTY / G_BUSY / G_LIVE / G_TOMB
  uint32_t fl;    // GF_* flags
  int32_t kg;     // key group
  int32_t cnt;    // CountTrigger's count
  int64_t key, start;
};

struct alignas(32) LPay {
  int64_t ts, val, ord, pad;
};

struct LState {
  GSlot* g;  // the group map: one 32-byte slot per group (a lookup reads one sector)
  uint32_t gmask;
  // session windows (FW_SESSION, fw_list.hip "session windows"): per slot its window end and list head / tail
  int64_t *wend, *whead, *wtail;
  LPay* lpay;  // the elements' payload, one 32-byte sector each (a gather reads one sector per element)
  int32_t* lgid;
  int64_t *rkey, *rstart, *rend, *rcnt, *rsum, *rmin, *rmax, *rfirst, *roff;
  int64_t *ets, *eval, *eord;
  int64_t ecap;
  int64_t *skey, *sts, *sval;
  LCounters* ctr;
};

// ---------------------------------------------------------------- windows
__device__ __forceinline__ bool event_time(const LCfg& c) { return c.assigner != FW_GLOBAL; }
__device__ __forceinline__ int64_t w_end(const LCfg& c, int64_t start) {
  return c.assigner == FW_GLOBAL ? LMAX : jadd(start, c.size);
}
// TimeWindow.maxTimestamp (end - 1); GlobalWindow.maxTimestamp = Long.MAX_VALUE
__device__ __forceinline__ int64_t w_max_ts(const LCfg& c, int64_t start) {
  return c.assigner == FW_GLOBAL ? LMAX : jsub(jadd(start, c.size), 1);
}
// WindowOperator.cleanupTime (:637-644); GlobalWindows are not event time: no cleanup timer (LMAX)
__device__ __forceinline__ int64_t w_cleanup(const LCfg& c, int64_t start) {
  if (!event_time(c)) return LMAX;
  const int64_t mx = w_max_ts(c, start);
  const int64_t t = jadd(mx, c.lateness);
  return t >= mx ? t : LMAX;
}
// TimeWindow.getWindowStartWithOffset (TimeWindow.java:254-256): Java's truncating % is C++'s
__device__ __forceinline__ int64_t w_start_of(int64_t ts, int64_t off, int64_t size) {
  return jsub(ts, jadd(jsub(ts, off), size) % size);
}
// every window of a record that is not late (WindowOperator.isWindowLate, :629-631), in the assigner's order
template <class F>
__device__ __forceinline__ void for_windows(const LCfg& c, int64_t ts, int64_t wm, F f) {
  if (c.assigner == FW_GLOBAL) {
    f(LMIN);
    return;
  }
  if (c.assigner == FW_TUMBLING) {
    const int64_t s = w_start_of(ts, c.offset, c.size);
    if (!(w_cleanup(c, s) <= wm)) f(s);
    return;
  }
  const int64_t last = w_start_of(ts, c.offset, c.slide);  // SlidingEventTimeWindows.java:67-81
  for (int64_t s = last; s > jsub(ts, c.size); s = jsub(s, c.slide))
    if (!(w_cleanup(c, s) <= wm)) f(s);
}

// ---------------------------------------------------------------- group map
__device__ __forceinline__ uint32_t g_hash(int64_t key, int64_t start) {
  return (uint32_t)fmix64((uint64_t)key ^ fmix64((uint64_t)start ^ 0x9E3779B97F4A7C15ull));
}
// Lookups read the state word with a relaxed agent-scope load (L2, no L1 invalidation as an acquire would cost on
// every probe) and, once it reads LIVE, the key and window the same way: the inserter's write-through stores of both
// complete before its store of LIVE, and the key loads are issued only after the state's value has arrived (they
// depend on it), so they read what the inserter wrote.
__device__ __forceinline__ int64_t ld_l2(const int64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// limit > 0: no new group beyond `limit` live ones (LF_MAP_FULL is raised instead, nothing inserted).  *ins counts
// the groups this call inserted (the caller adds them to live_groups, one atomic per workgroup).  live_groups lags
// the launch (its workgroups add their inserts when they finish), so a push with many new groups can fill the map
// past the limit before any lane sees it; a probe chain therefore stops at G_PROBE_CAP slots (at <= 3/4 load a
// chain that long means the map is overfull) and, past G_PROBE_CHECK slots, at a raised LF_MAP_FULL: the push is
// redone after a growth, so a full map costs each later insert a bounded walk, not one over the whole map.
constexpr uint32_t G_PROBE_CHECK = 32, G_PROBE_CAP = 1024;
__device__ int32_t g_find_insert(const LState& S, int64_t key, int64_t start, int32_t kg, unsigned long long limit,
                                 unsigned* ins) {
  uint32_t s = g_hash(key, start) & S.gmask;
  for (uint32_t probes = 0; probes <= S.gmask;) {
    if (limit && probes >= G_PROBE_CHECK &&
        (probes >= G_PROBE_CAP ||
         (__hip_atomic_load(&S.ctr->flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & LF_MAP_FULL)))
      break;
    const uint32_t cur = __hip_atomic_load(&S.g[s].st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_signal_fence(__ATOMIC_ACQUIRE);  // (the compiler keeps the key loads behind it)
    if (cur == G_LIVE) {
      if (ld_l2(&S.g[s].key) == key && ld_l2(&S.g[s].start) == start) return (int32_t)s;
    } else if (cur == G_BUSY) {
      continue;  // being published by another lane: read it again
    } else if (cur == G_EMPTY) {
      if (limit && __hip_atomic_load(&S.ctr->live_groups, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= limit) {
        atomicOr(&S.ctr->flags, LF_MAP_FULL);
        return -1;
      }
      if (atomicCAS(&S.g[s].st, G_EMPTY, G_BUSY) == G_EMPTY) {
        // publish without an L2 write-back per group (an agent-scope release is one): the fields are stored
        // write-through (relaxed agent-scope stores, sc1), this lane waits for them, then stores LIVE the same
        // way; readers poll the state and load the fields with relaxed agent-scope loads (sc1), the hand-off of
        // MI355X_MICROARCH.md's sc1 table (one lane signalling for all its own stores)
        __hip_atomic_store(&S.g[s].key, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&S.g[s].start, start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&S.g[s].kg, kg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&S.g[s].cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&S.g[s].fl, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&S.g[s].st, (uint32_t)G_LIVE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        (*ins)++;
        return (int32_t)s;
      }
      continue;  // lost the race for this slot: read it again
    }
    s = (s + 1) & S.gmask;  // live foreign group or tombstone
    probes++;
  }
  atomicOr(&S.ctr->flags, LF_MAP_FULL);
  return -1;
}
// per-workgroup minimum into a global one
__device__ __forceinline__ void block_min(long long* dst, long long v) {
  __shared__ long long acc;
  if (threadIdx.x == 0) acc = LMAX;
  __syncthreads();
  if (v != LMAX) atomicMin(&acc, v);
  __syncthreads();
  if (threadIdx.x == 0 && acc != LMAX) atomicMin(dst, acc);
}
// per-workgroup sum into a global counter (one atomic per workgroup instead of one per thread)
__device__ __forceinline__ void block_add(unsigned long long* dst, unsigned long long v) {
  __shared__ unsigned long long acc;
  if (threadIdx.x == 0) acc = 0;
  __syncthreads();
  if (v) atomicAdd(&acc, v);
  __syncthreads();
  if (threadIdx.x == 0 && acc) atomicAdd(dst, acc);
}

// ---------------------------------------------------------------- push
// per record: its non-late windows (wcnt), errors, late records (side output / numLateRecordsDropped)
__global__ __launch_bounds__(256) void k_lp_count(LCfg c, LState S, const int64_t* __restrict__ key,
                                                  const int64_t* __restrict__ ts, const int64_t* __restrict__ val,
                                                  const int32_t* __restrict__ kh, int64_t n, int64_t wm,
                                                  uint32_t* __restrict__ wcnt) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = ts[i];
    wcnt[i] = 0;
    if (event_time(c) && t == LMIN) {  // TumblingEventTimeWindows.java:69-71
      atomicOr(&S.ctr->flags, LF_NO_TS);
      continue;
    }
    const int32_t kg = key_group(key_hash_of(c.key_kind, key[i], kh, i), c.max_par);
    if ((uint32_t)(kg - c.kg0) >= (uint32_t)c.nkg) {
      atomicOr(&S.ctr->flags, LF_KEY_GROUP);
      continue;
    }
    uint32_t k = 0;
    for_windows(c, t, wm, [&](int64_t) { k++; });
    wcnt[i] = k;
    // skipped && isElementLate (:410-418, :620-622)
    if (k == 0 && event_time(c) && jadd(t, c.lateness) <= wm) {
      if (c.side_output) {
        const unsigned long long r = atomicAdd(&S.ctr->side, 1ull);
        S.skey[r] = key[i];
        S.sts[r] = t;
        S.sval[r] = val[i];
      } else {
        atomicAdd(&S.ctr->late, 1ull);
      }
    }
  }
}

// the entries: log[base + woff[i] + j] = (ts, value, ordinal, group) for the j-th non-late window of record i;
// groups whose elements fire while being processed are marked for the ordered walk.
// AU records per thread in flight: a one-window record's home slot is read as one 64-bit (state, flags) load for all
// of them, then the key and window of the LIVE ones, so the common case (its group already at its home slot) costs
// two dependent round trips per AU records; the rest (a probe chain, a new group, several windows) go through
// g_find_insert one by one.
constexpr int AU = 4;
__global__ __launch_bounds__(256) void k_lp_append(LCfg c, LState S, const int64_t* __restrict__ key,
                                                   const int64_t* __restrict__ ts, const int64_t* __restrict__ val,
                                                   const int32_t* __restrict__ kh, int64_t n, int64_t wm,
                                                   const uint32_t* __restrict__ wcnt, const uint32_t* __restrict__ woff,
                                                   int64_t base, int64_t ord_base, unsigned long long limit) {
  long long due = LMAX;  // the earliest timer these entries register
  unsigned ins = 0;
  bool seq = false;      // some entry fires while being processed (one store per workgroup, not per entry)
  // one entry: its payload and group, and the trigger's bookkeeping (fl: the group's flags as last read)
  auto put = [&](int64_t idx, int64_t i, int64_t t, int64_t v, int64_t s, int32_t g, uint32_t fl) {
    S.lpay[idx] = LPay{t, v, ord_base + i, 0};
    S.lgid[idx] = g;
    if (g < 0) {
      atomicOr(&S.ctr->flags, LF_MAP_FULL);
      return;
    }
    const int64_t mts = w_max_ts(c, s);
    due = min(due, (long long)(c.trigger == FW_TRIGGER_EVENT_TIME && mts > wm ? mts : w_cleanup(c, s)));
    if (c.trigger == FW_TRIGGER_COUNT || mts <= wm) {  // CountTrigger / late firing
      atomicOr(&S.g[g].fl, GF_TOUCH);
      seq = true;
    } else if (!(fl & GF_TIMER)) {  // EventTimeTrigger.onElement registers the timer at maxTimestamp
      atomicOr(&S.g[g].fl, GF_TIMER);
    }
  };
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * AU;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x * AU; i0 < n; i0 += stride) {
    int64_t k[AU], t[AU], v[AU], s[AU], idx[AU];
    uint32_t wc[AU], home[AU];
    int32_t kg[AU];
#pragma unroll
    for (int u = 0; u < AU; u++) {
      const int64_t i = i0 + u * blockDim.x + threadIdx.x;
      wc[u] = i < n ? wcnt[i] : 0u;
      k[u] = t[u] = v[u] = idx[u] = 0;
      if (wc[u]) {
        t[u] = ts[i];
        k[u] = key[i];
        v[u] = val[i];
        idx[u] = base + woff[i];
      }
    }
    uint64_t sf[AU];
#pragma unroll
    for (int u = 0; u < AU; u++) {
      const int64_t i = i0 + u * blockDim.x + threadIdx.x;
      s[u] = LMIN;
      kg[u] = 0;
      sf[u] = 0;
      if (!wc[u]) continue;
      kg[u] = key_group(key_hash_of(c.key_kind, k[u], kh, i), c.max_par);
      if (wc[u] != 1) continue;
      for_windows(c, t[u], wm, [&](int64_t w) { s[u] = w; });
      home[u] = g_hash(k[u], s[u]) & S.gmask;
      sf[u] = __hip_atomic_load(reinterpret_cast<const uint64_t*>(&S.g[home[u]].st), __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
    }
    __atomic_signal_fence(__ATOMIC_ACQUIRE);  // (the compiler keeps the key loads behind the state words)
    int64_t hk[AU], hs[AU];
#pragma unroll
    for (int u = 0; u < AU; u++) {
      hk[u] = hs[u] = 0;
      if (wc[u] == 1 && (uint32_t)sf[u] == G_LIVE) {
        hk[u] = ld_l2(&S.g[home[u]].key);
        hs[u] = ld_l2(&S.g[home[u]].start);
      }
    }
#pragma unroll
    for (int u = 0; u < AU; u++) {
      if (!wc[u]) continue;
      const int64_t i = i0 + u * blockDim.x + threadIdx.x;
      if (wc[u] == 1) {
        if ((uint32_t)sf[u] == G_LIVE && hk[u] == k[u] && hs[u] == s[u]) {
          put(idx[u], i, t[u], v[u], s[u], (int32_t)home[u], (uint32_t)(sf[u] >> 32));
        } else {
          const int32_t g = g_find_insert(S, k[u], s[u], kg[u], limit, &ins);
          put(idx[u], i, t[u], v[u], s[u], g, g >= 0 ? S.g[g].fl : 0u);
        }
        continue;
      }
      int64_t x = idx[u];
      for_windows(c, t[u], wm, [&](int64_t w) {
        const int32_t g = g_find_insert(S, k[u], w, kg[u], limit, &ins);
        put(x++, i, t[u], v[u], w, g, g >= 0 ? S.g[g].fl : 0u);
      });
    }
  }
  if (__syncthreads_or(seq) && threadIdx.x == 0) S.ctr->need_seq = 1u;
  block_min(&S.ctr->next_due, due);
  block_add(&S.ctr->live_groups, ins);
}

// ---------------------------------------------------------------- ordered walks
__global__ __launch_bounds__(256) void k_sel_flags(const LState S, int64_t n, uint32_t bit, uint8_t* __restrict__ f) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t g = S.lgid[i];
    f[i] = g >= 0 && (S.g[g].fl & bit) ? 1 : 0;
  }
}
__global__ __launch_bounds__(256) void k_sel_keys(const LState S, const uint32_t* __restrict__ idx, int64_t m,
                                                  uint32_t* __restrict__ keys) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
    keys[i] = (uint32_t)S.lgid[idx[i]];
}
__global__ __launch_bounds__(256) void k_seg_flags(const uint32_t* __restrict__ keys, int64_t m, uint8_t* __restrict__ f) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
    f[i] = i == 0 || keys[i] != keys[i - 1] ? 1 : 0;
}

// Double.compare / Float.compare order of f64 bits as a signed key (canonical NaN largest)
__device__ __forceinline__ int64_t fkey(int64_t b) {
  if ((b & 0x7ff0000000000000ll) == 0x7ff0000000000000ll && (b & 0x000fffffffffffffll)) b = 0x7ff8000000000000ll;
  return b >= 0 ? b : (b ^ 0x7fffffffffffffffll);
}
__device__ __forceinline__ int64_t canon(int64_t b) {
  return ((b & 0x7ff0000000000000ll) == 0x7ff0000000000000ll && (b & 0x000fffffffffffffll)) ? 0x7ff8000000000000ll : b;
}
// DeltaEvictor's built-in DeltaFunction: last.field - e.field in the field's Java arithmetic, as a double
__device__ __forceinline__ double delta_of(const LCfg& c, int64_t e, int64_t last) {
  switch (c.vt) {
    case FW_VAL_I64: return (double)jsub(last, e);
    case FW_VAL_F64: return __longlong_as_double(last) - __longlong_as_double(e);
    case FW_VAL_F32: return (double)((float)__longlong_as_double(last) - (float)__longlong_as_double(e));
    default: return (double)(int32_t)((uint32_t)(int32_t)last - (uint32_t)(int32_t)e);
  }
}

// The walk's view of the selected elements, gathered into list order (k_gather_sel): their timestamps, values and
// ordinals side by side, and whether each is still live; a kill also marks the log (group -1).
struct LView {
  const uint32_t* pos;  // log index of each sorted position
  const int64_t *ts, *val, *ord;
  uint8_t* alive;
  int32_t* lgid;
  __device__ __forceinline__ void kill(int64_t q) const {
    alive[q] = 0;
    lgid[pos[q]] = -1;
  }
};

// one list in the sorted positions [a .. j] of the view: which of its live elements the evictor removes
// (CountEvictor.evict :63-78, TimeEvictor.evict :67-96, DeltaEvictor.evict :72-80).
// mark = false: returns how many would remain; mark = true: kills the others and returns the remaining count.
__device__ int64_t evict(const LCfg& c, const LState& S, const LView& V, int64_t a, int64_t j, bool mark) {
  int64_t live = 0;
  for (int64_t q = a; q <= j; q++) live += V.alive[q];
  if (c.evictor == FW_EVICT_NONE || live == 0) return live;
  int64_t killed = 0;
  if (c.evictor == FW_EVICT_COUNT) {
    if (live <= c.ev_n) return live;
    const int64_t drop = live - c.ev_n;
    if (mark) {
      for (int64_t q = a; q <= j && killed < drop; q++)
        if (V.alive[q]) {
          V.kill(q);
          killed++;
        }
    } else {
      killed = drop;
    }
  } else if (c.evictor == FW_EVICT_TIME) {
    int64_t first_ts = 0, mx = LMIN;
    bool have = false;
    for (int64_t q = a; q <= j; q++) {
      if (!V.alive[q]) continue;
      if (!have) first_ts = V.ts[q];
      have = true;
      mx = max(mx, V.ts[q]);
    }
    if (first_ts == LMIN) return live;  // hasTimestamp of the first element
    const int64_t cutoff = jsub(mx, c.ev_n);
    for (int64_t q = a; q <= j; q++) {
      if (!V.alive[q] || !(V.ts[q] <= cutoff)) continue;
      if (mark) V.kill(q);
      killed++;
    }
  } else {  // FW_EVICT_DELTA
    int64_t last = 0;
    for (int64_t q = j; q >= a; q--)
      if (V.alive[q]) {
        last = V.val[q];
        break;
      }
    for (int64_t q = a; q <= j; q++) {
      if (!V.alive[q] || !(delta_of(c, V.val[q], last) >= c.thr)) continue;
      if (mark) V.kill(q);
      killed++;
    }
  }
  if (mark && killed) atomicAdd(&S.ctr->dead, (unsigned long long)killed);
  return live - killed;
}

// emitWindowContents (:334-366) of group g over the list [a .. j] of the view: evictBefore, one row (+ the
// elements), evictAfter.  False (nothing changed) when the element buffer cannot take the contents.
// rsv_row >= 0: the row and the elements were reserved by the caller (k_walk's wave-aggregated reservation).
__device__ __forceinline__ int64_t fired_count(const LCfg& c, const LState& S, const LView& V, int64_t a, int64_t j) {
  int64_t cnt = 0;  // the elements the function sees
  if (c.evict_after)
    for (int64_t q = a; q <= j; q++) cnt += V.alive[q];
  else
    cnt = evict(c, S, V, a, j, false);
  return cnt;
}
__device__ bool emit_firing(const LCfg& c, const LState& S, const LView& V, uint32_t g, int64_t a, int64_t j,
                            bool room, int64_t rsv_row = -1, int64_t rsv_elem = 0, int64_t rsv_cnt = 0) {
  const int64_t cnt = rsv_row >= 0 ? rsv_cnt : fired_count(c, S, V, a, j);
  int64_t eoff = 0;
  if (rsv_row >= 0) {
    eoff = c.emit && cnt ? rsv_elem : 0;
  } else if (c.emit && cnt && room) {  // the host sized the element buffer for every possible firing
    eoff = (int64_t)atomicAdd(&S.ctr->elems, (unsigned long long)cnt);
  } else if (c.emit && cnt) {  // reserve the elements (rows were sized by the host: one per possible firing)
    unsigned long long cur = __hip_atomic_load(&S.ctr->elems, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (true) {
      if ((int64_t)cur + cnt > S.ecap) {
        atomicOr(&S.ctr->flags, LF_ELEMS);
        return false;
      }
      const unsigned long long prev = atomicCAS(&S.ctr->elems, cur, cur + (unsigned long long)cnt);
      if (prev == cur) break;
      cur = prev;
    }
    eoff = (int64_t)cur;
  }
  if (!c.evict_after) evict(c, S, V, a, j, true);
  const bool fl = c.vt == FW_VAL_F64 || c.vt == FW_VAL_F32;
  double ds = 0.0;
  int64_t is = 0, mn = 0, mx = 0, first = -1, k = 0;
  for (int64_t q = a; q <= j; q++) {
    if (!V.alive[q]) continue;
    const int64_t v = V.val[q];
    if (k == 0) first = V.ord[q];
    if (fl) {
      const double d = __longlong_as_double(v);
      ds = k == 0 ? d : c.vt == FW_VAL_F32 ? (double)((float)ds + (float)d) : ds + d;
      if (k == 0 || fkey(v) < fkey(mn)) mn = v;
      if (k == 0 || fkey(v) > fkey(mx)) mx = v;
    } else {
      is = k == 0 ? v : jadd(is, v);
      if (k == 0 || v < mn) mn = v;
      if (k == 0 || v > mx) mx = v;
    }
    if (c.emit) {
      S.ets[eoff + k] = V.ts[q];
      S.eval[eoff + k] = v;
      S.eord[eoff + k] = V.ord[q];
    }
    k++;
  }
  const unsigned long long r = rsv_row >= 0 ? (unsigned long long)rsv_row : atomicAdd(&S.ctr->rows, 1ull);
  S.rkey[r] = S.g[g].key;
  S.rstart[r] = S.g[g].start;
  S.rend[r] = w_end(c, S.g[g].start);
  S.rcnt[r] = k;
  if (fl) {
    S.rsum[r] = __double_as_longlong(ds);
    S.rmin[r] = k ? canon(mn) : 0;
    S.rmax[r] = k ? canon(mx) : 0;
  } else {
    S.rsum[r] = c.vt == FW_VAL_I32 ? (int64_t)(int32_t)is : c.vt == FW_VAL_I16 ? (int64_t)(int16_t)is
              : c.vt == FW_VAL_I8 ? (int64_t)(int8_t)is : is;
    S.rmin[r] = mn;
    S.rmax[r] = mx;
  }
  S.rfirst[r] = first;
  S.roff[r] = c.emit ? eoff : 0;
  if (c.evict_after) evict(c, S, V, a, j, true);
  return true;
}
__device__ void purge(const LState& S, const LView& V, int64_t a, int64_t j) {
  int64_t killed = 0;
  for (int64_t q = a; q <= j; q++)
    if (V.alive[q]) {
      V.kill(q);
      killed++;
    }
  if (killed) atomicAdd(&S.ctr->dead, (unsigned long long)killed);
}

// the selected elements in list order, side by side (one pass of random reads, coalesced writes)
__global__ __launch_bounds__(256) void k_gather_sel(LState S, const uint32_t* __restrict__ pos, int64_t m,
                                                    int64_t* __restrict__ ts, int64_t* __restrict__ val,
                                                    int64_t* __restrict__ ord, uint8_t* __restrict__ alive) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t e = pos[i];
    const LPay p = S.lpay[e];
    ts[i] = p.ts;
    val[i] = p.val;
    ord[i] = p.ord;
    alive[i] = 1;  // selected entries are live
  }
}

// One thread per list.  PUSH: the list's elements appended by this push (log index >= base_new), in order:
// CountTrigger.onElement / EventTimeTrigger.onElement (maxTimestamp <= watermark: FIRE), the firing over the
// list up to the element, PurgingTrigger's purge (EvictingWindowOperator.java:186-222).  prog[s] = where a
// launch stopped (the element buffer was full); the host grows it and launches again.
// WATERMARK: the due lists fire over all their elements (onEventTime, :241-286).
template <bool PUSH>
__global__ __launch_bounds__(256) void k_walk(LCfg c, LState S, LView V, const uint32_t* __restrict__ keys,
                                              const uint32_t* __restrict__ seg, int64_t nseg, int64_t base_new,
                                              int64_t wm, int64_t* __restrict__ prog, bool room) {
  const uint32_t* __restrict__ pos = V.pos;
  if (!PUSH && room) {  // a watermark with room for every firing: one reservation of rows and elements per wave
    const int lane = __lane_id();
    for (int64_t s0 = (int64_t)blockIdx.x * blockDim.x; s0 < nseg; s0 += (int64_t)gridDim.x * blockDim.x) {
      const int64_t s = s0 + threadIdx.x;
      int64_t a = 0, b = 0;
      uint32_t g = 0;
      bool act = false;
      if (s < nseg) {
        a = seg[s];
        b = seg[s + 1];
        g = keys[a];
        act = (S.g[g].fl & GF_FIRE) != 0;
      }
      const int64_t cnt = act ? fired_count(c, S, V, a, b - 1) : 0;
      const unsigned long long rr = act ? 1ull : 0ull, ee = act && c.emit ? (unsigned long long)cnt : 0ull;
      unsigned long long xr = rr, xe = ee;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long yr = __shfl_up(xr, o, 64), ye = __shfl_up(xe, o, 64);
        if (lane >= o) {
          xr += yr;
          xe += ye;
        }
      }
      unsigned long long br = 0, be = 0;
      if (lane == 63) {
        if (xr) br = atomicAdd(&S.ctr->rows, xr);
        if (xe) be = atomicAdd(&S.ctr->elems, xe);
      }
      br = __shfl(br, 63, 64);
      be = __shfl(be, 63, 64);
      if (!act) continue;
      emit_firing(c, S, V, g, a, b - 1, true, (int64_t)(br + xr - rr), (int64_t)(be + xe - ee), cnt);
      if (c.purging) purge(S, V, a, b - 1);
      atomicAnd(&S.g[g].fl, ~GF_FIRE);
    }
    return;
  }
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = seg[s], b = seg[s + 1];
    const uint32_t g = keys[a];
    if (!PUSH) {
      if (!(S.g[g].fl & GF_FIRE)) continue;
      if (!emit_firing(c, S, V, g, a, b - 1, room)) continue;
      if (c.purging) purge(S, V, a, b - 1);
      atomicAnd(&S.g[g].fl, ~GF_FIRE);
      continue;
    }
    if (!(S.g[g].fl & GF_TOUCH)) continue;
    int64_t j = prog[s] >= 0 ? prog[s] : a;
    while (j < b && (int64_t)pos[j] < base_new) j++;
    const int64_t mts = w_max_ts(c, S.g[g].start);
    bool stopped = false;
    for (; j < b; j++) {
      bool fire;
      int64_t nc = 0;
      if (c.trigger == FW_TRIGGER_COUNT) {
        nc = S.g[g].cnt + 1;
        fire = nc >= c.trig_n;
      } else {
        fire = mts <= wm;
      }
      if (fire) {
        if (!emit_firing(c, S, V, g, a, j, room)) {
          prog[s] = j;
          stopped = true;
          break;
        }
        if (c.purging) purge(S, V, a, j);
      }
      if (c.trigger == FW_TRIGGER_COUNT) S.g[g].cnt = fire ? 0 : nc;
    }
    if (!stopped) atomicAnd(&S.g[g].fl, ~GF_TOUCH);
  }
}

// an upper bound of the elements one walk can emit: per list, its length times the firings it can see (every
// due list once at a watermark; in a push every new element of an event-time list, or every trig_n-th of a
// CountTrigger list)
template <bool PUSH>
__global__ __launch_bounds__(256) void k_walk_bound(LCfg c, LState S, const uint32_t* __restrict__ pos,
                                                    const uint32_t* __restrict__ keys, const uint32_t* __restrict__ seg,
                                                    int64_t nseg, int64_t base_new) {
  unsigned long long tot = 0;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = seg[s], b = seg[s + 1];
    if (!PUSH) {
      tot += (unsigned long long)(b - a);
      continue;
    }
    int64_t nn = 0;
    for (int64_t q = a; q < b; q++) nn += (int64_t)pos[q] >= base_new;
    const int64_t f = c.trigger == FW_TRIGGER_COUNT ? (S.g[keys[a]].cnt + nn) / max<int64_t>(1, c.trig_n) : nn;
    tot += (unsigned long long)(f * (b - a));
  }
  if (tot) atomicAdd(&S.ctr->count, tot);
}

// The watermark firing of the common apply shape (no evictor, an integer field, contents emitted): every selected
// element is live and every list fires once over all of them, so list s's row is rows_base + s and its contents
// are the elements' list-order positions [a, b) themselves — no reservations.  k_gather_emit writes the contents
// (one 32-byte sector read per element, coalesced writes), then one wave per list reduces them (integer sums wrap
// the same in any order) and writes its row.  Other shapes take k_walk<false>.
__global__ __launch_bounds__(256) void k_gather_emit(LState S, const uint32_t* __restrict__ pos, int64_t m, int64_t ebase) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const LPay p = S.lpay[pos[i]];
    S.ets[ebase + i] = p.ts;
    S.eval[ebase + i] = p.val;
    S.eord[ebase + i] = p.ord;
  }
}
__global__ __launch_bounds__(256) void k_walk_wm_fast(LCfg c, LState S, const uint32_t* __restrict__ pos,
                                                      const uint32_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ seg, int64_t nseg, int64_t rbase,
                                                      int64_t ebase) {
  const int lane = __lane_id();
  const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  unsigned long long killed = 0;
  for (int64_t s = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; s < nseg; s += waves) {
    const int64_t a = seg[s], b = seg[s + 1];
    const uint32_t g = keys[a];
    int64_t is = 0, mn = LMAX, mx = LMIN;
    for (int64_t q = a + lane; q < b; q += 64) {
      const int64_t v = S.eval[ebase + q];
      is = jadd(is, v);
      mn = min(mn, v);
      mx = max(mx, v);
      if (c.purging) {
        S.lgid[pos[q]] = -1;
        killed++;
      }
    }
    for (int o = 32; o; o >>= 1) {  // the wave's reduce
      is = jadd(is, __shfl_xor(is, o, 64));
      mn = min(mn, __shfl_xor(mn, o, 64));
      mx = max(mx, __shfl_xor(mx, o, 64));
    }
    if (lane == 0) {
      const int64_t r = rbase + s;
      S.rkey[r] = S.g[g].key;
      S.rstart[r] = S.g[g].start;
      S.rend[r] = w_end(c, S.g[g].start);
      S.rcnt[r] = b - a;
      S.rsum[r] = c.vt == FW_VAL_I32 ? (int64_t)(int32_t)is : c.vt == FW_VAL_I16 ? (int64_t)(int16_t)is
                : c.vt == FW_VAL_I8 ? (int64_t)(int8_t)is : is;
      S.rmin[r] = mn;
      S.rmax[r] = mx;
      S.rfirst[r] = S.eord[ebase + a];
      S.roff[r] = ebase + a;
    }
  }
  block_add(&S.ctr->dead, killed);
}

// ---------------------------------------------------------------- watermark
__global__ __launch_bounds__(256) void k_lw_due(LCfg c, LState S, int64_t wm) {
  unsigned long long nf = 0, nc = 0;
  long long due = LMAX;  // the remaining groups' earliest timer
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g <= (int64_t)S.gmask;
       g += (int64_t)gridDim.x * blockDim.x) {
    if (S.g[g].st != G_LIVE) continue;
    const int64_t st = S.g[g].start;
    const uint32_t f0 = S.g[g].fl;
    uint32_t f = f0;
    if ((f & GF_TIMER) && w_max_ts(c, st) <= wm) {  // the trigger timer fires (EventTimeTrigger.onEventTime)
      f = (f & ~GF_TIMER) | GF_FIRE;
      nf++;
    }
    const int64_t cl = w_cleanup(c, st);
    if (cl != LMAX && cl <= wm) {  // no cleanup timer is registered at Long.MAX_VALUE (registerCleanupTimer)
      f |= GF_CLEAN;
      nc++;
    } else {
      due = min(due, (long long)((f & GF_TIMER) ? w_max_ts(c, st) : cl));
    }
    if (f != f0) S.g[g].fl = f;
  }
  block_min(&S.ctr->next_due, due);
  block_add(&S.ctr->nfire, nf);
  block_add(&S.ctr->nclean, nc);
}
// clearAllState (:368-385): the cleaned-up groups' elements die, their namespaces become tombstones
__global__ __launch_bounds__(256) void k_lw_clean_log(LState S, int64_t n) {
  unsigned long long killed = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t g = S.lgid[i];
    if (g >= 0 && (S.g[g].fl & GF_CLEAN)) {
      S.lgid[i] = -1;
      killed++;
    }
  }
  if (killed) atomicAdd(&S.ctr->dead, killed);
}
__global__ __launch_bounds__(256) void k_lw_clean_map(LState S) {
  unsigned long long nt = 0;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g <= (int64_t)S.gmask;
       g += (int64_t)gridDim.x * blockDim.x) {
    if (S.g[g].st != G_LIVE) continue;
    const uint32_t f = S.g[g].fl;
    if (f & GF_CLEAN) {
      S.g[g].st = G_TOMB;
      nt++;
    } else if (f & GF_FIRE) {
      S.g[g].fl = f & ~GF_FIRE;  // a due timer of an empty list: nothing to fire
    }
  }
  block_add(&S.ctr->tombs, nt);
  block_add(&S.ctr->live_groups, (unsigned long long)(-(long long)nt));  // (wraps: a subtraction)
}

// ---------------------------------------------------------------- compaction / rebuild
__global__ __launch_bounds__(256) void k_rebuild_map(LCfg c, LState o, LState S, int32_t* __restrict__ remap) {
  unsigned ins = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t g0 = (int64_t)blockIdx.x * blockDim.x; g0 <= (int64_t)o.gmask; g0 += stride) {
    const int64_t g = g0 + threadIdx.x;
    if (g > (int64_t)o.gmask) continue;
    if (o.g[g].st != G_LIVE) {
      remap[g] = -1;
      continue;
    }
    const int32_t ng = g_find_insert(S, o.g[g].key, o.g[g].start, o.g[g].kg, 0, &ins);
    remap[g] = ng;
    if (ng >= 0) {
      S.g[ng].cnt = o.g[g].cnt;
      S.g[ng].fl = o.g[g].fl;
    }
  }
  block_add(&S.ctr->live_groups, ins);
}
__global__ __launch_bounds__(256) void k_alive_flags(const int32_t* __restrict__ gid, int64_t n, uint8_t* __restrict__ f) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    f[i] = gid[i] >= 0;
}
__global__ __launch_bounds__(256) void k_gather_log(LState o, LState S, const uint32_t* __restrict__ idx, int64_t m,
                                                    const int32_t* __restrict__ remap) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t e = idx[i];
    S.lpay[i] = o.lpay[e];
    S.lgid[i] = remap ? remap[o.lgid[e]] : o.lgid[e];
  }
}

// ---------------------------------------------------------------- stats / snapshot / restore
// live lists (groups with a live element) and timers (HeapInternalTimerService: the trigger timer and the
// cleanup timer of a (key, window), one timer when they coincide)
__global__ __launch_bounds__(256) void k_mark_lists(LState S, int64_t n, uint8_t* __restrict__ has) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t g = S.lgid[i];
    if (g >= 0) has[g] = 1;
  }
}
__global__ __launch_bounds__(256) void k_count_state(LCfg c, LState S, const uint8_t* __restrict__ has,
                                                     unsigned long long* out2) {
  unsigned long long lists = 0, timers = 0;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g <= (int64_t)S.gmask;
       g += (int64_t)gridDim.x * blockDim.x) {
    if (S.g[g].st != G_LIVE) continue;
    lists += has[g];
    const int64_t cl = w_cleanup(c, S.g[g].start);
    const bool creg = event_time(c) && cl != LMAX;
    timers += creg ? 1 : 0;
    if ((S.g[g].fl & GF_TIMER) && !(creg && cl == w_max_ts(c, S.g[g].start))) timers++;
  }
  if (lists) atomicAdd(&out2[0], lists);
  if (timers) atomicAdd(&out2[1], timers);
}
__global__ __launch_bounds__(256) void k_kg_flags_log(LState S, int64_t n, int32_t kg, uint8_t* __restrict__ f) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t g = S.lgid[i];
    f[i] = g >= 0 && S.g[g].kg == kg;
  }
}
__global__ __launch_bounds__(256) void k_kg_flags_map(LState S, int32_t kg, uint8_t* __restrict__ f) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g <= (int64_t)S.gmask;
       g += (int64_t)gridDim.x * blockDim.x)
    f[g] = S.g[g].st == G_LIVE && S.g[g].kg == kg;
}
// restore: one thread inserts the lists in order (their count and timer flag), then the elements are appended
__global__ void k_restore_groups(LCfg c, LState S, const int64_t* __restrict__ key, const int64_t* __restrict__ start,
                                 const int64_t* __restrict__ cnt, const int64_t* __restrict__ timer, int64_t n,
                                 int32_t kg, int32_t* __restrict__ gid_out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    unsigned ins = 0;
    const int32_t g = g_find_insert(S, key[i], start[i], kg, 0, &ins);
    if (ins) atomicAdd(&S.ctr->live_groups, 1ull);  // (one thread)
    gid_out[i] = g;
    if (g < 0) continue;
    S.g[g].cnt = cnt[i];
    if (timer[i]) atomicOr(&S.g[g].fl, GF_TIMER);
    atomicMin(&S.ctr->next_due, (long long)(timer[i] ? w_max_ts(c, start[i]) : w_cleanup(c, start[i])));
  }
}
__global__ __launch_bounds__(256) void k_restore_elems(LState S, const int64_t* __restrict__ ts,
                                                       const int64_t* __restrict__ val, const int64_t* __restrict__ ord,
                                                       const int32_t* __restrict__ gid, int64_t n, int64_t base) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    S.lpay[base + i] = LPay{ts[i], val[i], ord[i], 0};
    S.lgid[base + i] = gid[i];
  }
}

// ---------------------------------------------------------------- session windows (f4, merging assigners)
// EventTimeSessionWindows over ListState: EvictingWindowOperator.processElement's merging branch (:110-170; the
// plain WindowOperator's, WindowOperator.java:297-370, is the same without an evictor) with MergingWindowSet.addWindow
// (MergingWindowSet.java:150-225) and TimeWindow.mergeWindows (TimeWindow.java:201-244), onEventTime (:241-286) and
// emitWindowContents (:334-366).
// A live slot of the map is one in-flight window of a key together with its state window's list (MergingWindowSet's
// mapping is one to one, so the window carries its list): GSlot.key / start, wend[] its end, GSlot.cnt its live
// elements, GF_TIMER its trigger timer, whead / wtail its list -- a singly linked list through the log (LPay.pad =
// the next element, -1 at the end) in list order: the state window's list, then the other merged windows' lists in
// HashSet order (AbstractHeapMergingState.mergeNamespaces :67-93 with HeapListState's addAll), then the elements added
// since.  Slots are hashed by the key alone, so a key's windows all lie on its probe chain before the first EMPTY
// slot.  lgid: 0 live, -1 dead (evicted, purged, cleaned up, or dropped late).
// A push sorts its records by key (stable: arrival order within a key), places them in the log in that order, and
// one thread per key processes its elements in order.
constexpr int SL_MAXM = 4;  // in-flight windows one element's window can touch (2: they are >= gap long, disjoint)
__device__ __forceinline__ uint32_t sl_home(int64_t key) { return (uint32_t)fmix64((uint64_t)key ^ 0x5E551045u); }
__device__ __forceinline__ int64_t sl_max_ts(int64_t end) { return jsub(end, 1); }
__device__ __forceinline__ int64_t sl_cleanup(const LCfg& c, int64_t end) {  // WindowOperator.cleanupTime (:637-644)
  const int64_t mx = sl_max_ts(end);
  const int64_t t = jadd(mx, c.lateness);
  return t >= mx ? t : LMAX;
}
// TimeWindow.hashCode = MathUtils.longToIntWithBitMixing(start + end) (TimeWindow.java:102-104, MathUtils.java:177-182),
// then HashMap's bucket spread h ^ (h >>> 16)
__device__ __forceinline__ uint32_t sl_tw_bucket(int64_t start, int64_t end, uint32_t cap) {
  uint64_t in = (uint64_t)jadd(start, end);
  in = (in ^ (in >> 30)) * 0xbf58476d1ce4e5b9ull;
  in = (in ^ (in >> 27)) * 0x94d049bb133111ebull;
  in = in ^ (in >> 31);
  const uint32_t h = (uint32_t)in;
  return (h ^ (h >> 16)) & (cap - 1);
}
__device__ __forceinline__ int64_t sl_timer_of(const LCfg& c, uint32_t fl, int64_t end) {
  return (fl & GF_TIMER) ? sl_max_ts(end) : sl_cleanup(c, end);
}

// a new window slot for key on its chain (from `from`, a TOMB / EMPTY slot the walk met first): claimed with a CAS
// (other threads insert other keys), its fields stored write-through, then LIVE (g_find_insert's publication)
__device__ int32_t sl_insert(const LState& S, int64_t key, int32_t kg, int64_t start, int64_t end, uint32_t from) {
  uint32_t s = from;
  for (uint32_t probes = 0; probes <= S.gmask; probes++, s = (s + 1) & S.gmask) {
    uint32_t cur = __hip_atomic_load(&S.g[s].st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur != G_EMPTY && cur != G_TOMB) continue;
    if (atomicCAS(&S.g[s].st, cur, G_BUSY) != cur) continue;  // (taken meanwhile: it is some key's now)
    __hip_atomic_store(&S.g[s].key, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&S.g[s].start, start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&S.g[s].kg, kg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&S.g[s].cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&S.g[s].fl, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    S.wend[s] = end;
    S.whead[s] = -1;
    S.wtail[s] = -1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&S.g[s].st, (uint32_t)G_LIVE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == G_TOMB) atomicAdd(&S.ctr->tombs, (unsigned long long)-1ll);
    return (int32_t)s;
  }
  atomicOr(&S.ctr->flags, LF_MAP_FULL);
  return -1;
}

// kill element q of a list (unlinked by the caller)
__device__ __forceinline__ void sl_kill(const LState& S, int64_t q, unsigned long long* killed) {
  S.lgid[q] = -1;
  (*killed)++;
}
// the evictor over slot s's list (CountEvictor.evict :63-78, TimeEvictor.evict :67-96, DeltaEvictor.evict :72-80):
// mark = false: how many elements would remain; mark = true: the others are unlinked and killed, the count returned
__device__ int64_t sl_evict(const LCfg& c, const LState& S, int32_t s, bool mark, unsigned long long* killed) {
  const int64_t live = S.g[s].cnt;
  if (c.evictor == FW_EVICT_NONE || live == 0) return live;
  int64_t drop = 0, cutoff = 0, last = 0;
  if (c.evictor == FW_EVICT_COUNT) {
    if (live <= c.ev_n) return live;
    drop = live - c.ev_n;
  } else if (c.evictor == FW_EVICT_TIME) {
    const int64_t h = S.whead[s];
    if (S.lpay[h].ts == LMIN) return live;  // hasTimestamp of the first element
    int64_t mx = LMIN;
    for (int64_t q = h; q >= 0; q = S.lpay[q].pad) mx = max(mx, S.lpay[q].ts);
    cutoff = jsub(mx, c.ev_n);
  } else {
    last = S.lpay[S.wtail[s]].val;
  }
  int64_t removed = 0, prev = -1;
  for (int64_t q = S.whead[s]; q >= 0;) {
    const LPay p = S.lpay[q];
    const bool rm = c.evictor == FW_EVICT_COUNT ? removed < drop
                  : c.evictor == FW_EVICT_TIME  ? p.ts <= cutoff
                                                : delta_of(c, p.val, last) >= c.thr;
    if (rm) {
      removed++;
      if (mark) {
        if (prev < 0)
          S.whead[s] = p.pad;
        else
          S.lpay[prev].pad = p.pad;
        if (S.wtail[s] == q) S.wtail[s] = prev;
        sl_kill(S, q, killed);
      }
    } else {
      prev = q;
    }
    if (c.evictor == FW_EVICT_COUNT && removed >= drop && !mark) break;
    q = p.pad;
  }
  if (mark) S.g[s].cnt = (int32_t)(live - removed);
  return live - removed;
}
// clearing slot s's list (PurgingTrigger's windowState.clear(), clearAllState)
__device__ void sl_clear(const LState& S, int32_t s, unsigned long long* killed) {
  for (int64_t q = S.whead[s]; q >= 0; q = S.lpay[q].pad) sl_kill(S, q, killed);
  S.whead[s] = S.wtail[s] = -1;
  S.g[s].cnt = 0;
}
// emitWindowContents (:334-366) of slot s: evictBefore, one row (+ the elements in list order), evictAfter.
// atomic = false: the host sized rows and elements for every firing (plain reservations); else elements are reserved
// with compare-and-swap against ecap, and false (nothing changed) is returned when they do not fit.
__device__ bool sl_emit(const LCfg& c, const LState& S, int32_t s, bool atomic, unsigned long long* killed) {
  const int64_t cnt = c.evict_after ? (int64_t)S.g[s].cnt : sl_evict(c, S, s, false, killed);
  int64_t eoff = 0;
  if (c.emit && cnt) {
    if (!atomic) {
      eoff = (int64_t)atomicAdd(&S.ctr->elems, (unsigned long long)cnt);
    } else {
      unsigned long long cur = __hip_atomic_load(&S.ctr->elems, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      while (true) {
        if ((int64_t)cur + cnt > S.ecap) {
          atomicOr(&S.ctr->flags, LF_ELEMS);
          return false;
        }
        const unsigned long long prev = atomicCAS(&S.ctr->elems, cur, cur + (unsigned long long)cnt);
        if (prev == cur) break;
        cur = prev;
      }
      eoff = (int64_t)cur;
    }
  }
  if (!c.evict_after) sl_evict(c, S, s, true, killed);
  const bool fl = c.vt == FW_VAL_F64 || c.vt == FW_VAL_F32;
  double ds = 0.0;
  int64_t is = 0, mn = 0, mx = 0, first = -1, k = 0;
  for (int64_t q = S.whead[s]; q >= 0;) {
    const LPay p = S.lpay[q];
    const int64_t v = p.val;
    if (k == 0) first = p.ord;
    if (fl) {
      const double d = __longlong_as_double(v);
      ds = k == 0 ? d : c.vt == FW_VAL_F32 ? (double)((float)ds + (float)d) : ds + d;
      if (k == 0 || fkey(v) < fkey(mn)) mn = v;
      if (k == 0 || fkey(v) > fkey(mx)) mx = v;
    } else {
      is = k == 0 ? v : jadd(is, v);
      if (k == 0 || v < mn) mn = v;
      if (k == 0 || v > mx) mx = v;
    }
    if (c.emit) {
      S.ets[eoff + k] = p.ts;
      S.eval[eoff + k] = v;
      S.eord[eoff + k] = p.ord;
    }
    k++;
    q = p.pad;
  }
  const unsigned long long r = atomicAdd(&S.ctr->rows, 1ull);
  S.rkey[r] = S.g[s].key;
  S.rstart[r] = S.g[s].start;
  S.rend[r] = S.wend[s];
  S.rcnt[r] = k;
  if (fl) {
    S.rsum[r] = __double_as_longlong(ds);
    S.rmin[r] = k ? canon(mn) : 0;
    S.rmax[r] = k ? canon(mx) : 0;
  } else {
    S.rsum[r] = c.vt == FW_VAL_I32 ? (int64_t)(int32_t)is : c.vt == FW_VAL_I16 ? (int64_t)(int16_t)is
              : c.vt == FW_VAL_I8 ? (int64_t)(int8_t)is : is;
    S.rmin[r] = mn;
    S.rmax[r] = mx;
  }
  S.rfirst[r] = first;
  S.roff[r] = c.emit ? eoff : 0;
  if (c.evict_after) sl_evict(c, S, s, true, killed);
  return true;
}

// per record: its key group (errors flagged) and its sort key / payload (the key, the record's index)
__global__ __launch_bounds__(256) void k_sl_keys(LCfg c, LState S, const int64_t* __restrict__ key,
                                                 const int32_t* __restrict__ kh, int64_t n, uint64_t* __restrict__ sk,
                                                 uint32_t* __restrict__ si) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t kg = key_group(key_hash_of(c.key_kind, key[i], kh, i), c.max_par);
    if ((uint32_t)(kg - c.kg0) >= (uint32_t)c.nkg) atomicOr(&S.ctr->flags, LF_KEY_GROUP);
    sk[i] = (uint64_t)key[i];
    si[i] = (uint32_t)i;
  }
}
// the records in key order into the log at base (arrival order within a key), and the first position of each key
__global__ __launch_bounds__(256) void k_sl_place(LState S, const int64_t* __restrict__ ts, const int64_t* __restrict__ val,
                                                  const uint64_t* __restrict__ sk, const uint32_t* __restrict__ si,
                                                  int64_t n, int64_t base, int64_t ord_base, uint8_t* __restrict__ f) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t i = si[p];
    S.lpay[base + p] = LPay{ts[i], val[i], ord_base + (int64_t)i, -1};
    S.lgid[base + p] = 0;
    f[p] = p == 0 || sk[p] != sk[p - 1];
  }
}

// One thread per key: its elements of the push in arrival order, exactly EvictingWindowOperator.processElement's
// merging branch.  prog[r] = the log index of the element whose firing did not fit the element buffer (its window in
// pslot[r]); the host grows the buffer and launches again, which finishes that firing first.  LMAX: the key is done.
__global__ __launch_bounds__(256) void k_sl_process(LCfg c, LState S, const uint32_t* __restrict__ seg, int64_t nruns,
                                                    int64_t base, int64_t wm, const uint64_t* __restrict__ sk,
                                                    const int32_t* __restrict__ kh, const uint32_t* __restrict__ si,
                                                    int64_t* __restrict__ prog, int32_t* __restrict__ pslot) {
  long long due = LMAX;
  unsigned long long killed = 0, late = 0, ins = 0, tombs = 0;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nruns; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t q = prog[r];
    if (q == LMAX) continue;
    const int64_t a = seg[r], b = seg[r + 1];
    const int64_t key = (int64_t)sk[a];
    const int32_t kg = key_group(key_hash_of(c.key_kind, key, kh, (int64_t)si[a]), c.max_par);
    if (q >= 0) {  // a resumed firing: element q's window fires over its list
      const int32_t s = pslot[r];
      if (!sl_emit(c, S, s, true, &killed)) continue;
      if (c.purging) sl_clear(S, s, &killed);
      due = min(due, (long long)sl_timer_of(c, S.g[s].fl, S.wend[s]));
      q++;
    } else {
      q = base + a;
    }
    const uint32_t home = sl_home(key) & S.gmask;
    for (; q < base + b; q++) {
      const LPay e = S.lpay[q];
      const int64_t ws = e.ts, we = jadd(e.ts, c.size);  // EventTimeSessionWindows.assignWindows
      // the key's in-flight windows that intersect [ws, we] (TimeWindow.intersects), and the chain's first free slot
      int32_t m[SL_MAXM];
      int nm = 0;
      uint32_t freeslot = 0xffffffffu, s = home;
      for (uint32_t probes = 0; probes <= S.gmask; probes++, s = (s + 1) & S.gmask) {
        const uint32_t st = __hip_atomic_load(&S.g[s].st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (st == G_EMPTY) {
          if (freeslot == 0xffffffffu) freeslot = s;
          break;
        }
        if (st == G_TOMB) {
          if (freeslot == 0xffffffffu) freeslot = s;
          continue;
        }
        if (st != G_LIVE) continue;  // (BUSY: another key's window being published)
        __atomic_signal_fence(__ATOMIC_ACQUIRE);
        if (ld_l2(&S.g[s].key) != key) continue;
        const int64_t st0 = S.g[s].start, en0 = S.wend[s];
        if (!(st0 <= we && en0 >= ws)) continue;
        if (nm < SL_MAXM) m[nm] = (int32_t)s;
        nm++;
      }
      if (nm > SL_MAXM) {
        atomicOr(&S.ctr->flags, LF_MERGE_WIDE);
        break;
      }
      int32_t actual = -1;
      if (nm == 0) {  // a new window: MergingWindowSet.addWindow maps it to itself
        if (sl_cleanup(c, we) <= wm) {  // isWindowLate -> retireWindow; the element is skipped
          sl_kill(S, q, &killed);
          if (jadd(e.ts, c.lateness) <= wm) {  // isElementLate (:410-418)
            if (c.side_output) {
              const unsigned long long o = atomicAdd(&S.ctr->side, 1ull);
              S.skey[o] = key;
              S.sts[o] = e.ts;
              S.sval[o] = e.val;
            } else {
              late++;
            }
          }
          continue;
        }
        actual = sl_insert(S, key, kg, ws, we, freeslot == 0xffffffffu ? home : freeslot);
        if (actual < 0) break;
        ins++;
      } else {
        // the merge set: the windows met and the new one, in TimeWindow.mergeWindows' order (by start, the new one
        // after windows of an equal start: it was added last before the stable sort), iterated in HashSet order
        int64_t ms[SL_MAXM + 1], me[SL_MAXM + 1];
        int32_t mslot[SL_MAXM + 1];
        int n = 0;
        for (int i = 0; i < nm; i++) {  // insertion sort of the met windows by start
          const int64_t st0 = S.g[m[i]].start;
          int j = n;
          while (j > 0 && ms[j - 1] > st0) {
            ms[j] = ms[j - 1];
            me[j] = me[j - 1];
            mslot[j] = mslot[j - 1];
            j--;
          }
          ms[j] = st0;
          me[j] = S.wend[m[i]];
          mslot[j] = m[i];
          n++;
        }
        {
          int j = n;
          while (j > 0 && ms[j - 1] > ws) {
            ms[j] = ms[j - 1];
            me[j] = me[j - 1];
            mslot[j] = mslot[j - 1];
            j--;
          }
          ms[j] = ws;
          me[j] = we;
          mslot[j] = -1;
          n++;
        }
        int64_t cs = ms[0], ce = me[0];
        for (int i = 1; i < n; i++) ce = max(ce, me[i]);
        (void)cs;
        if (nm == 1 && S.g[m[0]].start <= ws && we <= S.wend[m[0]]) {
          actual = m[0];  // contained: the merge result is the window itself, no merge function
        } else {
          // HashSet<TimeWindow> iteration (capacity 16 for <= 12 members): by bucket, a bucket in insertion order
          uint32_t bk[SL_MAXM + 1];
          for (int i = 0; i < n; i++) bk[i] = sl_tw_bucket(ms[i], me[i], 16u);
          int ord[SL_MAXM + 1];
          for (int i = 0; i < n; i++) ord[i] = i;
          for (int i = 1; i < n; i++) {  // stable insertion sort by bucket
            const int x = ord[i];
            int j = i;
            while (j > 0 && bk[ord[j - 1]] > bk[x]) {
              ord[j] = ord[j - 1];
              j--;
            }
            ord[j] = x;
          }
          // merge function (WindowOperator.java:308-339): the result may not be late
          if (jadd(sl_max_ts(ce), c.lateness) <= wm) {
            atomicOr(&S.ctr->flags, LF_MERGE_LATE);
            break;
          }
          int32_t target = -1;
          for (int oi = 0; oi < n; oi++) {
            const int32_t sl = mslot[ord[oi]];
            if (sl < 0) continue;  // (the new window: removed from the merge set)
            if (target < 0) {
              target = sl;  // the state window of the first merged window
              continue;
            }
            // mergeNamespaces: the source's list appended to the target's; the source window leaves
            if (S.whead[sl] >= 0) {
              if (S.wtail[target] >= 0)
                S.lpay[S.wtail[target]].pad = S.whead[sl];
              else
                S.whead[target] = S.whead[sl];
              S.wtail[target] = S.wtail[sl];
              S.g[target].cnt += S.g[sl].cnt;
            }
            __hip_atomic_store(&S.g[sl].st, (uint32_t)G_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            tombs++;
          }
          int64_t lo = LMAX;
          for (int i = 0; i < n; i++) lo = min(lo, ms[i]);
          S.g[target].start = lo;
          S.wend[target] = ce;
          S.g[target].fl |= GF_TIMER;  // EventTimeTrigger.onMerge registers the merged window's maxTimestamp
          actual = target;
        }
      }
      // windowState.add(element): appended to the list
      if (S.wtail[actual] >= 0)
        S.lpay[S.wtail[actual]].pad = q;
      else
        S.whead[actual] = q;
      S.wtail[actual] = q;
      S.g[actual].cnt++;
      // EventTimeTrigger.onElement: FIRE when the window's maxTimestamp is not after the watermark
      if (sl_max_ts(S.wend[actual]) <= wm) {
        if (!sl_emit(c, S, actual, true, &killed)) {
          prog[r] = q;
          pslot[r] = actual;
          break;
        }
        if (c.purging) sl_clear(S, actual, &killed);
      } else {
        S.g[actual].fl |= GF_TIMER;
      }
      due = min(due, (long long)sl_timer_of(c, S.g[actual].fl, S.wend[actual]));
    }
    if (q >= base + b) prog[r] = LMAX;
  }
  block_min(&S.ctr->next_due, due);
  block_add(&S.ctr->dead, killed);
  block_add(&S.ctr->late, late);
  block_add(&S.ctr->live_groups, ins - tombs);  // (wraps: a net change)
  block_add(&S.ctr->tombs, tombs);
}

// watermark: each live window whose trigger timer (maxTimestamp) or cleanup timer is due; the firing ones' list
// lengths added up (the element buffer's bound)
__global__ __launch_bounds__(256) void k_sl_due(LCfg c, LState S, int64_t wm) {
  unsigned long long nf = 0, nc = 0, ne = 0;
  long long due = LMAX;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g <= (int64_t)S.gmask;
       g += (int64_t)gridDim.x * blockDim.x) {
    if (S.g[g].st != G_LIVE) continue;
    const int64_t end = S.wend[g];
    const uint32_t f0 = S.g[g].fl;
    uint32_t f = f0;
    if ((f & GF_TIMER) && sl_max_ts(end) <= wm) {  // EventTimeTrigger.onEventTime: FIRE
      f = (f & ~GF_TIMER) | GF_FIRE;
      nf++;
      ne += (unsigned long long)S.g[g].cnt;
    }
    const int64_t cl = sl_cleanup(c, end);
    if (cl != LMAX && cl <= wm) {
      f |= GF_CLEAN;
      nc++;
    } else {
      due = min(due, (long long)((f & GF_TIMER) ? sl_max_ts(end) : cl));
    }
    if (f != f0) S.g[g].fl = f;
  }
  block_min(&S.ctr->next_due, due);
  block_add(&S.ctr->nfire, nf);
  block_add(&S.ctr->nclean, nc);
  block_add(&S.ctr->count, ne);
}
// the due windows: onEventTime (:241-286) -- contents != null: emitWindowContents; PURGE: clear; cleanup time:
// clearAllState and the window leaves its MergingWindowSet (a tombstone)
__global__ __launch_bounds__(256) void k_sl_fire(LCfg c, LState S) {
  unsigned long long killed = 0, nt = 0;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g <= (int64_t)S.gmask;
       g += (int64_t)gridDim.x * blockDim.x) {
    if (S.g[g].st != G_LIVE) continue;
    const uint32_t f = S.g[g].fl;
    if (!(f & (GF_FIRE | GF_CLEAN))) continue;
    if (f & GF_FIRE) {
      if (S.g[g].cnt > 0) {
        sl_emit(c, S, (int32_t)g, false, &killed);
        if (c.purging) sl_clear(S, (int32_t)g, &killed);
      }
      S.g[g].fl = f & ~GF_FIRE;
    }
    if (f & GF_CLEAN) {
      sl_clear(S, (int32_t)g, &killed);
      S.g[g].st = G_TOMB;
      nt++;
    }
  }
  block_add(&S.ctr->dead, killed);
  block_add(&S.ctr->tombs, nt);
  block_add(&S.ctr->live_groups, (unsigned long long)(-(long long)nt));
}

// compaction: the live elements' new positions, the log gathered with its links remapped, the lists' ends remapped
__global__ __launch_bounds__(256) void k_sl_remap_set(const uint32_t* __restrict__ sel, int64_t m,
                                                      int64_t* __restrict__ remap) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
    remap[sel[i]] = i;
}
__global__ __launch_bounds__(256) void k_sl_gather_log(LState o, LState S, const uint32_t* __restrict__ sel, int64_t m,
                                                       const int64_t* __restrict__ remap) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    LPay p = o.lpay[sel[i]];
    p.pad = p.pad >= 0 ? remap[p.pad] : -1;
    S.lpay[i] = p;
    S.lgid[i] = 0;
  }
}
// the map rebuilt into S (another capacity, no tombstones); remap: the log's remap of the list ends (or null)
__global__ __launch_bounds__(256) void k_sl_rebuild(LState o, LState S, const int64_t* __restrict__ remap) {
  unsigned long long ins = 0;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g <= (int64_t)o.gmask;
       g += (int64_t)gridDim.x * blockDim.x) {
    if (o.g[g].st != G_LIVE) continue;
    const int64_t key = o.g[g].key;
    const int32_t s = sl_insert(S, key, o.g[g].kg, o.g[g].start, o.wend[g], sl_home(key) & S.gmask);
    if (s < 0) continue;
    S.g[s].fl = o.g[g].fl;
    S.g[s].cnt = o.g[g].cnt;
    const int64_t h = o.whead[g], t = o.wtail[g];
    S.whead[s] = h >= 0 && remap ? remap[h] : h;
    S.wtail[s] = t >= 0 && remap ? remap[t] : t;
    ins++;
  }
  block_add(&S.ctr->live_groups, ins);
}
// live lists (windows with elements) and timers: each window's cleanup timer, and its trigger timer when registered
// and not at the same time (HeapInternalTimerService keeps one timer per (timestamp, key, window))
__global__ __launch_bounds__(256) void k_sl_count_state(LCfg c, LState S, unsigned long long* out2) {
  unsigned long long lists = 0, timers = 0;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g <= (int64_t)S.gmask;
       g += (int64_t)gridDim.x * blockDim.x) {
    if (S.g[g].st != G_LIVE) continue;
    lists += S.g[g].cnt > 0;
    const int64_t cl = sl_cleanup(c, S.wend[g]);
    timers += cl != LMAX;
    if ((S.g[g].fl & GF_TIMER) && !(cl != LMAX && cl == sl_max_ts(S.wend[g]))) timers++;
  }
  if (lists) atomicAdd(&out2[0], lists);
  if (timers) atomicAdd(&out2[1], timers);
}

unsigned grid_for(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>(8192, (n + 255) / 256)); }

template <class T>
hipError_t dmalloc(T** p, size_t count) {
  *p = nullptr;
  return hipMalloc((void**)p, std::max<size_t>(count, 1) * sizeof(T));
}
template <class T>
void dfree(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

}  // namespace

struct fw_list {
  fw_list_config cfg{};
  LCfg c{};
  LState S{};
  hipStream_t stream = nullptr;
  int device = 0;
  std::string err;
  int64_t gcap = 0, lcap = 0, rcap = 0, scap = 0, max_batch = 0;
  int64_t n_log = 0, ord_base = 0, wm = LMIN, records_in = 0, fired_total = 0, grows = 0;
  LCounters* h_ctr = nullptr;  // pinned mirror
  // per-push scratch (max_batch) and selection scratch (grown with the log)
  int64_t *in_key = nullptr, *in_ts = nullptr, *in_val = nullptr;
  int32_t* in_kh = nullptr;
  uint32_t *wcnt = nullptr, *woff = nullptr;
  int64_t sel_cap = 0;
  uint8_t* flags8 = nullptr;
  uint32_t *sel = nullptr, *sel2 = nullptr, *keys = nullptr, *keys2 = nullptr, *seg = nullptr;
  int64_t *gts = nullptr, *gval = nullptr, *gord = nullptr;  // the walk's gathered view (LView)
  uint8_t* galive = nullptr;
  int64_t* prog = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  // session windows (FW_SESSION): the push's records sorted by key, and the per-key progress of k_sl_process
  uint64_t *sk = nullptr, *sk2 = nullptr;
  uint32_t *si = nullptr, *si2 = nullptr;
  int64_t* sprog = nullptr;
  int32_t* pslot = nullptr;
};

namespace {

int set_err(fw_list* op, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (op) op->err = buf;
  return code;
}
#define LHIP(op, expr)                                                                                   \
  do {                                                                                                   \
    hipError_t _e = (expr);                                                                              \
    if (_e != hipSuccess) return set_err(op, FW_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(_e)); \
  } while (0)
#define LRET(expr)          \
  do {                      \
    int _r = (expr);        \
    if (_r != FW_OK) return _r; \
  } while (0)

int read_ctr(fw_list* op) {
  LHIP(op, hipMemcpyAsync(op->h_ctr, op->S.ctr, sizeof(LCounters), hipMemcpyDeviceToHost, op->stream));
  LHIP(op, hipStreamSynchronize(op->stream));
  return FW_OK;
}
int ensure_tmp(fw_list* op, size_t bytes) {
  if (bytes <= op->tmp_bytes) return FW_OK;
  dfree(op->tmp);
  op->tmp_bytes = std::max(bytes, op->tmp_bytes * 2);
  LHIP(op, dmalloc((uint8_t**)&op->tmp, op->tmp_bytes));
  return FW_OK;
}
int alloc_map(fw_list* op, LState& S, int64_t cap) {
  LHIP(op, dmalloc(&S.g, (size_t)cap));
  LHIP(op, hipMemsetAsync(S.g, 0, (size_t)cap * sizeof(GSlot), op->stream));  // G_EMPTY
  S.gmask = (uint32_t)(cap - 1);
  return FW_OK;
}
void free_map(LState& S) {
  dfree(S.g);
}
int alloc_log(fw_list* op, LState& S, int64_t cap) {
  LHIP(op, dmalloc(&S.lpay, (size_t)cap));
  LHIP(op, dmalloc(&S.lgid, (size_t)cap));
  return FW_OK;
}
void free_log(LState& S) {
  dfree(S.lpay);
  dfree(S.lgid);
}
int ensure_sel(fw_list* op, int64_t n) {
  if (n <= op->sel_cap) return FW_OK;
  const int64_t cap = std::max<int64_t>(n, op->sel_cap * 2);
  dfree(op->flags8);
  dfree(op->sel);
  dfree(op->sel2);
  dfree(op->keys);
  dfree(op->keys2);
  dfree(op->seg);
  dfree(op->prog);
  dfree(op->gts);
  dfree(op->gval);
  dfree(op->gord);
  dfree(op->galive);
  LHIP(op, dmalloc(&op->gts, (size_t)cap));
  LHIP(op, dmalloc(&op->gval, (size_t)cap));
  LHIP(op, dmalloc(&op->gord, (size_t)cap));
  LHIP(op, dmalloc(&op->galive, (size_t)cap));
  LHIP(op, dmalloc(&op->flags8, (size_t)cap));
  LHIP(op, dmalloc(&op->sel, (size_t)cap));
  LHIP(op, dmalloc(&op->sel2, (size_t)cap));
  LHIP(op, dmalloc(&op->keys, (size_t)cap));
  LHIP(op, dmalloc(&op->keys2, (size_t)cap));
  LHIP(op, dmalloc(&op->seg, (size_t)cap + 1));
  LHIP(op, dmalloc(&op->prog, (size_t)cap));
  op->sel_cap = cap;
  return FW_OK;
}
// grows a row / element column set, keeping the first `keep` values
int grow_cols(fw_list* op, int64_t** cols[], int ncol, int64_t old_cap, int64_t cap, int64_t keep) {
  for (int i = 0; i < ncol; i++) {
    int64_t* n = nullptr;
    LHIP(op, dmalloc(&n, (size_t)cap));
    if (keep) LHIP(op, hipMemcpyAsync(n, *cols[i], (size_t)keep * 8, hipMemcpyDeviceToDevice, op->stream));
    LHIP(op, hipStreamSynchronize(op->stream));
    dfree(*cols[i]);
    *cols[i] = n;
  }
  (void)old_cap;
  return FW_OK;
}
int ensure_rows(fw_list* op, int64_t need) {
  if (need <= op->rcap) return FW_OK;
  const int64_t cap = std::max<int64_t>(need, op->rcap * 2);
  int64_t** cols[] = {&op->S.rkey, &op->S.rstart, &op->S.rend, &op->S.rcnt, &op->S.rsum, &op->S.rmin,
                      &op->S.rmax, &op->S.rfirst, &op->S.roff};
  LRET(grow_cols(op, cols, 9, op->rcap, cap, (int64_t)op->h_ctr->rows));
  op->rcap = cap;
  return FW_OK;
}
int ensure_elems(fw_list* op, int64_t need) {
  if (need <= op->S.ecap) return FW_OK;
  const int64_t cap = std::max<int64_t>(need, op->S.ecap * 2);
  int64_t** cols[] = {&op->S.ets, &op->S.eval, &op->S.eord};
  LRET(grow_cols(op, cols, 3, op->S.ecap, cap, (int64_t)op->h_ctr->elems));
  op->S.ecap = cap;
  return FW_OK;
}
int ensure_side(fw_list* op, int64_t need) {
  if (need <= op->scap) return FW_OK;
  const int64_t cap = std::max<int64_t>(need, op->scap * 2);
  int64_t** cols[] = {&op->S.skey, &op->S.sts, &op->S.sval};
  LRET(grow_cols(op, cols, 3, op->scap, cap, (int64_t)op->h_ctr->side));
  op->scap = cap;
  return FW_OK;
}

// stable selection of the log positions whose flag is set: sel[0 .. *m)
int select_positions(fw_list* op, const uint8_t* flags, int64_t n, uint32_t* out, int64_t* m) {
  rocprim::counting_iterator<uint32_t> it(0);
  unsigned long long* d_cnt = &op->S.ctr->count;
  size_t bytes = 0;
  LHIP(op, rocprim::select(nullptr, bytes, it, flags, out, d_cnt, (size_t)n, op->stream));
  LRET(ensure_tmp(op, bytes));
  bytes = op->tmp_bytes;
  LHIP(op, rocprim::select(op->tmp, bytes, it, flags, out, d_cnt, (size_t)n, op->stream));
  LRET(read_ctr(op));
  *m = (int64_t)op->h_ctr->count;
  return FW_OK;
}

// the live elements of the groups flagged `bit`, grouped by list (a stable radix sort by group keeps list
// order), then one walk over them; relaunched with a larger element buffer until every list is done
template <bool PUSH>
int walk_lists(fw_list* op, uint32_t bit, int64_t base_new) {
  LRET(ensure_sel(op, op->n_log));
  hipLaunchKernelGGL(k_sel_flags, dim3(grid_for(op->n_log)), dim3(256), 0, op->stream, op->S, op->n_log, bit,
                     op->flags8);
  int64_t m = 0;
  LRET(select_positions(op, op->flags8, op->n_log, op->sel, &m));
  if (m == 0) return FW_OK;
  hipLaunchKernelGGL(k_sel_keys, dim3(grid_for(m)), dim3(256), 0, op->stream, op->S, op->sel, m, op->keys);
  int bits = 1;
  while (((int64_t)1 << bits) <= (int64_t)op->S.gmask) bits++;
  size_t bytes = 0;
  LHIP(op, rocprim::radix_sort_pairs(nullptr, bytes, op->keys, op->keys2, op->sel, op->sel2, (size_t)m, 0, bits,
                                     op->stream));
  LRET(ensure_tmp(op, bytes));
  bytes = op->tmp_bytes;
  LHIP(op, rocprim::radix_sort_pairs(op->tmp, bytes, op->keys, op->keys2, op->sel, op->sel2, (size_t)m, 0, bits,
                                     op->stream));
  hipLaunchKernelGGL(k_seg_flags, dim3(grid_for(m)), dim3(256), 0, op->stream, op->keys2, m, op->flags8);
  int64_t nseg = 0;
  LRET(select_positions(op, op->flags8, m, op->seg, &nseg));
  const uint32_t mm = (uint32_t)m;
  LHIP(op, hipMemcpyAsync(op->seg + nseg, &mm, 4, hipMemcpyHostToDevice, op->stream));
  LHIP(op, hipMemsetAsync(op->prog, 0xff, (size_t)nseg * 8, op->stream));

  // with room for every possible firing the walk reserves elements with plain atomics; else (a bound beyond
  // FW_LIST_ROOM elements) it reserves with compare-and-swap and stops where the buffer is full
  bool room = !op->c.emit;
  if (op->c.emit) {
    LHIP(op, hipMemsetAsync(&op->S.ctr->count, 0, 8, op->stream));
    hipLaunchKernelGGL(k_walk_bound<PUSH>, dim3(grid_for(nseg)), dim3(256), 0, op->stream, op->c, op->S, op->sel2,
                       op->keys2, op->seg, nseg, base_new);
    LRET(read_ctr(op));
    const int64_t need = (int64_t)op->h_ctr->elems + (int64_t)op->h_ctr->count;
    if ((int64_t)op->h_ctr->count <= FW_LIST_ROOM) {
      LRET(ensure_elems(op, need));
      room = true;
    }
  }
  const bool fl = op->c.vt == FW_VAL_F64 || op->c.vt == FW_VAL_F32;
  if (!PUSH && room && op->c.emit && op->c.evictor == FW_EVICT_NONE && !fl) {  // the common apply shape
    LRET(read_ctr(op));
    const int64_t rbase = (int64_t)op->h_ctr->rows, ebase = (int64_t)op->h_ctr->elems;
    hipLaunchKernelGGL(k_gather_emit, dim3(grid_for(m)), dim3(256), 0, op->stream, op->S, op->sel2, m, ebase);
    hipLaunchKernelGGL(k_walk_wm_fast, dim3((unsigned)std::min<int64_t>(16384, (nseg + 3) / 4)), dim3(256), 0,
                       op->stream, op->c, op->S, op->sel2, op->keys2, op->seg, nseg, rbase, ebase);
    LHIP(op, hipGetLastError());
    const unsigned long long re[2] = {(unsigned long long)(rbase + nseg), (unsigned long long)(ebase + m)};
    LHIP(op, hipMemcpyAsync(&op->S.ctr->rows, re, 16, hipMemcpyHostToDevice, op->stream));  // rows, elems
    return read_ctr(op);
  }
  hipLaunchKernelGGL(k_gather_sel, dim3(grid_for(m)), dim3(256), 0, op->stream, op->S, op->sel2, m, op->gts, op->gval,
                     op->gord, op->galive);
  const LView V{op->sel2, op->gts, op->gval, op->gord, op->galive, op->S.lgid};
  for (int round = 0;; round++) {
    LHIP(op, hipMemsetAsync(&op->S.ctr->flags, 0, 4, op->stream));
    hipLaunchKernelGGL(k_walk<PUSH>, dim3(grid_for(nseg)), dim3(256), 0, op->stream, op->c, op->S, V, op->keys2,
                       op->seg, nseg, base_new, op->wm, op->prog, room);
    LHIP(op, hipGetLastError());
    LRET(read_ctr(op));
    if (!(op->h_ctr->flags & LF_ELEMS)) break;
    if (round > 64) return set_err(op, FW_ERR_STATE, "list walk made no progress");
    LRET(ensure_elems(op, op->S.ecap * 2));
  }
  return FW_OK;
}

// drops dead elements (stable) and tombstones; the map grows to hold `groups_needed` at <= 1/2 load
int compact(fw_list* op, int64_t groups_needed) {
  LState o = op->S, S = op->S;
  int64_t gcap = op->gcap;
  while (gcap < 2 * groups_needed) gcap *= 2;
  LRET(alloc_map(op, S, gcap));
  int32_t* remap = nullptr;
  LHIP(op, dmalloc(&remap, (size_t)op->gcap));
  LHIP(op, hipMemsetAsync(&op->S.ctr->live_groups, 0, 8, op->stream));
  LHIP(op, hipMemsetAsync(&op->S.ctr->tombs, 0, 8, op->stream));
  LHIP(op, hipMemsetAsync(&op->S.ctr->flags, 0, 4, op->stream));  // (a full map's flag is what called us)
  hipLaunchKernelGGL(k_rebuild_map, dim3(grid_for(op->gcap)), dim3(256), 0, op->stream, op->c, o, S, remap);
  // the live elements, in order, remapped
  LRET(ensure_sel(op, op->n_log));
  hipLaunchKernelGGL(k_alive_flags, dim3(grid_for(op->n_log)), dim3(256), 0, op->stream, o.lgid, op->n_log, op->flags8);
  int64_t m = 0;
  LRET(select_positions(op, op->flags8, op->n_log, op->sel, &m));
  LState L = S;
  LRET(alloc_log(op, L, op->lcap));
  hipLaunchKernelGGL(k_gather_log, dim3(grid_for(m)), dim3(256), 0, op->stream, o, L, op->sel, m, remap);
  LHIP(op, hipStreamSynchronize(op->stream));
  dfree(remap);
  free_map(o);
  free_log(o);
  op->S = L;
  op->gcap = gcap;
  op->n_log = m;
  LHIP(op, hipMemsetAsync(&op->S.ctr->dead, 0, 8, op->stream));
  LRET(read_ctr(op));
  if (op->h_ctr->flags & LF_MAP_FULL) return set_err(op, FW_ERR_CAPACITY, "list state map full");
  op->grows++;
  return FW_OK;
}

// room for `extra` more log entries: compaction when dead entries are the majority, else a larger log
int grow_log(fw_list* op, int64_t extra) {
  if (op->n_log + extra <= op->lcap) return FW_OK;
  if (2 * (int64_t)op->h_ctr->dead > op->n_log) {
    LRET(compact(op, (int64_t)op->h_ctr->live_groups));
    if (op->n_log + extra <= op->lcap) return FW_OK;
  }
  const int64_t cap = std::max<int64_t>(op->n_log + extra, op->lcap * 2);
  LState L = op->S;
  LRET(alloc_log(op, L, cap));
  if (op->n_log) {
    LHIP(op, hipMemcpyAsync(L.lpay, op->S.lpay, (size_t)op->n_log * sizeof(LPay), hipMemcpyDeviceToDevice,
                            op->stream));
    LHIP(op, hipMemcpyAsync(L.lgid, op->S.lgid, (size_t)op->n_log * 4, hipMemcpyDeviceToDevice, op->stream));
  }
  LHIP(op, hipStreamSynchronize(op->stream));
  free_log(op->S);
  op->S.lpay = L.lpay;
  op->S.lgid = L.lgid;
  op->lcap = cap;
  op->grows++;
  return FW_OK;
}

int maybe_compact(fw_list* op) {
  const int64_t dead = (int64_t)op->h_ctr->dead, tombs = (int64_t)op->h_ctr->tombs;
  if ((dead > (1 << 16) && 2 * dead > op->n_log) || 4 * tombs > op->gcap)
    return compact(op, (int64_t)op->h_ctr->live_groups);
  return FW_OK;
}

// ---------------------------------------------------------------- session windows (host)
bool sessions(const fw_list* op) { return op->c.assigner == FW_SESSION; }
int sl_alloc_map(fw_list* op, LState& S, int64_t cap) {
  LRET(alloc_map(op, S, cap));
  LHIP(op, dmalloc(&S.wend, (size_t)cap));
  LHIP(op, dmalloc(&S.whead, (size_t)cap));
  LHIP(op, dmalloc(&S.wtail, (size_t)cap));
  return FW_OK;
}
void sl_free_map(LState& S) {
  free_map(S);
  dfree(S.wend);
  dfree(S.whead);
  dfree(S.wtail);
}
// the map rebuilt at gcap slots (tombstones dropped); with `log`, the log compacted first (the live elements in
// order, their links and the lists' ends remapped)
int sl_compact(fw_list* op, int64_t gcap, bool log) {
  LState o = op->S, S = op->S;
  int64_t* remap = nullptr;
  int64_t m = op->n_log;
  if (log && op->n_log) {
    LRET(ensure_sel(op, op->n_log));
    hipLaunchKernelGGL(k_alive_flags, dim3(grid_for(op->n_log)), dim3(256), 0, op->stream, o.lgid, op->n_log,
                       op->flags8);
    LRET(select_positions(op, op->flags8, op->n_log, op->sel, &m));
    LHIP(op, dmalloc(&remap, (size_t)op->n_log));
    LHIP(op, hipMemsetAsync(remap, 0xff, (size_t)op->n_log * 8, op->stream));
    hipLaunchKernelGGL(k_sl_remap_set, dim3(grid_for(m)), dim3(256), 0, op->stream, op->sel, m, remap);
    LState L = S;
    LRET(alloc_log(op, L, op->lcap));
    hipLaunchKernelGGL(k_sl_gather_log, dim3(grid_for(m)), dim3(256), 0, op->stream, o, L, op->sel, m, remap);
    S.lpay = L.lpay;
    S.lgid = L.lgid;
  }
  LRET(sl_alloc_map(op, S, gcap));
  LHIP(op, hipMemsetAsync(&op->S.ctr->live_groups, 0, 16, op->stream));  // live_groups, tombs
  LHIP(op, hipMemsetAsync(&op->S.ctr->flags, 0, 4, op->stream));
  hipLaunchKernelGGL(k_sl_rebuild, dim3(grid_for(op->gcap)), dim3(256), 0, op->stream, o, S, remap);
  LHIP(op, hipGetLastError());
  LHIP(op, hipStreamSynchronize(op->stream));
  dfree(remap);
  sl_free_map(o);
  if (log && op->n_log) {
    free_log(o);
    op->n_log = m;
    LHIP(op, hipMemsetAsync(&S.ctr->dead, 0, 8, op->stream));
  }
  op->S = S;
  op->gcap = gcap;
  op->grows++;
  LRET(read_ctr(op));
  if (op->h_ctr->flags & LF_MAP_FULL) return set_err(op, FW_ERR_CAPACITY, "list state map full");
  return FW_OK;
}
int sl_maybe_compact(fw_list* op) {
  const int64_t dead = (int64_t)op->h_ctr->dead, tombs = (int64_t)op->h_ctr->tombs;
  const bool log = dead > (1 << 16) && 2 * dead > op->n_log;
  if (log || 4 * tombs > op->gcap) return sl_compact(op, op->gcap, log);
  return FW_OK;
}
int sl_check_flags(fw_list* op) {
  const uint32_t f = op->h_ctr->flags;
  if (f & LF_KEY_GROUP) return set_err(op, FW_ERR_KEY_GROUP, "a key of the batch is outside the handle's KeyGroupRange");
  if (f & LF_MERGE_LATE)
    return set_err(op, FW_ERR_UNSUPPORTED, "The end timestamp of an event-time window cannot become earlier than the "
                                           "current watermark by merging.");
  if (f & LF_MERGE_WIDE) return set_err(op, FW_ERR_STATE, "a session window met more than %d in-flight windows", SL_MAXM);
  if (f & LF_MAP_FULL) return set_err(op, FW_ERR_CAPACITY, "list state map full");
  return FW_OK;
}
// processElement for a batch of session-window records (EvictingWindowOperator.java:110-170)
int sl_push(fw_list* op, const int64_t* key, const int64_t* ts, const int64_t* val, const int32_t* kh, int64_t n) {
  LRET(read_ctr(op));
  if (op->c.side_output) LRET(ensure_side(op, (int64_t)op->h_ctr->side + n));
  // the map: every record may open a window; at most 3/4 of the slots live or tombstones during the push
  const int64_t live = (int64_t)op->h_ctr->live_groups, tombs = (int64_t)op->h_ctr->tombs;
  if (4 * (live + tombs + n) > 3 * op->gcap) {
    int64_t g = op->gcap;
    while (2 * (live + n) > g) g *= 2;
    LRET(sl_compact(op, g, 2 * (int64_t)op->h_ctr->dead > op->n_log));
  }
  // the log: the batch is appended
  if (op->n_log + n > op->lcap) {
    if (2 * (int64_t)op->h_ctr->dead > op->n_log) LRET(sl_compact(op, op->gcap, true));
    if (op->n_log + n > op->lcap) {
      const int64_t cap = std::max<int64_t>(op->n_log + n, op->lcap * 2);
      LState L = op->S;
      LRET(alloc_log(op, L, cap));
      if (op->n_log) {
        LHIP(op, hipMemcpyAsync(L.lpay, op->S.lpay, (size_t)op->n_log * sizeof(LPay), hipMemcpyDeviceToDevice,
                                op->stream));
        LHIP(op, hipMemcpyAsync(L.lgid, op->S.lgid, (size_t)op->n_log * 4, hipMemcpyDeviceToDevice, op->stream));
      }
      LHIP(op, hipStreamSynchronize(op->stream));
      free_log(op->S);
      op->S.lpay = L.lpay;
      op->S.lgid = L.lgid;
      op->lcap = cap;
      op->grows++;
    }
  }
  LRET(ensure_rows(op, (int64_t)op->h_ctr->rows + n));  // (at most one firing per element)
  LRET(ensure_sel(op, n));
  LHIP(op, hipMemsetAsync(&op->S.ctr->flags, 0, 8, op->stream));  // flags, need_seq
  hipLaunchKernelGGL(k_sl_keys, dim3(grid_for(n)), dim3(256), 0, op->stream, op->c, op->S, key, kh, n, op->sk, op->si);
  size_t bytes = 0;
  LHIP(op, rocprim::radix_sort_pairs(nullptr, bytes, op->sk, op->sk2, op->si, op->si2, (size_t)n, 0, 64, op->stream));
  LRET(ensure_tmp(op, bytes));
  bytes = op->tmp_bytes;
  LHIP(op, rocprim::radix_sort_pairs(op->tmp, bytes, op->sk, op->sk2, op->si, op->si2, (size_t)n, 0, 64, op->stream));
  const int64_t base = op->n_log;
  hipLaunchKernelGGL(k_sl_place, dim3(grid_for(n)), dim3(256), 0, op->stream, op->S, ts, val, op->sk2, op->si2, n, base,
                     op->ord_base, op->flags8);
  int64_t nruns = 0;
  LRET(select_positions(op, op->flags8, n, op->seg, &nruns));  // (reads the counters: flags are current)
  LRET(sl_check_flags(op));
  const uint32_t nn = (uint32_t)n;
  LHIP(op, hipMemcpyAsync(op->seg + nruns, &nn, 4, hipMemcpyHostToDevice, op->stream));
  LHIP(op, hipMemsetAsync(op->sprog, 0xff, (size_t)nruns * 8, op->stream));
  for (int round = 0;; round++) {
    LHIP(op, hipMemsetAsync(&op->S.ctr->flags, 0, 4, op->stream));
    hipLaunchKernelGGL(k_sl_process, dim3(grid_for(nruns)), dim3(256), 0, op->stream, op->c, op->S, op->seg, nruns,
                       base, op->wm, op->sk2, kh, op->si2, op->sprog, op->pslot);
    LHIP(op, hipGetLastError());
    LRET(read_ctr(op));
    LRET(sl_check_flags(op));
    if (!(op->h_ctr->flags & LF_ELEMS)) break;
    if (round > 64) return set_err(op, FW_ERR_STATE, "session list push made no progress");
    LRET(ensure_elems(op, op->S.ecap * 2));
  }
  op->n_log += n;
  op->ord_base += n;
  op->records_in += n;
  return sl_maybe_compact(op);
}
// processWatermark: the due windows fire and the cleaned-up ones leave (EvictingWindowOperator.onEventTime)
int sl_watermark(fw_list* op, int64_t wm) {
  LHIP(op, hipMemsetAsync(&op->S.ctr->nfire, 0, 24, op->stream));  // nfire, nclean, count
  hipLaunchKernelGGL(k_sl_due, dim3(grid_for(op->gcap)), dim3(256), 0, op->stream, op->c, op->S, wm);
  LRET(read_ctr(op));
  const int64_t nfire = (int64_t)op->h_ctr->nfire, nclean = (int64_t)op->h_ctr->nclean;
  if (!nfire && !nclean) return FW_OK;
  LRET(ensure_rows(op, (int64_t)op->h_ctr->rows + nfire));
  if (op->c.emit) LRET(ensure_elems(op, (int64_t)op->h_ctr->elems + (int64_t)op->h_ctr->count));
  hipLaunchKernelGGL(k_sl_fire, dim3(grid_for(op->gcap)), dim3(256), 0, op->stream, op->c, op->S);
  LHIP(op, hipGetLastError());
  LRET(read_ctr(op));
  return sl_maybe_compact(op);
}

int push_device(fw_list* op, const int64_t* key, const int64_t* ts, const int64_t* val, const int32_t* kh, int64_t n) {
  if (n == 0) return FW_OK;
  if (n > op->max_batch) return set_err(op, FW_ERR_ARG, "batch of %lld records exceeds max_batch %lld", (long long)n,
                                        (long long)op->max_batch);
  if (op->cfg.key_kind == FW_KEY_HASHED && !kh) return set_err(op, FW_ERR_ARG, "key_hash required for FW_KEY_HASHED");
  if (sessions(op)) return sl_push(op, key, ts, val, kh, n);
  if (op->c.side_output) {  // room for every record of the batch in the side output
    LRET(read_ctr(op));
    LRET(ensure_side(op, (int64_t)op->h_ctr->side + n));
  }
  LHIP(op, hipMemsetAsync(&op->S.ctr->flags, 0, 8, op->stream));  // flags, need_seq
  hipLaunchKernelGGL(k_lp_count, dim3(grid_for(n)), dim3(256), 0, op->stream, op->c, op->S, key, ts, val, kh, n, op->wm,
                     op->wcnt);
  size_t bytes = 0;
  LHIP(op, rocprim::inclusive_scan(nullptr, bytes, op->wcnt, op->woff + 1, (size_t)n, rocprim::plus<uint32_t>(),
                                   op->stream));
  LRET(ensure_tmp(op, bytes));
  bytes = op->tmp_bytes;
  LHIP(op, hipMemsetAsync(op->woff, 0, 4, op->stream));
  LHIP(op, rocprim::inclusive_scan(op->tmp, bytes, op->wcnt, op->woff + 1, (size_t)n, rocprim::plus<uint32_t>(),
                                   op->stream));
  uint32_t total = 0;
  LHIP(op, hipMemcpyAsync(&total, op->woff + n, 4, hipMemcpyDeviceToHost, op->stream));
  LRET(read_ctr(op));
  if (op->h_ctr->flags & LF_NO_TS)
    return set_err(op, FW_ERR_NO_TIMESTAMP,
                   "Record has Long.MIN_VALUE timestamp (= no timestamp marker). Is the time characteristic set to "
                   "'ProcessingTime', or did you forget to call 'DataStream.assignTimestampsAndWatermarks(...)'?");
  if (op->h_ctr->flags & LF_KEY_GROUP)
    return set_err(op, FW_ERR_KEY_GROUP, "a key of the batch is outside the handle's KeyGroupRange");
  const int64_t E = total;
  // room: the log, a row per possibly firing entry
  LRET(grow_log(op, E));
  LRET(ensure_rows(op, (int64_t)op->h_ctr->rows + E));
  // the entries, their groups inserted on the way at <= 3/4 load; when the map would pass it, nothing is lost: it
  // doubles (with a compaction of the log) and the append runs again from the start (it writes the same entries
  // and sets the same flags)
  int64_t base = op->n_log;
  for (int round = 0;; round++) {
    LHIP(op, hipMemsetAsync(&op->S.ctr->flags, 0, 8, op->stream));  // flags, need_seq
    hipLaunchKernelGGL(k_lp_append, dim3(grid_for(n)), dim3(256), 0, op->stream, op->c, op->S, key, ts, val, kh, n,
                       op->wm, op->wcnt, op->woff, base, op->ord_base, (unsigned long long)(op->gcap / 4 * 3));
    LRET(read_ctr(op));
    if (!(op->h_ctr->flags & LF_MAP_FULL)) break;
    if (round > 40) return set_err(op, FW_ERR_CAPACITY, "list state map full");
    // the map was too small for the push's new groups: four times the capacity (a push of many more new groups
    // than the map holds takes few rounds)
    LRET(compact(op, 2 * op->gcap));
    base = op->n_log;
  }
  LHIP(op, hipGetLastError());
  op->n_log += E;
  op->ord_base += n;
  op->records_in += n;
  // (the counters are current: read after the last append)
  if (op->h_ctr->need_seq) {
    LRET(walk_lists<true>(op, GF_TOUCH, base));
    LRET(read_ctr(op));
  }
  return maybe_compact(op);
}

}  // namespace

extern "C" {

int fw_list_create(const fw_list_config* cfg, fw_list** out) {
  if (!cfg || !out) return FW_ERR_ARG;
  *out = nullptr;
  fw_list* op = new fw_list();
  op->cfg = *cfg;
  const fw_list_config& c = *cfg;
  auto fail = [&](int code, const char* msg) {  // as fw_create: the handle carries the message; destroy it
    op->err = msg;
    *out = op;
    return code;
  };
  if (c.assigner != FW_TUMBLING && c.assigner != FW_SLIDING && c.assigner != FW_GLOBAL && c.assigner != FW_SESSION)
    return fail(FW_ERR_UNSUPPORTED, "assigner must be FW_TUMBLING, FW_SLIDING, FW_SESSION or FW_GLOBAL");
  if (c.assigner == FW_SESSION && c.size <= 0)
    return fail(FW_ERR_ARG, "EventTimeSessionWindows parameters must satisfy 0 < size");
  if (c.assigner == FW_SESSION && c.trigger != FW_TRIGGER_EVENT_TIME)
    return fail(FW_ERR_UNSUPPORTED, "session windows over ListState are offered with EventTimeTrigger (or PurgingTrigger "
                                    "of it)");
  if (c.assigner == FW_TUMBLING && (c.size <= 0 || c.offset < 0 || c.offset >= c.size))
    return fail(FW_ERR_ARG, "TumblingEventTimeWindows parameters must satisfy 0 <= offset < size");
  if (c.assigner == FW_SLIDING && (c.size <= 0 || c.slide <= 0 || c.slide > c.size || c.offset < 0 || c.offset >= c.slide))
    return fail(FW_ERR_ARG, "SlidingEventTimeWindows parameters must satisfy 0 <= offset < slide <= size");
  if (c.allowed_lateness < 0) return fail(FW_ERR_ARG, "The allowed lateness cannot be negative.");
  if (c.trigger != FW_TRIGGER_EVENT_TIME && c.trigger != FW_TRIGGER_COUNT) return fail(FW_ERR_ARG, "unknown trigger");
  if (c.trigger == FW_TRIGGER_COUNT && (c.trigger_count <= 0 || c.trigger_count > INT32_MAX))
    return fail(FW_ERR_ARG, "CountTrigger count must be in [1, 2^31)");
  if (c.evictor < FW_EVICT_NONE || c.evictor > FW_EVICT_DELTA) return fail(FW_ERR_ARG, "unknown evictor");
  if (c.evictor == FW_EVICT_COUNT && c.evict_count < 0) return fail(FW_ERR_ARG, "CountEvictor count must be >= 0");
  if (c.value_type < FW_VAL_I64 || c.value_type > FW_VAL_F32) return fail(FW_ERR_ARG, "unknown value type");
  if (c.key_kind < FW_KEY_LONG || c.key_kind > FW_KEY_HASHED) return fail(FW_ERR_ARG, "unknown key kind");
  const int32_t mp = c.max_parallelism ? c.max_parallelism : 128;
  const int32_t kg0 = c.key_group_start < 0 ? 0 : c.key_group_start;
  const int32_t kg1 = c.key_group_end < 0 ? mp - 1 : c.key_group_end;
  if (mp <= 0 || mp > 32768 || kg0 > kg1 || kg1 >= mp) return fail(FW_ERR_ARG, "invalid KeyGroupRange");
  op->c = LCfg{c.assigner, c.value_type, c.key_kind, c.trigger, c.purging, c.evictor, c.evict_after, c.side_output,
               c.emit_contents, mp, kg0, kg1 - kg0 + 1, c.size, c.slide, c.offset, c.allowed_lateness,
               c.trigger_count, c.evict_count, c.delta_threshold};
  op->device = c.device;
  if (hipSetDevice(c.device) != hipSuccess) return fail(FW_ERR_HIP, "hipSetDevice failed");
  if (hipStreamCreateWithFlags(&op->stream, hipStreamNonBlocking) != hipSuccess)
    return fail(FW_ERR_HIP, "hipStreamCreateWithFlags failed");
  op->max_batch = c.max_batch > 0 ? c.max_batch : (1 << 24);
  const int64_t fan = c.assigner == FW_SLIDING ? (c.size + c.slide - 1) / c.slide : 1;
  const int64_t exp = c.expected_elements > 0 ? c.expected_elements : std::min<int64_t>(op->max_batch * fan, 1 << 22);
  op->lcap = std::max<int64_t>(exp, 1024);
  int64_t g = 1024;  // groups: the map doubles when a push would pass 3/4 load (k_lp_append), so it stays the
  while (g < 2 * std::min<int64_t>(op->lcap, 1 << 20)) g <<= 1;  // smallest that holds them (MALL-resident slots)
  op->gcap = g;
  op->rcap = 1024;
  op->scap = 1024;
  op->S.ecap = 1024;
  int rc = FW_OK;
  if (hipHostMalloc((void**)&op->h_ctr, sizeof(LCounters), hipHostMallocDefault) != hipSuccess) rc = FW_ERR_HIP;
  if (rc == FW_OK) memset(op->h_ctr, 0, sizeof(LCounters));
  if (rc == FW_OK) rc = c.assigner == FW_SESSION ? sl_alloc_map(op, op->S, op->gcap) : alloc_map(op, op->S, op->gcap);
  if (rc == FW_OK && c.assigner == FW_SESSION) {
    const size_t mb = (size_t)op->max_batch;
    if (dmalloc(&op->sk, mb) != hipSuccess || dmalloc(&op->sk2, mb) != hipSuccess || dmalloc(&op->si, mb) != hipSuccess ||
        dmalloc(&op->si2, mb) != hipSuccess || dmalloc(&op->sprog, mb) != hipSuccess ||
        dmalloc(&op->pslot, mb) != hipSuccess)
      rc = FW_ERR_HIP;
  }
  if (rc == FW_OK) rc = alloc_log(op, op->S, op->lcap);
  auto al = [&](int64_t** p, int64_t n) {
    if (rc == FW_OK && dmalloc(p, (size_t)n) != hipSuccess) rc = FW_ERR_HIP;
  };
  for (int64_t** p : {&op->S.rkey, &op->S.rstart, &op->S.rend, &op->S.rcnt, &op->S.rsum, &op->S.rmin, &op->S.rmax,
                      &op->S.rfirst, &op->S.roff})
    al(p, op->rcap);
  for (int64_t** p : {&op->S.ets, &op->S.eval, &op->S.eord}) al(p, op->S.ecap);
  for (int64_t** p : {&op->S.skey, &op->S.sts, &op->S.sval}) al(p, op->scap);
  for (int64_t** p : {&op->in_key, &op->in_ts, &op->in_val}) al(p, op->max_batch);
  if (rc == FW_OK && dmalloc(&op->in_kh, (size_t)op->max_batch) != hipSuccess) rc = FW_ERR_HIP;
  if (rc == FW_OK && dmalloc(&op->wcnt, (size_t)op->max_batch) != hipSuccess) rc = FW_ERR_HIP;
  if (rc == FW_OK && dmalloc(&op->woff, (size_t)op->max_batch + 1) != hipSuccess) rc = FW_ERR_HIP;
  if (rc == FW_OK && dmalloc(&op->S.ctr, 1) != hipSuccess) rc = FW_ERR_HIP;
  if (rc == FW_OK && hipMemsetAsync(op->S.ctr, 0, sizeof(LCounters), op->stream) != hipSuccess) rc = FW_ERR_HIP;
  if (rc == FW_OK) {
    static const long long none = LMAX;
    if (hipMemcpyAsync(&op->S.ctr->next_due, &none, 8, hipMemcpyHostToDevice, op->stream) != hipSuccess) rc = FW_ERR_HIP;
  }
  if (rc == FW_OK && hipStreamSynchronize(op->stream) != hipSuccess) rc = FW_ERR_HIP;
  if (rc != FW_OK) return fail(rc, "device allocation failed");
  *out = op;
  return FW_OK;
}

void fw_list_destroy(fw_list* op) {
  if (!op) return;
  (void)hipSetDevice(op->device);
  if (op->stream) (void)hipStreamSynchronize(op->stream);
  sl_free_map(op->S);  // (the session columns are null for the other assigners)
  free_log(op->S);
  dfree(op->sk);
  dfree(op->sk2);
  dfree(op->si);
  dfree(op->si2);
  dfree(op->sprog);
  dfree(op->pslot);
  for (int64_t** p : {&op->S.rkey, &op->S.rstart, &op->S.rend, &op->S.rcnt, &op->S.rsum, &op->S.rmin, &op->S.rmax,
                      &op->S.rfirst, &op->S.roff, &op->S.ets, &op->S.eval, &op->S.eord, &op->S.skey, &op->S.sts,
                      &op->S.sval, &op->in_key, &op->in_ts, &op->in_val})
    dfree(*p);
  dfree(op->in_kh);
  dfree(op->wcnt);
  dfree(op->woff);
  dfree(op->S.ctr);
  dfree(op->flags8);
  dfree(op->sel);
  dfree(op->sel2);
  dfree(op->keys);
  dfree(op->keys2);
  dfree(op->seg);
  dfree(op->prog);
  dfree(op->gts);
  dfree(op->gval);
  dfree(op->gord);
  dfree(op->galive);
  if (op->tmp) (void)hipFree(op->tmp);
  if (op->h_ctr) (void)hipHostFree(op->h_ctr);
  if (op->stream) (void)hipStreamDestroy(op->stream);
  delete op;
}

const char* fw_list_last_error(const fw_list* op) { return op ? op->err.c_str() : "null handle"; }

int fw_list_push_batch_device(fw_list* op, const int64_t* key, const int64_t* ts, const void* val,
                              const int32_t* key_hash, int64_t n) {
  if (!op || n < 0 || (n && (!key || !ts || !val))) return set_err(op, FW_ERR_ARG, "invalid arguments");
  (void)hipSetDevice(op->device);
  return push_device(op, key, ts, (const int64_t*)val, key_hash, n);
}

int fw_list_push_batch(fw_list* op, const int64_t* key, const int64_t* ts, const void* val, const int32_t* key_hash,
                       int64_t n) {
  if (!op || n < 0 || (n && (!key || !ts || !val))) return set_err(op, FW_ERR_ARG, "invalid arguments");
  (void)hipSetDevice(op->device);
  for (int64_t o = 0; o < n; o += op->max_batch) {
    const int64_t m = std::min(op->max_batch, n - o);
    LHIP(op, hipMemcpyAsync(op->in_key, key + o, (size_t)m * 8, hipMemcpyHostToDevice, op->stream));
    LHIP(op, hipMemcpyAsync(op->in_ts, ts + o, (size_t)m * 8, hipMemcpyHostToDevice, op->stream));
    LHIP(op, hipMemcpyAsync(op->in_val, (const int64_t*)val + o, (size_t)m * 8, hipMemcpyHostToDevice, op->stream));
    if (key_hash)
      LHIP(op, hipMemcpyAsync(op->in_kh, key_hash + o, (size_t)m * 4, hipMemcpyHostToDevice, op->stream));
    LRET(push_device(op, op->in_key, op->in_ts, op->in_val, key_hash ? op->in_kh : nullptr, m));
  }
  return FW_OK;
}

int fw_list_advance_watermark(fw_list* op, int64_t wm, int64_t* n_pending_rows) {
  if (!op) return FW_ERR_ARG;
  (void)hipSetDevice(op->device);
  LRET(read_ctr(op));
  if (wm > op->wm && wm < op->h_ctr->next_due) {
    op->wm = wm;  // no timer is due
  } else if (wm > op->wm) {  // HeapInternalTimerService.advanceWatermark: timers <= wm, in any order across lists
    op->wm = wm;
    const long long none = LMAX;
    LHIP(op, hipMemcpyAsync(&op->S.ctr->next_due, &none, 8, hipMemcpyHostToDevice, op->stream));
    if (sessions(op)) {
      LRET(sl_watermark(op, wm));
      LRET(read_ctr(op));
      if (n_pending_rows) *n_pending_rows = (int64_t)op->h_ctr->rows;
      return FW_OK;
    }
    LHIP(op, hipMemsetAsync(&op->S.ctr->nfire, 0, 16, op->stream));
    hipLaunchKernelGGL(k_lw_due, dim3(grid_for(op->gcap)), dim3(256), 0, op->stream, op->c, op->S, wm);
    LRET(read_ctr(op));
    const int64_t nfire = (int64_t)op->h_ctr->nfire, nclean = (int64_t)op->h_ctr->nclean;
    if (nfire) {
      LRET(ensure_rows(op, (int64_t)op->h_ctr->rows + nfire));
      LRET(walk_lists<false>(op, GF_FIRE, 0));
    }
    if (nfire || nclean) {
      if (nclean)
        hipLaunchKernelGGL(k_lw_clean_log, dim3(grid_for(op->n_log)), dim3(256), 0, op->stream, op->S, op->n_log);
      hipLaunchKernelGGL(k_lw_clean_map, dim3(grid_for(op->gcap)), dim3(256), 0, op->stream, op->S);
      LHIP(op, hipGetLastError());
    }
    LRET(read_ctr(op));
    LRET(maybe_compact(op));
  }
  LRET(read_ctr(op));
  if (n_pending_rows) *n_pending_rows = (int64_t)op->h_ctr->rows;
  return FW_OK;
}

int fw_list_pending(fw_list* op, int64_t* n_rows, int64_t* n_elems, int64_t* n_side_rows) {
  if (!op) return FW_ERR_ARG;
  LRET(read_ctr(op));
  if (n_rows) *n_rows = (int64_t)op->h_ctr->rows;
  if (n_elems) *n_elems = (int64_t)op->h_ctr->elems;
  if (n_side_rows) *n_side_rows = (int64_t)op->h_ctr->side;
  return FW_OK;
}

int fw_list_drain(fw_list* op, const fw_list_rows* rows, int64_t cap_rows, const fw_list_elems* elems,
                  int64_t cap_elems, int64_t* n_rows, int64_t* n_elems) {
  if (!op || !rows) return set_err(op, FW_ERR_ARG, "invalid arguments");
  (void)hipSetDevice(op->device);
  LRET(read_ctr(op));
  const int64_t nr = (int64_t)op->h_ctr->rows, ne = (int64_t)op->h_ctr->elems;
  if (n_rows) *n_rows = nr;
  if (n_elems) *n_elems = ne;
  if (nr > cap_rows || (ne && (!elems || ne > cap_elems))) return set_err(op, FW_ERR_CAPACITY, "output too small");
  const int64_t* src[] = {op->S.rkey, op->S.rstart, op->S.rend, op->S.rcnt, op->S.rsum, op->S.rmin, op->S.rmax,
                          op->S.rfirst, op->S.roff};
  int64_t* dst[] = {rows->key, rows->start, rows->end, rows->count, rows->sum, rows->min, rows->max, rows->first,
                    rows->elem_off};
  for (int i = 0; i < 9; i++)
    if (dst[i] && nr) LHIP(op, hipMemcpyAsync(dst[i], src[i], (size_t)nr * 8, hipMemcpyDeviceToHost, op->stream));
  if (ne) {
    const int64_t* es[] = {op->S.ets, op->S.eval, op->S.eord};
    int64_t* ed[] = {elems->ts, elems->val, elems->ordinal};
    for (int i = 0; i < 3; i++)
      if (ed[i]) LHIP(op, hipMemcpyAsync(ed[i], es[i], (size_t)ne * 8, hipMemcpyDeviceToHost, op->stream));
  }
  LHIP(op, hipMemsetAsync(&op->S.ctr->rows, 0, 16, op->stream));  // rows, elems
  LHIP(op, hipStreamSynchronize(op->stream));
  op->fired_total += nr;
  op->h_ctr->rows = op->h_ctr->elems = 0;
  return FW_OK;
}

int fw_list_clear_pending(fw_list* op) {
  if (!op) return FW_ERR_ARG;
  (void)hipSetDevice(op->device);
  LRET(read_ctr(op));
  op->fired_total += (int64_t)op->h_ctr->rows;
  LHIP(op, hipMemsetAsync(&op->S.ctr->rows, 0, 16, op->stream));  // rows, elems
  LHIP(op, hipStreamSynchronize(op->stream));
  op->h_ctr->rows = op->h_ctr->elems = 0;
  return FW_OK;
}

int fw_list_drain_side(fw_list* op, const fw_side_rows* host_dst, int64_t cap, int64_t* n) {
  if (!op || !host_dst) return set_err(op, FW_ERR_ARG, "invalid arguments");
  (void)hipSetDevice(op->device);
  LRET(read_ctr(op));
  const int64_t ns = (int64_t)op->h_ctr->side;
  if (n) *n = ns;
  if (ns > cap) return set_err(op, FW_ERR_CAPACITY, "output too small");
  if (ns) {
    LHIP(op, hipMemcpyAsync(host_dst->key, op->S.skey, (size_t)ns * 8, hipMemcpyDeviceToHost, op->stream));
    LHIP(op, hipMemcpyAsync(host_dst->ts, op->S.sts, (size_t)ns * 8, hipMemcpyDeviceToHost, op->stream));
    LHIP(op, hipMemcpyAsync(host_dst->val, op->S.sval, (size_t)ns * 8, hipMemcpyDeviceToHost, op->stream));
  }
  LHIP(op, hipMemsetAsync(&op->S.ctr->side, 0, 8, op->stream));
  LHIP(op, hipStreamSynchronize(op->stream));
  return FW_OK;
}

int fw_list_get_stats(fw_list* op, fw_stats* out) {
  if (!op || !out) return set_err(op, FW_ERR_ARG, "invalid arguments");
  (void)hipSetDevice(op->device);
  uint8_t* has = nullptr;
  unsigned long long* d2 = nullptr;
  unsigned long long h2[2] = {0, 0};
  LHIP(op, dmalloc(&has, (size_t)op->gcap));
  LHIP(op, dmalloc(&d2, 2));
  LHIP(op, hipMemsetAsync(has, 0, (size_t)op->gcap, op->stream));
  LHIP(op, hipMemsetAsync(d2, 0, 16, op->stream));
  if (sessions(op)) {
    hipLaunchKernelGGL(k_sl_count_state, dim3(grid_for(op->gcap)), dim3(256), 0, op->stream, op->c, op->S, d2);
  } else {
    if (op->n_log)
      hipLaunchKernelGGL(k_mark_lists, dim3(grid_for(op->n_log)), dim3(256), 0, op->stream, op->S, op->n_log, has);
    hipLaunchKernelGGL(k_count_state, dim3(grid_for(op->gcap)), dim3(256), 0, op->stream, op->c, op->S, has, d2);
  }
  LHIP(op, hipMemcpyAsync(h2, d2, 16, hipMemcpyDeviceToHost, op->stream));
  LRET(read_ctr(op));
  dfree(has);
  dfree(d2);
  memset(out, 0, sizeof *out);
  out->records_in = op->records_in;
  out->late_records_dropped = (int64_t)op->h_ctr->late;
  out->keyed_state_entries = (int64_t)h2[0];
  out->event_time_timers = (int64_t)h2[1];
  out->current_watermark = op->wm;
  out->fired_rows_total = op->fired_total + (int64_t)op->h_ctr->rows;
  out->pending_rows = (int64_t)op->h_ctr->rows;
  out->pending_side_rows = (int64_t)op->h_ctr->side;
  out->table_capacity = op->gcap;
  out->table_grows = op->grows;
  return FW_OK;
}

int fw_list_snapshot_key_group(fw_list* op, int32_t key_group, const fw_list_state* dst, int64_t cap_lists,
                               int64_t cap_elems, int64_t* n_lists, int64_t* n_elems) {
  if (!op) return FW_ERR_ARG;
  (void)hipSetDevice(op->device);
  if (sessions(op)) return set_err(op, FW_ERR_UNSUPPORTED, "session windows' list state is not offered for snapshots");
  if ((uint32_t)(key_group - op->c.kg0) >= (uint32_t)op->c.nkg)
    return set_err(op, FW_ERR_KEY_GROUP, "key group %d is not in the handle's KeyGroupRange", key_group);
  // the key group's lists: its live groups, and its live elements grouped by list in list order
  LRET(ensure_sel(op, std::max(op->n_log, op->gcap)));
  hipLaunchKernelGGL(k_kg_flags_map, dim3(grid_for(op->gcap)), dim3(256), 0, op->stream, op->S, key_group, op->flags8);
  int64_t ng = 0;
  LRET(select_positions(op, op->flags8, op->gcap, op->seg, &ng));
  int64_t m = 0;
  if (op->n_log) {
    hipLaunchKernelGGL(k_kg_flags_log, dim3(grid_for(op->n_log)), dim3(256), 0, op->stream, op->S, op->n_log, key_group,
                       op->flags8);
    LRET(select_positions(op, op->flags8, op->n_log, op->sel, &m));
  }
  if (n_lists) *n_lists = ng;
  if (n_elems) *n_elems = m;
  if (!dst || ng > cap_lists || m > cap_elems) return FW_OK;
  std::vector<uint32_t> gids(ng), pos(m);
  std::vector<int32_t> lg(m);
  if (ng) LHIP(op, hipMemcpyAsync(gids.data(), op->seg, (size_t)ng * 4, hipMemcpyDeviceToHost, op->stream));
  if (m) LHIP(op, hipMemcpyAsync(pos.data(), op->sel, (size_t)m * 4, hipMemcpyDeviceToHost, op->stream));
  LHIP(op, hipStreamSynchronize(op->stream));
  // host gathers (a snapshot is a cold path): group columns, then the elements per list in log order
  std::vector<LPay> lpay(op->n_log);
  std::vector<int32_t> lgid(op->n_log);
  if (op->n_log) {
    LHIP(op, hipMemcpy(lpay.data(), op->S.lpay, (size_t)op->n_log * sizeof(LPay), hipMemcpyDeviceToHost));
    LHIP(op, hipMemcpy(lgid.data(), op->S.lgid, (size_t)op->n_log * 4, hipMemcpyDeviceToHost));
  }
  std::vector<int64_t> rank(op->gcap, -1);
  for (int64_t i = 0; i < ng; i++) rank[gids[i]] = i;
  std::vector<int64_t> cnt(ng, 0), off(ng + 1, 0);
  for (int64_t i = 0; i < m; i++) cnt[rank[lgid[pos[i]]]]++;
  for (int64_t i = 0; i < ng; i++) off[i + 1] = off[i] + cnt[i];
  std::vector<int64_t> fill(off.begin(), off.end() - 1);
  for (int64_t i = 0; i < m; i++) {
    const uint32_t e = pos[i];
    const int64_t k = fill[rank[lgid[e]]]++;
    if (dst->ts) dst->ts[k] = lpay[e].ts;
    if (dst->val) dst->val[k] = lpay[e].val;
    if (dst->ordinal) dst->ordinal[k] = lpay[e].ord;
  }
  for (int64_t i = 0; i < ng; i++) {
    const uint32_t g = gids[i];
    GSlot gs;
    LHIP(op, hipMemcpy(&gs, op->S.g + g, sizeof gs, hipMemcpyDeviceToHost));
    const int64_t key = gs.key, start = gs.start, c = gs.cnt;
    const uint32_t fl = gs.fl;
    dst->key[i] = key;
    dst->start[i] = start;
    dst->end[i] = op->c.assigner == FW_GLOBAL ? LMAX : (int64_t)((uint64_t)start + (uint64_t)op->c.size);
    dst->trigger_count[i] = c;
    dst->timer[i] = (fl & GF_TIMER) ? 1 : 0;
    dst->n_elems[i] = cnt[i];
  }
  return FW_OK;
}

int fw_list_restore_key_group(fw_list* op, int32_t key_group, const fw_list_state* src, int64_t n_lists,
                              int64_t n_elems) {
  if (!op || (n_lists && !src)) return set_err(op, FW_ERR_ARG, "invalid arguments");
  (void)hipSetDevice(op->device);
  if (sessions(op)) return set_err(op, FW_ERR_UNSUPPORTED, "session windows' list state is not offered for snapshots");
  if ((uint32_t)(key_group - op->c.kg0) >= (uint32_t)op->c.nkg)
    return set_err(op, FW_ERR_KEY_GROUP, "key group %d is not in the handle's KeyGroupRange", key_group);
  if (n_lists == 0) return FW_OK;
  int64_t total = 0, max_ord = -1;
  for (int64_t i = 0; i < n_lists; i++) {
    if (src->n_elems[i] < 0) return set_err(op, FW_ERR_ARG, "negative list length");
    total += src->n_elems[i];
    const int64_t s = src->start[i];
    const int64_t e = op->c.assigner == FW_GLOBAL ? LMAX : (int64_t)((uint64_t)s + (uint64_t)op->c.size);
    if (src->end[i] != e || (op->c.assigner == FW_GLOBAL && s != LMIN))
      return set_err(op, FW_ERR_ARG, "list %lld: window [%lld, %lld) is not one of the assigner's", (long long)i,
                     (long long)s, (long long)src->end[i]);
    if (op->c.key_kind != FW_KEY_HASHED) {
      const int64_t k = src->key[i];
      const int32_t h = op->c.key_kind == FW_KEY_INT ? (int32_t)k : (int32_t)(k ^ (int64_t)((uint64_t)k >> 32));
      // MathUtils.murmurHash (host restatement) % maxParallelism
      uint32_t c = (uint32_t)h;
      c *= 0xcc9e2d51u;
      c = (c << 15) | (c >> 17);
      c *= 0x1b873593u;
      c = (c << 13) | (c >> 19);
      c = c * 5u + 0xe6546b64u;
      c ^= 4u;
      c ^= c >> 16;
      c *= 0x85ebca6bu;
      c ^= c >> 13;
      c *= 0xc2b2ae35u;
      c ^= c >> 16;
      int32_t r = (int32_t)c;
      r = r >= 0 ? r : (r != INT32_MIN ? -r : 0);
      if (r % op->c.max_par != key_group)
        return set_err(op, FW_ERR_KEY_GROUP, "key %lld is not in key group %d", (long long)k, key_group);
    }
  }
  if (total != n_elems) return set_err(op, FW_ERR_ARG, "list lengths do not add up to n_elems");
  for (int64_t i = 0; i < n_elems; i++) max_ord = std::max(max_ord, src->ordinal[i]);
  LRET(read_ctr(op));
  if ((int64_t)op->h_ctr->live_groups + n_lists > op->gcap / 2) LRET(compact(op, (int64_t)op->h_ctr->live_groups + n_lists));
  LRET(grow_log(op, n_elems));
  // device copies of the lists' columns
  int64_t *dk = nullptr, *ds = nullptr, *dc = nullptr, *dt = nullptr, *ets = nullptr, *evl = nullptr, *eod = nullptr;
  int32_t *dg = nullptr, *eg = nullptr;
  LHIP(op, dmalloc(&dk, (size_t)n_lists));
  LHIP(op, dmalloc(&ds, (size_t)n_lists));
  LHIP(op, dmalloc(&dc, (size_t)n_lists));
  LHIP(op, dmalloc(&dt, (size_t)n_lists));
  LHIP(op, dmalloc(&dg, (size_t)n_lists));
  LHIP(op, hipMemcpy(dk, src->key, (size_t)n_lists * 8, hipMemcpyHostToDevice));
  LHIP(op, hipMemcpy(ds, src->start, (size_t)n_lists * 8, hipMemcpyHostToDevice));
  LHIP(op, hipMemcpy(dc, src->trigger_count, (size_t)n_lists * 8, hipMemcpyHostToDevice));
  LHIP(op, hipMemcpy(dt, src->timer, (size_t)n_lists * 8, hipMemcpyHostToDevice));
  // one thread: lists repeating a (key, window) append to it in order
  hipLaunchKernelGGL(k_restore_groups, dim3(1), dim3(1), 0, op->stream, op->c, op->S, dk, ds, dc, dt, n_lists,
                     key_group, dg);
  std::vector<int32_t> hg(n_lists), eg_h(n_elems);
  LHIP(op, hipMemcpyAsync(hg.data(), dg, (size_t)n_lists * 4, hipMemcpyDeviceToHost, op->stream));
  LHIP(op, hipStreamSynchronize(op->stream));
  for (int64_t i = 0, k = 0; i < n_lists; i++)
    for (int64_t j = 0; j < src->n_elems[i]; j++) eg_h[k++] = hg[i];
  if (n_elems) {
    LHIP(op, dmalloc(&ets, (size_t)n_elems));
    LHIP(op, dmalloc(&evl, (size_t)n_elems));
    LHIP(op, dmalloc(&eod, (size_t)n_elems));
    LHIP(op, dmalloc(&eg, (size_t)n_elems));
    LHIP(op, hipMemcpy(ets, src->ts, (size_t)n_elems * 8, hipMemcpyHostToDevice));
    LHIP(op, hipMemcpy(evl, src->val, (size_t)n_elems * 8, hipMemcpyHostToDevice));
    LHIP(op, hipMemcpy(eod, src->ordinal, (size_t)n_elems * 8, hipMemcpyHostToDevice));
    LHIP(op, hipMemcpy(eg, eg_h.data(), (size_t)n_elems * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_restore_elems, dim3(grid_for(n_elems)), dim3(256), 0, op->stream, op->S, ets, evl, eod, eg,
                       n_elems, op->n_log);
    LHIP(op, hipStreamSynchronize(op->stream));
  }
  for (auto p : {dk, ds, dc, dt, ets, evl, eod}) (void)hipFree(p);
  (void)hipFree(dg);
  (void)hipFree(eg);
  LRET(read_ctr(op));
  if (op->h_ctr->flags & LF_MAP_FULL) return set_err(op, FW_ERR_CAPACITY, "list state map full");
  for (int64_t i = 0; i < n_lists; i++)
    if (hg[i] < 0) return set_err(op, FW_ERR_CAPACITY, "list state map full");
  op->n_log += n_elems;
  op->ord_base = std::max(op->ord_base, max_ord + 1);
  return FW_OK;
}

}  // extern "C"
