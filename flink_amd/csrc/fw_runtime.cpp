// fw_runtime.cpp — host side of the C-ABI in include/flink_window.h.
//
// One fw_op = one WindowOperator subtask on one GPU: it owns the HBM state table of its
// KeyGroupRange, the per-batch scratch, the fired-row buffer and one HIP stream.  Every public
// call is serialised by the caller (the Flink task thread holds the checkpoint lock around
// processElement / processWatermark, StreamInputProcessor.java:211-222).
//
// Asynchrony.  Device pushes and count-less watermarks only queue work; every queued sequence ends
// with a copy of the device Status into pinned memory and an event (the "snapshot").  The next call
// that needs the status waits for the snapshot and settles the sequence: if a kernel suspended
// because a state region or the fired-row buffer lacked room, the table / buffer is grown and the
// suspended kernels are resumed where they stopped (and a watermark the suspension skipped is fired
// again); errors the sequence detected are returned by that call.
//
// A push queues its classify / scan / scatter kernels BEFORE it waits for the previous snapshot:
// they only read the batch and write this push's scratch set (two sets alternate), so they run
// while the host waits and settles, and the state kernels are queued before the GPU drains.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/flink_window.h"
#include "fw_internal.h"

namespace {

// per-batch scratch; two sets alternate so a push can be resumed while the next one is classified
struct Scratch {
  uint32_t* hist = nullptr;      // (P+2) x T histogram, scanned in place into offsets
  uint32_t* scan_tmp = nullptr;
  PRec* part = nullptr;          // the batch's normal records, partition-major
  int64_t *sk = nullptr, *stt = nullptr, *sv = nullptr;  // ordered-path list
  int32_t* skh = nullptr;
  int64_t* so = nullptr;         // FW_AGG_FIRST: arrival ordinal of each ordered-path record
  int64_t* byv = nullptr;        // FW_AGG_MINBY / MAXBY: the batch's value column (DevCfg::by_val)
  int64_t* rowc = nullptr;       // FW_AGG_ROW: the batch's value columns (column j at j * max_batch), DevCfg::row_cols
  uint8_t* rown = nullptr;       //             and NULL masks (DevCfg::row_nulls)
  int32_t T = 0;                 // tiles of the batch that used this set
  int64_t n = 0;                 // records of the batch
  bool split = false;            // its aggregate split long partitions (fw_op::hot)
  int64_t wm = INT64_MIN;        // watermark the batch was classified against
  int32_t compact = 0;           // DevCfg::compact / cbase of the batch (a resumed aggregate reads the same form)
  int32_t narrow = 0, ndn0 = 0;  // DevCfg::narrow / ndn0 of the batch's single pass
  int64_t cbase = 0;
  int64_t ord_base = 0;          // arrival ordinal of the batch's first record (ordinal aggregates)
  int32_t* wide = nullptr;       // DevCfg::wide of the batches that use this set
  PartialRec* pparts = nullptr;  // combining: a partials push's partials, partition-major (allocated on first use)
  bool partials = false;         // the set's latest push merged partials (fw_push_partials_device)
  // HyperLogLog partials (fw_push_hll_partials_device): the push's partials, registers and register offsets, for
  // the register raise that follows the merge (rerun after a resumed merge)
  PartialCols hin{};
  int64_t hn = 0;
  const uint32_t* hregs = nullptr;
  const uint32_t* hoff = nullptr;
  // gathered batches (fwdev::gather_mode): runs table [T8][P] and its transpose, the partitions' virtual
  // offsets (P + 1) and the ordered-path rows (2 x T8); T is then the batch's FW_GTILE tiles
  uint32_t *rt = nullptr, *rt_t = nullptr, *voffs = nullptr, *gsrow = nullptr, *gcb = nullptr;
  bool gather = false;
  // dense batches: the single-pass scatter's run lengths and flags (fwdev::launch_scatter_rsv), P + FW_RSV_WORDS
  uint32_t* rsv = nullptr;
  bool single = false;  // the set's latest batch went through it (its runs are then at p * fw_op::rcap ...)
  // DevCfg::wide of the set's latest batch: a word of rsv (zeroed with it) when the batch took the single pass
  int32_t* wide_word(int32_t P) const { return single ? reinterpret_cast<int32_t*>(rsv + P + FW_RSV_WIDE) : wide; }
  // the ordered-path rows of the batch: scanned counts per tile, then raw counts
  const uint32_t* srow(int32_t P) const { return gather ? gsrow : hist + (int64_t)P * T; }
  // the partitions' runs in part: offsets offs()[p * offT()] (a gathered batch: regrouped, virtual offsets)
  const uint32_t* offs() const { return gather ? voffs : hist; }
  int32_t offT() const { return gather ? 1 : T; }
};

}  // namespace

struct fw_op {
  fw_config cfg{};
  DevCfg dc{};
  int device = 0;
  hipStream_t stream = nullptr;
  // async input (fw_set_async_input): a device push's batch-only kernels (classify, scan, scatter) run on
  // bstream, beside the previous batch's aggregate and firing on `stream`; ev_scat[set] orders the batch's
  // aggregate after them, ev_done[set] the reuse of a scratch set after the aggregate of its previous batch
  hipStream_t bstream = nullptr;
  hipEvent_t ev_scat[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr};
  bool async_in = false;
  int64_t rcap = 0;          // single-pass scatter: each partition's run capacity in compact records
  int32_t rsv_seen = 0;      // Status::rsv_fallbacks at the latest settle
  int32_t rsv_misses = 0;    // consecutive settles that saw a single-pass batch redone
  int64_t resumptions = 0;   // fw_stats::push_resumptions
  bool rsv_off = false;      // after 3 of them the operator stops trying the single pass
  int32_t narrow_seen = 0;   // Status::narrow_misses last seen
  bool narrow_off = false;   // a narrow single pass met a record without a narrow form: 16-byte records from then on
  int64_t narrow_batches = 0;  // batches that took the narrow single pass (fw_stats)
  int64_t single_batches = 0;  // batches that took the single pass (fw_stats)
  uint32_t *xoffs = nullptr, *xscan = nullptr;  // combining: the combiner's live-count offsets and scan scratch
  // HyperLogLog combining: the extracted partials' register offsets (combiner) / the pushed ones' (receiver), with
  // their scan scratch and capacities
  uint32_t *xreg = nullptr, *xreg_tmp = nullptr, *hoff = nullptr, *hoff_tmp = nullptr;
  int64_t xreg_cap = 0, hoff_cap = 0, xreg_n = -1;
  std::string err;

  // state table
  DevTable tb{};
  int64_t table_slots = 0;
  int64_t grows = 0;

  // per-batch scratch
  int64_t max_batch = 0;
  int32_t tmax = 0;
  int64_t *in_key = nullptr, *in_ts = nullptr, *in_val = nullptr;
  int32_t* in_kh = nullptr;
  Scratch sc[2];
  int last_sc = 1;   // set of the most recent push
  AggProg prog{};    // k_aggregate resume points
  uint32_t taint_epoch = 0;  // sessions: epoch of the latest batch's taint set (DevCfg.taint_*)
  AggHot hot{};              // split-partition buffers (allocated by the first batch that may need them)
  TdBuf td{};                // FW_AGG_TDIGEST: per-push compression buffers
  DevCount cw{};             // FW_COUNT: count-window state
  bool td_export = false;    // FW_AGG_TDIGEST: fired rows keep their centroids (DevRows::dig)
  int64_t dig_stride = 0;    // words per row of DevRows::dig (t-digest export: 1 + delta; FW_AGG_ROW: 1 + aggregates)
  int64_t* iota = nullptr;   // FW_AGG_ROW: 0, 1, ... (a record's value is its index in the push)

  DevRows out{};
  DevSide side{};
  int64_t out_base = 0, side_base = 0;  // rows already handed to the caller
  Status* d_status = nullptr;
  Status* h_status = nullptr;           // written by the snapshot copy: read only when settled
  unsigned long long* d_stats3 = nullptr;

  int64_t wm = INT64_MIN;
  int64_t records_in = 0;

  // the queued, not yet settled sequence
  hipEvent_t snap = nullptr;
  bool unsynced = false;
  bool push_unsettled = false;  // it holds a push (in scratch set last_sc)
  bool fire_unsettled = false;  // it holds a watermark (fired again if the push suspended)
  bool clear_deferred = false;  // fw_clear_pending was called meanwhile

  // optional per-kernel event timing (fw_profile)
  uint32_t prof_mask = 0;  // kernel kinds timed (bit k = kind k)
  struct Pair {
    hipEvent_t a, b;
    int kind;
  };
  std::vector<Pair> prof_pending;
  std::vector<hipEvent_t> prof_free;
  double prof_ms[FW_NUM_KERNELS] = {0};
  int64_t prof_n[FW_NUM_KERNELS] = {0};
};

namespace {

int set_err(fw_op* op, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (op) op->err = buf;
  return code;
}

#define HIP_OR_RETURN(op, expr)                                                                          \
  do {                                                                                                   \
    hipError_t _e = (expr);                                                                              \
    if (_e != hipSuccess) return set_err(op, FW_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

template <class T>
hipError_t dmalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  return hipMalloc((void**)p, count * sizeof(T));
}
template <class T>
void dfree(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

int64_t next_pow2(int64_t x) {
  int64_t r = 1;
  while (r < x) r <<= 1;
  return r;
}
int ilog2(int64_t x) {
  int r = 0;
  while ((int64_t(1) << r) < x) r++;
  return r;
}

void free_table(DevTable& t) {
  for (int b = 0; b < 2; b++) {
    dfree(t.ent[b]);
    dfree(t.state[b]);
  }
}

int alloc_table(fw_op* op, DevTable& t, const DevCfg& c, bool with_meta) {
  const int64_t slots = (int64_t)c.P << c.log_r;
  for (int b = 0; b < 2; b++) {
    HIP_OR_RETURN(op, dmalloc(&t.ent[b], (size_t)slots));
    HIP_OR_RETURN(op, dmalloc(&t.state[b], (size_t)slots));
    HIP_OR_RETURN(op, hipMemsetAsync(t.state[b], 0, (size_t)slots * sizeof(uint32_t), op->stream));
  }
  if (with_meta) {
    HIP_OR_RETURN(op, dmalloc(&t.cur, (size_t)c.P));
    HIP_OR_RETURN(op, dmalloc(&t.live, (size_t)c.P));
    HIP_OR_RETURN(op, dmalloc(&t.next_timer, (size_t)c.P));
    HIP_OR_RETURN(op, dmalloc(&t.fire_e, (size_t)c.P));
    HIP_OR_RETURN(op, dmalloc(&t.fire_lo, (size_t)c.P));
    HIP_OR_RETURN(op, dmalloc(&t.pane_floor, (size_t)c.P));
    HIP_OR_RETURN(op, dmalloc(&t.passes, (size_t)c.P));
  }
  return FW_OK;
}

int alloc_scratch(fw_op* op, Scratch& s, int64_t mb, int64_t m) {
  HIP_OR_RETURN(op, dmalloc(&s.hist, m));
  HIP_OR_RETURN(op, dmalloc(&s.scan_tmp, m / 4096 + 2));
  HIP_OR_RETURN(op, dmalloc(&s.part, mb));
  HIP_OR_RETURN(op, dmalloc(&s.sk, mb));
  HIP_OR_RETURN(op, dmalloc(&s.stt, mb));
  HIP_OR_RETURN(op, dmalloc(&s.sv, mb));
  HIP_OR_RETURN(op, dmalloc(&s.skh, mb));
  HIP_OR_RETURN(op, dmalloc(&s.wide, 1));
  if (op->dc.dense) {  // (zero between batches: the aggregate's stream resets what a batch used)
    HIP_OR_RETURN(op, dmalloc(&s.rsv, (size_t)op->dc.P + FW_RSV_WORDS));
    HIP_OR_RETURN(op, hipMemset(s.rsv, 0, ((size_t)op->dc.P + FW_RSV_WORDS) * sizeof(uint32_t)));
  }
  if (op->cfg.aggregate >= FW_AGG_FIRST && op->cfg.aggregate <= FW_AGG_FIRST_MAX) HIP_OR_RETURN(op, dmalloc(&s.so, mb));
  if (op->cfg.aggregate == FW_AGG_MINBY || op->cfg.aggregate == FW_AGG_MAXBY) HIP_OR_RETURN(op, dmalloc(&s.byv, mb));
  if (op->cfg.aggregate == FW_AGG_ROW) {
    HIP_OR_RETURN(op, dmalloc(&s.rowc, (size_t)(mb * op->dc.row_nc)));
    HIP_OR_RETURN(op, dmalloc(&s.rown, (size_t)mb));
  }
  DevCfg probe = op->dc;
  probe.compact = 1;
  if (fwdev::gather_mode(probe, 1)) {
    const int64_t t8 = std::min<int64_t>((mb + FW_GTILE - 1) / FW_GTILE, FW_GMAX_T);
    HIP_OR_RETURN(op, dmalloc(&s.rt, (size_t)(t8 * op->dc.P)));
    HIP_OR_RETURN(op, dmalloc(&s.rt_t, (size_t)(t8 * op->dc.P)));
    HIP_OR_RETURN(op, dmalloc(&s.voffs, (size_t)op->dc.P + 1));
    HIP_OR_RETURN(op, dmalloc(&s.gsrow, (size_t)(2 * t8)));
    HIP_OR_RETURN(op, dmalloc(&s.gcb, (size_t)op->dc.P + 1));
  }
  return FW_OK;
}
void free_scratch(Scratch& s) {
  dfree(s.hist);
  dfree(s.scan_tmp);
  dfree(s.part);
  dfree(s.rowc);
  dfree(s.rown);
  dfree(s.sk);
  dfree(s.stt);
  dfree(s.sv);
  dfree(s.skh);
  dfree(s.wide);
  dfree(s.rsv);
  dfree(s.pparts);
  dfree(s.so);
  dfree(s.byv);
  dfree(s.rt);
  dfree(s.rt_t);
  dfree(s.voffs);
  dfree(s.gsrow);
  dfree(s.gcb);
}

// buffers of the split-partition aggregate (AggHot): deltas at record indices, so one Entry per record
// of the largest batch; one chunk count per partition and per FW_AGG_CHUNK records
int ensure_hot(fw_op* op) {
  if (op->hot.delta) return FW_OK;
  const int64_t P = op->dc.P;
  AggHot& h = op->hot;
  HIP_OR_RETURN(op, dmalloc(&h.delta, (size_t)op->max_batch));
  HIP_OR_RETURN(op, dmalloc(&h.chunk_base, (size_t)P + 1));
  HIP_OR_RETURN(op, dmalloc(&h.scan_tmp, 64));
  HIP_OR_RETURN(op, dmalloc(&h.nd, (size_t)(P + op->max_batch / FW_AGG_CHUNK + 1)));
  HIP_OR_RETURN(op, dmalloc(&h.pdone, (size_t)P));
  return FW_OK;
}
void free_hot(AggHot& h) {
  dfree(h.delta);
  dfree(h.chunk_base);
  dfree(h.scan_tmp);
  dfree(h.nd);
  dfree(h.pdone);
}

// the ordered path may fill the fired-row buffer up to cap - table slots, so a watermark always has
// room to fire every live window
void set_slow_limit(fw_op* op) { op->out.slow_limit = std::max<int64_t>(0, op->out.cap - op->table_slots); }

// grow the fired-row buffer to hold `need` rows, keeping the first `keep` (stream idle on exit)
int ensure_out_capacity(fw_op* op, int64_t need, int64_t keep) {
  if (need <= op->out.cap) {
    set_slow_limit(op);
    return FW_OK;
  }
  const int64_t cap = std::max(need, op->out.cap * 2);
  DevRows n{};
  int64_t** cols_new[7] = {&n.key, &n.start, &n.end, &n.cnt, &n.sum, &n.mn, &n.mx};
  int64_t** cols_old[7] = {&op->out.key, &op->out.start, &op->out.end, &op->out.cnt,
                           &op->out.sum, &op->out.mn, &op->out.mx};
  keep = std::min(keep, op->out.cap);
  for (int i = 0; i < 7; i++) {
    HIP_OR_RETURN(op, dmalloc(cols_new[i], (size_t)cap));
    if (keep > 0 && *cols_old[i])
      HIP_OR_RETURN(op, hipMemcpyAsync(*cols_new[i], *cols_old[i], keep * sizeof(int64_t), hipMemcpyDeviceToDevice,
                                       op->stream));
  }
  const int64_t dstride = op->dig_stride;  // t-digest export / FW_AGG_ROW results: one record per row
  if (op->dig_stride) {
    HIP_OR_RETURN(op, dmalloc(&n.dig, (size_t)(cap * dstride)));
    if (keep > 0 && op->out.dig)
      HIP_OR_RETURN(op, hipMemcpyAsync(n.dig, op->out.dig, keep * dstride * sizeof(int64_t), hipMemcpyDeviceToDevice,
                                       op->stream));
  }
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  for (int i = 0; i < 7; i++) dfree(*cols_old[i]);
  dfree(op->out.dig);
  n.cap = cap;
  op->out = n;
  set_slow_limit(op);
  return FW_OK;
}

int ensure_side_capacity(fw_op* op, int64_t need, int64_t keep) {
  if (need <= op->side.cap) return FW_OK;
  const int64_t cap = std::max(need, op->side.cap * 2);
  DevSide n{};
  int64_t** cols_new[3] = {&n.key, &n.ts, &n.val};
  int64_t** cols_old[3] = {&op->side.key, &op->side.ts, &op->side.val};
  keep = std::min(keep, op->side.cap);
  for (int i = 0; i < 3; i++) {
    HIP_OR_RETURN(op, dmalloc(cols_new[i], (size_t)cap));
    if (keep > 0 && *cols_old[i])
      HIP_OR_RETURN(op, hipMemcpyAsync(*cols_new[i], *cols_old[i], keep * sizeof(int64_t), hipMemcpyDeviceToDevice,
                                       op->stream));
  }
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  for (int i = 0; i < 3; i++) dfree(*cols_old[i]);
  n.cap = cap;
  op->side = n;
  return FW_OK;
}

enum { K_CLASSIFY = 0, K_SCAN, K_SCATTER, K_AGGREGATE, K_SLOW, K_FIRE, K_TDIGEST };
const char* const KERNEL_NAMES[FW_NUM_KERNELS] = {"k_classify_hist", "k_scan", "k_scatter", "k_aggregate",
                                                  "k_slow",          "k_fire", "k_tdigest"};

hipEvent_t prof_event(fw_op* op) {
  if (!op->prof_free.empty()) {
    hipEvent_t e = op->prof_free.back();
    op->prof_free.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  // timing only: no system-scope fence (a cache write-back and invalidation) when the marker completes, so the
  // markers do not slow the work they bracket (fw_profile_read synchronizes the stream before reading them)
  (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  return e;
}
// time the launches issued by `launch` on the handle's stream as one interval of `kind`.  ext: `launch` issues
// exactly one kernel of the kind (fwdev::FW_LAUNCH_MAIN), timed by its dispatch's own start / stop events
// (fwdev::g_ext) instead of two marker packets around it (each pair of markers cost C2 ~10 us per step)
template <class F>
void timed(fw_op* op, int kind, F&& launch, hipStream_t on = nullptr, bool ext = false) {
  if (!((op->prof_mask >> kind) & 1u)) {
    launch();
    return;
  }
  if (!on) on = op->stream;
  fw_op::Pair pr{prof_event(op), prof_event(op), kind};
  if (ext) {
    fwdev::g_ext = fwdev::ExtTiming{pr.a, pr.b, false};
    launch();
    const bool used = fwdev::g_ext.used;
    fwdev::g_ext = fwdev::ExtTiming{};
    if (used) {
      op->prof_pending.push_back(pr);
    } else {  // (no main kernel this time: nothing to time)
      op->prof_free.push_back(pr.a);
      op->prof_free.push_back(pr.b);
    }
    return;
  }
  (void)hipEventRecord(pr.a, on);
  launch();
  (void)hipEventRecord(pr.b, on);
  op->prof_pending.push_back(pr);
}
// fold the completed intervals into the totals (intervals still in flight stay pending)
void prof_collect(fw_op* op) {
  size_t keep = 0;
  for (size_t i = 0; i < op->prof_pending.size(); i++) {
    fw_op::Pair& pr = op->prof_pending[i];
    if (hipEventQuery(pr.b) != hipSuccess) {
      op->prof_pending[keep++] = pr;
      continue;
    }
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, pr.a, pr.b) == hipSuccess) {
      op->prof_ms[pr.kind] += ms;
      op->prof_n[pr.kind]++;
    }
    op->prof_free.push_back(pr.a);
    op->prof_free.push_back(pr.b);
  }
  op->prof_pending.resize(keep);
}

// queue the status snapshot that ends a sequence
int snapshot(fw_op* op) {
  HIP_OR_RETURN(op, hipMemcpyAsync(op->h_status, op->d_status, sizeof(Status), hipMemcpyDeviceToHost, op->stream));
  HIP_OR_RETURN(op, hipEventRecord(op->snap, op->stream));
  op->unsynced = true;
  return FW_OK;
}

// status of everything queued so far (stream idle on exit)
int sync_status(fw_op* op) {
  HIP_OR_RETURN(op, hipMemcpyAsync(op->h_status, op->d_status, sizeof(Status), hipMemcpyDeviceToHost, op->stream));
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  if (!op->prof_pending.empty()) prof_collect(op);
  return FW_OK;
}

// write one field of the device status from the host copy.  Only fields no queued kernel writes
// (the suspension bookkeeping, or counters while the stream is idle) are written this way.
template <class T>
int put_status_field(fw_op* op, T Status::*field) {
  const size_t off = (size_t)((char*)&(op->h_status->*field) - (char*)op->h_status);
  HIP_OR_RETURN(op, hipMemcpyAsync((char*)op->d_status + off, (char*)op->h_status + off, sizeof(T),
                                   hipMemcpyHostToDevice, op->stream));
  return FW_OK;
}

// FW_AGG_ROW's blocks are small (a RowAcc per value column), so its pool covers every slot the table can hold (the
// regions' load limit; merged and purged windows keep their slots until k_fire rebuilds the region) and grows with
// the table: a push cannot run it dry, however few entries were expected
int64_t row_pool_blocks(const DevCfg& c) { return (int64_t)c.P * region_limit(c.log_r) + 1024; }

// the block pool to `blocks` blocks, contents, free stack and deferred list kept (stream idle)
int grow_pool(fw_op* op, int64_t blocks) {
  DevCfg& c = op->dc;
  if (blocks <= c.pool_blocks) return FW_OK;
  if (blocks >= (int64_t(1) << 32)) return set_err(op, FW_ERR_CAPACITY, "accumulator block pool would exceed 2^32 blocks");
  uint8_t* np = nullptr;
  uint32_t *nf = nullptr, *nd = nullptr;
  const size_t ob = (size_t)(c.pool_blocks * c.pool_bytes), nb = (size_t)(blocks * c.pool_bytes);
  HIP_OR_RETURN(op, dmalloc(&np, nb));
  HIP_OR_RETURN(op, dmalloc(&nf, (size_t)blocks));
  HIP_OR_RETURN(op, dmalloc(&nd, (size_t)blocks));
  HIP_OR_RETURN(op, hipMemcpyAsync(np, c.pool, ob, hipMemcpyDeviceToDevice, op->stream));
  HIP_OR_RETURN(op, hipMemsetAsync(np + ob, 0, nb - ob, op->stream));  // (blocks start at zero)
  HIP_OR_RETURN(op, hipMemcpyAsync(nf, c.pool_free, (size_t)c.pool_blocks * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                                   op->stream));
  HIP_OR_RETURN(op, hipMemcpyAsync(nd, c.pool_defer, (size_t)c.pool_blocks * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                                   op->stream));
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  dfree(c.pool);
  dfree(c.pool_free);
  dfree(c.pool_defer);
  c.pool = np;
  c.pool_free = nf;
  c.pool_defer = nd;
  c.pool_blocks = blocks;
  return FW_OK;
}

// grow every region to new_log_r, re-inserting the live entries (stream idle on exit)
int grow_table(fw_op* op, int new_log_r) {
  if (new_log_r > 30) return set_err(op, FW_ERR_CAPACITY, "state region would exceed 2^30 slots");
  DevCfg nc = op->dc;
  nc.log_r = new_log_r;
  DevTable nt{};
  nt.cur = op->tb.cur;
  nt.live = op->tb.live;
  nt.next_timer = op->tb.next_timer;
  nt.fire_e = op->tb.fire_e;
  nt.fire_lo = op->tb.fire_lo;
  nt.pane_floor = op->tb.pane_floor;
  nt.passes = op->tb.passes;
  int rc = alloc_table(op, nt, nc, false);
  if (rc) {
    free_table(nt);
    return set_err(op, FW_ERR_CAPACITY, "cannot grow the state table to %lld slots: %s",
                   (long long)((int64_t)nc.P << nc.log_r), op->err.c_str());
  }
  fwdev::launch_rehash(op->dc, op->tb, nc, nt, op->stream);
  HIP_OR_RETURN(op, hipGetLastError());
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  free_table(op->tb);
  op->tb = nt;
  op->dc = nc;
  op->table_slots = (int64_t)nc.P << nc.log_r;
  op->grows++;
  if (op->dc.agg == FW_AGG_ROW && (rc = grow_pool(op, row_pool_blocks(op->dc)))) return rc;
  if (op->dc.agg == FW_AGG_TDIGEST) {  // the compression's per-slot index follows the table
    if (op->table_slots >= (int64_t(1) << 31)) return set_err(op, FW_ERR_CAPACITY, "t-digest table would exceed 2^31 slots");
    dfree(op->td.lidx);
    HIP_OR_RETURN(op, dmalloc(&op->td.lidx, (size_t)op->table_slots));
    op->td.lidx_slots = op->table_slots;
    dfree(op->td.dcnt);  // (zero between pushes)
    HIP_OR_RETURN(op, dmalloc(&op->td.dcnt, (size_t)op->table_slots));
    HIP_OR_RETURN(op, hipMemsetAsync(op->td.dcnt, 0, (size_t)op->table_slots * sizeof(uint32_t), op->stream));
    if (op->td.mover) {  // (no override is set between pushes)
      dfree(op->td.mover);
      HIP_OR_RETURN(op, dmalloc(&op->td.mover, (size_t)op->table_slots));
      HIP_OR_RETURN(op, hipMemsetAsync(op->td.mover, 0xff, (size_t)op->table_slots * sizeof(int32_t), op->stream));
    }
    if (op->dc.td_olast) {  // a push's late-firing chains, mid-push (settle): relinked over the moved slots
      dfree(op->dc.td_olast);
      HIP_OR_RETURN(op, dmalloc(&op->dc.td_olast, (size_t)op->table_slots));
      HIP_OR_RETURN(op, hipMemsetAsync(op->dc.td_olast, 0xff, (size_t)op->table_slots * sizeof(int32_t), op->stream));
      fwdev::launch_td_relink(op->dc, op->tb, op->stream);
      HIP_OR_RETURN(op, hipGetLastError());
    }
  }
  const int64_t rows = (int64_t)op->h_status->out_rows;
  return ensure_out_capacity(op, rows + op->table_slots, rows);
}

// smallest region size whose load limit leaves half the region free for `need` occupied slots
int log_r_for(const fw_op* op, int64_t need) {
  int log_r = op->dc.log_r + 1;
  while ((int64_t(1) << log_r) < 2 * need) log_r++;
  return log_r;
}

// Wait for the queued sequence and settle it (see the file comment).  Kernels queued after the
// snapshot (the next push's classify / scan / scatter) may still be running: they use the other
// scratch set and write no status field that is rewritten here.
int settle(fw_op* op) {
  if (!op->unsynced) return FW_OK;
  HIP_OR_RETURN(op, hipEventSynchronize(op->snap));
  if (!op->prof_pending.empty()) prof_collect(op);
  Status& s = *op->h_status;
  int rc;
  int rounds = 0;
  while (s.suspended) {
    if (++rounds > 64) return set_err(op, FW_ERR_STATE, "suspended push did not complete after 64 resumptions");
    op->resumptions++;
    const int susp = s.suspended;
    if (susp == FW_SUSP_FIRE) {  // pane windows did not fit the fired-row buffer: grow it and fire again
      if ((rc = ensure_out_capacity(op, std::max<int64_t>(2 * op->out.cap, (int64_t)s.need_out + op->table_slots),
                                    (int64_t)s.out_rows)))
        return rc;
      s.suspended = 0;
      s.need_out = 0;
      if ((rc = put_status_field(op, &Status::suspended)) || (rc = put_status_field(op, &Status::need_out))) return rc;
      timed(op, K_FIRE, [&] { fwdev::launch_fire(op->dc, op->wm, op->tb, op->out, op->d_status, op->stream); });
      HIP_OR_RETURN(op, hipGetLastError());
      if ((rc = sync_status(op))) return rc;
      continue;
    }
    if (s.need_live > region_limit(op->dc.log_r) && (rc = grow_table(op, log_r_for(op, s.need_live)))) return rc;
    if (s.need_out > op->out.slow_limit &&
        (rc = ensure_out_capacity(op, (int64_t)s.need_out + op->table_slots, (int64_t)s.out_rows)))
      return rc;
    s.suspended = 0;
    s.need_live = 0;
    s.need_out = 0;
    if ((rc = put_status_field(op, &Status::suspended)) || (rc = put_status_field(op, &Status::need_live)) ||
        (rc = put_status_field(op, &Status::need_out)))
      return rc;
    const Scratch& S = op->sc[op->last_sc];
    DevCfg c = op->dc;
    c.slow_ord = S.so;
    c.by_val = S.byv;
    c.compact = S.compact;
    c.cbase = S.cbase;
    c.narrow = S.narrow;
    c.ndn0 = S.ndn0;
    c.ord_base = S.ord_base;
    c.wide = S.wide_word(op->dc.P);
    c.row_cols = S.rowc;
    c.row_nulls = S.rown;
    c.row_stride = op->max_batch;
    if (S.partials) {  // a partials push: only its merge can have suspended
      c.nt_floor = fwdev::pane_nt_floor(c, S.wm);  // (panes: a new pane's first window)
      timed(op, K_AGGREGATE, [&] {
        fwdev::launch_pmerge(c, S.pparts, S.hist, S.T, op->tb, op->prog, 1, op->d_status, op->stream);
        if (S.hregs)  // (register max is idempotent: the whole push's registers again)
          fwdev::launch_hll_push_regs(c, S.wm, S.hin, S.hn, S.hregs, S.hoff, op->tb, op->d_status, op->stream);
      });
      if (op->fire_unsettled)
        timed(op, K_FIRE, [&] { fwdev::launch_fire(c, op->wm, op->tb, op->out, op->d_status, op->stream); });
      HIP_OR_RETURN(op, hipGetLastError());
      if ((rc = sync_status(op))) return rc;
      continue;
    }
    if (susp & FW_SUSP_AGG)
      timed(op, K_AGGREGATE, [&] {
        fwdev::launch_aggregate(c, S.wm, S.part, S.offs(), S.offT(), op->tb, op->prog, 1, S.split ? &op->hot : nullptr,
                                S.n, op->d_status, op->stream, nullptr, 0, S.single ? S.rsv : nullptr, op->rcap);
        // the update skipped itself behind the suspension; register max is idempotent, so it reruns whole (and the
        // Table aggregates' adds, which are not, never started)
        if (c.agg == FW_AGG_HLL)
          fwdev::launch_hll_update(c, S.part, S.offs(), S.offT(), S.n, op->tb, op->d_status, op->stream);
        if (c.agg == FW_AGG_ROW)
          fwdev::launch_row_update(c, S.part, S.offs(), S.offT(), S.n, op->tb, op->d_status, op->stream);
      });
    // after an aggregate suspension the ordered path never started; otherwise it resumes
    if (!c.dense) timed(op, K_SLOW, [&] {
      fwdev::launch_slow(c, S.wm, S.srow(op->dc.P), S.T, S.sk, S.stt, S.sv, S.skh, op->tb, op->out, op->side, op->d_status,
                         (susp & FW_SUSP_AGG) ? 0 : 1, op->stream);
    });
    // the t-digest compression skipped itself behind the suspension (it runs once, after the aggregate and the
    // ordered path completed)
    if ((susp & (FW_SUSP_AGG | FW_SUSP_SLOW)) && c.agg == FW_AGG_TDIGEST)
      timed(op, K_TDIGEST, [&] {
        fwdev::launch_tdigest(c, S.part, S.offs(), S.offT(), S.n, op->tb, op->td, op->d_status, op->stream);
      });
    // a watermark queued behind the push skipped itself; firing at the latest one is the same as
    // firing at each (nothing was pushed in between)
    if (op->fire_unsettled)
      timed(op, K_FIRE, [&] { fwdev::launch_fire(c, op->wm, op->tb, op->out, op->d_status, op->stream); });
    HIP_OR_RETURN(op, hipGetLastError());
    if ((rc = sync_status(op))) return rc;
  }
  if (rounds && op->sc[op->last_sc].single) {
    // the suspended push's aggregate left its single-pass words for the resumption (k_rsv_reset skips behind a
    // suspension): zero them now, before the set's next batch (which waits for ev_done)
    Scratch& L = op->sc[op->last_sc];
    HIP_OR_RETURN(op, hipMemsetAsync(L.rsv, 0, ((size_t)op->dc.P + FW_RSV_WORDS) * sizeof(uint32_t), op->stream));
    HIP_OR_RETURN(op, hipEventRecord(op->ev_done[op->last_sc], op->stream));
  }
  op->unsynced = op->push_unsettled = op->fire_unsettled = false;
  if (s.narrow_misses != op->narrow_seen) {  // a stream with wide keys or values keeps them: 16-byte records on
    op->narrow_seen = s.narrow_misses;
    op->narrow_off = true;
  }
  if (s.rsv_fallbacks != op->rsv_seen) {  // single-pass batches redone: a skewed stream stops trying after 3 in a row
    op->rsv_seen = s.rsv_fallbacks;
    if (++op->rsv_misses >= 3) op->rsv_off = true;
  } else {
    op->rsv_misses = 0;
  }
  if (op->clear_deferred) {
    // rows the next push's scatter may have added since are side rows; side output never queues
    // early (push_device), so both counts are exactly those of the cleared sequence
    op->out_base = (int64_t)s.out_rows;
    op->side_base = (int64_t)s.side_rows;
    op->clear_deferred = false;
  }
  if (s.flags & FW_STATUS_STATE_LOST)
    return set_err(op, FW_ERR_CAPACITY, "a window could not be stored (state region full)");
  if (s.flags & FW_STATUS_OUT_FULL) return set_err(op, FW_ERR_STATE, "fired-row buffer overflow");
  if (s.flags & FW_STATUS_TD_UNION)
    return set_err(op, FW_ERR_CAPACITY, "a late session firing joined more than %d t-digest centroids in one push",
                   op->dc.td_lateu_cap);
  if (s.flags & FW_STATUS_POOL)
    return set_err(op, FW_ERR_CAPACITY, "accumulator block pool exhausted (%lld blocks; raise expected_entries)",
                   (long long)op->dc.pool_blocks);
  if (s.flags & FW_STATUS_SIDE_FULL) return set_err(op, FW_ERR_STATE, "side-output buffer overflow");
  if (s.kg_errors) return set_err(op, FW_ERR_KEY_GROUP, "%d record(s) outside KeyGroupRange [%d, %d]", s.kg_errors,
                                   op->dc.kg0, op->dc.kg0 + op->dc.n_kg - 1);
  if (s.ts_errors)
    return set_err(op, FW_ERR_NO_TIMESTAMP,
                   "Record has Long.MIN_VALUE timestamp (= no timestamp marker). Is the time characteristic set to "
                   "'ProcessingTime', or did you forget to call 'DataStream.assignTimestampsAndWatermarks(...)'?");
  if (s.flags & FW_STATUS_MERGE_LATE)
    return set_err(op, FW_ERR_UNSUPPORTED,
                   "The end timestamp of an event-time window cannot become earlier than the current watermark by "
                   "merging. Current watermark: %lld",
                   (long long)op->wm);
  if (s.need_grow) {  // grow ahead of need, before a region has to suspend
    if ((rc = grow_table(op, op->dc.log_r + 1))) return rc;
    s.need_grow = 0;
    if ((rc = put_status_field(op, &Status::need_grow))) return rc;
  }
  return FW_OK;
}

// rows handed out are forgotten lazily: the counters restart at 0 once everything was consumed
// and the buffer is a quarter full (one status write every few watermarks, not per call).
// Settled only; no queued kernel writes these counters (side output never queues early).
int maybe_restart_rows(fw_op* op) {
  Status& s = *op->h_status;
  int rc;
  if (op->out_base == (int64_t)s.out_rows && s.out_rows > 0 && (int64_t)s.out_rows > op->out.cap / 4) {
    s.out_rows = 0;
    op->out_base = 0;
    if ((rc = put_status_field(op, &Status::out_rows))) return rc;
  }
  if (op->side_base == (int64_t)s.side_rows && s.side_rows > 0 && (int64_t)s.side_rows > op->side.cap / 4) {
    s.side_rows = 0;
    op->side_base = 0;
    if ((rc = put_status_field(op, &Status::side_rows))) return rc;
  }
  return FW_OK;
}

// FW_COUNT: count windows fire while the batch is processed; no state table, timers or suspension
int push_count(fw_op* op, const int64_t* key, const int64_t* val, int64_t n) {
  int rc;
  if ((rc = settle(op)) || (rc = maybe_restart_rows(op))) return rc;
  const int64_t rows = (int64_t)op->h_status->out_rows;
  // a key fires at most ceil(r / slide) times for its r elements of the batch
  const int64_t most = std::min<int64_t>(n, n / op->cw.slide + std::min<int64_t>(n, op->cw.max_keys));
  if ((rc = ensure_out_capacity(op, rows + most, rows)))
    return rc;
  DevCfg c = op->dc;
  c.ord_base = op->records_in;
  fwdev::launch_count(c, op->cw, key, val, n, op->out, op->d_status, op->stream);
  HIP_OR_RETURN(op, hipGetLastError());
  op->records_in += n;
  op->push_unsettled = true;
  return snapshot(op);
}

hipStream_t input_stream_of(const fw_op* op);  // the stream device pushes read their columns on
// FW_AGG_ROW input of a push: the caller's columns (column j of the push's record i at cols[j * stride + i]) and NULL
// masks (nullptr = none)
struct RowIn {
  const int64_t* cols;
  const uint8_t* nulls;
  int64_t stride;
};
int push_device(fw_op* op, const int64_t* key, const int64_t* ts, const int64_t* val, const int32_t* kh, int64_t n,
                bool async_ok, const RowIn* rin = nullptr) {
  if (n == 0) return FW_OK;
  if ((op->dc.agg == FW_AGG_ROW) != (rin != nullptr))
    return set_err(op, FW_ERR_ARG, rin ? "fw_push_row_batch needs an FW_AGG_ROW operator"
                                       : "an FW_AGG_ROW operator takes its records through fw_push_row_batch");
  if (op->cfg.assigner == FW_COUNT) return push_count(op, key, val, n);
  int rc;
  DevCfg c = op->dc;  // by value: a session batch stamps its taint epoch into it
  // queue the batch-only kernels before waiting for the previous sequence, except with side
  // output (the scatter appends late records to the side buffer, whose capacity and counters the
  // settle below must see unchanged)
  const bool early = op->unsynced && !c.side_output;
  if (!early && (rc = settle(op))) return rc;
  if (!early && c.side_output) {
    const int64_t rows = (int64_t)op->h_status->side_rows;
    if ((rc = ensure_side_capacity(op, rows + n, rows))) return rc;
  }
  const int nxt = op->last_sc ^ 1;
  Scratch& S = op->sc[nxt];
  c.ord_base = op->records_in;  // FW_AGG_FIRST: arrival ordinals of this batch start here
  c.slow_ord = S.so;
  c.wide = S.wide;
  auto aligned = [](const void* p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; };
  c.vec_in = aligned(key, 16) && aligned(ts, 16) && aligned(val, 16) && (!kh || aligned(kh, 8));
  if (c.compact) {
    // compact records: window deltas count from 2^(log_s - 1) windows (or panes) before the watermark's,
    // so the batch's windows on both sides of the watermark fit; no base for a watermark near Long.MIN_VALUE
    const __int128 u = c.slide, w = op->wm, off = c.offset;
    __int128 q = (w - off) / u;
    if ((w - off) % u < 0) q -= 1;  // floor
    const __int128 base = q * u + off - ((__int128)1 << (c.log_s - 1)) * u;
    if (base < (__int128)INT64_MIN || base > (__int128)INT64_MAX)
      c.compact = 0;
    else
      c.cbase = (int64_t)base;
  }
  const bool gather = S.rt && fwdev::gather_mode(c, n);
  const bool single = !gather && S.rsv && !op->rsv_off && op->rcap > 0 && fwdev::rsv_eligible(c);
  // narrow records: integer fields only (a narrow value is an int32), compact windows from the watermark's on
  static const bool no_narrow = getenv("FW_NO_NARROW") && atoi(getenv("FW_NO_NARROW"));
  c.narrow = single && !op->narrow_off && c.vtype != FW_VAL_F64 && c.log_s >= 1 && !no_narrow;
  c.ndn0 = c.narrow ? 1 << (c.log_s - 1) : 0;
  const int32_t T = gather ? (int32_t)((n + FW_GTILE - 1) / FW_GTILE) : (int32_t)((n + FW_TILE - 1) / FW_TILE);
  const int64_t m = (int64_t)(c.P + 1) * T;
  // async input: the batch-only kernels run on bstream, after the aggregate that last used this scratch set
  // (the same predicate as fw_input_stream, which the caller ordered its producer before: a batch that is not
  // gathered while gather scratch exists stays on the operator's stream)
  const bool two = async_ok && input_stream_of(op) == op->bstream && !gather;
  hipStream_t bs = two ? op->bstream : op->stream;
  if (two) HIP_OR_RETURN(op, hipStreamWaitEvent(bs, op->ev_done[nxt], 0));
  if (c.assigner == FW_SESSION) {
    // a new epoch empties the taint set; its slots are cleared only when the epochs wrap
    if (++op->taint_epoch >= 0x80000000u) {
      HIP_OR_RETURN(op, hipMemsetAsync(c.taint_state, 0, ((size_t)c.taint_mask + 1) * sizeof(uint32_t), bs));
      op->taint_epoch = 1;
    }
    c.taint_epoch = op->taint_epoch;
    HIP_OR_RETURN(op, hipMemsetAsync(&op->d_status->taint_any, 0, sizeof(int32_t), bs));
  }
  if (single) c.wide = reinterpret_cast<int32_t*>(S.rsv + c.P + FW_RSV_WIDE);  // (zero with the rest of rsv)
  else if (c.compact) HIP_OR_RETURN(op, hipMemsetAsync(S.wide, 0, sizeof(int32_t), bs));
  if (gather) {
    // classify, tile-local partition sort, runs table, ordered-path compaction: one pass over the input
    timed(op, K_SCATTER, [&] {
      fwdev::launch_stage(c, op->wm, key, ts, val, kh, n, S.part, op->max_batch, S.rt, S.rt_t, S.voffs, S.gsrow, S.gcb, S.sk,
                          S.stt, S.sv, S.skh, op->side, op->d_status, op->stream);
    });
  } else {
    // dense compact batches: one pass reserves each partition's run piece by piece; the classify / scan /
    // offset-scatter sequence behind it runs only when that pass could not take the batch (a record without a
    // compact form, a run beyond rcap)
    if (single) {  // (rsv is zero: reset behind the set's previous aggregate, k_rsv_reset, or by settle)
      timed(op, K_SCATTER, [&] { fwdev::launch_scatter_rsv(c, op->wm, key, ts, val, kh, n, T, S.part, S.rsv, op->rcap, bs); },
            bs, true);
    }
    const uint32_t* gate = single ? S.rsv + c.P : nullptr;
    if (single) {  // (fw_profile: the gated sequence counts as classify)
      timed(
          op, K_CLASSIFY,
          [&] {
            fwdev::launch_classify_hist(c, op->wm, key, ts, kh, n, T, S.hist, op->d_status, bs, S.rsv);
            fwdev::launch_scan(S.hist, m, S.scan_tmp, bs, gate);
            fwdev::launch_scatter(c, op->wm, key, ts, val, kh, n, T, S.hist, S.part, S.sk, S.stt, S.sv, S.skh, op->side,
                                  op->d_status, bs, gate);
          },
          bs);
    } else {
      timed(
          op, K_CLASSIFY,
          [&] {
            if (c.assigner == FW_SESSION) fwdev::launch_taint(c, op->wm, key, ts, n, op->d_status, bs);
            fwdev::launch_classify_hist(c, op->wm, key, ts, kh, n, T, S.hist, op->d_status, bs);
          },
          bs);
      timed(op, K_SCAN, [&] { fwdev::launch_scan(S.hist, m, S.scan_tmp, bs); }, bs);
      timed(
          op, K_SCATTER,
          [&] {
            fwdev::launch_scatter(c, op->wm, key, ts, val, kh, n, T, S.hist, S.part, S.sk, S.stt, S.sv, S.skh, op->side,
                                  op->d_status, bs);
          },
          bs);
    }
  }
  S.single = single;
  op->single_batches += single;
  op->narrow_batches += c.narrow;
  S.gather = gather;
  S.T = T;
  // minBy / maxBy: the aggregate reads the selected elements' fields back by batch index, possibly after the
  // caller's columns are gone (a resumed push), so the batch keeps its own copy
  if (S.byv) HIP_OR_RETURN(op, hipMemcpyAsync(S.byv, val, n * sizeof(int64_t), hipMemcpyDeviceToDevice, bs));
  HIP_OR_RETURN(op, hipGetLastError());
  if (two) {  // the batch's aggregate waits for its scatter
    HIP_OR_RETURN(op, hipEventRecord(op->ev_scat[nxt], bs));
    HIP_OR_RETURN(op, hipStreamWaitEvent(op->stream, op->ev_scat[nxt], 0));
  }
  if (S.rowc) {  // FW_AGG_ROW: the batch's columns and NULL masks, kept by the set (a resumed push reads them again)
    HIP_OR_RETURN(op, hipMemcpy2DAsync(S.rowc, (size_t)op->max_batch * sizeof(int64_t), rin->cols,
                                       (size_t)rin->stride * sizeof(int64_t), (size_t)n * sizeof(int64_t),
                                       (size_t)op->dc.row_nc, hipMemcpyDefault, op->stream));
    if (rin->nulls)
      HIP_OR_RETURN(op, hipMemcpyAsync(S.rown, rin->nulls, (size_t)n, hipMemcpyDefault, op->stream));
    else
      HIP_OR_RETURN(op, hipMemsetAsync(S.rown, 0, (size_t)n, op->stream));
  }
  if (early && (rc = settle(op))) return rc;
  if ((rc = maybe_restart_rows(op))) return rc;
  // the ordered path checks its room per chunk and suspends when it runs out; one chunk always fits
  const int64_t rows = (int64_t)op->h_status->out_rows;
  const int64_t chunk_rows = (int64_t)FW_SLOW_THREADS * (c.assigner == FW_SESSION ? 1 : c.wpr);
  if ((rc = ensure_out_capacity(op, rows + op->table_slots + chunk_rows, rows))) return rc;
  DevCfg cc = op->dc;  // settle may have grown the table
  cc.ord_base = c.ord_base;
  cc.slow_ord = S.so;
  cc.by_val = S.byv;
  cc.compact = c.compact;
  cc.cbase = c.cbase;
  cc.narrow = c.narrow;
  cc.ndn0 = c.ndn0;
  cc.wide = c.wide;
  cc.row_cols = S.rowc;
  cc.row_nulls = S.rown;
  cc.row_stride = op->max_batch;
  // a partition can outgrow one aggregate workgroup (hot keys) only when the batch is longer than a chunk
  const bool split = !cc.dense && (cc.wpr == 1 || cc.panes) && n > cc.agg_chunk;
  if (split && (rc = ensure_hot(op))) return rc;
  if (cc.agg == FW_AGG_TDIGEST && cc.assigner == FW_SESSION) {  // the push's merge log and ordered values start empty
    HIP_OR_RETURN(op, hipMemsetAsync(cc.td_mctr, 0, sizeof(int32_t), op->stream));
    HIP_OR_RETURN(op, hipMemsetAsync(cc.td_ovctr, 0, sizeof(int32_t), op->stream));
    HIP_OR_RETURN(op, hipMemsetAsync(op->td.uctr, 0, 2 * sizeof(unsigned long long), op->stream));
  }
  if (cc.agg == FW_AGG_TDIGEST && cc.td_olast) {  // (allowed lateness) ... and no window has a chain yet
    HIP_OR_RETURN(op, hipMemsetAsync(cc.td_ovctr, 0, sizeof(int32_t), op->stream));
    HIP_OR_RETURN(op, hipMemsetAsync(cc.td_olast, 0xff, (size_t)op->table_slots * sizeof(int32_t), op->stream));
    if (cc.td_bhead)  // (sessions: no block has merged blocks yet)
      HIP_OR_RETURN(op, hipMemsetAsync(cc.td_bhead, 0xff, (size_t)cc.pool_blocks * sizeof(int32_t), op->stream));
  }
  timed(
      op, K_AGGREGATE,
      [&] {
        fwdev::launch_aggregate(cc, op->wm, S.part, S.offs(), S.offT(), op->tb, op->prog, 0, split ? &op->hot : nullptr,
                                n, op->d_status, op->stream, nullptr, 0, single ? S.rsv : nullptr, op->rcap);
        if (cc.agg == FW_AGG_HLL)
          fwdev::launch_hll_update(cc, S.part, S.offs(), S.offT(), n, op->tb, op->d_status, op->stream);
        if (cc.agg == FW_AGG_ROW)
          fwdev::launch_row_update(cc, S.part, S.offs(), S.offT(), n, op->tb, op->d_status, op->stream);
      },
      nullptr, cc.dense);  // (the dense aggregate is one kernel)
  if (single) fwdev::launch_rsv_reset(S.rsv, cc.P + FW_RSV_WORDS, op->d_status, op->stream);
  if (!cc.dense)  // (tumbling windows without allowed lateness: no record needs arrival order)
    timed(op, K_SLOW, [&] {
      fwdev::launch_slow(cc, op->wm, S.srow(cc.P), S.T, S.sk, S.stt, S.sv, S.skh, op->tb, op->out, op->side, op->d_status,
                         0, op->stream);
    });
  // the t-digest compression closes the push: after the ordered path too (sessions: its merges and added values)
  if (cc.agg == FW_AGG_TDIGEST)
    timed(op, K_TDIGEST, [&] {
      fwdev::launch_tdigest(cc, S.part, S.offs(), S.offT(), n, op->tb, op->td, op->d_status, op->stream);
    });
  HIP_OR_RETURN(op, hipGetLastError());
  HIP_OR_RETURN(op, hipEventRecord(op->ev_done[nxt], op->stream));  // the set's last use by this batch (see settle)
  S.T = T;
  S.n = n;
  S.partials = false;
  S.split = split;
  S.wm = op->wm;
  S.compact = c.compact;
  S.cbase = c.cbase;
  S.narrow = c.narrow;
  S.ndn0 = c.ndn0;
  S.ord_base = c.ord_base;
  op->last_sc = nxt;
  op->records_in += n;
  op->push_unsettled = true;
  return snapshot(op);
}


// ---- pre-shuffle combining (fw_combine_extract_device / fw_push_partials_device)
// tumbling windows, or sliding windows kept as panes (size % slide == 0): a pane's partial is classified by its
// start exactly as each of its elements is (they all share the pane's newest window), so merging it at the receiver
// equals pushing its records (round 4)
bool combine_eligible(const fw_config& c) {
  const bool panes = c.assigner == FW_SLIDING && c.slide > 0 && c.size > c.slide && c.size % c.slide == 0 &&
                     !(getenv("FW_NO_PANES") && atoi(getenv("FW_NO_PANES")));
  return (c.assigner == FW_TUMBLING || panes) && c.aggregate == FW_AGG_COUNT_SUM_MIN_MAX &&
         c.allowed_lateness == 0 && !c.side_output && (c.key_kind == FW_KEY_LONG || c.key_kind == FW_KEY_INT);
}
// HyperLogLog partials (register lists): tumbling windows, no allowed lateness, Long or Integer keys
bool combine_eligible_hll(const fw_config& c) {
  return c.assigner == FW_TUMBLING && c.aggregate == FW_AGG_HLL && c.allowed_lateness == 0 && !c.side_output &&
         (c.key_kind == FW_KEY_LONG || c.key_kind == FW_KEY_INT);
}
// what a partial's representation depends on (fw_partials.config); never 0, so a zeroed struct never matches
uint64_t combine_config_tag(const fw_config& c) {
  const int64_t f[] = {c.assigner, c.size, c.offset, c.value_type, c.key_kind, c.max_parallelism, c.aggregate,
                       c.assigner == FW_SLIDING ? c.slide : 0,
                       c.aggregate == FW_AGG_HLL ? (c.hll_precision ? c.hll_precision : 14) : 0};
  uint64_t h = 0x9E3779B97F4A7C15ull;
  for (int64_t x : f) {
    h ^= (uint64_t)x + 0x632BE59BD9B4E019ull + (h << 6) + (h >> 2);
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
  }
  return h | 1;
}
int push_partials(fw_op* op, const PartialCols& in, int64_t n, const uint32_t* hregs = nullptr,
                  const uint32_t* hoff = nullptr) {
  int rc;
  if ((rc = settle(op)) || (rc = maybe_restart_rows(op))) return rc;
  const int nxt = op->last_sc ^ 1;
  Scratch& S = op->sc[nxt];
  if (!S.pparts) HIP_OR_RETURN(op, dmalloc(&S.pparts, (size_t)op->max_batch));
  DevCfg c = op->dc;
  c.compact = 0;
  c.wide = S.wide;
  const int32_t T = (int32_t)((n + FW_TILE - 1) / FW_TILE);
  const int64_t m = (int64_t)(c.P + 1) * T;
  // the partials' partitions and classes, their window start standing for the timestamp
  timed(op, K_CLASSIFY, [&] {
    fwdev::launch_classify_hist(c, op->wm, in.key, in.start, nullptr, n, T, S.hist, op->d_status, op->stream);
  });
  timed(op, K_SCAN, [&] { fwdev::launch_scan(S.hist, m, S.scan_tmp, op->stream); });
  timed(op, K_SCATTER, [&] {
    fwdev::launch_pscatter(c, op->wm, in, n, T, S.hist, S.pparts, op->d_status, op->stream);
  });
  c.nt_floor = fwdev::pane_nt_floor(c, op->wm);  // (panes: a new pane's first window, lds_delta)
  timed(op, K_AGGREGATE, [&] {
    fwdev::launch_pmerge(c, S.pparts, S.hist, T, op->tb, op->prog, 0, op->d_status, op->stream);
    // HyperLogLog: the partials' registers into their windows' blocks (skipped behind a suspended merge)
    if (hregs) fwdev::launch_hll_push_regs(c, op->wm, in, n, hregs, hoff, op->tb, op->d_status, op->stream);
  });
  HIP_OR_RETURN(op, hipGetLastError());
  HIP_OR_RETURN(op, hipEventRecord(op->ev_done[nxt], op->stream));
  S.hin = in;
  S.hn = n;
  S.hregs = hregs;
  S.hoff = hoff;
  S.T = T;
  S.n = n;
  S.partials = true;
  S.single = false;
  S.split = false;
  S.gather = false;
  S.wm = op->wm;
  S.compact = 0;
  S.cbase = 0;
  S.narrow = 0;
  S.ord_base = op->records_in;
  op->last_sc = nxt;
  op->push_unsettled = true;
  return snapshot(op);
}
}  // namespace

// ============================================================================ C-ABI
extern "C" {

int fw_create(const fw_config* cfg_in, fw_op** out) {
  if (!cfg_in || !out) return FW_ERR_ARG;
  *out = nullptr;
  fw_config cfg = *cfg_in;
  char msg[256] = {0};
  // argument checks mirror the reference's constructors
  if (cfg.assigner == FW_TUMBLING) {
    if (cfg.size <= 0 || cfg.offset < 0 || cfg.offset >= cfg.size)
      snprintf(msg, sizeof msg, "TumblingEventTimeWindows parameters must satisfy 0 <= offset < size");
    cfg.slide = cfg.size;
  } else if (cfg.assigner == FW_SLIDING) {
    if (cfg.offset < 0 || cfg.offset >= cfg.slide || cfg.size <= 0 || cfg.slide <= 0)
      snprintf(msg, sizeof msg,
               "SlidingEventTimeWindows parameters must satisfy 0 <= offset < slide and size > 0");
    else if ((cfg.size + cfg.slide - 1) / cfg.slide > (1 << 20))
      snprintf(msg, sizeof msg, "a sliding window may overlap at most 2^20 others (size / slide)");
  } else if (cfg.assigner == FW_SESSION) {
    if (cfg.gap <= 0) snprintf(msg, sizeof msg, "EventTimeSessionWindows parameters must satisfy 0 < size");
  } else if (cfg.assigner == FW_COUNT) {
    if (cfg.size <= 0 || cfg.slide <= 0 || cfg.size > (1 << 16) || cfg.slide > (1 << 16))
      snprintf(msg, sizeof msg, "count windows need 0 < size <= 65536 and 0 < slide <= 65536");
    else if (cfg.aggregate != FW_AGG_FIRST)
      snprintf(msg, sizeof msg, "count windows are offered for countWindow(size, slide).sum(pos) (FW_AGG_FIRST)");
  } else {
    snprintf(msg, sizeof msg, "unknown assigner %d", cfg.assigner);
  }
  if (!msg[0] && cfg.allowed_lateness < 0) snprintf(msg, sizeof msg, "The allowed lateness cannot be negative.");
  if (!msg[0] && (cfg.value_type < FW_VAL_I64 || cfg.value_type > FW_VAL_F32))
    snprintf(msg, sizeof msg, "unknown value type %d", cfg.value_type);
  if (!msg[0] && (cfg.key_kind < FW_KEY_LONG || cfg.key_kind > FW_KEY_HASHED))
    snprintf(msg, sizeof msg, "unknown key kind %d", cfg.key_kind);
  if (cfg.max_parallelism == 0) cfg.max_parallelism = 128;
  if (!msg[0] && (cfg.max_parallelism < 1 || cfg.max_parallelism > (1 << 15)))
    snprintf(msg, sizeof msg, "Operator parallelism not within bounds: %d", cfg.max_parallelism);
  if (cfg.key_group_start < 0 && cfg.key_group_end < 0) {
    cfg.key_group_start = 0;
    cfg.key_group_end = cfg.max_parallelism - 1;
  }
  if (!msg[0] && (cfg.key_group_start < 0 || cfg.key_group_end < cfg.key_group_start ||
                  cfg.key_group_end >= cfg.max_parallelism))
    snprintf(msg, sizeof msg, "invalid KeyGroupRange [%d, %d]", cfg.key_group_start, cfg.key_group_end);
  if (!msg[0] && cfg.sub_partitions != 0 && (cfg.sub_partitions & (cfg.sub_partitions - 1)))
    snprintf(msg, sizeof msg, "sub_partitions must be a power of two");
  if (!msg[0] && (cfg.aggregate < FW_AGG_COUNT_SUM_MIN_MAX || cfg.aggregate > FW_AGG_ROW))
    snprintf(msg, sizeof msg, "unknown aggregate %d", cfg.aggregate);
  const int32_t hll_p = cfg.hll_precision ? cfg.hll_precision : 14;
  if (!msg[0] && cfg.aggregate == FW_AGG_HLL && (hll_p < 4 || hll_p > 16))
    snprintf(msg, sizeof msg, "HyperLogLog precision must be in [4, 16], got %d", hll_p);
  bool unsupported = false;
  if (!msg[0] && cfg.aggregate == FW_AGG_HLL &&
      ((cfg.assigner != FW_TUMBLING && cfg.assigner != FW_SLIDING && cfg.assigner != FW_SESSION) ||
       cfg.value_type != FW_VAL_I64)) {
    snprintf(msg, sizeof msg, "the HyperLogLog aggregate is offered for tumbling, sliding and session windows over a "
                              "Long item column");
    unsupported = true;
  }
  const int32_t td_delta = cfg.tdigest_compression ? cfg.tdigest_compression : 100;
  if (cfg.aggregate == FW_AGG_TDIGEST && cfg.tdigest_quantiles[0] == 0 && cfg.tdigest_quantiles[1] == 0 &&
      cfg.tdigest_quantiles[2] == 0) {
    cfg.tdigest_quantiles[0] = 0.5;
    cfg.tdigest_quantiles[1] = 0.95;
    cfg.tdigest_quantiles[2] = 0.99;
  }
  if (!msg[0] && cfg.aggregate == FW_AGG_TDIGEST && (td_delta < 10 || td_delta > 500 || (td_delta & 1)))
    snprintf(msg, sizeof msg, "t-digest compression must be even and in [10, 500], got %d", td_delta);
  for (int i = 0; i < 3 && !msg[0] && cfg.aggregate == FW_AGG_TDIGEST; i++)
    if (!(cfg.tdigest_quantiles[i] >= 0.0 && cfg.tdigest_quantiles[i] <= 1.0))
      snprintf(msg, sizeof msg, "t-digest quantiles must be in [0, 1]");
  if (!msg[0] && cfg.aggregate == FW_AGG_TDIGEST && cfg.value_type != FW_VAL_F64) {
    snprintf(msg, sizeof msg, "the t-digest aggregate is offered over a Double field");
    unsupported = true;
  }
  if (!msg[0] && cfg.aggregate == FW_AGG_TDIGEST && cfg.assigner == FW_SLIDING && cfg.slide > 0 &&
      (cfg.size + cfg.slide - 1) / cfg.slide > 4096) {
    snprintf(msg, sizeof msg, "the t-digest aggregate takes at most 4096 windows per element");
    unsupported = true;
  }
  if (!msg[0] && cfg.aggregate == FW_AGG_ROW) {
    // the Table API's group windows (DataStreamGroupWindowAggregate.scala:197-294): event-time tumbling / sliding /
    // session windows with the assigner's EventTimeTrigger, no allowed lateness and no side output
    if (cfg.row_columns < 1 || cfg.row_columns > 8 || cfg.row_aggregates < 1 || cfg.row_aggregates > 16) {
      snprintf(msg, sizeof msg, "FW_AGG_ROW needs 1 .. 8 value columns and 1 .. 16 aggregates");
    } else {
      for (int j = 0; j < cfg.row_columns && !msg[0]; j++)
        if (cfg.row_column_type[j] < FW_VAL_I64 || cfg.row_column_type[j] > FW_VAL_F32)
          snprintf(msg, sizeof msg, "FW_AGG_ROW: unknown type %d of column %d", cfg.row_column_type[j], j);
      for (int q = 0; q < cfg.row_aggregates && !msg[0]; q++) {
        const int fn = cfg.row_aggregate[q] >> 8, col = cfg.row_aggregate[q] & 0xff;
        if (fn < FW_ROW_COUNT_STAR || fn > FW_ROW_AVG || col >= cfg.row_columns)
          snprintf(msg, sizeof msg, "FW_AGG_ROW: aggregate %d is not FW_ROW_* << 8 | column", q);
      }
    }
    if (!msg[0] && (cfg.assigner == FW_COUNT || cfg.allowed_lateness != 0 || cfg.purging || cfg.side_output)) {
      snprintf(msg, sizeof msg, "FW_AGG_ROW is offered for the Table API's event-time group windows: tumbling, sliding "
                                "or session windows, EventTimeTrigger, no allowed lateness, no side output");
      unsupported = true;
    }
  }
  if (!msg[0] && cfg.aggregate >= FW_AGG_FIRST && cfg.aggregate <= FW_AGG_FIRST_MAX && cfg.assigner == FW_SLIDING && cfg.slide > 0 &&
      (cfg.size + cfg.slide - 1) / cfg.slide > 65535) {
    snprintf(msg, sizeof msg, "the first-element aggregate takes at most 65535 windows per element");
    unsupported = true;
  }
  fw_op* op = new fw_op();
  op->cfg = cfg;
  if (msg[0]) {
    op->err = msg;
    *out = op;
    return unsupported ? FW_ERR_UNSUPPORTED : FW_ERR_ARG;
  }
  *out = op;
  op->device = cfg.device;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  HIP_OR_RETURN(op, hipStreamCreateWithFlags(&op->stream, hipStreamNonBlocking));
  HIP_OR_RETURN(op, hipStreamCreateWithFlags(&op->bstream, hipStreamNonBlocking));
  for (hipEvent_t* e : {&op->ev_scat[0], &op->ev_scat[1], &op->ev_done[0], &op->ev_done[1]})
    HIP_OR_RETURN(op, hipEventCreateWithFlags(e, hipEventDisableTiming));
  for (hipEvent_t e : {op->ev_done[0], op->ev_done[1]}) HIP_OR_RETURN(op, hipEventRecord(e, op->stream));
  HIP_OR_RETURN(op, hipEventCreateWithFlags(&op->snap, hipEventDisableTiming));

  DevCfg& c = op->dc;
  c.assigner = cfg.assigner;
  // Short / Byte fields run as Integer and Float as Double inside; rows and snapshots take the field's width
  c.vtype = cfg.value_type == FW_VAL_F32 ? FW_VAL_F64 : (cfg.value_type == FW_VAL_I16 || cfg.value_type == FW_VAL_I8)
                                                           ? FW_VAL_I32 : cfg.value_type;
  c.sum_bits = cfg.value_type == FW_VAL_I32 ? 32 : cfg.value_type == FW_VAL_I16 ? 16 : cfg.value_type == FW_VAL_I8 ? 8 : 64;
  c.f32 = cfg.value_type == FW_VAL_F32;
  c.key_kind = cfg.key_kind;
  c.purging = cfg.purging;
  c.side_output = cfg.side_output;
  c.max_par = cfg.max_parallelism;
  c.kg0 = cfg.key_group_start;
  c.n_kg = cfg.key_group_end - cfg.key_group_start + 1;
  // dense regions (DevCfg::dense): tumbling windows, count/sum/min/max, no allowed lateness (FW_NO_DENSE=1 disables),
  // and not for a handful of keys: a dense region's run is one workgroup's, so a few hot keys would serialise the
  // batch (C1, 170 words: k_dt_aggregate 2.4 ms per step against 0.45 ms for k_aggregate's split partitions)
  c.dense = cfg.assigner == FW_TUMBLING && cfg.aggregate == FW_AGG_COUNT_SUM_MIN_MAX && cfg.allowed_lateness == 0 &&
            (cfg.expected_entries == 0 || cfg.expected_entries >= 65536) &&
            !(getenv("FW_NO_DENSE") && atoi(getenv("FW_NO_DENSE")));
  int64_t s = cfg.sub_partitions;
  if (s == 0 && c.dense) {
    // about 3/4 of k_dt_aggregate's LDS table of live entries per region (C2: 2M live entries -> 1024 regions), at
    // least 4 per key group (the compact records' window delta)
    const int64_t keys = cfg.expected_entries > 0 ? cfg.expected_entries : 0;
    const int64_t target = std::max<int64_t>(256, next_pow2((keys + FW_DT_SLOTS * 3 / 4 - 1) / (FW_DT_SLOTS * 3 / 4)));
    s = std::max<int64_t>(4, next_pow2(std::max<int64_t>(1, target / c.n_kg)));
  } else if (s == 0) {
    // about 2048 partitions, more when the expected keys would put more than ~512 keys in one: a
    // partition's (key, window) deltas of a batch must fit k_aggregate's LDS table, or it flushes
    // several times into its region (C3, 2M keys: 4096 partitions halve k_aggregate's time)
    const int64_t wins = cfg.assigner == FW_SLIDING ? cfg.size / cfg.slide + 1 : 2;  // live windows per key
    const int64_t keys = cfg.expected_entries > 0 ? cfg.expected_entries / wins : 0;
    // tumbling count/sum/min/max: ~256 keys, so a batch that spans a window boundary (two windows per key)
    // still fits the LDS table once (C2: 4096 partitions, k_aggregate 0.36 -> 0.28 ms; sessions, HLL and
    // t-digest measured no better or worse with the smaller partitions)
    const int64_t per = cfg.assigner == FW_TUMBLING && cfg.aggregate == FW_AGG_COUNT_SUM_MIN_MAX ? 256 : 512;
    const int64_t target = std::min<int64_t>(16384, std::max<int64_t>(2048, next_pow2(std::max<int64_t>(1, keys / per))));
    s = std::max<int64_t>(1, next_pow2(std::max<int64_t>(1, target / c.n_kg)));
  }
  c.log_s = ilog2(s);
  c.P = c.n_kg << c.log_s;
  c.size = cfg.size;
  c.slide = cfg.assigner == FW_SLIDING ? cfg.slide : cfg.size;
  c.offset = cfg.offset;
  c.gap = cfg.gap;
  c.lateness = cfg.allowed_lateness;
  // FW_DIAG: ablation bits for pricing kernel stages in diagnostic runs only (results are wrong)
  if (const char* d = getenv("FW_DIAG")) c.diag = atoi(d);
  c.wpr = cfg.assigner == FW_SLIDING ? (int32_t)((cfg.size + cfg.slide - 1) / cfg.slide) : 1;
  // sliding windows whose size is a multiple of the slide, without allowed lateness, are kept as panes:
  // one state update per element instead of size/slide (DevCfg::panes; FW_NO_PANES=1 disables it)
  c.panes = cfg.assigner == FW_SLIDING && cfg.allowed_lateness == 0 && cfg.size > cfg.slide &&
            cfg.size % cfg.slide == 0 && cfg.aggregate != FW_AGG_HLL &&  // (HLL, t-digest, rows: a block per window)
            cfg.aggregate != FW_AGG_TDIGEST && cfg.aggregate != FW_AGG_ROW &&
            !(getenv("FW_NO_PANES") && atoi(getenv("FW_NO_PANES")));
  if (cfg.assigner != FW_SESSION) {
    make_div_inv((uint64_t)c.size, &c.mag_size, &c.l_size);
    make_div_inv((uint64_t)c.slide, &c.mag_slide, &c.l_slide);
  }
  // compact 16-byte partitioned records (DevCfg::compact): one window per record, an order-free aggregate,
  // and at least 2 bits of sub-partition to carry the window delta (FW_NO_COMPACT=1 disables them)
  c.compact = (cfg.assigner == FW_TUMBLING || c.panes) &&
              (cfg.aggregate == FW_AGG_COUNT_SUM_MIN_MAX || cfg.aggregate == FW_AGG_HLL ||
               cfg.aggregate == FW_AGG_TDIGEST || cfg.aggregate == FW_AGG_ROW) && c.log_s >= 2 &&
              !(getenv("FW_NO_COMPACT") && atoi(getenv("FW_NO_COMPACT")));
  const int64_t expected = cfg.expected_entries > 0 ? cfg.expected_entries : (int64_t)c.P * 512;
  if (cfg.aggregate >= FW_AGG_FIRST) c.agg = cfg.aggregate;  // (FW_AGG_HLL is set below)
  // records per aggregate workgroup of a split (hot) partition: HyperLogLog over time windows takes twice as many
  // (its aggregate keeps the count only; C5 1.00e10 -> 1.08e10 records/s; C4 and C5t measured no better)
  c.agg_chunk = cfg.aggregate == FW_AGG_HLL && cfg.assigner != FW_SESSION ? FW_HLL_AGG_CHUNK_MUL * FW_AGG_CHUNK : FW_AGG_CHUNK;
  if (cfg.aggregate == FW_AGG_HLL) {
    // register pool: one 2^p-byte block per live (key, window); expected_entries live entries, plus
    // a quarter for entries created before the watermark that retires their predecessors
    c.agg = FW_AGG_HLL;
    c.hll_p = hll_p;
    c.pool_bytes = ((int64_t)1 << hll_p) + hll_hdr_bytes(hll_p);  // touched-chunk bitmap + registers
  } else if (cfg.aggregate == FW_AGG_TDIGEST) {
    // digest pool: a head and two halves of delta/2 centroids per live (key, window) (TdHead, TdCent)
    c.td_nb = td_delta / 2;
    c.pool_bytes = ((int64_t)sizeof(TdHead) + 2 * c.td_nb * (int64_t)sizeof(TdCent) + 63) / 64 * 64;
    for (int i = 0; i < 3; i++) c.td_quant[i] = cfg.tdigest_quantiles[i];
    // the k1 scale function's unit steps qb[b] = sin(pi b / delta)^2 (the oracle computes the same table)
    std::vector<double> qb(c.td_nb + 1);
    for (int b = 0; b <= c.td_nb; b++) {
      const double sn = std::sin(M_PI * (double)b / (double)td_delta);
      qb[b] = sn * sn;
    }
    qb[0] = 0.0;
    qb[c.td_nb] = 1.0;
    double* dq = nullptr;
    HIP_OR_RETURN(op, dmalloc(&dq, qb.size()));
    HIP_OR_RETURN(op, hipMemcpy(dq, qb.data(), qb.size() * sizeof(double), hipMemcpyHostToDevice));
    c.td_qb = dq;
    op->td_export = cfg.tdigest_export != 0;
    if (op->td_export) op->dig_stride = 1 + 2 * (int64_t)c.td_nb;
  } else if (cfg.aggregate == FW_AGG_ROW) {
    // one RowAcc per value column per live (key, window), zero = empty (fw_internal.h)
    c.agg = FW_AGG_ROW;
    c.vtype = FW_VAL_I64;  // (a record's value is its index in the push)
    c.sum_bits = 64;
    c.f32 = 0;
    c.row_nc = cfg.row_columns;
    c.row_ns = cfg.row_aggregates;
    int32_t ts[24];
    for (int j = 0; j < 8; j++) ts[j] = j < cfg.row_columns ? cfg.row_column_type[j] : 0;
    for (int q = 0; q < 16; q++) ts[8 + q] = q < cfg.row_aggregates ? cfg.row_aggregate[q] : 0;
    int32_t* dts = nullptr;
    HIP_OR_RETURN(op, dmalloc(&dts, 24));
    HIP_OR_RETURN(op, hipMemcpy(dts, ts, sizeof ts, hipMemcpyHostToDevice));
    c.row_ts = dts;
    c.pool_bytes = ((int64_t)sizeof(RowAcc) * c.row_nc + 15) / 16 * 16;
    op->dig_stride = 1 + (int64_t)c.row_ns;
  }
  // regions sized for the expected entries at 1/FW_TABLE_SLACK load (default 4: 25 %; the limit is 3/4)
  const int64_t slack = getenv("FW_TABLE_SLACK") ? std::max(1, atoi(getenv("FW_TABLE_SLACK"))) : c.dense ? 2 : 4;
  c.log_r = std::max(8, ilog2(slack * ((expected + c.P - 1) / c.P)));  // (dense: a region's groups, densely)
  if (c.pool_bytes) {
    c.pool_blocks = std::max<int64_t>(1024, expected + expected / 4);
    if (c.agg == FW_AGG_ROW) c.pool_blocks = std::max(c.pool_blocks, row_pool_blocks(c));
    HIP_OR_RETURN(op, dmalloc(&c.pool, (size_t)(c.pool_blocks * c.pool_bytes)));
    if (c.agg == FW_AGG_HLL || c.agg == FW_AGG_ROW)  // registers / row accumulators start at zero (and are zeroed
      HIP_OR_RETURN(op, hipMemsetAsync(c.pool, 0, (size_t)(c.pool_blocks * c.pool_bytes), op->stream));  // when freed)
    HIP_OR_RETURN(op, dmalloc(&c.pool_free, (size_t)c.pool_blocks));
    HIP_OR_RETURN(op, dmalloc(&c.pool_defer, (size_t)c.pool_blocks));
    HIP_OR_RETURN(op, dmalloc(&c.pool_ctr, 3));
    HIP_OR_RETURN(op, hipMemsetAsync(c.pool_ctr, 0, 3 * sizeof(int32_t), op->stream));
  }
  op->table_slots = (int64_t)c.P << c.log_r;

  op->max_batch = cfg.max_batch > 0 ? std::min<int64_t>(cfg.max_batch, int64_t(1) << 31) : (int64_t(1) << 24);
  op->tmax = (int32_t)((op->max_batch + FW_TILE - 1) / FW_TILE);
  int rc = alloc_table(op, op->tb, c, true);
  if (rc) return rc;
  fwdev::launch_reset_regions(c, op->tb, op->stream);
  const int64_t mb = op->max_batch;
  const int64_t m = (int64_t)(c.P + 2) * op->tmax;  // P partition rows + ordered row (scanned) + per-tile ordered counts
  HIP_OR_RETURN(op, dmalloc(&op->in_key, mb));
  HIP_OR_RETURN(op, dmalloc(&op->in_ts, mb));
  HIP_OR_RETURN(op, dmalloc(&op->in_val, mb));
  HIP_OR_RETURN(op, dmalloc(&op->in_kh, mb));
  for (Scratch& sc : op->sc)
    if ((rc = alloc_scratch(op, sc, mb, m))) return rc;
  if (c.agg == FW_AGG_ROW) {  // the records' values: their index in the push
    std::vector<int64_t> h((size_t)mb);
    for (int64_t i = 0; i < mb; i++) h[(size_t)i] = i;
    HIP_OR_RETURN(op, dmalloc(&op->iota, (size_t)mb));
    HIP_OR_RETURN(op, hipMemcpy(op->iota, h.data(), (size_t)mb * sizeof(int64_t), hipMemcpyHostToDevice));
  }
  c.wide = op->sc[0].wide;  // (every push sets its own set's word)
  // single-pass scatter: a partition's run may take twice its share of the largest batch (part holds mb PRecs
  // = 2 mb compact records), whole 128-byte lines apart
  if (c.dense) op->rcap = ((2 * mb) / c.P) & ~(int64_t)7;
  if (c.assigner == FW_SESSION) {
    // the batches' taint set (k_taint): 2x the batch, at most 2^22 slots; a batch whose ordered-path
    // keys overflow it replays all of its records in arrival order
    const int64_t cap = std::min<int64_t>(next_pow2(2 * mb), int64_t(1) << 22);
    HIP_OR_RETURN(op, dmalloc(&c.taint_key, (size_t)cap));
    HIP_OR_RETURN(op, dmalloc(&c.taint_state, (size_t)cap));
    HIP_OR_RETURN(op, hipMemsetAsync(c.taint_state, 0, (size_t)cap * sizeof(uint32_t), op->stream));
    c.taint_mask = (uint32_t)(cap - 1);
  }
  if (c.agg == FW_AGG_TDIGEST) {
    TdBuf& t = op->td;
    // the compression sorts one item per (record, window): sliding windows fan out wpr items per record
    const int64_t mi = mb * (c.assigner == FW_SLIDING ? c.wpr : 1);
    for (int b = 0; b < 2; b++) {
      HIP_OR_RETURN(op, dmalloc(&t.gs[b], (size_t)mi));
      HIP_OR_RETURN(op, dmalloc(&t.v[b], (size_t)mi));
    }
    HIP_OR_RETURN(op, dmalloc(&t.binv, (size_t)c.pool_blocks));
    HIP_OR_RETURN(op, hipMemsetAsync(t.binv, 0xff, (size_t)c.pool_blocks * sizeof(uint32_t), op->stream));
    // the grouping and the sorts (launch_tdigest): per digest its count / run start, per position its digest, the
    // runs for the LDS sort (digests of 65 .. 4096 values, and the MSD bins: at most 2 per 2048 values of a long run
    // per level) and for the MSD levels (runs of more than 4096 values), their key ranges and bins
    HIP_OR_RETURN(op, dmalloc(&t.dcnt, (size_t)op->table_slots));
    HIP_OR_RETURN(op, hipMemsetAsync(t.dcnt, 0, (size_t)op->table_slots * sizeof(uint32_t), op->stream));
    HIP_OR_RETURN(op, dmalloc(&t.gsort, (size_t)mi));
    t.lrun_cap = mi / 48 + 4096;
    t.brun_cap = mi / 4096 + 2;
    HIP_OR_RETURN(op, dmalloc(&t.lrun, (size_t)t.lrun_cap));
    for (int b = 0; b < 3; b++) HIP_OR_RETURN(op, dmalloc(&t.brun[b], (size_t)t.brun_cap));
    HIP_OR_RETURN(op, dmalloc(&t.msd, (size_t)t.brun_cap));
    HIP_OR_RETURN(op, dmalloc(&t.spl, (size_t)t.brun_cap * 2047));
    HIP_OR_RETURN(op, dmalloc(&t.hist, (size_t)t.brun_cap * 4096));
    HIP_OR_RETURN(op, dmalloc(&t.lctr, FW_TD_LC_WORDS));
    HIP_OR_RETURN(op, dmalloc(&t.tslot, (size_t)mi));
    HIP_OR_RETURN(op, dmalloc(&t.tbeg, (size_t)mi + 1));  // (+ the runs' end)
    HIP_OR_RETURN(op, dmalloc(&t.ctr, 3));
    // a wave-tier digest has more than FW_TD_T1 - delta/2 values in the batch, a large one more than
    // FW_TD_T3 - delta/2
    HIP_OR_RETURN(op, dmalloc(&t.mid, (size_t)mi));
    t.max_large = (int32_t)(mi / std::max<int64_t>(1, FW_TD_T3 - c.td_nb) + 1);
    HIP_OR_RETURN(op, dmalloc(&t.large, (size_t)t.max_large));
    HIP_OR_RETURN(op, dmalloc(&t.nstart, (size_t)t.max_large * c.td_nb));
    HIP_OR_RETURN(op, dmalloc(&t.ostart, (size_t)t.max_large * c.td_nb));
    HIP_OR_RETURN(op, dmalloc(&t.okey, (size_t)t.max_large * c.td_nb));
    if (op->table_slots >= (int64_t(1) << 31)) return set_err(op, FW_ERR_CAPACITY, "t-digest table would exceed 2^31 slots");
    HIP_OR_RETURN(op, dmalloc(&t.lidx, (size_t)op->table_slots));
    t.lidx_slots = op->table_slots;
    if (c.assigner == FW_SESSION || c.lateness > 0) {  // the ordered path's added elements (DevCfg::td_ovk ...)
      HIP_OR_RETURN(op, dmalloc(&c.td_ovk, (size_t)mb));
      HIP_OR_RETURN(op, dmalloc(&c.td_ovt, (size_t)mb));
      HIP_OR_RETURN(op, dmalloc(&c.td_ovv, (size_t)mb));
      HIP_OR_RETURN(op, dmalloc(&c.td_ovp, (size_t)mb));
      HIP_OR_RETURN(op, dmalloc(&c.td_ovctr, 1));
      HIP_OR_RETURN(op, hipMemsetAsync(c.td_ovctr, 0, sizeof(int32_t), op->stream));
    }
    if (c.lateness > 0) {  // late firings (DevCfg::td_olast ...)
      if (c.assigner != FW_SESSION) HIP_OR_RETURN(op, dmalloc(&c.td_ovn, (size_t)mb));
      HIP_OR_RETURN(op, dmalloc(&c.td_olink, (size_t)(mb * c.wpr)));
      HIP_OR_RETURN(op, dmalloc(&c.td_olast, (size_t)op->table_slots));
      HIP_OR_RETURN(op, dmalloc(&c.td_late, (size_t)FW_SLOW_THREADS * c.td_nb));
      if (c.assigner == FW_SESSION) {  // merged digests' unions (DevCfg::td_bhead ...)
        c.td_lateu_cap = 16 * c.td_nb;
        HIP_OR_RETURN(op, dmalloc(&c.td_bhead, (size_t)c.pool_blocks));
        HIP_OR_RETURN(op, dmalloc(&c.td_bnext, (size_t)c.pool_blocks));
        HIP_OR_RETURN(op, dmalloc(&c.td_lateu, (size_t)FW_SLOW_THREADS * c.td_lateu_cap));
      }
    }
    if (c.assigner == FW_SESSION) {  // session merges (DevCfg::td_mdst, TdBuf::fwd ...; launch_tdigest)
      const size_t pb = (size_t)c.pool_blocks;
      HIP_OR_RETURN(op, dmalloc(&c.td_mdst, pb));
      HIP_OR_RETURN(op, dmalloc(&c.td_msrc, pb));
      HIP_OR_RETURN(op, dmalloc(&c.td_mctr, 1));
      HIP_OR_RETURN(op, hipMemsetAsync(c.td_mctr, 0, sizeof(int32_t), op->stream));
      HIP_OR_RETURN(op, dmalloc(&t.fwd, pb));
      HIP_OR_RETURN(op, dmalloc(&t.mhead, pb));
      HIP_OR_RETURN(op, dmalloc(&t.mnext, pb));
      HIP_OR_RETURN(op, dmalloc(&t.ovr, pb));
      HIP_OR_RETURN(op, dmalloc(&t.uni, pb * (size_t)c.td_nb));
      HIP_OR_RETURN(op, dmalloc(&t.uctr, 2));
      HIP_OR_RETURN(op, dmalloc(&t.mover, (size_t)op->table_slots));
      HIP_OR_RETURN(op, hipMemsetAsync(t.fwd, 0xff, pb * sizeof(uint32_t), op->stream));
      HIP_OR_RETURN(op, hipMemsetAsync(t.mhead, 0xff, pb * sizeof(int32_t), op->stream));
      HIP_OR_RETURN(op, hipMemsetAsync(t.mover, 0xff, (size_t)op->table_slots * sizeof(int32_t), op->stream));
      HIP_OR_RETURN(op, hipMemsetAsync(t.uctr, 0, 2 * sizeof(unsigned long long), op->stream));
    }
  }
  if (cfg.assigner == FW_COUNT) {
    DevCount& w = op->cw;
    w.size = cfg.size;
    w.slide = cfg.slide;
    w.wl = cfg.count_evict_after ? cfg.size + cfg.slide : cfg.size;
    w.max_keys = (int32_t)std::min<int64_t>(cfg.expected_entries > 0 ? cfg.expected_entries : (1 << 20), 1 << 30);
    const int64_t cap = next_pow2(2 * (int64_t)w.max_keys);
    w.cap_mask = (uint32_t)(cap - 1);
    HIP_OR_RETURN(op, dmalloc(&w.mkey, (size_t)cap));
    HIP_OR_RETURN(op, dmalloc(&w.mstate, (size_t)cap));
    HIP_OR_RETURN(op, hipMemsetAsync(w.mstate, 0, (size_t)cap * sizeof(uint32_t), op->stream));
    HIP_OR_RETURN(op, dmalloc(&w.mslot, (size_t)cap));
    HIP_OR_RETURN(op, dmalloc(&w.nslots, 1));
    HIP_OR_RETURN(op, hipMemsetAsync(w.nslots, 0, sizeof(int32_t), op->stream));
    HIP_OR_RETURN(op, dmalloc(&w.cnt, (size_t)w.max_keys));
    HIP_OR_RETURN(op, hipMemsetAsync(w.cnt, 0, (size_t)w.max_keys * sizeof(int64_t), op->stream));
    const size_t ring = (size_t)w.max_keys * (size_t)std::max<int64_t>(1, w.wl - 1);
    if (ring * 16 > (size_t(64) << 30))
      return set_err(op, FW_ERR_CAPACITY, "count windows: expected_entries * (window length - 1) * 16 B exceeds 64 GiB");
    HIP_OR_RETURN(op, dmalloc(&w.ring_v, ring));
    HIP_OR_RETURN(op, dmalloc(&w.ring_o, ring));
    for (int b = 0; b < 2; b++) {
      HIP_OR_RETURN(op, dmalloc(&w.sk[b], (size_t)mb));
      HIP_OR_RETURN(op, dmalloc(&w.sv[b], (size_t)mb));
    }
    w.tmp_bytes = fwdev::count_sort_bytes(mb);
    HIP_OR_RETURN(op, dmalloc((uint8_t**)&w.tmp, w.tmp_bytes));
    HIP_OR_RETURN(op, dmalloc(&w.sbeg, (size_t)w.max_keys));
    HIP_OR_RETURN(op, dmalloc(&w.send, (size_t)w.max_keys));
  }
  HIP_OR_RETURN(op, dmalloc(&op->prog.rb, (size_t)c.P));
  HIP_OR_RETURN(op, dmalloc(&op->prog.tp, (size_t)c.P * FW_AGG_THREADS));
  HIP_OR_RETURN(op, dmalloc(&op->prog.done, (size_t)c.P));
  HIP_OR_RETURN(op, dmalloc(&op->d_status, 1));
  HIP_OR_RETURN(op, dmalloc(&op->d_stats3, 4));
  HIP_OR_RETURN(op, hipMemsetAsync(op->d_status, 0, sizeof(Status), op->stream));
  HIP_OR_RETURN(op, hipHostMalloc((void**)&op->h_status, sizeof(Status), hipHostMallocDefault));
  memset(op->h_status, 0, sizeof(Status));
  if ((rc = ensure_out_capacity(op, 2 * op->table_slots, 0))) return rc;
  if ((rc = ensure_side_capacity(op, cfg.side_output ? mb : 1, 0))) return rc;
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  return FW_OK;
}

void fw_destroy(fw_op* op) {
  if (!op) return;
  if (op->stream) {
    (void)hipSetDevice(op->device);
    if (op->bstream) (void)hipStreamSynchronize(op->bstream);
    (void)hipStreamSynchronize(op->stream);
  }
  free_table(op->tb);
  dfree(op->tb.cur);
  dfree(op->tb.live);
  dfree(op->tb.next_timer);
  dfree(op->tb.fire_e);
  dfree(op->tb.fire_lo);
  dfree(op->tb.pane_floor);
  dfree(op->tb.passes);
  dfree(op->in_key);
  dfree(op->in_ts);
  dfree(op->in_val);
  dfree(op->in_kh);
  for (Scratch& sc : op->sc) free_scratch(sc);
  dfree(op->prog.rb);
  dfree(op->prog.tp);
  dfree(op->prog.done);
  dfree(op->dc.taint_key);
  dfree(op->dc.pool);
  dfree(op->dc.pool_free);
  dfree(op->dc.pool_defer);
  dfree(op->dc.pool_ctr);
  {
    double* q = const_cast<double*>(op->dc.td_qb);
    dfree(q);
    int32_t* rts = const_cast<int32_t*>(op->dc.row_ts);
    dfree(rts);
    TdBuf& t = op->td;
    for (int b = 0; b < 2; b++) {
      dfree(t.gs[b]);
      dfree(t.v[b]);
    }
    dfree(t.binv);
    dfree(t.dcnt);
    dfree(t.gsort);
    dfree(t.lrun);
    for (int b = 0; b < 3; b++) dfree(t.brun[b]);
    dfree(t.msd);
    dfree(t.spl);
    dfree(t.hist);
    dfree(t.lctr);
    dfree(t.tslot);
    dfree(t.tbeg);
    dfree(t.ctr);
    dfree(t.large);
    dfree(t.mid);
    dfree(t.okey);
    dfree(t.nstart);
    dfree(t.ostart);
    dfree(t.lidx);
    for (uint32_t* q : {op->dc.td_mdst, op->dc.td_msrc, t.fwd}) dfree(q);
    for (int32_t* q : {op->dc.td_mctr, op->dc.td_ovctr, op->dc.td_ovp, op->dc.td_ovn, op->dc.td_olink, op->dc.td_olast,
                       op->dc.td_bhead, op->dc.td_bnext, t.mhead, t.mnext, t.mover})
      dfree(q);
    dfree(op->dc.td_late);
    dfree(op->dc.td_lateu);
    for (int64_t* q : {op->dc.td_ovk, op->dc.td_ovt, op->dc.td_ovv}) dfree(q);
    dfree(t.ovr);
    dfree(t.uni);
    dfree(t.uctr);
    DevCount& w = op->cw;
    dfree(w.mkey);
    dfree(w.mstate);
    dfree(w.mslot);
    dfree(w.nslots);
    dfree(w.cnt);
    dfree(w.ring_v);
    dfree(w.ring_o);
    for (int b = 0; b < 2; b++) {
      dfree(w.sk[b]);
      dfree(w.sv[b]);
    }
    uint8_t* wt = (uint8_t*)w.tmp;
    dfree(wt);
    dfree(w.sbeg);
    dfree(w.send);
  }
  dfree(op->dc.taint_state);
  free_hot(op->hot);
  for (int64_t** col : {&op->out.key, &op->out.start, &op->out.end, &op->out.cnt, &op->out.sum, &op->out.mn,
                        &op->out.mx, &op->out.dig, &op->side.key, &op->side.ts, &op->side.val})
    dfree(*col);
  dfree(op->d_status);
  dfree(op->d_stats3);
  dfree(op->xoffs);
  dfree(op->xscan);
  dfree(op->xreg);
  dfree(op->xreg_tmp);
  dfree(op->hoff);
  dfree(op->hoff_tmp);
  dfree(op->iota);
  for (auto& pr : op->prof_pending) {
    (void)hipEventDestroy(pr.a);
    (void)hipEventDestroy(pr.b);
  }
  for (hipEvent_t e : op->prof_free) (void)hipEventDestroy(e);
  if (op->snap) (void)hipEventDestroy(op->snap);
  if (op->h_status) (void)hipHostFree(op->h_status);
  for (hipEvent_t e : {op->ev_scat[0], op->ev_scat[1], op->ev_done[0], op->ev_done[1]})
    if (e) (void)hipEventDestroy(e);
  if (op->bstream) (void)hipStreamDestroy(op->bstream);
  if (op->stream) (void)hipStreamDestroy(op->stream);
  delete op;
}

const char* fw_last_error(const fw_op* op) { return op ? op->err.c_str() : "null handle"; }

int fw_push_batch(fw_op* op, const int64_t* key, const int64_t* ts, const void* val, const int32_t* key_hash,
                  int64_t n) {
  if (!op || n < 0 || (n > 0 && (!key || !ts || !val))) return op ? set_err(op, FW_ERR_ARG, "null column") : FW_ERR_ARG;
  if (op->cfg.key_kind == FW_KEY_HASHED && n > 0 && !key_hash)
    return set_err(op, FW_ERR_ARG, "key_hash required for FW_KEY_HASHED");
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  for (int64_t b = 0; b < n; b += op->max_batch) {
    const int64_t m = std::min(op->max_batch, n - b);
    HIP_OR_RETURN(op, hipMemcpyAsync(op->in_key, key + b, m * 8, hipMemcpyHostToDevice, op->stream));
    HIP_OR_RETURN(op, hipMemcpyAsync(op->in_ts, ts + b, m * 8, hipMemcpyHostToDevice, op->stream));
    HIP_OR_RETURN(op, hipMemcpyAsync(op->in_val, (const int64_t*)val + b, m * 8, hipMemcpyHostToDevice, op->stream));
    if (op->cfg.key_kind == FW_KEY_HASHED)
      HIP_OR_RETURN(op, hipMemcpyAsync(op->in_kh, key_hash + b, m * 4, hipMemcpyHostToDevice, op->stream));
    int rc = push_device(op, op->in_key, op->in_ts, op->in_val, op->in_kh, m, false);
    if (rc) return rc;
  }
  return settle(op);  // host columns: the caller may reuse them when this returns
}

namespace {
// the stream a device push reads its columns on: the input stream when async input applies to the operator's
// batches (push_device's `two`: not with side output, count windows or gathered batches)
hipStream_t input_stream_of(const fw_op* op) {
  const bool two = op->async_in && !op->dc.side_output && op->cfg.assigner != FW_COUNT && !op->sc[0].rt;
  return two ? op->bstream : op->stream;
}

int push_device_batches(fw_op* op, const int64_t* key, const int64_t* ts, const void* val, const int32_t* key_hash,
                        int64_t n, bool async_ok) {
  if (!op || n < 0 || (n > 0 && (!key || !ts || !val))) return op ? set_err(op, FW_ERR_ARG, "null column") : FW_ERR_ARG;
  if (op->cfg.key_kind == FW_KEY_HASHED && n > 0 && !key_hash)
    return set_err(op, FW_ERR_ARG, "key_hash required for FW_KEY_HASHED");
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  for (int64_t b = 0; b < n; b += op->max_batch) {
    const int64_t m = std::min(op->max_batch, n - b);
    int rc = push_device(op, key + b, ts + b, (const int64_t*)val + b, key_hash ? key_hash + b : nullptr, m, async_ok);
    if (rc) return rc;
  }
  return FW_OK;
}
}  // namespace

int fw_push_batch_device(fw_op* op, const int64_t* key, const int64_t* ts, const void* val, const int32_t* key_hash,
                         int64_t n) {
  return push_device_batches(op, key, ts, val, key_hash, n, true);
}

int fw_push_row_batch_device(fw_op* op, const int64_t* key, const int64_t* ts, const int64_t* cols,
                             const uint8_t* nulls, const int32_t* key_hash, int64_t n) {
  if (!op || n < 0 || (n > 0 && (!key || !ts || !cols))) return op ? set_err(op, FW_ERR_ARG, "null column") : FW_ERR_ARG;
  if (op->dc.agg != FW_AGG_ROW) return set_err(op, FW_ERR_ARG, "fw_push_row_batch needs an FW_AGG_ROW operator");
  if (op->cfg.key_kind == FW_KEY_HASHED && n > 0 && !key_hash)
    return set_err(op, FW_ERR_ARG, "key_hash required for FW_KEY_HASHED");
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  for (int64_t b = 0; b < n; b += op->max_batch) {
    const int64_t m = std::min(op->max_batch, n - b);
    const RowIn rin{cols + b, nulls ? nulls + b : nullptr, n};
    int rc = push_device(op, key + b, ts + b, op->iota, key_hash ? key_hash + b : nullptr, m, true, &rin);
    if (rc) return rc;
  }
  return FW_OK;
}

int fw_push_row_batch(fw_op* op, const int64_t* key, const int64_t* ts, const int64_t* cols, const uint8_t* nulls,
                      const int32_t* key_hash, int64_t n) {
  if (!op || n < 0 || (n > 0 && (!key || !ts || !cols))) return op ? set_err(op, FW_ERR_ARG, "null column") : FW_ERR_ARG;
  if (op->dc.agg != FW_AGG_ROW) return set_err(op, FW_ERR_ARG, "fw_push_row_batch needs an FW_AGG_ROW operator");
  if (op->cfg.key_kind == FW_KEY_HASHED && n > 0 && !key_hash)
    return set_err(op, FW_ERR_ARG, "key_hash required for FW_KEY_HASHED");
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  for (int64_t b = 0; b < n; b += op->max_batch) {
    const int64_t m = std::min(op->max_batch, n - b);
    HIP_OR_RETURN(op, hipMemcpyAsync(op->in_key, key + b, m * 8, hipMemcpyHostToDevice, op->stream));
    HIP_OR_RETURN(op, hipMemcpyAsync(op->in_ts, ts + b, m * 8, hipMemcpyHostToDevice, op->stream));
    if (op->cfg.key_kind == FW_KEY_HASHED)
      HIP_OR_RETURN(op, hipMemcpyAsync(op->in_kh, key_hash + b, m * 4, hipMemcpyHostToDevice, op->stream));
    // (the columns go from host memory straight into the push's copy, on the operator's stream)
    const RowIn rin{cols + b, nulls ? nulls + b : nullptr, n};
    int rc = push_device(op, op->in_key, op->in_ts, op->iota, op->in_kh, m, false, &rin);
    if (rc) return rc;
  }
  return settle(op);  // host columns: the caller may reuse them when this returns
}

int fw_drain_row_results(fw_op* op, int64_t* values, uint32_t* null_mask, int64_t cap, int64_t* n) {
  if (!op) return FW_ERR_ARG;
  if (op->dc.agg != FW_AGG_ROW) return set_err(op, FW_ERR_UNSUPPORTED, "fw_drain_row_results needs FW_AGG_ROW");
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc = settle(op);
  if (rc) return rc;
  const int64_t base = op->out_base, have = (int64_t)op->h_status->out_rows - base;
  if (n) *n = have;
  if (cap < have) return set_err(op, FW_ERR_ARG, "drain capacity %lld < pending rows %lld", (long long)cap, (long long)have);
  if (have <= 0) return FW_OK;
  const int64_t ns = op->dc.row_ns, stride = op->dig_stride;
  std::vector<int64_t> h((size_t)(have * stride));
  HIP_OR_RETURN(op, hipMemcpyAsync(h.data(), op->out.dig + base * stride, h.size() * sizeof(int64_t),
                                   hipMemcpyDeviceToHost, op->stream));
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  for (int64_t i = 0; i < have; i++) {
    const int64_t* d = h.data() + i * stride;
    if (null_mask) null_mask[i] = (uint32_t)d[0];
    if (values)
      for (int64_t q = 0; q < ns; q++) values[i * ns + q] = d[1 + q];
  }
  return FW_OK;
}

int fw_set_async_input(fw_op* op, int enable) {
  if (!op) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc = fw_synchronize(op);
  if (rc) return rc;
  op->async_in = enable != 0;
  return FW_OK;
}

void* fw_input_stream(fw_op* op) { return op ? (void*)input_stream_of(op) : nullptr; }

int fw_advance_watermark(fw_op* op, int64_t wm, int64_t* n_pending) {
  if (!op) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc;
  if (op->cfg.assigner == FW_COUNT) {  // GlobalWindow: nothing fires by time (GlobalWindows.java NeverTrigger)
    op->wm = wm;
    if (!n_pending) return FW_OK;
    if ((rc = settle(op))) return rc;
    *n_pending = (int64_t)op->h_status->out_rows - op->out_base;
    return FW_OK;
  }
  // settled: the host knows the row count; unsettled: the ordered path left cap - table slots free
  // and an earlier watermark of the sequence found the buffer with that room as well
  if (!op->unsynced) {
    const int64_t rows = (int64_t)op->h_status->out_rows;
    if ((rc = ensure_out_capacity(op, rows + op->table_slots, rows))) return rc;
  } else if (op->fire_unsettled && (rc = settle(op))) {
    return rc;  // two watermarks in one sequence: the second needs the first's row count
  }
  timed(op, K_FIRE, [&] { fwdev::launch_fire(op->dc, wm, op->tb, op->out, op->d_status, op->stream); });
  HIP_OR_RETURN(op, hipGetLastError());
  op->wm = wm;  // HeapInternalTimerService.advanceWatermark: currentWatermark = time
  op->fire_unsettled = true;
  if ((rc = snapshot(op))) return rc;
  if (!n_pending) return FW_OK;  // asynchronous: the count is left to the next settling call
  if ((rc = settle(op))) return rc;
  *n_pending = (int64_t)op->h_status->out_rows - op->out_base;
  return FW_OK;
}

int fw_pending(fw_op* op, int64_t* n_rows, int64_t* n_side) {
  if (!op) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc = settle(op);
  if (rc) return rc;
  if (n_rows) *n_rows = (int64_t)op->h_status->out_rows - op->out_base;
  if (n_side) *n_side = (int64_t)op->h_status->side_rows - op->side_base;
  return FW_OK;
}

int fw_drain_rows(fw_op* op, const fw_rows* dst, int64_t cap, int64_t* n) {
  if (!op || !dst) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc = settle(op);
  if (rc) return rc;
  const int64_t base = op->out_base, have = (int64_t)op->h_status->out_rows - base;
  if (cap < have) {
    if (n) *n = have;
    return set_err(op, FW_ERR_ARG, "drain capacity %lld < pending rows %lld", (long long)cap, (long long)have);
  }
  if (have > 0) {
    int64_t* d[7] = {dst->key, dst->start, dst->end, dst->count, dst->sum, dst->min, dst->max};
    int64_t* s[7] = {op->out.key, op->out.start, op->out.end, op->out.cnt, op->out.sum, op->out.mn, op->out.mx};
    for (int i = 0; i < 7; i++)
      if (d[i]) HIP_OR_RETURN(op, hipMemcpyAsync(d[i], s[i] + base, have * 8, hipMemcpyDefault, op->stream));  // host or HBM
  }
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  op->out_base += have;
  if (n) *n = have;
  return maybe_restart_rows(op);
}

int fw_drain_side(fw_op* op, const fw_side_rows* dst, int64_t cap, int64_t* n) {
  if (!op || !dst) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc = settle(op);
  if (rc) return rc;
  const int64_t base = op->side_base, have = (int64_t)op->h_status->side_rows - base;
  if (cap < have) {
    if (n) *n = have;
    return set_err(op, FW_ERR_ARG, "drain capacity %lld < pending side rows %lld", (long long)cap, (long long)have);
  }
  if (have > 0) {
    int64_t* d[3] = {dst->key, dst->ts, dst->val};
    int64_t* s[3] = {op->side.key, op->side.ts, op->side.val};
    for (int i = 0; i < 3; i++)
      if (d[i]) HIP_OR_RETURN(op, hipMemcpyAsync(d[i], s[i] + base, have * 8, hipMemcpyDefault, op->stream));  // host or HBM
  }
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  op->side_base += have;
  if (n) *n = have;
  return maybe_restart_rows(op);
}

int fw_rows_device(fw_op* op, fw_rows* view, int64_t* n) {
  if (!op || !view) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc = settle(op);
  if (rc) return rc;
  const int64_t b = op->out_base;
  view->key = op->out.key + b;
  view->start = op->out.start + b;
  view->end = op->out.end + b;
  view->count = op->out.cnt + b;
  view->sum = op->out.sum + b;
  view->min = op->out.mn + b;
  view->max = op->out.mx + b;
  if (n) *n = (int64_t)op->h_status->out_rows - b;
  return FW_OK;
}

int fw_drain_digests(fw_op* op, int64_t* n_cent, double* sum, int64_t* weight, int64_t cap, int64_t* n) {
  if (!op) return FW_ERR_ARG;
  if (!op->td_export) return set_err(op, FW_ERR_UNSUPPORTED, "fw_drain_digests needs FW_AGG_TDIGEST with tdigest_export");
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc = settle(op);
  if (rc) return rc;
  const int64_t base = op->out_base, have = (int64_t)op->h_status->out_rows - base;
  if (n) *n = have;
  if (cap < have) return set_err(op, FW_ERR_ARG, "drain capacity %lld < pending rows %lld", (long long)cap, (long long)have);
  if (have <= 0) return FW_OK;
  const int64_t nb = op->dc.td_nb, stride = 1 + 2 * nb;
  std::vector<int64_t> h((size_t)(have * stride));
  HIP_OR_RETURN(op, hipMemcpyAsync(h.data(), op->out.dig + base * stride, h.size() * sizeof(int64_t),
                                   hipMemcpyDeviceToHost, op->stream));
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  for (int64_t i = 0; i < have; i++) {
    const int64_t* d = h.data() + i * stride;
    if (n_cent) n_cent[i] = d[0];
    for (int64_t k = 0; k < d[0] && k < nb; k++) {
      if (sum) memcpy(&sum[i * nb + k], &d[1 + 2 * k], sizeof(double));
      if (weight) weight[i * nb + k] = d[2 + 2 * k];
    }
  }
  return FW_OK;
}

int fw_clear_pending(fw_op* op) {
  if (!op) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  if (op->unsynced) {  // applied when the queued sequence settles: no wait here
    op->clear_deferred = true;
    return FW_OK;
  }
  op->out_base = (int64_t)op->h_status->out_rows;
  op->side_base = (int64_t)op->h_status->side_rows;
  return maybe_restart_rows(op);
}

int fw_get_stats(fw_op* op, fw_stats* o) {
  if (!op || !o) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc = settle(op);
  if (rc) return rc;
  HIP_OR_RETURN(op, hipMemsetAsync(op->d_stats3, 0, 4 * sizeof(unsigned long long), op->stream));
  fwdev::launch_table_stats(op->dc, op->tb, op->d_stats3, op->stream);
  unsigned long long h3[4];
  HIP_OR_RETURN(op, hipMemcpyAsync(h3, op->d_stats3, sizeof h3, hipMemcpyDeviceToHost, op->stream));
  if ((rc = sync_status(op))) return rc;
  const Status& s = *op->h_status;
  o->records_in = op->records_in + (int64_t)s.partial_records;  // + the records inside merged partials
  o->late_records_dropped = (int64_t)s.late_dropped;
  o->keyed_state_entries = (int64_t)h3[0];
  o->event_time_timers = (int64_t)h3[1];
  o->current_watermark = op->wm;
  o->fired_rows_total = (int64_t)s.fired_total;
  o->pending_rows = (int64_t)s.out_rows - op->out_base;
  o->pending_side_rows = (int64_t)s.side_rows - op->side_base;
  o->table_capacity = op->table_slots;
  o->table_grows = op->grows;
  o->slow_path_records = (int64_t)s.slow_total;
  o->state_merges = (int64_t)s.merged;
  o->digest_centroids_fired = (int64_t)s.td_cent;
  o->single_pass_batches = op->single_batches;
  o->single_pass_redone = (int64_t)s.rsv_fallbacks;
  o->narrow_pass_batches = op->narrow_batches;
  o->narrow_pass_redone = (int64_t)s.narrow_misses;
  o->push_resumptions = op->resumptions;
  return FW_OK;
}

int fw_profile(fw_op* op, int enable) {
  if (!op) return FW_ERR_ARG;
  op->prof_mask = enable == 0 ? 0u : (enable & FW_PROFILE_KINDS) ? (uint32_t)(enable & 0xff) : 0xffu;
  return FW_OK;
}

int fw_profile_read(fw_op* op, double* ms, int64_t* launches, int reset) {
  if (!op) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  prof_collect(op);
  for (int k = 0; k < FW_NUM_KERNELS; k++) {
    if (ms) ms[k] = op->prof_ms[k];
    if (launches) launches[k] = op->prof_n[k];
    if (reset) {
      op->prof_ms[k] = 0;
      op->prof_n[k] = 0;
    }
  }
  return FW_OK;
}

const char* fw_kernel_name(int kind) { return kind >= 0 && kind < FW_NUM_KERNELS ? KERNEL_NAMES[kind] : ""; }

static int fw_combine_extract_device_any(fw_op* op, int32_t world, fw_partials* out, int64_t cap, int64_t* counts,
                                         int64_t* n);
int fw_combine_extract_device(fw_op* op, int32_t world, fw_partials* out, int64_t cap, int64_t* counts,
                              int64_t* n) {
  if (!op || !n || world < 1 || (world > 1 && !counts)) return op ? set_err(op, FW_ERR_ARG, "null argument") : FW_ERR_ARG;
  if (!combine_eligible(op->cfg))
    return set_err(op, FW_ERR_UNSUPPORTED,
                   "combining needs tumbling windows or sliding windows kept as panes, the count/sum/min/max aggregate, no "
                   "allowed lateness, no side output and Long or Integer keys (HyperLogLog: "
                   "fw_combine_extract_hll_device)");
  return fw_combine_extract_device_any(op, world, out, cap, counts, n);
}
// the drain itself (count/sum/min/max and HyperLogLog partial rows alike)
static int fw_combine_extract_device_any(fw_op* op, int32_t world, fw_partials* out, int64_t cap, int64_t* counts,
                                  int64_t* n) {
  if (op->wm != INT64_MIN)
    return set_err(op, FW_ERR_STATE, "a combiner's watermark is never advanced (it would fire or drop partials)");
  if (world > op->cfg.max_parallelism) return set_err(op, FW_ERR_ARG, "more subtasks than key groups");
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc = fw_synchronize(op);
  if (rc) return rc;
  const DevCfg& c = op->dc;
  if (!op->xoffs) {
    HIP_OR_RETURN(op, dmalloc(&op->xoffs, (size_t)c.P + 1));
    HIP_OR_RETURN(op, dmalloc(&op->xscan, (size_t)(c.P + 1) / 4096 + 2));
  }
  fwdev::launch_live_offsets(c, op->tb, op->xoffs, op->xscan, op->stream);
  std::vector<uint32_t> h((size_t)c.P + 1);
  HIP_OR_RETURN(op, hipMemcpyAsync(h.data(), op->xoffs, h.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, op->stream));
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  *n = h[c.P];
  // destination d owns computeKeyGroupRangeForOperatorIndex(maxPar, world, d); its partitions are contiguous
  const int32_t M = op->cfg.max_parallelism, k0 = c.kg0, k1 = c.kg0 + c.n_kg;  // [k0, k1)
  for (int32_t d = 0; counts && d < world; d++) {
    const int32_t a = std::max((d * M + world - 1) / world, k0), b = std::min(((d + 1) * M - 1) / world + 1, k1);
    counts[d] = a < b ? (int64_t)h[(size_t)(b - k0) << c.log_s] - (int64_t)h[(size_t)(a - k0) << c.log_s] : 0;
  }
  if (*n > cap) return set_err(op, FW_ERR_CAPACITY, "%lld partials do not fit the %lld-row output", (long long)*n,
                               (long long)cap);
  if (*n > 0 && (!out || !out->key || !out->start || !out->cnt || !out->sum || !out->min || !out->max))
    return set_err(op, FW_ERR_ARG, "null output column");
  if (out) out->config = combine_config_tag(op->cfg);
  if (*n > 0) {
    fwdev::launch_extract(c, op->tb, op->xoffs, PartialCols{out->key, out->start, out->cnt, out->sum, out->min, out->max},
                          op->stream);
  }
  HIP_OR_RETURN(op, hipGetLastError());
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  return FW_OK;
}

int fw_push_partials_device(fw_op* op, const fw_partials* in, int64_t n) {
  if (!op || !in || n < 0) return op ? set_err(op, FW_ERR_ARG, "null argument") : FW_ERR_ARG;
  if (!combine_eligible(op->cfg))
    return set_err(op, FW_ERR_UNSUPPORTED,
                   "combining needs tumbling windows or sliding windows kept as panes, the count/sum/min/max aggregate, no "
                   "allowed lateness, no side output and Long or Integer keys");
  if (n > 0 && (!in->key || !in->start || !in->cnt || !in->sum || !in->min || !in->max))
    return set_err(op, FW_ERR_ARG, "null column");
  if (in->config != combine_config_tag(op->cfg))
    return set_err(op, FW_ERR_ARG,
                   "partials from a combiner configured differently (assigner, size, offset, value type, key kind, max "
                   "parallelism or aggregate) than this operator");
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  for (int64_t b = 0; b < n; b += op->max_batch) {
    const int64_t m = std::min(op->max_batch, n - b);
    const int rc = push_partials(op, PartialCols{in->key + b, in->start + b, in->cnt + b, in->sum + b, in->min + b,
                                                 in->max + b}, m);
    if (rc) return rc;
  }
  return FW_OK;
}

namespace {
int grow_u32(fw_op* op, uint32_t** p, uint32_t** tmp, int64_t* cap, int64_t need) {
  if (need <= *cap) return FW_OK;
  const int64_t c = std::max<int64_t>(need, 2 * *cap);
  dfree(*p);
  dfree(*tmp);
  *cap = 0;
  HIP_OR_RETURN(op, dmalloc(p, (size_t)c));
  HIP_OR_RETURN(op, dmalloc(tmp, (size_t)c / 4096 + 2));
  *cap = c;
  return FW_OK;
}
}  // namespace

int fw_combine_extract_hll_device(fw_op* op, int32_t world, fw_partials* out, int64_t cap, int64_t* counts,
                                  int64_t* reg_counts, int64_t* n, int64_t* nregs) {
  if (!op || !n || !nregs || world < 1 || (world > 1 && (!counts || !reg_counts)))
    return op ? set_err(op, FW_ERR_ARG, "null argument") : FW_ERR_ARG;
  if (!combine_eligible_hll(op->cfg))
    return set_err(op, FW_ERR_UNSUPPORTED, "HyperLogLog combining needs tumbling windows, no allowed lateness, no side "
                                           "output and Long or Integer keys");
  if (op->xreg_n >= 0)
    return set_err(op, FW_ERR_STATE, "the previous extraction's registers were not taken (fw_combine_hll_registers_device)");
  int rc = fw_combine_extract_device_any(op, world, out, cap, counts, n);
  if (rc) return rc;
  *nregs = 0;
  if (reg_counts)
    for (int32_t d = 0; d < world; d++) reg_counts[d] = 0;
  const DevCfg& c = op->dc;
  if (*n > 0) {
    if ((rc = grow_u32(op, &op->xreg, &op->xreg_tmp, &op->xreg_cap, *n + 1))) return rc;
    const PartialCols pc{out->key, out->start, out->cnt, out->sum, out->min, out->max};
    fwdev::launch_hll_extract_counts(c, pc, *n, op->xreg, op->xreg_tmp, op->stream);
    HIP_OR_RETURN(op, hipGetLastError());
    // the register offsets at every destination's first partial (its partials are one contiguous slice)
    std::vector<uint32_t> at((size_t)world + 1);
    int64_t first = 0;
    for (int32_t d = 0; d <= world; d++) {
      HIP_OR_RETURN(op, hipMemcpyAsync(&at[(size_t)d], op->xreg + first, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                       op->stream));
      if (d < world) first += counts ? counts[d] : *n;
    }
    HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
    *nregs = at[(size_t)world];
    for (int32_t d = 0; reg_counts && d < world; d++) reg_counts[d] = (int64_t)at[(size_t)d + 1] - (int64_t)at[(size_t)d];
  }
  op->xreg_n = *n;
  return FW_OK;
}

int fw_combine_hll_registers_device(fw_op* op, const fw_partials* out, int64_t n, uint32_t* regs, int64_t regs_cap) {
  if (!op || !out || n < 0) return op ? set_err(op, FW_ERR_ARG, "null argument") : FW_ERR_ARG;
  if (op->xreg_n < 0 || n != op->xreg_n)
    return set_err(op, FW_ERR_STATE, "no extraction of %lld HyperLogLog partials to take the registers of", (long long)n);
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  if (n > 0) {
    uint32_t total = 0;
    HIP_OR_RETURN(op, hipMemcpy(&total, op->xreg + n, sizeof total, hipMemcpyDeviceToHost));
    if ((int64_t)total > regs_cap)
      return set_err(op, FW_ERR_CAPACITY, "%lld registers do not fit the %lld-entry output", (long long)total,
                     (long long)regs_cap);
    if (total > 0 && !regs) return set_err(op, FW_ERR_ARG, "null register output");
    fwdev::launch_hll_extract_regs(op->dc, PartialCols{out->key, out->start, out->cnt, out->sum, out->min, out->max}, n,
                                   op->xreg, regs, op->stream);
    HIP_OR_RETURN(op, hipGetLastError());
    HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  }
  op->xreg_n = -1;
  return FW_OK;
}

int fw_push_hll_partials_device(fw_op* op, const fw_partials* in, int64_t n, const uint32_t* regs, int64_t nregs) {
  if (!op || !in || n < 0 || nregs < 0) return op ? set_err(op, FW_ERR_ARG, "null argument") : FW_ERR_ARG;
  if (!combine_eligible_hll(op->cfg))
    return set_err(op, FW_ERR_UNSUPPORTED, "HyperLogLog combining needs tumbling windows, no allowed lateness, no side "
                                           "output and Long or Integer keys");
  if (n > 0 && (!in->key || !in->start || !in->cnt || !in->sum || !in->min || !in->max || (nregs > 0 && !regs)))
    return set_err(op, FW_ERR_ARG, "null column");
  if (in->config != combine_config_tag(op->cfg))
    return set_err(op, FW_ERR_ARG,
                   "partials from a combiner configured differently (assigner, size, offset, value type, key kind, max "
                   "parallelism, aggregate or precision) than this operator");
  if (n == 0) return FW_OK;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc;
  // the previous push settled first: a resumed merge of it reruns its register raise with the offsets it had
  if ((rc = settle(op))) return rc;
  if ((rc = grow_u32(op, &op->hoff, &op->hoff_tmp, &op->hoff_cap, n + 1))) return rc;
  const PartialCols all{in->key, in->start, in->cnt, in->sum, in->min, in->max};
  fwdev::launch_hll_reg_offsets(all, n, op->hoff, op->hoff_tmp, op->stream);
  HIP_OR_RETURN(op, hipGetLastError());
  {  // the register list must hold exactly what the partials' sum columns say (the raise reads it unguarded)
    uint32_t tot = 0;
    HIP_OR_RETURN(op, hipMemcpyAsync(&tot, op->hoff + n, sizeof tot, hipMemcpyDeviceToHost, op->stream));
    HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
    if ((int64_t)tot != nregs)
      return set_err(op, FW_ERR_ARG, "the partials' sum columns count %lld registers, the register list has %lld",
                     (long long)tot, (long long)nregs);
  }
  for (int64_t b = 0; b < n; b += op->max_batch) {
    const int64_t m = std::min(op->max_batch, n - b);
    // (the offsets index the whole register list: partial b + i's are at hoff[b + i])
    rc = push_partials(op, PartialCols{in->key + b, in->start + b, in->cnt + b, in->sum + b, in->min + b, in->max + b}, m,
                       regs, op->hoff + b);
    if (rc) return rc;
  }
  return FW_OK;
}

int fw_synchronize(fw_op* op) {
  if (!op) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc = settle(op);
  if (rc) return rc;
  HIP_OR_RETURN(op, hipStreamSynchronize(op->bstream));
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  return FW_OK;
}

void* fw_stream(fw_op* op) { return op ? (void*)op->stream : nullptr; }

// ---- keyed-state snapshot / restore per key group (see flink_window.h)
namespace {
int kg_check(fw_op* op, int32_t kg) {
  if (kg < op->dc.kg0 || kg >= op->dc.kg0 + op->dc.n_kg)
    return set_err(op, FW_ERR_KEY_GROUP, "key group %d is not in this operator's KeyGroupRange [%d, %d]", kg,
                   op->dc.kg0, op->dc.kg0 + op->dc.n_kg - 1);
  return FW_OK;
}
int alloc_state_cols(fw_op* op, StateCols& c, int64_t n) {
  int64_t** cols[8] = {&c.key, &c.start, &c.end, &c.cnt, &c.sum, &c.mn, &c.mx, &c.timer};
  for (int i = 0; i < 8; i++) HIP_OR_RETURN(op, dmalloc(cols[i], (size_t)std::max<int64_t>(n, 1)));
  return FW_OK;
}
void free_state_cols(StateCols& c) {
  int64_t** cols[8] = {&c.key, &c.start, &c.end, &c.cnt, &c.sum, &c.mn, &c.mx, &c.timer};
  for (int i = 0; i < 8; i++) dfree(*cols[i]);
}
}  // namespace

int64_t fw_state_block_bytes(fw_op* op) {
  if (!op) return 0;
  if (op->dc.agg == FW_AGG_HLL) return (int64_t)1 << op->dc.hll_p;
  if (op->dc.agg == FW_AGG_TDIGEST) return (1 + 2 * (int64_t)op->dc.td_nb) * (int64_t)sizeof(int64_t);
  if (op->dc.agg == FW_AGG_ROW) return 5 * (int64_t)op->dc.row_nc * (int64_t)sizeof(int64_t);
  return 0;
}

int fw_snapshot_key_group(fw_op* op, int32_t kg, const fw_state_rows* dst, int64_t cap, int64_t* n) {
  if (op && op->dc.pool_bytes)
    return set_err(op, FW_ERR_UNSUPPORTED, "the HyperLogLog and t-digest accumulators are not in fw_state_rows: "
                                           "use fw_snapshot_key_group_blocks");
  return fw_snapshot_key_group_blocks(op, kg, dst, nullptr, cap, n);
}

int fw_snapshot_key_group_blocks(fw_op* op, int32_t kg, const fw_state_rows* dst, uint8_t* blocks, int64_t cap,
                                 int64_t* n) {
  if (op && op->cfg.assigner == FW_COUNT)
    return set_err(op, FW_ERR_UNSUPPORTED, "keyed-state snapshots of count windows are not offered");
  if (!op || !n) return op ? set_err(op, FW_ERR_ARG, "null argument") : FW_ERR_ARG;
  const int64_t bb = fw_state_block_bytes(op);
  if (bb && dst && cap > 0 && !blocks) return set_err(op, FW_ERR_ARG, "null accumulator blocks");
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc;
  if ((rc = kg_check(op, kg)) || (rc = settle(op))) return rc;
  const DevCfg& c = op->dc;
  const int32_t np = 1 << c.log_s, p0 = (kg - c.kg0) << c.log_s;
  // occupied slots of the key group's regions bound its live entries
  std::vector<int32_t> live(np);
  HIP_OR_RETURN(op, hipMemcpyAsync(live.data(), op->tb.live + p0, np * sizeof(int32_t), hipMemcpyDeviceToHost,
                                   op->stream));
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  int64_t bound = 0;
  for (int32_t v : live) bound += v;
  StateCols d{};
  uint8_t* acc = nullptr;
  auto release = [&]() {
    free_state_cols(d);
    dfree(d.blk);
    dfree(acc);
  };
  if ((rc = alloc_state_cols(op, d, bound)) ||
      (bb && dmalloc(&d.blk, (size_t)std::max<int64_t>(bound, 1)) != hipSuccess && (rc = FW_ERR_HIP))) {
    release();
    return rc == FW_ERR_HIP ? set_err(op, rc, "snapshot: allocation failed") : rc;
  }
  HIP_OR_RETURN(op, hipMemsetAsync(op->d_stats3, 0, sizeof(unsigned long long), op->stream));
  fwdev::launch_snapshot(c, op->tb, p0, np, d, op->d_stats3, op->stream);
  unsigned long long got = 0;
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(&got, op->d_stats3, sizeof got, hipMemcpyDeviceToHost, op->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(op->stream);
  if (e == hipSuccess && dst && cap >= (int64_t)got && got > 0) {
    int64_t* hs[8] = {dst->key, dst->start, dst->end, dst->count, dst->sum, dst->min, dst->max, dst->timer};
    int64_t* ds[8] = {d.key, d.start, d.end, d.cnt, d.sum, d.mn, d.mx, d.timer};
    for (int i = 0; i < 8 && e == hipSuccess; i++)
      if (hs[i]) e = hipMemcpyAsync(hs[i], ds[i], got * sizeof(int64_t), hipMemcpyDeviceToHost, op->stream);
    if (e == hipSuccess && bb) {  // the rows' accumulators in their snapshot form
      e = dmalloc(&acc, (size_t)(got * bb));
      if (e == hipSuccess) {
        fwdev::launch_block_export(c, d.blk, (int64_t)got, acc, op->stream);
        e = hipGetLastError();
      }
      if (e == hipSuccess) e = hipMemcpyAsync(blocks, acc, got * bb, hipMemcpyDeviceToHost, op->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(op->stream);
  }
  release();
  if (e != hipSuccess) return set_err(op, FW_ERR_HIP, "snapshot: %s", hipGetErrorString(e));
  *n = (int64_t)got;
  return FW_OK;
}

}  // extern "C"
namespace {
// restore into dense regions: the rows (already checked to belong to kg) become partial accumulators in
// partition-major runs and are merged like a combining push; a region whose buffers are too small suspends the
// merge, the table grows and the merge resumes (synchronous)
int restore_dense(fw_op* op, int32_t kg, const fw_state_rows* src, int64_t n) {
  const int32_t P = op->dc.P;
  const int32_t T = (int32_t)((n + FW_TILE - 1) / FW_TILE);
  const int64_t m = (int64_t)(P + 1) * T;
  StateCols d{};
  int32_t* rp = nullptr;
  uint32_t *hist = nullptr, *scan_tmp = nullptr;
  PartialRec *tmp = nullptr, *part = nullptr;
  auto done = [&](int code) {
    free_state_cols(d);
    dfree(rp);
    dfree(hist);
    dfree(scan_tmp);
    dfree(tmp);
    dfree(part);
    return code;
  };
  int rc;
  if ((rc = alloc_state_cols(op, d, n))) return done(rc);
  const int64_t* hs[8] = {src->key, src->start, src->end, src->count, src->sum, src->min, src->max, src->timer};
  int64_t* ds[8] = {d.key, d.start, d.end, d.cnt, d.sum, d.mn, d.mx, d.timer};
  for (int i = 0; i < 8; i++)
    if (hipMemcpyAsync(ds[i], hs[i], n * sizeof(int64_t), hipMemcpyHostToDevice, op->stream) != hipSuccess)
      return done(set_err(op, FW_ERR_HIP, "restore: copy failed"));
  if (dmalloc(&rp, (size_t)n) != hipSuccess || dmalloc(&hist, (size_t)m) != hipSuccess ||
      dmalloc(&scan_tmp, (size_t)(m / 4096 + 2)) != hipSuccess || dmalloc(&tmp, (size_t)n) != hipSuccess ||
      dmalloc(&part, (size_t)n) != hipSuccess)
    return done(set_err(op, FW_ERR_HIP, "restore: allocation failed"));
  fwdev::launch_dt_restore_runs(op->dc, kg, d, n, rp, hist, scan_tmp, tmp, part, op->d_status, op->stream);
  for (int resume = 0, rounds = 0;; resume = 1) {
    if (++rounds > 64) return done(set_err(op, FW_ERR_STATE, "restore did not complete after 64 resumptions"));
    fwdev::launch_pmerge(op->dc, part, hist, T, op->tb, op->prog, resume, op->d_status, op->stream);
    if (hipGetLastError() != hipSuccess) return done(set_err(op, FW_ERR_HIP, "restore kernel failed"));
    if ((rc = sync_status(op))) return done(rc);
    Status& s = *op->h_status;
    if (!s.suspended) break;
    if ((rc = grow_table(op, log_r_for(op, s.need_live)))) return done(rc);
    s.suspended = 0;
    s.need_live = 0;
    if ((rc = put_status_field(op, &Status::suspended)) || (rc = put_status_field(op, &Status::need_live)))
      return done(rc);
  }
  done(FW_OK);
  if (op->h_status->flags & FW_STATUS_STATE_LOST) return set_err(op, FW_ERR_CAPACITY, "restore: region full");
  const int64_t rows = (int64_t)op->h_status->out_rows;
  return ensure_out_capacity(op, rows + op->table_slots, rows);  // a watermark may fire every restored window
}
}  // namespace
extern "C" {

int fw_restore_key_group(fw_op* op, int32_t kg, const fw_state_rows* src, int64_t n) {
  if (op && op->dc.pool_bytes)
    return set_err(op, FW_ERR_UNSUPPORTED, "the HyperLogLog and t-digest accumulators are not in fw_state_rows: "
                                           "use fw_restore_key_group_blocks");
  return fw_restore_key_group_blocks(op, kg, src, nullptr, n);
}

int fw_restore_key_group_blocks(fw_op* op, int32_t kg, const fw_state_rows* src, const uint8_t* blocks, int64_t n) {
  if (op && op->cfg.assigner == FW_COUNT)
    return set_err(op, FW_ERR_UNSUPPORTED, "keyed-state snapshots of count windows are not offered");
  if (!op || (n > 0 && !src) || n < 0) return op ? set_err(op, FW_ERR_ARG, "null argument") : FW_ERR_ARG;
  const int64_t bb = fw_state_block_bytes(op);
  if (bb && n > 0 && !blocks) return set_err(op, FW_ERR_ARG, "null accumulator blocks");
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc;
  if ((rc = kg_check(op, kg)) || (rc = settle(op))) return rc;
  if (n == 0) return FW_OK;
  const int64_t* hs[8] = {src->key, src->start, src->end, src->count, src->sum, src->min, src->max, src->timer};
  for (const int64_t* h : hs)
    if (!h) return set_err(op, FW_ERR_ARG, "null state column");
  // first-element reduces: records pushed after the restore are numbered after every restored first
  // element, so the earlier element keeps winning in the caller's numbering
  // (minBy / maxBy: `max` is the selected element's ordinal, likewise)
  if (op->dc.agg >= FW_AGG_FIRST && op->dc.agg <= FW_AGG_FIRST_MAX)
    for (int64_t i = 0; i < n; i++) op->records_in = std::max(op->records_in, src->max[i] + 1);
  // rows of this call that restore the same (key, window): a round per repetition (launch_restore)
  std::vector<int32_t> round_of((size_t)n);
  int32_t rounds = 1;
  {
    struct KW {
      int64_t k, s, e;
      bool operator==(const KW& o) const { return k == o.k && s == o.s && e == o.e; }
    };
    struct H {
      size_t operator()(const KW& x) const {
        return std::hash<int64_t>()(x.k * 0x9E3779B97F4A7C15ll ^ x.s * 0x632BE59BD9B4E019ll ^ x.e);
      }
    };
    std::unordered_map<KW, int32_t, H> seen;
    seen.reserve((size_t)n);
    for (int64_t i = 0; i < n; i++) {
      int32_t& c = seen[KW{src->key[i], src->start[i], src->end[i]}];
      round_of[(size_t)i] = c++;
      rounds = std::max(rounds, c);
    }
  }
  StateCols d{};
  int32_t* demand = nullptr;
  uint8_t* acc = nullptr;
  auto fail = [&](int code) {
    free_state_cols(d);
    dfree(demand);
    dfree(acc);
    dfree(d.blk);
    dfree(d.used);
    return code;
  };
  if ((rc = alloc_state_cols(op, d, n))) return fail(rc);
  int64_t* ds[8] = {d.key, d.start, d.end, d.cnt, d.sum, d.mn, d.mx, d.timer};
  for (int i = 0; i < 8; i++)
    if (hipMemcpyAsync(ds[i], hs[i], n * sizeof(int64_t), hipMemcpyHostToDevice, op->stream) != hipSuccess)
      return fail(set_err(op, FW_ERR_HIP, "restore: copy failed"));
  // the rows' demand per partition: grow the table first if a region would pass its load limit
  const int32_t P = op->dc.P;
  if (dmalloc(&demand, (size_t)P) != hipSuccess || hipMemsetAsync(demand, 0, P * sizeof(int32_t), op->stream) != hipSuccess)
    return fail(set_err(op, FW_ERR_HIP, "restore: allocation failed"));
  fwdev::launch_restore(op->dc, kg, d, n, demand, op->tb, op->d_status, nullptr, 0, op->stream);
  std::vector<int32_t> dem(P), live(P);
  if (hipMemcpyAsync(dem.data(), demand, P * sizeof(int32_t), hipMemcpyDeviceToHost, op->stream) != hipSuccess ||
      hipMemcpyAsync(live.data(), op->tb.live, P * sizeof(int32_t), hipMemcpyDeviceToHost, op->stream) != hipSuccess ||
      (rc = sync_status(op)))
    return fail(rc ? rc : set_err(op, FW_ERR_HIP, "restore: copy failed"));
  if (op->h_status->kg_errors) {
    const int bad = op->h_status->kg_errors;
    op->h_status->kg_errors = 0;
    put_status_field(op, &Status::kg_errors);
    return fail(set_err(op, FW_ERR_KEY_GROUP, "%d restored row(s) do not belong to key group %d", bad, kg));
  }
  if (op->dc.dense) {  // the rows as partials in partition-major runs, merged region by region (k_dt_aggregate)
    fail(FW_OK);
    return restore_dense(op, kg, src, n);
  }
  int64_t need = 0;
  for (int32_t p = 0; p < P; p++) need = std::max<int64_t>(need, (int64_t)live[p] + dem[p]);
  if (need > region_limit(op->dc.log_r) && (rc = grow_table(op, log_r_for(op, need)))) return fail(rc);
  // pool aggregates: n blocks off the free stack / the pool's tail for the rows' new windows, the accumulators
  // imported by k_restore, the blocks it did not use back on the stack
  int32_t ctr[2] = {0, 0};
  int32_t take = 0;
  if (bb) {
    if (hipMemcpy(ctr, op->dc.pool_ctr, sizeof ctr, hipMemcpyDeviceToHost) != hipSuccess)
      return fail(set_err(op, FW_ERR_HIP, "restore: copy failed"));
    take = (int32_t)std::min<int64_t>(ctr[0], n);
    if (ctr[1] + (n - take) > op->dc.pool_blocks)
      return fail(set_err(op, FW_ERR_CAPACITY, "restore: %lld rows do not fit the accumulator block pool (%lld blocks, "
                          "%d free; raise expected_entries)", (long long)n, (long long)op->dc.pool_blocks,
                          (int)(op->dc.pool_blocks - ctr[1] + ctr[0])));
    if (dmalloc(&acc, (size_t)(n * bb)) != hipSuccess || dmalloc(&d.blk, (size_t)n) != hipSuccess ||
        dmalloc(&d.used, 1) != hipSuccess || hipMemsetAsync(d.used, 0, sizeof(int32_t), op->stream) != hipSuccess ||
        hipMemcpyAsync(acc, blocks, n * bb, hipMemcpyHostToDevice, op->stream) != hipSuccess)
      return fail(set_err(op, FW_ERR_HIP, "restore: allocation failed"));
    d.acc = acc;
    d.acc_bytes = bb;
    fwdev::launch_pool_take(op->dc, ctr[0], take, ctr[1], n, d.blk, op->stream);
    const int32_t nc[2] = {ctr[0] - take, (int32_t)(ctr[1] + (n - take))};
    if (hipMemcpyAsync(op->dc.pool_ctr, nc, sizeof nc, hipMemcpyHostToDevice, op->stream) != hipSuccess ||
        hipStreamSynchronize(op->stream) != hipSuccess)
      return fail(set_err(op, FW_ERR_HIP, "restore: copy failed"));
  }
  int32_t* d_round = nullptr;
  if (rounds > 1) {
    if (dmalloc(&d_round, (size_t)n) != hipSuccess ||
        hipMemcpyAsync(d_round, round_of.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, op->stream) != hipSuccess)
      return fail(set_err(op, FW_ERR_HIP, "restore: allocation failed"));
  }
  fwdev::launch_restore(op->dc, kg, d, n, nullptr, op->tb, op->d_status, d_round, rounds, op->stream);
  const bool launched = hipGetLastError() == hipSuccess;
  rc = sync_status(op);
  dfree(d_round);
  if (!launched || rc) return fail(rc ? rc : set_err(op, FW_ERR_HIP, "restore kernel failed"));
  if (bb) {
    int32_t used = 0;
    if (hipMemcpy(&used, d.used, sizeof used, hipMemcpyDeviceToHost) != hipSuccess)
      return fail(set_err(op, FW_ERR_HIP, "restore: copy failed"));
    const int32_t h = ctr[0] - take, back = (int32_t)(n - used);
    fwdev::launch_pool_give(op->dc, d.blk + used, back, h, op->stream);
    const int32_t height = h + back;
    if (hipMemcpyAsync(op->dc.pool_ctr, &height, sizeof height, hipMemcpyHostToDevice, op->stream) != hipSuccess ||
        hipStreamSynchronize(op->stream) != hipSuccess)
      return fail(set_err(op, FW_ERR_HIP, "restore: copy failed"));
    if (op->h_status->acc_refused) {
      const int bad = op->h_status->acc_refused;
      op->h_status->acc_refused = 0;
      put_status_field(op, &Status::acc_refused);
      return fail(set_err(op, FW_ERR_STATE, "%d restored t-digest row(s) refused: a malformed digest, or a window "
                          "that is already present (digests are not merged on restore)", bad));
    }
  }
  fail(FW_OK);
  if (op->h_status->flags & FW_STATUS_STATE_LOST) return set_err(op, FW_ERR_CAPACITY, "restore: region full");
  const int64_t rows = (int64_t)op->h_status->out_rows;
  return ensure_out_capacity(op, rows + op->table_slots, rows);  // a watermark may fire every restored window
}

int fw_key_groups_device(const int64_t* key, const int32_t* key_hash, int32_t key_kind, int64_t n,
                         int32_t max_parallelism, int32_t* kg_out, void* stream) {
  if (n < 0 || max_parallelism < 1 || (key_kind == FW_KEY_HASHED && !key_hash)) return FW_ERR_ARG;
  fwdev::launch_key_groups(key, key_hash, key_kind, n, max_parallelism, kg_out, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? FW_OK : FW_ERR_HIP;
}

int64_t fw_route_scratch_bytes(int64_t n, int32_t parallelism) {
  const int64_t T = (n + FW_TILE - 1) / FW_TILE;
  const int64_t m = (int64_t)parallelism * T;
  return (m + m / 4096 + 64) * (int64_t)sizeof(uint32_t);
}

int fw_route_device(const int64_t* key, const int64_t* ts, const int64_t* val, const int32_t* key_hash,
                    int32_t key_kind, int64_t n, int32_t max_parallelism, int32_t parallelism, int64_t* key_out,
                    int64_t* ts_out, int64_t* val_out, int32_t* hash_out, int64_t* counts, void* scratch,
                    int64_t scratch_bytes, void* stream) {
  if (n < 0 || parallelism < 1 || parallelism > max_parallelism || parallelism > 1024) return FW_ERR_ARG;
  if (key_kind == FW_KEY_HASHED && !key_hash) return FW_ERR_ARG;
  if (scratch_bytes < fw_route_scratch_bytes(n, parallelism)) return FW_ERR_ARG;
  fwdev::launch_route(key, ts, val, key_hash, key_kind, n, max_parallelism, parallelism, key_out, ts_out, val_out,
                      hash_out, counts, (uint32_t*)scratch, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? FW_OK : FW_ERR_HIP;
}

// ---- keyBy exchange over RCCL (see flink_window.h)
}  // extern "C"
struct fw_comm {
  ncclComm_t nc = nullptr;
  int32_t world = 1, rank = 0, device = 0;
  int64_t cap = 0;                                        // records the routed (send) columns hold
  int64_t rcap = 0;                                       // records the received columns hold
  int64_t *rk = nullptr, *rt = nullptr, *rv = nullptr;    // received columns
  int32_t* rh = nullptr;
  int64_t *sk = nullptr, *st = nullptr, *sv = nullptr;    // routed (send) columns
  int32_t* sh = nullptr;
  void* scratch = nullptr;
  int64_t scratch_bytes = 0;
  int64_t* counts = nullptr;  // [2 world + 4]: send counts, recv counts, wm in / min, batch size in / sum
  int64_t* h_counts = nullptr;                            // pinned host copy
  fw_comm_stats stats{};                                   // exchange counters (fw_comm_get_stats)
  int64_t pcap = 0;                                       // combining: partials the send / receive columns hold
  int64_t* ps[6] = {};                                    // send partials (key, start, cnt, sum, min, max)
  int64_t* pr[6] = {};                                    // received partials
  uint32_t *rs = nullptr, *rr = nullptr;                  // HyperLogLog partials' registers: sent / received
  int64_t rscap = 0, rrcap = 0;
  int64_t *rgc = nullptr, *h_rgc = nullptr;               // their per-peer counts [2 world] (device / pinned host)
};
namespace {
template <class T>
void cfree(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}
// the routed columns (and the route's scratch) for n records; their contents are not kept.  On failure every column
// is freed and the capacity is 0, so the next call allocates afresh.
int comm_reserve_send(fw_op* op, fw_comm* c, int64_t need) {
  if (need <= c->cap) return FW_OK;
  const int64_t cap = std::max<int64_t>(need, c->cap * 2);
  c->cap = 0;
  for (int64_t** p : {&c->sk, &c->st, &c->sv}) cfree(*p);
  cfree(c->sh);
  cfree(c->scratch);
  bool ok = dmalloc(&c->sk, (size_t)cap) == hipSuccess && dmalloc(&c->st, (size_t)cap) == hipSuccess &&
            dmalloc(&c->sv, (size_t)cap) == hipSuccess && dmalloc(&c->sh, (size_t)cap) == hipSuccess;
  c->scratch_bytes = fw_route_scratch_bytes(cap, c->world);
  ok = ok && dmalloc((uint8_t**)&c->scratch, (size_t)c->scratch_bytes) == hipSuccess;
  if (!ok) {
    for (int64_t** p : {&c->sk, &c->st, &c->sv}) cfree(*p);
    cfree(c->sh);
    cfree(c->scratch);
    return set_err(op, FW_ERR_HIP, "exchange: cannot allocate the routed columns for %lld records", (long long)cap);
  }
  c->cap = cap;
  return FW_OK;
}
// the received columns for `need` records (a skewed batch can bring more than the subtask sent); the stream that
// last read them must be idle
int comm_reserve_recv(fw_op* op, fw_comm* c, int64_t need) {
  if (need <= c->rcap) return FW_OK;
  const int64_t cap = std::max<int64_t>(need, c->rcap * 2);
  c->rcap = 0;
  for (int64_t** p : {&c->rk, &c->rt, &c->rv}) cfree(*p);
  cfree(c->rh);
  const bool ok = dmalloc(&c->rk, (size_t)cap) == hipSuccess && dmalloc(&c->rt, (size_t)cap) == hipSuccess &&
                  dmalloc(&c->rv, (size_t)cap) == hipSuccess && dmalloc(&c->rh, (size_t)cap) == hipSuccess;
  if (!ok) {
    for (int64_t** p : {&c->rk, &c->rt, &c->rv}) cfree(*p);
    cfree(c->rh);
    return set_err(op, FW_ERR_HIP, "exchange: cannot allocate the received columns for %lld records", (long long)cap);
  }
  c->rcap = cap;
  return FW_OK;
}
#define NCCL_OR_RETURN(op, expr)                                                                            \
  do {                                                                                                      \
    ncclResult_t _r = (expr);                                                                               \
    if (_r != ncclSuccess) return set_err(op, FW_ERR_HIP, "%s failed: %s", #expr, ncclGetErrorString(_r)); \
  } while (0)
// inside ncclGroupStart ... ncclGroupEnd: a failed enqueue still closes the group before returning, so the
// communicator's next collective does not run inside a half-built group
#define NCCL_IN_GROUP(op, expr)                                                                                \
  do {                                                                                                         \
    ncclResult_t _r = (expr);                                                                                  \
    if (_r != ncclSuccess) {                                                                                   \
      (void)ncclGroupEnd();                                                                                    \
      return set_err(op, FW_ERR_HIP, "%s failed: %s", #expr, ncclGetErrorString(_r));                          \
    }                                                                                                          \
  } while (0)
// the counts round: per-peer counts all-to-all, the watermark's minimum and the batch sizes' sum (the bound on
// what any subtask can receive in this batch) over all subtasks, one group on stream s
int comm_counts_round(fw_op* op, fw_comm* c, hipStream_t s) {
  const int W = c->world;
  NCCL_OR_RETURN(op, ncclGroupStart());
  NCCL_IN_GROUP(op, ncclAllToAll(c->counts, c->counts + W, 1, ncclInt64, c->nc, s));
  NCCL_IN_GROUP(op, ncclAllReduce(c->counts + 2 * W, c->counts + 2 * W + 1, 1, ncclInt64, ncclMin, c->nc, s));
  NCCL_IN_GROUP(op, ncclAllReduce(c->counts + 2 * W + 2, c->counts + 2 * W + 3, 1, ncclInt64, ncclSum, c->nc, s));
  NCCL_OR_RETURN(op, ncclGroupEnd());
  HIP_OR_RETURN(op, hipMemcpyAsync(c->h_counts, c->counts, (2 * W + 4) * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  HIP_OR_RETURN(op, hipStreamSynchronize(s));
  return FW_OK;
}
// the receive-side bookkeeping of one batch from the counts round (fw_exchange_plan) plus the counters
void comm_account(fw_comm* c, const fw_exchange_plan_t& pl, int64_t bytes_per_item) {
  c->stats.batches++;
  c->stats.items_sent += pl.items_sent;
  c->stats.items_received += pl.items_received;
  c->stats.bytes_sent += pl.items_sent * bytes_per_item;
  c->stats.bytes_received += pl.items_received * bytes_per_item;
}
}  // namespace
extern "C" {

int fw_comm_unique_id(void* id128) {
  if (!id128) return FW_ERR_ARG;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return FW_ERR_HIP;
  memcpy(id128, &id, sizeof id);
  return FW_OK;
}

int fw_comm_init(const void* id128, int32_t world, int32_t rank, int32_t device, fw_comm** out) {
  if (!id128 || !out || world < 1 || rank < 0 || rank >= world) return FW_ERR_ARG;
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return FW_ERR_HIP;
  fw_comm* c = new fw_comm();
  c->world = world;
  c->rank = rank;
  c->device = device;
  ncclUniqueId id;
  memcpy(&id, id128, sizeof id);
  if (ncclCommInitRank(&c->nc, world, id, rank) != ncclSuccess || dmalloc(&c->counts, 2 * (size_t)world + 4) != hipSuccess ||
      hipHostMalloc((void**)&c->h_counts, (2 * (size_t)world + 4) * sizeof(int64_t), hipHostMallocDefault) != hipSuccess) {
    fw_comm_destroy(c);
    return FW_ERR_HIP;
  }
  *out = c;
  return FW_OK;
}

void fw_comm_destroy(fw_comm* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->nc) (void)ncclCommDestroy(c->nc);
  for (int64_t** p : {&c->rk, &c->rt, &c->rv, &c->sk, &c->st, &c->sv, &c->counts}) cfree(*p);
  for (int32_t** p : {&c->rh, &c->sh}) cfree(*p);
  for (int i = 0; i < 6; i++) {
    cfree(c->ps[i]);
    cfree(c->pr[i]);
  }
  cfree(c->scratch);
  cfree(c->rs);
  cfree(c->rr);
  cfree(c->rgc);
  if (c->h_counts) (void)hipHostFree(c->h_counts);
  if (c->h_rgc) (void)hipHostFree(c->h_rgc);
  delete c;
}

int fw_exchange_plan(int32_t world, int32_t rank, const int64_t* counts, int64_t* send_off, int64_t* recv_off,
                     fw_exchange_plan_t* out) {
  if (world < 1 || rank < 0 || rank >= world || !counts || !send_off || !recv_off || !out) return FW_ERR_ARG;
  const int W = world;
  *out = fw_exchange_plan_t{};
  send_off[0] = recv_off[0] = 0;
  for (int p = 0; p < W; p++) {
    if (counts[p] < 0 || counts[W + p] < 0) return FW_ERR_STATE;
    send_off[p + 1] = send_off[p] + counts[p];
    recv_off[p + 1] = recv_off[p] + counts[W + p];
    if (p != rank) {
      out->items_sent += counts[p];
      out->items_received += counts[W + p];
    }
  }
  out->send_total = send_off[W];
  out->recv_total = recv_off[W];
  out->recv_bound = counts[2 * W + 3];
  // what a subtask receives is part of the batch of all subtasks; the own share is sent to itself
  if (out->recv_total > out->recv_bound || counts[rank] != counts[W + rank]) return FW_ERR_STATE;
  return FW_OK;
}

int fw_comm_get_stats(fw_comm* c, fw_comm_stats* out) {
  if (!c || !out) return FW_ERR_ARG;
  *out = c->stats;
  int n = 0, r = 0;
  if (ncclCommCount(c->nc, &n) != ncclSuccess || ncclCommUserRank(c->nc, &r) != ncclSuccess) return FW_ERR_HIP;
  out->world = n;
  out->rank = r;
  out->recv_capacity = std::max(c->rcap, c->pcap);
  return FW_OK;
}

int fw_keyby_push_device(fw_comm* c, fw_op* op, const int64_t* key, const int64_t* ts, const void* val,
                         const int32_t* key_hash, int64_t n, int64_t local_wm, int64_t* combined_wm) {
  if (!c || !op || n < 0 || (n > 0 && (!key || !ts || !val))) return op ? set_err(op, FW_ERR_ARG, "null argument") : FW_ERR_ARG;
  const bool hashed = op->cfg.key_kind == FW_KEY_HASHED;
  if (hashed && n > 0 && !key_hash) return set_err(op, FW_ERR_ARG, "key_hash required for FW_KEY_HASHED");
  int32_t kg0, kg1;
  {
    const int32_t M = op->cfg.max_parallelism, W = c->world, r = c->rank;
    kg0 = (r * M + W - 1) / W;  // KeyGroupRangeAssignment.computeKeyGroupRangeForOperatorIndex (:85-99)
    kg1 = ((r + 1) * M - 1) / W;
  }
  if (op->cfg.key_group_start != kg0 || op->cfg.key_group_end != kg1)
    return set_err(op, FW_ERR_ARG, "the operator's KeyGroupRange [%d, %d] is not subtask %d of %d's [%d, %d]",
                   op->cfg.key_group_start, op->cfg.key_group_end, c->rank, c->world, kg0, kg1);
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc;
  if ((rc = comm_reserve_send(op, c, std::max<int64_t>(n, 1)))) return rc;
  const int W = c->world;
  // the exchange runs on the stream the operator reads device batches on (fw_input_stream): with async input
  // that is not the stream of the previous batch's aggregation, so the count round trip below waits only for
  // the previous batch's partitioning (which read the received columns) and this batch's route
  hipStream_t s = input_stream_of(op);
  // group by destination subtask (stable), counts[W] on the device
  fwdev::launch_route(key, ts, (const int64_t*)val, key_hash, op->cfg.key_kind, n, op->cfg.max_parallelism, W, c->sk,
                      c->st, c->sv, c->sh, c->counts, (uint32_t*)c->scratch, s);
  HIP_OR_RETURN(op, hipGetLastError());
  c->h_counts[2 * W] = local_wm;
  c->h_counts[2 * W + 2] = n;
  HIP_OR_RETURN(op, hipMemcpyAsync(c->counts + 2 * W, c->h_counts + 2 * W, 3 * sizeof(int64_t), hipMemcpyHostToDevice, s));
  // the receive sizes: the one host round trip of the exchange
  if ((rc = comm_counts_round(op, c, s))) return rc;
  std::vector<int64_t> soff(W + 1, 0), roff(W + 1, 0);
  fw_exchange_plan_t pl;
  if ((rc = fw_exchange_plan(W, c->rank, c->h_counts, soff.data(), roff.data(), &pl)))
    return set_err(op, rc, "exchange: inconsistent counts round (received %lld records of a %lld-record batch)",
                   (long long)pl.recv_total, (long long)pl.recv_bound);
  const int64_t total = pl.recv_total;
  // the received columns grow geometrically with what this subtask receives (x1.25 over the batch that needs more,
  // capped by the bound from the counts round, the whole batch of all subtasks; comm_reserve_recv at least doubles),
  // so skew costs a few reallocations (counted in the stats) and not world-size times the memory (s is idle here,
  // and the previous batch's partitioning, the last reader of the received columns, ran on s)
  if (total > c->rcap) {
    const int64_t want = std::max(std::min(pl.recv_bound, total + total / 4), std::max<int64_t>(total, 1));
    if ((rc = comm_reserve_recv(op, c, want))) return rc;
    c->stats.recv_reallocs++;
  }
  comm_account(c, pl, hashed ? 28 : 24);
  // the columns peer to peer: each peer pair over its own xGMI link
  NCCL_OR_RETURN(op, ncclGroupStart());
  for (int p = 0; p < W; p++) {
    const size_t sc = (size_t)c->h_counts[p], rcn = (size_t)c->h_counts[W + p];
    NCCL_IN_GROUP(op, ncclSend(c->sk + soff[p], sc, ncclInt64, p, c->nc, s));
    NCCL_IN_GROUP(op, ncclSend(c->st + soff[p], sc, ncclInt64, p, c->nc, s));
    NCCL_IN_GROUP(op, ncclSend(c->sv + soff[p], sc, ncclInt64, p, c->nc, s));
    if (hashed) NCCL_IN_GROUP(op, ncclSend(c->sh + soff[p], sc, ncclInt32, p, c->nc, s));
    NCCL_IN_GROUP(op, ncclRecv(c->rk + roff[p], rcn, ncclInt64, p, c->nc, s));
    NCCL_IN_GROUP(op, ncclRecv(c->rt + roff[p], rcn, ncclInt64, p, c->nc, s));
    NCCL_IN_GROUP(op, ncclRecv(c->rv + roff[p], rcn, ncclInt64, p, c->nc, s));
    if (hashed) NCCL_IN_GROUP(op, ncclRecv(c->rh + roff[p], rcn, ncclInt32, p, c->nc, s));
  }
  NCCL_OR_RETURN(op, ncclGroupEnd());
  if (combined_wm) *combined_wm = c->h_counts[2 * W + 1];
  // processElement for the received batch (stream-ordered behind the receives: they ran on the stream the push
  // reads its columns on)
  return push_device_batches(op, c->rk, c->rt, c->rv, hashed ? c->rh : nullptr, total, true);
}

int fw_keyby_combine_push_device(fw_comm* c, fw_op* comb, fw_op* op, const int64_t* key, const int64_t* ts,
                                 const void* val, int64_t n, int64_t local_wm, int64_t* combined_wm) {
  if (!c || !comb || !op || n < 0 || (n > 0 && (!key || !ts || !val)))
    return op ? set_err(op, FW_ERR_ARG, "null argument") : FW_ERR_ARG;
  const int W = c->world;
  {
    const int32_t M = op->cfg.max_parallelism, r = c->rank;
    if (op->cfg.key_group_start != (r * M + W - 1) / W || op->cfg.key_group_end != ((r + 1) * M - 1) / W)
      return set_err(op, FW_ERR_ARG, "the operator's KeyGroupRange is not subtask %d of %d's", r, W);
  }
  if (combine_config_tag(comb->cfg) != combine_config_tag(op->cfg))
    return set_err(op, FW_ERR_ARG,
                   "the combiner is configured differently (assigner, size, offset, value type, key kind, max "
                   "parallelism or aggregate) than the operator");
  // HyperLogLog: the partial rows travel with their non-zero registers (fw_combine_extract_hll_device)
  const bool hll = op->cfg.aggregate == FW_AGG_HLL;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc;
  // HyperLogLog: a merge of the previous batch that suspended reruns its register raise from c->pr / c->rr when it is
  // settled, so it is settled before this batch reallocates those buffers or receives into them
  if (hll && (rc = settle(op))) return rc;
  // the batch into the combiner, ordered after the columns' producer (the caller's fw_stream(op) order)
  hipEvent_t ready = nullptr;
  HIP_OR_RETURN(op, hipEventCreateWithFlags(&ready, hipEventDisableTiming));
  HIP_OR_RETURN(op, hipEventRecord(ready, op->stream));
  HIP_OR_RETURN(op, hipStreamWaitEvent(comb->stream, ready, 0));
  (void)hipEventDestroy(ready);
  if ((rc = push_device_batches(comb, key, ts, val, nullptr, n, false))) return set_err(op, rc, "%s", comb->err.c_str());
  // drain it: the partials in key-group order, per-peer counts (and, for HLL, per-peer register counts)
  std::vector<int64_t> counts(W), rcounts(W, 0);
  int64_t np = 0, nr = 0;
  auto extract = [&](fw_partials* o) {
    return hll ? fw_combine_extract_hll_device(comb, W, o, c->pcap, counts.data(), rcounts.data(), &np, &nr)
               : fw_combine_extract_device(comb, W, o, c->pcap, counts.data(), &np);
  };
  fw_partials out{c->ps[0], c->ps[1], c->ps[2], c->ps[3], c->ps[4], c->ps[5]};
  rc = extract(&out);
  if (rc == FW_ERR_CAPACITY && np > c->pcap) {
    const int64_t cap = std::max<int64_t>(np, 2 * c->pcap);
    for (int i = 0; i < 6; i++) {
      cfree(c->ps[i]);
      cfree(c->pr[i]);
      HIP_OR_RETURN(op, dmalloc(&c->ps[i], (size_t)cap));
      HIP_OR_RETURN(op, dmalloc(&c->pr[i], (size_t)cap));
    }
    c->pcap = cap;
    out = fw_partials{c->ps[0], c->ps[1], c->ps[2], c->ps[3], c->ps[4], c->ps[5]};
    rc = extract(&out);
  }
  if (rc) return set_err(op, rc, "%s", comb->err.c_str());
  if (hll) {  // the registers, in partial order (each destination's one slice)
    if (nr > c->rscap) {
      const int64_t cap = std::max<int64_t>(nr, 2 * c->rscap);
      cfree(c->rs);
      c->rscap = 0;
      HIP_OR_RETURN(op, dmalloc(&c->rs, (size_t)cap));
      c->rscap = cap;
    }
    if ((rc = fw_combine_hll_registers_device(comb, &out, np, c->rs, c->rscap))) return set_err(op, rc, "%s", comb->err.c_str());
  }
  hipStream_t s = op->stream;
  for (int p = 0; p < W; p++) c->h_counts[p] = counts[p];
  c->h_counts[2 * W] = local_wm;
  c->h_counts[2 * W + 2] = np;
  HIP_OR_RETURN(op, hipMemcpyAsync(c->counts, c->h_counts, W * sizeof(int64_t), hipMemcpyHostToDevice, s));
  HIP_OR_RETURN(op, hipMemcpyAsync(c->counts + 2 * W, c->h_counts + 2 * W, 3 * sizeof(int64_t), hipMemcpyHostToDevice, s));
  if ((rc = comm_counts_round(op, c, s))) return rc;
  std::vector<int64_t> soff(W + 1, 0), roff(W + 1, 0), rsoff(W + 1, 0), rroff(W + 1, 0);
  fw_exchange_plan_t pl;
  if ((rc = fw_exchange_plan(W, c->rank, c->h_counts, soff.data(), roff.data(), &pl)))
    return set_err(op, rc, "exchange: inconsistent counts round (received %lld partials of %lld)",
                   (long long)pl.recv_total, (long long)pl.recv_bound);
  const int64_t total = pl.recv_total;
  int64_t rtotal = 0;
  if (hll) {  // the register counts: one more all-to-all (the receive sizes of the register lists)
    if (!c->rgc) {
      HIP_OR_RETURN(op, dmalloc(&c->rgc, 2 * (size_t)W));
      HIP_OR_RETURN(op, hipHostMalloc((void**)&c->h_rgc, 2 * (size_t)W * sizeof(int64_t), hipHostMallocDefault));
    }
    for (int p = 0; p < W; p++) c->h_rgc[p] = rcounts[p];
    HIP_OR_RETURN(op, hipMemcpyAsync(c->rgc, c->h_rgc, W * sizeof(int64_t), hipMemcpyHostToDevice, s));
    NCCL_OR_RETURN(op, ncclAllToAll(c->rgc, c->rgc + W, 1, ncclInt64, c->nc, s));
    HIP_OR_RETURN(op, hipMemcpyAsync(c->h_rgc, c->rgc, 2 * W * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIP_OR_RETURN(op, hipStreamSynchronize(s));
    for (int p = 0; p < W; p++) {
      rsoff[p + 1] = rsoff[p] + c->h_rgc[p];
      rroff[p + 1] = rroff[p] + c->h_rgc[W + p];
    }
    rtotal = rroff[W];
    if (rtotal > c->rrcap) {
      cfree(c->rr);
      const int64_t cap = std::max<int64_t>(rtotal, 2 * c->rrcap);
      c->rrcap = 0;
      HIP_OR_RETURN(op, dmalloc(&c->rr, (size_t)cap));
      c->rrcap = cap;
      c->stats.recv_reallocs++;
    }
  }
  if (total > c->pcap) {  // the receive columns for what this subtask receives (geometric, as fw_keyby_push_device)
    const int64_t cap = std::max(std::min(pl.recv_bound, total + total / 4), std::max<int64_t>(total, 2 * c->pcap));
    for (int i = 0; i < 6; i++) {
      cfree(c->pr[i]);
      HIP_OR_RETURN(op, dmalloc(&c->pr[i], (size_t)cap));
    }
    int64_t* ns[6] = {};
    for (int i = 0; i < 6; i++) {
      HIP_OR_RETURN(op, dmalloc(&ns[i], (size_t)cap));
      if (np) HIP_OR_RETURN(op, hipMemcpyAsync(ns[i], c->ps[i], np * 8, hipMemcpyDeviceToDevice, s));
    }
    HIP_OR_RETURN(op, hipStreamSynchronize(s));
    for (int i = 0; i < 6; i++) {
      cfree(c->ps[i]);
      c->ps[i] = ns[i];
    }
    c->pcap = cap;
    c->stats.recv_reallocs++;
  }
  comm_account(c, pl, 48);
  if (hll) {
    int64_t rs_other = 0, rr_other = 0;
    for (int p = 0; p < W; p++)
      if (p != c->rank) {
        rs_other += c->h_rgc[p];
        rr_other += c->h_rgc[W + p];
      }
    c->stats.bytes_sent += 4 * rs_other;
    c->stats.bytes_received += 4 * rr_other;
  }
  NCCL_OR_RETURN(op, ncclGroupStart());
  for (int p = 0; p < W; p++) {
    const size_t sc = (size_t)c->h_counts[p], rcn = (size_t)c->h_counts[W + p];
    for (int i = 0; i < 6; i++) {
      NCCL_IN_GROUP(op, ncclSend(c->ps[i] + soff[p], sc, ncclInt64, p, c->nc, s));
      NCCL_IN_GROUP(op, ncclRecv(c->pr[i] + roff[p], rcn, ncclInt64, p, c->nc, s));
    }
    if (hll) {
      NCCL_IN_GROUP(op, ncclSend(c->rs + rsoff[p], (size_t)c->h_rgc[p], ncclUint32, p, c->nc, s));
      NCCL_IN_GROUP(op, ncclRecv(c->rr + rroff[p], (size_t)c->h_rgc[W + p], ncclUint32, p, c->nc, s));
    }
  }
  NCCL_OR_RETURN(op, ncclGroupEnd());
  if (combined_wm) *combined_wm = c->h_counts[2 * W + 1];
  const fw_partials in{c->pr[0], c->pr[1], c->pr[2], c->pr[3], c->pr[4], c->pr[5], out.config};
  return hll ? fw_push_hll_partials_device(op, &in, total, c->rr, rtotal) : fw_push_partials_device(op, &in, total);
}

int fw_generate_device(uint64_t seed, int64_t first, int64_t n, int64_t num_keys, const double* zipf_cdf,
                       int64_t ts_base, int64_t rate, int64_t jitter, int64_t* key, int64_t* ts, int64_t* val,
                       int64_t* max_ts, void* stream) {
  if (n < 0 || num_keys < 1 || rate < 1 || jitter < 0) return FW_ERR_ARG;
  fwdev::launch_generate(seed, first, n, num_keys, zipf_cdf, ts_base, rate, jitter, key, ts, val, max_ts,
                         (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? FW_OK : FW_ERR_HIP;
}

}  // extern "C"
