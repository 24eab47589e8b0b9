// fw_runtime.cpp — host side of the C-ABI in include/flink_window.h.
//
// One fw_op = one WindowOperator subtask on one GPU: it owns the HBM state table of its
// KeyGroupRange, the per-batch scratch, the fired-row buffer and one HIP stream.  Every public
// call is serialised by the caller (the Flink task thread holds the checkpoint lock around
// processElement / processWatermark, StreamInputProcessor.java:211-222).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/flink_window.h"
#include "fw_internal.h"

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

}  // namespace

struct fw_op {
  fw_config cfg{};
  DevCfg dc{};
  int device = 0;
  hipStream_t stream = nullptr;
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
  uint32_t *hist = nullptr, *scan_tmp = nullptr;
  PRec* part = nullptr;  // partitioned records of the current batch
  int64_t *sk = nullptr, *stt = nullptr, *sv = nullptr;
  int32_t* skh = nullptr;

  DevRows out{};
  DevSide side{};
  DevOverflow ov{};
  Status* d_status = nullptr;
  Status* h_status = nullptr;
  unsigned long long* d_stats3 = nullptr;

  int64_t wm = INT64_MIN;
  int64_t records_in = 0;

  // optional per-kernel event timing (fw_profile)
  bool prof = false;
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
  }
  return FW_OK;
}

int ensure_out_capacity(fw_op* op, int64_t need) {
  if (need <= op->out.cap) return FW_OK;
  const int64_t cap = std::max(need, op->out.cap * 2);
  DevRows n{};
  int64_t** cols_new[7] = {&n.key, &n.start, &n.end, &n.cnt, &n.sum, &n.mn, &n.mx};
  int64_t** cols_old[7] = {&op->out.key, &op->out.start, &op->out.end, &op->out.cnt,
                           &op->out.sum, &op->out.mn, &op->out.mx};
  const int64_t keep = std::min<int64_t>((int64_t)op->h_status->out_rows, op->out.cap);
  for (int i = 0; i < 7; i++) {
    HIP_OR_RETURN(op, dmalloc(cols_new[i], (size_t)cap));
    if (keep > 0 && *cols_old[i])
      HIP_OR_RETURN(op, hipMemcpyAsync(*cols_new[i], *cols_old[i], keep * sizeof(int64_t), hipMemcpyDeviceToDevice,
                                       op->stream));
  }
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  for (int i = 0; i < 7; i++) dfree(*cols_old[i]);
  n.cap = cap;
  op->out = n;
  return FW_OK;
}

int ensure_side_capacity(fw_op* op, int64_t need) {
  if (need <= op->side.cap) return FW_OK;
  const int64_t cap = std::max(need, op->side.cap * 2);
  DevSide n{};
  int64_t** cols_new[3] = {&n.key, &n.ts, &n.val};
  int64_t** cols_old[3] = {&op->side.key, &op->side.ts, &op->side.val};
  const int64_t keep = std::min<int64_t>((int64_t)op->h_status->side_rows, op->side.cap);
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

enum { K_CLASSIFY = 0, K_SCAN, K_SCATTER, K_AGGREGATE, K_SLOW, K_FIRE };
const char* const KERNEL_NAMES[FW_NUM_KERNELS] = {"k_classify_hist", "k_scan", "k_scatter",
                                                  "k_aggregate",     "k_slow", "k_fire"};

hipEvent_t prof_event(fw_op* op) {
  if (!op->prof_free.empty()) {
    hipEvent_t e = op->prof_free.back();
    op->prof_free.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}
// time the launches issued by `launch` on the handle's stream as one interval of `kind`
template <class F>
void timed(fw_op* op, int kind, F&& launch) {
  if (!op->prof) {
    launch();
    return;
  }
  fw_op::Pair pr{prof_event(op), prof_event(op), kind};
  (void)hipEventRecord(pr.a, op->stream);
  launch();
  (void)hipEventRecord(pr.b, op->stream);
  op->prof_pending.push_back(pr);
}
void prof_collect(fw_op* op) {
  for (auto& pr : op->prof_pending) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, pr.a, pr.b) == hipSuccess) {
      op->prof_ms[pr.kind] += ms;
      op->prof_n[pr.kind]++;
    }
    op->prof_free.push_back(pr.a);
    op->prof_free.push_back(pr.b);
  }
  op->prof_pending.clear();
}

int sync_status(fw_op* op) {
  HIP_OR_RETURN(op, hipMemcpyAsync(op->h_status, op->d_status, sizeof(Status), hipMemcpyDeviceToHost, op->stream));
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  if (!op->prof_pending.empty()) prof_collect(op);
  return FW_OK;
}

// write one field of the device status from the host copy
template <class T>
int put_status_field(fw_op* op, T Status::*field) {
  const size_t off = (size_t)((char*)&(op->h_status->*field) - (char*)op->h_status);
  HIP_OR_RETURN(op, hipMemcpyAsync((char*)op->d_status + off, (char*)op->h_status + off, sizeof(T),
                                   hipMemcpyHostToDevice, op->stream));
  return FW_OK;
}

// grow every region to new_log_r, re-inserting the live entries and then the parked overflow
int grow_table(fw_op* op, int new_log_r) {
  DevCfg nc = op->dc;
  nc.log_r = new_log_r;
  DevTable nt{};
  nt.cur = op->tb.cur;
  nt.live = op->tb.live;
  nt.next_timer = op->tb.next_timer;
  int rc = alloc_table(op, nt, nc, false);
  if (rc) return rc;
  fwdev::launch_rehash(op->dc, op->tb, nc, nt, op->stream);
  if (op->h_status->overflow_count > 0) fwdev::launch_merge_overflow(nc, nt, op->ov, op->d_status, op->stream);
  HIP_OR_RETURN(op, hipGetLastError());
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  free_table(op->tb);
  op->tb = nt;
  op->dc = nc;
  op->table_slots = (int64_t)nc.P << nc.log_r;
  op->grows++;
  op->h_status->overflow_count = 0;
  if ((rc = put_status_field(op, &Status::overflow_count))) return rc;
  // the parked deltas may have been larger than the slack: re-grow the overflow list with the table
  const int64_t ovcap = std::max<int64_t>(op->table_slots / 2, 1 << 16);
  if (ovcap > op->ov.cap) {
    dfree(op->ov.ent);
    dfree(op->ov.part);
    HIP_OR_RETURN(op, dmalloc(&op->ov.ent, (size_t)ovcap));
    HIP_OR_RETURN(op, dmalloc(&op->ov.part, (size_t)ovcap));
    op->ov.cap = ovcap;
  }
  return ensure_out_capacity(op, (int64_t)op->h_status->out_rows + op->table_slots);
}

// after every push / watermark: surface errors, grow the table when a region is over half full
int after_sync(fw_op* op) {
  Status& s = *op->h_status;
  if (s.flags & FW_STATUS_OVERFLOW_LOST)
    return set_err(op, FW_ERR_CAPACITY,
                   "state table overflowed beyond its overflow list (raise fw_config.expected_entries)");
  if (s.flags & FW_STATUS_OUT_FULL) return set_err(op, FW_ERR_STATE, "fired-row buffer overflow");
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
  const int64_t R = int64_t(1) << op->dc.log_r;
  int log_r = op->dc.log_r;
  if (s.overflow_count > 0 || s.max_live > R / 2) {
    int64_t need = std::max<int64_t>(s.max_live, 1) + (int64_t)s.overflow_count;
    while ((int64_t(1) << log_r) < 2 * need || log_r == op->dc.log_r) log_r++;
    int rc = grow_table(op, log_r);
    if (rc) return rc;
  }
  s.max_live = 0;
  return put_status_field(op, &Status::max_live);
}

int push_device(fw_op* op, const int64_t* key, const int64_t* ts, const int64_t* val, const int32_t* kh, int64_t n) {
  if (n == 0) return FW_OK;
  int rc;
  const DevCfg& c = op->dc;
  // every record may be replayed on the ordered path and late-fire all its windows
  if ((rc = ensure_out_capacity(op, (int64_t)op->h_status->out_rows + op->table_slots + n * c.wpr))) return rc;
  if (c.side_output && (rc = ensure_side_capacity(op, (int64_t)op->h_status->side_rows + n))) return rc;
  const DevCfg& cc = op->dc;
  const int32_t T = (int32_t)((n + FW_TILE - 1) / FW_TILE);
  const int64_t m = (int64_t)(cc.P + 1) * T;
  op->h_status->slow_count = 0;
  if ((rc = put_status_field(op, &Status::slow_count))) return rc;
  timed(op, K_CLASSIFY, [&] {
    fwdev::launch_classify_hist(cc, op->wm, key, ts, kh, n, T, op->hist, op->d_status, op->stream);
  });
  timed(op, K_SCAN, [&] { fwdev::launch_scan(op->hist, m, op->scan_tmp, op->stream); });
  timed(op, K_SCATTER, [&] {
    fwdev::launch_scatter(cc, op->wm, key, ts, val, kh, n, T, op->hist, op->part, op->sk, op->stt, op->sv, op->skh,
                          op->side, op->d_status, op->stream);
  });
  timed(op, K_AGGREGATE, [&] {
    fwdev::launch_aggregate(cc, op->wm, op->part, op->hist, T, op->tb, op->ov, op->d_status, op->stream);
  });
  timed(op, K_SLOW, [&] {
    fwdev::launch_slow(cc, op->wm, op->sk, op->stt, op->sv, op->skh, op->tb, op->out, op->side, op->d_status,
                       op->stream);
  });
  HIP_OR_RETURN(op, hipGetLastError());
  op->records_in += n;
  if ((rc = sync_status(op))) return rc;
  return after_sync(op);
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
  } else if (cfg.assigner == FW_SESSION) {
    if (cfg.gap <= 0) snprintf(msg, sizeof msg, "EventTimeSessionWindows parameters must satisfy 0 < size");
  } else {
    snprintf(msg, sizeof msg, "unknown assigner %d", cfg.assigner);
  }
  if (!msg[0] && cfg.allowed_lateness < 0) snprintf(msg, sizeof msg, "The allowed lateness cannot be negative.");
  if (!msg[0] && (cfg.value_type < FW_VAL_I64 || cfg.value_type > FW_VAL_F64))
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
  fw_op* op = new fw_op();
  op->cfg = cfg;
  if (msg[0]) {
    op->err = msg;
    *out = op;
    return FW_ERR_ARG;
  }
  *out = op;
  op->device = cfg.device;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  HIP_OR_RETURN(op, hipStreamCreateWithFlags(&op->stream, hipStreamNonBlocking));

  DevCfg& c = op->dc;
  c.assigner = cfg.assigner;
  c.vtype = cfg.value_type;
  c.key_kind = cfg.key_kind;
  c.purging = cfg.purging;
  c.side_output = cfg.side_output;
  c.max_par = cfg.max_parallelism;
  c.kg0 = cfg.key_group_start;
  c.n_kg = cfg.key_group_end - cfg.key_group_start + 1;
  int64_t s = cfg.sub_partitions;
  if (s == 0) s = std::max<int64_t>(1, next_pow2(std::max<int64_t>(1, 2048 / c.n_kg)));
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
  if (cfg.assigner != FW_SESSION) {
    make_div_inv((uint64_t)c.size, &c.mag_size, &c.l_size);
    make_div_inv((uint64_t)c.slide, &c.mag_slide, &c.l_slide);
  }
  const int64_t expected = cfg.expected_entries > 0 ? cfg.expected_entries : (int64_t)c.P * 512;
  c.log_r = std::max(8, ilog2(4 * ((expected + c.P - 1) / c.P)));
  op->table_slots = (int64_t)c.P << c.log_r;

  op->max_batch = cfg.max_batch > 0 ? cfg.max_batch : (int64_t(1) << 24);
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
  HIP_OR_RETURN(op, dmalloc(&op->hist, m));
  HIP_OR_RETURN(op, dmalloc(&op->scan_tmp, m / 4096 + 2));
  HIP_OR_RETURN(op, dmalloc(&op->part, mb));
  HIP_OR_RETURN(op, dmalloc(&op->sk, mb));
  HIP_OR_RETURN(op, dmalloc(&op->stt, mb));
  HIP_OR_RETURN(op, dmalloc(&op->sv, mb));
  HIP_OR_RETURN(op, dmalloc(&op->skh, mb));
  const int64_t ovcap = std::max<int64_t>(op->table_slots / 2, 1 << 16);
  HIP_OR_RETURN(op, dmalloc(&op->ov.ent, ovcap));
  HIP_OR_RETURN(op, dmalloc(&op->ov.part, ovcap));
  op->ov.cap = ovcap;
  HIP_OR_RETURN(op, dmalloc(&op->d_status, 1));
  HIP_OR_RETURN(op, dmalloc(&op->d_stats3, 4));
  HIP_OR_RETURN(op, hipMemsetAsync(op->d_status, 0, sizeof(Status), op->stream));
  HIP_OR_RETURN(op, hipHostMalloc((void**)&op->h_status, sizeof(Status), hipHostMallocDefault));
  memset(op->h_status, 0, sizeof(Status));
  if ((rc = ensure_out_capacity(op, 2 * op->table_slots))) return rc;
  if ((rc = ensure_side_capacity(op, cfg.side_output ? mb : 1))) return rc;
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  return FW_OK;
}

void fw_destroy(fw_op* op) {
  if (!op) return;
  if (op->stream) {
    (void)hipSetDevice(op->device);
    (void)hipStreamSynchronize(op->stream);
  }
  free_table(op->tb);
  dfree(op->tb.cur);
  dfree(op->tb.live);
  dfree(op->tb.next_timer);
  dfree(op->in_key);
  dfree(op->in_ts);
  dfree(op->in_val);
  dfree(op->in_kh);
  dfree(op->hist);
  dfree(op->scan_tmp);
  dfree(op->part);
  dfree(op->sk);
  dfree(op->stt);
  dfree(op->sv);
  dfree(op->skh);
  dfree(op->ov.ent);
  dfree(op->ov.part);
  for (int64_t** col : {&op->out.key, &op->out.start, &op->out.end, &op->out.cnt, &op->out.sum, &op->out.mn,
                        &op->out.mx, &op->side.key, &op->side.ts, &op->side.val})
    dfree(*col);
  dfree(op->d_status);
  dfree(op->d_stats3);
  for (auto& pr : op->prof_pending) {
    (void)hipEventDestroy(pr.a);
    (void)hipEventDestroy(pr.b);
  }
  for (hipEvent_t e : op->prof_free) (void)hipEventDestroy(e);
  if (op->h_status) (void)hipHostFree(op->h_status);
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
    int rc = push_device(op, op->in_key, op->in_ts, op->in_val, op->in_kh, m);
    if (rc) return rc;
  }
  return FW_OK;
}

int fw_push_batch_device(fw_op* op, const int64_t* key, const int64_t* ts, const void* val, const int32_t* key_hash,
                         int64_t n) {
  if (!op || n < 0 || (n > 0 && (!key || !ts || !val))) return op ? set_err(op, FW_ERR_ARG, "null column") : FW_ERR_ARG;
  if (op->cfg.key_kind == FW_KEY_HASHED && n > 0 && !key_hash)
    return set_err(op, FW_ERR_ARG, "key_hash required for FW_KEY_HASHED");
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  for (int64_t b = 0; b < n; b += op->max_batch) {
    const int64_t m = std::min(op->max_batch, n - b);
    int rc = push_device(op, key + b, ts + b, (const int64_t*)val + b, key_hash ? key_hash + b : nullptr, m);
    if (rc) return rc;
  }
  return FW_OK;
}

int fw_advance_watermark(fw_op* op, int64_t wm, int64_t* n_pending) {
  if (!op) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  int rc = ensure_out_capacity(op, (int64_t)op->h_status->out_rows + op->table_slots);
  if (rc) return rc;
  timed(op, K_FIRE, [&] { fwdev::launch_fire(op->dc, wm, op->tb, op->out, op->d_status, op->stream); });
  HIP_OR_RETURN(op, hipGetLastError());
  op->wm = wm;  // HeapInternalTimerService.advanceWatermark: currentWatermark = time
  if ((rc = sync_status(op))) return rc;
  if ((rc = after_sync(op))) return rc;
  if (n_pending) *n_pending = (int64_t)op->h_status->out_rows;
  return FW_OK;
}

int fw_pending(fw_op* op, int64_t* n_rows, int64_t* n_side) {
  if (!op) return FW_ERR_ARG;
  if (n_rows) *n_rows = (int64_t)op->h_status->out_rows;
  if (n_side) *n_side = (int64_t)op->h_status->side_rows;
  return FW_OK;
}

int fw_drain_rows(fw_op* op, const fw_rows* dst, int64_t cap, int64_t* n) {
  if (!op || !dst) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  const int64_t have = (int64_t)op->h_status->out_rows;
  if (cap < have) {
    if (n) *n = have;
    return set_err(op, FW_ERR_ARG, "drain capacity %lld < pending rows %lld", (long long)cap, (long long)have);
  }
  if (have > 0) {
    int64_t* d[7] = {dst->key, dst->start, dst->end, dst->count, dst->sum, dst->min, dst->max};
    int64_t* s[7] = {op->out.key, op->out.start, op->out.end, op->out.cnt, op->out.sum, op->out.mn, op->out.mx};
    for (int i = 0; i < 7; i++)
      if (d[i]) HIP_OR_RETURN(op, hipMemcpyAsync(d[i], s[i], have * 8, hipMemcpyDeviceToHost, op->stream));
  }
  op->h_status->out_rows = 0;
  int rc = put_status_field(op, &Status::out_rows);
  if (rc) return rc;
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  if (n) *n = have;
  return FW_OK;
}

int fw_drain_side(fw_op* op, const fw_side_rows* dst, int64_t cap, int64_t* n) {
  if (!op || !dst) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  const int64_t have = (int64_t)op->h_status->side_rows;
  if (cap < have) {
    if (n) *n = have;
    return set_err(op, FW_ERR_ARG, "drain capacity %lld < pending side rows %lld", (long long)cap, (long long)have);
  }
  if (have > 0) {
    int64_t* d[3] = {dst->key, dst->ts, dst->val};
    int64_t* s[3] = {op->side.key, op->side.ts, op->side.val};
    for (int i = 0; i < 3; i++)
      if (d[i]) HIP_OR_RETURN(op, hipMemcpyAsync(d[i], s[i], have * 8, hipMemcpyDeviceToHost, op->stream));
  }
  op->h_status->side_rows = 0;
  int rc = put_status_field(op, &Status::side_rows);
  if (rc) return rc;
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  if (n) *n = have;
  return FW_OK;
}

int fw_rows_device(fw_op* op, fw_rows* view, int64_t* n) {
  if (!op || !view) return FW_ERR_ARG;
  view->key = op->out.key;
  view->start = op->out.start;
  view->end = op->out.end;
  view->count = op->out.cnt;
  view->sum = op->out.sum;
  view->min = op->out.mn;
  view->max = op->out.mx;
  if (n) *n = (int64_t)op->h_status->out_rows;
  return FW_OK;
}

int fw_clear_pending(fw_op* op) {
  if (!op) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  op->h_status->out_rows = 0;
  op->h_status->side_rows = 0;
  int rc = put_status_field(op, &Status::out_rows);
  if (!rc) rc = put_status_field(op, &Status::side_rows);
  return rc;
}

int fw_get_stats(fw_op* op, fw_stats* o) {
  if (!op || !o) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipSetDevice(op->device));
  HIP_OR_RETURN(op, hipMemsetAsync(op->d_stats3, 0, 4 * sizeof(unsigned long long), op->stream));
  fwdev::launch_table_stats(op->dc, op->tb, op->d_stats3, op->stream);
  unsigned long long h3[4];
  HIP_OR_RETURN(op, hipMemcpyAsync(h3, op->d_stats3, sizeof h3, hipMemcpyDeviceToHost, op->stream));
  int rc = sync_status(op);
  if (rc) return rc;
  const Status& s = *op->h_status;
  o->records_in = op->records_in;
  o->late_records_dropped = (int64_t)s.late_dropped;
  o->keyed_state_entries = (int64_t)h3[0];
  o->event_time_timers = (int64_t)h3[1];
  o->current_watermark = op->wm;
  o->fired_rows_total = (int64_t)s.fired_total;
  o->pending_rows = (int64_t)s.out_rows;
  o->pending_side_rows = (int64_t)s.side_rows;
  o->table_capacity = op->table_slots;
  o->table_grows = op->grows;
  o->slow_path_records = (int64_t)s.slow_total;
  o->state_merges = (int64_t)s.merged;
  return FW_OK;
}

int fw_profile(fw_op* op, int enable) {
  if (!op) return FW_ERR_ARG;
  op->prof = enable != 0;
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

int fw_synchronize(fw_op* op) {
  if (!op) return FW_ERR_ARG;
  HIP_OR_RETURN(op, hipStreamSynchronize(op->stream));
  return FW_OK;
}

void* fw_stream(fw_op* op) { return op ? (void*)op->stream : nullptr; }

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

int fw_generate_device(uint64_t seed, int64_t first, int64_t n, int64_t num_keys, const double* zipf_cdf,
                       int64_t ts_base, int64_t rate, int64_t jitter, int64_t* key, int64_t* ts, int64_t* val,
                       int64_t* max_ts, void* stream) {
  if (n < 0 || num_keys < 1 || rate < 1 || jitter < 0) return FW_ERR_ARG;
  fwdev::launch_generate(seed, first, n, num_keys, zipf_cdf, ts_base, rate, jitter, key, ts, val, max_ts,
                         (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? FW_OK : FW_ERR_HIP;
}

}  // extern "C"
