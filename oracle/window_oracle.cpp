// window_oracle.cpp — CPU restatement of Flink's keyed event-time WindowOperator.
// TEST INFRASTRUCTURE ONLY (parity checker + cpu_baseline).  See window_oracle.h for
// the list of reference files restated here.  Paths below are relative to
// /root/reference/flink-streaming-java/src/main/java/org/apache/flink/streaming/ unless
// they start with flink-*.
#include "window_oracle.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <deque>
#include <map>
#include <queue>
#include <set>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

// ---------------------------------------------------------------- Java arithmetic
inline int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
inline int64_t jsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
const int64_t LMAX = INT64_MAX;
const int64_t LMIN = INT64_MIN;

// flink-core/src/main/java/org/apache/flink/util/MathUtils.java:191-198
inline int32_t bit_mix(int32_t in) {
  uint32_t x = (uint32_t)in;
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return (int32_t)x;
}
inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
// MathUtils.java:134-154
inline int32_t murmur(int32_t code) {
  uint32_t c = (uint32_t)code;
  c *= 0xcc9e2d51u;
  c = rotl32(c, 15);
  c *= 0x1b873593u;
  c = rotl32(c, 13);
  c = c * 5u + 0xe6546b64u;
  c ^= 4u;
  int32_t r = bit_mix((int32_t)c);
  if (r >= 0) return r;
  if (r != INT32_MIN) return -r;
  return 0;
}
inline int32_t long_hash(int64_t v) { return (int32_t)(v ^ (int64_t)((uint64_t)v >> 32)); }

// TimeWindow.java:254-256  (Java: timestamp - (timestamp - offset + windowSize) % windowSize)
inline int64_t window_start(int64_t ts, int64_t offset, int64_t size) {
  int64_t t = jadd(jsub(ts, offset), size);
  return jsub(ts, t % size);
}

// Double.doubleToLongBits (canonical NaN) and Double.compare ordering as a signed key.
inline int64_t dbits(double d) {
  if (std::isnan(d)) return 0x7ff8000000000000LL;
  int64_t b;
  memcpy(&b, &d, 8);
  return b;
}
inline double bitsd(int64_t b) {
  double d;
  memcpy(&d, &b, 8);
  return d;
}
inline int java_double_compare(double a, double b) {
  if (a < b) return -1;
  if (a > b) return 1;
  int64_t x = dbits(a), y = dbits(b);
  return x == y ? 0 : (x < y ? -1 : 1);
}

// ---------------------------------------------------------------- TimeWindow
struct TW {
  int64_t start, end;
  int64_t maxTs() const { return jsub(end, 1); }  // TimeWindow.java:83-85
  bool operator==(const TW& o) const { return start == o.start && end == o.end; }
  bool operator<(const TW& o) const { return start != o.start ? start < o.start : end < o.end; }
  bool intersects(const TW& o) const { return start <= o.end && end >= o.start; }  // :117-119
  TW cover(const TW& o) const { return TW{std::min(start, o.start), std::max(end, o.end)}; }  // :124-126
};

struct Acc {
  int64_t cnt = 0;
  int64_t isum = 0;
  double dsum = 0.0;
  int64_t imn = 0, imx = 0;
  double dmn = 0.0, dmx = 0.0;
  std::vector<uint8_t> regs;  // OR_AGG_HLL registers (2^p)
  int64_t first = 0;          // OR_AGG_FIRST: arrival ordinal of the element that created the state
  int64_t by_val = 0, by_ord = 0;  // OR_AGG_MINBY / MAXBY: the selected element's field and ordinal
  std::vector<double> td_sum;      // OR_AGG_TDIGEST: centroids (sum, weight), in order
  std::vector<int64_t> td_w;
  std::vector<int64_t> td_buf;     // values added since the last compression (f64 bits)
  bool td_merged = false;          // centroids of merged digests joined since the last compression
  // OR_AGG_ROW: per value column, the accumulators of the Table aggregates over it (window_oracle.h)
  struct RowCol {
    int64_t nn = 0;        // non-null values (CountAggFunction / the Sum, Min, Max accumulators' f1 flag)
    __int128 isum = 0;     // exact integral sum (BigIntegralAvgAccumulator; its low bits are the wrapped sums)
    double dsum = 0.0;     // Double sum (SumAggFunction[Double], FloatingAvgAccumulator over doubleValue())
    double fsum = 0.0;     // Float sum, rounded to float after every addition (SumAggFunction[Float])
    int64_t imn = 0, imx = 0;
    double dmn = 0.0, dmx = 0.0;
  };
  std::vector<RowCol> row;
};

// ---------------------------------------------------------------- t-digest (window_oracle.h OR_AGG_TDIGEST)
// Double.compare order of f64 bits as an unsigned key (canonical NaN largest)
inline uint64_t td_key(int64_t bits) {
  if ((bits & 0x7ff0000000000000LL) == 0x7ff0000000000000LL && (bits & 0x000fffffffffffffLL)) bits = 0x7ff8000000000000LL;
  const int64_t s = bits >= 0 ? bits : (bits ^ 0x7fffffffffffffffLL);
  return (uint64_t)s ^ 0x8000000000000000ULL;
}
// qb[b] = sin(pi b / delta)^2, b = 0 .. delta/2 (the k1 scale function's unit steps)
std::vector<double> td_bounds(int delta) {
  const int nb = delta / 2;
  std::vector<double> q(nb + 1);
  for (int b = 0; b <= nb; b++) {
    const double s = std::sin(M_PI * (double)b / (double)delta);
    q[b] = s * s;
  }
  q[0] = 0.0;
  q[nb] = 1.0;
  return q;
}
// group of an item of weight w whose predecessors weigh c (W = total weight): the bucket of its midpoint,
// the largest b < nb with W*qb[b] <= c + w/2
inline int td_slot(const std::vector<double>& q, double W, int64_t c, int64_t w) {
  const int nb = (int)q.size() - 1;
  const double mid = (double)c + (double)w * 0.5;
  int lo = 0, hi = nb - 1;
  while (lo < hi) {
    const int m = (lo + hi + 1) >> 1;
    if (W * q[m] <= mid)
      lo = m;
    else
      hi = m - 1;
  }
  return lo;
}
// sum of up to 64 values as the perfect binary tree over 64 slots in order (empty slots contribute nothing)
struct TreeSum {
  double v;
  bool any;
};
TreeSum td_tree(const double* x, int n, int lo, int width) {
  if (lo >= n) return TreeSum{0.0, false};
  if (width == 1) return TreeSum{x[lo], true};
  const TreeSum a = td_tree(x, n, lo, width / 2), b = td_tree(x, n, lo + width / 2, width / 2);
  if (!b.any) return a;
  return TreeSum{a.v + b.v, true};
}
// merge the buffered values into the centroids (the compression at the end of a batch)
void td_compress(Acc& a, const std::vector<double>& q) {
  if (a.td_buf.empty() && !a.td_merged) return;
  a.td_merged = false;
  std::vector<uint64_t> nv(a.td_buf.size());
  for (size_t i = 0; i < nv.size(); i++) nv[i] = td_key(a.td_buf[i]);
  std::sort(nv.begin(), nv.end());
  a.td_buf.clear();
  int64_t W = 0;
  for (int64_t w : a.td_w) W += w;
  W += (int64_t)nv.size();
  const double Wd = (double)W;
  std::vector<double> os;
  std::vector<int64_t> ow;
  os.swap(a.td_sum);
  ow.swap(a.td_w);
  // one group: its old centroid sums added left to right, its new values in blocks of 64 (each a tree sum),
  // the block sums added left to right
  struct Group {
    double old_sum = 0.0, new_sum = 0.0;
    bool any_old = false, any_new = false;
    int64_t w = 0;
    std::vector<double> blk;
  } g;
  auto flush_block = [&]() {
    if (g.blk.empty()) return;
    const double t = td_tree(g.blk.data(), (int)g.blk.size(), 0, 64).v;
    g.new_sum = g.any_new ? g.new_sum + t : t;
    g.any_new = true;
    g.blk.clear();
  };
  auto emit = [&]() {
    flush_block();
    if (g.w == 0) return;
    a.td_sum.push_back(g.any_old && g.any_new ? g.old_sum + g.new_sum : g.any_old ? g.old_sum : g.new_sum);
    a.td_w.push_back(g.w);
    g = Group{};
  };
  size_t i = 0, j = 0;
  int64_t c = 0;
  int cur = -1;
  while (i < nv.size() || j < os.size()) {
    bool take_new = j == os.size();
    if (!take_new && i < nv.size()) {
      int64_t mb;
      const double mean = os[j] / (double)ow[j];
      memcpy(&mb, &mean, 8);
      take_new = nv[i] <= td_key(mb);
    }
    double x;
    int64_t w;
    if (take_new) {
      const int64_t s = (int64_t)(nv[i++] ^ 0x8000000000000000ULL);
      x = bitsd(s >= 0 ? s : (s ^ 0x7fffffffffffffffLL));
      w = 1;
    } else {
      x = os[j];
      w = ow[j++];
    }
    const int slot = td_slot(q, Wd, c, w);
    if (slot != cur) emit();
    cur = slot;
    if (take_new) {
      g.blk.push_back(x);
      if (g.blk.size() == 64) flush_block();
    } else {
      g.old_sum = g.any_old ? g.old_sum + x : x;
      g.any_old = true;
    }
    g.w += w;
    c += w;
  }
  emit();
}
// piecewise-linear quantile through (0, min), (centre_i, mean_i), (W, max)
double td_quantile(const Acc& a, double mn, double mx, double qv) {
  const size_t n = a.td_sum.size();
  if (n == 0) return NAN;
  double W = 0.0;
  for (int64_t w : a.td_w) W += (double)w;
  const double x = qv * W;
  double x0 = 0.0, y0 = mn, before = 0.0;
  for (size_t i = 0; i < n; i++) {
    const double t = before + (double)a.td_w[i] * 0.5;
    const double m = a.td_sum[i] / (double)a.td_w[i];
    if (t >= x) return y0 + (m - y0) * ((x - x0) / (t - x0));
    x0 = t;
    y0 = m;
    before += (double)a.td_w[i];
  }
  return y0 + (mx - y0) * ((x - x0) / (W - x0));
}

// AggregateFunction.merge of two t-digests (this build's definition, window_oracle.h OR_AGG_TDIGEST): the union of
// their centroids, ordered by (mean key, weight, sum key), and of their buffered values; the union is compressed with
// the buffered values at the end of the batch (td_compress), so a merge of several digests in one batch gives the
// same result in any order (the GPU merges a session's whole connected component at once)
inline uint64_t td_cent_mean_key(double sum, int64_t w) {
  const double m = sum / (double)w;
  int64_t b;
  memcpy(&b, &m, 8);
  return td_key(b);
}
void td_union(Acc& r, const Acc& b) {
  std::vector<size_t> idx(r.td_sum.size() + b.td_sum.size());
  std::vector<double> s(idx.size());
  std::vector<int64_t> w(idx.size());
  for (size_t i = 0; i < r.td_sum.size(); i++) s[i] = r.td_sum[i], w[i] = r.td_w[i];
  for (size_t i = 0; i < b.td_sum.size(); i++) s[r.td_sum.size() + i] = b.td_sum[i], w[r.td_sum.size() + i] = b.td_w[i];
  for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
  auto sk = [&](size_t i) {
    int64_t bits;
    memcpy(&bits, &s[i], 8);
    return td_key(bits);
  };
  std::sort(idx.begin(), idx.end(), [&](size_t x, size_t y) {
    const uint64_t mx = td_cent_mean_key(s[x], w[x]), my = td_cent_mean_key(s[y], w[y]);
    if (mx != my) return mx < my;
    if (w[x] != w[y]) return w[x] < w[y];
    return sk(x) < sk(y);
  });
  r.td_sum.resize(idx.size());
  r.td_w.resize(idx.size());
  for (size_t i = 0; i < idx.size(); i++) r.td_sum[i] = s[idx[i]], r.td_w[i] = w[idx[i]];
  r.td_buf.insert(r.td_buf.end(), b.td_buf.begin(), b.td_buf.end());
  r.td_merged = true;
}

// ---------------------------------------------------------------- HyperLogLog (window_oracle.h)
inline uint64_t hll_fmix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}
inline void hll_add(std::vector<uint8_t>& regs, int p, uint64_t item) {
  const uint64_t h = hll_fmix64(item);
  const uint64_t j = h >> (64 - p);
  const uint64_t w = (h << p) | (1ULL << (p - 1));
  const uint8_t rank = (uint8_t)(__builtin_clzll(w) + 1);
  if (regs[j] < rank) regs[j] = rank;
}
inline double hll_alpha(int64_t m) {
  if (m == 16) return 0.673;
  if (m == 32) return 0.697;
  if (m == 64) return 0.709;
  return 0.7213 / (1.0 + 1.079 / (double)m);
}
// estimate, zero-register count V, and the low 64 bits of S
inline void hll_result(const std::vector<uint8_t>& regs, int p, double* est, int64_t* zeros, int64_t* lo64) {
  const int64_t m = (int64_t)1 << p;
  const int rmax = 65 - p;
  unsigned __int128 S = 0;
  int64_t V = 0;
  for (int64_t j = 0; j < m; j++) {
    S += (unsigned __int128)1 << (rmax - regs[j]);
    V += regs[j] == 0;
  }
  const uint64_t hi = (uint64_t)(S >> 64), lo = (uint64_t)S;
  const double sd = (double)hi * 18446744073709551616.0 + (double)lo;
  const double raw = (hll_alpha(m) * (double)m * (double)m) * std::ldexp(1.0, rmax) / sd;
  *est = (raw <= 2.5 * (double)m && V > 0) ? (double)m * std::log((double)m / (double)V) : raw;
  *zeros = V;
  *lo64 = (int64_t)lo;
}

struct KW {
  int64_t key;
  TW w;
  bool operator==(const KW& o) const { return key == o.key && w == o.w; }
};
inline uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}
struct KWHash {
  size_t operator()(const KW& k) const {
    return mix64((uint64_t)k.key * 0x9E3779B97F4A7C15ULL ^ mix64((uint64_t)k.w.start) ^ ((uint64_t)k.w.end << 1));
  }
};

// InternalTimer: (timestamp, key, namespace).  Ordering by timestamp only
// (InternalTimer.java:62-64); ties are broken deterministically here — the
// reference leaves them in PriorityQueue heap order, i.e. undefined.
struct Timer {
  int64_t ts, key;
  TW w;
  bool operator==(const Timer& o) const { return ts == o.ts && key == o.key && w == o.w; }
};
struct TimerHash {
  size_t operator()(const Timer& t) const { return KWHash()(KW{t.key, t.w}) ^ mix64((uint64_t)t.ts); }
};
struct TimerGreater {
  bool operator()(const Timer& a, const Timer& b) const {
    if (a.ts != b.ts) return a.ts > b.ts;
    if (a.key != b.key) return a.key > b.key;
    return b.w < a.w;
  }
};

struct OpError {
  int code;
};

class WindowOperatorOracle {
 public:
  explicit WindowOperatorOracle(const oracle_cfg& c) : cfg(c) {
    if (cfg.aggregate == OR_AGG_TDIGEST) td_q = td_bounds(cfg.td_delta);
  }

  oracle_cfg cfg;
  std::vector<double> td_q;                                    // OR_AGG_TDIGEST bucket bounds qb[]
  std::vector<KW> td_touched;                                  // digests with buffered values
  std::vector<std::vector<std::pair<double, int64_t>>> row_digest;  // per emitted row: its centroids
  // end of a processElements batch: the t-digests compress their buffered values
  void end_batch() {
    for (const KW& k : td_touched) {
      auto it = state.find(k);
      if (it != state.end()) td_compress(it->second, td_q);
    }
    td_touched.clear();
  }
  int64_t wm = LMIN;  // HeapInternalTimerService.currentWatermark initial value
  int64_t epoch = 0;
  int64_t late_dropped = 0;
  std::vector<oracle_row> rows;
  std::vector<oracle_side_row> side;

  std::unordered_map<KW, Acc, KWHash> state;  // window-contents (key, namespace) -> ACC
  // event-time timers: dedup set + min-heap with lazy deletion
  std::unordered_set<Timer, TimerHash> timer_set;
  std::priority_queue<Timer, std::vector<Timer>, TimerGreater> timer_q;
  // MergingWindowSet per key: window -> state window
  std::unordered_map<int64_t, std::map<TW, TW>> merging;

  bool is_merging() const { return cfg.assigner == OR_SESSION; }

  // ------------------------------------------------ accumulator (CountSumMinMax)
  // (OR_AGG_FIRST: HeapReducingState.add, HeapReducingState.java:72-84 — the element that finds no
  // state becomes it, and SumAggregator.reduce / ComparableAggregator.reduce keep a copy of their first
  // argument (SumAggregator.java:66-76, ComparableAggregator.java:72-94): the first element survives)
  // Comparator.MinByComparator / MaxByComparator order the field with compareTo: Long / Integer by value,
  // Double by Double.compare (Comparator.java:35-108)
  bool is_float() const { return cfg.value_type == OR_VAL_F64 || cfg.value_type == OR_VAL_F32; }
  // the sum in the field's type: Integer / Short / Byte sums wrap to their width (SumFunction.java:56-107)
  int64_t wrap_sum(int64_t s) const {
    return cfg.value_type == OR_VAL_I32 ? (int64_t)(int32_t)s : cfg.value_type == OR_VAL_I16 ? (int64_t)(int16_t)s
         : cfg.value_type == OR_VAL_I8 ? (int64_t)(int8_t)s : s;
  }
  int by_cmp(int64_t x, int64_t y) const {
    if (is_float()) return java_double_compare(bitsd(x), bitsd(y));
    return x < y ? -1 : x > y ? 1 : 0;
  }
  void acc_add(Acc& a, int64_t v) const {
    if (a.cnt == 0) a.first = ordinal;
    // minBy/maxBy (Comparator.MinByComparator / MaxByComparator, first = true): a strictly smaller (larger)
    // field replaces the kept element; an equal one leaves the earlier element
    if (a.cnt == 0 || (cfg.aggregate == OR_AGG_MINBY && by_cmp(v, a.by_val) < 0) ||
        (cfg.aggregate == OR_AGG_MAXBY && by_cmp(v, a.by_val) > 0)) {
      a.by_val = v;
      a.by_ord = ordinal;
    }
    if (cfg.aggregate == OR_AGG_HLL) {
      if (a.regs.empty()) a.regs.assign((size_t)1 << cfg.hll_p, 0);
      hll_add(a.regs, cfg.hll_p, (uint64_t)v);
      a.cnt += 1;
      return;
    }
    if (cfg.aggregate == OR_AGG_ROW) {  // v: the record's index in the batch of oracle_process_rows
      row_add(a, v);
      a.cnt += 1;
      return;
    }
    if (cfg.aggregate == OR_AGG_TDIGEST) a.td_buf.push_back(v);  // compressed at the end of the batch
    if (is_float()) {
      double d = bitsd(v);
      if (a.cnt == 0) {
        a.dmn = a.dmx = d;
      } else {
        if (java_double_compare(d, a.dmn) < 0) a.dmn = d;
        if (java_double_compare(d, a.dmx) > 0) a.dmx = d;
      }
      // FloatSum adds in float (SumFunction.java:92-99): every partial sum rounds to float
      a.dsum = cfg.value_type == OR_VAL_F32 ? (double)((float)a.dsum + (float)d) : a.dsum + d;
    } else {
      if (a.cnt == 0) {
        a.imn = a.imx = v;
      } else {
        a.imn = std::min(a.imn, v);
        a.imx = std::max(a.imx, v);
      }
      a.isum = jadd(a.isum, v);
    }
    a.cnt += 1;
  }
  // ------------------------------------------------ OR_AGG_ROW (Table group-window aggregates, window_oracle.h)
  const int64_t* row_cols = nullptr;  // the batch being processed: column j of record i at row_cols[j * row_n + i]
  const uint8_t* row_nulls = nullptr;
  int64_t row_n = 0;
  std::vector<std::vector<int64_t>> row_res;  // per emitted row: its aggregates, then the null mask
  bool row_float(int j) const { return cfg.row_type[j] == OR_VAL_F64 || cfg.row_type[j] == OR_VAL_F32; }
  // accumulate(acc, value) of every aggregate over each non-null column (the Table functions skip nulls)
  void row_add(Acc& a, int64_t i) const {
    if (a.row.empty()) a.row.resize((size_t)cfg.row_nc);
    const uint8_t nm = row_nulls ? row_nulls[i] : 0;
    for (int j = 0; j < cfg.row_nc; j++) {
      if ((nm >> j) & 1) continue;
      const int64_t x = row_cols[(int64_t)j * row_n + i];
      Acc::RowCol& c = a.row[(size_t)j];
      if (row_float(j)) {
        const double d = bitsd(x);
        if (c.nn == 0 || java_double_compare(d, c.dmn) < 0) c.dmn = d;  // MinAggFunction.accumulate
        if (c.nn == 0 || java_double_compare(d, c.dmx) > 0) c.dmx = d;  // MaxAggFunction.accumulate
        c.dsum = d + c.dsum;                                             // numeric.plus(v, acc) / acc.f0 += v
        c.fsum = (double)((float)d + (float)c.fsum);                     // Float plus
      } else {
        if (c.nn == 0 || x < c.imn) c.imn = x;
        if (c.nn == 0 || x > c.imx) c.imx = x;
        c.isum += (__int128)x;
      }
      c.nn++;
    }
  }
  // merge(acc, its) of every aggregate (SumAggFunction.merge: plus of the flagged sums; Min/Max: accumulate(a.f0))
  void row_merge(Acc& r, const Acc& b) const {
    if (b.row.empty()) return;
    if (r.row.empty()) r.row.resize((size_t)cfg.row_nc);
    for (int j = 0; j < cfg.row_nc; j++) {
      Acc::RowCol& c = r.row[(size_t)j];
      const Acc::RowCol& o = b.row[(size_t)j];
      if (o.nn == 0) continue;
      if (c.nn == 0) {
        c = o;
        continue;
      }
      if (row_float(j)) {
        if (java_double_compare(o.dmn, c.dmn) < 0) c.dmn = o.dmn;
        if (java_double_compare(o.dmx, c.dmx) > 0) c.dmx = o.dmx;
        c.dsum = c.dsum + o.dsum;
        c.fsum = (double)((float)c.fsum + (float)o.fsum);
      } else {
        c.imn = std::min(c.imn, o.imn);
        c.imx = std::max(c.imx, o.imx);
        c.isum += o.isum;
      }
      c.nn += o.nn;
    }
  }
  // getValue of aggregate s (OR_ROW_* << 8 | column): the value (integers sign-extended from the type's width,
  // floating results as f64 bits) or NULL
  int64_t row_value(const Acc& a, int s, bool* null) const {
    const int fn = cfg.row_spec[s] >> 8, j = cfg.row_spec[s] & 0xff;
    *null = false;
    if (fn == OR_ROW_COUNT_STAR) return a.cnt;
    const Acc::RowCol c = a.row.empty() ? Acc::RowCol{} : a.row[(size_t)j];
    if (fn == OR_ROW_COUNT) return c.nn;
    if (c.nn == 0) {
      *null = true;
      return 0;
    }
    const int t = cfg.row_type[j];
    auto narrow = [t](int64_t v) -> int64_t {
      return t == OR_VAL_I32 ? (int64_t)(int32_t)v : t == OR_VAL_I16 ? (int64_t)(int16_t)v
           : t == OR_VAL_I8 ? (int64_t)(int8_t)v : v;
    };
    auto fbits = [](double d) {  // (the double of a Float result)
      int64_t b;
      memcpy(&b, &d, 8);
      return b;
    };
    switch (fn) {
      case OR_ROW_SUM:
        if (t == OR_VAL_F64) return fbits(c.dsum);
        if (t == OR_VAL_F32) return fbits(c.fsum);
        return narrow((int64_t)(uint64_t)(unsigned __int128)c.isum);
      case OR_ROW_MIN:
        return row_float(j) ? fbits(c.dmn) : c.imn;
      case OR_ROW_MAX:
        return row_float(j) ? fbits(c.dmx) : c.imx;
      default: {  // OR_ROW_AVG
        if (t == OR_VAL_F64) return fbits(c.dsum / (double)c.nn);
        if (t == OR_VAL_F32) return fbits((double)(float)(c.dsum / (double)c.nn));
        if (t == OR_VAL_I64) return (int64_t)(c.isum / (__int128)c.nn);  // BigInteger.divide: truncating
        const int64_t lsum = (int64_t)(uint64_t)(unsigned __int128)c.isum;  // the Long accumulator (wraps)
        return narrow(lsum / c.nn);                                         // Java long division, then toInt ...
      }
    }
  }

  // AggregateFunction.merge(a, b)
  Acc acc_merge(const Acc& a, const Acc& b) const {
    if (a.cnt == 0) return b;
    if (b.cnt == 0) return a;
    Acc r = a;
    r.cnt = a.cnt + b.cnt;
    // OR_AGG_FIRST: mergeState(a, b) = reduce(a, b) keeps a's first element (HeapReducingState.java:91-93),
    // and which state window is `a` follows HashSet order in the reference (AbstractHeapMergingState.java
    // :67-93, MergingWindowSet.java:190-205): parity unpinned, defined here as the earlier element
    r.first = std::min(a.first, b.first);  // (OR_AGG_FIRST and OR_AGG_FIRST_MAX)
    // minBy/maxBy merge: the reference keeps reduce(a, b)'s first argument on a tie, `a` chosen by HashSet
    // order (parity unpinned); defined here as the earlier element, like the accumulation order
    const int cmp = by_cmp(b.by_val, a.by_val);
    const bool b_wins = cfg.aggregate == OR_AGG_MINBY   ? (cmp < 0 || (cmp == 0 && b.by_ord < a.by_ord))
                        : cfg.aggregate == OR_AGG_MAXBY ? (cmp > 0 || (cmp == 0 && b.by_ord < a.by_ord))
                                                        : false;
    if (b_wins) {
      r.by_val = b.by_val;
      r.by_ord = b.by_ord;
    }
    if (cfg.aggregate == OR_AGG_HLL) {
      for (size_t j = 0; j < r.regs.size(); j++) r.regs[j] = std::max(r.regs[j], b.regs[j]);
      return r;
    }
    if (cfg.aggregate == OR_AGG_TDIGEST) td_union(r, b);
    if (cfg.aggregate == OR_AGG_ROW) {
      row_merge(r, b);
      return r;
    }
    if (is_float()) {
      r.dsum = cfg.value_type == OR_VAL_F32 ? (double)((float)a.dsum + (float)b.dsum) : a.dsum + b.dsum;
      r.dmn = java_double_compare(b.dmn, a.dmn) < 0 ? b.dmn : a.dmn;
      r.dmx = java_double_compare(b.dmx, a.dmx) > 0 ? b.dmx : a.dmx;
    } else {
      r.isum = jadd(a.isum, b.isum);
      r.imn = std::min(a.imn, b.imn);
      r.imx = std::max(a.imx, b.imx);
    }
    return r;
  }

  // ------------------------------------------------ timers (HeapInternalTimerService.java:224-248)
  void register_timer(int64_t ts, int64_t key, const TW& w) {
    Timer t{ts, key, w};
    if (timer_set.insert(t).second) timer_q.push(t);
  }
  void delete_timer(int64_t ts, int64_t key, const TW& w) { timer_set.erase(Timer{ts, key, w}); }

  // ------------------------------------------------ WindowOperator.java:576-651
  int64_t cleanup_time(const TW& w) const {
    int64_t c = jadd(w.maxTs(), cfg.lateness);
    return c >= w.maxTs() ? c : LMAX;
  }
  bool is_window_late(const TW& w) const { return cleanup_time(w) <= wm; }
  bool is_element_late(int64_t ts) const { return jadd(ts, cfg.lateness) <= wm; }
  void register_cleanup_timer(int64_t key, const TW& w) {
    int64_t c = cleanup_time(w);
    if (c == LMAX) return;
    register_timer(c, key, w);
  }
  void delete_cleanup_timer(int64_t key, const TW& w) {
    int64_t c = cleanup_time(w);
    if (c == LMAX) return;
    delete_timer(c, key, w);
  }

  void emit(int64_t key, const TW& w, const Acc& a_in) {
    Acc a = a_in;
    oracle_row r;
    r.key = key;
    r.start = w.start;
    r.end = w.end;
    r.count = a.cnt;
    row_digest.emplace_back();
    if (cfg.aggregate == OR_AGG_ROW) {
      std::vector<int64_t> res((size_t)cfg.row_ns + 1, 0);
      for (int q = 0; q < cfg.row_ns; q++) {
        bool nl;
        res[(size_t)q] = row_value(a, q, &nl);
        if (nl) res[(size_t)cfg.row_ns] |= (int64_t)1 << q;
      }
      row_res.push_back(res);
      r.sum = r.min = r.max = 0;
      r.epoch = epoch;
      rows.push_back(r);
      return;
    }
    if (cfg.aggregate == OR_AGG_TDIGEST) {
      if (!a_in.td_buf.empty() || a_in.td_merged) td_compress(a, td_q);  // getResult within a batch sees every value
      const double q[3] = {td_quantile(a, a.dmn, a.dmx, cfg.td_q[0]), td_quantile(a, a.dmn, a.dmx, cfg.td_q[1]),
                           td_quantile(a, a.dmn, a.dmx, cfg.td_q[2])};
      memcpy(&r.sum, &q[0], 8);
      memcpy(&r.min, &q[1], 8);
      memcpy(&r.max, &q[2], 8);
      for (size_t i = 0; i < a.td_sum.size(); i++) row_digest.back().emplace_back(a.td_sum[i], a.td_w[i]);
      r.epoch = epoch;
      rows.push_back(r);
      return;
    }
    if (cfg.aggregate == OR_AGG_HLL) {
      double est;
      hll_result(a.regs, cfg.hll_p, &est, &r.min, &r.max);
      memcpy(&r.sum, &est, 8);
    } else if (is_float()) {
      r.sum = dbits(a.dsum);
      r.min = dbits(a.dmn);
      r.max = dbits(a.dmx);
      // keep raw (non-canonical) sum bits: sums are compared with tolerance
      memcpy(&r.sum, &a.dsum, 8);
    } else {
      r.sum = wrap_sum(a.isum);
      r.min = a.imn;
      r.max = a.imx;
    }
    if (cfg.aggregate == OR_AGG_FIRST) r.max = a.first;
    if (cfg.aggregate == OR_AGG_FIRST_MAX) {  // max(pos): the first element with the field's maximum
      r.min = is_float() ? dbits(a.dmx) : a.imx;
      r.max = a.first;
    }
    if (cfg.aggregate == OR_AGG_MINBY || cfg.aggregate == OR_AGG_MAXBY) {
      r.min = a.by_val;
      r.max = a.by_ord;
    }
    r.epoch = epoch;
    rows.push_back(r);
  }

  // ------------------------------------------------ assigners
  void assign(int64_t ts, std::vector<TW>& out) const {
    out.clear();
    if (cfg.assigner == OR_SESSION) {  // EventTimeSessionWindows.java:59-61
      out.push_back(TW{ts, jadd(ts, cfg.gap)});
      return;
    }
    if (ts == LMIN) throw OpError{OR_ERR_NO_TIMESTAMP};
    if (cfg.assigner == OR_TUMBLING) {  // TumblingEventTimeWindows.java:63-73
      int64_t s = window_start(ts, cfg.offset, cfg.size);
      out.push_back(TW{s, jadd(s, cfg.size)});
      return;
    }
    // SlidingEventTimeWindows.java:67-81
    int64_t last = window_start(ts, cfg.offset, cfg.slide);
    for (int64_t s = last; s > jsub(ts, cfg.size); s = jsub(s, cfg.slide)) out.push_back(TW{s, jadd(s, cfg.size)});
  }

  // ------------------------------------------------ MergingWindowSet.java:150-225 (+ TimeWindow.mergeWindows)
  // Returns the window the new window ended up in; calls the merge function of
  // WindowOperator.java:305-339 inline.
  TW add_window(int64_t key, std::map<TW, TW>& mapping, const TW& nw) {
    std::vector<TW> ws;
    ws.reserve(mapping.size() + 1);
    for (auto& kv : mapping) ws.push_back(kv.first);
    ws.push_back(nw);
    std::stable_sort(ws.begin(), ws.end(), [](const TW& a, const TW& b) { return a.start < b.start; });
    // sweep (TimeWindow.java:201-244)
    std::vector<std::pair<TW, std::set<TW>>> merged;
    bool have = false;
    std::pair<TW, std::set<TW>> cur;
    for (const TW& c : ws) {
      if (!have) {
        cur.first = c;
        cur.second.clear();
        cur.second.insert(c);
        have = true;
      } else if (cur.first.intersects(c)) {
        cur.first = cur.first.cover(c);
        cur.second.insert(c);
      } else {
        merged.push_back(cur);
        cur.first = c;
        cur.second.clear();
        cur.second.insert(c);
      }
    }
    if (have) merged.push_back(cur);
    std::vector<std::pair<TW, std::set<TW>>> results;
    for (auto& m : merged)
      if (m.second.size() > 1) results.push_back(m);

    TW result = nw;
    bool merged_new = false;
    for (auto& r : results) {
      const TW merge_result = r.first;
      std::set<TW> mws = r.second;
      if (mws.erase(nw)) {
        merged_new = true;
        result = merge_result;
      }
      // "pick any of the merged windows": deterministic first here (the reference uses
      // HashSet iteration order; the choice only decides where state lives).
      TW merged_state_window = mapping.at(*mws.begin());
      std::vector<TW> merged_state_windows;
      for (const TW& m : mws) {
        auto it = mapping.find(m);
        if (it != mapping.end()) {
          merged_state_windows.push_back(it->second);
          mapping.erase(it);
        }
      }
      mapping[merge_result] = merged_state_window;
      merged_state_windows.erase(
          std::remove(merged_state_windows.begin(), merged_state_windows.end(), merged_state_window),
          merged_state_windows.end());
      if (!(mws.count(merge_result) && mws.size() == 1)) {
        merge_function(key, merge_result, mws, mapping[merge_result], merged_state_windows);
      }
    }
    if (results.empty() || (result == nw && !merged_new)) mapping[result] = result;
    return result;
  }

  // WindowOperator.java:308-339
  void merge_function(int64_t key, const TW& merge_result, const std::set<TW>& merged_windows,
                      const TW& state_window_result, const std::vector<TW>& merged_state_windows) {
    if (jadd(merge_result.maxTs(), cfg.lateness) <= wm) throw OpError{OR_ERR_MERGE_LATE};
    // EventTimeTrigger.onMerge (EventTimeTrigger.java:70-73): unconditional registration
    register_timer(merge_result.maxTs(), key, merge_result);
    for (const TW& m : merged_windows) {
      delete_timer(m.maxTs(), key, m);  // triggerContext.clear() -> EventTimeTrigger.clear
      delete_cleanup_timer(key, m);
    }
    // AbstractHeapMergingState.mergeNamespaces (:67-93)
    if (merged_state_windows.empty()) return;
    bool have = false;
    Acc acc;
    for (const TW& s : merged_state_windows) {
      auto it = state.find(KW{key, s});
      if (it == state.end()) continue;
      Acc src = it->second;
      state.erase(it);
      acc = have ? acc_merge(acc, src) : src;
      have = true;
    }
    if (have) {
      auto it = state.find(KW{key, state_window_result});
      if (it != state.end())
        it->second = acc_merge(it->second, acc);
      else
        state[KW{key, state_window_result}] = acc;
      // (a merged t-digest is compressed at the end of the batch, whatever its buffer)
      if (cfg.aggregate == OR_AGG_TDIGEST) td_touched.push_back(KW{key, state_window_result});
    }
  }

  // ------------------------------------------------ WindowOperator.processElement (:291-421)
  std::vector<TW> wbuf;
  int64_t ordinal = -1;  // arrival ordinal of the element being processed
  void process_element(int64_t key, int64_t ts, int64_t val) {
    ordinal++;
    assign(ts, wbuf);
    bool skipped = true;
    if (is_merging()) {
      std::map<TW, TW>& mapping = merging[key];
      for (const TW& w : wbuf) {
        TW actual = add_window(key, mapping, w);
        if (is_window_late(actual)) {
          // MergingWindowSet.retireWindow
          if (!mapping.erase(actual)) throw OpError{OR_ERR_ILLEGAL_STATE};
          continue;
        }
        skipped = false;
        auto it = mapping.find(actual);
        if (it == mapping.end()) throw OpError{OR_ERR_ILLEGAL_STATE};
        TW sw = it->second;
        Acc& a = state[KW{key, sw}];
        acc_add(a, val);
        if (cfg.aggregate == OR_AGG_TDIGEST && a.td_buf.size() == 1) td_touched.push_back(KW{key, sw});
        // EventTimeTrigger.onElement
        if (actual.maxTs() <= wm) {
          emit(key, actual, a);
          if (cfg.purging) state.erase(KW{key, sw});
        } else {
          register_timer(actual.maxTs(), key, actual);
        }
        register_cleanup_timer(key, actual);
      }
      if (mapping.empty()) merging.erase(key);
    } else {
      for (const TW& w : wbuf) {
        if (is_window_late(w)) continue;
        skipped = false;
        KW kw{key, w};
        Acc& a = state[kw];
        acc_add(a, val);
        if (cfg.aggregate == OR_AGG_TDIGEST && a.td_buf.size() == 1) td_touched.push_back(kw);
        if (w.maxTs() <= wm) {
          emit(key, w, a);
          if (cfg.purging) state.erase(kw);
        } else {
          register_timer(w.maxTs(), key, w);
        }
        register_cleanup_timer(key, w);
      }
    }
    if (skipped && is_element_late(ts)) {
      if (cfg.side_output)
        side.push_back(oracle_side_row{key, ts, val, epoch});
      else
        late_dropped++;
    }
  }

  // ------------------------------------------------ WindowOperator.onEventTime (:424-469)
  void on_event_time(const Timer& t) {
    const int64_t key = t.key;
    const TW& w = t.w;
    TW sw = w;
    std::map<TW, TW>* mapping = nullptr;
    if (is_merging()) {
      auto mit = merging.find(key);
      if (mit == merging.end()) return;
      auto it = mit->second.find(w);
      if (it == mit->second.end()) return;
      sw = it->second;
      mapping = &mit->second;
    }
    KW kw{key, sw};
    auto it = state.find(kw);
    if (it != state.end()) {
      if (t.ts == w.maxTs()) {  // EventTimeTrigger.onEventTime
        emit(key, w, it->second);
        if (cfg.purging) state.erase(kw);
      }
    }
    if (t.ts == cleanup_time(w)) {  // isCleanupTime -> clearAllState (:526-538)
      state.erase(kw);
      delete_timer(w.maxTs(), key, w);
      if (mapping) {
        if (!mapping->erase(w)) throw OpError{OR_ERR_ILLEGAL_STATE};
        if (mapping->empty()) merging.erase(key);
      }
    }
  }

  // ------------------------------------------------ AbstractStreamOperator.processWatermark (:735-740)
  void process_watermark(int64_t w) {
    wm = w;  // HeapInternalTimerService.advanceWatermark (:276-290)
    while (!timer_q.empty() && timer_q.top().ts <= w) {
      Timer t = timer_q.top();
      timer_q.pop();
      auto it = timer_set.find(t);
      if (it == timer_set.end()) continue;  // lazily deleted
      timer_set.erase(it);
      on_event_time(t);
    }
    epoch++;
  }
};

}  // namespace

// =========================================================================== C API
// ---------------------------------------------------------------- a14: count windows (C1 CPU reference)
// KeyedStream.countWindow(size, slide) = window(GlobalWindows.create()).evictor(CountEvictor.of(size))
//   .trigger(CountTrigger.of(slide)) (KeyedStream.java:383-397).
// EvictingWindowOperator.processElement (EvictingWindowOperator.java:102-239): the element is appended to
// the window's ListState; CountTrigger.onElement (CountTrigger.java:47-55) adds 1 to its count and FIREs
// (clearing the count) when it reaches `slide`.  emitWindowContents (:334-366): evictBefore, the window
// function over the remaining elements, evictAfter; the evictor removes from the front
// (CountEvictor.evict, CountEvictor.java:63-78: keep the last maxCount).  GlobalWindow never fires by time.
struct CountWindowOracle {
  CountWindowOracle(int64_t sz, int64_t sl, bool after, int32_t vt)
      : size(sz), slide(sl), evict_after(after), value_type(vt) {}
  int64_t size, slide;
  bool evict_after;
  int32_t value_type;
  int64_t ordinal = -1;
  struct Elem {
    int64_t val, ord;
  };
  struct KeyState {
    std::deque<Elem> list;
    int64_t count = 0;  // CountTrigger's ReducingState
  };
  std::unordered_map<int64_t, KeyState> state;
  std::vector<oracle_row> rows;

  void evict(std::deque<Elem>& l) const {
    while ((int64_t)l.size() > size) l.pop_front();
  }
  void process(int64_t key, int64_t val) {
    ordinal++;
    KeyState& s = state[key];
    s.list.push_back(Elem{val, ordinal});
    if (++s.count < slide) return;
    s.count = 0;
    if (!evict_after) evict(s.list);
    // ReduceApplyWindowFunction over the iterable, SumAggregator.reduce: first element kept, field summed
    oracle_row r{};
    r.key = key;
    r.start = LMIN;
    r.end = LMAX;
    r.count = (int64_t)s.list.size();
    r.min = LMAX;
    const bool fl = value_type == OR_VAL_F64 || value_type == OR_VAL_F32;
    double ds = 0.0, dm = 0.0;
    bool first = true;
    for (const Elem& e : s.list) {  // ReduceFunction applied in order: SumAggregator / SumFunction
      if (fl) {
        const double d = bitsd(e.val);
        ds = first ? d : value_type == OR_VAL_F32 ? (double)((float)ds + (float)d) : ds + d;
        if (first || java_double_compare(d, dm) < 0) dm = d;
      } else {
        r.sum = jadd(r.sum, e.val);
        r.min = std::min(r.min, e.val);
      }
      first = false;
    }
    if (fl) {
      memcpy(&r.sum, &ds, 8);
      r.min = dbits(dm);
    } else {
      r.sum = value_type == OR_VAL_I32 ? (int64_t)(int32_t)r.sum : value_type == OR_VAL_I16 ? (int64_t)(int16_t)r.sum
            : value_type == OR_VAL_I8 ? (int64_t)(int8_t)r.sum : r.sum;
    }
    r.max = s.list.front().ord;
    rows.push_back(r);
    if (evict_after) evict(s.list);
  }
};

extern "C" {

void* oracle_count_create(int64_t size, int64_t slide, int32_t evict_after, int32_t value_type) {
  if (size <= 0 || slide <= 0) return nullptr;
  return new CountWindowOracle(size, slide, evict_after != 0, value_type);
}
void oracle_count_destroy(void* op) { delete static_cast<CountWindowOracle*>(op); }
void oracle_count_process(void* op, const int64_t* key, const int64_t* val, int64_t n) {
  auto* o = static_cast<CountWindowOracle*>(op);
  for (int64_t i = 0; i < n; i++) o->process(key[i], val[i]);
}
int64_t oracle_count_num_rows(void* op) { return (int64_t)static_cast<CountWindowOracle*>(op)->rows.size(); }
void oracle_count_get_rows(void* op, oracle_row* out) {
  auto* o = static_cast<CountWindowOracle*>(op);
  std::copy(o->rows.begin(), o->rows.end(), out);
}

void* oracle_create(const oracle_cfg* cfg) { return new WindowOperatorOracle(*cfg); }
void oracle_destroy(void* op) { delete static_cast<WindowOperatorOracle*>(op); }

int oracle_process(void* p, const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n) {
  auto* op = static_cast<WindowOperatorOracle*>(p);
  try {
    for (int64_t i = 0; i < n; i++) op->process_element(key[i], ts[i], val[i]);
  } catch (const OpError& e) {
    op->end_batch();
    return e.code;
  }
  op->end_batch();
  return OR_OK;
}
int oracle_watermark(void* p, int64_t wm) {
  try {
    static_cast<WindowOperatorOracle*>(p)->process_watermark(wm);
  } catch (const OpError& e) {
    return e.code;
  }
  return OR_OK;
}
int64_t oracle_num_rows(void* p) { return (int64_t) static_cast<WindowOperatorOracle*>(p)->rows.size(); }
void oracle_get_rows(void* p, oracle_row* out) {
  auto* op = static_cast<WindowOperatorOracle*>(p);
  if (!op->rows.empty()) memcpy(out, op->rows.data(), op->rows.size() * sizeof(oracle_row));
}
void oracle_clear_rows(void* p) {
  static_cast<WindowOperatorOracle*>(p)->rows.clear();
  static_cast<WindowOperatorOracle*>(p)->row_digest.clear();
  static_cast<WindowOperatorOracle*>(p)->row_res.clear();
}
int oracle_process_rows(void* p, const int64_t* key, const int64_t* ts, const int64_t* cols, const uint8_t* nulls,
                        int64_t n) {
  auto* op = static_cast<WindowOperatorOracle*>(p);
  if (op->cfg.aggregate != OR_AGG_ROW) return OR_ERR_ILLEGAL_STATE;
  op->row_cols = cols;
  op->row_nulls = nulls;
  op->row_n = n;
  int rc = OR_OK;
  try {
    for (int64_t i = 0; i < n; i++) op->process_element(key[i], ts[i], i);
  } catch (const OpError& e) {
    rc = e.code;
  }
  op->row_cols = nullptr;
  op->row_nulls = nullptr;
  op->end_batch();
  return rc;
}
int32_t oracle_row_results(void* p, int64_t row, int64_t* vals, uint32_t* null_mask) {
  auto* op = static_cast<WindowOperatorOracle*>(p);
  if (row < 0 || row >= (int64_t)op->row_res.size()) return -1;
  const auto& r = op->row_res[(size_t)row];
  for (int q = 0; q < op->cfg.row_ns; q++) vals[q] = r[(size_t)q];
  *null_mask = (uint32_t)r[(size_t)op->cfg.row_ns];
  return op->cfg.row_ns;
}
int64_t oracle_row_digest(void* p, int64_t row, double* sum, int64_t* weight, int64_t cap) {
  auto* op = static_cast<WindowOperatorOracle*>(p);
  if (row < 0 || row >= (int64_t)op->row_digest.size()) return -1;
  const auto& d = op->row_digest[(size_t)row];
  for (int64_t i = 0; i < (int64_t)d.size() && i < cap; i++) {
    sum[i] = d[(size_t)i].first;
    weight[i] = d[(size_t)i].second;
  }
  return (int64_t)d.size();
}
int64_t oracle_num_side_rows(void* p) { return (int64_t) static_cast<WindowOperatorOracle*>(p)->side.size(); }
void oracle_get_side_rows(void* p, oracle_side_row* out) {
  auto* op = static_cast<WindowOperatorOracle*>(p);
  if (!op->side.empty()) memcpy(out, op->side.data(), op->side.size() * sizeof(oracle_side_row));
}
int64_t oracle_late_dropped(void* p) { return static_cast<WindowOperatorOracle*>(p)->late_dropped; }
int64_t oracle_num_state_entries(void* p) { return (int64_t) static_cast<WindowOperatorOracle*>(p)->state.size(); }
int64_t oracle_num_timers(void* p) { return (int64_t) static_cast<WindowOperatorOracle*>(p)->timer_set.size(); }
int64_t oracle_current_watermark(void* p) { return static_cast<WindowOperatorOracle*>(p)->wm; }

int32_t oracle_long_hash(int64_t v) { return long_hash(v); }
int32_t oracle_murmur_hash(int32_t code) { return murmur(code); }
int32_t oracle_key_group(int32_t h, int32_t max_par) { return murmur(h) % max_par; }
int32_t oracle_operator_index(int32_t max_par, int32_t par, int32_t kg) { return kg * par / max_par; }
void oracle_key_group_range(int32_t max_par, int32_t par, int32_t idx, int32_t* s, int32_t* e) {
  *s = (idx * max_par + par - 1) / par;
  *e = ((idx + 1) * max_par - 1) / par;
}
void oracle_key_groups_long(const int64_t* keys, int64_t n, int32_t max_par, int32_t* out) {
  for (int64_t i = 0; i < n; i++) out[i] = murmur(long_hash(keys[i])) % max_par;
}
int64_t oracle_window_start(int64_t ts, int64_t offset, int64_t size) { return window_start(ts, offset, size); }
int32_t oracle_string_hash(const char* s, int64_t len) {
  uint32_t h = 0;
  for (int64_t i = 0; i < len; i++) h = 31u * h + (uint32_t)(unsigned char)s[i];
  return (int32_t)h;
}

int64_t oracle_run_parallel(const oracle_cfg* cfg, const int64_t* key, const int64_t* ts, const int64_t* val,
                            int64_t n, int64_t batch, const int64_t* wms, int64_t n_wms, int32_t max_par,
                            int32_t threads, int64_t* late_dropped) {
  if (threads < 1) threads = 1;
  // Phase 1 (the upstream KeyGroupStreamPartitioner, KeyGroupStreamPartitioner.java:53-65):
  // chunk-parallel routing of record indices to subtasks, arrival order kept per subtask.
  const int64_t chunk = (n + threads - 1) / threads;
  std::vector<std::vector<std::vector<int64_t>>> routed(threads, std::vector<std::vector<int64_t>>(threads));
  auto router = [&](int c) {
    int64_t lo = c * chunk, hi = std::min(n, lo + chunk);
    for (int64_t i = lo; i < hi; i++) {
      int32_t kg = murmur(long_hash(key[i])) % max_par;
      routed[c][kg * threads / max_par].push_back(i);
    }
  };
  {
    std::vector<std::thread> th;
    for (int c = 1; c < threads; c++) th.emplace_back(router, c);
    router(0);
    for (auto& t : th) t.join();
  }
  // Phase 2: one WindowOperator per subtask; watermark after each `batch` input records.
  std::vector<int64_t> total_rows(threads, 0), total_late(threads, 0);
  auto worker = [&](int t) {
    WindowOperatorOracle op(*cfg);
    int64_t b = 0;  // next watermark index
    for (int c = 0; c < threads; c++) {
      for (int64_t i : routed[c][t]) {
        while (b < n_wms && i >= (b + 1) * batch) {
          op.end_batch();
          op.process_watermark(wms[b++]);
          total_rows[t] += (int64_t)op.rows.size();  // discarding sink
          op.rows.clear();
          op.row_digest.clear();
        }
        op.process_element(key[i], ts[i], val[i]);
      }
    }
    op.end_batch();
    for (; b < n_wms; b++) op.process_watermark(wms[b]);
    total_rows[t] += (int64_t)op.rows.size();
    total_late[t] = op.late_dropped;
  };
  std::vector<std::thread> ts_;
  for (int t = 1; t < threads; t++) ts_.emplace_back(worker, t);
  worker(0);
  for (auto& th : ts_) th.join();
  int64_t rows = 0, late = 0;
  for (int t = 0; t < threads; t++) {
    rows += total_rows[t];
    late += total_late[t];
  }
  if (late_dropped) *late_dropped = late;
  return rows;
}

}  // extern "C"
