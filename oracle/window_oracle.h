/*
 * window_oracle.h — CPU restatement of Flink's keyed event-time WindowOperator.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker ("oracle") for the
 * MI355X path in flink_amd/.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product path never links or
 * calls anything under oracle/.
 *
 * It restates, element by element and with Java arithmetic (two's-complement
 * wrap, truncating %), the semantics of (paths relative to /root/reference):
 *   flink-core/src/main/java/org/apache/flink/util/MathUtils.java:134-198         murmurHash, bitMix
 *   flink-runtime/.../state/KeyGroupRangeAssignment.java:47-135                    key groups / operator index
 *   flink-streaming-java/.../api/windowing/windows/TimeWindow.java:83-256         maxTimestamp, intersects, cover,
 *                                                                                  mergeWindows, getWindowStartWithOffset
 *   .../api/windowing/assigners/TumblingEventTimeWindows.java:63-73               tumbling assignment
 *   .../api/windowing/assigners/SlidingEventTimeWindows.java:67-81                sliding assignment
 *   .../api/windowing/assigners/EventTimeSessionWindows.java:59-61                session assignment
 *   .../api/windowing/triggers/EventTimeTrigger.java:37-73, PurgingTrigger.java    trigger results
 *   .../runtime/operators/windowing/WindowOperator.java:291-651                   processElement/onEventTime/lateness
 *   .../runtime/operators/windowing/MergingWindowSet.java:81-225                  addWindow / retireWindow
 *   .../api/operators/HeapInternalTimerService.java:224-290                       timer dedup + advanceWatermark
 *   flink-runtime/.../state/heap/AbstractHeapMergingState.java:67-93              mergeNamespaces
 *
 * Aggregation: the build's built-in AggregateFunction "CountSumMinMax" over a
 * value column (i64, i32 with 32-bit wrap of the sum, or f64 with
 * Double.compare ordering for min/max and canonical NaN), i.e. the accumulator
 * {count, sum, min, max} — see DESIGN.md §"Aggregates".
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_TUMBLING = 0, OR_SLIDING = 1, OR_SESSION = 2 };
/* Long / Integer / Double fields, and Short / Byte (sums wrap to the width: SumFunction.ShortSum / ByteSum)
 * and Float (sums added in float, SumFunction.FloatSum; values passed as f64 bits of the float) */
enum { OR_VAL_I64 = 0, OR_VAL_I32 = 1, OR_VAL_F64 = 2, OR_VAL_I16 = 3, OR_VAL_I8 = 4, OR_VAL_F32 = 5 };

/* error codes returned by oracle_process / oracle_watermark */
enum {
  OR_OK = 0,
  OR_ERR_NO_TIMESTAMP = -1,   /* Long.MIN_VALUE timestamp: TumblingEventTimeWindows.java:69-71 */
  OR_ERR_MERGE_LATE = -2,     /* UnsupportedOperationException, WindowOperator.java:313-317 */
  OR_ERR_ILLEGAL_STATE = -3,  /* IllegalStateException, MergingWindowSet.java:127 / WindowOperator.java:355 */
};

typedef struct {
  int32_t assigner;      /* OR_TUMBLING / OR_SLIDING / OR_SESSION */
  int32_t value_type;    /* OR_VAL_* */
  int64_t size;          /* tumbling/sliding window size */
  int64_t slide;         /* sliding slide */
  int64_t offset;        /* tumbling/sliding offset */
  int64_t gap;           /* session gap */
  int64_t lateness;      /* allowedLateness */
  int32_t purging;       /* PurgingTrigger.of(EventTimeTrigger) */
  int32_t side_output;   /* late records go to the side output instead of numLateRecordsDropped */
  int32_t aggregate;     /* OR_AGG_* */
  int32_t hll_p;         /* HyperLogLog precision p (registers m = 2^p), OR_AGG_HLL only */
  int32_t td_delta;      /* t-digest compression delta (even), OR_AGG_TDIGEST only */
  int32_t td_pad;
  double td_q[3];        /* t-digest quantiles reported in a row's sum / min / max */
  int32_t row_nc;        /* OR_AGG_ROW: value columns per record (1 .. 8) */
  int32_t row_ns;        /* OR_AGG_ROW: output aggregates (1 .. 16) */
  int32_t row_type[8];   /* OR_AGG_ROW: OR_VAL_* of each column */
  int32_t row_spec[16];  /* OR_AGG_ROW: OR_ROW_* << 8 | column */
} oracle_cfg;

/* The user AggregateFunctions of SURVEY.md §8d C5.  OR_AGG_HLL is a HyperLogLog distinct count
 * (Flajolet, Fusy, Gandouet, Meunier 2007) over the value column read as a u64 item:
 *   h = fmix64(item) (MurmurHash3's 64-bit finaliser); register j = h >> (64 - p);
 *   rank = clz64((h << p) | (1 << (p - 1))) + 1  (1 .. 65 - p);  M[j] = max(M[j], rank);
 *   S = sum_j 2^(65 - p - M[j]) (exact, 128-bit); V = #{j : M[j] == 0};
 *   raw = (alpha_m * m * m) * 2^(65 - p) / S, S converted as hi * 2^64 + lo (two doubles);
 *   E = raw <= 2.5 m && V > 0 ? m * log(m / V) : raw  (small-range correction; no large-range
 *   correction with a 64-bit hash).
 * Row: count = elements, sum = E (f64 bits), min = V, max = low 64 bits of S (an exact register
 * checksum).  AggregateFunction.merge = register-wise max. */
/* OR_AGG_FIRST: count/sum/min with max = arrival ordinal of the window's first element (the passthrough
 * fields of sum(pos)/min(pos)); ordinals count every element processed, from 0. */
/* OR_AGG_MINBY / OR_AGG_MAXBY: minBy(pos) / maxBy(pos) with first = true (ComparableAggregator.java:72-94):
 * min = the selected field value, max = the arrival ordinal of the selected element. */
/* OR_AGG_TDIGEST: a merging t-digest (Dunning & Ertl, "Computing extremely accurate quantiles using
 * t-digests", 2019) of an f64 value column, compression delta, scale function k1(q) = delta/(2 pi)
 * asin(2q - 1), in its bucketed form — defined by this build (Flink 1.5 ships no t-digest; SURVEY §8d C5
 * names it as a user AggregateFunction):
 *   qb[b] = sin(pi b / delta)^2 for b = 0 .. nb = delta/2 (qb[0] = 0, qb[nb] = 1): the k1 values -delta/4 + b.
 *   add(v) buffers v; at the end of every processElements batch (a micro-batch / push) each digest with
 *   buffered values is compressed: the values, sorted by Double.compare order, and the centroids (sum, w)
 *   in their order are merged into one sequence (a value goes before a centroid whose mean sum/w is
 *   equal or larger in Double.compare order), W = total weight, and each item, with c = the weight
 *   before it, falls into the bucket of its midpoint: the largest b < nb with W*qb[b] <= c + w/2.
 *   Consecutive items of one bucket form one centroid: weight = sum of weights; sum = S_old + S_new, where
 *   S_old = its old centroids' sums added left to right and S_new = its new values in blocks of 64 (from
 *   its first new value on), each block summed as the perfect binary tree over its 64 slots in order (an
 *   empty slot contributes nothing), the block sums added left to right (only S_old or only S_new when
 *   the group has only old or only new items).  At most delta/2 centroids.
 *   getResult: count = W; sum / min / max = quantile(td_q[0..2]) as f64 bits, where quantile(q) is the
 *   piecewise-linear interpolation at x = q*W through (0, min), (cum_{i-1} + w_i/2, mean_i) ..., (W, max).
 * The arithmetic is IEEE-754 double without fused multiply-add, so the GPU's digests are bit-exact. */
/* OR_AGG_ROW: the Table API's group-window aggregation (flink-libraries/flink-table, DataStreamGroupWindowAggregate
 * .scala:197-294): ONE accumulator Row per (key, window) holding several built-in aggregates over nullable value
 * columns (the generated AggregateFunction of AggregateUtil.createDataStreamAggregateFunction); each record carries
 * row_nc columns and a null mask.  The aggregates (.../table/functions/aggfunctions/):
 *   OR_ROW_COUNT_STAR  COUNT(*) / COUNT(1): every record (CountAggFunction.accumulate(acc), :41-43)
 *   OR_ROW_COUNT       COUNT(col): the non-null values (CountAggFunction.scala:51-55); never null
 *   OR_ROW_SUM         SUM(col): null when the column had no non-null value; Long / Int / Short / Byte sums wrap to
 *                      their width, Float adds in float, Double in double (SumAggFunction.scala:28-100, Scala Numeric)
 *   OR_ROW_MIN/MAX     MIN / MAX(col): null when empty; Double / Float by Ordering.Double / Float (java.lang compare)
 *                      (MinAggFunction.scala, MaxAggFunction.scala:28-100)
 *   OR_ROW_AVG         AVG(col): null when empty; Long: the exact (BigInteger) sum / count truncated (BigIntegral-
 *                      AvgAggFunction, AvgAggFunction.scala:130-185); Int / Short / Byte: the Long sum / count (Java
 *                      long division) narrowed to the type (IntegralAvgAggFunction, :39-120); Double / Float: the
 *                      double sum of the values / count (FloatingAvgAggFunction, :187-250; Float narrowed)
 * merge (sessions, AbstractHeapMergingState.mergeNamespaces) = each function's merge.  A row's count is COUNT(*);
 * its results come from oracle_row_results: one int64 per aggregate (integers sign-extended, floating results as
 * f64 bits, a Float result as the double of the float) and a null mask (bit s = aggregate s is NULL). */
enum { OR_ROW_COUNT_STAR = 0, OR_ROW_COUNT = 1, OR_ROW_SUM = 2, OR_ROW_MIN = 3, OR_ROW_MAX = 4, OR_ROW_AVG = 5 };
enum { OR_AGG_COUNT_SUM_MIN_MAX = 0, OR_AGG_HLL = 1, OR_AGG_FIRST = 2, OR_AGG_MINBY = 3, OR_AGG_MAXBY = 4,
       OR_AGG_FIRST_MAX = 5 /* max(pos): as OR_AGG_FIRST with min = the field's maximum */,
       OR_AGG_TDIGEST = 6, OR_AGG_ROW = 7 };

/* One fired row.  sum/min/max hold i64 values (I64/I32) or f64 bit patterns (F64).
 * epoch = number of watermarks fully processed before the row was emitted, so
 * every row preceding the k-th output watermark has epoch k (TestHarnessUtil
 * compares watermark positions exactly and records sorted in between). */
typedef struct {
  int64_t key, start, end, count, sum, min, max, epoch;
} oracle_row;

typedef struct {
  int64_t key, ts, val, epoch;
} oracle_side_row;

void*   oracle_create(const oracle_cfg* cfg);
void    oracle_destroy(void* op);
/* process n elements in order; val holds i64 values or f64 bits */
int     oracle_process(void* op, const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n);
int     oracle_watermark(void* op, int64_t wm);
/* OR_AGG_ROW: n records with row_nc value columns (cols + j * n: column j; i64 values or f64 bits) and a null mask
 * per record (bit j = column j is NULL; nulls may be NULL = none) */
int     oracle_process_rows(void* op, const int64_t* key, const int64_t* ts, const int64_t* cols, const uint8_t* nulls,
                            int64_t n);
/* OR_AGG_ROW: the aggregates of emitted row `row` (row_ns values) and their null mask; returns row_ns, -1 = no row */
int32_t oracle_row_results(void* op, int64_t row, int64_t* vals, uint32_t* null_mask);
int64_t oracle_num_rows(void* op);
/* a14 — count windows (SURVEY §8a, config C1 CPU reference): GlobalWindows + CountTrigger.of(slide) +
 * CountEvictor.of(size, evict_after) over a ListState of elements, the window function reducing the
 * remaining elements in order with sum (KeyedStream.countWindow(size, slide).sum(pos),
 * KeyedStream.java:383-397; EvictingWindowOperator.java:102-239,334-366).  Rows: start = Long.MIN_VALUE,
 * end = Long.MAX_VALUE (GlobalWindow; row timestamp Long.MAX_VALUE), count = elements reduced,
 * sum (wrapped to value_type width), min, max = arrival ordinal of the first reduced element (the
 * passthrough fields of sum(pos), as OR_AGG_FIRST). */
void*   oracle_count_create(int64_t size, int64_t slide, int32_t evict_after, int32_t value_type);
void    oracle_count_destroy(void* op);
void    oracle_count_process(void* op, const int64_t* key, const int64_t* val, int64_t n);
int64_t oracle_count_num_rows(void* op);
void    oracle_count_get_rows(void* op, oracle_row* out);
void    oracle_get_rows(void* op, oracle_row* out);       /* copies all rows emitted so far */
/* OR_AGG_TDIGEST: centroids (sum, weight) of row `row` (index into the rows emitted so far); returns
 * their number (copies at most cap) */
int64_t oracle_row_digest(void* op, int64_t row, double* sum, int64_t* weight, int64_t cap);
void    oracle_clear_rows(void* op);
int64_t oracle_num_side_rows(void* op);
void    oracle_get_side_rows(void* op, oracle_side_row* out);
int64_t oracle_late_dropped(void* op);
int64_t oracle_num_state_entries(void* op);  /* ≙ numKeyedStateEntries (window-contents) */
int64_t oracle_num_timers(void* op);         /* ≙ numEventTimeTimers */
int64_t oracle_current_watermark(void* op);

/* Java hashing / key-group restatement (MathUtils.java:134-198, KeyGroupRangeAssignment.java:47-135) */
int32_t oracle_long_hash(int64_t v);              /* Long.hashCode */
int32_t oracle_murmur_hash(int32_t code);         /* MathUtils.murmurHash */
int32_t oracle_key_group(int32_t key_hash, int32_t max_parallelism);
int32_t oracle_operator_index(int32_t max_par, int32_t par, int32_t key_group);
void    oracle_key_group_range(int32_t max_par, int32_t par, int32_t op_index, int32_t* start, int32_t* end);
void    oracle_key_groups_long(const int64_t* keys, int64_t n, int32_t max_par, int32_t* out);
int64_t oracle_window_start(int64_t ts, int64_t offset, int64_t size);
int32_t oracle_string_hash(const char* s, int64_t len);  /* String.hashCode over UTF-16 units (ASCII input) */

/* Multi-threaded CPU baseline: p subtasks, each a WindowOperator over its KeyGroupRange
 * (computeKeyGroupRangeForOperatorIndex), fed the records routed to it (murmur key groups),
 * with a watermark after every `batch` records (wms[b]) and a final watermark if given.
 * Returns total fired rows; *late_dropped gets the sum over subtasks. */
int64_t oracle_run_parallel(const oracle_cfg* cfg, const int64_t* key, const int64_t* ts,
                            const int64_t* val, int64_t n, int64_t batch, const int64_t* wms,
                            int64_t n_wms, int32_t max_par, int32_t threads, int64_t* late_dropped);

#ifdef __cplusplus
}
#endif
