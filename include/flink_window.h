/*
 * flink_window.h — C-ABI of the MI355X keyed event-time window operator ("fw_").
 *
 * Drop-in boundary for Flink's WindowOperator + heap keyed state backend + event-time
 * timer service (paths relative to /root/reference/flink-streaming-java/src/main/java/
 * org/apache/flink/streaming/ unless they start with flink-*).  Plain pointers and sizes,
 * no C++ or torch types; every call returns an int status (FW_OK = 0, < 0 error) and
 * fw_last_error() gives the message (the Java shim throws IOException(message), as
 * HeapAggregatingState.java:90-92 wraps state errors).  Calls on one handle are serialised
 * by the caller (one handle per subtask, as one task thread owns one operator:
 * runtime/io/StreamInputProcessor.java:211-222); handles on different GPUs may be driven
 * concurrently.
 *
 * Micro-batch contract: records handed to one fw_push_* call are processed against the
 * current watermark exactly as WindowOperator.processElement would process them one by one
 * (WindowOperator.java:291-421); fw_advance_watermark is processWatermark
 * (api/operators/AbstractStreamOperator.java:735-740 -> HeapInternalTimerService.java:276-290).
 * The host therefore cuts batches at watermarks.
 */
#ifndef FLINK_WINDOW_H
#define FLINK_WINDOW_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define FW_OK 0
#define FW_ERR_ARG (-1)          /* invalid argument (IllegalArgumentException in the reference) */
#define FW_ERR_HIP (-2)          /* HIP runtime failure */
#define FW_ERR_NO_TIMESTAMP (-3) /* Long.MIN_VALUE timestamp: TumblingEventTimeWindows.java:69-71 */
#define FW_ERR_KEY_GROUP (-4)    /* key outside the handle's KeyGroupRange (KeyGroupRangeOffsets / StateTable) */
#define FW_ERR_CAPACITY (-5)     /* state could not be stored (HBM exhausted) */
#define FW_ERR_UNSUPPORTED (-6)  /* configuration not offered on the GPU path */
#define FW_ERR_STATE (-7)        /* corrupted / inconsistent handle state */

/* ---- assigner, value and key kinds ---- */
#define FW_TUMBLING 0 /* api/windowing/assigners/TumblingEventTimeWindows.java:53-73 */
#define FW_SLIDING 1  /* api/windowing/assigners/SlidingEventTimeWindows.java:57-81   */
#define FW_SESSION 2  /* api/windowing/assigners/EventTimeSessionWindows.java:59-61  */
#define FW_COUNT 3    /* count windows: KeyedStream.countWindow(size, slide) = GlobalWindows + CountTrigger.of(slide) +
                         CountEvictor.of(size) (api/datastream/KeyedStream.java:383-397; EvictingWindowOperator.java
                         :102-239,334-366; CountTrigger.java:47-55; CountEvictor.java:63-78), and countWindow(size) =
                         PurgingTrigger.of(CountTrigger.of(size)) with slide = size.  Every slide-th element of a key
                         fires the key's last min(size, elements) elements, reduced in arrival order, while the
                         element is processed (no timers; watermarks only delimit the output).  Rows: start =
                         Long.MIN_VALUE, end = Long.MAX_VALUE (GlobalWindow, timestamp Long.MAX_VALUE), count, sum,
                         min, and max = the arrival ordinal of the window's first element (the passthrough fields of
                         sum(pos)); aggregate must be FW_AGG_FIRST.  expected_entries bounds the distinct keys. */

#define FW_VAL_I64 0 /* Long field: sum wraps at 64 bits (SumFunction.LongSum)            */
#define FW_VAL_I32 1 /* Integer field: sum wraps at 32 bits (SumFunction.IntSum)          */
#define FW_VAL_F64 2 /* Double field: min/max by Double.compare, sum within 1e-6 relative */
#define FW_VAL_I16 3 /* Short field: sum wraps at 16 bits (SumFunction.ShortSum); values sign-extended */
#define FW_VAL_I8 4  /* Byte field: sum wraps at 8 bits (SumFunction.ByteSum); values sign-extended   */
#define FW_VAL_F32 5 /* Float field passed as the double of the float: min/max by Float.compare, sum
                        rounded to float (SumFunction.FloatSum adds in float: within 1e-5 relative)  */

/* the AggregateFunction (fw_config.aggregate) */
#define FW_AGG_COUNT_SUM_MIN_MAX 0 /* built-in {count, sum, min, max} accumulator                        */
#define FW_AGG_HLL 1               /* HyperLogLog distinct count of the value column read as a u64 item
                                      (definition in DESIGN.md §HLL): fired rows carry
                                      count, sum = estimate (f64 bits), min = zero registers, max = the
                                      low 64 bits of sum_j 2^(65-p-M[j]); the accumulator is the registers
                                      and the count (a snapshot row's sum / min / max are 0 / Long.MAX_VALUE
                                      / Long.MIN_VALUE, not value statistics).  Tumbling and sliding windows
                                      (one register block per window), any allowed lateness (a window fires
                                      at maxTimestamp and keeps its registers until its cleanup time), and
                                      session windows (merged sessions take the register max of their blocks,
                                      AbstractHeapMergingState.mergeNamespaces; not with PurgingTrigger:
                                      FW_ERR_UNSUPPORTED); expected_entries sizes the register pool
                                      (2^p B/entry). */
#define FW_AGG_FIRST 2             /* the reduce aggregations sum(pos) / min(pos) of DataStream / WindowedStream
                                      (SumAggregator.java:66-76, ComparableAggregator.java:72-94 over
                                      HeapReducingState.add, HeapReducingState.java:72-84): the result is a
                                      copy of the FIRST element of the window with the field replaced.  Rows
                                      carry count, sum, min as usual and max = the arrival ordinal of that
                                      first element (0-based index of the record among all records pushed
                                      into the handle), from which the caller takes the passthrough fields.
                                      Merged sessions keep the smaller ordinal.  At most 65535 windows per
                                      record. */
#define FW_AGG_MINBY 3             /* minBy(pos) / maxBy(pos) with the first-tie rule (ComparableAggregator.java
                                      :72-94, Comparator.java MinBy/MaxBy): the whole element with the smallest
                                      (largest) field, the earlier one among equal fields; Integer, Long or
                                      Double (Double.compare order) fields.  Rows carry count, sum, min = the
                                      selected field value and max = the arrival ordinal of the selected element
                                      (exact: (field, ordinal) pairs compare in full).  Sliding windows keep
                                      panes like the other aggregates: a window's element is the smallest
                                      (field, ordinal) pair over its panes. */
#define FW_AGG_MAXBY 4
#define FW_AGG_TDIGEST 6           /* t-digest quantiles of a Double field (definition in DESIGN.md
                                      §t-digest and oracle/window_oracle.h): a merging t-digest with the k1 scale
                                      function, compression tdigest_compression (delta), at most delta/2
                                      centroids; add buffers, and every push compresses the values it added.
                                      Rows carry count = elements and sum / min / max = the estimated quantiles
                                      tdigest_quantiles[0..2] (f64 bits).  Tumbling and sliding windows (one
                                      digest per window; allowed lateness without PurgingTrigger: a late firing
                                      reports the digest with the push's values so far) and session windows
                                      (merged sessions' digests merge: the union of their centroids, compressed
                                      with the push's values; AbstractHeapMergingState.mergeNamespaces; with
                                      allowed lateness, no PurgingTrigger), FW_VAL_F64; expected_entries sizes
                                      the digest pool.  Keyed-state snapshots
                                      carry the digest as an accumulator block (fw_snapshot_key_group_blocks). */
#define FW_AGG_FIRST_MAX 5         /* max(pos) (ComparableAggregator.java:72-94, Comparator.MaxComparator): as
                                      FW_AGG_FIRST, but the min column holds the field's MAXIMUM (the first
                                      element with the field replaced by the max) */

#define FW_AGG_ROW 7               /* the Table API's group-window aggregation (flink-libraries/flink-table
                                      DataStreamGroupWindowAggregate.scala:197-294 -> WindowedStream.aggregate of
                                      one accumulator Row): several built-in aggregates over up to 8 nullable value
                                      columns (row_columns, row_column_type[], row_aggregate[] = FW_ROW_* << 8 |
                                      column), pushed with fw_push_row_batch(_device).  Semantics of the Table
                                      functions (.../table/functions/aggfunctions/ *AggFunction.scala; oracle/window_oracle.h
                                      OR_AGG_ROW): COUNT(col) counts non-null values; SUM / MIN / MAX / AVG are
                                      NULL when the column had none; integral SUM wraps to the column's width;
                                      integral AVG = the Long sum / count (Java division; Long: the exact sum)
                                      narrowed to the type; Double / Float AVG = the double sum / count.  Tumbling,
                                      sliding and session windows (merged sessions merge every aggregate), allowed
                                      lateness 0, EventTimeTrigger, no side output (the Table planner sets none).
                                      Rows carry count = COUNT(*) (sum / min / max 0); fw_drain_row_results gives
                                      each row's aggregates and their NULL mask.  Keyed-state snapshots carry the
                                      accumulator as a block (fw_snapshot_key_group_blocks): per column its
                                      non-null count, the sum's low and high words (floating: the f64 sum, 0),
                                      min and max (the column's value; 0 when the count is 0), int64 each. */
#define FW_ROW_COUNT_STAR 0 /* COUNT(*) / COUNT(1): every record (CountAggFunction.accumulate(acc))           */
#define FW_ROW_COUNT 1      /* COUNT(col): the non-null values (CountAggFunction.scala:51-55)                   */
#define FW_ROW_SUM 2        /* SUM(col) (SumAggFunction.scala)                                                  */
#define FW_ROW_MIN 3        /* MIN(col) (MinAggFunction.scala; Double / Float by their compare)                 */
#define FW_ROW_MAX 4        /* MAX(col) (MaxAggFunction.scala)                                                  */
#define FW_ROW_AVG 5        /* AVG(col) (AvgAggFunction.scala: Integral / BigIntegral / Floating)               */

#define FW_KEY_LONG 0   /* key is a Long: hashCode = (int)(v ^ (v >>> 32))               */
#define FW_KEY_INT 1    /* key is an Integer: hashCode = value                              */
#define FW_KEY_HASHED 2 /* caller passes key.hashCode() per record (String, Tuple, POJO);
                           the i64 key column is then the caller's dictionary id of the key */

/* Operator configuration: the arguments of the WindowOperator constructor
 * (runtime/operators/windowing/WindowOperator.java:179-212) restricted to the GPU-eligible
 * shapes (event-time assigner above, EventTimeTrigger or PurgingTrigger.of(EventTimeTrigger),
 * AggregatingStateDescriptor/ReducingStateDescriptor with the built-in count/sum/min/max
 * accumulator), plus the keyed-backend arguments of
 * flink-runtime/.../state/StateBackend.java:130 (numberOfKeyGroups, keyGroupRange). */
typedef struct fw_config {
  int32_t assigner;            /* FW_TUMBLING / FW_SLIDING / FW_SESSION                      */
  int32_t value_type;          /* FW_VAL_*                                                   */
  int32_t key_kind;            /* FW_KEY_*                                                   */
  int32_t purging;             /* 1 = PurgingTrigger.of(EventTimeTrigger.create())           */
  int32_t side_output;         /* 1 = late records go to the side output (lateDataOutputTag) */
  int32_t max_parallelism;     /* number of key groups (0 -> 128, ExecutionJobVertex.java:176) */
  int32_t key_group_start;     /* KeyGroupRange owned by this handle, inclusive             */
  int32_t key_group_end;       /*   (-1/-1 -> the whole range [0, max_parallelism-1])        */
  int32_t device;              /* HIP device ordinal                                         */
  int32_t sub_partitions;      /* state partitions per key group, power of two (0 = auto)   */
  int64_t size;                /* window size (tumbling, sliding)                            */
  int64_t slide;               /* slide (sliding)                                            */
  int64_t offset;              /* window offset (tumbling, sliding)                          */
  int64_t gap;                 /* session gap (session)                                      */
  int64_t allowed_lateness;    /* WindowedStream.allowedLateness, >= 0                       */
  int64_t expected_entries;    /* sizing hint: live (key, window) pairs (0 = default)        */
  int64_t max_batch;           /* largest n passed to one push (0 = 1 << 24)                */
  int32_t aggregate;           /* FW_AGG_* (0 = count/sum/min/max)                           */
  int32_t hll_precision;       /* FW_AGG_HLL: p in [4, 16], m = 2^p registers (0 -> 14)       */
  int32_t tdigest_compression; /* FW_AGG_TDIGEST: delta, even, in [10, 500] (0 -> 100)         */
  int32_t tdigest_export;      /* FW_AGG_TDIGEST: 1 = fired rows also keep their centroids for
                                  fw_drain_digests                                             */
  double tdigest_quantiles[3]; /* FW_AGG_TDIGEST: the quantiles of a row (all 0 -> .5 .95 .99) */
  int32_t count_evict_after;   /* FW_COUNT: 1 = CountEvictor.of(size, true): evict after the window function
                                  (the fired window is the last min(elements, size + slide)) */
  int32_t pad0;
  int32_t row_columns;         /* FW_AGG_ROW: value columns per record, 1 .. 8                   */
  int32_t row_aggregates;      /* FW_AGG_ROW: aggregates of a row, 1 .. 16                       */
  int32_t row_column_type[8];  /* FW_AGG_ROW: FW_VAL_* of each column                            */
  int32_t row_aggregate[16];   /* FW_AGG_ROW: FW_ROW_* << 8 | column                             */
} fw_config;

typedef struct fw_op fw_op;

/* Fired window rows (struct of arrays).  One row per emitted window result:
 * the built-in AggregateFunction.getResult {count, sum, min, max} plus the key and the
 * TimeWindow; the record timestamp of the row is end - 1 = TimeWindow.maxTimestamp()
 * (TimestampedCollector.setAbsoluteTimestamp, WindowOperator.java:544-548).  For
 * FW_VAL_F64 / FW_VAL_F32, sum/min/max hold IEEE-754 double bit patterns. */
typedef struct fw_rows {
  int64_t* key;
  int64_t* start;
  int64_t* end;
  int64_t* count;
  int64_t* sum;
  int64_t* min;
  int64_t* max;
} fw_rows;

/* Late records routed to the side output (WindowOperator.sideOutput, :556-558). */
typedef struct fw_side_rows {
  int64_t* key;
  int64_t* ts;
  int64_t* val;
} fw_side_rows;

typedef struct fw_stats {
  int64_t records_in;             /* numRecordsIn                                            */
  int64_t late_records_dropped;   /* numLateRecordsDropped (WindowOperator.java:138-140,418) */
  int64_t keyed_state_entries;    /* numKeyedStateEntries of "window-contents"               */
  int64_t event_time_timers;      /* numEventTimeTimers                                      */
  int64_t current_watermark;      /* InternalTimerService.currentWatermark()                 */
  int64_t fired_rows_total;       /* all rows emitted since creation                         */
  int64_t pending_rows;           /* rows emitted and not yet drained                        */
  int64_t pending_side_rows;      /* side-output rows not yet drained                        */
  int64_t table_capacity;         /* slots in the HBM state table                            */
  int64_t table_grows;            /* times the table was resized                             */
  int64_t slow_path_records;      /* records replayed in arrival order (late firing / drop)  */
  int64_t state_merges;           /* pre-aggregated (key, window) deltas merged into HBM       */
  int64_t digest_centroids_fired; /* FW_AGG_TDIGEST: centroids of all digests fired so far      */
  int64_t single_pass_batches;    /* device batches partitioned in one pass (dense tumbling)    */
  int64_t single_pass_redone;     /* ... of which went through classify / scan / scatter after  */
  int64_t narrow_pass_batches;    /* ... of which wrote 8-byte records (key, window, int32 value) */
  int64_t narrow_pass_redone;     /* ... of which had a record without that form (then 16 bytes) */
  int64_t push_resumptions;       /* suspended sequences resumed after the host grew the table / row buffer */
} fw_stats;

/* Lifecycle — StreamOperator.setup/open/close/dispose (api/operators/StreamOperator.java:57-127). */
int fw_create(const fw_config* cfg, fw_op** out);
void fw_destroy(fw_op* op);
const char* fw_last_error(const fw_op* op);

/* processElement for a micro-batch (WindowOperator.java:291-421).
 *   fw_push_batch:        host buffers (a Java DirectByteBuffer in native byte order); the
 *                         batch is processed completely before the call returns, and errors
 *                         (FW_ERR_KEY_GROUP, FW_ERR_NO_TIMESTAMP, ...) are returned by it.
 *   fw_push_batch_device: device pointers already resident in HBM on the handle's device;
 *                         enqueued on the handle's stream and returns without waiting.  The
 *                         buffers must stay valid until the stream has passed the push (the
 *                         next fw_* call that returns a count, or fw_synchronize).  Errors the
 *                         batch raised are returned by that next call.
 * The state table grows on demand: a kernel that finds a region (or the fired-row buffer) short
 * of room stops before changing anything it could not keep, and the next synchronising call
 * grows the table and resumes it where it stopped, so no batch size is too large for the state.
 * key_hash may be NULL unless key_kind == FW_KEY_HASHED.  val points to n int64 (FW_VAL_I64 /
 * FW_VAL_I32, the latter already sign-extended) or n doubles (FW_VAL_F64). */
int fw_push_batch(fw_op* op, const int64_t* key, const int64_t* ts, const void* val, const int32_t* key_hash,
                  int64_t n);
int fw_push_batch_device(fw_op* op, const int64_t* key, const int64_t* ts, const void* val, const int32_t* key_hash,
                         int64_t n);

/* processWatermark: fires every (key, window) whose event-time timer is <= wm, clears state
 * whose cleanup time (maxTimestamp + allowedLateness, WindowOperator.java:637-644) is <= wm,
 * and returns the number of rows now pending (emitted since the last drain, including
 * late firings emitted while processing elements).  Rows pending at this point all precede
 * the watermark in the operator's output (AbstractStreamOperator.java:735-740). */
int fw_advance_watermark(fw_op* op, int64_t wm, int64_t* n_pending_rows);

/* Pending output.  *_host copy into caller-owned arrays of capacity cap and clear the pending
 * set (fw_drain_rows: host or device memory, a NULL column is skipped); fw_rows_device exposes the pending rows in HBM without copying (valid until the
 * next fw_* call) and fw_clear_pending drops them.  Each of these first settles an unsettled
 * device push. */
int fw_pending(fw_op* op, int64_t* n_rows, int64_t* n_side_rows);
int fw_drain_rows(fw_op* op, const fw_rows* host_dst, int64_t cap, int64_t* n);
int fw_drain_side(fw_op* op, const fw_side_rows* host_dst, int64_t cap, int64_t* n);
int fw_rows_device(fw_op* op, fw_rows* dev_view, int64_t* n);
/* FW_AGG_TDIGEST with tdigest_export: the centroids of the pending rows (the AggregateFunction's accumulator at
 * getResult), without draining them: for pending row i, n_centroids[i] and the centroids' sums (f64) and
 * weights at [i * delta/2 + k], k < n_centroids[i].  Call before fw_drain_rows. */
int fw_drain_digests(fw_op* op, int64_t* n_centroids, double* sum, int64_t* weight, int64_t cap_rows, int64_t* n);
int fw_clear_pending(fw_op* op);
/* FW_AGG_ROW: processElement for n records of the Table API's input rows (DataStreamGroupWindowAggregate's
 * WindowedStream.aggregate): row_columns value columns, column-major (cols + j * n = column j: int64 values
 * sign-extended, Double / Float as f64 bits), and per record a NULL mask (bit j = column j is NULL; nulls = NULL:
 * no NULLs).  Host buffers (processed before return) or HBM (_device, stream-ordered as fw_push_batch_device). */
int fw_push_row_batch(fw_op* op, const int64_t* key, const int64_t* ts, const int64_t* cols, const uint8_t* nulls,
                      const int32_t* key_hash, int64_t n);
int fw_push_row_batch_device(fw_op* op, const int64_t* key, const int64_t* ts, const int64_t* cols,
                             const uint8_t* nulls, const int32_t* key_hash, int64_t n);
/* FW_AGG_ROW: the aggregates of the pending rows (the generated AggregateFunction's getValue per aggregate:
 * values[i * row_aggregates + s], integers sign-extended, floating results as f64 bits, a Float result as the
 * double of the float) and null_mask[i] (bit s = aggregate s is NULL), without draining them: call before
 * fw_drain_rows.  Either output may be NULL. */
int fw_drain_row_results(fw_op* op, int64_t* values, uint32_t* null_mask, int64_t cap_rows, int64_t* n);

int fw_get_stats(fw_op* op, fw_stats* out);

/* Per-kernel timing with HIP events recorded around every launch on the handle's stream
 * (rocprofv3 --kernel-trace measures the same launches from outside).  Kernel kinds, in order:
 * classify_hist, scan, scatter, aggregate, slow, fire, tdigest (the t-digest compression of a push).  fw_profile_read returns accumulated
 * milliseconds and launch counts per kind (arrays of FW_NUM_KERNELS) and optionally resets them.
 * enable: 0 = off, 1 = every kind, FW_PROFILE_KINDS | (1 << kind) | ... = only those kinds (each timed launch
 * adds two event markers to its stream, so a measurement that needs one kernel's duration times only that one). */
#define FW_NUM_KERNELS 7
#define FW_PROFILE_KINDS 0x100
int fw_profile(fw_op* op, int enable);
int fw_profile_read(fw_op* op, double* ms, int64_t* launches, int reset);
const char* fw_kernel_name(int kind);
/* wait for every queued push / watermark and return the error any of them raised */
int fw_synchronize(fw_op* op);
void* fw_stream(fw_op* op); /* the hipStream_t the handle enqueues on */
/* Async input (StreamInputProcessor hands the next buffer over while the operator still works on the previous
 * one, StreamInputProcessor.java:211-223).  Enabled, fw_push_batch_device reads its columns on
 * fw_input_stream(op) — the caller orders the columns' producer before that stream (not before fw_stream) —
 * and the batch's partitioning kernels run there, beside the previous batch's aggregation and firing on
 * fw_stream.  Disabled (the default), or with side output or count windows, fw_input_stream(op) ==
 * fw_stream(op).  fw_keyby_push_device reads its columns and runs its exchange on fw_input_stream(op) too; host
 * pushes read theirs in fw_stream order. */
int fw_set_async_input(fw_op* op, int enable);
void* fw_input_stream(fw_op* op);

/* Pre-shuffle combining for the keyBy exchange: partial accumulators instead of records cross the
 * network when the aggregate is decomposable (AggregateFunction.merge, flink-core/.../AggregateFunction.java:160).
 * Eligible: tumbling windows or sliding windows kept as panes (size a multiple of slide; a partial is then one
 * (key, pane) accumulator), FW_AGG_COUNT_SUM_MIN_MAX, allowed lateness 0, no side output, Long or Integer keys.
 * A combiner is an ordinary handle over the subtask's whole input (any KeyGroupRange covering it; its watermark is
 * never advanced) into which the subtask pushes its batch; fw_combine_extract_device then drains the combiner's
 * state into the partials (device columns, the accumulators in the handle's own representation: only
 * fw_push_partials_device of a handle with the same configuration reads them) in key-group order, so destination
 * d of `world` subtasks (KeyGroupRangeAssignment.computeOperatorIndexForKeyGroup, :115-117) owns the contiguous
 * slice counts[d]; it empties the combiner.  When the partials exceed cap, *n is set, nothing is drained and
 * FW_ERR_CAPACITY is returned.  fw_push_partials_device is processElement for the partials of the receiving
 * subtask's KeyGroupRange: a partial whose window is late is dropped and its count added to the late records
 * (WindowOperator.java:402-418; with allowed lateness 0 every record of a late window is late). */
typedef struct {
  int64_t *key, *start, *cnt, *sum, *min, *max;
  /* the producing combiner's configuration tag (written by fw_combine_extract_device): assigner, size, slide,
     offset, value type, key kind, max parallelism and aggregate.  fw_push_partials_device refuses partials whose tag is
     not its own (FW_ERR_ARG): the accumulators are in the handle's internal representation (f64 min/max in
     sortable form, window starts of its own size and offset), so a differently configured receiver would
     misread them. */
  uint64_t config;
} fw_partials;
int fw_combine_extract_device(fw_op* combiner, int32_t world, fw_partials* out, int64_t cap, int64_t* counts,
                              int64_t* n);
int fw_push_partials_device(fw_op* op, const fw_partials* in, int64_t n);

/* Keyed-state snapshot and restore, one key group at a time: the heap backend writes its state per
 * key group (flink-runtime/.../state/heap/HeapKeyedStateBackend.java:289-399, offsets per key group
 * :370-381) and the timers likewise (api/operators/InternalTimeServiceManager.java:114), which is
 * what lets a restore re-shard the key groups over a different parallelism.  One row per live
 * (key, window) accumulator of "window-contents"; `timer` = 1 when the window's event-time trigger
 * timer (maxTimestamp) is registered, 0 when only its cleanup timer is pending (the cleanup timer is
 * implied by the window: cleanupTime, WindowOperator.java:637-644).  sum/min/max are in the form of
 * the fired rows (fw_rows).  Rows come out in no particular order.
 *   fw_snapshot_key_group: copies the key group's rows into caller-owned host arrays of capacity cap;
 *     with cap too small (or dst NULL) it only returns the row count in *n.
 *   fw_restore_key_group: inserts rows into the handle (which must own the key group); a row whose
 *     (key, window) is already present is merged into it (AggregateFunction.merge).  Long/Integer
 *     keys outside the key group are refused with FW_ERR_KEY_GROUP.  First-element reduces (FW_AGG_FIRST,
 *     FW_AGG_FIRST_MAX, FW_AGG_MINBY, FW_AGG_MAXBY): `max` is the element's ordinal, and later pushes are
 *     numbered after the largest restored one.  Rows of one call that restore the same (key, window) are merged
 *     in order.  HyperLogLog and t-digest handles keep their accumulator beside the row: these two calls
 *     refuse them (FW_ERR_UNSUPPORTED) and the _blocks variants below carry it. */
typedef struct fw_state_rows {
  int64_t* key;
  int64_t* start;
  int64_t* end;
  int64_t* count;
  int64_t* sum;
  int64_t* min;
  int64_t* max;
  int64_t* timer;
} fw_state_rows;
int fw_snapshot_key_group(fw_op* op, int32_t key_group, const fw_state_rows* host_dst, int64_t cap, int64_t* n);
int fw_restore_key_group(fw_op* op, int32_t key_group, const fw_state_rows* host_src, int64_t n);

/* The same with each row's accumulator block, for the aggregates whose accumulator is not in the row
 * (FW_AGG_HLL, FW_AGG_TDIGEST; any other handle takes them with blocks NULL).  The heap backend stores the
 * accumulator in the state's value column through the AggregateFunction's accumulator serializer
 * (HeapAggregatingState.java:73-93 keeps the ACC object; its TypeSerializer writes it per mapping at snapshot,
 * HeapKeyedStateBackend.java:370-381); this build's accumulators are fixed-size blocks of
 * fw_state_block_bytes(op) bytes, row i's at blocks + i * fw_state_block_bytes(op):
 *   FW_AGG_HLL      the 2^p registers M[0..m), one byte each (the rank, 0 = untouched);
 *   FW_AGG_TDIGEST  int64 little-endian words: n, then (sum as f64 bits, weight) of centroids 0..n-1 in
 *                   mean order, zero-padded to 1 + 2 * floor(delta / 2) words (the fw_rows.digests layout).
 * fw_snapshot_key_group_blocks: rows as fw_snapshot_key_group plus the blocks (host buffer of cap rows; NULL
 *   with cap 0 only counts).
 * fw_restore_key_group_blocks: rows as fw_restore_key_group; a new (key, window) takes a pool block holding the
 *   imported accumulator.  A HyperLogLog row whose (key, window) is already present merges by register max
 *   (AggregateFunction.merge); a t-digest one is refused with FW_ERR_STATE (the digest is not re-compressed).
 *   Rows must fit the pool (expected_entries): FW_ERR_CAPACITY otherwise, before anything changes. */
int64_t fw_state_block_bytes(fw_op* op);
int fw_snapshot_key_group_blocks(fw_op* op, int32_t key_group, const fw_state_rows* host_dst, uint8_t* host_blocks,
                                 int64_t cap, int64_t* n);
int fw_restore_key_group_blocks(fw_op* op, int32_t key_group, const fw_state_rows* host_src,
                                const uint8_t* host_blocks, int64_t n);

/* Key routing (both sides of keyBy).
 *   fw_key_groups_device: kg[i] = KeyGroupRangeAssignment.assignToKeyGroup(key_i, maxParallelism)
 *     (flink-runtime/.../state/KeyGroupRangeAssignment.java:58-71, MathUtils.java:134-154).
 *   fw_route_device: KeyGroupStreamPartitioner.selectChannels (runtime/partitioner/
 *     KeyGroupStreamPartitioner.java:53-65): groups the batch by destination operator index
 *     computeOperatorIndexForKeyGroup(maxPar, parallelism, kg) (KeyGroupRangeAssignment.java:115-117),
 *     keeping arrival order inside each destination; writes the reordered columns and
 *     counts[parallelism] (int64, device).  All pointers are device pointers on `device`;
 *     the call is asynchronous on `stream` (a hipStream_t, NULL = default stream). */
int fw_key_groups_device(const int64_t* key, const int32_t* key_hash, int32_t key_kind, int64_t n,
                         int32_t max_parallelism, int32_t* kg_out, void* stream);
int fw_route_device(const int64_t* key, const int64_t* ts, const int64_t* val, const int32_t* key_hash,
                    int32_t key_kind, int64_t n, int32_t max_parallelism, int32_t parallelism, int64_t* key_out,
                    int64_t* ts_out, int64_t* val_out, int32_t* hash_out, int64_t* counts, void* scratch,
                    int64_t scratch_bytes, void* stream);
int64_t fw_route_scratch_bytes(int64_t n, int32_t parallelism);

/* Pre-shuffle combining of HyperLogLog ("combining is results-equal for count/sum/min/max/HLL"): a
 * combiner's windows cross the exchange as partial rows plus their non-zero registers, the receiver merges them
 * with AggregateFunction.merge = register max (flink-core/.../AggregateFunction.java:160).  Tumbling windows, no
 * allowed lateness, Long or Integer keys (FW_ERR_UNSUPPORTED otherwise).
 *   fw_combine_extract_hll_device: drains the combiner like fw_combine_extract_device; a row's sum = how many of
 *     its window's registers are non-zero (min holds an opaque block id until the registers are taken),
 *     reg_counts[d] = the registers of destination d's partials (in partial order), *nregs their total.
 *   fw_combine_hll_registers_device: then writes the n rows' registers into regs[0, nregs) as u32
 *     (register index << 8 | rank), in row order, and releases the combiner's blocks (FW_ERR_CAPACITY, with
 *     nothing taken, when regs_cap < nregs; FW_ERR_STATE without a preceding extraction of n rows).
 *   fw_push_hll_partials_device: merges received partial rows (counts) and raises their registers (regs: the rows'
 *     register lists concatenated in row order) into this operator's windows; late rows are dropped with their
 *     records, as fw_push_partials_device does. */
int fw_combine_extract_hll_device(fw_op* op, int32_t world, fw_partials* out, int64_t cap, int64_t* counts,
                                  int64_t* reg_counts, int64_t* n, int64_t* nregs);
int fw_combine_hll_registers_device(fw_op* op, const fw_partials* out, int64_t n, uint32_t* regs, int64_t regs_cap);
int fw_push_hll_partials_device(fw_op* op, const fw_partials* in, int64_t n, const uint32_t* regs, int64_t nregs);

/* keyBy across the GPUs of one node behind the C-ABI (the RecordWriter -> KeyGroupStreamPartitioner ->
 * network -> input gate path: flink-runtime/.../io/network/api/writer/RecordWriter.java:88-115,
 * runtime/partitioner/KeyGroupStreamPartitioner.java:53-65; watermark valve runtime/streamstatus/
 * StatusWatermarkValve.java:173-191), over RCCL.  One communicator per subtask / GPU:
 *   fw_comm_unique_id: rank 0 creates the id (128 bytes) and hands it to the other subtasks (e.g. through the
 *     JobManager); fw_comm_init: every subtask joins with its rank (= its operator index) on its device.
 *   fw_keyby_push_device: this subtask's device batch is grouped by destination subtask
 *     (computeOperatorIndexForKeyGroup), the per-peer counts are exchanged (all-to-all of one int64 each, then
 *     read by the host: the receive sizes), the key / timestamp / value (/ key hash) columns go peer to peer
 *     (grouped ncclSend / ncclRecv, one pair per peer), and the records received from subtasks 0 .. world-1, each
 *     source's arrival order kept, are pushed into `op` (fw_push_batch_device), whose KeyGroupRange must be
 *     computeKeyGroupRangeForOperatorIndex(maxParallelism, world, rank).  *combined_wm = min over the subtasks of
 *     local_wm (the operator's input watermark), for the caller's fw_advance_watermark.  Collective: every
 *     subtask calls it once per batch.  Enqueued on fw_input_stream(op); the host waits once per batch, for the
 *     route and the count exchange on that stream (with async input not for the previous batch's aggregation). */
typedef struct fw_comm fw_comm;
int fw_comm_unique_id(void* id128);
int fw_comm_init(const void* id128, int32_t world, int32_t rank, int32_t device, fw_comm** out);
void fw_comm_destroy(fw_comm* comm);
int fw_keyby_push_device(fw_comm* comm, fw_op* op, const int64_t* key, const int64_t* ts, const void* val,
                         const int32_t* key_hash, int64_t n, int64_t local_wm, int64_t* combined_wm);
/* The same with pre-shuffle combining (see fw_combine_extract_device): the batch goes into `combiner` (this
 * subtask's combiner handle, same configuration -- FW_ERR_ARG otherwise --, never given a watermark), which is
 * drained into partials; the
 * partials' per-peer counts and six columns cross the exchange instead of the records, and the received ones are
 * merged into `op` (fw_push_partials_device).  Eligible configurations only. */
int fw_keyby_combine_push_device(fw_comm* comm, fw_op* combiner, fw_op* op, const int64_t* key, const int64_t* ts,
                                 const void* val, int64_t n, int64_t local_wm, int64_t* combined_wm);
/* The exchange's counters (the sending side of RecordWriter's numBytesOut / numRecordsOut,
 * flink-runtime/.../io/network/api/writer/RecordWriter.java:88-115): world / rank as the RCCL communicator reports
 * them (ncclCommCount / ncclCommUserRank), batches exchanged, items (records, or partials when combining) and
 * bytes sent to and received from the OTHER subtasks (a subtask's own share never leaves the GPU), how often the
 * receive columns were reallocated and what they hold. */
typedef struct fw_comm_stats {
  int32_t world, rank;
  int64_t batches, items_sent, items_received, bytes_sent, bytes_received, recv_reallocs, recv_capacity;
} fw_comm_stats;
int fw_comm_get_stats(fw_comm* comm, fw_comm_stats* out);
/* The host arithmetic of one exchange round, from the counts round's int64[2 world + 4] (send counts per peer,
 * receive counts per peer, watermark in / min, batch size in / sum over subtasks): send and receive offsets
 * ([world + 1] each, prefix sums: records from subtask 0 first, then 1, ..., as the input gate's channels) and
 * the totals.  recv_bound = the sum of every subtask's batch: no subtask can receive more, so the receive columns
 * are sized for it once.  FW_ERR_STATE when the counts contradict themselves (negative, more received than the
 * whole batch, the own share sent != received). */
typedef struct fw_exchange_plan_t {
  int64_t send_total, recv_total, items_sent, items_received, recv_bound;
} fw_exchange_plan_t;
int fw_exchange_plan(int32_t world, int32_t rank, const int64_t* counts, int64_t* send_off, int64_t* recv_off,
                     fw_exchange_plan_t* out);

/* ---- f2: Flink's wire format for one input channel <-> device columns.
 * The byte stream of a channel is its network buffers in order: SpanningRecordSerializer.addRecord writes each
 * StreamElement as a 4-byte big-endian length and then its bytes (flink-runtime/.../io/network/api/serialization/
 * SpanningRecordSerializer.java:76-98), StreamElementSerializer (SJ/runtime/streamrecord/StreamElementSerializer
 * .java:54-58, 167-221) writes a tag byte then
 *   0 record with timestamp: BE i64 timestamp, the value      1 record without timestamp: the value
 *   2 watermark: BE i64       3 latency marker: BE i64 marked time, BE i64 x 2 operator id, BE i32 subtask
 *   4 stream status: BE i32   (any other tag: "Corrupt stream, found tag: X")
 * and the value is a Tuple (TupleSerializer: fields in order, no null mask) of fixed-size fields, or one bare
 * field: Long / Integer / Short / Byte / Boolean (BE two's complement) and Double / Float (BE
 * doubleToLongBits / floatToIntBits), or String (StringSerializer -> StringValue.writeString, StringValue.java:
 * 789-817: length + 1 as a base-128 varint, 0 = null, then each UTF-16 char as a base-128 varint).  A String
 * field is the key (FW_ROLE_KEY) or skipped: the key column then holds the chars' 64-bit id (FNV-1a 64 over the
 * UTF-16 chars, then fmix64 of it ^ the length) and the key_hash column String.hashCode, the two columns
 * FW_KEY_HASHED takes; a null String key is a corrupt element (KeyGroupStreamPartitioner cannot hash it).  A
 * record with String fields is decoded when it is at most 64 bytes with its length prefix (WindowWordCount's
 * Tuple2<String, Integer> with a timestamp: words of up to 46 ASCII chars).
 *   fw_wire_decode_device: a device byte stream -> key / ts / val columns in arrival order (records without a
 *     timestamp get Long.MIN_VALUE, StreamRecord.getTimestamp), ready for fw_push_batch_device.  The field whose
 *     role is FW_ROLE_KEY becomes the key (an integer kind), FW_ROLE_VALUE the value (integers sign-extended,
 *     Double as its bits, Float widened to double bits); other fields are skipped.  stats: the frames of each
 *     kind, the last watermark (Long.MIN_VALUE if none: the caller's processWatermark), the last stream status
 *     (StreamStatus ACTIVE 0 / IDLE -1; 0 if none), and `consumed` = the bytes up to the end of the last complete element (a trailing partial element is
 *     the start of the next call's stream, SpillingAdaptiveSpanningRecordDeserializer's role).  Frames are
 *     found in parallel: every 2 KiB chunk is parsed from each of its 64 possible first-frame offsets, and the
 *     chunks' transfer functions are composed (a decoded element is at most 64 bytes with its length prefix:
 *     value fields of at most 51 bytes).
 *   fw_wire_encode_device: fired rows -> elements of one output channel: tag 0, timestamp = end - 1 (the
 *     window's maxTimestamp, WindowOperator.emitWindowContents' TimestampedCollector), a Tuple of the row
 *     fields the layout's roles name (FW_ROLE_KEY / START / END / COUNT / SUM / MIN / MAX).
 * Both return FW_ERR_ARG for an unsupported layout and FW_ERR_STATE for a corrupt stream (message in
 * fw_wire_last_error) or too small an output; they run on the codec's own stream and return when done. */
#define FW_WIRE_LONG 0
#define FW_WIRE_INT 1
#define FW_WIRE_DOUBLE 2
#define FW_WIRE_SHORT 3
#define FW_WIRE_BYTE 4
#define FW_WIRE_FLOAT 5
#define FW_WIRE_BOOL 6
#define FW_WIRE_STRING 7
#define FW_ROLE_SKIP 0
#define FW_ROLE_KEY 1
#define FW_ROLE_VALUE 2
#define FW_ROLE_START 3
#define FW_ROLE_END 4
#define FW_ROLE_COUNT 5
#define FW_ROLE_SUM 6
#define FW_ROLE_MIN 7
#define FW_ROLE_MAX 8
#define FW_WIRE_MAX_FIELDS 8
typedef struct {
  int32_t nfields;                     /* 1 = a bare field, > 1 = a Tuple of that arity */
  int32_t kind[FW_WIRE_MAX_FIELDS];    /* FW_WIRE_* */
  int32_t role[FW_WIRE_MAX_FIELDS];    /* FW_ROLE_* */
} fw_wire_layout;
typedef struct {
  int64_t records, watermarks, latency_markers, statuses;
  int64_t consumed;                    /* bytes of complete elements */
  int64_t watermark;                   /* the last watermark, Long.MIN_VALUE if none */
  int32_t status;                      /* the last stream status (0 ACTIVE, -1 IDLE), 0 if none */
  int32_t pad;
} fw_wire_stats;
typedef struct fw_wire fw_wire;
/* max_bytes: the largest stream of one decode call; device: the HIP device of the buffers */
int fw_wire_create(const fw_wire_layout* layout, int64_t max_bytes, int32_t device, fw_wire** out);
void fw_wire_destroy(fw_wire* w);
const char* fw_wire_last_error(const fw_wire* w);
int fw_wire_decode_device(fw_wire* w, const uint8_t* bytes, int64_t nbytes, int64_t* key, int64_t* ts, int64_t* val,
                          int64_t cap, fw_wire_stats* stats);
/* the same with the key_hash column (int32, the key's Java hashCode: String.hashCode of a String key, 0 for the
 * other kinds, whose hash the operator derives itself); required when the key field is a String */
int fw_wire_decode_keyed_device(fw_wire* w, const uint8_t* bytes, int64_t nbytes, int64_t* key, int32_t* key_hash,
                                int64_t* ts, int64_t* val, int64_t cap, fw_wire_stats* stats);
/* rows: a device view (fw_rows_device); f64 = the rows' sum/min/max are double bits (FW_VAL_F64 aggregates);
 * out: device bytes of capacity cap; *written = n * element size */
int fw_wire_encode_device(fw_wire* w, const fw_rows* rows, int64_t n, int32_t f64, uint8_t* out, int64_t cap,
                          int64_t* written);

/* ---- f4: window contents (ListState) — WindowedStream.apply / process with an Iterable window function, and
 * evictors (SJ/api/datastream/WindowedStream.java:1080-1123 builds a WindowOperator over a ListStateDescriptor, or an
 * EvictingWindowOperator when an evictor is set).  The handle keeps every (key, window)'s list of elements in HBM
 * and applies, element by element, EvictingWindowOperator.processElement / onEventTime / emitWindowContents
 * (runtime/operators/windowing/EvictingWindowOperator.java:102-366; without an evictor WindowOperator.java:291-469):
 *   assigners  FW_TUMBLING, FW_SLIDING (every window of a record holds a copy), FW_GLOBAL (GlobalWindows: never
 *              late, never cleaned up; rows have start = Long.MIN_VALUE, end = Long.MAX_VALUE = their timestamp);
 *   triggers   FW_TRIGGER_EVENT_TIME (EventTimeTrigger.java:37-73) or FW_TRIGGER_COUNT (CountTrigger.of(n),
 *              CountTrigger.java:47-70), either wrapped in PurgingTrigger (purging = 1);
 *   evictors   CountEvictor.of(n[, after]) (CountEvictor.java:50-78), TimeEvictor.of(ms[, after]) (TimeEvictor.java
 *              :54-104; a timestamp of Long.MIN_VALUE is "no timestamp": nothing is evicted when the first element
 *              has none), DeltaEvictor.of(threshold, f[, after]) with the built-in f(e, last) = last.field - e.field
 *              in the field's Java arithmetic (DeltaEvictor.java:59-80).
 * Every firing emits one row: the window, count = elements the function sees (after evictBefore), the built-in
 * reduce over them in list order (sum wrapped to the field width, min, max; Double / Float fields by compare
 * order, sums in list order, so f64 sums are exact), first = the arrival ordinal of the first element (-1 if none;
 * the passthrough fields of reduce / sum(pos)), and with emit_contents the elements themselves in list order
 * (timestamp, value, ordinal) for the host's Iterable function (InternalIterableWindowFunction).  A push is
 * processed completely before the call returns (late firings and count triggers are ordered per (key, window)). */
#define FW_GLOBAL 4
#define FW_TRIGGER_EVENT_TIME 0
#define FW_TRIGGER_COUNT 1
#define FW_EVICT_NONE 0
#define FW_EVICT_COUNT 1
#define FW_EVICT_TIME 2
#define FW_EVICT_DELTA 3
typedef struct fw_list_config {
  int32_t assigner;          /* FW_TUMBLING / FW_SLIDING / FW_GLOBAL / FW_SESSION (size = the gap)  */
  int32_t value_type;        /* FW_VAL_*                                                          */
  int32_t key_kind;          /* FW_KEY_*                                                          */
  int32_t trigger;           /* FW_TRIGGER_*                                                      */
  int32_t purging;           /* PurgingTrigger.of(trigger)                                        */
  int32_t evictor;           /* FW_EVICT_*                                                        */
  int32_t evict_after;       /* doEvictAfter                                                      */
  int32_t side_output;       /* late records to the side output instead of numLateRecordsDropped */
  int32_t emit_contents;     /* 1 = fired rows carry their elements                               */
  int32_t max_parallelism;   /* as fw_config                                                      */
  int32_t key_group_start;
  int32_t key_group_end;
  int32_t device;
  int32_t pad0;
  int64_t size, slide, offset, allowed_lateness;
  int64_t trigger_count;     /* CountTrigger.of(n)                                                */
  int64_t evict_count;       /* CountEvictor maxCount, TimeEvictor windowSize (ms)                */
  double delta_threshold;    /* DeltaEvictor threshold                                            */
  int64_t expected_elements; /* sizing hint: elements held at once (0 = default)                  */
  int64_t max_batch;         /* largest n of one push (0 = 1 << 24)                               */
} fw_list_config;
typedef struct fw_list_rows {
  int64_t *key, *start, *end, *count, *sum, *min, *max;
  int64_t* first;            /* arrival ordinal of the row's first element, -1 if none          */
  int64_t* elem_off;         /* index of the row's first element among the drained elements     */
} fw_list_rows;
typedef struct fw_list_elems {
  int64_t *ts, *val, *ordinal;
} fw_list_elems;
/* A key group's list state, for snapshot / restore (the heap backend writes "window-contents" per key group:
 * HeapKeyedStateBackend.java:370-381): per (key, window) its list, CountTrigger's count and whether its
 * EventTimeTrigger timer is registered; the elements of all lists concatenated in list order. */
typedef struct fw_list_state {
  int64_t *key, *start, *end, *trigger_count, *timer, *n_elems;  /* per list   */
  int64_t *ts, *val, *ordinal;                                   /* elements   */
} fw_list_state;
typedef struct fw_list fw_list;
/* as fw_create: on an error *out may hold a handle that carries the message (fw_list_last_error); destroy it */
int fw_list_create(const fw_list_config* cfg, fw_list** out);
void fw_list_destroy(fw_list* op);
const char* fw_list_last_error(const fw_list* op);
/* processElement for a batch: host buffers, or device buffers on the handle's device (key_hash as fw_push_batch) */
int fw_list_push_batch(fw_list* op, const int64_t* key, const int64_t* ts, const void* val, const int32_t* key_hash,
                       int64_t n);
int fw_list_push_batch_device(fw_list* op, const int64_t* key, const int64_t* ts, const void* val,
                              const int32_t* key_hash, int64_t n);
/* processWatermark: the EventTimeTrigger timers <= wm fire their lists, cleanup timers drop them */
int fw_list_advance_watermark(fw_list* op, int64_t wm, int64_t* n_pending_rows);
int fw_list_pending(fw_list* op, int64_t* n_rows, int64_t* n_elems, int64_t* n_side_rows);
/* copies the pending rows (and elements: elem_off counts from the first drained element) into host arrays and
 * clears them; FW_ERR_CAPACITY (nothing drained) when either capacity is too small */
int fw_list_drain(fw_list* op, const fw_list_rows* rows, int64_t cap_rows, const fw_list_elems* elems,
                  int64_t cap_elems, int64_t* n_rows, int64_t* n_elems);
int fw_list_drain_side(fw_list* op, const fw_side_rows* host_dst, int64_t cap, int64_t* n);
/* drops the pending rows and elements without copying them (a discarding sink) */
int fw_list_clear_pending(fw_list* op);
int fw_list_get_stats(fw_list* op, fw_stats* out);
/* per key group: the lists (dst NULL or a capacity too small: only the counts) / restored into the handle, appended
 * to a list already present */
int fw_list_snapshot_key_group(fw_list* op, int32_t key_group, const fw_list_state* dst, int64_t cap_lists,
                               int64_t cap_elems, int64_t* n_lists, int64_t* n_elems);
int fw_list_restore_key_group(fw_list* op, int32_t key_group, const fw_list_state* src, int64_t n_lists,
                              int64_t n_elems);

/* Synthetic source used by the benchmarks (the same counter-based generator as the CPU
 * baseline and the tests): record i of stream `seed` has
 *   key = splitmix64(seed ^ 4i) mod num_keys  (uniform)  or Zipf(zipf_s) over num_keys,
 *   val = (int32) splitmix64(seed ^ (4i+1)),
 *   ts  = ts_base + floor(i * 1000 / rate) - (splitmix64(seed ^ (4i+2)) mod jitter).
 * Writes records [first, first + n) to device buffers; returns max(ts) over them in *max_ts
 * (device int64, may be NULL).  zipf_cdf (device, num_keys doubles) is used when non-NULL. */
int fw_generate_device(uint64_t seed, int64_t first, int64_t n, int64_t num_keys, const double* zipf_cdf,
                       int64_t ts_base, int64_t rate, int64_t jitter, int64_t* key, int64_t* ts, int64_t* val,
                       int64_t* max_ts, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FLINK_WINDOW_H */
