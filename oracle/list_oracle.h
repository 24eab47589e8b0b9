/*
 * list_oracle.h — CPU restatement of Flink's window-contents (ListState) window paths.
 *
 * TEST INFRASTRUCTURE ONLY (the parity checker of flink_amd's fw_list_* operator).  Only tests/ and
 * bench.py's cpu_baseline leg may load it; the product path never links or calls anything under oracle/.
 *
 * Restates, element by element (paths relative to /root/reference/flink-streaming-java/src/main/java/
 * org/apache/flink/streaming/):
 *   runtime/operators/windowing/EvictingWindowOperator.java:102-239   processElement (non-merging assigners, and the
 *                                                                       merging branch :110-170 for session windows:
 *                                                                       MergingWindowSet.java:150-225, the merged lists
 *                                                                       in mergeNamespaces order: the state window's
 *                                                                       list, then the others' in HashSet order,
 *                                                                       AbstractHeapMergingState.java:67-93)
 *   runtime/operators/windowing/EvictingWindowOperator.java:241-286   onEventTime
 *   runtime/operators/windowing/EvictingWindowOperator.java:334-366   emitWindowContents (evictBefore, the
 *                                                                       function, evictAfter, the list re-stored)
 *   runtime/operators/windowing/WindowOperator.java:291-469, 544-548  the same without an evictor (ListState +
 *                                                                       InternalIterableWindowFunction: apply/process)
 *   runtime/operators/windowing/WindowOperator.java:576-651           lateness / cleanup time / side output
 *   api/windowing/triggers/EventTimeTrigger.java:37-73, CountTrigger.java:47-70, PurgingTrigger.java:45-59
 *   api/windowing/evictors/CountEvictor.java:50-78, TimeEvictor.java:54-104, DeltaEvictor.java:59-80
 *   api/windowing/assigners/GlobalWindows.java (isEventTime false: never late, no cleanup timer)
 *   api/operators/HeapInternalTimerService.java:224-290                timer dedup + advanceWatermark
 *
 * The window function is the caller's (an Iterable function on the host): every firing records the
 * contents it saw (after evictBefore), in list order, plus the build's reduce over them: count, the
 * field's sum in list order (SumAggregator over the Iterable: wrapped to the field width, Float sums in
 * float), min and max (Double.compare / Float.compare order for floating fields), and `first` = the
 * arrival ordinal of the first element.  DeltaEvictor's DeltaFunction is the built-in field difference
 * delta(e, last) = last.field - e.field in the field's Java arithmetic (int subtraction for Integer /
 * Short / Byte, long for Long, double / float for Double / Float), widened to double.
 * A timestamp of Long.MIN_VALUE is "no timestamp" (StreamRecord.hasTimestamp false: the wire codec's
 * decoding of a record without one); TimeEvictor then evicts nothing when the first element has none.
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_GLOBAL = 3 };
enum { OR_TRIG_EVENT_TIME = 0, OR_TRIG_COUNT = 1 };
enum { OR_EVICT_NONE = 0, OR_EVICT_COUNT = 1, OR_EVICT_TIME = 2, OR_EVICT_DELTA = 3 };

typedef struct {
  int32_t assigner;        /* OR_TUMBLING / OR_SLIDING / OR_GLOBAL / OR_SESSION (size = the gap; EventTimeTrigger) */
  int32_t value_type;      /* OR_VAL_* */
  int64_t size, slide, offset, lateness;
  int32_t trigger;         /* OR_TRIG_* */
  int32_t purging;         /* PurgingTrigger.of(trigger) */
  int64_t trigger_count;   /* CountTrigger.of(n) */
  int32_t evictor;         /* OR_EVICT_* */
  int32_t evict_after;     /* doEvictAfter */
  int64_t evict_count;     /* CountEvictor maxCount / TimeEvictor windowSize (ms) */
  double delta_threshold;  /* DeltaEvictor threshold */
  int32_t side_output;
  int32_t pad;
} oracle_list_cfg;

typedef struct {
  int64_t key, start, end, count, sum, min, max, first, elem_off, epoch;
} oracle_list_row;

typedef struct {
  int64_t ts, val, ord;
} oracle_list_elem;

void*   oracle_list_create(const oracle_list_cfg* cfg);
void    oracle_list_destroy(void* op);
int     oracle_list_process(void* op, const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n);
int     oracle_list_watermark(void* op, int64_t wm);
int64_t oracle_list_num_rows(void* op);
int64_t oracle_list_num_elems(void* op);
void    oracle_list_get_rows(void* op, oracle_list_row* out);
void    oracle_list_get_elems(void* op, oracle_list_elem* out);
int64_t oracle_list_num_side_rows(void* op);
void    oracle_list_get_side_rows(void* op, int64_t* key, int64_t* ts, int64_t* val, int64_t* epoch);
int64_t oracle_list_late_dropped(void* op);
int64_t oracle_list_num_state_entries(void* op); /* live (key, window) lists */
int64_t oracle_list_num_timers(void* op);

#ifdef __cplusplus
}
#endif
