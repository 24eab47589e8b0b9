"""Window assigners, triggers, time and the built-in aggregate of the GPU path — the host mirror
of the reference's API objects.  They only carry parameters (validated exactly as the reference's
constructors do); assignment itself runs in the HIP kernels.

Reference (flink-streaming-java/src/main/java/org/apache/flink/streaming/api/):
  windowing/assigners/TumblingEventTimeWindows.java:53-126
  windowing/assigners/SlidingEventTimeWindows.java:50-146
  windowing/assigners/EventTimeSessionWindows.java:45-113
  windowing/triggers/EventTimeTrigger.java, PurgingTrigger.java
  windowing/time/Time.java
"""
from dataclasses import dataclass

from . import _native as N


class Time:
    """windowing/time/Time.java: a size in milliseconds."""

    def __init__(self, ms):
        self.ms = int(ms)

    @staticmethod
    def milliseconds(v):
        return Time(v)

    @staticmethod
    def seconds(v):
        return Time(v * 1000)

    @staticmethod
    def minutes(v):
        return Time(v * 60_000)

    @staticmethod
    def hours(v):
        return Time(v * 3_600_000)

    @staticmethod
    def days(v):
        return Time(v * 86_400_000)

    def to_milliseconds(self):
        return self.ms


def _ms(t):
    return t.ms if isinstance(t, Time) else int(t)


class WindowAssigner:
    kind = None
    is_event_time = True

    def config(self):
        raise NotImplementedError


class TumblingEventTimeWindows(WindowAssigner):
    """TumblingEventTimeWindows.of(size[, offset]) (TumblingEventTimeWindows.java:53-58,104-121)."""
    kind = N.FW_TUMBLING

    def __init__(self, size, offset=0):
        if offset < 0 or offset >= size:
            raise ValueError("TumblingEventTimeWindows parameters must satisfy 0 <= offset < size")
        self.size, self.offset = size, offset

    @staticmethod
    def of(size, offset=0):
        return TumblingEventTimeWindows(_ms(size), _ms(offset))

    def config(self):
        return dict(assigner=self.kind, size=self.size, slide=self.size, offset=self.offset)

    def __repr__(self):
        return f"TumblingEventTimeWindows({self.size})"


class SlidingEventTimeWindows(WindowAssigner):
    """SlidingEventTimeWindows.of(size, slide[, offset]) (SlidingEventTimeWindows.java:57-64,120-141)."""
    kind = N.FW_SLIDING

    def __init__(self, size, slide, offset=0):
        if offset < 0 or offset >= slide or size <= 0:
            raise ValueError("SlidingEventTimeWindows parameters must satisfy 0 <= offset < slide and size > 0")
        self.size, self.slide, self.offset = size, slide, offset

    @staticmethod
    def of(size, slide, offset=0):
        return SlidingEventTimeWindows(_ms(size), _ms(slide), _ms(offset))

    def config(self):
        return dict(assigner=self.kind, size=self.size, slide=self.slide, offset=self.offset)

    def __repr__(self):
        return f"SlidingEventTimeWindows({self.size}, {self.slide})"


class EventTimeSessionWindows(WindowAssigner):
    """EventTimeSessionWindows.withGap(gap) (EventTimeSessionWindows.java:52-57,94-96)."""
    kind = N.FW_SESSION

    def __init__(self, gap):
        if gap <= 0:
            raise ValueError("EventTimeSessionWindows parameters must satisfy 0 < size")
        self.gap = gap

    @staticmethod
    def with_gap(gap):
        return EventTimeSessionWindows(_ms(gap))

    withGap = with_gap

    def config(self):
        return dict(assigner=self.kind, gap=self.gap)

    def __repr__(self):
        return f"EventTimeSessionWindows({self.gap})"


class CountWindows(WindowAssigner):
    """KeyedStream.countWindow(size, slide) = window(GlobalWindows.create()).evictor(CountEvictor.of(size))
    .trigger(CountTrigger.of(slide)), and countWindow(size) = PurgingTrigger.of(CountTrigger.of(size))
    (KeyedStream.java:383-397): every slide-th element of a key fires its last `size` elements (the last
    size + slide with evict_after, CountEvictor.of(size, true)).  Rows have start = Long.MIN_VALUE, end =
    Long.MAX_VALUE (GlobalWindow) and are emitted while the elements are processed."""
    kind = N.FW_COUNT
    is_event_time = False

    def __init__(self, size, slide=None, evict_after=False):
        slide = size if slide is None else slide
        if size <= 0 or slide <= 0:
            raise ValueError("count windows need positive size and slide")
        self.size, self.slide, self.evict_after = int(size), int(slide), bool(evict_after)

    @staticmethod
    def of(size, slide=None, evict_after=False):
        return CountWindows(size, slide, evict_after)

    def config(self):
        return dict(assigner=self.kind, size=self.size, slide=self.slide, count_evict_after=int(self.evict_after))

    def __repr__(self):
        return f"CountWindows({self.size}, {self.slide})"


class Trigger:
    purging = False


class EventTimeTrigger(Trigger):
    """EventTimeTrigger.create() (EventTimeTrigger.java:37-73)."""

    @staticmethod
    def create():
        return EventTimeTrigger()


class PurgingTrigger(Trigger):
    """PurgingTrigger.of(EventTimeTrigger.create()) (PurgingTrigger.java:45-59); around CountTrigger.of(n) for the
    window-contents operator only."""
    purging = True

    def __init__(self, nested):
        if not isinstance(nested, (EventTimeTrigger, CountTrigger)):
            raise ValueError("the GPU path offers PurgingTrigger only around EventTimeTrigger or CountTrigger")
        self.nested = nested

    @staticmethod
    def of(nested):
        return PurgingTrigger(nested)


class GlobalWindows(WindowAssigner):
    """GlobalWindows.create() (GlobalWindows.java): one window per key, not event time (never late, no cleanup
    timer); for the window-contents operator (GpuListWindowOperator)."""
    kind = N.FW_GLOBAL

    @staticmethod
    def create():
        return GlobalWindows()

    def config(self):
        return dict(assigner=self.kind)

    def __repr__(self):
        return "GlobalWindows()"


class CountTrigger(Trigger):
    """CountTrigger.of(n) (CountTrigger.java:47-70): FIRE at every n-th element of a (key, window)."""

    def __init__(self, count):
        if count <= 0:
            raise ValueError("count must be positive")
        self.count = count

    @staticmethod
    def of(count):
        return CountTrigger(count)


class Evictor:
    kind = N.FW_EVICT_NONE
    evict_after = False
    arg = 0
    threshold = 0.0


@dataclass(frozen=True)
class CountEvictor(Evictor):
    """CountEvictor.of(maxCount[, doEvictAfter]) (CountEvictor.java:50-78): keeps the last maxCount elements."""
    arg: int = 0
    evict_after: bool = False
    kind = N.FW_EVICT_COUNT

    @staticmethod
    def of(max_count, evict_after=False):
        return CountEvictor(max_count, evict_after)


@dataclass(frozen=True)
class TimeEvictor(Evictor):
    """TimeEvictor.of(windowSize[, doEvictAfter]) (TimeEvictor.java:54-104): drops the elements with a timestamp
    <= max timestamp - windowSize (none when the first element has no timestamp)."""
    arg: int = 0
    evict_after: bool = False
    kind = N.FW_EVICT_TIME

    @staticmethod
    def of(window_size, evict_after=False):
        return TimeEvictor(int(window_size), evict_after)


@dataclass(frozen=True)
class DeltaEvictor(Evictor):
    """DeltaEvictor.of(threshold, f[, doEvictAfter]) (DeltaEvictor.java:59-80) with the built-in DeltaFunction
    f(e, last) = last.field - e.field (the field's Java arithmetic): drops the elements with f >= threshold."""
    threshold: float = 0.0
    evict_after: bool = False
    kind = N.FW_EVICT_DELTA

    @staticmethod
    def of(threshold, evict_after=False):
        return DeltaEvictor(float(threshold), evict_after)


# the field types of the built-in aggregations (SumFunction.java:34-107): Short / Byte sums wrap to their width,
# Float fields are passed as doubles and their sums rounded to float
VALUE_TYPES = {"long": N.FW_VAL_I64, "int": N.FW_VAL_I32, "double": N.FW_VAL_F64, "short": N.FW_VAL_I16,
               "byte": N.FW_VAL_I8, "float": N.FW_VAL_F32}
FLOAT_TYPES = ("double", "float")


@dataclass(frozen=True)
class CountSumMinMax:
    """The built-in AggregateFunction of the GPU path: ACC = OUT = (count, sum, min, max) of one
    numeric field.  `value_type` is "long" (sum wraps at 64 bits), "int" (SumFunction.IntSum:
    wraps at 32 bits, so `sum(pos)` on an Integer field), "short" / "byte" (ShortSum / ByteSum: wrap at
    16 / 8 bits), "double" (min/max by Double.compare, sum within 1e-6 relative of the reference's
    left-to-right order) or "float" (the float values as doubles; FloatSum rounds every partial sum to
    float, the GPU rounds the sum once: within 1e-5 relative).
    sum/min/max of WindowedStream (WindowedStream.java:1354-1535) are projections of this
    accumulator onto one field."""
    value_type: str = "long"

    def native(self):
        return VALUE_TYPES[self.value_type]

    def hll_precision(self):
        return 0

    def tdigest(self):
        return None

    def aggregate_kind(self):
        return N.FW_AGG_COUNT_SUM_MIN_MAX


@dataclass(frozen=True)
class FirstElementReduce:
    """The reduce aggregations `sum(pos)` / `min(pos)` of WindowedStream (WindowedStream.java:1354-1439):
    a ReducingState (HeapReducingState.add, HeapReducingState.java:72-84) whose reduce keeps a copy of
    its FIRST argument with the field replaced (SumAggregator.reduce, SumAggregator.java:66-76;
    ComparableAggregator.reduce, ComparableAggregator.java:72-94).  The GPU keeps count/sum/min of the
    field and the arrival ordinal of the window's first element (fired rows: max = that ordinal);
    `first_element_results` rebuilds the reference's output tuples from it.  Merged sessions keep the
    earlier element (the reference's choice follows HashSet order: parity unpinned).
    `field="max"` is `max(pos)`: the rows' min column then holds the field's maximum."""
    value_type: str = "int"
    field: str = "sum"

    def native(self):
        return VALUE_TYPES[self.value_type]

    def hll_precision(self):
        return 0

    def tdigest(self):
        return None

    def aggregate_kind(self):
        return N.FW_AGG_FIRST_MAX if self.field == "max" else N.FW_AGG_FIRST


@dataclass(frozen=True)
class ExtremalElementReduce:
    """`minBy(pos)` / `maxBy(pos)` of WindowedStream (first = true): the whole element whose field is the
    smallest (largest), the earlier one among equal fields (ComparableAggregator.reduce,
    ComparableAggregator.java:72-94; Comparator MinBy/MaxBy): Integer ("int"), Long ("long") or Double
    ("double", Double.compare order) fields.  Fired rows: min = the selected field, max = the selected
    element's arrival ordinal (`selected_elements` returns the elements)."""
    kind: str = "min"
    value_type: str = "int"

    def native(self):
        return VALUE_TYPES[self.value_type]

    def hll_precision(self):
        return 0

    def tdigest(self):
        return None

    def aggregate_kind(self):
        return N.FW_AGG_MINBY if self.kind == "min" else N.FW_AGG_MAXBY


def selected_elements(rows, elements):
    """The output elements of minBy/maxBy: the element at each row's ordinal (`max`)."""
    return [tuple(elements[int(r["max"])]) for r in rows]


def first_element_results(rows, elements, pos, field="sum"):
    """The output tuples of `sum(pos)` (field "sum") or `min(pos)` (field "min") from fired rows of a
    FirstElementReduce operator: a copy of the window's first element (its arrival ordinal is the row's
    `max`) with field `pos` replaced, as SumAggregator.reduce / ComparableAggregator.reduce leave it
    (SumAggregator.java:66-76, ComparableAggregator.java:72-94).  `elements[i]` is the i-th element the
    operator was given (the caller keeps the passthrough fields; the GPU keeps only the ordinal)."""
    out = []
    for r in rows:
        t = list(elements[int(r["max"])])
        t[pos] = int(r[field])
        out.append(tuple(t))
    return out


@dataclass(frozen=True)
class HyperLogLog:
    """User AggregateFunction of SURVEY §8d C5: a HyperLogLog distinct count of a Long item field with
    2^precision one-byte registers per (key, window) (definition: DESIGN.md §HLL, restated in
    oracle/window_oracle.h).  add = register max of the item's hash; merge = register-wise max;
    getResult = (count, estimate).  Fired rows: count, sum = estimate (f64 bits), min = zero registers,
    max = the low 64 bits of sum_j 2^(65 - p - M[j]) (an exact register checksum).  Offered on the GPU
    for tumbling, sliding and session windows, with allowed lateness and PurgingTrigger."""
    precision: int = 14
    value_type: str = "long"

    def native(self):
        return N.FW_VAL_I64

    def hll_precision(self):
        return self.precision

    def tdigest(self):
        return None

    def aggregate_kind(self):
        return N.FW_AGG_HLL


ROW_FUNCTIONS = {"count_star": N.FW_ROW_COUNT_STAR, "count": N.FW_ROW_COUNT, "sum": N.FW_ROW_SUM, "min": N.FW_ROW_MIN,
                 "max": N.FW_ROW_MAX, "avg": N.FW_ROW_AVG}


@dataclass(frozen=True)
class RowAggregate:
    """The Table API's group-window accumulator (DataStreamGroupWindowAggregate.scala:197-294: one generated
    AggregateFunction over a Row holding several built-in aggregates): `column_types` are the value columns' types
    ("long", "int", "short", "byte", "double", "float"; up to 8, nullable), `aggregates` the select list's built-in
    aggregates as (function, column index) with function in count_star / count / sum / min / max / avg (up to 16).
    Semantics of flink-table's CountAggFunction, SumAggFunction, Min/MaxAggFunction and AvgAggFunction (restated in
    oracle/window_oracle.h OR_AGG_ROW).  Records go in through GpuWindowOperator.process_rows; fired rows carry
    count = COUNT(*) and drain_row_results gives each row's aggregate values and NULL mask."""
    column_types: tuple = ("long",)
    aggregates: tuple = (("count_star", 0),)
    value_type: str = "long"  # (a record's value column is its index in the push)

    def native(self):
        return N.FW_VAL_I64

    def hll_precision(self):
        return 0

    def tdigest(self):
        return None

    def aggregate_kind(self):
        return N.FW_AGG_ROW

    def spec_words(self):
        return [(ROW_FUNCTIONS[f] << 8) | int(c) for f, c in self.aggregates]

    def type_codes(self):
        return [VALUE_TYPES[t] for t in self.column_types]


@dataclass(frozen=True)
class TDigest:
    """User AggregateFunction of SURVEY §8d C5: quantiles of a Double field per key and window from a merging
    t-digest with the k1 scale function and compression `compression` (delta; at most delta/2 centroids).
    Definition: DESIGN.md §t-digest, restated in oracle/window_oracle.h.  add buffers the value; every
    micro-batch (push) compresses the values it added into the centroids (AggregateFunction.merge of the
    batch's digest); getResult = (count, the quantiles `quantiles`).  Fired rows: count, sum / min / max =
    the three quantile estimates (f64 bits).  With export=True the operator also keeps each fired row's
    centroids (GpuWindowOperator.drain_digests).  Offered for tumbling, sliding and session windows, with allowed
    lateness and PurgingTrigger."""
    compression: int = 100
    quantiles: tuple = (0.5, 0.95, 0.99)
    export: bool = False
    value_type: str = "double"

    def native(self):
        return N.FW_VAL_F64

    def hll_precision(self):
        return 0

    def tdigest(self):
        return self

    def aggregate_kind(self):
        return N.FW_AGG_TDIGEST


def tdigest_quantile(sums, weights, mn, mx, q):
    """Quantile q of a digest's centroids (sum, weight) with the window's min / max: the read-out of
    TDigest's getResult (piecewise-linear through (0, min), (centre_i, mean_i), (W, max)), for a row's
    exported centroids."""
    W = float(sum(int(w) for w in weights))
    if not len(sums):
        return float("nan")
    x = q * W
    x0, y0, before = 0.0, mn, 0.0
    for s, w in zip(sums, weights):
        t = before + float(w) * 0.5
        m = float(s) / float(w)
        if t >= x:
            return y0 + (m - y0) * ((x - x0) / (t - x0))
        x0, y0, before = t, m, before + float(w)
    return y0 + (mx - y0) * ((x - x0) / (W - x0))
