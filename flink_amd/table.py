"""Table API group windows on the GPU path -- the host mirror of
flink-libraries/flink-table/src/main/scala/org/apache/flink/table/plan/nodes/datastream/
DataStreamGroupWindowAggregate.scala:197-294 for event-time windows: `table.window(Tumble | Slide | Session ...)
.groupBy('w, keys).select(keys, aggregates, 'w.start, 'w.end)` becomes keyBy(keys).window(assigner).aggregate(the
generated Row accumulator, the window-property function).  Here the accumulator is RowAggregate (FW_AGG_ROW: the
built-in COUNT(*) / COUNT / SUM / MIN / MAX / AVG over nullable columns in HBM), and the window function appends
w.start / w.end (AggregateUtil.createAggregationGroupWindowFunction).  The planner's rewrite of a query into this
operator needs the JVM and is not rebuilt; a host that has planned a query hands the select list to this class.
"""
import numpy as np

from .windowing import (EventTimeSessionWindows, FLOAT_TYPES, RowAggregate, SlidingEventTimeWindows,
                        TumblingEventTimeWindows, _ms)


class Tumble:
    """Tumble over <size> on 'rowtime (TumblingGroupWindow -> TumblingEventTimeWindows.of(size))."""

    def __init__(self, size):
        self.size = _ms(size)

    @staticmethod
    def over(size):
        return Tumble(size)

    def assigner(self):
        return TumblingEventTimeWindows.of(self.size)


class Slide:
    """Slide over <size> every <slide> on 'rowtime (SlidingGroupWindow -> SlidingEventTimeWindows.of(size, slide))."""

    def __init__(self, size, slide=None):
        self.size, self.slide = _ms(size), None if slide is None else _ms(slide)

    @staticmethod
    def over(size):
        return Slide(size)

    def every(self, slide):
        return Slide(self.size, slide)

    def assigner(self):
        return SlidingEventTimeWindows.of(self.size, self.slide)


class Session:
    """Session withGap <gap> on 'rowtime (SessionGroupWindow -> EventTimeSessionWindows.withGap(gap))."""

    def __init__(self, gap):
        self.gap = _ms(gap)

    @staticmethod
    def with_gap(gap):
        return Session(gap)

    withGap = with_gap

    def assigner(self):
        return EventTimeSessionWindows.with_gap(self.gap)


def _decode(fn, t, v):
    """A result word as the aggregate's SQL value: COUNTs are Long; SUM / MIN / MAX / AVG have the column's type."""
    if fn in ("count_star", "count") or t not in FLOAT_TYPES:
        return int(v)
    return float(np.array([v], dtype=np.int64).view(np.float64)[0])


class GroupWindowAggregate:
    """One keyed event-time group window with a select list of built-in aggregates over value columns.
    `column_types`: the aggregated columns' types; `aggregates`: [(function, column index)], function one of
    count_star, count, sum, min, max, avg.  Records: process(keys, rowtimes, columns, nulls[, key_hash]);
    watermark(wm) returns the rows fired by it as [(key, [aggregate values, None = NULL], w.start, w.end)]."""

    def __init__(self, window, column_types, aggregates, key_type="long", device=0, expected_entries=0, max_batch=0,
                 **kw):
        from .operator import GpuWindowOperator
        self.column_types = tuple(column_types)
        self.aggregates = tuple((f, int(c)) for f, c in aggregates)
        self.agg = RowAggregate(self.column_types, self.aggregates)
        self.op = GpuWindowOperator(window.assigner(), self.agg, key_type=key_type, device=device,
                                    expected_entries=expected_entries, max_batch=max_batch, **kw)

    def process(self, keys, rowtimes, columns, nulls=None, key_hash=None):
        self.op.process_row_batch(keys, rowtimes, columns, nulls, key_hash)

    def watermark(self, wm):
        self.op.advance_watermark(wm)
        vals, nm = self.op.drain_row_results()
        rows = self.op.drain_rows(self.op.epoch - 1)
        out = []
        for i, r in enumerate(rows):
            v = [None if (int(nm[i]) >> q) & 1 else _decode(f, self.column_types[c], vals[i][q])
                 for q, (f, c) in enumerate(self.aggregates)]
            out.append((int(r["key"]), v, int(r["start"]), int(r["end"])))
        return out

    def close(self):
        self.op.close()
