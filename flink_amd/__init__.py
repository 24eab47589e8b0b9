"""flink_amd — MI355X-native keyed event-time window aggregation (Flink WindowOperator drop-in).

The hot path (key-group hashing, window assignment, HBM state table, watermark firing) runs in the
HIP kernels of libflinkwin.so (flink_amd/csrc, gfx950).  This package is the host-side mirror of the
reference's operator interface for that path; see DESIGN.md and INTEGRATION.md.
"""
from .keygroups import (KeyGroupRange, assign_key_to_parallel_operator, assign_to_key_group,  # noqa: F401
                        compute_default_max_parallelism, compute_key_group_range_for_operator_index,
                        compute_operator_index_for_key_group, long_hash_code, murmur_hash, string_hash_code)
from .windowing import (CountEvictor, CountTrigger, DeltaEvictor, GlobalWindows, TimeEvictor,  # noqa: F401
                        CountSumMinMax, CountWindows, ExtremalElementReduce, FirstElementReduce, HyperLogLog, TDigest,  # noqa: F401
                        RowAggregate,
                        EventTimeSessionWindows, EventTimeTrigger, PurgingTrigger, SlidingEventTimeWindows, Time,
                        TumblingEventTimeWindows, first_element_results, selected_elements, tdigest_quantile)


def __getattr__(name):
    # the operator needs the native library; import lazily so host-only helpers work without it
    if name == "GpuWindowOperator":
        from .operator import GpuWindowOperator
        return GpuWindowOperator
    if name in ("GroupWindowAggregate", "Tumble", "Slide", "Session"):
        from . import table
        return getattr(table, name)
    if name == "GpuListWindowOperator":
        from .listwindow import GpuListWindowOperator
        return GpuListWindowOperator
    raise AttributeError(name)
