"""Shared by the oracle and GPU tests of f3 (Table API group windows, DataStreamGroupWindowAggregate.scala:197-294):
the reference ITCases' inputs (tests/golden/reference_kats.json "table_group_windows") as batches, and the row
comparison (one row per (key, window) with the select list's values and NULLs)."""
import numpy as np

MAX = (1 << 63) - 1


def case_cfg(case):
    """Assigner keyword arguments of the oracle / the GPU operator for a KAT case."""
    a = case["assigner"]
    if a == "tumbling":
        return dict(assigner="tumbling", size=case["size"])
    if a == "sliding":
        return dict(assigner="sliding", size=case["size"], slide=case["slide"])
    return dict(assigner="session", gap=case["gap"])


def case_events(case):
    """The input as (keys, ts, cols, nulls) per element, each followed by the punctuated watermark ts - offset
    (TimestampAndWatermarkWithOffset), then Long.MAX_VALUE; keys are dictionary ids of the grouping key strings
    (None = the null key).  Returns (key_names, [(keys, ts, cols, nulls, watermark), ...])."""
    names = []
    for _, _, k in case["input"]:
        if k not in names:
            names.append(k)
    nc = len(case["types"])
    steps = []
    for t, vals, k in case["input"]:
        cols = [np.array([0 if vals[j] is None else vals[j]], dtype=np.int64) for j in range(nc)]
        nm = np.array([sum(1 << j for j in range(nc) if vals[j] is None)], dtype=np.uint8)
        steps.append((np.array([names.index(k)], dtype=np.int64), np.array([t], dtype=np.int64), cols, nm,
                      t - case["offset"]))
    empty = np.zeros(0, dtype=np.int64)
    steps.append((empty, empty, [empty] * nc, np.zeros(0, dtype=np.uint8), MAX))
    return names, steps


def expected_rows(case, names):
    """Sorted [(key id, start, end, (values with None for NULL))] of the ITCase's expected output."""
    return sorted((names.index(k), s, e, tuple(v)) for k, s, e, v in case["expected"])


def rows_with_values(rows, vals, nulls):
    """Sorted [(key, start, end, (values, None for NULL))] of fired rows and their result matrix."""
    out = []
    for i, r in enumerate(rows):
        v = tuple(None if (int(nulls[i]) >> q) & 1 else int(vals[i][q]) for q in range(vals.shape[1]))
        out.append((int(r["key"]), int(r["start"]), int(r["end"]), v))
    return sorted(out)
