"""The N>1 path on CPU: KeyGroupExchange (flink_amd/exchange.py) at world size 2 over gloo.

Each rank generates its slice of the global stream (as bench.py does), routes it by destination
operator index kg*G/maxPar (KeyGroupRangeAssignment.java:115-117), exchanges counts and records with
all_to_all_single and combines watermarks with all_reduce(MIN) (StatusWatermarkValve.java:173-191).
The window operator behind the exchange is the oracle here (no GPU on this container); the test checks
the exchange: every record arrives at the rank owning its key group, per-source arrival order is kept,
and the union of both ranks' fired rows equals one operator over the whole stream.
"""
import os
import socket

import numpy as np
import pytest

from flink_amd.keygroups import (compute_key_group_range_for_operator_index,
                                 compute_operator_index_for_key_group)
from oracle import oracle as orc

MAX_PAR = 128
WORLD = 2
BATCH = 4096
STEPS = 6
KEYS = 3000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _slice(rank, step):
    from flink_amd.datagen import generate_host
    first = (step * WORLD + rank) * BATCH
    return generate_host(0x5EED, first, BATCH, KEYS, ts_base=0, rate=100_000, jitter=300)


def _host_route(keys, ts, vals, max_par, par, key_hash=None, key_kind=0):
    """CPU stand-in for fw_route_device: stable grouping by destination (test-side key groups; Long keys)."""
    import torch
    k = keys.numpy()
    dest = (orc.key_groups_long(k, max_par).astype(np.int64) * par) // max_par
    order = np.argsort(dest, kind="stable")
    counts = np.bincount(dest, minlength=par).astype(np.int64)
    pick = torch.from_numpy(order)
    return (keys[pick], ts[pick], vals[pick], None), torch.from_numpy(counts)


def _worker(rank, port, out_dir):
    import torch
    import torch.distributed as dist
    from flink_amd.exchange import KeyGroupExchange
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    ex = KeyGroupExchange(MAX_PAR, WORLD, rank, route_fn=_host_route)
    op = orc.WindowOperatorOracle(assigner="tumbling", size=1000)
    got_keys, mx = [], -(1 << 63)
    for s in range(STEPS):
        k, t, v = (torch.from_numpy(np.ascontiguousarray(x)) for x in _slice(rank, s))
        mx = max(mx, int(t.max()))
        rk, rt, rv = ex.exchange(k, t, v)
        wm = ex.combine_watermark(mx - 200)
        op.process(rk.numpy(), rt.numpy(), rv.numpy())
        op.watermark(wm)
        got_keys.append(rk.numpy())
        np.save(os.path.join(out_dir, f"recv_{rank}_{s}.npy"), np.stack([rk.numpy(), rt.numpy(), rv.numpy()]))
    op.watermark((1 << 63) - 1)
    np.save(os.path.join(out_dir, f"rows_{rank}.npy"), op.rows())
    dist.destroy_process_group()


def test_exchange_world2_gloo(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    # routing: every received record belongs to the receiving rank's KeyGroupRange, and each step's
    # receive buffer is source 0's records then source 1's, each in arrival order
    for r in range(WORLD):
        kgr = compute_key_group_range_for_operator_index(MAX_PAR, WORLD, r)
        for s in range(STEPS):
            rk, rt, rv = np.load(tmp_path / f"recv_{r}_{s}.npy")
            kg = orc.key_groups_long(rk, MAX_PAR)
            assert ((kg >= kgr.start_key_group) & (kg <= kgr.end_key_group)).all()
            assert all(compute_operator_index_for_key_group(MAX_PAR, WORLD, int(g)) == r for g in kg[:50])
            exp = []
            for src in range(WORLD):
                k, t, v = _slice(src, s)
                d = (orc.key_groups_long(k, MAX_PAR).astype(np.int64) * WORLD) // MAX_PAR
                sel = d == r
                exp.append(np.stack([k[sel], t[sel], v[sel]]))
            np.testing.assert_array_equal(np.concatenate(exp, axis=1), np.stack([rk, rt, rv]))
    # results: both ranks' rows == one operator over the whole stream with the global watermarks
    rows = np.concatenate([np.load(tmp_path / f"rows_{r}.npy") for r in range(WORLD)])
    ref = orc.WindowOperatorOracle(assigner="tumbling", size=1000)
    mx = [-(1 << 63)] * WORLD
    for s in range(STEPS):
        parts = [_slice(r, s) for r in range(WORLD)]
        for r in range(WORLD):
            mx[r] = max(mx[r], int(parts[r][1].max()))
        # the same per-rank arrival order the exchange produced (source-major)
        for src in range(WORLD):
            ref.process(*parts[src])
        ref.watermark(min(m - 200 for m in mx))
    ref.watermark((1 << 63) - 1)
    r = ref.rows()
    key = lambda a: np.lexsort((a["start"], a["key"]))
    a, b = rows[key(rows)], r[key(r)]
    assert len(a) == len(b) > 0
    for f in ("key", "start", "end", "count", "sum", "min", "max"):
        np.testing.assert_array_equal(a[f], b[f])
