"""CPU checks of the keyBy exchange's host arithmetic (fw_exchange_plan, no GPU): the per-peer send / receive
offsets a subtask derives from one counts round (all-to-all of per-destination counts, the watermark's MIN and the
batch sizes' SUM), for world 8 with skewed routing, and its rejection of inconsistent rounds.

Reference: RecordWriter.emit -> KeyGroupStreamPartitioner.selectChannels
(flink-runtime/.../io/network/api/writer/RecordWriter.java:88-115, KeyGroupRangeAssignment.java:85-117): records
of one destination stay in arrival order, and a subtask's input gate holds channel 0's records first."""
import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd.exchange import exchange_plan
from flink_amd.keygroups import (assign_to_key_group, compute_key_group_range_for_operator_index,
                                 compute_operator_index_for_key_group, long_hash_code)


def rounds(sent):
    """sent[r][p] = records subtask r routes to p: each subtask's counts round as the collectives leave it."""
    W = len(sent)
    batch = [int(sum(row)) for row in sent]
    out = []
    for r in range(W):
        c = [int(sent[r][p]) for p in range(W)] + [int(sent[p][r]) for p in range(W)]
        c += [1000 + r, 1000, batch[r], sum(batch)]  # wm in, wm min, batch in, batch sum
        out.append(c)
    return out


def skewed_counts(W=8, n=1 << 16, seed=7):
    """Zipf(1.1) Long keys over 10^4 keys routed by key group: a few hot keys pile onto one subtask."""
    rng = np.random.default_rng(seed)
    sent = np.zeros((W, W), dtype=np.int64)
    for r in range(W):
        keys = rng.zipf(1.1, n) % 10_000
        dest = [compute_operator_index_for_key_group(128, W, assign_to_key_group(long_hash_code(int(k)), 128)) for k in keys[:4096]]
        sent[r] = np.bincount(dest, minlength=W) * (n // 4096)
    return sent


@pytest.mark.parametrize("world", [1, 2, 8])
def test_plan_offsets_and_totals(world):
    sent = skewed_counts(world) if world > 1 else np.array([[12345]])
    for r, c in enumerate(rounds(sent)):
        so, ro, pl = exchange_plan(world, r, c)
        assert so == [0] + list(np.cumsum(sent[r]))
        assert ro == [0] + list(np.cumsum(sent[:, r]))
        assert pl["send_total"] == sent[r].sum() and pl["recv_total"] == sent[:, r].sum()
        assert pl["items_sent"] == sent[r].sum() - sent[r, r]
        assert pl["items_received"] == sent[:, r].sum() - sent[r, r]
        assert pl["recv_bound"] == sent.sum()
        assert pl["recv_total"] <= pl["recv_bound"]


def test_skew_is_real_and_bounded():
    # the hottest subtask receives far more than it sent, yet never more than the bound the receive columns are
    # sized for on the first batch (so a skewed batch does not reallocate them)
    sent = skewed_counts(8)
    recv = sent.sum(axis=0)
    assert recv.max() > 1.3 * sent.sum(axis=1).mean()
    for r, c in enumerate(rounds(sent)):
        _, _, pl = exchange_plan(8, r, c)
        assert pl["recv_total"] == recv[r] <= pl["recv_bound"]


def test_plan_rejects_inconsistent_rounds():
    sent = skewed_counts(8)
    c = rounds(sent)[3]
    bad = list(c)
    bad[8 + 2] = -1  # negative receive count
    with pytest.raises(N.NativeError) as e:
        exchange_plan(8, 3, bad)
    assert e.value.code == N.FW_ERR_STATE
    bad = list(c)
    bad[2 * 8 + 3] = sum(c[8:16]) - 1  # more received than the whole batch
    with pytest.raises(N.NativeError):
        exchange_plan(8, 3, bad)
    bad = list(c)
    bad[8 + 3] += 1  # own share sent != received
    with pytest.raises(N.NativeError):
        exchange_plan(8, 3, bad)
    with pytest.raises(N.NativeError) as e:
        exchange_plan(8, 8, c)  # rank out of range
    assert e.value.code == N.FW_ERR_ARG


def test_key_group_ranges_cover_world_8():
    # the ranges the plan's destinations own: contiguous, disjoint, 16 key groups each at M = 128
    cover = []
    for r in range(8):
        kgr = compute_key_group_range_for_operator_index(128, 8, r)
        a, b = kgr.start_key_group, kgr.end_key_group
        assert b - a + 1 == 16
        cover += list(range(a, b + 1))
        for kg in (a, b):
            assert compute_operator_index_for_key_group(128, 8, kg) == r
    assert cover == list(range(128))
