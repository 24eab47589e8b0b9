"""The keyBy exchange across GPUs of one node: one process per GPU, each owning the contiguous
KeyGroupRange computeKeyGroupRangeForOperatorIndex(maxPar, world, rank).

Reference path being replaced: RecordWriterOutput -> RecordWriter.emit -> KeyGroupStreamPartitioner.
selectChannels (flink-streaming-java/.../runtime/partitioner/KeyGroupStreamPartitioner.java:53-65,
flink-runtime/.../io/network/api/writer/RecordWriter.java:88-115) and the Netty / local input channels
on the receiving side; watermarks are broadcast to every channel and the receiver takes the minimum
over channels (flink-streaming-java/.../runtime/streamstatus/StatusWatermarkValve.java:173-191).

On MI355X: the batch is grouped by destination on the GPU (fw_route_device, stable), the per-peer
counts are exchanged (all_to_all_single of P int64), then the key, timestamp and value columns go
peer-to-peer, one all_to_all_single each (RCCL over xGMI: each peer pair has its own link).  The watermark is one int64
all_reduce(MIN).  The collectives are torch.distributed's, so the same code runs over "nccl" (RCCL) on
the GPU box and over "gloo" in the CPU tests, where the caller supplies the routing function.
"""
import ctypes

from . import _native as N
from .keygroups import compute_key_group_range_for_operator_index


def route_device(keys, ts, vals, max_parallelism, parallelism, key_hash=None, key_kind=N.FW_KEY_LONG):
    """Stable grouping of a device-resident batch by destination operator index.
    Returns ((keys, ts, vals, hashes) reordered, counts[parallelism] int64) as CUDA tensors."""
    import torch
    n = keys.numel()
    dev = keys.device
    ko, to, vo = torch.empty_like(keys), torch.empty_like(ts), torch.empty_like(vals)
    ho = torch.empty(n, dtype=torch.int32, device=dev)
    counts = torch.empty(parallelism, dtype=torch.int64, device=dev)
    nbytes = N.lib().fw_route_scratch_bytes(n, parallelism)
    scratch = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    rc = N.lib().fw_route_device(keys.data_ptr(), ts.data_ptr(), vals.data_ptr(),
                                 key_hash.data_ptr() if key_hash is not None else None, key_kind, n,
                                 max_parallelism, parallelism, ko.data_ptr(), to.data_ptr(), vo.data_ptr(),
                                 ho.data_ptr(), counts.data_ptr(), scratch.data_ptr(), nbytes, stream)
    N.check(rc)
    return (ko, to, vo, ho), counts


class KeyGroupExchange:
    """Per-batch keyBy shuffle between the `world` operator subtasks (ranks) of one job vertex."""

    def __init__(self, max_parallelism, world, rank, route_fn=route_device, group=None):
        self.max_parallelism = max_parallelism
        self.world = world
        self.rank = rank
        self.route_fn = route_fn
        self.group = group
        self.key_group_range = compute_key_group_range_for_operator_index(max_parallelism, world, rank)
        self.bytes_sent = 0

    def exchange(self, keys, ts, vals):
        """Returns this rank's (keys, ts, vals): records from rank 0 first, then rank 1, ...,
        each source's arrival order kept (the per-channel order Flink guarantees)."""
        import torch
        import torch.distributed as dist
        if self.world == 1:
            return keys, ts, vals
        (k, t, v, _), counts = self.route_fn(keys, ts, vals, self.max_parallelism, self.world)
        recv_counts = torch.empty_like(counts)
        dist.all_to_all_single(recv_counts, counts, group=self.group)
        in_split = counts.tolist()
        out_split = recv_counts.tolist()
        total = sum(out_split)
        # one all-to-all per SoA column, straight from the routed columns into the operator's input
        # columns: no interleave before the send or split after it (each would cost 48 B/record of HBM)
        out = []
        for col in (k, t, v):
            r = torch.empty(total, dtype=col.dtype, device=col.device)
            dist.all_to_all_single(r, col, output_split_sizes=out_split, input_split_sizes=in_split,
                                   group=self.group)
            out.append(r)
        self.bytes_sent += 24 * (sum(in_split) - in_split[self.rank])
        return out[0], out[1], out[2]

    def combine_watermark(self, local_wm, device=None):
        """StatusWatermarkValve: the operator's input watermark is the minimum over its channels."""
        import torch
        import torch.distributed as dist
        if self.world == 1:
            return int(local_wm)
        t = torch.tensor([int(local_wm)], dtype=torch.int64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return int(t.item())


del ctypes
