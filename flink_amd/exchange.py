"""The keyBy exchange across GPUs of one node: one process per GPU, each owning the contiguous
KeyGroupRange computeKeyGroupRangeForOperatorIndex(maxPar, world, rank).

Reference path being replaced: RecordWriterOutput -> RecordWriter.emit -> KeyGroupStreamPartitioner.
selectChannels (flink-streaming-java/.../runtime/partitioner/KeyGroupStreamPartitioner.java:53-65,
flink-runtime/.../io/network/api/writer/RecordWriter.java:88-115) and the Netty / local input channels
on the receiving side; watermarks are broadcast to every channel and the receiver takes the minimum
over channels (flink-streaming-java/.../runtime/streamstatus/StatusWatermarkValve.java:173-191).

On MI355X: the batch is grouped by destination on the GPU (fw_route_device, stable), the per-peer
counts are exchanged (all_to_all_single of P int64), then the key, timestamp and value columns (and the
key hashes of String / Tuple keys) go peer-to-peer, one all_to_all_single each (RCCL over xGMI: each peer
pair has its own link).  The watermark is one int64 all_reduce(MIN).  KeyGroupExchange uses
torch.distributed's collectives, so the same code runs over "nccl" (RCCL) and over "gloo" (CUDA columns
staged through host memory); NativeKeyByExchange is the same sequence inside libflinkwin.so
(fw_keyby_push_device over the library's own RCCL communicator), the path a JNI host calls.
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


def exchange_plan(world, rank, counts):
    """fw_exchange_plan: send / receive offsets and totals of one exchange round from the counts round's
    int64[2 world + 4] (send counts, receive counts, watermark in / min, batch size in / sum).  Pure host arithmetic
    (no GPU).  Returns (send_off, recv_off, plan dict); raises NativeError(FW_ERR_STATE) on inconsistent counts."""
    c = (ctypes.c_int64 * (2 * world + 4))(*[int(x) for x in counts])
    so, ro = (ctypes.c_int64 * (world + 1))(), (ctypes.c_int64 * (world + 1))()
    pl = N.FwExchangePlan()
    rc = N.lib().fw_exchange_plan(world, rank, c, so, ro, ctypes.byref(pl))
    if rc != N.FW_OK:
        raise N.NativeError(rc, "inconsistent exchange counts")
    return list(so), list(ro), {f: getattr(pl, f) for f, _ in N.FwExchangePlan._fields_}


_KEY_KINDS = {"long": N.FW_KEY_LONG, "int": N.FW_KEY_INT, "hashed": N.FW_KEY_HASHED}


class KeyGroupExchange:
    """Per-batch keyBy shuffle between the `world` operator subtasks (ranks) of one job vertex.
    key_type: "long" (Long keys), "int" (Integer keys: Integer.hashCode) or "hashed" (the caller passes
    key.hashCode() per record, which travels with the record)."""

    def __init__(self, max_parallelism, world, rank, route_fn=route_device, group=None, key_type="long"):
        self.max_parallelism = max_parallelism
        self.world = world
        self.rank = rank
        self.route_fn = route_fn
        self.group = group
        self.key_kind = _KEY_KINDS[key_type]
        self.key_group_range = compute_key_group_range_for_operator_index(max_parallelism, world, rank)
        self.bytes_sent = self.items_sent = self.bytes_received = 0

    def exchange(self, keys, ts, vals, key_hash=None):
        """Returns this rank's (keys, ts, vals) — and key hashes as a 4th column when key_hash is given:
        records from rank 0 first, then rank 1, ..., each source's arrival order kept (the per-channel order
        Flink guarantees)."""
        import torch
        import torch.distributed as dist
        if self.key_kind == N.FW_KEY_HASHED and key_hash is None:
            raise ValueError("key_hash is required for hashed (String / Tuple) keys")
        if self.world == 1:
            return (keys, ts, vals) if key_hash is None else (keys, ts, vals, key_hash)
        (k, t, v, h), counts = self.route_fn(keys, ts, vals, self.max_parallelism, self.world, key_hash=key_hash,
                                             key_kind=self.key_kind)
        # gloo moves host tensors: CUDA columns are staged through host memory (the nccl backend takes them as is)
        staged = keys.is_cuda and dist.get_backend(self.group) == "gloo"
        move = (lambda x: x.cpu()) if staged else (lambda x: x)
        back = (lambda x: x.to(keys.device)) if staged else (lambda x: x)
        counts = move(counts)
        recv_counts = torch.empty_like(counts)
        dist.all_to_all_single(recv_counts, counts, group=self.group)
        in_split = counts.tolist()
        out_split = recv_counts.tolist()
        total = sum(out_split)
        # one all-to-all per SoA column, straight from the routed columns into the operator's input
        # columns: no interleave before the send or split after it (each would cost 48 B/record of HBM)
        cols = (k, t, v) + ((h,) if key_hash is not None else ())
        out = []
        for col in cols:
            col = move(col)
            r = torch.empty(total, dtype=col.dtype, device=col.device)
            dist.all_to_all_single(r, col, output_split_sizes=out_split, input_split_sizes=in_split,
                                   group=self.group)
            out.append(back(r))
        rec = 24 + (4 if key_hash is not None else 0)
        self.items_sent += sum(in_split) - in_split[self.rank]
        self.bytes_sent += rec * (sum(in_split) - in_split[self.rank])
        self.bytes_received += rec * (total - out_split[self.rank])
        return tuple(out)

    def combine_watermark(self, local_wm, device=None):
        """StatusWatermarkValve: the operator's input watermark is the minimum over its channels."""
        import torch
        import torch.distributed as dist
        if self.world == 1:
            return int(local_wm)
        t = torch.tensor([int(local_wm)], dtype=torch.int64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return int(t.item())


class NativeKeyByExchange:
    """fw_keyby_push_device: route, count exchange, peer-to-peer columns and the push into the operator, all
    inside libflinkwin.so over its own RCCL communicator (the sequence a JNI host calls).
    `unique_id` (128 bytes) comes from rank 0's NativeKeyByExchange.new_unique_id(), shared by the caller."""

    def __init__(self, op, world, rank, unique_id):
        self.op = op
        self.world, self.rank = world, rank
        self._c = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(unique_id), 128)
        rc = N.lib().fw_comm_init(buf, world, rank, op.device, ctypes.byref(self._c))
        if rc != N.FW_OK:
            raise N.NativeError(rc, "fw_comm_init failed")

    @staticmethod
    def new_unique_id():
        buf = ctypes.create_string_buffer(128)
        N.check(N.lib().fw_comm_unique_id(buf))
        return buf.raw

    def push(self, keys, ts, vals, local_wm, key_hash=None):
        """Exchanges this subtask's device batch and pushes what it receives; returns the combined watermark."""
        import torch
        wm = ctypes.c_int64()
        n = keys.numel()
        # the library's input stream reads the columns: it waits for their producer first
        self.op._input_stream(keys.device).wait_stream(torch.cuda.current_stream(keys.device))
        rc = N.lib().fw_keyby_push_device(self._c, self.op._h, keys.data_ptr(), ts.data_ptr(), vals.data_ptr(),
                                          key_hash.data_ptr() if key_hash is not None else None, n, int(local_wm),
                                          ctypes.byref(wm))
        N.check(rc, self.op._h)
        self.op._inflight = (keys, ts, vals, key_hash)
        return wm.value

    def push_combined(self, combiner, keys, ts, vals, local_wm):
        """fw_keyby_combine_push_device: the batch aggregated by `combiner` (a GpuWindowOperator of the same
        configuration over the whole key space), its partials exchanged and merged into the operator."""
        import torch
        wm = ctypes.c_int64()
        self.op._torch_stream(keys.device).wait_stream(torch.cuda.current_stream(keys.device))
        rc = N.lib().fw_keyby_combine_push_device(self._c, combiner._h, self.op._h, keys.data_ptr(), ts.data_ptr(),
                                                  vals.data_ptr(), keys.numel(), int(local_wm), ctypes.byref(wm))
        N.check(rc, self.op._h)
        self.op._inflight = (keys, ts, vals)
        return wm.value

    def stats(self):
        """fw_comm_get_stats: the communicator's world / rank (ncclCommCount / ncclCommUserRank) and the exchange's
        counters (items and bytes to and from the other subtasks, receive-column reallocations) as a dict."""
        st = N.FwCommStats()
        N.check(N.lib().fw_comm_get_stats(self._c, ctypes.byref(st)))
        return {f: getattr(st, f) for f, _ in N.FwCommStats._fields_}

    def close(self):
        if self._c:
            N.lib().fw_comm_destroy(self._c)
            self._c = None

    def __del__(self):
        self.close()


class CombiningExchange:
    """Pre-shuffle combining in front of a KeyGroupExchange: the subtask's batch is aggregated by a
    combiner operator (a GpuWindowOperator of the same configuration over the whole key space, its watermark never
    advanced), drained into partial accumulators in key-group order (fw_combine_extract_device), and the partials
    -- one per (key, window) of the batch instead of one per record -- go to their subtasks, which merge them
    (fw_push_partials_device; AggregateFunction.merge, flink-core/.../AggregateFunction.java:160).  Results equal
    the uncombined exchange for the decomposable count/sum/min/max on tumbling windows without allowed lateness
    (float sums within the usual tolerance), on tumbling and on sliding windows kept as panes (a partial is a pane's);
    first-element, minBy/maxBy, HLL and t-digest aggregates do not combine."""

    def __init__(self, exchange: KeyGroupExchange, combiner):
        self.exchange = exchange
        self.combiner = combiner
        self.partials_sent = 0

    def push(self, op, keys, ts, vals, local_wm):
        """Combines, exchanges and merges one batch of this subtask; returns the combined watermark."""
        import torch
        import torch.distributed as dist
        ex = self.exchange
        self.combiner.process_batch(keys, ts, vals)
        if self.combiner.aggregate.aggregate_kind() == N.FW_AGG_HLL:
            return self._push_hll(op, keys, local_wm)
        cols, counts = self.combiner.combine_extract(ex.world)
        config = cols.config
        if ex.world > 1:
            staged = cols[0].is_cuda and dist.get_backend(ex.group) == "gloo"
            move = (lambda x: x.cpu()) if staged else (lambda x: x)
            back = (lambda x: x.to(keys.device)) if staged else (lambda x: x)
            send = move(torch.tensor(counts, dtype=torch.int64, device=cols[0].device))
            recv = torch.empty_like(send)
            dist.all_to_all_single(recv, send, group=ex.group)
            out_split = recv.tolist()
            total = sum(out_split)
            got = []
            for col in cols:
                col = move(col)
                r = torch.empty(total, dtype=col.dtype, device=col.device)
                dist.all_to_all_single(r, col, output_split_sizes=out_split, input_split_sizes=counts, group=ex.group)
                got.append(back(r))
            cols = tuple(got)
            self.partials_sent += sum(counts) - counts[ex.rank]
        else:  # the combiner reuses its output buffers; the operator reads the partials asynchronously
            cols = tuple(c.clone() for c in cols)
        op.push_partials(*cols, config=config)
        return ex.combine_watermark(local_wm, device=keys.device)

    def _push_hll(self, op, keys, local_wm):
        """HyperLogLog partials: the rows and, per destination, their registers (index << 8 | rank) cross the
        exchange; the receiver merges the counts and raises the registers (register max)."""
        import torch
        import torch.distributed as dist
        ex = self.exchange
        cols, counts, regs, rcounts = self.combiner.combine_extract_hll(ex.world)
        config = cols.config
        if ex.world > 1:
            staged = cols[0].is_cuda and dist.get_backend(ex.group) == "gloo"
            move = (lambda x: x.cpu()) if staged else (lambda x: x)
            back = (lambda x: x.to(keys.device)) if staged else (lambda x: x)

            def a2a(col, send_split):
                send = move(torch.tensor(send_split, dtype=torch.int64, device=keys.device))
                recv = torch.empty_like(send)
                dist.all_to_all_single(recv, send, group=ex.group)
                out_split = recv.tolist()
                col = move(col)
                r = torch.empty(sum(out_split), dtype=col.dtype, device=col.device)
                dist.all_to_all_single(r, col, output_split_sizes=out_split, input_split_sizes=send_split,
                                       group=ex.group)
                return back(r)
            cols = tuple(a2a(c, counts) for c in cols)
            regs = a2a(regs, rcounts)
            self.partials_sent += sum(counts) - counts[ex.rank]
            self.registers_sent = getattr(self, "registers_sent", 0) + sum(rcounts) - rcounts[ex.rank]
        else:  # the combiner reuses its output buffers; the operator reads the partials asynchronously
            cols = tuple(c.clone() for c in cols)
            regs = regs.clone()
        op.push_hll_partials(*cols, regs=regs, config=config)
        return ex.combine_watermark(local_wm, device=keys.device)
