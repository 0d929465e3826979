"""Read sharding across GPUs of one node: replicas only, no data-path collective.

Every rank holds a full index replica in its own HBM and aligns a contiguous shard of the read
batch; the only communication is (i) the max-over-ranks elapsed time for the benchmark and
(ii) an optional gather of SAM text to rank 0, concatenated in rank order so the merged output
is byte-identical to a single-GPU run (the reference emits in input order, A/Align.java:187-195).
Works with any torch.distributed backend (gloo on CPU in tests, nccl=RCCL on the GPU box).
"""
import os


def world():
    """(rank, world_size, local_rank) from the torchrun environment; (0, 1, 0) standalone."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_bounds(n, rank, world_size):
    """Contiguous shard [lo, hi) of n reads for `rank`; shard sizes differ by at most one."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError("bad rank %d / world %d" % (rank, world_size))
    q, r = divmod(n, world_size)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def max_over_ranks(value):
    """Max of a float over all ranks (the benchmark's step time); identity when not distributed."""
    import torch
    import torch.distributed as td
    if not (td.is_available() and td.is_initialized()) or td.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64)
    td.all_reduce(t, op=td.ReduceOp.MAX)
    return float(t[0])


def all_gather_floats(value):
    """[value of rank 0, value of rank 1, ...] on every rank; [value] when not distributed."""
    import torch
    import torch.distributed as td
    if not (td.is_available() and td.is_initialized()) or td.get_world_size() == 1:
        return [float(value)]
    out = [torch.zeros(1, dtype=torch.float64) for _ in range(td.get_world_size())]
    td.all_gather(out, torch.tensor([float(value)], dtype=torch.float64))
    return [float(t[0]) for t in out]


def device_for(local_rank, n_devices):
    """GPU ordinal of a local rank: ranks beyond the node's GPU count share GPUs round-robin (so a
    2-rank run works on a 1-GPU box, each rank holding its own index replica)."""
    if n_devices < 1:
        raise RuntimeError("no GPU visible")
    return local_rank % n_devices


def gather_sam(sam_text, dst=0):
    """Gather each rank's SAM text to `dst`, concatenated in rank order (None on other ranks)."""
    import torch.distributed as td
    if not (td.is_available() and td.is_initialized()) or td.get_world_size() == 1:
        return sam_text
    parts = [None] * td.get_world_size() if td.get_rank() == dst else None
    td.gather_object(sam_text, parts, dst=dst)
    return "".join(parts) if td.get_rank() == dst else None


def gather_sam_device(sam, dst=0):
    """Gather each rank's SAM text held in a uint8 tensor (on the GPU with the nccl backend = RCCL over
    xGMI, or on the CPU with gloo) to `dst`, concatenated in rank order = input order.  One all-gather
    of the lengths (8 bytes per rank), then every other rank sends its text once, point to point, into
    its slice of the merged buffer on `dst`, all receives posted together (`batch_isend_irecv`): each text crosses the fabric once and no rank but `dst`
    holds more than its own (an all-gather of padded texts would move N x the data into every rank).
    Returns the merged uint8 tensor on `dst`, None on the other ranks; the tensor itself without
    torch.distributed."""
    import torch
    import torch.distributed as td
    if not (td.is_available() and td.is_initialized()) or td.get_world_size() == 1:
        return sam
    w, me = td.get_world_size(), td.get_rank()
    sam = sam.contiguous().view(-1)
    n = torch.tensor([sam.numel()], dtype=torch.int64, device=sam.device)
    lens = [torch.zeros_like(n) for _ in range(w)]
    td.all_gather(lens, n)
    lens = [int(x.item()) for x in lens]
    if me != dst:
        if lens[me]:
            for req in td.batch_isend_irecv([td.P2POp(td.isend, sam, dst)]):
                req.wait()
        return None
    out = torch.empty(sum(lens), dtype=torch.uint8, device=sam.device)
    # every receive posted at once (one batch): under RCCL the texts of up to 7 peers arrive over
    # their own xGMI links concurrently instead of one link at a time
    ops, off = [], 0
    for r, ln in enumerate(lens):
        if r == dst:
            out[off:off + ln].copy_(sam)
        elif ln:
            ops.append(td.P2POp(td.irecv, out[off:off + ln], r))
        off += ln
    if ops:
        for req in td.batch_isend_irecv(ops):
            req.wait()
    return out
