"""N>1 path on CPU: world-size-2 gloo ranks shard a read batch, align their shard, gather the SAM
to rank 0 and take the max elapsed time (genome-weaver-align_amd/dist.py).

The CPU oracle stands in for the per-rank GPU aligner here (tests may use it as the checker);
the merged SAM must be byte-identical to one unsharded run, as the reference emits in input order.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "genome-weaver-align_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tools")]

import dist  # noqa: E402


def test_shard_bounds_cover_exactly():
    for n in [0, 1, 7, 100, 1001]:
        for w in [1, 2, 3, 8]:
            spans = [dist.shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        dist.shard_bounds(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case():
    import synth
    codes, names, lengths = synth.genome([("chr1", 30000), ("chr2", 20000)], config_id=7)
    seqs, rn = synth.reads(codes, lengths, 120, 100, 2, config_id=5)
    strs = synth.to_strings(seqs)
    return codes, names, lengths, [(rn[i], strs[i], "I" * 100) for i in range(len(strs))]


def _rank_main(rank, world_size, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world_size))
    import time
    import torch.distributed as td
    import oracle as O
    td.init_process_group("gloo", rank=rank, world_size=world_size)
    codes, names, lengths, reads = _case()
    oi = O.Index.from_arrays(codes, names, lengths)
    lo, hi = dist.shard_bounds(len(reads), rank, world_size)
    t0 = time.perf_counter()
    sam = oi.align(reads[lo:hi], O.OrcConfig.default(k=2.0))
    dt = time.perf_counter() - t0 + 0.05 * rank  # ranks differ; the max must win
    mx = dist.max_over_ranks(dt)
    merged = dist.gather_sam(sam)
    # the tensor form (the GPU path gathers device buffers over RCCL; gloo here, on the CPU)
    import torch
    dev_merged = dist.gather_sam_device(torch.frombuffer(bytearray(sam.encode()), dtype=torch.uint8))
    if rank == 0:
        with open(os.path.join(outdir, "merged.sam"), "w") as f:
            f.write(merged)
        with open(os.path.join(outdir, "merged_tensor.sam"), "wb") as f:
            f.write(dev_merged.numpy().tobytes())
        with open(os.path.join(outdir, "max.txt"), "w") as f:
            f.write("%r %r" % (mx, dt))
    else:
        assert dev_merged is None
        with open(os.path.join(outdir, "rank1.txt"), "w") as f:
            f.write("%r %r" % (mx, dt))
    td.barrier()
    td.destroy_process_group()


def test_two_rank_shard_gather_equals_single(tmp_path):
    import oracle as O
    port = _free_port()
    mp.start_processes(_rank_main, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    codes, names, lengths, reads = _case()
    oi = O.Index.from_arrays(codes, names, lengths)
    single = oi.align(reads, O.OrcConfig.default(k=2.0))
    merged = open(tmp_path / "merged.sam").read()
    assert merged == single
    assert open(tmp_path / "merged_tensor.sam").read() == single
    m0, d0 = map(float, open(tmp_path / "max.txt").read().split())
    m1, d1 = map(float, open(tmp_path / "rank1.txt").read().split())
    assert m0 == m1 == max(d0, d1)


def _gather_main(rank, world_size, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world_size))
    import torch
    import torch.distributed as td
    td.init_process_group("gloo", rank=rank, world_size=world_size)
    # uneven texts, one rank with none: each rank sends its own bytes once, rank 0 merges in rank order
    text = b"" if rank == 1 else (b"rank%d line\n" % rank) * (1000 * (rank + 1))
    out = dist.gather_sam_device(torch.frombuffer(bytearray(text), dtype=torch.uint8) if text
                                 else torch.empty(0, dtype=torch.uint8))
    if rank == 0:
        with open(os.path.join(outdir, "g.bin"), "wb") as f:
            f.write(out.numpy().tobytes())
    else:
        assert out is None
    td.barrier()
    td.destroy_process_group()


def test_three_rank_point_to_point_gather(tmp_path):
    mp.start_processes(_gather_main, args=(3, _free_port(), str(tmp_path)), nprocs=3, join=True, start_method="spawn")
    exp = b"".join(b"" if r == 1 else (b"rank%d line\n" % r) * (1000 * (r + 1)) for r in range(3))
    assert (tmp_path / "g.bin").read_bytes() == exp
