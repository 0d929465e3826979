"""C2 and C4 (-m bsf and -m sf) on the full-size BASELINE stand-in genome: hg19 contig lengths,
i.i.d. ACGT with hg19-like N-gap runs (tools/synth.genome_ngaps, what bench.py measures).  As in
test_gpu_configs.py: a large batch on the GPU, a random sample plus every read that needed a search
tier >= 1 compared byte for byte with the oracle, whose index takes the GPU suffix arrays only after
the complete O(n) check of both."""
import os
import sys
import time

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from test_gpu_configs import O, _batch_and_check, _say, _threads, synth  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hg19_full(request):
    import gwa
    t0 = time.time()
    codes, names, lengths = synth.genome_ngaps(synth.HG19_CONTIGS, config_id=1)
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths)
    _say(request, "hg19 (N gaps) genome + GPU index in %.0fs" % (time.time() - t0))
    t0 = time.time()
    T = _threads()
    sa_f = gi.suffixArray(0)
    O.check_cyclic_sa_full(codes, sa_f, threads=T)
    sa_r = gi.suffixArray(1)
    O.check_cyclic_sa_full(np.ascontiguousarray(codes[::-1]), sa_r, threads=T)
    oi = O.Index.from_arrays(codes, names, lengths, sa_f=sa_f, sa_r=sa_r)
    del sa_f, sa_r
    _say(request, "complete SA check + oracle index in %.0fs" % (time.time() - t0))
    yield codes, names, lengths, gi, oi
    gi.close()


@pytest.mark.timeout(900)
def test_c2_full_size_hg19_k2(hg19_full, request):
    """C2: 100 bp, 0-2 substitutions, -k 2, -m bsf: 2M reads, 200k random + every tier >= 1 read."""
    codes, names, lengths, gi, oi = hg19_full
    strs = synth.to_strings(synth.reads_codes(codes, lengths, 2_000_000, 100, 2, config_id=2))
    _batch_and_check(request, gi, oi, strs, 100, 2.0, "bsf", 200_000)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("strategy", ["bsf", "sf"])
def test_c4_full_size_hg19_indels_k5(hg19_full, request, strategy):
    """C4: 150 bp, 0-5 edits with 1-bp indels, -k 5: 100k reads, 50k random + every tier >= 1 read."""
    codes, names, lengths, gi, oi = hg19_full
    strs = synth.to_strings(synth.reads_codes(codes, lengths, 100_000, 150, 2, config_id=4, indels=True,
                                              max_edits=5))
    _batch_and_check(request, gi, oi, strs, 150, 5.0, strategy, 50_000)


def _oracle_pairs(oi, t1, t2, cfg):
    """orc_align_pairs over chunks on the host threads (ctypes releases the GIL), in pair order"""
    from concurrent.futures import ThreadPoolExecutor
    T = _threads()
    step = max(1, (len(t1) + T - 1) // T)
    chunks = [(a, min(a + step, len(t1))) for a in range(0, len(t1), step)]
    with ThreadPoolExecutor(T) as ex:
        parts = list(ex.map(lambda c: oi.align_pairs(t1[c[0]:c[1]], t2[c[0]:c[1]], cfg), chunks))
    return "".join(parts)


@pytest.mark.timeout(900)
def test_c5_full_size_hg19_pairs(hg19_full, request):
    """C5: 2x100 bp pairs (insert ~ N(300, 30), 0-2 substitutions per mate), -k 2, on the full-size hg19
    stand-in: 1M pairs on the GPU; 20k random pairs plus EVERY pair with a mate without candidates (mate
    rescue) or with several candidates (pair choice among them) compared with orc_align_pairs byte for
    byte.  (The pairing rules are this build's own: the reference has no paired-end path.)"""
    import gwa
    codes, names, lengths, gi, oi = hg19_full
    pairs, m = 1_000_000, 100
    m1, m2 = synth.pairs_codes(codes, lengths, pairs, m, config_id=5)
    s1, s2 = synth.SYM[m1].tobytes(), synth.SYM[m2].tobytes()
    del m1, m2
    off = np.arange(0, m * (pairs + 1), m, dtype=np.uint64)
    nb, no = synth.name_blob(pairs)
    q1, q2 = b"I" * (m * pairs), b"J" * (m * pairs)
    t0 = time.time()
    b = gwa.Batch(gi, gwa.AlignmentConfig(k=2.0), pair_blobs=((nb, no, s1, off, q1, off), (nb, no, s2, off, q2, off)))
    b.run()
    c = b.read_counters()
    h1, h2 = c[:pairs, 7].astype(np.int64), c[pairs:, 7].astype(np.int64)
    special = np.nonzero((h1 == 0) | (h2 == 0) | (h1 > 1) | (h2 > 1))[0]
    rng = np.random.default_rng(23)
    samp = np.unique(np.concatenate([rng.choice(pairs, 20_000, replace=False), special])).astype(np.uint32)
    got, _ = b.results_select(samp)
    st = b.stats()
    b.close()
    t1 = time.time()
    tp1 = [(nb[10 * i:10 * i + 10].decode(), s1[m * i:m * i + m].decode(), "I" * m) for i in samp]
    tp2 = [(nb[10 * i:10 * i + 10].decode(), s2[m * i:m * i + m].decode(), "J" * m) for i in samp]
    exp = _oracle_pairs(oi, tp1, tp2, O.OrcConfig.default(k=2.0))
    _say(request, "C5: %d pairs on the GPU (%.1fs, heavy %d), %d compared (%d with a candidate-less or multi-candidate "
         "mate) in %.1fs" % (pairs, t1 - t0, st.heavy_pairs, len(samp), len(special), time.time() - t1))
    assert len(special) > 100
    from test_gpu_configs import _compare
    _compare(got, exp)


# ---- C3 at full size: two processes, one full index replica each, contiguous shards ----

def _c3_full_rank(rank, world_size, port, outdir, n_reads):
    # a fresh interpreter (spawn): nothing has touched the GPU in this process yet
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world_size),
                      LOCAL_RANK=str(rank))
    sys.path[:0] = [os.path.join(os.path.dirname(HERE), "tools"), os.path.join(os.path.dirname(HERE), "genome-weaver-align_amd")]
    import torch
    import torch.distributed as td
    import dist
    import gwa
    import synth as S
    td.init_process_group("gloo", rank=rank, world_size=world_size)
    codes, names, lengths = S.genome_ngaps(S.HG19_CONTIGS, config_id=1)
    dev = dist.device_for(rank, gwa.lib().gwa_device_count())
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths, device=dev)
    lo, hi = dist.shard_bounds(n_reads, rank, world_size)
    strs = S.to_strings(S.reads_codes(codes, lengths, n_reads, 100, 2, config_id=2))[lo:hi]
    del codes
    b = gwa.Batch(gi, gwa.AlignmentConfig(k=2.0), [("r%09d" % (lo + i), s, "I" * 100) for i, s in enumerate(strs)])
    b.run()
    b.format_device()
    mine = b.sam_device().cpu()  # gloo moves host tensors; RCCL would move the device tensor itself
    b.close()
    gi.close()
    merged = dist.gather_sam_device(mine)
    if rank == 0:
        with open(os.path.join(outdir, "merged.sam"), "wb") as f:
            f.write(merged.numpy().tobytes())
    with open(os.path.join(outdir, "rank%d.txt" % rank), "w") as f:
        f.write("%d %d %d %d\n" % (dev, lo, hi, int(mine.numel())))
    td.barrier()
    td.destroy_process_group()


@pytest.mark.timeout(900)
def test_c3_full_size_two_processes(hg19_full, request, tmp_path):
    """C3-shaped at full size: two processes (spawned before they touch the GPU), each building its own
    full hg19-size index replica (33 GB of HBM each) and aligning a contiguous shard of 2M C2 reads
    through libgwa; the SAM texts are gathered to rank 0 in rank order (dist.gather_sam_device: one
    point-to-point send per rank).  The merged SAM equals a one-process run over all reads byte for
    byte, and a 20k-read sample equals the oracle's."""
    import socket
    import gwa
    import torch.multiprocessing as mp
    codes, names, lengths, gi, oi = hg19_full
    n = 2_000_000
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    t0 = time.time()
    mp.start_processes(_c3_full_rank, args=(2, port, str(tmp_path), n), nprocs=2, join=True, start_method="spawn")
    _say(request, "C3: two full-size replicas aligned their shards in %.0fs" % (time.time() - t0))
    merged = (tmp_path / "merged.sam").read_bytes().decode()
    spans = [tuple(map(int, open(tmp_path / ("rank%d.txt" % r)).read().split())) for r in range(2)]
    assert spans[0][1] == 0 and spans[0][2] == spans[1][1] and spans[1][2] == n
    assert spans[0][3] + spans[1][3] == len(merged)
    strs = synth.to_strings(synth.reads_codes(codes, lengths, n, 100, 2, config_id=2))
    reads = [("r%09d" % i, strs[i], "I" * 100) for i in range(n)]
    b = gwa.Batch(gi, gwa.AlignmentConfig(k=2.0), reads)
    b.run()
    one, _ = b.results()
    b.close()
    assert merged == one
    lines = merged.splitlines(True)
    assert len(lines) == n  # besthit: one line per read (no split chains among these reads)
    samp = np.sort(np.random.default_rng(29).choice(n, 20_000, replace=False))
    exp = oi.align([reads[i] for i in samp], O.OrcConfig.default(k=2.0), threads=_threads())
    assert "".join(lines[i] for i in samp) == exp
