"""Every BASELINE.json config as a GPU parity test at its own scale.

- C2 / C4 on the FULL-SIZE hg19-like genome (here: tools/synth.genome_repeats at hg19 contig lengths,
  3.1 Gbp with N gaps, repeat families, satellites and segmental duplications) and on the full-size
  hg19 stand-in with N gaps (test_gpu_configs_hg19.py): a large batch runs
  on the GPU; the SAM of a random sample plus EVERY read that needed a search tier >= 1 is compared
  byte for byte with the oracle.  The oracle index takes the GPU suffix arrays only after the
  complete O(n) check of both (oracle/ orc_check_cyclic_sa_full: permutation + every adjacent pair),
  so no GPU SA entry is trusted unchecked.
- C3: two processes started by torch.multiprocessing (spawn) before they touch the GPU, each aligning
  its contiguous shard through libgwa on device rank % count; the merged SAM equals the oracle's.
- C1 (E. coli-size, exact) and C5 (paired-end) are in test_gpu_parity.py.
"""
import os
import socket
import sys
import time

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "tools"), os.path.join(REPO, "genome-weaver-align_amd"), os.path.join(REPO, "oracle")]

import oracle as O  # noqa: E402
import synth  # noqa: E402

pytestmark = pytest.mark.gpu


def _threads():
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(float(q) / float(per) + 0.5)))
    except (OSError, ValueError):
        pass
    return max(1, min(n, 16))


def _say(request, msg):
    """progress on the real terminal (a full-size fixture runs for minutes)"""
    capman = request.config.pluginmanager.getplugin("capturemanager")
    with capman.global_and_fixture_disabled():
        print("[configs] %s" % msg, flush=True)


def _compare(got, exp, what=""):
    if got != exp:
        g, e = got.splitlines(), exp.splitlines()
        bad = [(a, b) for a, b in zip(g, e) if a != b][:3]
        raise AssertionError("SAM differs%s: %d vs %d lines; first diffs: %r" % (what, len(g), len(e), bad))


@pytest.fixture(scope="module")
def hg19r_full(request):
    import gwa
    t0 = time.time()
    codes, names, lengths = synth.genome_repeats(synth.HG19_CONTIGS, config_id=1)
    _say(request, "hg19r genome %d bp generated in %.0fs" % (len(codes), time.time() - t0))
    t0 = time.time()
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths)
    _say(request, "GPU index built in %.0fs (%.1f GB)" % (time.time() - t0, gi.deviceBytes() / 1e9))
    t0 = time.time()
    T = _threads()
    sa_f = gi.suffixArray(0)
    O.check_cyclic_sa_full(codes, sa_f, threads=T)
    sa_r = gi.suffixArray(1)
    O.check_cyclic_sa_full(np.ascontiguousarray(codes[::-1]), sa_r, threads=T)
    _say(request, "both GPU suffix arrays pass the complete check in %.0fs" % (time.time() - t0))
    t0 = time.time()
    oi = O.Index.from_arrays(codes, names, lengths, sa_f=sa_f, sa_r=sa_r)
    del sa_f, sa_r
    _say(request, "oracle index in %.0fs" % (time.time() - t0))
    yield codes, names, lengths, gi, oi
    gi.close()


class _Heartbeat:
    """a line every 60 s while a long step runs (a silent GPU-box step is taken for a hang): appended
    to gpurun_out/heartbeat.log when that directory exists (pytest captures fd 2 during a test)"""

    def __init__(self, what):
        import threading
        self.what, self.t0, self.stop = what, time.time(), threading.Event()
        self.th = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        d = os.path.join(REPO, "gpurun_out")
        while not self.stop.wait(60):
            line = "[configs] ... %s %.0fs\n" % (self.what, time.time() - self.t0)
            if os.path.isdir(d):
                with open(os.path.join(d, "heartbeat.log"), "a") as f:
                    f.write(line)

    def __enter__(self):
        self.th.start()
        return self

    def __exit__(self, *a):
        self.stop.set()


def _batch_and_check(request, gi, oi, strs, m, k, strategy, n_random):
    """Run the whole batch on the GPU; compare a random sample plus every tier >= 1 read."""
    import gwa
    n = len(strs)
    reads = [("r%09d" % i, strs[i], "I" * m) for i in range(n)]
    cfg = gwa.AlignmentConfig(k=k, strategy=strategy)
    t0 = time.time()
    b = gwa.Batch(gi, cfg, reads)
    with _Heartbeat("GPU batch"):
        b.run()
    st = b.stats()
    c = b.read_counters()
    deep = np.nonzero(c[:, 12] >= 1)[0]
    rng = np.random.default_rng(17)
    samp = np.unique(np.concatenate([rng.choice(n, min(n_random, n), replace=False), deep])).astype(np.uint32)
    got, _ = b.results_select(samp)
    b.close()
    t1 = time.time()
    with _Heartbeat("oracle"):
        exp = oi.align([reads[i] for i in samp], O.OrcConfig.default(k=k, strategy=gwa.STRATEGIES[strategy]),
                       threads=_threads())
    _say(request, "%s k=%g m=%d: %d reads on the GPU (tiers %s, %.1fs), %d compared (%d from tiers >= 1) in %.1fs"
         % (strategy, k, m, n, list(st.tier_reads), t1 - t0, len(samp), len(deep), time.time() - t1))
    _compare(got, exp, " (compared: %d of %d reads = %d random + every tier >= 1 read, %d of them)"
             % (len(samp), n, min(n_random, n), len(deep)))
    return st, deep


@pytest.mark.timeout(900)
def test_c2_full_size_hg19r_k2(hg19r_full, request):
    """C2: 100 bp, 0-2 substitutions, -k 2, -m bsf, on the full-size hg19-like genome: 2M reads on
    the GPU, 200k random + every tier >= 1 read against the oracle."""
    codes, names, lengths, gi, oi = hg19r_full
    strs = synth.to_strings(synth.reads_codes(codes, lengths, 2_000_000, 100, 2, config_id=2))
    st, deep = _batch_and_check(request, gi, oi, strs, 100, 2.0, "bsf", 200_000)
    assert len(deep) > 1000  # the repeats send thousands of reads to the deeper tiers


@pytest.mark.timeout(900)
def test_c4_full_size_hg19r_indels_k5(hg19r_full, request):
    """C4: 150 bp, 0-5 edits (60 % substitutions, 20 % 1-bp insertions, 20 % 1-bp deletions), -k 5,
    -m bsf on the full-size hg19-like genome: 100k reads on the GPU, 50k random + every tier >= 1 read."""
    codes, names, lengths, gi, oi = hg19r_full
    strs = synth.to_strings(synth.reads_codes(codes, lengths, 100_000, 150, 2, config_id=4, indels=True,
                                              max_edits=5))
    _batch_and_check(request, gi, oi, strs, 150, 5.0, "bsf", 50_000)


@pytest.mark.timeout(900)
def test_c4_full_size_hg19r_indels_k5_sf(hg19r_full, request):
    """C4 with -m sf on the full-size hg19-like genome.  The reference's SuffixFilter loop has no
    search cap (S/SuffixFilter.java:257-290): on the full-size repeat families (1M Alu-like copies) a
    few reads in a thousand queue over 200k states at once and verify over 500k candidate positions
    (tools/diag_sf.py: 1.6M SFStates, 511k DP verifications for the heaviest of 2000; the oracle needs
    7 s for it on one core).  Such reads reach the grown last tier, run by the cooperative kernel
    (search_kernels.h sf_search_kernel COOP: lane 0 searches, deferring its verifications; lanes 1-63
    run them in passes of 63; a roll-back when a result would lower minMismatches) -- round 5 took
    the 2000-read batch from 228 s to ~60 s on the GPU.  4000 reads of the C4 stream on the GPU;
    3000 random + every tier >= 1 read compared byte for byte with the oracle (16 threads); both
    times are printed."""
    codes, names, lengths, gi, oi = hg19r_full
    strs = synth.to_strings(synth.reads_codes(codes, lengths, 4000, 150, 2, config_id=4, indels=True, max_edits=5))
    st, deep = _batch_and_check(request, gi, oi, strs, 150, 5.0, "sf", 3000)
    assert st.tier_reads[3] > 0 and len(deep) > 200


# ---- C3: reads sharded over processes, one index replica per process ----

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _c3_case():
    codes, names, lengths = synth.genome_ngaps([(n, L) for n, L in synth.HG19_CONTIGS], config_id=3, scale=0.002)
    strs = synth.to_strings(synth.reads_codes(codes, lengths, 30_000, 100, 2, config_id=3))
    return codes, names, lengths, [("r%09d" % i, s, "I" * 100) for i, s in enumerate(strs)]


def _c3_rank(rank, world_size, port, outdir):
    # a fresh interpreter (spawn): nothing has touched the GPU in this process yet
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world_size),
                      LOCAL_RANK=str(rank))
    sys.path[:0] = [os.path.join(REPO, "tools"), os.path.join(REPO, "genome-weaver-align_amd")]
    import torch.distributed as td
    import dist
    import gwa
    td.init_process_group("gloo", rank=rank, world_size=world_size)
    codes, names, lengths, reads = _c3_case()
    dev = dist.device_for(rank, gwa.lib().gwa_device_count())
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths, device=dev)
    lo, hi = dist.shard_bounds(len(reads), rank, world_size)
    sam = gwa.BidirectionalSuffixFilter(gi, gwa.AlignmentConfig(k=2.0)).align_batch(reads[lo:hi])
    merged = dist.gather_sam(sam)
    if rank == 0:
        with open(os.path.join(outdir, "merged.sam"), "w") as f:
            f.write(merged)
    with open(os.path.join(outdir, "rank%d.txt" % rank), "w") as f:
        f.write("%d %d %d %d\n" % (dev, lo, hi, len(sam.splitlines())))
    gi.close()
    td.barrier()
    td.destroy_process_group()


@pytest.mark.timeout(600)
def test_c3_two_processes_shard_through_libgwa(tmp_path):
    """C3-shaped: 2 processes (torch.multiprocessing spawn), each with its own index replica on GPU
    rank % count, align contiguous shards through libgwa; the SAM gathered to rank 0 in rank order
    equals the oracle's SAM of the whole batch."""
    import torch.multiprocessing as mp
    mp.start_processes(_c3_rank, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    codes, names, lengths, reads = _c3_case()
    exp = O.Index.from_arrays(codes, names, lengths).align(reads, O.OrcConfig.default(k=2.0), threads=_threads())
    got = open(tmp_path / "merged.sam").read()
    _compare(got, exp)
    spans = [tuple(map(int, open(tmp_path / ("rank%d.txt" % r)).read().split())) for r in range(2)]
    assert spans[0][1] == 0 and spans[0][2] == spans[1][1] and spans[1][2] == len(reads)
    assert spans[0][3] + spans[1][3] == len(exp.splitlines())
