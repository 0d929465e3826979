"""GPU parity: the HIP path through the C-ABI against the CPU oracle (bit-exact SAM text), plus
size-independent properties of the GPU-built index.  Needs an MI355X (`-m gpu`)."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
sys.path.insert(0, HERE)

import oracle as O  # noqa: E402
import synth  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gwa():
    import gwa as g
    return g


def _both(codes, names, lengths):
    import gwa
    return gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths), O.Index.from_arrays(codes, names, lengths)


def _check(gi, oi, reads, **cfg):
    import gwa
    c = gwa.AlignmentConfig(**cfg)
    got = gwa.aligner(gi, c).align_batch(reads)
    rt = {"besthit": 0, "allhits": 1, "topl": 2}[c.reportType.lower()]
    exp = oi.align(reads, O.OrcConfig.default(k=float(c.k), report_type=rt, strategy=gwa.STRATEGIES[c.strategy],
                                              num_split=c.numSplitAlowed))
    if got != exp:
        g, e = got.splitlines(), exp.splitlines()
        bad = [(a, b) for a, b in zip(g, e) if a != b][:3]
        raise AssertionError("SAM differs: %d vs %d lines; first diffs: %r" % (len(g), len(e), bad))
    return got


@pytest.fixture(scope="module")
def random_pair():
    codes, names, lengths = synth.genome([("c1", 300000), ("c2", 200000)], 1)
    gi, oi = _both(codes, names, lengths)
    return codes, names, lengths, gi, oi


def test_known_answers_on_gpu(gwa):
    import json
    G = json.load(open(os.path.join(HERE, "golden", "reference_known_answers.json")))
    gi = gwa.FMIndexOnGenome.buildFromSequence("seq", G["bsf"]["reference"])
    oi = O.Index.from_sequence("seq", G["bsf"]["reference"])
    reads = [("read", c["query"], None) for c in G["bsf"]["cases"]]
    _check(gi, oi, reads, k=2.0)
    # BWAlignTest.align3 (CLI-built index of test2.fa, default k)
    fa = open(os.path.join(HERE, "golden", "fixtures", "test2.fa")).read()
    gi2 = gwa.FMIndexOnGenome.buildFromFasta(fa)
    sam = gwa.BidirectionalSuffixFilter(gi2).align_batch([("read", "TAAAGTAT", None)])
    f = sam.split("\t")
    assert (f[1], f[2], f[3]) == ("82", "seq2", "9")
    assert gi2.samHeader() == "@SQ\tSN:seq1\tLN:27\n@SQ\tSN:seq2\tLN:28\n"


def test_gpu_index_sa_matches_oracle(random_pair):
    codes, names, lengths, gi, oi = random_pair
    for s in (0, 1):
        assert np.array_equal(gi.suffixArray(s).astype(np.int64), oi.sa(s))


@pytest.mark.parametrize("k", [2.0, 0.1, 0.0])
def test_random_substitutions(random_pair, k):
    codes, names, lengths, gi, oi = random_pair
    seqs, rn = synth.reads(codes, lengths, 3000, 100, 2)
    strs = synth.to_strings(seqs)
    _check(gi, oi, [(rn[i], strs[i], "I" * 100) for i in range(len(strs))], k=k)


def test_indels_150_k5(random_pair):
    codes, names, lengths, gi, oi = random_pair
    seqs, rn = synth.reads(codes, lengths, 500, 150, config_id=4, indels=True, max_edits=5)
    strs = synth.to_strings(seqs)
    _check(gi, oi, [(rn[i], strs[i], "I" * 150) for i in range(len(strs))], k=5.0)


@pytest.fixture(scope="module")
def repetitive_pair():
    from test_hostcore import repetitive_genome as rg  # noqa
    rng = np.random.default_rng(11)
    seg = rng.integers(0, 4, 3000).astype(np.uint8)
    parts = []
    for i in range(40):
        s = seg.copy()
        mut = rng.integers(0, 3000, rng.integers(0, 60))
        s[mut] = rng.integers(0, 4, len(mut))
        parts.append(s)
        parts.append(rng.integers(0, 4, rng.integers(10, 2000)).astype(np.uint8))
        if i % 7 == 0:
            parts.append(np.full(rng.integers(1, 50), 4, np.uint8))
        if i % 5 == 0:
            parts.append(np.tile(rng.integers(0, 4, rng.integers(1, 6)).astype(np.uint8), 40))
    codes = np.concatenate(parts)
    L = len(codes)
    names, lengths = ["chrA", "chrB", "chr10"], [L // 3, L // 3, L - 2 * (L // 3)]
    gi, oi = _both(codes, names, lengths)
    return codes, gi, oi


@pytest.mark.parametrize("m,k,sub", [(100, 2.0, 2), (100, 0.1, 5), (150, 5.0, 5), (50, 0.1, 3)])
@pytest.mark.parametrize("chim", [False, True])
def test_repetitive(repetitive_pair, m, k, sub, chim):
    from test_hostcore import _mk
    codes, gi, oi = repetitive_pair
    _check(gi, oi, _mk(codes, 400, m, sub, chim, seed=m * 7 + int(chim)), k=k)


@pytest.mark.parametrize("rt", ["allhits", "topl"])
def test_report_modes(repetitive_pair, rt):
    from test_hostcore import _mk
    codes, gi, oi = repetitive_pair
    _check(gi, oi, _mk(codes, 300, 100, 2, rt == "topl", seed=99), k=2.0, reportType=rt)


def test_edge_reads(random_pair):
    codes, names, lengths, gi, oi = random_pair
    rng = np.random.default_rng(5)
    seqs, rn = synth.reads(codes, lengths, 300, 100, 2)
    strs = synth.to_strings(seqs)
    reads = []
    for i in range(300):
        s = list(strs[i])
        for j in rng.integers(0, 100, rng.integers(0, 4)):
            s[j] = "N"
        reads.append(("n%d" % i, "".join(s), "I" * 100))
    reads += [("x%d" % i, "".join(rng.choice(list("ACGT"), 100)), None) for i in range(100)]
    reads += [("short", "ACG", None), ("lower", strs[0].lower(), None), ("u", strs[1].replace("T", "U"), None)]
    # reads with and without a quality in one batch (FASTA reads have none: QUAL "*", per read)
    _check(gi, oi, reads, k=2.0)
    _check(gi, oi, [(a, b, c if c else "I" * len(b)) for a, b, c in reads], k=2.0)
    _check(gi, oi, [(a, b, None) for a, b, c in reads], k=2.0)


from test_hostcore import LONG_CASES  # noqa: E402


@pytest.mark.parametrize("strategy,m,k", LONG_CASES)
def test_long_reads_on_gpu(random_pair, gwa, strategy, m, k):
    """Reads of 257..512 bp (QW = 16 kernels).  Above ~223 bp the reference's StaircaseFilter (byte)
    chunk starts wrap and some reads make it throw: the reads the oracle aligns give its SAM as one
    batch; a batch holding a read the oracle throws on fails as the reference's run aborts; a read
    over 512 bp fails the batch at creation, with the limit in the message."""
    codes, names, lengths, gi, oi = random_pair
    seqs, rn = synth.reads(codes, lengths, 60, m, 3, config_id=4 + m)
    strs = synth.to_strings(seqs)
    strat = ["bsf", "sf"][strategy]
    good, bad = [], []
    for i, s_ in enumerate(strs):
        r = ("r%d" % i, s_, "I" * m)
        try:
            oi.align([r], O.OrcConfig.default(k=k, strategy=strategy))
            good.append(r)
        except RuntimeError:
            bad.append(r)
    assert good
    _check(gi, oi, good, k=k, strategy=strat)
    if bad:
        with pytest.raises(gwa.GwaError, match="reference would abort"):
            gwa.aligner(gi, gwa.AlignmentConfig(k=k, strategy=strat)).align_batch(good[:3] + bad[:1])
    with pytest.raises(gwa.GwaError, match="512"):
        gwa.aligner(gi, gwa.AlignmentConfig(k=k, strategy=strat)).align_batch([good[0], ("long", strs[0] * 2 + "A", None)])


def test_reads_up_to_256_bp(random_pair):
    """200 and 256 bp reads (QW = 8) align as the oracle does."""
    codes, names, lengths, gi, oi = random_pair
    for m in (200, 256):
        seqs, rn = synth.reads(codes, lengths, 60, m, 2, config_id=7)
        strs = synth.to_strings(seqs)
        reads = []
        for i, s_ in enumerate(strs):
            try:
                oi.align([(rn[i], s_, None)], O.OrcConfig.default(k=2.0))
                reads.append((rn[i], s_, None))
            except RuntimeError:
                pass
        _check(gi, oi, reads, k=2.0)


def test_ecoli_c1_exact(gwa):
    """Config 1: E. coli-size index, 10k exact 100 bp reads (-k 0)."""
    codes, names, lengths = synth.genome(synth.ECOLI, 1)
    gi, oi = _both(codes, names, lengths)
    seqs, rn = synth.reads(codes, lengths, 10000, 100, 0, config_id=1)
    strs = synth.to_strings(seqs)
    reads = [(rn[i], strs[i], "I" * 100) for i in range(len(strs))]
    sam = _check(gi, oi, reads, k=0.0)
    assert all(l.split("\t")[1] in ("66", "82") for l in sam.splitlines())


@pytest.mark.parametrize("ns", [0, 2])
def test_num_split_other_than_one(repetitive_pair, ns):
    # single-row text mode is off at -s 2 (exact for -s <= 1 only)
    from test_hostcore import _mk
    codes, gi, oi = repetitive_pair
    _check(gi, oi, _mk(codes, 300, 100, 3, True, seed=50 + ns), k=0.1, numSplitAlowed=ns)


# ---- -m sf (S/SuffixFilter.java) ----

@pytest.mark.parametrize("k", [2.0, 0.1, 0.0])
def test_sf_random_substitutions(random_pair, k):
    codes, names, lengths, gi, oi = random_pair
    seqs, rn = synth.reads(codes, lengths, 3000, 100, 2, config_id=21)
    strs = synth.to_strings(seqs)
    _check(gi, oi, [(rn[i], strs[i], "I" * 100) for i in range(len(strs))], k=k, strategy="sf")


def test_sf_indels_150_k5(random_pair):
    codes, names, lengths, gi, oi = random_pair
    seqs, rn = synth.reads(codes, lengths, 500, 150, config_id=24, indels=True, max_edits=5)
    strs = synth.to_strings(seqs)
    _check(gi, oi, [(rn[i], strs[i], "I" * 150) for i in range(len(strs))], k=5.0, strategy="sf")


@pytest.mark.parametrize("m,k,sub", [(100, 2.0, 2), (50, 0.1, 3)])
@pytest.mark.parametrize("chim", [False, True])
def test_sf_repetitive(repetitive_pair, m, k, sub, chim):
    from test_hostcore import _mk
    codes, gi, oi = repetitive_pair
    _check(gi, oi, _mk(codes, 300, m, sub, chim, seed=m * 11 + int(chim)), k=k, strategy="sf")


@pytest.mark.parametrize("rt", ["allhits", "topl"])
def test_sf_report_modes(repetitive_pair, rt):
    from test_hostcore import _mk
    codes, gi, oi = repetitive_pair
    _check(gi, oi, _mk(codes, 300, 100, 2, False, seed=77), k=2.0, reportType=rt, strategy="sf")


def test_sf_edge_reads(random_pair):
    codes, names, lengths, gi, oi = random_pair
    rng = np.random.default_rng(15)
    seqs, rn = synth.reads(codes, lengths, 300, 100, 2, config_id=25)
    strs = synth.to_strings(seqs)
    reads = []
    for i in range(300):
        s = list(strs[i])
        for j in rng.integers(0, 100, rng.integers(0, 4)):
            s[j] = "N"
        reads.append(("n%d" % i, "".join(s), "I" * 100))
    reads += [("x%d" % i, "".join(rng.choice(list("ACGT"), 100)), "I" * 100) for i in range(100)]
    reads += [("short", "ACG", "III"), ("lower", strs[0].lower(), "I" * 100), ("noqual", strs[2], None)]
    _check(gi, oi, reads, k=2.0, strategy="sf")


@pytest.mark.parametrize("k", [6.0, 12.0])
def test_sf_short_reads_large_k(random_pair, k):
    """Reads of 8-31 bp at a large k: their prefix-scan chunks wrap or run past the read
    (sfChunksWrap), so the batch runs the -m sf instance with the wrapped-offset staircase path;
    compared with the oracle (errors and unmapped reads included), and the same reads with -m bsf."""
    codes, names, lengths, gi, oi = random_pair
    rng = np.random.default_rng(int(k) + 40)
    L = len(codes)
    reads = []
    for i in range(400):
        m = int(rng.integers(8, 32))
        a = int(rng.integers(0, L - m))
        s = codes[a:a + m].copy()
        for j in rng.integers(0, m, rng.integers(0, 3)):
            s[j] = (s[j] + 1) % 4 if s[j] < 4 else s[j]
        reads.append(("s%d" % i, synth.SYM[s].tobytes().decode(), None))
    _check(gi, oi, reads, k=k, strategy="sf")
    _check(gi, oi, reads, k=k, strategy="bsf")


def test_sf_known_answer_queries_on_gpu(gwa):
    # the two SuffixFilterTest queries (T/strategy/SuffixFilterTest.java:67-76) on sample3.fa
    fa = open(os.path.join(HERE, "golden", "fixtures", "sample3.fa")).read()
    gi, oi = gwa.FMIndexOnGenome.buildFromFasta(fa), O.Index.from_fasta(fa)
    reads = [("exact", "CACTTTAGTATAATTGTTTTTAGTTTTTGGCAAAACTATTGTCTAAACAG", None),
             ("insertion", "CACTTTAGTATAATTGTTTTTAGCCTTTTTGGCAAAACTATTGTCTAAACAG", None)]
    _check(gi, oi, reads, strategy="sf")


@pytest.mark.parametrize("strategy", ["bsf", "sf"])
def test_text_ends_and_word_boundaries_on_gpu(gwa, strategy):
    # reads at the very start / end of the text and across contig joins, where the 32-base text
    # compares (quick scan, search run-ahead) meet the text ends and the cyclic wrap
    rng = np.random.default_rng(123)
    lengths = [97, 1500, 2301, 64]
    codes = rng.integers(0, 4, sum(lengths)).astype(np.uint8)
    names = ["c%d" % i for i in range(len(lengths))]
    gi, oi = _both(codes, names, lengths)
    L = len(codes)
    reads = []
    for i, a in enumerate(list(range(0, 40)) + list(range(L - 140, L - 60)) + [95, 1590, 3890, L - 100]):
        for m in (36, 60, 100):
            if a + m > L:
                continue
            s = codes[a:a + m].copy()
            for j in rng.integers(0, m, rng.integers(0, 3)):
                s[j] = (s[j] + rng.integers(1, 4)) % 4
            if rng.random() < 0.5:
                s = synth.COMP[s[::-1]]
            reads.append(("e%d_%d" % (i, m), synth.SYM[s].tobytes().decode(), "I" * m))
    for k in (2.0, 0.1):
        _check(gi, oi, reads, k=k, strategy=strategy)


# ---- more reported chains than a read's fixed output slot (OutSlots pool) ----

@pytest.fixture(scope="module")
def many_hits_pair():
    import genomes
    codes, names, lengths, reads = genomes.many_hits()
    gi, oi = _both(codes, names, lengths)
    return gi, oi, reads


@pytest.mark.parametrize("strategy", ["bsf", "sf"])
@pytest.mark.parametrize("rt", ["allhits", "topl"])
def test_many_equal_hits_on_gpu(many_hits_pair, strategy, rt):
    import genomes
    gi, oi, reads = many_hits_pair
    sam = _check(gi, oi, reads, k=5.0, reportType=rt, strategy=strategy)
    assert genomes.max_lines_per_read(sam) >= 5


@pytest.mark.parametrize("stage", ["1024", "4096"])
def test_sam_writer_direct_write_fallback(many_hits_pair, random_pair, monkeypatch, stage):
    # samWriteKernel stages a workgroup's 64 records in LDS and writes them out in 16-B chunks; a
    # workgroup whose records do not fit writes them directly, next to staged neighbours that write
    # the shared edge chunks bytewise.  A small staging buffer (GWA_SAM_STAGE) sends the many-hit reads'
    # workgroups (hundreds of lines) and, at 1024 B, every workgroup down the direct path: same bytes
    gi, oi, reads = many_hits_pair
    monkeypatch.setenv("GWA_SAM_STAGE", stage)
    _check(gi, oi, reads, k=5.0, reportType="allhits")
    codes, names, lengths, gi2, oi2 = random_pair
    seqs, rn = synth.reads(codes, lengths, 700, 100, 2, config_id=31)
    strs = synth.to_strings(seqs)
    mix = [(rn[i], strs[i][: 10 + (i * 37) % 91], None if i % 3 else "I" * (10 + (i * 37) % 91)) for i in range(700)]
    _check(gi2, oi2, mix, k=2.0)


def test_output_pool_growth(many_hits_pair, monkeypatch):
    # a 4-hit initial pool: the reads that overflow it are rerun after the pool grows
    gi, oi, reads = many_hits_pair
    monkeypatch.setenv("GWA_OUT_POOL", "4")
    _check(gi, oi, reads, k=5.0, reportType="allhits")


def test_three_piece_chimeras_two_splits_on_gpu(random_pair):
    import genomes
    codes, names, lengths, gi, oi = random_pair
    for m in (90, 120):
        _check(gi, oi, genomes.three_fragment_reads(codes, 200, m=m), k=5.0, numSplitAlowed=2)


def test_pipeline_two_handles_in_memory(random_pair):
    # gwa_pipeline_align over two index replicas on GPU 0: batches dealt to both, merged in order
    import gwa
    codes, names, lengths, gi, oi = random_pair
    gi2 = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths)
    seqs, rn = synth.reads(codes, lengths, 5000, 100, 2, config_id=31)
    strs = synth.to_strings(seqs)
    reads = [(rn[i], strs[i], "I" * 100) for i in range(len(strs))]
    pipe = gwa.Pipeline([gi, gi2], gwa.AlignmentConfig(k=2.0), batch_reads=333)
    got = pipe.align_batch(reads)
    st = pipe.stats()
    pipe.close()
    gi2.close()
    assert got == oi.align(reads, O.OrcConfig.default(k=2.0))
    assert st.batches == (5000 + 332) // 333 and st.reads == 5000
    assert st.device_kernel_s[0] > 0 and st.device_kernel_s[1] > 0


def test_sam_device_copy_matches_results(random_pair):
    # gwa_batch_sam_copy: the SAM text gwa_batch_format wrote in HBM, copied device to device into a
    # torch buffer (the source of dist.gather_sam_device), equals the host results
    import gwa
    codes, names, lengths, gi, oi = random_pair
    seqs, rn = synth.reads(codes, lengths, 1500, 100, 2, config_id=33)
    strs = synth.to_strings(seqs)
    reads = [(rn[i], strs[i], "I" * 100) for i in range(len(strs))]
    b = gwa.Batch(gi, gwa.AlignmentConfig(k=2.0), reads)
    b.run()
    n = b.format_device()
    t = b.sam_device()
    sam, _ = b.results()
    b.close()
    assert t.numel() == n and t.cpu().numpy().tobytes().decode() == sam == oi.align(reads, O.OrcConfig.default(k=2.0))


def test_per_read_counters_match_oracle_stats(random_pair):
    # numFMIndexSearches, FMQuickScan steps and DP verifications per read, device vs the oracle's
    # instrumented restatement (the oracle defines the algorithmic counts)
    import gwa
    codes, names, lengths, gi, oi = random_pair
    seqs, rn = synth.reads(codes, lengths, 2000, 100, 2, config_id=32)
    strs = synth.to_strings(seqs)
    reads = [(rn[i], strs[i], "I" * 100) for i in range(len(strs))]
    b = gwa.Batch(gi, gwa.AlignmentConfig(k=2.0), reads)
    b.run()
    c = b.read_counters()
    b.close()
    _, st = oi.align(reads, O.OrcConfig.default(k=2.0), with_stats=True)
    fm = np.array([x.fm_searches for x in st])
    # the device's FMQuickScan stops at the (k+1)-th mismatch (only numMismatches <= k is consumed)
    qs = np.array([x.quick_steps_cut for x in st])
    assert (qs <= np.array([x.quick_steps for x in st])).all()
    sw = np.array([x.sw for x in st])
    assert np.array_equal(c[:, 1], fm), np.nonzero(c[:, 1] != fm)[0][:5]
    assert np.array_equal(c[:, 2], qs), np.nonzero(c[:, 2] != qs)[0][:5]
    assert np.array_equal(c[:, 16], sw), np.nonzero(c[:, 16] != sw)[0][:5]


# ---- hg19-like repetitive genome (tools/synth.genome_repeats): N gaps, repeat families, satellites,
# segmental duplications at 0.5 % of hg19 size ----

@pytest.fixture(scope="module")
def hg19r_pair():
    import gwa
    codes, names, lengths = synth.genome_repeats(synth.HG19_CONTIGS, config_id=1, scale=0.005)
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths)
    # the oracle index takes the GPU suffix arrays after the complete independent check of them
    # (permutation + every adjacent pair, orc_check_cyclic_sa_full)
    sa_f, sa_r = gi.suffixArray(0), gi.suffixArray(1)
    O.check_cyclic_sa_full(codes, sa_f)
    O.check_cyclic_sa_full(np.ascontiguousarray(codes[::-1]), sa_r)
    oi = O.Index.from_arrays(codes, names, lengths, sa_f=sa_f, sa_r=sa_r)
    return codes, lengths, gi, oi


@pytest.mark.parametrize("strategy", ["bsf", "sf"])
def test_hg19r_c2_k2(hg19r_pair, strategy):
    codes, lengths, gi, oi = hg19r_pair
    strs = synth.to_strings(synth.reads_codes(codes, lengths, 4000, 100, 2, config_id=2))
    sam = _check(gi, oi, [("r%d" % i, strs[i], "I" * 100) for i in range(len(strs))], k=2.0, strategy=strategy)
    # repeats make multi-hit (X0 > 1) records common
    assert sum(1 for l in sam.splitlines() if "\tX0:i:1" not in l) > 50


@pytest.mark.parametrize("strategy", ["bsf", "sf"])
def test_hg19r_c4_indels_k5(hg19r_pair, strategy):
    codes, lengths, gi, oi = hg19r_pair
    strs = synth.to_strings(synth.reads_codes(codes, lengths, 600, 150, 2, config_id=4, indels=True, max_edits=5))
    _check(gi, oi, [("r%d" % i, strs[i], "I" * 150) for i in range(len(strs))], k=5.0, strategy=strategy)


def test_hg19r_allhits(hg19r_pair):
    codes, lengths, gi, oi = hg19r_pair
    strs = synth.to_strings(synth.reads_codes(codes, lengths, 1500, 100, 2, config_id=6))
    _check(gi, oi, [("r%d" % i, strs[i], "I" * 100) for i in range(len(strs))], k=2.0, reportType="allhits")


def _to_sam_line(text, names, r, split=None, has_segments=None, is_first=True, each_mapped=True):
    """AlignmentRecord.toSAMLine (R/AlignmentRecord.java:109-170) from gwa_record_t fields -- what a
    JVM binding does with the objects it builds from the records."""
    s = lambda off, n: text[off:off + n]
    if has_segments is None:
        has_segments = split is not None
    flag = 0x1 if has_segments else 0
    if r.strand == 1:
        flag |= 0x10
    if is_first:
        flag |= 0x40
        if r.x0 <= 0 or (split is not None and split.x0 <= 0):
            each_mapped = False
    elif split is None:
        flag |= 0x80
    if each_mapped:
        flag |= 0x2
    if r.x0 <= 0:
        flag |= 0x4
    if split is not None and split.x0 <= 0:
        flag |= 0x8
    chr_ = "*" if r.ref < 0 else names[r.ref]
    cols = [s(r.name_off, r.name_len), str(flag), chr_, str(r.pos), "1", s(r.cigar_off, r.cigar_len)]
    if split is None:
        cols += ["*", "0", "0"]
    else:
        sc = "*" if split.ref < 0 else names[split.ref]
        cols += ["=" if chr_ != "*" and chr_ == sc else sc, str(split.pos), str(split.end - r.pos)]
    cols += [s(r.seq_off, r.seq_len), "*" if r.qual_null else s(r.qual_off, r.qual_len)]
    if r.x0 > 0:
        if r.nm >= 0:
            cols.append("NM:i:%d" % r.nm)
        cols += ["XP:Z:" + s(r.state_off, r.state_len), "X0:i:%d" % r.x0]
    line = "\t".join(cols)
    if split is not None:
        line += "\n" + _to_sam_line(text, names, split, None, has_segments, False, each_mapped)
    return line


def test_results_records_rebuild_the_sam(repetitive_pair):
    # gwa_results_records: the AlignmentRecord fields of every line; rebuilding each top-level record
    # with toSAMLine gives the SAM text back (chimeric reads -> split records, unmapped reads)
    import gwa
    from test_hostcore import _mk
    codes, gi, oi = repetitive_pair
    rng = np.random.default_rng(72)
    reads = _mk(codes, 400, 100, 3, True, seed=71) + [("x%d" % i, "".join(rng.choice(list("ACGT"), 100)), "I" * 100)
                                                       for i in range(20)]
    b = gwa.Batch(gi, gwa.AlignmentConfig(k=0.1), reads)
    b.run()
    sam, recs = b.records(gi)
    b.close()
    names = ["chrA", "chrB", "chr10"]
    assert len(recs) == len(sam.splitlines())
    assert any(r.split >= 0 for r in recs) and any(r.ref < 0 for r in recs)
    rebuilt = [_to_sam_line(sam, names, r, recs[r.split] if r.split >= 0 else None) for r in recs if not r.is_split]
    assert "\n".join(rebuilt) + "\n" == sam


# ---- paired-end (config C5; the build's own pairing, checked against the oracle's restatement) ----

def _pairs(codes, lengths, n, seed):
    m1, m2 = synth.pairs_codes(codes, lengths, n, config_id=seed)
    s1, s2 = synth.to_strings(m1), synth.to_strings(m2)
    return ([("p%d/1" % i, s1[i], "I" * 100) for i in range(n)], [("p%d/2" % i, s2[i], "J" * 100) for i in range(n)])


@pytest.mark.parametrize("genome", ["random", "repetitive"])
def test_paired_end_matches_oracle(random_pair, repetitive_pair, genome):
    import gwa
    if genome == "random":
        codes, names, lengths, gi, oi = random_pair
    else:
        codes, gi, oi = repetitive_pair
        lengths = [len(codes) // 3, len(codes) // 3, len(codes) - 2 * (len(codes) // 3)]
    r1, r2 = _pairs(codes, lengths, 2000, 51)
    got = gwa.PairedEndAligner(gi, gwa.AlignmentConfig(k=2.0)).align_pairs(r1, r2)
    exp = oi.align_pairs(r1, r2, O.OrcConfig.default(k=2.0))
    assert got == exp
    flags = [int(l.split("\t")[1]) for l in got.splitlines()]
    # proper pairs: most on the random genome; on the repetitive one a multi-hit mate reports one position
    assert len(flags) == 4000 and sum(1 for f in flags if f & 0x2) > (3000 if genome == "random" else 1000)


def test_paired_end_insert_window_and_unmapped_mates(random_pair):
    import gwa
    codes, names, lengths, gi, oi = random_pair
    r1, r2 = _pairs(codes, lengths, 500, 52)
    rng = np.random.default_rng(53)
    # some mates unmappable, a narrow insert window (most pairs fail it)
    r2 = [(n, "".join(rng.choice(list("ACGT"), 100)) if i % 7 == 0 else s, q) for i, (n, s, q) in enumerate(r2)]
    got = gwa.PairedEndAligner(gi, gwa.AlignmentConfig(k=2.0), 295, 305).align_pairs(r1, r2)
    assert got == oi.align_pairs(r1, r2, O.OrcConfig.default(k=2.0), 295, 305)
    # mate 2 without qualities (a FASTA mate file) and single mate-1 reads without one
    r1q = [(n, s, None if i % 5 == 0 else q) for i, (n, s, q) in enumerate(r1)]
    r2q = [(n, s, None) for n, s, q in r2]
    got = gwa.PairedEndAligner(gi, gwa.AlignmentConfig(k=2.0)).align_pairs(r1q, r2q)
    assert got == oi.align_pairs(r1q, r2q, O.OrcConfig.default(k=2.0))


def test_paired_end_mate_rescue_matches_oracle(random_pair):
    """Rule 3 (mate rescue, pair_rescue_kernel): one mate carries 3-8 substitutions (or N runs),
    beyond what -k 2 lets the search find; the DP inside the insert window beside the other mate
    (window <= 320 bp, <= max(k, m/10) differences) rescues it.  Either mate may be the damaged one,
    fragments sit at contig edges (clipped windows) and some are too damaged to rescue."""
    import gwa
    codes, names, lengths, gi, oi = random_pair
    rng = np.random.default_rng(57)
    starts = np.concatenate([[0], np.cumsum(lengths)])
    r1, r2 = [], []
    for i in range(1500):
        c = int(rng.integers(0, len(lengths)))
        ins = int(rng.integers(260, 340))
        if i % 50 == 0:
            s = int(starts[c])  # fragment at the contig's left end
        elif i % 50 == 1:
            s = int(starts[c + 1]) - ins  # ... and at its right end
        else:
            s = int(starts[c] + rng.integers(0, lengths[c] - ins))
        frag = codes[s:s + ins]
        m1, m2 = frag[:100].copy(), synth.COMP[frag[ins - 100:][::-1]].copy()
        if i % 3 == 1:
            m1, m2 = m2, m1  # mate 1 on the reverse strand
        bad = m2 if i % 4 else m1
        nsub = int(rng.integers(3, 13)) if i % 11 else 0
        for p in rng.choice(100, nsub, replace=False):
            bad[p] = (bad[p] + int(rng.integers(1, 4))) % 4
        if i % 13 == 0:
            bad[40:43] = 4
        q2 = None if i % 6 == 0 else "J" * 100
        r1.append(("p%d/1" % i, synth.SYM[m1].tobytes().decode(), "I" * 100))
        r2.append(("p%d/2" % i, synth.SYM[m2].tobytes().decode(), q2))
    got = gwa.PairedEndAligner(gi, gwa.AlignmentConfig(k=2.0)).align_pairs(r1, r2)
    exp = oi.align_pairs(r1, r2, O.OrcConfig.default(k=2.0))
    if got != exp:
        g, e = got.splitlines(), exp.splitlines()
        bad = [(a, b) for a, b in zip(g, e) if a != b][:3]
        raise AssertionError("SAM differs: %d vs %d lines; first diffs: %r" % (len(g), len(e), bad))
    flags = [int(l.split("\t")[1]) for l in got.splitlines()]
    assert sum(1 for f in flags if f & 0x2) > 2000  # most damaged mates are rescued into proper pairs


def _frag_pairs(codes, n, seed, subs, ins=(150, 300)):
    """pairs from fragments anywhere in `codes` (both orientations), each mate with 0..subs substitutions"""
    rng = np.random.default_rng(seed)
    r1, r2 = [], []
    for i in range(n):
        L = int(rng.integers(ins[0], ins[1] + 1))
        s = int(rng.integers(0, len(codes) - L))
        frag = codes[s:s + L]
        m1, m2 = frag[:100].copy(), synth.COMP[frag[L - 100:][::-1]].copy()
        for m in (m1, m2):
            for p in rng.choice(100, int(rng.integers(0, subs + 1)), replace=False):
                m[p] = (m[p] + int(rng.integers(1, 4))) % 4
        if i % 2:
            m1, m2 = m2, m1
        r1.append(("f%d/1" % i, synth.SYM[m1].tobytes().decode(), "I" * 100))
        r2.append(("f%d/2" % i, synth.SYM[m2].tobytes().decode(), "J" * 100))
    return r1, r2


def _blobs(reads):
    out = []
    for f in range(3):
        parts = [x[f].encode() for x in reads]
        out += [b"".join(parts), np.concatenate([[0], np.cumsum([len(x) for x in parts])]).astype(np.uint64)]
    return tuple(out)


@pytest.mark.parametrize("mode", ["sweep", "spread"])
def test_paired_end_sorted_sweep_choice(random_pair, repetitive_pair, monkeypatch, mode):
    """Rules 1-2 (fewest differences, ties by mate-1 then mate-2 report order) through
    pair_choose_kernel: GWA_PAIR_QUAD=0 sends every pair whose mates both have candidates to the
    LDS-sorted sliding-window sweep ("sweep"); GWA_PAIR_SORT_CAP=1 to its all-pairs loop spread over
    the workgroup ("spread").  Genomes: random, repetitive, and the many-equal-hits one (200 copies of
    a 300-base segment; -k 5 gives several candidates per mate), insert windows tight to unbounded."""
    import gwa
    import genomes
    monkeypatch.setenv("GWA_PAIR_QUAD", "0")
    if mode == "spread":
        monkeypatch.setenv("GWA_PAIR_SORT_CAP", "1")
    mh_codes, mh_names, mh_lengths, _ = genomes.many_hits()
    mh_gi, mh_oi = _both(mh_codes, mh_names, mh_lengths)
    rep_codes, rep_gi, rep_oi = repetitive_pair
    codes, names, lengths, gi, oi = random_pair
    cases = [(gi, oi, _frag_pairs(codes, 600, 63, 2), 2.0), (rep_gi, rep_oi, _frag_pairs(rep_codes, 600, 64, 2), 2.0),
             (mh_gi, mh_oi, _frag_pairs(mh_codes, 600, 65, 3), 5.0)]
    heavy = 0
    for g, o, (r1, r2), k in cases:
        for lo, hi in ((210, 390), (250, 260), (1, 1 << 20), (0, 200)):
            got = gwa.PairedEndAligner(g, gwa.AlignmentConfig(k=k), lo, hi).align_pairs(r1, r2)
            exp = o.align_pairs(r1, r2, O.OrcConfig.default(k=k), lo, hi)
            if got != exp:
                gl, el = got.splitlines(), exp.splitlines()
                bad = [(x, y) for x, y in zip(gl, el) if x != y][:3]
                raise AssertionError("k %g insert [%d, %d]: SAM differs: first diffs %r" % (k, lo, hi, bad))
        b = gwa.Batch(g, gwa.AlignmentConfig(k=k), pair_blobs=(_blobs(r1), _blobs(r2)))
        b.run()
        heavy += b.stats().heavy_pairs
        b.close()
    assert heavy > 1000
    mh_gi.close()


def test_results_records_of_a_paired_batch(random_pair):
    # gwa_results_records on paired-end results: two mate lines per pair, each its own record (no
    # split linking: FLAG 0x41 / 0x81 are mates here, not a split record pair)
    import gwa
    codes, names, lengths, gi, oi = random_pair
    m1, m2 = synth.pairs_codes(codes, lengths, 300, config_id=54)
    off = np.arange(0, 100 * 301, 100, dtype=np.uint64)
    nb, no = synth.name_blob(300)
    s1, s2 = synth.SYM[m1].tobytes(), synth.SYM[m2].tobytes()
    b = gwa.Batch(gi, gwa.AlignmentConfig(k=2.0), pair_blobs=((nb, no, s1, off, b"I" * 30000, off),
                                                              (nb, no, s2, off, b"J" * 30000, off)))
    b.run()
    sam, recs = b.records(gi)
    b.close()
    lines = sam.splitlines()
    assert len(recs) == len(lines) == 600
    assert all(r.split == -1 and r.is_split == 0 for r in recs)
    assert [r.read for r in recs] == [i // 2 for i in range(600)]
    assert all((r.flag & 0x40) if i % 2 == 0 else (r.flag & 0x80) for i, r in enumerate(recs))
    for r, line in zip(recs, lines):
        f = line.split("\t")
        assert r.pos == int(f[3]) and r.flag == int(f[1])


def test_gpu_cyclic_sa_known_answers(gwa):
    # the GPU suffix-array builder on CyclicSAISTest's texts (T/sais/CyclicSAISTest.java:45-90),
    # relabelled order-preservingly to the index alphabet
    import json
    from test_oracle_golden import _relabel
    G = json.load(open(os.path.join(HERE, "golden", "reference_known_answers.json")))
    for case in G["cyclic_sa"]:
        codes = np.array(_relabel(case["text"]), dtype=np.uint8)
        gi = gwa.FMIndexOnGenome.buildFromCodes(codes, ["t"], [len(codes)])
        assert list(gi.suffixArray(0)) == case["expect"], case["name"]
        gi.close()


@pytest.mark.parametrize("strat,k", [("bsf", 2.0), ("bsf", 4.0), ("sf", 4.0)])
def test_search_order_and_refill_do_not_change_results(random_pair, monkeypatch, strat, k):
    # round 6: the first-tier search list sorted by quick-scan key (radix sort) and the wavefront-wide
    # refill threshold only reorder work; with both off (GWA_SEARCH_SORT=0, GWA_REFILL=1: input
    # order, a lane refilled as soon as it empties) the SAM text is byte-identical and equals the oracle
    import gwa
    codes, names, lengths, gi, oi = random_pair
    seqs, rn = synth.reads(codes, lengths, 3000, 100, int(k) + 1, config_id=61)
    strs = synth.to_strings(seqs)
    reads = [(rn[i], strs[i], "I" * 100) for i in range(len(strs))]
    cfg = gwa.AlignmentConfig(k=k, strategy=strat)
    sam_default = gwa.aligner(gi, cfg).align_batch(reads)
    monkeypatch.setenv("GWA_SEARCH_SORT", "0")
    monkeypatch.setenv("GWA_REFILL", "1")
    sam_plain = gwa.aligner(gi, cfg).align_batch(reads)
    assert sam_default == sam_plain
    assert sam_default == oi.align(reads, O.OrcConfig.default(k=k, strategy=["bsf", "sf"].index(strat)))


@pytest.mark.parametrize("strat,arena", [("bsf", "64"), ("sf", None)])
def test_concurrent_batches_small_scratch_budget(random_pair, monkeypatch, strat, arena):
    # batches of several host threads size their search scratch at the same time.
    # Under a small budget (GWA_SCRATCH_BUDGET_MB), and for -m bsf with a small first-tier arena so that
    # reads overflow into the deep tiers, three concurrent batches all finish and equal the oracle.
    import threading
    import gwa
    codes, names, lengths, gi, oi = random_pair
    monkeypatch.setenv("GWA_SCRATCH_BUDGET_MB", "256")
    if arena:
        monkeypatch.setenv("GWA_TIER_ARENA", arena)
    cfg = gwa.AlignmentConfig(k=4.0, strategy=strat)
    batches = []
    for j in range(3):
        seqs, rn = synth.reads(codes, lengths, 1500, 100, 5, config_id=70 + j)
        strs = synth.to_strings(seqs)
        batches.append([("b%d_%s" % (j, rn[i]), strs[i], "I" * 100) for i in range(len(strs))])
    got, deep, errs = [None] * 3, [0] * 3, []

    def work(j):
        try:
            b = gwa.Batch(gi, cfg, batches[j])
            b.run()
            deep[j] = sum(list(b.stats().tier_reads)[1:])
            got[j] = b.results()[0]
            b.close()
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(repr(e))
    th = [threading.Thread(target=work, args=(j,)) for j in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs
    if arena:
        assert min(deep) > 0, deep  # every batch ran deep tiers
    for j in range(3):
        assert got[j] == oi.align(batches[j], O.OrcConfig.default(k=4.0, strategy=["bsf", "sf"].index(strat)))
