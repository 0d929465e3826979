"""The kernel logic (bsf_core.h) compiled for the CPU, against the oracle: random and
repetitive references, substitutions/indels/N/chimeric reads, all report modes.  This is a
debugging harness for the device code (the GPU parity tests are tests/test_gpu_parity.py)."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "hostcore"))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))

import oracle as O  # noqa: E402
import synth  # noqa: E402
import hostcore  # noqa: E402


def _cmp(codes, names, lengths, reads, k, rt=0, strategy=0, num_split=1):
    oi = O.Index.from_arrays(codes, names, lengths)
    hc = hostcore.HostCore(codes, names, lengths)
    b = oi.align(reads, O.OrcConfig.default(k=k, report_type=rt, strategy=strategy, num_split=num_split))
    a = hc.align(reads, k=k, report_type=rt, strategy=strategy, num_split=num_split)
    assert a == b


@pytest.fixture(scope="module")
def random_genome():
    return synth.genome([("c1", 300000), ("c2", 200000)], 1)


@pytest.fixture(scope="module")
def repetitive_genome():
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
    return codes, ["chrA", "chrB", "chr10"], [L // 3, L // 3, L - 2 * (L // 3)]


def _mk(codes, n, m, sub, chim, seed):
    rng = np.random.default_rng(seed)
    L = len(codes)
    out = []
    for i in range(n):
        if chim:
            a, b, cut = rng.integers(0, L - m), rng.integers(0, L - m), rng.integers(8, m - 8)
            s = np.concatenate([codes[a:a + cut], codes[b + cut:b + m]])
        else:
            a = rng.integers(0, L - m)
            s = codes[a:a + m].copy()
        for j in rng.integers(0, m, rng.integers(0, sub + 1)):
            if s[j] < 4:
                s[j] = (s[j] + rng.integers(1, 4)) % 4
        if rng.random() < 0.5:
            s = synth.COMP[s[::-1]]
        out.append(("q%05d" % i, synth.SYM[s].tobytes().decode(), "I" * m))
    return out


@pytest.mark.parametrize("k", [2.0, 0.1, 0.0])
def test_random_genome_substitutions(random_genome, k):
    codes, names, lengths = random_genome
    seqs, rn = synth.reads(codes, lengths, 600, 100, 2)
    strs = synth.to_strings(seqs)
    _cmp(codes, names, lengths, [(rn[i], strs[i], "I" * 100) for i in range(len(strs))], k)


def test_random_genome_indels_150(random_genome):
    codes, names, lengths = random_genome
    seqs, rn = synth.reads(codes, lengths, 200, 150, config_id=4, indels=True, max_edits=5)
    strs = synth.to_strings(seqs)
    _cmp(codes, names, lengths, [(rn[i], strs[i], None) for i in range(len(strs))], 5.0)


@pytest.mark.parametrize("m,k,sub", [(100, 2.0, 2), (100, 0.1, 5), (150, 5.0, 5), (50, 0.1, 3), (36, 2.0, 2)])
@pytest.mark.parametrize("chim", [False, True])
def test_repetitive_genome(repetitive_genome, m, k, sub, chim):
    codes, names, lengths = repetitive_genome
    _cmp(codes, names, lengths, _mk(codes, 200, m, sub, chim, seed=m * 7 + int(chim)), k)


@pytest.mark.parametrize("rt", [1, 2])
def test_report_modes(repetitive_genome, rt):
    codes, names, lengths = repetitive_genome
    _cmp(codes, names, lengths, _mk(codes, 200, 100, 2, rt == 2, seed=99), 2.0, rt=rt)


def test_reads_with_n_and_unmappable(random_genome):
    codes, names, lengths = random_genome
    rng = np.random.default_rng(5)
    seqs, rn = synth.reads(codes, lengths, 200, 100, 2)
    strs = synth.to_strings(seqs)
    reads = []
    for i in range(200):
        s = list(strs[i])
        for j in rng.integers(0, 100, rng.integers(0, 4)):
            s[j] = "N"
        reads.append(("n%d" % i, "".join(s), "I" * 100))
    reads += [("x%d" % i, "".join(rng.choice(list("ACGT"), 100)), None) for i in range(100)]
    reads += [("e0", "", None), ("short", "ACG", None), ("lower", strs[0].lower(), None)]
    _cmp(codes, names, lengths, reads, 2.0)


@pytest.mark.parametrize("ns", [0, 2])
def test_num_split_other_than_one(repetitive_genome, ns):
    # -s 0 / -s 2: single-row text mode is exact for -s <= 1 only and is off at -s 2 (bsf_core.h nextSi)
    codes, names, lengths = repetitive_genome
    _cmp(codes, names, lengths, _mk(codes, 150, 100, 3, True, seed=40 + ns), 0.1, num_split=ns)


# ---- -m sf (S/SuffixFilter.java): sf_core.h on the CPU against the oracle's SuffixFilter ----

@pytest.mark.parametrize("k", [2.0, 0.1, 0.0])
def test_sf_random_genome(random_genome, k):
    codes, names, lengths = random_genome
    seqs, rn = synth.reads(codes, lengths, 400, 100, 2, config_id=21)
    strs = synth.to_strings(seqs)
    _cmp(codes, names, lengths, [(rn[i], strs[i], "I" * 100) for i in range(len(strs))], k, strategy=1)


def test_sf_indels_150(random_genome):
    codes, names, lengths = random_genome
    seqs, rn = synth.reads(codes, lengths, 150, 150, config_id=24, indels=True, max_edits=5)
    strs = synth.to_strings(seqs)
    _cmp(codes, names, lengths, [(rn[i], strs[i], None) for i in range(len(strs))], 5.0, strategy=1)


@pytest.mark.parametrize("m,k,sub", [(100, 2.0, 2), (50, 0.1, 3), (36, 2.0, 2)])
@pytest.mark.parametrize("chim", [False, True])
def test_sf_repetitive_genome(repetitive_genome, m, k, sub, chim):
    codes, names, lengths = repetitive_genome
    _cmp(codes, names, lengths, _mk(codes, 120, m, sub, chim, seed=m * 11 + int(chim)), k, strategy=1)


@pytest.mark.parametrize("case", ["indels150", "rep100", "rep50chim", "rep_rt2"])
def test_sf_cooperative_deferred_verification(random_genome, repetitive_genome, case, monkeypatch):
    """-m sf through the cooperative kernel's algorithm (search_kernels.h sf_search_kernel COOP, run
    by the GPU on the sparse last tier), here on every tier: the owner lane defers its verifications
    and goes on searching, 63 helper lanes run them in passes, the owner commits them in order and
    rolls the search back (undo log + register copy) when a result lowers minMismatches after
    later polls.  The SAM must equal the oracle's."""
    monkeypatch.setenv("HC_SF_COOP", "1")
    j0, p0, r0 = hostcore.spec_stats()
    if case == "indels150":
        codes, names, lengths = random_genome
        seqs, rn = synth.reads(codes, lengths, 150, 150, config_id=24, indels=True, max_edits=5)
        strs = synth.to_strings(seqs)
        _cmp(codes, names, lengths, [(rn[i], strs[i], None) for i in range(len(strs))], 5.0, strategy=1)
    else:
        codes, names, lengths = repetitive_genome
        m, sub, chim, rt = {"rep100": (100, 2, False, 0), "rep50chim": (50, 3, True, 0), "rep_rt2": (100, 2, False, 2)}[case]
        _cmp(codes, names, lengths, _mk(codes, 120, m, sub, chim, seed=m * 13 + int(chim)), 2.0, rt=rt, strategy=1)
    j1, p1, r1 = hostcore.spec_stats()
    print("helper verifications %d in %d passes, %d roll-backs" % (j1 - j0, p1 - p0, r1 - r0))
    assert j1 - j0 > 0 and p1 - p0 > 0


@pytest.mark.parametrize("rt", [1, 2])
def test_sf_report_modes(repetitive_genome, rt):
    codes, names, lengths = repetitive_genome
    _cmp(codes, names, lengths, _mk(codes, 120, 100, 2, False, seed=77), 2.0, rt=rt, strategy=1)


def test_sf_reads_with_n_and_unmappable(random_genome):
    codes, names, lengths = random_genome
    rng = np.random.default_rng(15)
    seqs, rn = synth.reads(codes, lengths, 120, 100, 2, config_id=25)
    strs = synth.to_strings(seqs)
    reads = []
    for i in range(120):
        s = list(strs[i])
        for j in rng.integers(0, 100, rng.integers(0, 4)):
            s[j] = "N"
        reads.append(("n%d" % i, "".join(s), "I" * 100))
    reads += [("x%d" % i, "".join(rng.choice(list("ACGT"), 100)), None) for i in range(40)]
    reads += [("short", "ACG", None), ("lower", strs[0].lower(), None)]
    _cmp(codes, names, lengths, reads, 2.0, strategy=1)
    # an empty read: StaircaseFilter(0, k + 1) throws in the reference (BitVector._not), both abort
    oi = O.Index.from_arrays(codes, names, lengths)
    with pytest.raises(RuntimeError):
        oi.align([("e0", "", None)], O.OrcConfig.default(k=2.0, strategy=1))
    with pytest.raises(RuntimeError):
        hostcore.HostCore(codes, names, lengths).align([("e0", "", None)], k=2.0, strategy=1)


@pytest.mark.parametrize("strategy", [0, 1])
def test_text_ends_and_word_boundaries(strategy):
    # reads at the very start / end of the text and straddling contig joins: the text-mode runs
    # (quick scan and search, 32 bases per compare) meet the text ends and the cyclic wrap there
    rng = np.random.default_rng(123)
    lengths = [97, 1500, 2301, 64]
    codes = rng.integers(0, 4, sum(lengths)).astype(np.uint8)
    names = ["c%d" % i for i in range(len(lengths))]
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
            reads.append(("e%d_%d" % (i, m), synth.SYM[s].tobytes().decode(), None))
    for k in (2.0, 0.1):
        _cmp(codes, names, lengths, reads, k, strategy=strategy)


# ---- more reported chains than a fixed output slot holds (OutSlots pool), 3-fragment chains ----

@pytest.mark.parametrize("strategy", [0, 1])
@pytest.mark.parametrize("rt", [1, 2])
def test_many_equal_hits(strategy, rt):
    import genomes
    codes, names, lengths, reads = genomes.many_hits()
    oi = O.Index.from_arrays(codes, names, lengths)
    exp = oi.align(reads, O.OrcConfig.default(k=5.0, report_type=rt, strategy=strategy))
    # some read reports more than 4 chains (allhits) / exactly -L 5 (topL)
    assert genomes.max_lines_per_read(exp) >= 5
    _cmp(codes, names, lengths, reads, 5.0, rt=rt, strategy=strategy)


def test_three_piece_chimeras_two_splits():
    # three-piece chimeras at -s 2: the reference keeps at most one split on these (XP has two
    # states); sam.cpp converts the head and its first split of any longer chain, as
    # R/AlignmentRecord.java:201-206 does, instead of failing the batch
    import genomes
    codes, names, lengths = synth.genome([("c1", 200000), ("c2", 100000)], 5)
    for m in (90, 120):
        reads = genomes.three_fragment_reads(codes, 200, m=m)
        _cmp(codes, names, lengths, reads, 5.0, num_split=2)


@pytest.mark.parametrize("strategy", [0, 1])
def test_dp_slice_fallback(random_genome, repetitive_genome, monkeypatch, strategy):
    """The first tier keeps a 32-row slice of the DP history around the read's diagonal; a traceback
    leaving it overflows the read into the next tier (whole columns).  With the slice moved off the
    diagonal every edit takes that path, and the SAM is unchanged."""
    monkeypatch.setenv("GWA_TEST_SLICE_SHIFT", "40")
    codes, names, lengths = random_genome
    seqs, rn = synth.reads(codes, lengths, 120, 150, config_id=4, indels=True, max_edits=5)
    strs = synth.to_strings(seqs)
    _cmp(codes, names, lengths, [(rn[i], strs[i], None) for i in range(len(strs))], 5.0, strategy=strategy)
    codes, names, lengths = repetitive_genome
    _cmp(codes, names, lengths, _mk(codes, 150, 100, 2, True, seed=5), 2.0, strategy=strategy)


def test_byte_parallel_to3bit_matches_acgt_table():
    # text_core.h to3bit4 (the encode kernels: four text bytes per word) against ACGT.to3bitCode
    # (A/ACGT.java:36-43) for every byte value in every byte lane
    import ctypes
    from hostcore import lib as hlib
    L = hlib()
    L.hc_to3bit4.restype = ctypes.c_uint32
    L.hc_to3bit4.argtypes = [ctypes.c_uint32]
    table = {ord(c): v for c, v in zip("AaCcGgTtUu", [0, 0, 1, 1, 2, 2, 3, 3, 3, 3])}
    for b in range(256):
        for lane in range(4):
            x = (b << (8 * lane)) | (ord("G") << (8 * ((lane + 1) % 4)))
            got = L.hc_to3bit4(x)
            assert (got >> (8 * lane)) & 0xFF == table.get(b, 4), (b, lane)
            assert (got >> (8 * ((lane + 1) % 4))) & 0xFF == 2


# ---- reads of 257..512 bp (QW = 16): read by read against the oracle, errors included ----

def _long_cases():
    codes, names, lengths = synth.genome([("chrA", 150000), ("chrB", 50000)], config_id=3)
    return codes, names, lengths


LONG_CASES = [(0, 257, 2.0), (0, 300, 5.0), (0, 333, 10.0), (0, 400, 2.0), (0, 480, 0.06), (0, 512, 31.0),
              (1, 300, 31.0), (1, 333, 2.0), (1, 400, 5.0), (1, 400, 0.06), (1, 480, 5.0), (1, 512, 2.0)]


@pytest.mark.parametrize("strategy,m,k", LONG_CASES)
def test_long_reads_read_by_read(strategy, m, k):
    """Above ~223 bp the reference's StaircaseFilter (byte) chunk starts wrap: some (m, minMismatches)
    filters throw in their constructor (the run aborts where the reference builds that filter), others
    give negative chunk starts and widths (-m sf seeds scanning nothing, staircase offsets outside
    [-k, m]).  Each read alone: the host core reports the oracle's SAM, or fails where the oracle
    throws."""
    codes, names, lengths = _long_cases()
    oi = O.Index.from_arrays(codes, names, lengths)
    hc = hostcore.HostCore(codes, names, lengths)
    seqs, rn = synth.reads(codes, lengths, 60, m, 3, config_id=4 + m)
    strs = synth.to_strings(seqs)
    errs = ok = 0
    for i, s in enumerate(strs):
        r = [("r%d" % i, s, "I" * m)]
        try:
            e = oi.align(r, O.OrcConfig.default(k=k, strategy=strategy))
        except RuntimeError:
            e = None
        try:
            g = hc.align(r, k=k, strategy=strategy)
        except RuntimeError:
            g = None
        assert g == e, (m, k, strategy, i)
        errs += e is None
        ok += e is not None
    assert ok > 0


def test_sf_wrap_instance_rule():
    """The -m sf kernel instance without the wrapped-offset staircase path is picked only for batches
    whose reads' prefix-scan chunks stay inside the read (sfChunksWrap false): the usual lengths
    (36-150 bp, k <= 10) do; reads of <= 31 bp at a large k and some 129-512 bp lengths do not, and
    their batches run the WRAP instance (launchSfSearchT)."""
    import ctypes
    L = hostcore.lib()
    L.hc_sf_chunks_wrap.restype = ctypes.c_int
    L.hc_sf_chunks_wrap.argtypes = [ctypes.c_int, ctypes.c_int]
    assert not any(L.hc_sf_chunks_wrap(m, k + 1) for m in (36, 50, 100, 128, 150) for k in range(0, 11))
    wraps = [(m, kk) for m in range(1, 129) for kk in range(1, 33) if L.hc_sf_chunks_wrap(m, kk)]
    assert wraps and max(m for m, _ in wraps) <= 31
    assert any(L.hc_sf_chunks_wrap(m, kk) for m in range(129, 257) for kk in range(1, 33))
    assert any(L.hc_sf_chunks_wrap(m, kk) for m in range(257, 513) for kk in range(1, 33))


# ---- suspend / resume across capacity tiers (BsfLane::suspendTo / resumeFrom) ----

@pytest.mark.parametrize("arena", [24, 48])
def test_suspend_resume_across_tiers(random_genome, repetitive_genome, monkeypatch, arena):
    """A read about to outgrow its tier is suspended between micro-steps (or before a report, which an
    overflow rolls back) and resumed on the next tier from its record instead of restarting from the
    seeds.  The first tier's kernel does not suspend (its overflows restart); with tiny first and
    second tiers most searches restart on the second and suspend there; the SAM and every read's
    FM-search and DP counts equal the oracle's, and equal a replay where every overflow restarts."""
    monkeypatch.setenv("HC_T0_ARENA", str(arena))
    monkeypatch.setenv("HC_T1_ARENA", str(arena))
    cases = []
    codes, names, lengths = random_genome
    seqs, rn = synth.reads(codes, lengths, 150, 150, config_id=4, indels=True, max_edits=5)
    strs = synth.to_strings(seqs)
    cases.append((random_genome, [(rn[i], strs[i], None) for i in range(len(strs))], 5.0))
    cases.append((repetitive_genome, _mk(repetitive_genome[0], 150, 100, 2, True, seed=9), 2.0))
    for (codes, names, lengths), reads, k in cases:
        oi = O.Index.from_arrays(codes, names, lengths)
        hc = hostcore.HostCore(codes, names, lengths)
        s0 = hostcore.suspends()
        got, st = hc.align(reads, k=k, stats=True)
        assert hostcore.suspends() - s0 >= 10
        exp, est = oi.align(reads, O.OrcConfig.default(k=k), with_stats=True)
        assert got == exp
        assert np.array_equal(st[:, 0], np.array([x.fm_searches for x in est]))
        monkeypatch.setenv("HC_NO_RESUME", "1")
        assert hc.align(reads, k=k) == got
        monkeypatch.delenv("HC_NO_RESUME")
