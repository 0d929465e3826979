"""The kernel logic (bsf_core.h, sf_core.h, sam_core.h) compiled for the CPU as a standalone program
under AddressSanitizer + UndefinedBehaviorSanitizer (g++) and MemorySanitizer (clang++), on the host
suite's cases: every SAM must equal the oracle's and no sanitizer may report (the programs are
built with -fno-sanitize-recover, so the first report aborts the run).

These are the standing CPU checks for undefined behaviour in the device code:
out-of-range shifts, out-of-slice reads and writes, reads of uninitialised lane fields.  The
binaries take ~10 min to build, so the tests run when they are up to date (`make -C tests/hostcore
hc_asan hc_msan`) or with GWA_SANITIZE=1 (which builds them); otherwise they are skipped."""
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
HC = os.path.join(HERE, "hostcore")
sys.path.insert(0, HC)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))

import oracle as O  # noqa: E402
import synth  # noqa: E402

SANITIZERS = ["hc_asan", "hc_msan"]


def _binary(name):
    up_to_date = subprocess.call(["make", "-s", "-q", "-C", HC, name]) == 0
    if not up_to_date:
        if os.environ.get("GWA_SANITIZE") != "1":
            pytest.skip("%s not built or stale: make -C tests/hostcore %s (or GWA_SANITIZE=1)" % (name, name))
        subprocess.check_call(["make", "-s", "-C", HC, name])
    return os.path.join(HC, name)


def _write_genome(path, codes, names, lengths):
    with open(path, "wb") as f:
        f.write(("%d\n" % len(names)).encode())
        for n, L in zip(names, lengths):
            f.write(("%s %d\n" % (n, L)).encode())
        f.write(np.ascontiguousarray(codes, dtype=np.uint8).tobytes())


def _run(binary, genome, reads, k, rt=0, ns=1, strategy=0, env=None):
    """SAM text, or None where the program reports the batch failed as the reference would throw"""
    codes, names, lengths = genome
    with tempfile.TemporaryDirectory() as d:
        gp, rp = os.path.join(d, "g.bin"), os.path.join(d, "r.tsv")
        _write_genome(gp, codes, names, lengths)
        with open(rp, "w") as f:
            for n, s, q in reads:
                f.write("%s\t%s\t%s\n" % (n, s, q if q is not None else "*"))
        e = dict(os.environ)
        e.update({"ASAN_OPTIONS": "detect_leaks=0:abort_on_error=0:halt_on_error=1:verify_asan_link_order=0",
                  "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1",
                  "MSAN_OPTIONS": "halt_on_error=1", "OMP_NUM_THREADS": "2"})
        e.update(env or {})
        p = subprocess.run([binary, gp, rp, repr(float(k)), str(rt), str(ns), str(strategy)], capture_output=True,
                           env=e, timeout=1800)
    err = p.stderr.decode(errors="replace")
    for tag in ("Sanitizer", "runtime error"):
        assert tag not in err, err[-6000:]
    if p.returncode == 3:
        return None
    assert p.returncode == 0, (p.returncode, err[-4000:])
    return p.stdout.decode()


_ORACLE = {}


def _expect(genome, reads, k, rt=0, ns=1, strategy=0):
    codes, names, lengths = genome
    key = (len(codes), tuple(names), tuple(lengths), int(codes[:4096].sum()))
    if key not in _ORACLE:  # (one oracle index per genome: the long-read cases align read by read)
        _ORACLE[key] = O.Index.from_arrays(codes, names, lengths)
    oi = _ORACLE[key]
    try:
        return oi.align(reads, O.OrcConfig.default(k=k, report_type=rt, strategy=strategy, num_split=ns))
    except RuntimeError:
        return None


@pytest.fixture(scope="module")
def random_genome():
    return synth.genome([("c1", 120000), ("c2", 80000)], 1)


@pytest.fixture(scope="module")
def repetitive_genome():
    rng = np.random.default_rng(11)
    seg = rng.integers(0, 4, 3000).astype(np.uint8)
    parts = []
    for i in range(30):
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


def _mk(codes, n, m, sub, chim, seed, indels=False):
    rng = np.random.default_rng(seed)
    L = len(codes)
    out = []
    for i in range(n):
        if chim:
            a, b, cut = rng.integers(0, L - m), rng.integers(0, L - m), rng.integers(8, m - 8)
            s = np.concatenate([codes[a:a + cut], codes[b + cut:b + m]])
        else:
            a = rng.integers(0, L - m - 8)
            s = codes[a:a + m + 8].copy()
            if indels:
                for _ in range(rng.integers(0, 3)):
                    j = int(rng.integers(1, len(s) - 1))
                    s = np.delete(s, j) if rng.random() < 0.5 else np.insert(s, j, rng.integers(0, 4))
            s = s[:m].copy()
        for j in rng.integers(0, m, rng.integers(0, sub + 1)):
            if s[j] < 4:
                s[j] = (s[j] + rng.integers(1, 4)) % 4
        if rng.random() < 0.5:
            s = synth.COMP[s[::-1]]
        out.append(("q%05d" % i, synth.SYM[s].tobytes().decode(), "I" * m))
    return out


# (genome, m, k, substitutions, chimeric, indels, report type, -s, env)
CASES = {
    "bsf_rand_k2": ("rand", 100, 2.0, 2, False, False, 0, 1, {}),
    "bsf_rand_k01": ("rand", 100, 0.1, 4, False, False, 0, 1, {}),
    "bsf_indels150_k5": ("rand", 150, 5.0, 3, False, True, 0, 1, {}),
    "bsf_rep_chim": ("rep", 100, 2.0, 2, True, False, 0, 1, {}),
    "bsf_rep_allhits": ("rep", 100, 2.0, 2, False, False, 1, 1, {}),
    "bsf_rep_topl_s2": ("rep", 90, 0.1, 3, True, False, 2, 2, {}),
    "bsf_rep_s0": ("rep", 100, 0.1, 3, True, False, 0, 0, {}),
    "bsf_slice_fallback": ("rand", 150, 5.0, 3, False, True, 0, 1, {"GWA_TEST_SLICE_SHIFT": "40"}),
    "bsf_suspend_resume": ("rep", 100, 2.0, 2, True, False, 0, 1, {"HC_T0_ARENA": "24", "HC_T1_ARENA": "24"}),
    "bsf_rep_50": ("rep", 50, 0.1, 3, False, False, 0, 1, {}),
    "sf_rand_k2": ("rand", 100, 2.0, 2, False, False, 0, 1, {}),
    "sf_indels150_k5": ("rand", 150, 5.0, 3, False, True, 0, 1, {}),
    "sf_rep_chim": ("rep", 50, 0.1, 3, True, False, 0, 1, {}),
    "sf_rep_topl": ("rep", 100, 2.0, 2, False, False, 2, 1, {}),
    "sf_coop_rep": ("rep", 100, 2.0, 2, False, False, 0, 1, {"HC_SF_COOP": "1"}),
    "sf_coop_indels150": ("rand", 150, 5.0, 3, False, True, 0, 1, {"HC_SF_COOP": "1"}),
    "sf_coop_rep_allhits": ("rep", 100, 2.0, 2, False, False, 1, 1, {"HC_SF_COOP": "1"}),
}


@pytest.mark.parametrize("san", SANITIZERS)
@pytest.mark.parametrize("case", sorted(CASES))
def test_sanitized_hostcore_matches_oracle(san, case, random_genome, repetitive_genome):
    binary = _binary(san)
    g, m, k, sub, chim, indels, rt, ns, env = CASES[case]
    genome = random_genome if g == "rand" else repetitive_genome
    strategy = 1 if case.startswith("sf") else 0
    reads = _mk(genome[0], 60, m, sub, chim, seed=sum(map(ord, case)), indels=indels)
    if case == "bsf_rand_k2":  # N, empty, short and lowercase reads
        reads += [("n0", "N" * 100, None), ("short", "ACG", None), ("e0", "", None), ("low", reads[0][1].lower(), None)]
    exp = _expect(genome, reads, k, rt, ns, strategy)
    got = _run(binary, genome, reads, k, rt, ns, strategy, env)
    assert got == exp


# 257..512 bp reads (QW = 16) at the k's of test_hostcore.py::LONG_CASES, on the same 60 reads per case
# as tests/test_gpu_parity.py::test_long_reads_on_gpu -- including the -m sf 400 bp k = 0.06 case whose
# reads r19, r23 and r39 the GPU lost in round 5 (gpurun_out/j13/long_coop.log): the reads the oracle
# aligns as one batch (its SAM), and each read the reference throws on alone (the program must fail)
LONG = [(0, 300, 5.0), (0, 400, 2.0), (0, 512, 31.0), (1, 400, 0.06), (1, 400, 5.0), (1, 480, 5.0), (1, 333, 2.0)]


@pytest.mark.parametrize("san", SANITIZERS)
@pytest.mark.parametrize("strategy,m,k", LONG)
def test_sanitized_long_reads(san, strategy, m, k):
    binary = _binary(san)
    genome = synth.genome([("c1", 300000), ("c2", 200000)], 1)  # (test_gpu_parity.py random_pair)
    seqs, rn = synth.reads(genome[0], genome[2], 60, m, 3, config_id=4 + m)
    strs = synth.to_strings(seqs)
    good, bad = [], []
    for i, s in enumerate(strs):
        r = ("r%d" % i, s, "I" * m)
        (good if _expect(genome, [r], k, strategy=strategy) is not None else bad).append(r)
    assert good
    assert _run(binary, genome, good, k, strategy=strategy) == _expect(genome, good, k, strategy=strategy), (m, k)
    for r in bad[:1]:  # (the program fails where the reference throws; each run rebuilds the index)
        assert _run(binary, genome, [r], k, strategy=strategy) is None, (m, k, r[0])
