"""Small synthetic references and reads for the report-mode and split-chain edge cases (test data,
shared by the CPU hostcore tests and the GPU parity tests)."""
import numpy as np

import synth


def many_hits(n_reads=1000, seed=21):
    """A genome of 200 copies of one 300-base segment (each copy with up to 4 substitutions) between
    random spacers, and 100-base reads from it with up to 5 substitutions: at -k 5 (or 0.1) the
    best-first search keeps several equal-score hits for some reads (up to 8 here), so -R allhits /
    topL report more chains than a fixed output slot holds.  Returns (codes, names, lengths, reads)."""
    from test_hostcore import _mk
    rng = np.random.default_rng(seed)
    seg = rng.integers(0, 4, 300).astype(np.uint8)
    parts = []
    for i in range(200):
        s = seg.copy()
        mut = rng.integers(0, 300, rng.integers(0, 5))
        s[mut] = (s[mut] + rng.integers(1, 4, len(mut))) % 4
        parts.append(s)
        parts.append(rng.integers(0, 4, rng.integers(10, 500)).astype(np.uint8))
    codes = np.concatenate(parts)
    L = len(codes)
    return codes, ["chrM1", "chrM2"], [L // 2, L - L // 2], _mk(codes, n_reads, 100, 5, False, seed=5)


def max_lines_per_read(sam):
    import collections
    c = collections.Counter(l.split("\t", 1)[0] for l in sam.splitlines())
    return max(c.values()) if c else 0


def three_fragment_reads(codes, n, m=120, seed=7):
    """Chimeric reads made of three pieces from distant places (reachable as 3-fragment hit chains at
    -s 2, R/AlignmentRecord.java:201-206 converts the first two)."""
    rng = np.random.default_rng(seed)
    L = len(codes)
    out = []
    for i in range(n):
        c1, c2 = sorted(rng.choice(np.arange(25, m - 25), 2, replace=False))
        if c2 - c1 < 25:
            c2 = c1 + 25
        a, b, c = rng.integers(0, L - m, 3)
        s = np.concatenate([codes[a:a + c1], codes[b + c1:b + c2], codes[c + c2:c + m]])
        if rng.random() < 0.5:
            s = synth.COMP[s[::-1]]
        out.append(("tri%04d" % i, synth.SYM[s].tobytes().decode(), "I" * len(s)))
    return out
