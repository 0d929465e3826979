"""Synthetic genome / read generator shared by tests and bench.py.

Genome: i.i.d. uniform ACGT contigs (labelled synthetic).  Reads: name r%09d, start uniform
over the contig, strand 50/50 (- = reverse complement), QUAL 'I'*m, per-config edits.
Seeds: 0x6A09E667 ^ config_id (+ shard).  numpy PCG64 streams (not xoshiro).
"""
import numpy as np

HG19_CONTIGS = [  # hg19 chr1..22, X, Y, M lengths (stand-in sizes only)
    ("chr1", 249250621), ("chr2", 243199373), ("chr3", 198022430), ("chr4", 191154276), ("chr5", 180915260),
    ("chr6", 171115067), ("chr7", 159138663), ("chr8", 146364022), ("chr9", 141213431), ("chr10", 135534747),
    ("chr11", 135006516), ("chr12", 133851895), ("chr13", 115169878), ("chr14", 107349540), ("chr15", 102531392),
    ("chr16", 90354753), ("chr17", 81195210), ("chr18", 78077248), ("chr19", 59128983), ("chr20", 63025520),
    ("chr21", 48129895), ("chr22", 51304566), ("chrX", 155270560), ("chrY", 59373566), ("chrM", 16571)]
ECOLI = [("U00096.3", 4641652)]
SEED0 = 0x6A09E667
SYM = np.frombuffer(b"ACGTN", dtype=np.uint8)
COMP = np.array([3, 2, 1, 0, 4], dtype=np.uint8)


def genome(contigs, config_id=1, scale=1.0):
    """-> (codes uint8 [N], names, lengths)"""
    rng = np.random.Generator(np.random.PCG64(SEED0 ^ config_id))
    names = [c[0] for c in contigs]
    lengths = [max(1, int(c[1] * scale)) for c in contigs]
    n = sum(lengths)
    codes = np.empty(n, dtype=np.uint8)
    step = 1 << 26
    for s in range(0, n, step):
        e = min(n, s + step)
        codes[s:e] = rng.integers(0, 4, e - s, dtype=np.uint8)
    return codes, names, lengths


def reads(codes, lengths, n, m=100, max_subs=2, config_id=2, shard=0, indels=False, max_edits=5):
    """-> (seqs uint8 [n, m] codes, names list) ; substitutions: #subs uniform {0..max_subs},
    distinct positions, base uniform over the other 3."""
    seqs = reads_codes(codes, lengths, n, m, max_subs, config_id, shard, indels, max_edits)
    return seqs, ["r%09d" % i for i in range(n)]


def reads_codes(codes, lengths, n, m=100, max_subs=2, config_id=2, shard=0, indels=False, max_edits=5,
                chunk=1 << 20):
    """Chunked generator core: -> uint8 [n, m] read codes."""
    rng = np.random.Generator(np.random.PCG64((SEED0 ^ config_id) + shard))
    N = len(codes)
    offs = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    L = np.array(lengths, dtype=np.int64)
    p = np.where(L >= m + 2, L - m - 1, 0).astype(np.float64)
    p /= p.sum()
    out = np.empty((n, m), dtype=np.uint8)
    for c0 in range(0, n, chunk):
        c = min(chunk, n - c0)
        ci = rng.choice(len(L), size=c, p=p)
        starts = offs[ci] + (rng.random(c) * (L[ci] - m - 1)).astype(np.int64)
        if not indels:
            idx = starts[:, None] + np.arange(m)[None, :]
            blk = codes[np.minimum(idx, N - 1)]
            nsub = rng.integers(0, max_subs + 1, c)
            prev = None
            for j in range(max_subs):
                sel = nsub > j
                pos = rng.integers(0, m, c)
                if prev is not None:
                    pos = np.where(sel & (pos == prev), (pos + 1) % m, pos)
                else:
                    prev = pos
                r = rng.integers(1, 4, c).astype(np.uint8)
                rows = np.nonzero(sel)[0]
                blk[rows, pos[rows]] = (blk[rows, pos[rows]] + r[rows]) % 4
        else:
            idx = starts[:, None] + np.arange(m + 8)[None, :]
            win = codes[np.minimum(idx, N - 1)]
            blk = np.empty((c, m), dtype=np.uint8)
            ne = rng.integers(0, max_edits + 1, c)
            for i in range(c):
                s = list(win[i])
                for _ in range(ne[i]):
                    t = rng.random()
                    p_ = int(rng.integers(5, m - 5))
                    if t < 0.6:
                        s[p_] = (s[p_] + int(rng.integers(1, 4))) % 4
                    elif t < 0.8:
                        s.insert(p_, int(rng.integers(0, 4)))
                    else:
                        del s[p_]
                blk[i] = np.array((s + [0] * m)[:m], dtype=np.uint8)
        strand = rng.integers(0, 2, c)
        rc = COMP[blk[:, ::-1]]
        out[c0:c0 + c] = np.where(strand[:, None] == 1, rc, blk)
    return out


def name_blob(n, start=0):
    """names r%09d as one bytes blob + offsets (10 bytes each)."""
    ids = np.arange(start, start + n, dtype=np.int64)
    digits = np.empty((n, 10), dtype=np.uint8)
    digits[:, 0] = ord("r")
    for d in range(9):
        digits[:, 9 - d] = ord("0") + (ids // (10 ** d)) % 10
    return digits.tobytes(), np.arange(0, 10 * (n + 1), 10, dtype=np.uint64)


def to_strings(seqs):
    return [SYM[row].tobytes().decode() for row in seqs]


def fasta_text(codes, names, lengths, width=60):
    parts = []
    off = 0
    for nm, L in zip(names, lengths):
        parts.append(">" + nm + "\n")
        s = SYM[codes[off:off + L]].tobytes().decode()
        parts.extend(s[i:i + width] + "\n" for i in range(0, L, width))
        off += L
    return "".join(parts)
