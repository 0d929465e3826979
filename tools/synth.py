"""Synthetic genome / read generator shared by tests and bench.py.

Genomes: `genome` = i.i.d. uniform ACGT contigs; `genome_repeats` = hg19-like composition (N gaps,
interspersed repeat families with divergence, tandem repeats and satellites, segmental
duplications) at hg19 contig lengths (both labelled synthetic).  Reads: name r%09d, start uniform
over N-free windows, strand 50/50 (- = reverse complement), QUAL 'I'*m, per-config edits.
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


# hg19 gaps that are not sequence: acrocentric short arms and the big chrY heterochromatin block
_ACRO = {"chr13": 19.0e6, "chr14": 19.0e6, "chr15": 20.0e6, "chr21": 9.4e6, "chr22": 16.0e6}


def _mutate(rng, block, div):
    """Substitute each base of block (uint8 [c, L]) with probability div[c] (per row)."""
    hit = rng.random(block.shape, dtype=np.float32) < div[:, None]
    block[hit] = (block[hit] + rng.integers(1, 4, int(hit.sum()), dtype=np.uint8)) % 4
    return block


def _scatter(rng, codes, starts, block):
    """codes[starts[i] : starts[i] + L] = block[i], keeping N positions (gaps) N."""
    L = block.shape[1]
    idx = starts[:, None] + np.arange(L, dtype=np.int64)[None, :]
    old = codes[idx]
    codes[idx] = np.where(old == 4, np.uint8(4), block)


def genome_repeats(contigs, config_id=1, scale=1.0, log=None):
    """hg19-like synthetic genome at the given contig lengths -> (codes, names, lengths).

    Composition (approximate hg19 fractions, SURVEY.md §8d "hg19-like N-gap runs", plus the repeat
    load that makes multi-hit suffix intervals common):
      N gaps ~6 %: 10 kb telomeres, a 3 Mb centromere per chromosome, acrocentric short arms,
        chrY heterochromatin, ~8 scattered 50-100 kb gaps per chromosome;
      Alu-like family (300 bp, ~10 % of sequence, 2-20 % divergence per copy);
      L1-like family (6 kb consensus, 5'-truncated copies of mean ~1 kb, ~17 %, 3-20 % divergence);
      24 further interspersed families (150-3000 bp, ~12 %, 5-30 % divergence);
      alpha-satellite-like 171 bp arrays around centromeres (~2 %, 2-10 % monomer divergence);
      microsatellites (period 1-6, 20-400 bp, ~1.5 %);
      segmental duplications (10-200 kb copies of other places, ~4 %, 0.5-5 % divergence).
    Deterministic for (contigs, config_id, scale)."""
    rng = np.random.Generator(np.random.PCG64(SEED0 ^ (config_id + 0x5EED)))
    codes, names, lengths = genome(contigs, config_id, scale)
    N = len(codes)
    offs = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)

    def say(msg):
        if log:
            log(msg)

    def spots(count, L):
        """count random start positions of L-base copies (within one contig each)."""
        ci = rng.choice(len(lengths), size=count, p=np.array(lengths, np.float64) / N)
        span = np.maximum(np.array(lengths, np.int64)[ci] - L, 1)
        return offs[ci] + (rng.random(count) * span).astype(np.int64)

    def family(cons_len, n_copies, dmin, dmax, trunc_mean=None, chunk=100000):
        cons = rng.integers(0, 4, cons_len, dtype=np.uint8)
        done = 0
        while done < n_copies:
            c = min(chunk, n_copies - done)
            if trunc_mean is None:
                L = cons_len
                blk = np.broadcast_to(cons, (c, L)).copy()
                _scatter(rng, codes, spots(c, L), _mutate(rng, blk, rng.uniform(dmin, dmax, c).astype(np.float32)))
            else:  # 5'-truncated copies: a few length classes per chunk
                for L in np.unique(np.minimum(cons_len, (rng.exponential(trunc_mean, 8) + 200).astype(np.int64))):
                    cc = max(1, c // 8)
                    blk = np.broadcast_to(cons[cons_len - L:], (cc, L)).copy()
                    _scatter(rng, codes, spots(cc, L), _mutate(rng, blk, rng.uniform(dmin, dmax, cc).astype(np.float32)))
            done += c
        return cons_len

    # interspersed families (copy counts scale with the genome)
    g = N / 3.1e9
    family(300, int(1.0e6 * g), 0.02, 0.20)
    say("alu-like done")
    family(6000, int(5.0e5 * g), 0.03, 0.20, trunc_mean=900)
    say("l1-like done")
    for f in range(24):
        L = int(rng.integers(150, 3000))
        family(L, max(1, int(0.12 * N / 24 / L)), 0.05, 0.30)
    say("other families done")
    # microsatellites
    n_ms = int(0.015 * N / 150)
    for _ in range(8):
        per = int(rng.integers(1, 7))
        unit = rng.integers(0, 4, per, dtype=np.uint8)
        L = 150
        blk = np.tile(unit, (n_ms // 8, L // per + 1))[:, :L].copy()
        _scatter(rng, codes, spots(n_ms // 8, L), _mutate(rng, blk, np.full(n_ms // 8, 0.02, np.float32)))
    say("microsatellites done")
    # segmental duplications: copies of other places
    sd_total, sd = int(0.04 * N), 0
    while sd < sd_total:
        L = int(min(rng.integers(10000, 200000), N // 4))
        src = spots(1, L)[0]
        dst = spots(1, L)[0]
        blk = codes[src:src + L][None, :].copy()
        blk[blk == 4] = 0
        _scatter(rng, codes, np.array([dst]), _mutate(rng, blk, np.array([rng.uniform(0.005, 0.05)], np.float32)))
        sd += L
    say("segmental duplications done")
    # N gaps and centromeric satellites, per chromosome
    alpha = rng.integers(0, 4, 171, dtype=np.uint8)
    for i, (nm, L) in enumerate(zip(names, lengths)):
        o = offs[i]
        tel = min(10000, L // 20)
        codes[o:o + tel] = 4
        codes[o + L - tel:o + L] = 4
        if L < 5e6 * scale and L < 2e7:
            continue
        if nm in _ACRO:
            codes[o:o + int(_ACRO[nm] * scale)] = 4
        if nm == "chrY":
            a = o + int(0.45 * L)
            codes[a:a + int(0.5 * L)] = 4
        cen = o + int(L * rng.uniform(0.3, 0.55))
        cl = int(3.0e6 * scale)
        codes[cen:cen + cl] = 4
        for side in (cen - int(4e5 * scale), cen + cl):  # satellite arrays flanking the centromere gap
            reps = max(1, int(4e5 * scale) // 171)
            blk = np.broadcast_to(alpha, (reps, 171)).copy()
            _mutate(rng, blk, rng.uniform(0.02, 0.10, reps).astype(np.float32))
            seg = blk.reshape(-1)
            a = max(o, min(side, o + L - len(seg)))
            codes[a:a + len(seg)] = np.where(codes[a:a + len(seg)] == 4, np.uint8(4), seg)
        for _ in range(int(rng.poisson(8))):
            gl = int(rng.integers(50000, 100000) * scale)
            a = o + int(rng.random() * max(1, L - gl))
            codes[a:a + gl] = 4
    say("gaps done")
    return codes, names, lengths


def genome_ngaps(contigs, config_id=1, scale=1.0):
    """The BASELINE stand-in: i.i.d. uniform ACGT at the given contig lengths with
    hg19-like N-gap runs and no repeats -> (codes, names, lengths).  Gaps per chromosome as in
    genome_repeats: 10 kb telomeres, a 3 Mb centromere (chromosomes >= 20 Mb), the acrocentric short
    arms, chrY heterochromatin, ~8 scattered 50-100 kb gaps (about 6 % N at hg19 size).
    Deterministic for (contigs, config_id, scale)."""
    codes, names, lengths = genome(contigs, config_id, scale)
    rng = np.random.Generator(np.random.PCG64(SEED0 ^ (config_id + 0x6A95)))
    o = 0
    for nm, L in zip(names, lengths):
        tel = min(10000, L // 20)
        codes[o:o + tel] = 4
        codes[o + L - tel:o + L] = 4
        if L >= 5e6 * scale or L >= 2e7:
            if nm in _ACRO:
                codes[o:o + int(_ACRO[nm] * scale)] = 4
            if nm == "chrY":
                a = o + int(0.45 * L)
                codes[a:a + int(0.5 * L)] = 4
            cen = o + int(L * rng.uniform(0.3, 0.55))
            codes[cen:cen + int(3.0e6 * scale)] = 4
            for _ in range(int(rng.poisson(8))):
                gl = int(rng.integers(50000, 100000) * scale)
                a = o + int(rng.random() * max(1, L - gl))
                codes[a:a + gl] = 4
        o += L
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
        # start uniform over N-free windows: redraw the windows that hold an N (only redrawn windows
        # are checked again: the others are unchanged, so the draws are those of a full re-check)
        W = m + (8 if indels else 0)
        chk = np.arange(c)
        for _ in range(64):
            win = codes[np.minimum(starts[chk][:, None] + np.arange(W)[None, :], N - 1)]
            bad = chk[(win == 4).any(axis=1)]
            if len(bad) == 0:
                break
            cj = rng.choice(len(L), size=len(bad), p=p)
            starts[bad] = offs[cj] + (rng.random(len(bad)) * (L[cj] - m - 1)).astype(np.int64)
            chk = bad
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


def pairs_codes(codes, lengths, n, m=100, mean=300, sd=30, max_subs=2, config_id=5, shard=0):
    """Paired-end reads (config C5): fragment length ~ N(mean, sd) (at least m), start uniform over
    N-free fragment windows; mate 1 = the fragment's first m bases and mate 2 = the reverse complement
    of its last m (or, for half the pairs, the fragment of the other strand: mates swapped and both
    reverse-complemented); each mate gets uniform {0..max_subs} substitutions.
    -> (mate1 codes uint8 [n, m], mate2 codes uint8 [n, m])."""
    rng = np.random.Generator(np.random.PCG64((SEED0 ^ config_id) + shard))
    N = len(codes)
    offs = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    L = np.array(lengths, dtype=np.int64)
    flen = np.maximum(m, np.rint(rng.normal(mean, sd, n))).astype(np.int64)
    W = int(flen.max())
    p = np.where(L >= W + 2, L - W - 1, 0).astype(np.float64)
    p /= p.sum()
    ci = rng.choice(len(L), size=n, p=p)
    starts = offs[ci] + (rng.random(n) * (L[ci] - W - 1)).astype(np.int64)
    for _ in range(64):  # N-free fragments
        win = codes[np.minimum(starts[:, None] + np.arange(W)[None, :], N - 1)]
        bad = np.nonzero(((win == 4) & (np.arange(W)[None, :] < flen[:, None])).any(axis=1))[0]
        if len(bad) == 0:
            break
        cj = rng.choice(len(L), size=len(bad), p=p)
        starts[bad] = offs[cj] + (rng.random(len(bad)) * (L[cj] - W - 1)).astype(np.int64)
    a = codes[starts[:, None] + np.arange(m)[None, :]]
    b = codes[(starts + flen - m)[:, None] + np.arange(m)[None, :]]
    b = COMP[b[:, ::-1]]
    swap = rng.integers(0, 2, n).astype(bool)
    m1 = np.where(swap[:, None], b, a)
    m2 = np.where(swap[:, None], a, b)
    for mate in (m1, m2):
        nsub = rng.integers(0, max_subs + 1, n)
        for j in range(max_subs):
            rows = np.nonzero(nsub > j)[0]
            pos = rng.integers(0, m, len(rows))
            mate[rows, pos] = (mate[rows, pos] + rng.integers(1, 4, len(rows)).astype(np.uint8)) % 4
    return m1, m2


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


_TO3BIT = np.full(256, 4, dtype=np.uint8)
for _c, _v in ((b"Aa", 0), (b"Cc", 1), (b"Gg", 2), (b"TtUu", 3)):
    for _b in _c:
        _TO3BIT[_b] = _v


def fasta_codes(path):
    """A FASTA file (e.g. $GWA_HG19) as (codes, names, lengths), the same values the library's packFasta
    (genome-weaver-align_amd/csrc/host_index.cpp; A/PackFasta.java:81-108) gives: every sequence line
    trimmed of bytes <= ' ' at both ends and each byte through to3bit (A/ACGT.java:36-43), the contig
    name the first token of its '>' line (up to whitespace or '|').  Vectorised over the whole file."""
    raw = np.fromfile(path, dtype=np.uint8)
    nl = np.flatnonzero(raw == 10)
    starts = np.concatenate([[0], nl + 1])
    ends = np.concatenate([nl, [raw.size]])
    keep = starts < ends
    starts, ends = starts[keep], ends[keep]
    hdr = raw[starts] == ord(">")
    names, seq_parts, lengths = [], [], []
    hidx = np.flatnonzero(hdr)
    for j, h in enumerate(hidx):
        s, e = int(starts[h]) + 1, int(ends[h])
        line = raw[s:e].tobytes().rstrip(b"\r").decode("latin-1")
        tok = line.strip().split()[0] if line.strip() else ""
        names.append(tok.split("|")[0])
        lo = int(ends[h]) + 1
        hi = int(starts[hidx[j + 1]]) if j + 1 < len(hidx) else raw.size
        block = raw[lo:hi]
        ws = block <= 32
        cr = np.flatnonzero(block == 13)
        if np.count_nonzero(ws) == np.count_nonzero(block == 10) + cr.size and \
                np.all((cr + 1 >= block.size) | (block[np.minimum(cr + 1, block.size - 1)] == 10)):
            # the usual file: the only bytes <= ' ' are line ends ("\n", "\r\n")
            seq = _TO3BIT[block[~ws]]
            seq_parts.append(seq)
            lengths.append(int(seq.size))
            continue
        # per line: drop bytes <= ' ' (the newline too) that lead or trail the line
        lid = np.cumsum(block == 10) - (block == 10)  # line index of every byte (a newline ends its line)
        solid = ~ws
        # first / last solid byte position of each line
        nlines = int(lid[-1]) + 1 if block.size else 0
        first = np.full(nlines, block.size, dtype=np.int64)
        last = np.full(nlines, -1, dtype=np.int64)
        pos = np.flatnonzero(solid)
        if pos.size:
            np.minimum.at(first, lid[pos], pos)
            np.maximum.at(last, lid[pos], pos)
        idx = np.arange(block.size)
        inner = (idx >= first[lid]) & (idx <= last[lid]) if block.size else np.zeros(0, bool)
        del ws, solid, pos, idx
        seq = _TO3BIT[block[inner]]
        seq_parts.append(seq)
        lengths.append(int(seq.size))
    codes = np.concatenate(seq_parts) if seq_parts else np.zeros(0, np.uint8)
    return codes, names, lengths


def fasta_text(codes, names, lengths, width=60):
    parts = []
    off = 0
    for nm, L in zip(names, lengths):
        parts.append(">" + nm + "\n")
        s = SYM[codes[off:off + L]].tobytes().decode()
        parts.extend(s[i:i + width] + "\n" for i in range(0, L, width))
        off += L
    return "".join(parts)


if __name__ == "__main__":
    # python tools/synth.py hg19r|hg19 OUT.npy : write a genome's codes (bench.py generates the hg19r
    # leg's genome in a child process while its main leg runs)
    import sys
    kind, out = sys.argv[1], sys.argv[2]
    c, _, _ = (genome_repeats if kind == "hg19r" else genome_ngaps)(HG19_CONTIGS, config_id=1)
    np.save(out, c)
