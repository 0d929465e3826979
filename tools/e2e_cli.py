"""End-to-end `align` timing through the CLI (first bullet): FASTQ file -> SAM file,
index load excluded, on a synthetic genome written as FASTA (GPU box; writes under $TMPDIR).

  python tools/e2e_cli.py [--genome hg19|<Mbp>] [--reads N] [--gz]
"""
import argparse
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tools")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genome", default="hg19")
    ap.add_argument("--reads", type=int, default=2_000_000)
    ap.add_argument("--gz", action="store_true")
    ap.add_argument("--saved-index", action="store_true", help="run the `bwt` command first; align loads its index")
    ap.add_argument("--devices", default=None)
    ap.add_argument("--workers", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 20)
    a = ap.parse_args()
    import gzip
    import numpy as np
    import synth
    contigs = synth.HG19_CONTIGS if a.genome == "hg19" else [("chr%d" % (i + 1), int(float(a.genome) * 1e6 / 4)) for i in range(4)]
    codes, names, lengths = synth.genome(contigs, config_id=1)
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    fa, fq = os.path.join(d, "ref.fa"), os.path.join(d, "reads.fq" + (".gz" if a.gz else ""))
    t0 = time.time()
    with open(fa, "wb") as f:  # 60 bases a line, written as a (rows, 61) byte array per contig
        off = 0
        for nm, L in zip(names, lengths):
            f.write(b">%s\n" % nm.encode())
            s = synth.SYM[codes[off:off + L]]
            rows = (L + 59) // 60
            blk = np.full((rows, 61), ord("\n"), dtype=np.uint8)
            flat = np.zeros(rows * 60, dtype=np.uint8)
            flat[:L] = s
            blk[:, :60] = flat.reshape(rows, 60)
            data = blk.tobytes()
            tail = rows * 60 - L  # drop the padding of the last line, keep its newline
            f.write(data[:len(data) - 1 - tail] + b"\n" if tail else data)
            off += L
    m = 100
    seqs = synth.reads_codes(codes, lengths, a.reads, m, 2, config_id=2)
    sb = synth.SYM[seqs]
    with (gzip.open(fq, "wb", compresslevel=1) if a.gz else open(fq, "wb")) as f:
        for c0 in range(0, a.reads, 1 << 18):
            c1 = min(a.reads, c0 + (1 << 18))
            f.write(b"".join(b"@r%09d\n%s\n+\n%s\n" % (i, sb[i].tobytes(), b"I" * m) for i in range(c0, c1)))
    print("[e2e] inputs written in %.1fs: %s (%.2f GB), %s (%.2f GB)"
          % (time.time() - t0, fa, os.path.getsize(fa) / 1e9, fq, os.path.getsize(fq) / 1e9), flush=True)
    out = os.path.join(d, "out.sam")
    cli = [sys.executable, os.path.join(REPO, "genome-weaver-align_amd", "gwa_cli.py")]
    if a.saved_index:
        t0 = time.time()
        r = subprocess.run(cli + ["bwt", fa], stderr=subprocess.PIPE, text=True)
        print("[e2e] bwt (FASTA -> saved index) %.1fs rc %d %s" % (time.time() - t0, r.returncode, r.stderr.strip()), flush=True)
    t0 = time.time()
    extra = (["--devices", a.devices] if a.devices else []) + ["--workers", str(a.workers), "--batch", str(a.batch)]
    r = subprocess.run(cli + ["align", "-r", fa, "-k", "2", "--timing"] + extra + [fq], stdout=open(out, "wb"),
                       stderr=subprocess.PIPE, text=True)
    print(r.stderr.strip(), flush=True)
    print("[e2e] CLI wall %.1fs, SAM %.2f GB, rc %d" % (time.time() - t0, os.path.getsize(out) / 1e9, r.returncode))
    for p in (fa, fq, out, fa + ".gwa.idx"):
        if os.path.exists(p):
            os.remove(p)
    os.rmdir(d)
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
