"""`align` command of genome-weaver on MI355X (A/Align.java:57-110 and the options of
A/AlignmentConfig.java:40-72, A/AlignmentScoreConfig.java:37-77).

  python genome-weaver-align_amd/gwa_cli.py align -r ref.fa [-q SEQ | reads.fq[.gz] | reads.fa[.gz]]
         [-k 0.1] [-m bsf|sf] [-R besthit|allhits|topL] [-L 5] [-g 1] [-e 4] [-s 1] [-M 1] [-N 3]
         [-G 11] [-E 4] [-S 11] [-P 5] [-W 31] [--silent] [--device 0] [--batch 1048576]

Writes SAM to stdout: the `@SQ` header (SequenceBoundary.toSAMHeader, A/SequenceBoundary.java:81-87)
then one record per read in input order, as SAMOutput does (A/SAMOutput.java:56-82).  Reads are
aligned in batches on one GPU; the index is built on the GPU from the FASTA at start-up (the
reference instead loads the files of its `bwt` command, A/FMIndexOnGenome.java:60-86).

Read input follows ReadReaderFactory.createReader (R/ReadReaderFactory.java:126-151): `.fa`,
`.fasta`, `.fan`, `.fastq`, `.fq`, optionally `.gz`; `-q` aligns one query named "read" with no
qualities (R/ReadReaderFactory.java:167-180).  Read names are the first whitespace-delimited token
of the header line (utgb FastqReader / FASTAPullParser are unvendored: parity unpinned).
"""
import argparse
import gzip
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import gwa  # noqa: E402


def _open(path):
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path, "rt")


def _kind(path):
    p = path[:-3] if path.endswith(".gz") else path
    if p.endswith((".fa", ".fasta", ".fan")):
        return "fasta"
    if p.endswith((".fastq", ".fq")):
        return "fastq"
    raise gwa.GwaError("Unsupported file type: " + path)


def read_fasta(f):
    """(name, seq, None) per record; multi-line sequences are concatenated."""
    name, parts = None, []
    for line in f:
        line = line.rstrip("\r\n")
        if line.startswith(">"):
            if name is not None:
                yield name, "".join(parts), None
            hdr = line[1:].split()
            name, parts = (hdr[0] if hdr else ""), []
        elif name is not None:
            parts.append(line.strip())
    if name is not None:
        yield name, "".join(parts), None


def read_fastq(f):
    """(name, seq, qual) per 4-line record."""
    while True:
        h = f.readline()
        if not h:
            return
        h = h.rstrip("\r\n")
        if not h:
            continue
        if not h.startswith("@"):
            raise gwa.GwaError("malformed FASTQ header: %r" % h[:80])
        seq = f.readline().rstrip("\r\n")
        plus = f.readline()
        qual = f.readline().rstrip("\r\n")
        if not plus.startswith("+") or len(qual) != len(seq):
            raise gwa.GwaError("malformed FASTQ record: %r" % h[:80])
        hdr = h[1:].split()
        yield (hdr[0] if hdr else ""), seq, qual


def reads_of(path):
    kind = _kind(path)  # unsupported suffixes fail before the file is opened
    f = _open(path)
    try:
        yield from (read_fasta(f) if kind == "fasta" else read_fastq(f))
    finally:
        f.close()


def native_chunks(path, chunk=64 << 20):
    """The read file as library-parsed chunks (gwa.ParsedReads, include/gwa.h gwa_reads_parse): the
    host side of the pipeline stays native for large files; read_fasta / read_fastq state the same
    record rules in Python (tests/test_cli.py holds the two to identical output)."""
    kind = _kind(path)
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        carry = b""
        while True:
            data = f.read(chunk)
            final = not data
            buf = carry + data
            if not buf:
                return
            pr = gwa.ParsedReads(buf, kind, final)
            yield pr
            carry = buf[pr.consumed:]
            if final:
                return


def build_parser():
    ap = argparse.ArgumentParser(prog="gwa", description="genome-weaver read alignment on MI355X")
    sub = ap.add_subparsers(dest="cmd", required=True)
    a = sub.add_parser("align", help="read alignment")
    a.add_argument("-r", dest="refSeq", required=True, help="reference sequence (FASTA)")
    a.add_argument("-q", dest="query", help="single query sequence")
    a.add_argument("readFiles", nargs="*", help="read file (single-end)")
    a.add_argument("--silent", action="store_true", help="disable output")
    a.add_argument("-m", dest="strategy", default="bsf", help="alignment strategy: bsf (default), sf")
    a.add_argument("-R", dest="reportType", default="besthit", help="besthit (default), allhits, topL")
    a.add_argument("-L", dest="topL", type=int, default=5)
    a.add_argument("-k", dest="k", type=float, default=0.1,
                   help="maximum edit distances. float (fraction of read length) or int [0.1]")
    a.add_argument("-g", dest="numGapOpenAllowed", type=int, default=1)
    a.add_argument("-e", dest="numGapExtensionAllowed", type=int, default=4)
    a.add_argument("-s", dest="numSplitAlowed", type=int, default=1)
    a.add_argument("-M", dest="matchScore", type=int, default=1)
    a.add_argument("-N", dest="mismatchPenalty", type=int, default=3)
    a.add_argument("-G", dest="gapOpenPenalty", type=int, default=11)
    a.add_argument("-E", dest="gapExtensionPenalty", type=int, default=4)
    a.add_argument("-S", dest="splitOpenPenalty", type=int, default=11)
    a.add_argument("-P", dest="indelEndSkip", type=int, default=5)
    a.add_argument("-W", dest="bandWidth", type=int, default=31)
    a.add_argument("--device", type=int, default=0, help="GPU ordinal")
    a.add_argument("--batch", type=int, default=1 << 20, help="reads per device batch")
    a.add_argument("--timing", action="store_true", help="index / align wall times and reads/s on stderr")
    return ap


def config_of(ns):
    cfg = gwa.AlignmentConfig(k=ns.k, strategy=ns.strategy, reportType=ns.reportType, topL=ns.topL,
                              numGapOpenAllowed=ns.numGapOpenAllowed, numGapExtensionAllowed=ns.numGapExtensionAllowed,
                              numSplitAlowed=ns.numSplitAlowed, matchScore=ns.matchScore,
                              mismatchPenalty=ns.mismatchPenalty, gapOpenPenalty=ns.gapOpenPenalty,
                              gapExtensionPenalty=ns.gapExtensionPenalty, splitOpenPenalty=ns.splitOpenPenalty,
                              indelEndSkip=ns.indelEndSkip, bandWidth=ns.bandWidth)
    cfg._c()  # validates strategy / report type (raises GwaError)
    return cfg


def align(ns, out=sys.stdout):
    if ns.query is None and not ns.readFiles:
        raise gwa.GwaError("no query is given")
    if ns.query is None and len(ns.readFiles) != 1:
        raise gwa.GwaError("# of input read files must be one (single-end)")
    cfg = config_of(ns)
    if ns.query is None:
        _kind(ns.readFiles[0])  # unsupported suffixes fail before the index is built
    t0 = time.perf_counter()
    fm = gwa.FMIndexOnGenome.load(ns.refSeq, device=ns.device)
    t1 = time.perf_counter()
    bsf = gwa.aligner(fm, cfg)
    w = (lambda s: None) if ns.silent else out.write
    w(fm.samHeader())
    n = 0
    if ns.query is not None:
        w(bsf.align_batch([("read", ns.query, None)]))
        n = 1
    else:
        for pr in native_chunks(ns.readFiles[0]):
            for i in range(0, pr.n, ns.batch):
                c = min(ns.batch, pr.n - i)
                w(gwa.align_reads(bsf, pr.slice(i, c)))
                n += c
            pr.close()
    t2 = time.perf_counter()
    fm.close()
    if ns.timing:
        print("[gwa] index load %.2fs; align (read file -> SAM, index load excluded) %.2fs: %.0f reads/s"
              % (t1 - t0, t2 - t1, n / max(t2 - t1, 1e-9)), file=sys.stderr)
    return n


def main(argv=None):
    ns = build_parser().parse_args(argv)
    try:
        if ns.cmd == "align":
            n = align(ns)
            print("[gwa] %d reads aligned" % n, file=sys.stderr)
    except gwa.GwaError as e:
        print("[gwa] error: %s" % e, file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
