"""`align` command of genome-weaver on MI355X (A/Align.java:57-110 and the options of
A/AlignmentConfig.java:40-72, A/AlignmentScoreConfig.java:37-77).

  python genome-weaver-align_amd/gwa_cli.py bwt ref.fa            (writes ref.fa.gwa.idx)
  python genome-weaver-align_amd/gwa_cli.py align -r ref.fa [-q SEQ | reads.fq[.gz|.snap] | reads.fa[.gz|.snap]]
         [-k 0.1] [-m bsf|sf|bd|bwa] [-R besthit|allhits|topL] [-L 5] [-g 1] [-e 4] [-s 1] [-M 1] [-N 3]
         [-G 11] [-E 4] [-S 11] [-P 5] [-W 31] [--silent] [--devices 0,1,..] [--batch 1048576]

Writes SAM to stdout: the `@SQ` header (SequenceBoundary.toSAMHeader, A/SequenceBoundary.java:81-87)
then one record per read in input order, as SAMOutput does (A/SAMOutput.java:56-82).  Read files go
through the library's multi-device pipeline (gwa_pipeline_align_file): batches dealt to one index
replica per GPU in --devices, SAM written back in input order.  Like the reference, which loads the
files its `bwt` command wrote next to the FASTA (A/FMIndexOnGenome.java:60-86, A/BWTFiles.java:40-80),
`align -r ref.fa` loads `ref.fa.gwa.idx` when `bwt` made one, and otherwise builds the index on the GPU
from the FASTA.

Read input follows ReadReaderFactory.createReader (R/ReadReaderFactory.java:126-151): `.fa`,
`.fasta`, `.fan`, `.fastq`, `.fq`, optionally `.gz` or `.snap` (snappy-java stream); `-q` aligns one query named "read" with no
qualities (R/ReadReaderFactory.java:167-180).  Read names are the first whitespace-delimited token
of the header line (utgb FastqReader / FASTAPullParser are unvendored: parity unpinned).
"""
import argparse
import gzip
import io
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import gwa  # noqa: E402


def _open(path):
    if path.endswith(".snap"):  # snappy-java stream (R/ReadReaderFactory.java:130-139)
        with open(path, "rb") as f:
            return io.TextIOWrapper(io.BytesIO(gwa.snappy_decompress(f.read())))
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path, "rt")


def _open_bytes(path):
    if path.endswith(".snap"):
        with open(path, "rb") as f:
            return io.BytesIO(gwa.snappy_decompress(f.read()))
    return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")


def _kind(path):
    p = path[:-3] if path.endswith(".gz") else path[:-5] if path.endswith(".snap") else path
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


def build_parser():
    ap = argparse.ArgumentParser(prog="gwa", description="genome-weaver read alignment on MI355X")
    sub = ap.add_subparsers(dest="cmd", required=True)
    a = sub.add_parser("align", help="read alignment")
    a.add_argument("-r", dest="refSeq", required=True, help="reference sequence (FASTA)")
    a.add_argument("-q", dest="query", help="single query sequence")
    a.add_argument("readFiles", nargs="*", help="read file (single-end), or two mate files (paired-end)")
    a.add_argument("--silent", action="store_true", help="disable output")
    a.add_argument("-m", dest="strategy", default="bsf", help="alignment strategy: bsf (default), sf, bd, bwa")
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
    a.add_argument("--device", type=int, default=0, help="GPU ordinal (one device)")
    a.add_argument("--devices", default=None, help="comma-separated GPU ordinals: one index replica per GPU")
    a.add_argument("--workers", type=int, default=3, help="host worker threads per device")
    b = sub.add_parser("bwt", help="build and save the index of a FASTA (loaded by align -r)")
    b.add_argument("fasta")
    b.add_argument("-o", dest="out", default=None, help="index file (default: <fasta>.gwa.idx)")
    b.add_argument("--device", type=int, default=0)
    a.add_argument("--batch", type=int, default=1 << 20, help="reads per device batch")
    a.add_argument("--timing", action="store_true", help="index / align wall times and reads/s on stderr")
    a.add_argument("--warm-passes", type=int, default=1,
                   help="timing runs: align the read file N times, the first N - 1 into /dev/null; --timing then "
                        "reports the last pass only")
    a.add_argument("--insert-min", type=int, default=210, help="paired-end: smallest template length of a proper pair")
    a.add_argument("--insert-max", type=int, default=390,
                   help="paired-end: largest template length of a proper pair (mate rescue needs max - min + read "
                        "length + 2k <= 320 bases; wider ranges pair without rescue)")
    a.add_argument("--sync", default=None, metavar="DIR:N",
                   help="timing runs of N processes (--shard): after the warm passes, wait until all N have written a "
                        "ready file into DIR, so their timed passes run at the same time; --timing then also prints "
                        "the timed pass's CLOCK_MONOTONIC start and end")
    a.add_argument("--shard", default=None, metavar="R/N",
                   help="one process per GPU: align contiguous shard R of N of the (plain) read file; the SAM "
                        "header is written by shard 0 only, so the shards' outputs concatenated in order are "
                        "the one-process SAM")
    return ap


def sync_wait(spec, timeout=600.0):
    """--sync DIR:N: write DIR/ready.<pid>, then wait until N ready files exist"""
    d, n = spec.rsplit(":", 1)
    n = int(n)
    open(os.path.join(d, "ready.%d" % os.getpid()), "w").close()
    t0 = time.monotonic()
    while sum(1 for x in os.listdir(d) if x.startswith("ready.")) < n:
        if time.monotonic() - t0 > timeout:
            raise gwa.GwaError("--sync %s: the other processes did not arrive" % spec)
        time.sleep(0.0005)


def shard_of(ns):
    """--shard R/N as (R, N), or None"""
    if ns.shard is None:
        return None
    try:
        r, n = (int(x) for x in ns.shard.split("/"))
    except ValueError:
        raise gwa.GwaError("--shard takes R/N (e.g. 0/8), got %r" % ns.shard)
    if n < 1 or not 0 <= r < n:
        raise gwa.GwaError("--shard %s: need 0 <= R < N" % ns.shard)
    return r, n


def config_of(ns):
    cfg = gwa.AlignmentConfig(k=ns.k, strategy=ns.strategy, reportType=ns.reportType, topL=ns.topL,
                              numGapOpenAllowed=ns.numGapOpenAllowed, numGapExtensionAllowed=ns.numGapExtensionAllowed,
                              numSplitAlowed=ns.numSplitAlowed, matchScore=ns.matchScore,
                              mismatchPenalty=ns.mismatchPenalty, gapOpenPenalty=ns.gapOpenPenalty,
                              gapExtensionPenalty=ns.gapExtensionPenalty, splitOpenPenalty=ns.splitOpenPenalty,
                              indelEndSkip=ns.indelEndSkip, bandWidth=ns.bandWidth)
    cfg._c()  # validates strategy / report type (raises GwaError)
    return cfg


def index_path(ref):
    """The saved index the `bwt` command writes for a FASTA (or the path itself when it is one)."""
    return ref + ".gwa.idx"


def load_indexes(ref, devices):
    """One FMIndexOnGenome per device (built in parallel; each GPU holds a full replica)."""
    import threading
    src = index_path(ref) if os.path.exists(index_path(ref)) else ref
    out, errs = [None] * len(devices), []

    def one(i, d):
        try:
            out[i] = gwa.FMIndexOnGenome.load(src, device=d)
        except gwa.GwaError as e:
            errs.append(e)

    th = [threading.Thread(target=one, args=(i, d)) for i, d in enumerate(devices)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        for x in out:
            if x is not None:
                x.close()
        raise errs[0]
    return out


def align(ns, out=sys.stdout):
    if ns.query is None and not ns.readFiles:
        raise gwa.GwaError("no query is given")
    if ns.query is None and len(ns.readFiles) not in (1, 2):
        raise gwa.GwaError("give one read file (single-end) or two mate files (paired-end)")
    cfg = config_of(ns)
    shard = shard_of(ns)
    if shard is not None and (ns.query is not None or len(ns.readFiles) != 1):
        raise gwa.GwaError("--shard splits one single-end read file")
    if ns.query is None:
        for f in ns.readFiles:
            _kind(f)  # unsupported suffixes fail before the index is built
    if shard is not None:
        gwa.shard_range(ns.readFiles[0], *shard)  # (a .gz or missing file fails before the index is built)
    devices = [int(x) for x in ns.devices.split(",")] if ns.devices else [ns.device]
    t0 = time.perf_counter()
    fms = load_indexes(ns.refSeq, devices)
    t1 = time.perf_counter()
    w = (lambda s: None) if ns.silent else out.write
    if shard is None or shard[0] == 0:
        w(fms[0].samHeader())
    n = 0
    t_open = 0.0
    try:
        if ns.query is not None:
            w(gwa.aligner(fms[0], cfg).align_batch([("read", ns.query, None)]))
            n = 1
        elif len(ns.readFiles) == 2:
            n = align_pairs(ns, fms[0], cfg, w)
        else:
            out.flush()
            tp = time.perf_counter()
            pipe = gwa.Pipeline(fms, cfg, batch_reads=ns.batch, workers_per_device=ns.workers)  # pins host buffers
            t_open = time.perf_counter() - tp
            try:
                # --warm-passes N: N - 1 untimed passes over the file into /dev/null first (pinned buffers,
                # device caches and the page cache warm), then the timed pass that writes the SAM
                for _ in range(max(0, ns.warm_passes - 1)):
                    with open(os.devnull, "wb") as dn:
                        pipe.align_file(ns.readFiles[0], dn.fileno(), shard=shard)
                if ns.sync:
                    sync_wait(ns.sync)
                if ns.warm_passes > 1 or ns.sync:
                    t1, t_open = time.perf_counter(), 0.0
                mono0 = time.monotonic_ns()
                if ns.silent:
                    with open(os.devnull, "wb") as dn:
                        n = pipe.align_file(ns.readFiles[0], dn.fileno(), shard=shard)
                else:
                    try:
                        fd = out.fileno()
                    except (AttributeError, io.UnsupportedOperation):
                        fd = None
                    if fd is not None:
                        n = pipe.align_file(ns.readFiles[0], fd, shard=shard)
                        if ns.timing:
                            st = pipe.stats()
                            print("[gwa] pipeline %.2fs: read %.2fs, frame %.2fs; summed over %d worker threads: parse %.2fs, "
                                  "set-up %.2fs, kernels %s s, SAM format %.2fs, write %.2fs, order wait %.2fs"
                                  % (st.wall_s, st.read_s, st.frame_s, ns.workers * len(devices), st.parse_s, st.setup_s,
                                     "/".join("%.2f" % st.device_kernel_s[i] for i in range(len(devices))),
                                     st.format_s, st.write_s, st.order_wait_s), file=sys.stderr)
                    else:  # an in-memory stream (tests): through a temporary file
                        with tempfile.TemporaryFile() as tf:
                            n = pipe.align_file(ns.readFiles[0], tf.fileno(), shard=shard)
                            tf.seek(0)
                            out.write(tf.read().decode())
            finally:
                t2 = time.perf_counter()  # (the SAM is written; unpinning the buffers is teardown)
                if ns.timing and ns.sync:
                    print("[gwa] timed pass monotonic_ns %d %d" % (mono0, time.monotonic_ns()), file=sys.stderr)
                pipe.close()
        if ns.query is not None or len(ns.readFiles) == 2:
            t2 = time.perf_counter()
    finally:
        for fm in fms:
            fm.close()
    if ns.timing:
        print("[gwa] index load %.2fs (%d device(s)); align (read file -> SAM, index load excluded) %.2fs: %.0f reads/s; "
              "of which pipeline open (pinning host buffers) %.2fs, after it %.0f reads/s"
              % (t1 - t0, len(devices), t2 - t1, n / max(t2 - t1, 1e-9), t_open, n / max(t2 - t1 - t_open, 1e-9)),
              file=sys.stderr)
    return n


def align_pairs(ns, fm, cfg, w):
    """Paired-end: mate i of the first file with mate i of the second (gwa_align_pairs, one GPU),
    two SAM lines per pair.  The reference prints only the header for two read files: its paired
    reader is a stub (R/ReadReaderFactory.java:60-84); the pairing rules are this build's own
    (include/gwa.h gwa_batch_create_pairs)."""
    if cfg.strategy.lower() != "bsf":
        raise gwa.GwaError("paired-end alignment runs -m bsf")
    pe = gwa.PairedEndAligner(fm, cfg, ns.insert_min, ns.insert_max)
    with _open_bytes(ns.readFiles[0]) as f1, _open_bytes(ns.readFiles[1]) as f2:
        p1 = gwa.ParsedReads(f1.read(), _kind(ns.readFiles[0]))
        p2 = gwa.ParsedReads(f2.read(), _kind(ns.readFiles[1]))
    try:
        if p1.n != p2.n:
            raise gwa.GwaError("the mate files hold %d and %d reads" % (p1.n, p2.n))
        for i in range(0, p1.n, ns.batch):
            c = min(ns.batch, p1.n - i)
            w(pe.align_pair_structs(p1.slice(i, c), p2.slice(i, c)))
        return p1.n
    finally:
        p1.close()
        p2.close()


def bwt(ns):
    """Build the index of a FASTA on the GPU and save it (the reference's `bwt` command,
    A/BWTransform.java:72-179, in this build's own format: include/gwa.h gwa_index_save)."""
    out = ns.out or index_path(ns.fasta)
    fm = gwa.FMIndexOnGenome.load(ns.fasta, device=ns.device)
    try:
        fm.save(out)
    finally:
        fm.close()
    print("[gwa] index of %s saved to %s" % (ns.fasta, out), file=sys.stderr)


def main(argv=None):
    ns = build_parser().parse_args(argv)
    try:
        if ns.cmd == "align":
            n = align(ns)
            print("[gwa] %d reads aligned" % n, file=sys.stderr)
        elif ns.cmd == "bwt":
            bwt(ns)
    except gwa.GwaError as e:
        print("[gwa] error: %s" % e, file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
