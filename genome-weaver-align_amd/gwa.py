"""gwa -- Python host mirror of genome-weaver's `align` plugin surface over the C-ABI (libgwa.so).

Mirrors (names, argument meaning, error behaviour) the reference's Java interface for this path:
  AlignmentConfig / AlignmentScoreConfig   A/AlignmentConfig.java:40-72, A/AlignmentScoreConfig.java:37-77
  FMIndexOnGenome.load / buildFromSequence A/FMIndexOnGenome.java:60-115
  Aligner.align(read, reporter)            A/Aligner.java:30-33   (batched: align_batch)
  SAMOutput (header + one emit per read)   A/SAMOutput.java:56-82
The compute path is the HIP extension: importing works without a GPU, but every call that aligns
or builds an index raises GwaError when no MI355X is present or libgwa.so is missing.
"""
import ctypes
import os
from dataclasses import dataclass, fields

_HERE = os.path.dirname(os.path.abspath(__file__))
# A process that also uses torch on the GPU must import torch before this library loads: torch's bundled
# HIP runtime and the system ROCm one libgwa.so links have the same SONAME (libamdhip64.so.7), so the
# first one loaded serves both, and torch initialises its device only on its own.
LIBPATH = os.path.join(_HERE, os.environ.get("GWA_LIB", "libgwa.so"))  # GWA_LIB=libgwa_prof.so: profiling build


class GwaError(RuntimeError):
    pass


class _Config(ctypes.Structure):
    _fields_ = [("k", ctypes.c_float)] + [(n, ctypes.c_int32) for n in (
        "strategy", "report_type", "top_l", "num_gap_open", "num_gap_ext", "num_split", "match", "mismatch",
        "gap_open", "gap_ext", "split_open", "indel_end_skip", "band_width")]


class _Reads(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("name", ctypes.c_void_p), ("seq", ctypes.c_void_p), ("qual", ctypes.c_void_p),
                ("name_off", ctypes.c_void_p), ("seq_off", ctypes.c_void_p), ("qual_off", ctypes.c_void_p),
                ("qual_null", ctypes.c_void_p)]


class _ReadBuf(ctypes.Structure):
    _fields_ = [("reads", _Reads), ("priv", ctypes.c_void_p)]


class Record(ctypes.Structure):
    """gwa_record_t: one SAM record as AlignmentRecord fields (string fields index the SAM text)."""
    _fields_ = [(n, ctypes.c_uint32) for n in ("read", "flag")] + [(n, ctypes.c_int32) for n in (
        "ref", "pos", "end", "strand", "nm", "x0", "split", "is_split", "qual_null", "pad_")] + [
        (n, ctypes.c_uint64) for n in ("line_off", "name_off", "cigar_off", "seq_off", "qual_off", "state_off")] + [
        (n, ctypes.c_uint32) for n in ("line_len", "name_len", "cigar_len", "seq_len", "qual_len", "state_len")]


class _Results(ctypes.Structure):
    _fields_ = [("n_reads", ctypes.c_uint32), ("sam", ctypes.c_void_p), ("sam_len", ctypes.c_uint64),
                ("line_off", ctypes.c_void_p), ("records", ctypes.c_void_p), ("n_records", ctypes.c_uint64),
                ("paired", ctypes.c_uint32)]


class BatchStats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("quickscan_ms", ctypes.c_double), ("search_ms", ctypes.c_double),
                ("fm_searches", ctypes.c_uint64), ("quick_steps", ctypes.c_uint64), ("blocks", ctypes.c_uint64),
                ("quick_blocks", ctypes.c_uint64), ("states", ctypes.c_uint64), ("sa_reads", ctypes.c_uint64), ("tier_reads", ctypes.c_uint32 * 4),
                ("n_mapped", ctypes.c_uint32), ("n_unmapped", ctypes.c_uint32), ("kmer_lookups", ctypes.c_uint64),
                ("quick_short_steps", ctypes.c_uint64), ("quick_sa_reads", ctypes.c_uint64),
                ("search_short_steps", ctypes.c_uint64), ("tier_ms", ctypes.c_float * 4),
                ("num_sw", ctypes.c_uint64), ("verify_bytes", ctypes.c_uint64),
                ("quick_text_runs", ctypes.c_uint64), ("encode_ms", ctypes.c_double), ("format_ms", ctypes.c_double),
                ("rescue_ms", ctypes.c_double), ("heavy_pairs", ctypes.c_uint64),
                ("rescue_window_skipped", ctypes.c_uint64)]


def shard_range(path, shard, nshards):
    """Byte range [begin, end) of contiguous shard `shard` of `nshards` of a plain read file, cut at record
    starts (include/gwa.h gwa_reads_shard_range): the shards' SAM concatenated in order is a one-process
    run's SAM."""
    b, e = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().gwa_reads_shard_range(path.encode(), shard, nshards, ctypes.byref(b), ctypes.byref(e)))
    return b.value, e.value


def snappy_decompress(data):
    """The bytes of a `.snap` file (R/ReadReaderFactory.java:130-139, snappy-java SnappyInputStream),
    decompressed by the library (include/gwa.h gwa_snappy_decompress; host only)."""
    out, n = ctypes.c_void_p(), ctypes.c_uint64()
    _check(lib().gwa_snappy_decompress(data, len(data), ctypes.byref(out), ctypes.byref(n)))
    try:
        return ctypes.string_at(out, n.value)
    finally:
        lib().gwa_free(out)


class PipelineStats(ctypes.Structure):
    _fields_ = [("reads", ctypes.c_uint64), ("batches", ctypes.c_uint64), ("wall_s", ctypes.c_double),
                ("read_s", ctypes.c_double), ("device_kernel_s", ctypes.c_double * 16), ("parse_s", ctypes.c_double),
                ("setup_s", ctypes.c_double), ("format_s", ctypes.c_double), ("write_s", ctypes.c_double),
                ("order_wait_s", ctypes.c_double), ("frame_s", ctypes.c_double), ("pinned_bufs", ctypes.c_uint64)]


_lib = None

# every symbol include/gwa.h declares (checked by tests/test_cabi.py)
EXPORTS = ["gwa_config_default", "gwa_last_error", "gwa_device_count", "gwa_index_build_fasta", "gwa_index_open",
           "gwa_index_build_codes", "gwa_index_save", "gwa_index_text_size", "gwa_index_device_bytes", "gwa_index_export_sa",
           "gwa_sam_header", "gwa_index_close", "gwa_align_batch", "gwa_results_free", "gwa_free",
           "gwa_batch_create", "gwa_batch_create_pairs", "gwa_align_pairs", "gwa_batch_run", "gwa_batch_stats", "gwa_batch_results", "gwa_batch_free",
           "gwa_batch_read_counters", "gwa_batch_results_range", "gwa_results_records", "gwa_batch_results_select", "gwa_batch_format",
           "gwa_batch_sam_copy",
           "gwa_pipeline_open", "gwa_pipeline_align", "gwa_pipeline_align_file", "gwa_pipeline_align_file_range",
           "gwa_reads_shard_range", "gwa_pipeline_stats",
           "gwa_pipeline_close", "gwa_reads_parse", "gwa_reads_free", "gwa_snappy_decompress"]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIBPATH):
            raise GwaError("libgwa.so is not built (run __graft_entry__.build() or make -C genome-weaver-align_amd)")
        L = ctypes.CDLL(LIBPATH)
        V, P, I, U64 = ctypes.c_void_p, ctypes.POINTER, ctypes.c_int, ctypes.c_uint64
        L.gwa_last_error.restype = ctypes.c_char_p
        L.gwa_config_default.argtypes = [P(_Config)]
        L.gwa_index_build_fasta.argtypes = [ctypes.c_char_p, U64, I, P(V)]
        L.gwa_index_open.argtypes = [ctypes.c_char_p, I, P(V)]
        L.gwa_index_build_codes.argtypes = [V, U64, ctypes.c_int32, V, V, I, P(V)]
        L.gwa_index_save.argtypes = [V, ctypes.c_char_p]
        L.gwa_index_text_size.restype = U64
        L.gwa_index_text_size.argtypes = [V]
        L.gwa_index_device_bytes.restype = U64
        L.gwa_index_device_bytes.argtypes = [V]
        L.gwa_index_export_sa.argtypes = [V, I, V]
        L.gwa_sam_header.argtypes = [V, P(V), P(U64)]
        L.gwa_index_close.argtypes = [V]
        L.gwa_align_batch.argtypes = [V, P(_Config), P(_Reads), P(_Results)]
        L.gwa_results_free.argtypes = [P(_Results)]
        L.gwa_results_records.argtypes = [V, P(_Results)]
        L.gwa_free.argtypes = [V]
        L.gwa_batch_create.argtypes = [V, P(_Config), P(_Reads), P(V)]
        L.gwa_batch_run.argtypes = [V]
        L.gwa_batch_create_pairs.argtypes = [V, P(_Config), P(_Reads), P(_Reads), ctypes.c_int32, ctypes.c_int32, P(V)]
        L.gwa_align_pairs.argtypes = [V, P(_Config), P(_Reads), P(_Reads), ctypes.c_int32, ctypes.c_int32, P(_Results)]
        L.gwa_batch_stats.argtypes = [V, P(BatchStats)]
        L.gwa_batch_results.argtypes = [V, P(_Results)]
        L.gwa_batch_free.argtypes = [V]
        L.gwa_batch_read_counters.argtypes = [V, V]
        L.gwa_batch_results_range.argtypes = [V, ctypes.c_uint32, ctypes.c_uint32, P(_Results)]
        L.gwa_batch_results_select.argtypes = [V, V, ctypes.c_uint32, P(_Results)]
        L.gwa_batch_format.argtypes = [V, P(U64)]
        L.gwa_batch_sam_copy.argtypes = [V, V, P(U64)]
        L.gwa_reads_parse.argtypes = [ctypes.c_char_p, U64, I, I, P(_ReadBuf), P(U64)]
        L.gwa_reads_free.argtypes = [P(_ReadBuf)]
        L.gwa_pipeline_open.argtypes = [V, I, P(_Config), ctypes.c_uint32, I, P(V)]
        L.gwa_pipeline_align.argtypes = [V, P(_Reads), P(_Results)]
        L.gwa_pipeline_align_file.argtypes = [V, ctypes.c_char_p, I, P(U64)]
        L.gwa_pipeline_align_file_range.argtypes = [V, ctypes.c_char_p, I, U64, U64, P(U64)]
        L.gwa_reads_shard_range.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, P(U64), P(U64)]
        L.gwa_pipeline_stats.argtypes = [V, P(PipelineStats)]
        L.gwa_pipeline_close.argtypes = [V]
        if hasattr(L, "gwa_snappy_decompress"):  # (older libraries in A/B runs lack it)
            L.gwa_snappy_decompress.argtypes = [ctypes.c_char_p, U64, P(V), P(U64)]
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise GwaError(lib().gwa_last_error().decode())


STRATEGIES = {"bsf": 0, "sf": 1, "bd": 2, "bwa": 3}
REPORT_TYPES = {"besthit": 0, "allhits": 1, "topl": 2}


@dataclass
class AlignmentConfig:
    """AlignmentConfig + AlignmentScoreConfig, same defaults and CLI symbols."""
    k: float = 0.1             # -k  max edits (fraction of read length when in (0,1))
    strategy: str = "bsf"      # -m
    reportType: str = "besthit"  # -R
    topL: int = 5              # -L
    numGapOpenAllowed: int = 1  # -g
    numGapExtensionAllowed: int = 4  # -e
    numSplitAlowed: int = 1    # -s
    matchScore: int = 1        # -M
    mismatchPenalty: int = 3   # -N
    gapOpenPenalty: int = 11   # -G
    gapExtensionPenalty: int = 4  # -E
    splitOpenPenalty: int = 11  # -S
    indelEndSkip: int = 5      # -P
    bandWidth: int = 31        # -W

    def getMaximumEditDistance(self, readLength):
        # A/AlignmentScoreConfig.java:40-47 (float arithmetic)
        import numpy as np
        if 0 < self.k < 1:
            return int(np.floor(np.float32(readLength) * np.float32(self.k)))
        return int(self.k)

    def _c(self):
        if self.strategy.lower() not in STRATEGIES:
            raise GwaError("%s mode is not supported on the device path" % self.strategy)
        c = _Config()
        c.k = self.k
        c.strategy = STRATEGIES[self.strategy.lower()]
        c.report_type = REPORT_TYPES[self.reportType.lower()]
        c.top_l = self.topL
        c.num_gap_open, c.num_gap_ext, c.num_split = self.numGapOpenAllowed, self.numGapExtensionAllowed, self.numSplitAlowed
        c.match, c.mismatch, c.gap_open = self.matchScore, self.mismatchPenalty, self.gapOpenPenalty
        c.gap_ext, c.split_open = self.gapExtensionPenalty, self.splitOpenPenalty
        c.indel_end_skip, c.band_width = self.indelEndSkip, self.bandWidth
        return c


def _pack(strs):
    import numpy as np
    bs = [s.encode() if isinstance(s, str) else s for s in strs]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(b) for b in bs])
    blob = b"".join(bs)
    return blob, off


class FMIndexOnGenome:
    """An FM-index resident in one GPU's HBM (both strands, full SA, 2-bit text, contig table)."""

    def __init__(self, handle, device):
        self.h = handle
        self.device = device

    @classmethod
    def load(cls, fasta_path, device=0):
        h = ctypes.c_void_p()
        _check(lib().gwa_index_open(fasta_path.encode(), device, ctypes.byref(h)))
        return cls(h, device)

    @classmethod
    def buildFromFasta(cls, text, device=0):
        b = text.encode() if isinstance(text, str) else text
        h = ctypes.c_void_p()
        _check(lib().gwa_index_build_fasta(b, len(b), device, ctypes.byref(h)))
        return cls(h, device)

    @classmethod
    def buildFromSequence(cls, name, seq, device=0):
        return cls.buildFromFasta(">%s\n%s\n" % (name, seq), device)

    @classmethod
    def buildFromCodes(cls, codes, names, lengths, device=0):
        import numpy as np
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        ln = np.ascontiguousarray(lengths, dtype=np.int64)
        arr = (ctypes.c_char_p * len(names))(*[n.encode() for n in names])
        h = ctypes.c_void_p()
        _check(lib().gwa_index_build_codes(codes.ctypes.data, len(codes), len(names), ctypes.cast(arr, ctypes.c_void_p),
                                          ln.ctypes.data, device, ctypes.byref(h)))
        return cls(h, device)

    def save(self, path):
        """Write the index (gwa_index_save); FMIndexOnGenome.load(path) reads it back without the FASTA."""
        _check(lib().gwa_index_save(self.h, path.encode()))

    def textSize(self):
        return lib().gwa_index_text_size(self.h)

    def deviceBytes(self):
        return lib().gwa_index_device_bytes(self.h)

    def suffixArray(self, strand):
        import numpy as np
        out = np.zeros(self.textSize(), dtype=np.uint32)
        _check(lib().gwa_index_export_sa(self.h, strand, out.ctypes.data))
        return out

    def samHeader(self):
        p = ctypes.c_void_p()
        n = ctypes.c_uint64()
        _check(lib().gwa_sam_header(self.h, ctypes.byref(p), ctypes.byref(n)))
        s = ctypes.string_at(p, n.value).decode()
        lib().gwa_free(p)
        return s

    def close(self):
        if self.h:
            lib().gwa_index_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _reads_struct(reads, keep):
    """gwa_reads_t of [(name, seq, qual-or-None)]: a read whose qual is None prints QUAL "*" (the
    reference's Read.getQual(0) == null, R/AlignmentRecord.java:157), per read (qual_null)."""
    import numpy as np
    names, seqs, quals = zip(*reads) if reads else ((), (), ())
    nb, no = _pack(names)
    sb, so = _pack(seqs)
    any_q = any(q is not None for q in quals)
    r = _Reads()
    r.n = len(reads)
    keep.extend([nb, no, sb, so])
    r.name, r.seq = ctypes.cast(ctypes.c_char_p(nb), ctypes.c_void_p), ctypes.cast(ctypes.c_char_p(sb), ctypes.c_void_p)
    r.name_off, r.seq_off = no.ctypes.data, so.ctypes.data
    r.qual, r.qual_off, r.qual_null = None, None, None
    if any_q:
        qb, qo = _pack([q if q is not None else "" for q in quals])
        keep.extend([qb, qo])
        r.qual, r.qual_off = ctypes.cast(ctypes.c_char_p(qb), ctypes.c_void_p), qo.ctypes.data
        if any(q is None for q in quals):
            qn = np.array([q is None for q in quals], dtype=np.uint8)
            keep.append(qn)
            r.qual_null = qn.ctypes.data
    return r


def _take_results(res):
    import numpy as np
    try:
        s = ctypes.string_at(res.sam, res.sam_len).decode() if res.sam_len else ""
        off = np.ctypeslib.as_array((ctypes.c_uint64 * (res.n_reads + 1)).from_address(res.line_off)).copy()
        return s, off
    finally:
        lib().gwa_results_free(ctypes.byref(res))


class BidirectionalSuffixFilter:
    """The `-m bsf` Aligner (S/BidirectionalSuffixFilter.java), batched on one GPU."""

    def __init__(self, fmIndex, config=None):
        self.fmIndex = fmIndex
        self.config = config or AlignmentConfig()

    def align_batch(self, reads):
        """reads: list of (name, seq, qual-or-None) -> SAM text (no header), input order."""
        keep = []
        r = _reads_struct(reads, keep)
        res = _Results()
        c = self.config._c()
        _check(lib().gwa_align_batch(self.fmIndex.h, ctypes.byref(c), ctypes.byref(r), ctypes.byref(res)))
        return _take_results(res)[0]

    def align(self, read, reporter):
        """Aligner.align(Read, Reporter): reporter(line) once per emitted SAM line."""
        for line in self.align_batch([read]).splitlines():
            reporter(line)


class ParsedReads:
    """Reads parsed from FASTA / FASTQ text by the library (gwa_reads_parse): the records of a text
    chunk as a gwa_reads_t over library-owned blobs.  consumed = bytes of the chunk parsed (the
    rest starts an unfinished record unless final)."""

    def __init__(self, text, fmt, final=True):
        self._buf = _ReadBuf()
        self._text = bytes(text)
        used = ctypes.c_uint64()
        _check(lib().gwa_reads_parse(self._text, len(self._text), {"fasta": 0, "fastq": 1}[fmt], 1 if final else 0,
                                     ctypes.byref(self._buf), ctypes.byref(used)))
        self.consumed = used.value
        self.n = self._buf.reads.n

    def slice(self, first, count):
        """A gwa_reads_t for reads [first, first + count) (offsets stay absolute)."""
        r0 = self._buf.reads
        r = _Reads()
        r.n = count
        r.name, r.seq, r.qual = r0.name, r0.seq, r0.qual
        r.name_off = r0.name_off + 8 * first
        r.seq_off = r0.seq_off + 8 * first
        r.qual_off = (r0.qual_off + 8 * first) if r0.qual_off else None
        r.qual_null = (r0.qual_null + first) if r0.qual_null else None
        return r

    def records(self):
        """[(name, seq, qual-or-None)] (tests)."""
        import numpy as np
        r = self._buf.reads
        out = []
        if r.n == 0:
            return out
        offs = [np.ctypeslib.as_array((ctypes.c_uint64 * (r.n + 1)).from_address(a)) if a else None
                for a in (r.name_off, r.seq_off, r.qual_off)]
        blobs = [ctypes.string_at(p, int(o[-1])) if o is not None else None
                 for p, o in zip((r.name, r.seq, r.qual), offs)]
        for i in range(r.n):
            f = [b[o[i]:o[i + 1]].decode() if o is not None else None for b, o in zip(blobs, offs)]
            out.append((f[0], f[1], f[2]))
        return out

    def close(self):
        if self._buf.priv:
            lib().gwa_reads_free(ctypes.byref(self._buf))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def align_reads(aligner_, reads_struct):
    """SAM text of a gwa_reads_t (ParsedReads.slice) through aligner_'s index and config."""
    res = _Results()
    c = aligner_.config._c()
    _check(lib().gwa_align_batch(aligner_.fmIndex.h, ctypes.byref(c), ctypes.byref(reads_struct), ctypes.byref(res)))
    s = ctypes.string_at(res.sam, res.sam_len).decode() if res.sam_len else ""
    lib().gwa_results_free(ctypes.byref(res))
    return s


class SuffixFilter(BidirectionalSuffixFilter):
    """The `-m sf` Aligner (S/SuffixFilter.java), batched on one GPU."""

    def __init__(self, fmIndex, config=None):
        import dataclasses
        super().__init__(fmIndex, dataclasses.replace(config or AlignmentConfig(), strategy="sf"))


class PairedEndAligner:
    """Paired-end alignment (config C5) on one GPU: mate1[i] and mate2[i] form pair i; two SAM lines
    per pair (include/gwa.h gwa_align_pairs; the build's own pairing rules -- the reference's
    paired-end path is a stub, R/ReadReaderFactory.java:60-84, WeaverAlign.scala:259-278)."""

    def __init__(self, fmIndex, config=None, min_insert=210, max_insert=390):
        self.fmIndex = fmIndex
        self.config = config or AlignmentConfig()
        self.min_insert, self.max_insert = min_insert, max_insert

    def align_pairs(self, mates1, mates2):
        """mates: lists of (name, seq, qual-or-None) -> SAM text (no header), pair order."""
        keep = []
        r1, r2 = _reads_struct(mates1, keep), _reads_struct(mates2, keep)
        return self.align_pair_structs(r1, r2)

    def align_pair_structs(self, r1, r2):
        res = _Results()
        c = self.config._c()
        _check(lib().gwa_align_pairs(self.fmIndex.h, ctypes.byref(c), ctypes.byref(r1), ctypes.byref(r2),
                                     self.min_insert, self.max_insert, ctypes.byref(res)))
        return _take_results(res)[0]


class BidirectionalBWT(BidirectionalSuffixFilter):
    """`-m bd` / `-m bwa` (S/BidirectionalBWT.java): the reference reports BWAState / AlignmentSA
    objects that SAMOutput.emit drops (A/SAMOutput.java:73-82), so its SAM holds the header only;
    align_batch returns no records, as the reference prints none."""


def aligner(fmIndex, config):
    """Align.query's strategy switch (A/Align.java:116-137): the Aligner for config.strategy."""
    s = config.strategy.lower()
    if s == "sf":
        return SuffixFilter(fmIndex, config)
    if s == "bsf":
        return BidirectionalSuffixFilter(fmIndex, config)
    if s in ("bd", "bwa"):
        return BidirectionalBWT(fmIndex, config)
    raise GwaError("%s mode is not supported" % config.strategy)


class Pipeline:
    """Multi-device driver (include/gwa.h gwa_pipeline_*): read batches dealt to several index replicas
    (one per GPU), SAM in input order.  indexes: FMIndexOnGenome handles, one per device."""

    def __init__(self, indexes, config, batch_reads=1 << 20, workers_per_device=0):
        self.indexes = list(indexes)
        arr = (ctypes.c_void_p * len(self.indexes))(*[ix.h.value if hasattr(ix.h, "value") else ix.h
                                                       for ix in self.indexes])
        self.config = config
        self.h = ctypes.c_void_p()
        c = config._c()
        _check(lib().gwa_pipeline_open(ctypes.cast(arr, ctypes.c_void_p), len(self.indexes), ctypes.byref(c),
                                       batch_reads, workers_per_device, ctypes.byref(self.h)))

    def align_batch(self, reads):
        """reads: list of (name, seq, qual-or-None) -> SAM text (no header), input order."""
        keep = []
        r = _reads_struct(reads, keep)
        res = _Results()
        _check(lib().gwa_pipeline_align(self.h, ctypes.byref(r), ctypes.byref(res)))
        return _take_results(res)[0]

    def align_reads(self, reads_struct):
        res = _Results()
        _check(lib().gwa_pipeline_align(self.h, ctypes.byref(reads_struct), ctypes.byref(res)))
        return _take_results(res)[0]

    def align_file(self, path, fd, shard=None):
        """Stream a FASTA/FASTQ[.gz] read file through the devices; SAM records to file descriptor fd.
        shard=(r, N): only the records of contiguous shard r of N (a plain file; shard_range)."""
        n = ctypes.c_uint64()
        if shard is None:
            _check(lib().gwa_pipeline_align_file(self.h, path.encode(), fd, ctypes.byref(n)))
        else:
            b, e = shard_range(path, *shard)
            _check(lib().gwa_pipeline_align_file_range(self.h, path.encode(), fd, b, e, ctypes.byref(n)))
        return n.value

    def stats(self):
        st = PipelineStats()
        _check(lib().gwa_pipeline_stats(self.h, ctypes.byref(st)))
        return st

    def close(self):
        if self.h:
            lib().gwa_pipeline_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def reads_from_blobs(name_blob, name_off, seq_blob, seq_off, qual_blob=None, qual_off=None):
    """A gwa_reads_t over caller-built blobs (used for large synthetic batches)."""
    r = _Reads()
    r.n = len(name_off) - 1
    r.name = ctypes.cast(ctypes.c_char_p(name_blob), ctypes.c_void_p)
    r.seq = ctypes.cast(ctypes.c_char_p(seq_blob), ctypes.c_void_p)
    r.name_off, r.seq_off = name_off.ctypes.data, seq_off.ctypes.data
    if qual_blob is not None:
        r.qual, r.qual_off = ctypes.cast(ctypes.c_char_p(qual_blob), ctypes.c_void_p), qual_off.ctypes.data
    else:
        r.qual, r.qual_off = None, None
    return r


class Batch:
    """Split form for benchmarking: reads resident in HBM, run() = the timed kernels."""

    def __init__(self, fmIndex, config, reads=None, blobs=None, pair_blobs=None, insert=(210, 390)):
        """reads: [(name, seq, qual)] or blobs = (name, name_off, seq, seq_off, qual, qual_off); pair_blobs =
        (mate-1 blobs, mate-2 blobs) makes a paired-end batch (gwa_batch_create_pairs)."""
        self._keep = []
        self.h = ctypes.c_void_p()
        self.device = fmIndex.device  # the GPU holding the batch (its index's)
        c = config._c()
        if pair_blobs is not None:
            self._keep.append(pair_blobs)
            r1, r2 = reads_from_blobs(*pair_blobs[0]), reads_from_blobs(*pair_blobs[1])
            self.n = r1.n
            self.n_reads = 2 * r1.n
            _check(lib().gwa_batch_create_pairs(fmIndex.h, ctypes.byref(c), ctypes.byref(r1), ctypes.byref(r2),
                                                insert[0], insert[1], ctypes.byref(self.h)))
            return
        if blobs is not None:
            self._keep.append(blobs)
            r = reads_from_blobs(*blobs)
            self.n = r.n
        else:
            r = _reads_struct(reads, self._keep)
            self.n = len(reads)
        _check(lib().gwa_batch_create(fmIndex.h, ctypes.byref(c), ctypes.byref(r), ctypes.byref(self.h)))

    def run(self):
        _check(lib().gwa_batch_run(self.h))

    def format_device(self):
        """Write the batch's SAM text in HBM only (pairing included for paired batches); its size."""
        n = ctypes.c_uint64()
        _check(lib().gwa_batch_format(self.h, ctypes.byref(n)))
        return n.value

    def stats(self):
        st = BatchStats()
        _check(lib().gwa_batch_stats(self.h, ctypes.byref(st)))
        return st

    def sam_device(self):
        """The SAM text of the last format_device() as a uint8 torch tensor on the batch's GPU (a
        device-to-device copy; for dist.gather_sam_device over RCCL)."""
        import torch
        n = ctypes.c_uint64()
        _check(lib().gwa_batch_sam_copy(self.h, None, ctypes.byref(n)))
        t = torch.empty(n.value, dtype=torch.uint8, device=torch.device("cuda", self.device))
        if n.value:
            _check(lib().gwa_batch_sam_copy(self.h, ctypes.c_void_p(t.data_ptr()), ctypes.byref(n)))
        return t

    def results(self, first=0, count=None):
        res = _Results()
        if count is None:
            _check(lib().gwa_batch_results(self.h, ctypes.byref(res)))
        else:
            _check(lib().gwa_batch_results_range(self.h, first, count, ctypes.byref(res)))
        return _take_results(res)

    def results_select(self, idx):
        """(SAM text, line offsets) of the reads idx (any order, as given)."""
        import numpy as np
        idx = np.ascontiguousarray(idx, dtype=np.uint32)
        res = _Results()
        _check(lib().gwa_batch_results_select(self.h, idx.ctypes.data, len(idx), ctypes.byref(res)))
        return _take_results(res)

    def records(self, index, first=0, count=None):
        """(SAM text, [Record]) of reads [first, first + count): the AlignmentRecord fields of every line
        (include/gwa.h gwa_results_records)."""
        res = _Results()
        _check(lib().gwa_batch_results_range(self.h, first, self.n - first if count is None else count,
                                             ctypes.byref(res)))
        try:
            _check(lib().gwa_results_records(index.h, ctypes.byref(res)))
            recs = [Record.from_buffer_copy(ctypes.string_at(res.records + i * ctypes.sizeof(Record), ctypes.sizeof(Record)))
                    for i in range(res.n_records)]
            return (ctypes.string_at(res.sam, res.sam_len).decode() if res.sam_len else ""), recs
        finally:
            lib().gwa_results_free(ctypes.byref(res))

    def sam_size(self):
        """Format the whole batch's SAM text in the library (D2H of the records + host formatting) and
        return its size in bytes without copying it into Python (host-pipeline timing)."""
        res = _Results()
        _check(lib().gwa_batch_results(self.h, ctypes.byref(res)))
        n = res.sam_len
        lib().gwa_results_free(ctypes.byref(res))
        return n

    READ_COUNTERS = 20  # include/gwa.h GWA_READ_COUNTERS

    def read_counters(self):
        """per read (include/gwa.h gwa_batch_read_counters): status, fm_searches, quick_steps, quickscan_blocks,
        search_blocks, states, sa_reads, n_hits, quick-scan mismatches/starts x4, deepest tier, k-mer lookups,
        quick short steps, search text steps, DP verifications, verify bytes"""
        import numpy as np
        out = np.zeros((getattr(self, "n_reads", self.n), self.READ_COUNTERS), dtype=np.int32)
        _check(lib().gwa_batch_read_counters(self.h, out.ctypes.data))
        return out

    def close(self):
        if self.h:
            lib().gwa_batch_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
