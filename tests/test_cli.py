"""The `align` command (genome-weaver-align_amd/gwa_cli.py): read parsing and option handling on
CPU; end-to-end FASTA/FASTQ(.gz) -> SAM on the GPU, byte-identical to the oracle's header + records
(A/Align.java:57-110, A/SAMOutput.java:56-82)."""
import gzip
import io
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "genome-weaver-align_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tools")]

import gwa  # noqa: E402
import gwa_cli  # noqa: E402


def test_fasta_reader_multiline_and_names():
    f = io.StringIO(">r1 some description\nACGT\nACG\n>r2\n\nTTTT\n>empty\n")
    assert list(gwa_cli.read_fasta(f)) == [("r1", "ACGTACG", None), ("r2", "TTTT", None), ("empty", "", None)]


def test_fastq_reader_and_errors():
    f = io.StringIO("@q1 x\nACGT\n+\nIIII\n@q2\nAC\n+q2\nII\n")
    assert list(gwa_cli.read_fastq(f)) == [("q1", "ACGT", "IIII"), ("q2", "AC", "II")]
    with pytest.raises(gwa.GwaError):
        list(gwa_cli.read_fastq(io.StringIO("@q1\nACGT\n+\nII\n")))
    with pytest.raises(gwa.GwaError):
        list(gwa_cli.read_fastq(io.StringIO("q1\nACGT\n+\nIIII\n")))


def test_reference_fixture_counts(tmp_path):
    # the reference's own fixtures (T/record/ReadSequenceReaderTest.java:38-55: 3 reads)
    n = sum(1 for _ in gwa_cli.reads_of(os.path.join(HERE, "golden", "fixtures", "sample.fastq")))
    assert n == 3
    p = tmp_path / "r.fq.gz"
    with gzip.open(p, "wt") as f:
        f.write("@a\nACGT\n+\nIIII\n")
    assert list(gwa_cli.reads_of(str(p))) == [("a", "ACGT", "IIII")]
    with pytest.raises(gwa.GwaError):
        list(gwa_cli.reads_of(str(tmp_path / "x.txt")))


def test_options_and_errors():
    ns = gwa_cli.build_parser().parse_args(["align", "-r", "ref.fa", "-k", "2", "-R", "topL", "-L", "3", "r.fq"])
    cfg = gwa_cli.config_of(ns)
    assert cfg.k == 2.0 and cfg.reportType == "topL" and cfg.topL == 3 and cfg.bandWidth == 31
    ns = gwa_cli.build_parser().parse_args(["align", "-r", "ref.fa", "-m", "sf", "r.fq"])
    assert gwa_cli.config_of(ns).strategy == "sf"
    for m in ("bd", "bwa"):  # BidirectionalBWT: accepted, header-only output (A/Align.java:124-132)
        ns = gwa_cli.build_parser().parse_args(["align", "-r", "ref.fa", "-m", m, "r.fq"])
        assert gwa_cli.config_of(ns).strategy == m
    ns = gwa_cli.build_parser().parse_args(["align", "-r", "ref.fa", "-m", "xyz", "r.fq"])
    with pytest.raises(gwa.GwaError):
        gwa_cli.config_of(ns)
    ns = gwa_cli.build_parser().parse_args(["align", "-r", "ref.fa"])
    with pytest.raises(gwa.GwaError):
        gwa_cli.align(ns, out=io.StringIO())


def _py_records(text, fmt):
    f = io.StringIO(text.decode(), newline=None)  # text mode: universal newlines, as _open
    return list(gwa_cli.read_fasta(f) if fmt == "fasta" else gwa_cli.read_fastq(f))


def _native_records(text, fmt, chunk):
    # the CLI's chunked native parse (gwa_reads_parse with the unparsed tail carried over)
    out, carry, pos = [], b"", 0
    while True:
        data = text[pos:pos + chunk]
        pos += len(data)
        final = not data
        buf = carry + data
        if not buf:
            return out
        pr = gwa.ParsedReads(buf, fmt, final)
        out += pr.records()
        carry = buf[pr.consumed:]
        pr.close()
        if final:
            return out


FASTA_CASES = [b">r1 desc\nACGT\n  AC GT \r\n>r2\r\nNNNN\r>  \nAC\n", b"junk\n>a\n\nAC\n\n>b x y\nG", b"",
               b">only\n", b">\t t\x0bz\nac\x1cgt\n\n", b"no header\nat all\n"]
FASTQ_CASES = [b"@a x\nACGT\n+\nIIII\n\n@b\r\nAC\r\n+b\r\nII\r\n", b"\n\n@r\nA\n+\nI", b"",
               b"@\tq1\x0c extra\nACGN\n+q1\n!!!!\n@q2\n\n+\n\n",
               b"@c1\rACGT\r+\rIIII\r@c2 x\rGG\r+\r!!\r"]  # "\r" line ends only


@pytest.mark.parametrize("i", range(len(FASTA_CASES)))
def test_native_fasta_parser_matches_python(i):
    t = FASTA_CASES[i]
    exp = _py_records(t, "fasta")
    for chunk in range(1, len(t) + 2):
        assert _native_records(t, "fasta", chunk) == exp, chunk


@pytest.mark.parametrize("i", range(len(FASTQ_CASES)))
def test_native_fastq_parser_matches_python(i):
    t = FASTQ_CASES[i]
    exp = _py_records(t, "fastq")
    for chunk in range(1, len(t) + 2):
        assert _native_records(t, "fastq", chunk) == exp, chunk


def test_native_parser_cr_only_text_is_linear():
    # FASTQ with "\r" line ends only: the line scanner stops at the first "\r" of a bounded window
    # instead of searching to the end of the text for a "\n" on every line (quadratic before)
    import time
    rec = b"@r%d\r" + b"ACGT" * 25 + b"\r+\r" + b"I" * 100 + b"\r"
    t = b"".join(rec % k for k in range(40000))  # 8.6 MB, 160k lines
    t0 = time.perf_counter()
    pr = gwa.ParsedReads(t, "fastq", True)
    dt = time.perf_counter() - t0
    assert pr.n == 40000 and pr.consumed == len(t)
    assert pr.records()[123] == ("r123", "ACGT" * 25, "I" * 100)
    pr.close()
    assert dt < 2.0, dt


def test_native_parser_fixtures_and_errors():
    for name, fmt in (("sample.fastq", "fastq"), ("test2.fa", "fasta")):
        t = open(os.path.join(HERE, "golden", "fixtures", name), "rb").read()
        assert _native_records(t, fmt, 1 << 20) == _py_records(t, fmt)
        assert _native_records(t, fmt, 7) == _py_records(t, fmt)
    for bad in (b"@a\nAC\n+\nI\n", b"x\nAC\n+\nII\n", b"@a\nAC\n-\nII\n", b"@a\nAC\n"):
        with pytest.raises(gwa.GwaError):
            gwa.ParsedReads(bad, "fastq", True)
        with pytest.raises(gwa.GwaError):
            _py_records(bad, "fastq")


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", ["fq.gz", "fa"])
def test_cli_end_to_end_matches_oracle(tmp_path, fmt):
    import oracle as O
    import synth
    codes, names, lengths = synth.genome([("chrA", 60000), ("chr2", 41000)], config_id=9)
    ref = tmp_path / "ref.fa"
    ref.write_text(synth.fasta_text(codes, names, lengths))
    seqs, rn = synth.reads(codes, lengths, 700, 100, 2, config_id=10)
    strs = synth.to_strings(seqs)
    reads = [(rn[i], strs[i], "I" * 100 if fmt.startswith("fq") else None) for i in range(len(strs))]
    rp = tmp_path / ("reads." + fmt)
    opener = gzip.open if fmt.endswith(".gz") else open
    with opener(rp, "wt") as f:
        for n, s, q in reads:
            f.write("@%s\n%s\n+\n%s\n" % (n, s, q) if q else ">%s\n%s\n" % (n, s))
    out = io.StringIO()
    ns = gwa_cli.build_parser().parse_args(["align", "-r", str(ref), "-k", "2", "--batch", "256", str(rp)])
    assert gwa_cli.align(ns, out=out) == len(reads)
    oi = O.Index.from_fasta(ref.read_text())
    exp = oi.sam_header() + oi.align(reads, O.OrcConfig.default(k=2.0))
    assert out.getvalue() == exp


def _e2e_inputs(tmp_path, fmt, n=700, cid=10):
    import synth
    codes, names, lengths = synth.genome([("chrA", 60000), ("chr2", 41000)], config_id=9)
    ref = tmp_path / "ref.fa"
    ref.write_text(synth.fasta_text(codes, names, lengths))
    seqs, rn = synth.reads(codes, lengths, n, 100, 2, config_id=cid)
    strs = synth.to_strings(seqs)
    reads = [(rn[i], strs[i], "I" * 100 if fmt.startswith("fq") else None) for i in range(len(strs))]
    rp = tmp_path / ("reads." + fmt)
    opener = gzip.open if fmt.endswith(".gz") else open
    with opener(rp, "wt") as f:
        for nm, sq, q in reads:
            f.write("@%s\n%s\n+\n%s\n" % (nm, sq, q) if q else ">%s\n%s\n" % (nm, sq))
    return ref, rp, reads


@pytest.mark.gpu
def test_cli_two_device_handles_match_oracle(tmp_path):
    # the multi-device pipeline with two index replicas (both on GPU 0 here), small batches dealt
    # to both, SAM merged in input order == the oracle's
    import oracle as O
    ref, rp, reads = _e2e_inputs(tmp_path, "fq", n=3000, cid=11)
    out = io.StringIO()
    ns = gwa_cli.build_parser().parse_args(["align", "-r", str(ref), "-k", "2", "--batch", "97", "--devices", "0,0",
                                            str(rp)])
    assert gwa_cli.align(ns, out=out) == len(reads)
    oi = O.Index.from_fasta(ref.read_text())
    assert out.getvalue() == oi.sam_header() + oi.align(reads, O.OrcConfig.default(k=2.0))


@pytest.mark.gpu
def test_saved_index_and_bwt_command(tmp_path):
    import oracle as O
    ref, rp, reads = _e2e_inputs(tmp_path, "fq", n=500, cid=12)
    assert gwa_cli.main(["bwt", str(ref)]) == 0
    assert os.path.exists(str(ref) + ".gwa.idx")
    out = io.StringIO()
    ns = gwa_cli.build_parser().parse_args(["align", "-r", str(ref), "-k", "2", str(rp)])
    assert gwa_cli.align(ns, out=out) == len(reads)
    oi = O.Index.from_fasta(ref.read_text())
    assert out.getvalue() == oi.sam_header() + oi.align(reads, O.OrcConfig.default(k=2.0))
    # the saved file itself loads as an index
    fm = gwa.FMIndexOnGenome.load(str(ref) + ".gwa.idx")
    assert fm.samHeader() == oi.sam_header()
    fm.close()


@pytest.mark.gpu
@pytest.mark.parametrize("m", ["bd", "bwa"])
def test_bd_bwa_print_the_header_only(tmp_path, m):
    import oracle as O
    ref, rp, reads = _e2e_inputs(tmp_path, "fq", n=50, cid=13)
    out = io.StringIO()
    ns = gwa_cli.build_parser().parse_args(["align", "-r", str(ref), "-m", m, str(rp)])
    assert gwa_cli.align(ns, out=out) == len(reads)
    assert out.getvalue() == O.Index.from_fasta(ref.read_text()).sam_header()


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(len(FASTQ_CASES)))
def test_cli_device_fastq_parse_edge_cases(tmp_path, i):
    # the pipeline locates FASTQ fields on the GPU (batch_io.hip fastqFieldsKernel): CRLF / CR line
    # ends, blank lines between records, odd header whitespace, empty reads and a missing final newline
    # give the records the host parser (and gwa_cli.read_fastq) gives
    import oracle as O
    import synth
    codes, names, lengths = synth.genome([("chrA", 30000)], config_id=14)
    ref = tmp_path / "ref.fa"
    ref.write_text(synth.fasta_text(codes, names, lengths))
    s = synth.to_strings(synth.reads(codes, lengths, 40, 60, 1, config_id=15)[0])
    body = b"".join(b"@r%d desc\r\n%s\r\n+\r\n%s\r\n%s" % (k, s[k].encode(), b"I" * 60, b"\n" if k % 3 == 0 else b"")
                    for k in range(40))
    text = FASTQ_CASES[i] + b"\n" + body
    rp = tmp_path / "reads.fq"
    rp.write_bytes(text)
    recs = _py_records(text, "fastq")
    out = io.StringIO()
    ns = gwa_cli.build_parser().parse_args(["align", "-r", str(ref), "-k", "1", "--batch", "7", str(rp)])
    assert gwa_cli.align(ns, out=out) == len(recs)
    oi = O.Index.from_fasta(ref.read_text())
    assert out.getvalue() == oi.sam_header() + oi.align(recs, O.OrcConfig.default(k=1.0))


@pytest.mark.gpu
def test_cli_malformed_fastq_reports_the_record(tmp_path):
    import synth
    codes, names, lengths = synth.genome([("chrA", 30000)], config_id=14)
    ref = tmp_path / "ref.fa"
    ref.write_text(synth.fasta_text(codes, names, lengths))
    rp = tmp_path / "bad.fq"
    rp.write_bytes(b"@a\nACGT\n+\nIIII\n@b\nACGT\n+\nIII\n")
    ns = gwa_cli.build_parser().parse_args(["align", "-r", str(ref), str(rp)])
    with pytest.raises(gwa.GwaError, match="malformed FASTQ record"):
        gwa_cli.align(ns, out=io.StringIO())


@pytest.mark.gpu
def test_cli_paired_end_files(tmp_path):
    import oracle as O
    import synth
    codes, names, lengths = synth.genome([("chrA", 60000), ("chr2", 41000)], config_id=9)
    ref = tmp_path / "ref.fa"
    ref.write_text(synth.fasta_text(codes, names, lengths))
    m1, m2 = synth.pairs_codes(codes, lengths, 600, config_id=16)
    s1, s2 = synth.to_strings(m1), synth.to_strings(m2)
    r1 = [("q%d" % i, s1[i], "I" * 100) for i in range(600)]
    r2 = [("q%d" % i, s2[i], "I" * 100) for i in range(600)]
    for path, rs in ((tmp_path / "r_1.fq", r1), (tmp_path / "r_2.fq", r2)):
        path.write_text("".join("@%s\n%s\n+\n%s\n" % r for r in rs))
    out = io.StringIO()
    ns = gwa_cli.build_parser().parse_args(["align", "-r", str(ref), "-k", "2", "--batch", "250",
                                            str(tmp_path / "r_1.fq"), str(tmp_path / "r_2.fq")])
    assert gwa_cli.align(ns, out=out) == 600
    oi = O.Index.from_fasta(ref.read_text())
    assert out.getvalue() == oi.sam_header() + oi.align_pairs(r1, r2, O.OrcConfig.default(k=2.0))


@pytest.mark.gpu
def test_pipeline_appends_in_input_order(tmp_path):
    # an O_APPEND descriptor (shell ">>", open(..., "a")): pwrite would ignore the batch offsets and
    # append in completion order, so such output takes the in-order write path; several workers
    # over two handles and small batches give the same bytes as the oracle, after the old content
    import oracle as O
    ref, rp, reads = _e2e_inputs(tmp_path, "fq", n=2500, cid=17)
    fm = gwa.FMIndexOnGenome.load(str(ref))
    fm2 = gwa.FMIndexOnGenome.load(str(ref))
    out = tmp_path / "out.sam"
    out.write_bytes(b"@HD\tVN:1.0\n")
    pipe = gwa.Pipeline([fm, fm2], gwa.AlignmentConfig(k=2.0), batch_reads=61, workers_per_device=4)
    with open(out, "ab") as f:
        assert pipe.align_file(str(rp), f.fileno()) == len(reads)
    with open(out, "ab") as f:  # and once more: appended after the first run's records
        assert pipe.align_file(str(rp), f.fileno()) == len(reads)
    pipe.close()
    fm.close()
    fm2.close()
    oi = O.Index.from_fasta(ref.read_text())
    sam = oi.align(reads, O.OrcConfig.default(k=2.0))
    assert out.read_text() == "@HD\tVN:1.0\n" + sam + sam


# ---- --shard R/N: contiguous shards of one read file (one process per GPU, C3) ----

def _tricky_fastq(n, seed=5):
    """FASTQ whose quality lines often start with '@' or '+' (the shard cut must not sync on them),
    with blank lines, CRLF records and empty reads mixed in"""
    import random
    rnd = random.Random(seed)
    out = []
    for i in range(n):
        m = rnd.choice([0, 1, 7, 60, 100, 151])
        seq = "".join(rnd.choice("ACGTN") for _ in range(m))
        qual = "".join(rnd.choice("@+!#IJ5") for _ in range(m))
        if m and rnd.random() < 0.4:
            qual = rnd.choice("@+") + qual[1:]
        eol = "\r\n" if rnd.random() < 0.1 else "\n"
        out.append("@r%d x%s%s%s+%s%s%s" % (i, eol, seq, eol, eol, qual, eol))
        if rnd.random() < 0.05:
            out.append("\n")
    return "".join(out).encode()


@pytest.mark.parametrize("fmt", ["fq", "fa"])
def test_shard_ranges_tile_the_file_at_record_starts(tmp_path, fmt):
    # gwa_reads_shard_range (host code only): for every shard count the ranges tile the file, each
    # starts at a record, and the records of the shards in order are the file's records
    if fmt == "fq":
        text = _tricky_fastq(3000)
    else:
        import random
        rnd = random.Random(9)
        text = "".join(">s%d d\n%s\n%s\n" % (i, "".join(rnd.choice("ACGT>") for _ in range(rnd.randint(1, 70))).replace(">", "A"),
                                             "ACGT" * rnd.randint(0, 9)) for i in range(2000)).encode()
    p = tmp_path / ("reads." + fmt)
    p.write_bytes(text)
    whole = _native_records(text, "fastq" if fmt == "fq" else "fasta", 1 << 30)
    assert len(whole) == (3000 if fmt == "fq" else 2000)
    for nsh in (1, 2, 3, 7, 16, 64):
        ranges = [gwa.shard_range(str(p), r, nsh) for r in range(nsh)]
        assert ranges[0][0] == 0 and ranges[-1][1] == len(text)
        assert all(ranges[i][1] == ranges[i + 1][0] for i in range(nsh - 1))
        got = []
        for b, e in ranges:
            part = text[b:e]
            if part:
                assert part[:1] == (b"@" if fmt == "fq" else b">")
            got += _native_records(part, "fastq" if fmt == "fq" else "fasta", 1 << 30)
        assert got == whole, nsh


def test_shard_options_and_errors(tmp_path):
    p = tmp_path / "r.fq.gz"
    with gzip.open(p, "wt") as f:
        f.write("@a\nACGT\n+\nIIII\n")
    with pytest.raises(gwa.GwaError, match="uncompressed"):
        gwa.shard_range(str(p), 0, 2)
    q = tmp_path / "r.fq"
    q.write_text("@a\nACGT\n+\nIIII\n")
    with pytest.raises(gwa.GwaError):
        gwa.shard_range(str(q), 2, 2)
    assert gwa.shard_range(str(q), 1, 2)[1] == q.stat().st_size
    for bad in ("3", "2/2", "a/b", "-1/2"):
        ns = gwa_cli.build_parser().parse_args(["align", "-r", "ref.fa", "--shard=" + bad, str(q)])
        with pytest.raises(gwa.GwaError):
            gwa_cli.shard_of(ns)
    ns = gwa_cli.build_parser().parse_args(["align", "-r", "ref.fa", "--shard", "1/4", str(q)])
    assert gwa_cli.shard_of(ns) == (1, 4)


@pytest.mark.gpu
def test_cli_shards_concatenate_to_the_one_process_sam(tmp_path):
    # `align --shard r/N` for every r: the outputs concatenated in shard order are byte-identical to
    # one run over the whole file (header from shard 0 only), and to the oracle
    import oracle as O
    ref, rp, reads = _e2e_inputs(tmp_path, "fq", n=4000, cid=18)
    one = io.StringIO()
    ns = gwa_cli.build_parser().parse_args(["align", "-r", str(ref), "-k", "2", "--batch", "300", str(rp)])
    assert gwa_cli.align(ns, out=one) == len(reads)
    for nsh in (2, 5):
        parts, total = [], 0
        for r in range(nsh):
            out = tmp_path / ("shard%d_%d.sam" % (nsh, r))
            with open(out, "w") as f:
                ns = gwa_cli.build_parser().parse_args(["align", "-r", str(ref), "-k", "2", "--batch", "300",
                                                        "--shard", "%d/%d" % (r, nsh), str(rp)])
                total += gwa_cli.align(ns, out=f)
            parts.append(out.read_text())
        assert total == len(reads)
        assert "".join(parts) == one.getvalue()
    oi = O.Index.from_fasta(ref.read_text())
    assert one.getvalue() == oi.sam_header() + oi.align(reads, O.OrcConfig.default(k=2.0))


@pytest.mark.gpu
def test_pipeline_small_file_then_large_file_pins_for_the_large_one(tmp_path):
    # a pipeline that first aligns a small file pins small read-text buffers; a later large file must
    # not run on pageable memory because of them (they are unpinned and replaced by buffers of the
    # large file's chunk size); results stay identical
    ref, small, _ = _e2e_inputs(tmp_path, "fq", n=300, cid=19)
    big = tmp_path / "big.fq"
    rec = small.read_bytes()
    with open(big, "wb") as f:  # > 2 chunks of kChunk = 256 MiB is too slow here: the rule is per size
        for _ in range(200):
            f.write(rec)
    fm = gwa.FMIndexOnGenome.load(str(ref))
    pipe = gwa.Pipeline([fm], gwa.AlignmentConfig(k=2.0), batch_reads=4096, workers_per_device=2)
    with open(tmp_path / "a.sam", "wb") as f:
        pipe.align_file(str(small), f.fileno())
    n_small = pipe.stats().pinned_bufs
    with open(tmp_path / "b.sam", "wb") as f:
        pipe.align_file(str(big), f.fileno())
    st = pipe.stats()
    pipe.close()
    fm.close()
    assert n_small >= 3 and st.pinned_bufs >= 3
    assert (tmp_path / "b.sam").read_bytes() == (tmp_path / "a.sam").read_bytes() * 200
