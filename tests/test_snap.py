"""`.snap` read files (R/ReadReaderFactory.java:130-139: org.xerial.snappy.SnappyInputStream).  The
decoder (csrc/snappy_stream.cpp, gwa_snappy_decompress) is pinned by the fixtures
tests/golden/fixtures/*.snap, written by tests/golden/make_snap.py (a restatement of the published
snappy-java stream and Snappy block formats; snappy-java itself is not vendored with the reference,
SURVEY.md 8c, so the format is "parity unpinned" against the library's own encoder).  CPU: the decoder
and the CLI readers; GPU: a .snap FASTQ through the pipeline, SAM identical to the oracle's."""
import gzip
import io
import os
import struct
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
FX = os.path.join(HERE, "golden", "fixtures")
sys.path[:0] = [os.path.join(REPO, "genome-weaver-align_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tools"),
                os.path.join(HERE, "golden")]

import gwa  # noqa: E402
import gwa_cli  # noqa: E402
import snap_reads  # noqa: E402


def _read(name):
    with open(os.path.join(FX, name), "rb") as f:
        return f.read()


def test_stream_fixture_decodes_to_the_reads():
    data = _read("reads_c1.fq.snap")
    assert data[:8] == b"\x82SNAPPY\x00" and struct.unpack(">ii", data[8:16]) == (1, 1)
    assert gwa.snappy_decompress(data) == snap_reads.fastq_text()


def test_bare_block_fixture_decodes_to_the_reference_fixture():
    assert gwa.snappy_decompress(_read("sample.fastq.snap")) == _read("sample.fastq")


def test_corrupt_streams_fail():
    data = _read("reads_c1.fq.snap")
    with pytest.raises(gwa.GwaError):
        gwa.snappy_decompress(data[:-7])  # truncated chunk
    bad = bytearray(_read("sample.fastq.snap"))
    bad[-1] ^= 0xFF
    bare = bytes([5, 2 | (3 << 2), 0x40, 0x00])  # 5 bytes, then a copy at offset 64 of an empty output
    with pytest.raises(gwa.GwaError):
        gwa.snappy_decompress(bare)
    with pytest.raises(gwa.GwaError):
        gwa.snappy_decompress(bytes([0x80]))  # unterminated length varint
    # lengths that would size terabytes of output before any element is checked: a 6-byte varint
    # (Snappy's length is a uint32) and a 5-byte one far beyond what 10 input bytes can expand to
    with pytest.raises(gwa.GwaError):
        gwa.snappy_decompress(bytes([0xFF] * 5 + [0x7F, 0, 0, 0, 0]))
    with pytest.raises(gwa.GwaError):
        gwa.snappy_decompress(bytes([0xFF, 0xFF, 0xFF, 0xFF, 0x0F, 0, 0, 0, 0, 0]))
    # a stream chunk claiming more bytes than the data holds
    hdr = data[:16]
    with pytest.raises(gwa.GwaError):
        gwa.snappy_decompress(hdr + bytes([0x7F, 0xFF, 0xFF, 0xFF, 1, 0]))


def test_cli_reads_of_snap_equals_plain(tmp_path):
    plain = tmp_path / "reads_c1.fq"
    plain.write_bytes(snap_reads.fastq_text())
    snap = tmp_path / "reads_c1.fq.snap"
    snap.write_bytes(_read("reads_c1.fq.snap"))
    got = list(gwa_cli.reads_of(str(snap)))
    assert len(got) == 400 and got == list(gwa_cli.reads_of(str(plain)))
    # the reference's fixture, as a bare block: 3 reads (T/record/ReadSequenceReaderTest.java:38-55)
    s2 = tmp_path / "sample.fastq.snap"
    s2.write_bytes(_read("sample.fastq.snap"))
    assert len(list(gwa_cli.reads_of(str(s2)))) == 3
    with pytest.raises(gwa.GwaError):
        gwa.shard_range(str(snap), 0, 2)  # a shard needs an uncompressed file


@pytest.mark.gpu
def test_pipeline_snap_file_matches_oracle(tmp_path):
    import oracle as O
    import synth
    codes, names, lengths = snap_reads.genome()
    ref = tmp_path / "ref.fa"
    ref.write_text(synth.fasta_text(codes, names, lengths))
    snap = tmp_path / "reads_c1.fq.snap"
    snap.write_bytes(_read("reads_c1.fq.snap"))
    gz = tmp_path / "reads_c1.fq.gz"
    with gzip.open(gz, "wb") as f:
        f.write(snap_reads.fastq_text())
    reads = list(gwa_cli.reads_of(str(gz)))
    outs = []
    for rp in (snap, gz):
        out = io.StringIO()
        ns = gwa_cli.build_parser().parse_args(["align", "-r", str(ref), "-k", "2", "--batch", "64", str(rp)])
        assert gwa_cli.align(ns, out=out) == len(reads)
        outs.append(out.getvalue())
    oi = O.Index.from_fasta(ref.read_text())
    assert outs[0] == outs[1] == oi.sam_header() + oi.align(reads, O.OrcConfig.default(k=2.0))


@pytest.mark.gpu
def test_pipeline_snap_chunk_longer_than_file_fails(tmp_path):
    # the streaming reader (SnapReader, the pipeline's IO thread) checks a chunk's length against the
    # bytes left in the file before sizing its buffer: a clean error, not a 2 GiB allocation
    codes, names, lengths = snap_reads.genome()
    import synth
    ref = tmp_path / "ref.fa"
    ref.write_text(synth.fasta_text(codes, names, lengths))
    bad = tmp_path / "bad.fq.snap"
    bad.write_bytes(_read("reads_c1.fq.snap")[:16] + bytes([0x7F, 0xFF, 0xFF, 0xFF]) + b"\x01\x00")
    ns = gwa_cli.build_parser().parse_args(["align", "-r", str(ref), "-k", "2", "--batch", "64", str(bad)])
    with pytest.raises(gwa.GwaError, match="snappy"):
        gwa_cli.align(ns, out=io.StringIO())
