"""Writes the `.snap` read-file fixtures (tests/golden/fixtures/*.snap) that pin the library's snappy-java
stream decoder (genome-weaver-align_amd/csrc/snappy_stream.cpp, include/gwa.h gwa_snappy_decompress).

The reference reads `.snap` files through org.xerial.snappy.SnappyInputStream
(R/ReadReaderFactory.java:130-139); snappy-java is not vendored with it and no snappy
library exists here, so this script restates the published formats as an encoder:
  * SnappyOutputStream: magic 0x82 "SNAPPY" 0x00, big-endian int32 version 1 and compatible version 1,
    then per chunk (at most 32 KiB of input, snappy-java's default block size) a big-endian int32 length
    and one Snappy block;
  * Snappy block: varint uncompressed length, then literal / copy elements (a greedy 4-byte hash
    matcher here; the element kinds are rotated so every tag form -- literals with 0, 1 and 2 length
    bytes, copies with 1-, 2- and 4-byte offsets, overlapping copies -- appears in the fixtures).

  python tests/golden/make_snap.py      # rewrites the fixtures
Fixtures:
  reads_c1.fq.snap  -- 400 reads of 100 bp (tests/golden/snap_reads.py builds the same FASTQ text)
                       as a SnappyOutputStream stream of several chunks
  sample.fastq.snap -- the reference's own fixture sample.fastq as one bare Snappy block (the
                       SnappyInputStream fallback for Snappy.compress(byte[]) output)
"""
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import snap_reads  # noqa: E402

MAGIC = b"\x82SNAPPY\x00"


def varint(n):
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def literal(data):
    out = bytearray()
    n = len(data) - 1
    if n < 60:
        out.append(n << 2)
    elif n < 256:
        out += bytes([60 << 2, n])
    elif n < 65536:
        out += bytes([61 << 2]) + struct.pack("<H", n)
    else:
        out += bytes([62 << 2]) + struct.pack("<I", n)[:3]
    return bytes(out) + data


def copy(offset, length, form):
    """one copy element; form 1/2/4 = offset bytes (form 1 needs 4 <= length <= 11, offset < 2048)"""
    if form == 1:
        return bytes([1 | ((length - 4) << 2) | ((offset >> 8) << 5), offset & 0xFF])
    if form == 2:
        return bytes([2 | ((length - 1) << 2)]) + struct.pack("<H", offset)
    return bytes([3 | ((length - 1) << 2)]) + struct.pack("<I", offset)


def block(data, lit_head=0):
    """one Snappy block of data; its first lit_head bytes go out as one literal (long literals with
    1- and 2-byte lengths appear in the fixtures)"""
    out = bytearray(varint(len(data)))
    table = {}
    i, lit0, rot = min(lit_head, len(data)), 0, 0
    n = len(data)
    while i + 4 <= n:
        key = data[i:i + 4]
        j = table.get(key)
        table[key] = i
        if j is None or i - j > 65535:
            i += 1
            continue
        ln = 4
        while i + ln < n and data[j + ln] == data[i + ln] and ln < 64:
            ln += 1
        if lit0 < i:
            out += literal(data[lit0:i])
        off = i - j
        rot += 1
        if 4 <= ln <= 11 and off < 2048 and rot % 3 == 0:
            out += copy(off, ln, 1)
        elif rot % 5 == 0:
            out += copy(off, ln, 4)
        else:
            out += copy(off, ln, 2)
        i += ln
        lit0 = i
    if lit0 < n:
        out += literal(data[lit0:])
    return bytes(out)


def stream(data, chunk=32 * 1024):
    out = bytearray(MAGIC + struct.pack(">ii", 1, 1))
    for a in range(0, len(data), chunk):
        b = block(data[a:a + chunk], lit_head=300 if a == 0 else 0)
        out += struct.pack(">i", len(b)) + b
    return bytes(out)


def main():
    fx = os.path.join(HERE, "fixtures")
    with open(os.path.join(fx, "reads_c1.fq.snap"), "wb") as f:
        f.write(stream(snap_reads.fastq_text()))
    with open(os.path.join(fx, "sample.fastq"), "rb") as f:
        sample = f.read()
    # a bare block: one 100-byte literal (1 length byte) and the rest matched
    with open(os.path.join(fx, "sample.fastq.snap"), "wb") as f:
        f.write(block(sample, lit_head=100))


if __name__ == "__main__":
    main()
