"""The FASTQ text inside fixtures/reads_c1.fq.snap (make_snap.py): 400 reads of 100 bp with 0-2
substitutions drawn from a 200 kb synthetic genome (tools/synth.py, fixed seeds), and qualities from a
fixed PCG64 stream.  Deterministic: the tests rebuild the text and compare it with the decoded fixture."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
import synth  # noqa: E402


def genome():
    return synth.genome([("snapA", 120000), ("snapB", 80000)], 21)


def fastq_text():
    codes, names, lengths = genome()
    seqs, rn = synth.reads(codes, lengths, 400, 100, 2, config_id=22)
    strs = synth.to_strings(seqs)
    rng = np.random.Generator(np.random.PCG64(2024))
    out = []
    for i, s in enumerate(strs):
        q = bytes(rng.integers(33, 74, len(s), dtype=np.uint8)).decode()
        out.append("@%s\n%s\n+\n%s\n" % (rn[i], s, q))
    return "".join(out).encode()
