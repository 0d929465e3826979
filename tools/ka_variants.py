"""GPU box: the reference's BSF known answers (tests/golden) and a small random/repetitive batch through
each given libgwa build, compared with the oracle; prints the differing lines per build.

  python tools/ka_variants.py lib1.so lib2.so ...
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [HERE, os.path.join(REPO, "genome-weaver-align_amd"), os.path.join(REPO, "oracle")]
import oracle as O  # noqa: E402
import synth  # noqa: E402
from ab import load_variant  # noqa: E402


def main():
    G = json.load(open(os.path.join(REPO, "tests", "golden", "reference_known_answers.json")))
    ref = G["bsf"]["reference"]
    oi = O.Index.from_sequence("seq", ref)
    reads = [("read", c["query"], None) for c in G["bsf"]["cases"]]
    exp = oi.align(reads, O.OrcConfig.default(k=2.0))
    codes, names, lengths = synth.genome([("c1", 300000), ("c2", 200000)], 1)
    oi2 = O.Index.from_arrays(codes, names, lengths)
    seqs, rn = synth.reads(codes, lengths, 3000, 100, 2)
    strs = synth.to_strings(seqs)
    r2 = [(rn[i], strs[i], "I" * 100) for i in range(len(strs))]
    exp2 = oi2.align(r2, O.OrcConfig.default(k=2.0))
    for lib in sys.argv[1:]:
        g = load_variant(lib)
        gi = g.FMIndexOnGenome.buildFromSequence("seq", ref)
        for name, got, want in (("known answers", g.BidirectionalSuffixFilter(gi, g.AlignmentConfig(k=2.0)).align_batch(reads), exp),):
            print("[ka] %s %s: %s" % (os.path.basename(lib), name, got == want), flush=True)
            if got != want:
                for a, b in zip(got.splitlines(), want.splitlines()):
                    if a != b:
                        print("   got ", a, "\n   want", b)
        gi.close()
        gi2 = g.FMIndexOnGenome.buildFromCodes(codes, names, lengths)
        got2 = g.BidirectionalSuffixFilter(gi2, g.AlignmentConfig(k=2.0)).align_batch(r2)
        print("[ka] %s random 3000: %s" % (os.path.basename(lib), got2 == exp2), flush=True)
        gi2.close()


if __name__ == "__main__":
    main()
