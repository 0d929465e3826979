"""Diagnostic (GPU box): -m sf / -m bsf at k = 5 on the full-size hg19-like genome, small batches,
per-tier reads and times, then the oracle per chunk with progress lines.

  python tools/diag_sf.py [reads] [strategy]
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "genome-weaver-align_amd"), os.path.join(os.path.dirname(HERE), "oracle")]
import numpy as np  # noqa: E402
import synth  # noqa: E402
import gwa  # noqa: E402


def say(*a):
    print("[diag]", *a, flush=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    strategies = sys.argv[2].split(",") if len(sys.argv) > 2 else ["sf"]
    t0 = time.time()
    codes, names, lengths = synth.genome_repeats(synth.HG19_CONTIGS, config_id=1)
    say("genome %.0fs" % (time.time() - t0))
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths)
    say("index %.0fs" % (time.time() - t0))
    strs = synth.to_strings(synth.reads_codes(codes, lengths, n, 150, 2, config_id=4, indels=True, max_edits=5))
    reads = [("r%09d" % i, strs[i], "I" * 150) for i in range(n)]
    for strat in strategies:
        for sz in (100, 1000, n):
            if sz > n:
                continue
            b = gwa.Batch(gi, gwa.AlignmentConfig(k=5.0, strategy=strat), reads[:sz])
            t1 = time.time()
            b.run()
            st = b.stats()
            c = b.read_counters()
            say("%s %d reads: %.2fs tiers %s tier_ms %s fm/read %.0f states max %d fm max %d" % (
                strat, sz, time.time() - t1, list(st.tier_reads), [round(x) for x in st.tier_ms],
                st.fm_searches / sz, c[:, 5].max(), c[:, 1].max()))
            top = np.argsort(-c[:, 1])[:5]
            say("  heaviest reads (fm searches, states, tier):", [(int(i), int(c[i, 1]), int(c[i, 5]), int(c[i, 12])) for i in top])
            b.close()


if __name__ == "__main__":
    main()
