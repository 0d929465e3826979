"""Lane idleness of the one-read-per-lane quick scan (GPU box): per-read loop iterations from the
batch's read counters (k-mer lookups + Occ steps + 32-base text runs, estimated), grouped 64 reads
per wavefront in launch order; prints the work a wavefront waits for (its slowest lane) against the
work its lanes do.  tools only.
  python tools/quick_idle.py [--genome hg19|hg19r] [--reads N]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "genome-weaver-align_amd"), os.path.join(REPO, "tools")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genome", default="hg19")
    ap.add_argument("--reads", type=int, default=2_000_000)
    a = ap.parse_args()
    import numpy as np
    import synth
    import gwa
    if a.genome == "hg19r":
        codes, names, lengths = synth.genome_repeats(synth.HG19_CONTIGS, config_id=1)
    else:
        codes, names, lengths = synth.genome(synth.HG19_CONTIGS, config_id=1)
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths, device=0)
    m = 100
    strs = synth.to_strings(synth.reads_codes(codes, lengths, a.reads, m, 2, config_id=2, shard=0))
    b = gwa.Batch(gi, gwa.AlignmentConfig(k=2.0), [("r%d" % i, s, None) for i, s in enumerate(strs)])
    b.run()
    c = b.read_counters().astype(np.int64)
    quick, kmer, short = c[:, 2], c[:, 13], c[:, 14]
    occ = quick - short                       # steps on Occ blocks
    text_steps = np.maximum(short - 14 * kmer, 0)
    runs = (text_steps + 31) // 32 + (text_steps > 0)  # (estimate: 32 per run, +1 for the run that stops)
    it = occ + kmer + runs
    n = len(it) // 64 * 64
    w = it[:n].reshape(-1, 64)
    busy = w.sum() / (w.max(axis=1).sum() * 64)
    print("quick-scan loop iterations per read: mean %.1f, p50 %d, p90 %d, p99 %d, max %d"
          % (it.mean(), np.percentile(it, 50), np.percentile(it, 90), np.percentile(it, 99), it.max()))
    print("wavefronts of 64 reads in launch order: lanes busy %.1f %% of the slowest lane's iterations" % (100 * busy))
    srt = np.sort(it[:n]).reshape(-1, 64)
    print("(the same reads sorted by their iterations: %.1f %%)" % (100 * srt.sum() / (srt.max(axis=1).sum() * 64)))
    b.close()
    gi.close()


if __name__ == "__main__":
    main()
