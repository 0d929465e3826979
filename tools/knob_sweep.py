"""Sweep a batch-creation env knob (e.g. GWA_WAITQ16) on one resident index + read batch (GPU box).

  python tools/knob_sweep.py --genome hg19 --reads 10000000 --var GWA_WAITQ16 8 12 16
Prints one line per value: quickscan / search ms (HIP events, mean of --steps after one warmup).
A value "A=1;B=2" (with --var multi) sets several variables at once; "-" unsets.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "genome-weaver-align_amd"), os.path.join(REPO, "tools")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genome", default="hg19")
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--k", type=float, default=2.0)
    ap.add_argument("--c4", action="store_true", help="150 bp reads with 0-5 edits incl. indels (bench --workload c4)")
    ap.add_argument("--strategy", default="bsf")
    ap.add_argument("--var", required=True)
    ap.add_argument("values", nargs="+")
    a = ap.parse_args()
    import numpy as np
    import synth
    import gwa
    if a.genome == "hg19r":
        codes, names, lengths = synth.genome_repeats(synth.HG19_CONTIGS, config_id=1)
    else:
        contigs = synth.HG19_CONTIGS if a.genome == "hg19" else [("chr%d" % (i + 1), int(float(a.genome) * 1e6 / 4))
                                                                   for i in range(4)]
        codes, names, lengths = synth.genome(contigs, config_id=1)
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths, device=0)
    m = 150 if a.c4 else 100
    seqs = synth.reads_codes(codes, lengths, a.reads, m, 2, config_id=4 if a.c4 else 2, shard=0, indels=a.c4,
                             max_edits=5)
    seq_blob = synth.SYM[seqs].tobytes()
    seq_off = np.arange(0, m * (a.reads + 1), m, dtype=np.uint64)
    name_blob, name_off = synth.name_blob(a.reads)
    qual_blob = b"I" * (m * a.reads)
    ref = None
    touched = set()
    for v in a.values:
        for t in touched:
            os.environ.pop(t, None)
        if "=" in v:
            for kv in v.split(";"):
                k_, v_ = kv.split("=", 1)
                os.environ[k_] = v_
                touched.add(k_)
        elif v == "-":
            os.environ.pop(a.var, None)  # "-" = unset
        else:
            os.environ[a.var] = v
            touched.add(a.var)
        b = gwa.Batch(gi, gwa.AlignmentConfig(k=a.k, strategy=a.strategy), blobs=(name_blob, name_off, seq_blob, seq_off, qual_blob, seq_off))
        b.run()
        q = s = 0.0
        tms = [0.0] * 4
        for _ in range(a.steps):
            b.run()
            st = b.stats()
            q += st.quickscan_ms
            s += st.search_ms
            tms = [x + y for x, y in zip(tms, st.tier_ms)]
        sam, _ = b.results(0, 2000)
        same = ref is None or sam == ref
        ref = ref or sam
        print("%s=%s quickscan_ms=%.2f search_ms=%.2f tier_ms=%s tier_reads=%s same_sam=%s"
              % (a.var, v, q / a.steps, s / a.steps, [round(x / a.steps, 1) for x in tms], list(st.tier_reads), same),
              flush=True)
        b.close()


if __name__ == "__main__":
    main()
