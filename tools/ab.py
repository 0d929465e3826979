"""A/B timing of libgwa builds in one process (GPU box): each library (ctypes, RTLD_LOCAL) gets its
own index replica of the same genome and its own batch of the same reads; the whole-path step
(run + format) is timed alternately, and the SAM of every build is compared with the first.

  python tools/ab.py [--workload c2|c4] [--genome hg19|hg19r] [--reads N] [--steps K] lib1.so lib2.so ...
"""
import argparse
import ctypes
import importlib
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [HERE, os.path.join(REPO, "genome-weaver-align_amd")]


def say(*a):
    print("[ab]", *a, flush=True)


def load_variant(path):
    import gwa
    mod = importlib.util.module_from_spec(importlib.util.find_spec("gwa"))
    mod.__spec__.loader.exec_module(mod)
    mod.LIBPATH = os.path.abspath(path)
    mod._lib = None
    mod.lib()
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--genome", default="hg19")
    ap.add_argument("--reads", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--strategy", default="bsf")
    ap.add_argument("--env", action="append", default=[], help="per-variant env: IDX:VAR=VAL (applied around its calls)")
    args = ap.parse_args()
    import numpy as np
    import synth
    c4 = args.workload == "c4"
    m = 150 if c4 else 100
    n = args.reads or (1_000_000 if c4 else 10_000_000)
    t0 = time.time()
    gen = synth.genome_repeats if args.genome == "hg19r" else synth.genome_ngaps
    codes, names, lengths = gen(synth.HG19_CONTIGS, config_id=1)
    seqs = synth.reads_codes(codes, lengths, n, m, 2, config_id=4 if c4 else 2, indels=c4, max_edits=5)
    seq_blob = synth.SYM[seqs].tobytes()
    del seqs
    off = np.arange(0, m * (n + 1), m, dtype=np.uint64)
    nb, no = synth.name_blob(n)
    blobs = (nb, no, seq_blob, off, b"I" * (m * n), off)
    say("genome + %d reads in %.0fs" % (n, time.time() - t0))
    envs = {}
    for e in args.env:
        i, kv = e.split(":", 1)
        k, v = kv.split("=", 1)
        envs.setdefault(int(i), {})[k] = v
    vs = []
    for i, p in enumerate(args.libs):
        g = load_variant(p)
        t0 = time.time()
        gi = g.FMIndexOnGenome.buildFromCodes(codes, names, lengths)
        for k, v in envs.get(i, {}).items():
            os.environ[k] = v
        b = g.Batch(gi, g.AlignmentConfig(k=5.0 if c4 else 2.0, strategy=args.strategy), blobs=blobs)
        for k in envs.get(i, {}):
            del os.environ[k]
        vs.append((p, g, gi, b))
        say("variant %d %s: index + batch %.0fs" % (i, p, time.time() - t0))
    times = {p: [] for p, *_ in vs}
    for rep in range(args.steps + 1):
        for i, (p, g, gi, b) in enumerate(vs):
            for k, v in envs.get(i, {}).items():
                os.environ[k] = v
            t0 = time.perf_counter()
            b.run()
            b.format_device()
            st = b.stats()
            dt = time.perf_counter() - t0
            for k in envs.get(i, {}):
                del os.environ[k]
            if rep > 0:
                times[p].append((dt * 1e3, st.encode_ms, st.quickscan_ms, st.search_ms, st.format_ms, list(st.tier_ms),
                                 list(st.tier_reads)))
    ref = None
    rng = np.random.default_rng(5)
    samp = np.sort(rng.choice(n, min(n, 200000), replace=False)).astype(np.uint32)
    for i, (p, g, gi, b) in enumerate(vs):
        ts = times[p]
        med = sorted(t[0] for t in ts)[len(ts) // 2]
        sam, _ = b.results_select(samp)
        same = "ref" if ref is None else (sam == ref)
        ref = ref if ref is not None else sam
        say("%-40s step %.1f ms (median of %d) = %.2f M reads/s; encode %.2f qs %.2f search %.2f format %.2f tiers %s "
            "(reads %s); SAM %s"
            % (os.path.basename(p) + str(envs.get(i, "")), med, len(ts), n / med / 1e3, ts[-1][1], ts[-1][2], ts[-1][3],
               ts[-1][4], [round(x, 1) for x in ts[-1][5]], ts[-1][6], same))


if __name__ == "__main__":
    main()
