"""Diagnostic (GPU box): -m sf (or bsf) at k = 5 on the full-size hg19-like genome -- per-tier reads
and times, the heaviest reads (states created, FM searches, tier), then the oracle on every read that
needed a tier >= 1, one at a time, with its state count and time, SAM compared.

  python tools/diag_sf.py [reads] [strategy] [oracle: 0/1]
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


def heartbeat():
    import threading
    t0 = time.time()

    def beat():
        while True:
            time.sleep(30)
            say("... %.0fs" % (time.time() - t0))
    threading.Thread(target=beat, daemon=True).start()


def main():
    heartbeat()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    strat = sys.argv[2] if len(sys.argv) > 2 else "sf"
    run_oracle = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    t0 = time.time()
    codes, names, lengths = synth.genome_repeats(synth.HG19_CONTIGS, config_id=1)
    say("genome %.0fs" % (time.time() - t0))
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths)
    say("index %.0fs" % (time.time() - t0))
    strs = synth.to_strings(synth.reads_codes(codes, lengths, n, 150, 2, config_id=4, indels=True, max_edits=5))
    reads = [("r%09d" % i, strs[i], "I" * 150) for i in range(n)]
    b = gwa.Batch(gi, gwa.AlignmentConfig(k=5.0, strategy=strat), reads)
    t1 = time.time()
    b.run()
    st = b.stats()
    c = b.read_counters()
    say("%s %d reads: %.2fs tiers %s tier_ms %s search %.1f ms fm/read %.0f states max %d fm max %d" % (
        strat, n, time.time() - t1, list(st.tier_reads), [round(x) for x in st.tier_ms], st.search_ms,
        st.fm_searches / n, c[:, 5].max(), c[:, 1].max()))
    deep = np.nonzero(c[:, 12] >= 1)[0]
    say("tier histogram:", {int(t): int((c[:, 12] == t).sum()) for t in np.unique(c[:, 12])})
    top = np.argsort(-c[:, 5])[:12]
    say("heaviest reads (read, fm searches, states, tier):", [(int(i), int(c[i, 1]), int(c[i, 5]), int(c[i, 12])) for i in top])
    got, _ = b.results_select(deep.astype(np.uint32))
    b.close()
    if not run_oracle or len(deep) == 0:
        return
    import oracle as O
    t0 = time.time()
    sa_f = gi.suffixArray(0)
    O.check_cyclic_sa_full(codes, sa_f, threads=16)
    sa_r = gi.suffixArray(1)
    O.check_cyclic_sa_full(np.ascontiguousarray(codes[::-1]), sa_r, threads=16)
    oi = O.Index.from_arrays(codes, names, lengths, sa_f=sa_f, sa_r=sa_r)
    del sa_f, sa_r
    say("SA check + oracle index %.0fs" % (time.time() - t0))
    cfg = O.OrcConfig.default(k=5.0, strategy=gwa.STRATEGIES[strat])
    lines = got.splitlines(True)
    order = np.argsort(-c[deep, 5])
    heavy = [int(deep[j]) for j in order[:16]]
    for r in heavy:
        t2 = time.time()
        s, stt = oi.align([reads[r]], cfg, with_stats=True)
        say("oracle read %d: %.2fs states %d fm %d (gpu states %d fm %d tier %d)" % (
            r, time.time() - t2, stt[0].states, stt[0].fm_searches, c[r, 5], c[r, 1], c[r, 12]))
    t2 = time.time()
    exp = oi.align([reads[i] for i in deep], cfg, threads=16)
    say("oracle on %d deep reads %.1fs, identical: %s" % (len(deep), time.time() - t2, exp == got))
    if exp != got:
        g, e = got.splitlines(), exp.splitlines()
        say("first diffs:", [(a, bb) for a, bb in zip(g, e) if a != bb][:3])


if __name__ == "__main__":
    main()
