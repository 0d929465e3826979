"""Diagnostic (GPU box): -m sf (or bsf) at k = 5 on the full-size hg19-like genome.  Runs a batch of C4
reads (per-tier reads and times with GWA_VERBOSE=1), then -- whether or not the batch finished --
the oracle on the heaviest reads, each in a child process with a state cap (ORC_MAX_STATES) and a
time limit, to show how far the reference algorithm gets on them; then the oracle on every read
that needed a tier >= 1 when the batch finished, SAM compared.

  python tools/diag_sf.py [reads] [strategy] [oracle reads] [state cap]

(oracle reads 0: the GPU batch only.)
"""
import multiprocessing as mp
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


_ORC = {}


def _orc_one(args):
    """child process: one read through the oracle with the state cap; (seconds, error or None, stats)"""
    read, strat, cap = args
    import oracle as O
    os.environ["ORC_MAX_STATES"] = str(cap)
    t0 = time.time()
    try:
        _, st = _ORC["oi"].align([read], O.OrcConfig.default(k=5.0, strategy=strat), with_stats=True)
        return time.time() - t0, None, (st[0].states, st[0].fm_searches, st[0].sw, st[0].max_heap)
    except RuntimeError as e:
        return time.time() - t0, str(e), None


def main():
    heartbeat()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    strat = sys.argv[2] if len(sys.argv) > 2 else "sf"
    n_orc = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    cap = int(sys.argv[4]) if len(sys.argv) > 4 else 20_000_000
    t0 = time.time()
    codes, names, lengths = synth.genome_repeats(synth.HG19_CONTIGS, config_id=1)
    say("genome %.0fs" % (time.time() - t0))
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths)
    say("index %.0fs" % (time.time() - t0))
    strs = synth.to_strings(synth.reads_codes(codes, lengths, n, 150, 2, config_id=4, indels=True, max_edits=5))
    reads = [("r%09d" % i, strs[i], "I" * 150) for i in range(n)]
    b = gwa.Batch(gi, gwa.AlignmentConfig(k=5.0, strategy=strat), reads)
    t1 = time.time()
    ok = True
    try:
        b.run()
    except gwa.GwaError as e:
        ok = False
        say("batch failed after %.1fs: %s" % (time.time() - t1, e))
    st = b.stats()
    c = b.read_counters()
    say("%s %d reads: %.2fs tiers %s tier_ms %s" % (strat, n, time.time() - t1, list(st.tier_reads),
                                                   [round(x) for x in st.tier_ms]))
    say("deepest tier per read:", {int(t): int((c[:, 12] == t).sum()) for t in np.unique(c[:, 12])})
    deep = np.nonzero(c[:, 12] >= 1)[0]
    if ok:
        top = np.argsort(-c[:, 5])[:12]
        say("heaviest reads (read, fm searches, states, tier):", [(int(i), int(c[i, 1]), int(c[i, 5]), int(c[i, 12])) for i in top])
        got, _ = b.results_select(deep.astype(np.uint32))
    heavy = [int(i) for i in np.argsort(-c[:, 12], kind="stable")[:n_orc]]
    b.close()
    if n_orc == 0:  # GPU side only (e.g. GWA_LIB=libgwa_prof.so: per-region cycles per tier)
        gi.close()
        return
    import oracle as O
    t0 = time.time()
    sa_f = gi.suffixArray(0)
    O.check_cyclic_sa_full(codes, sa_f, threads=16)
    sa_r = gi.suffixArray(1)
    O.check_cyclic_sa_full(np.ascontiguousarray(codes[::-1]), sa_r, threads=16)
    _ORC["oi"] = O.Index.from_arrays(codes, names, lengths, sa_f=sa_f, sa_r=sa_r)
    del sa_f, sa_r
    gi.close()
    say("SA check + oracle index %.0fs" % (time.time() - t0))
    strat_i = gwa.STRATEGIES[strat]
    ctx = mp.get_context("fork")  # (the oracle index is inherited; the child touches no GPU)
    with ctx.Pool(min(len(heavy), 8)) as pool:
        res = [pool.apply_async(_orc_one, ((reads[r], strat_i, cap),)) for r in heavy]
        for r, h in zip(heavy, res):
            try:
                secs, err, stt = h.get(timeout=400)
                say("oracle read %d (GPU tier %d): %.1fs %s" % (r, c[r, 12], secs, err or
                    "states %d fm %d sw %d max queue %d" % stt))
            except mp.TimeoutError:
                say("oracle read %d (GPU tier %d): not finished in 400 s" % (r, c[r, 12]))
        pool.terminate()
    if ok and len(deep):
        t2 = time.time()
        exp = _ORC["oi"].align([reads[i] for i in deep], O.OrcConfig.default(k=5.0, strategy=strat_i), threads=16)
        say("oracle on %d deep reads %.1fs, identical: %s" % (len(deep), time.time() - t2, exp == got))


if __name__ == "__main__":
    main()
