"""fv_isolate.py -- does the 400-bp -m sf loss of a flag-form variant library depend on
which reads share the batch?  Diagnostic tool (run with GWA_LIB=libgwa_fv_<v>.so), not a test.
The reads are test_long_reads_on_gpu[1-400-0.06]'s; prints one JSON line per arrangement: the reads
whose SAM line differs from the oracle's when run (a) as the whole batch, (b) the batch reversed,
(c) each lost read alone, (d) each lost read with the 8 reads before it, (e) with each other read (both lane
orders) and with 8 copies of itself.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "genome-weaver-align_amd"), os.path.join(REPO, "tools"), os.path.join(REPO, "oracle")]

import oracle as O  # noqa: E402
import synth  # noqa: E402
import gwa  # noqa: E402


def main():
    m, k = 400, 0.06
    codes, names, lengths = synth.genome([("c1", 300000), ("c2", 200000)], 1)
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths)
    oi = O.Index.from_arrays(codes, names, lengths)
    seqs, rn = synth.reads(codes, lengths, 60, m, 3, config_id=4 + m)
    strs = synth.to_strings(seqs)
    good = []
    for i, s_ in enumerate(strs):
        r = ("r%d" % i, s_, "I" * m)
        try:
            oi.align([r], O.OrcConfig.default(k=k, strategy=1))
            good.append(r)
        except RuntimeError:
            pass
    exp = {}
    for line in oi.align(good, O.OrcConfig.default(k=k, strategy=1)).splitlines():
        exp.setdefault(line.split("\t")[0], []).append(line)
    al = gwa.aligner(gi, gwa.AlignmentConfig(k=k, strategy="sf"))

    dbg = None
    if hasattr(gwa.lib(), "gwa_dbg_read"):  # instrumented variants: children taken with an empty interval
        import ctypes
        buf = (ctypes.c_uint * 4)()

        def dbg():
            assert gwa.lib().gwa_dbg_read(buf) == 0
            return [int(x) for x in buf]
        dbg()

    def lost(reads):
        got = {}
        for line in al.align_batch(reads).splitlines():
            got.setdefault(line.split("\t")[0], []).append(line)
        out = sorted((r[0] for r in reads if got.get(r[0]) != exp[r[0]]), key=lambda s: (len(s), s))
        if dbg:
            out.append(dict(zip(os.environ.get("GWA_DBG_NAMES", "c0,c1,c2,c3").split(","), dbg())))
        return out

    whole = lost(good)
    print(json.dumps({"arrangement": "whole batch", "reads": len(good), "lost": whole}), flush=True)
    print(json.dumps({"arrangement": "reversed", "lost": lost(good[::-1])}), flush=True)
    idx = {r[0]: j for j, r in enumerate(good)}
    whole = [x for x in whole if isinstance(x, str)]
    for name in whole:
        j = idx[name]
        print(json.dumps({"arrangement": "alone", "read": name, "lost": lost([good[j]])}), flush=True)
        print(json.dumps({"arrangement": "with 8 before", "read": name,
                          "lost": lost(good[max(0, j - 8):j + 1])}), flush=True)
    # pairs: each lost read with every other read, both lane orders; and with copies of itself
    for name in whole[:3] if os.environ.get("GWA_ISO_PAIRS", "1") != "0" else []:
        j = idx[name]
        first = [good[i][0] for i in range(len(good)) if i != j and name in lost([good[j], good[i]])]
        second = [good[i][0] for i in range(len(good)) if i != j and name in lost([good[i], good[j]])]
        copies = [(name + "c%d" % c, good[j][1], good[j][2]) for c in range(8)]
        for c in copies:
            exp[c[0]] = [l.replace(name + "\t", c[0] + "\t", 1) for l in exp[name]]
        if first:  # 32 copies in lanes 0-31 (or 1-32) and one partner: neighbours only, or every copy?
            partner = good[idx[first[0]]]
            many = [good[j]] + copies + [(name + "d%d" % c, good[j][1], good[j][2]) for c in range(23)]
            for c in many[9:]:
                exp[c[0]] = [l.replace(name + "\t", c[0] + "\t", 1) for l in exp[name]]
            print(json.dumps({"arrangement": "32 copies then partner", "read": name, "partner": partner[0],
                              "lost": lost(many + [partner])}), flush=True)
            print(json.dumps({"arrangement": "partner then 32 copies", "read": name, "partner": partner[0],
                              "lost": lost([partner] + many)}), flush=True)
        print(json.dumps({"arrangement": "pairs", "read": name, "partners_losing_it_when_first": first,
                          "partners_losing_it_when_second": second,
                          "copies_lost": lost([good[j]] + copies)}), flush=True)


if __name__ == "__main__":
    main()
