"""overlap.py -- do two batches in flight on one GPU (two host threads, each batch on its own HIP
stream, as gwa_pipeline's workers run them) align faster than the same batches one after another?
Experiment tool, not part of libgwa or the bench.  C2 hg19 workload (bench.py's default), 10M reads
per batch; prints one JSON line per mode and whether the SAM text sizes agree.
  python tools/overlap.py [reads_per_batch] [rounds]
"""
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "genome-weaver-align_amd"), os.path.join(REPO, "tools"), REPO]

import numpy as np  # noqa: E402
import synth  # noqa: E402
import gwa  # noqa: E402
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    import torch
    torch.cuda.set_device(0)
    t0 = time.time()
    codes, names, lengths = synth.genome_ngaps(synth.HG19_CONTIGS, config_id=1)
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths, device=0)
    print("index %.1fs" % (time.time() - t0), file=sys.stderr, flush=True)
    cfg = gwa.AlignmentConfig(k=2.0, strategy="bsf")
    batches = []
    for r in range(2):
        blobs = bench.make_reads(synth, np, codes, lengths, n, 100, False, r)
        batches.append(gwa.Batch(gi, cfg, blobs=blobs))
    print("batches ready", file=sys.stderr, flush=True)

    def step(b, out, j):
        b.run()
        out[j] = b.format_device()

    for b in batches:  # warmup
        step(b, [0], 0)
    torch.cuda.synchronize()
    res = {}
    for mode in ("serial", "overlap", "serial", "overlap"):
        sizes = [0, 0]
        t0 = time.perf_counter()
        if mode == "serial":
            for _ in range(rounds):
                for j, b in enumerate(batches):
                    step(b, sizes, j)
        else:
            def worker(j):
                for _ in range(rounds):
                    step(batches[j], sizes, j)
            th = [threading.Thread(target=worker, args=(j,)) for j in range(2)]
            for t in th:
                t.start()
            for t in th:
                t.join()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        rate = 2 * rounds * n / dt
        res.setdefault(mode, []).append(rate)
        print(json.dumps({"mode": mode, "reads_per_s": rate, "ms_per_batch": dt / (2 * rounds) * 1e3,
                          "sam_bytes": sizes}), flush=True)
    print(json.dumps({"serial_best": max(res["serial"]), "overlap_best": max(res["overlap"]),
                      "ratio": max(res["overlap"]) / max(res["serial"])}), flush=True)
    for b in batches:
        b.close()


if __name__ == "__main__":
    main()
