"""FASTQ file -> SAM file through gwa_pipeline_align_file on one resident index (GPU box): the same
file aligned under several (workers, batch) settings, each twice on one pipeline (cold: first use of
its buffers; warm: second pass).

  python tools/e2e_sweep.py [--genome hg19] [--reads 10000000] 2:1048576 3:1048576 ...
"""
import argparse
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "genome-weaver-align_amd"), os.path.join(REPO, "tools")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genome", default="hg19")
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("configs", nargs="+")
    a = ap.parse_args()
    import numpy as np
    import synth
    import gwa
    contigs = synth.HG19_CONTIGS if a.genome == "hg19" else [("chr%d" % (i + 1), int(float(a.genome) * 1e6 / 4))
                                                               for i in range(4)]
    codes, names, lengths = synth.genome(contigs, config_id=1)
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths, device=0)
    m, n = 100, a.reads
    seqs = synth.reads_codes(codes, lengths, n, m, 2, config_id=2, shard=0)
    name_blob, _ = synth.name_blob(n)
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    fq, so = os.path.join(d, "reads.fq"), os.path.join(d, "out.sam")
    rec = np.empty((n, 12 + m + 3 + m + 1), dtype=np.uint8)
    rec[:, 0] = ord("@")
    rec[:, 1:11] = np.frombuffer(name_blob, dtype=np.uint8).reshape(n, 10)
    rec[:, 11] = ord("\n")
    rec[:, 12:12 + m] = synth.SYM[seqs]
    rec[:, 12 + m:15 + m] = np.frombuffer(b"\n+\n", dtype=np.uint8)
    rec[:, 15 + m:15 + 2 * m] = ord("I")
    rec[:, 15 + 2 * m] = ord("\n")
    with open(fq, "wb") as f:
        f.write(rec.data)
    del rec, seqs
    for c in a.configs:
        w, b = (int(x) for x in c.split(":"))
        p = gwa.Pipeline([gi], gwa.AlignmentConfig(k=2.0), batch_reads=b, workers_per_device=w)
        for leg in ("cold", "warm"):
            with open(so, "wb") as f:
                t0 = time.perf_counter()
                got = p.align_file(fq, f.fileno())
                dt = time.perf_counter() - t0
            st = p.stats()
            print("workers=%d batch=%d %s: %.2f M reads/s (%.3f s) read %.2f frame %.2f setup %.2f kernels %.2f "
                  "format %.2f write %.2f wait %.2f" % (w, b, leg, got / dt / 1e6, dt, st.read_s, st.frame_s, st.setup_s,
                                                       st.device_kernel_s[0], st.format_s, st.write_s, st.order_wait_s),
                  flush=True)
        p.close()
    for x in (fq, so):
        os.remove(x)
    os.rmdir(d)


if __name__ == "__main__":
    main()
