"""GPU debug run of one parity case (repetitive genome): SAM + per-read trace of one read."""
import os
import sys
sys.path[:0] = ['genome-weaver-align_amd', 'oracle', 'tools', 'tests', 'tests/hostcore']
import numpy as np
import gwa
from test_hostcore import _mk

READ = int(os.environ.get("DBG_READ", "42"))
rng = np.random.default_rng(11)
seg = rng.integers(0, 4, 3000).astype(np.uint8)
parts = []
for i in range(40):
    s = seg.copy()
    mut = rng.integers(0, 3000, rng.integers(0, 60))
    s[mut] = rng.integers(0, 4, len(mut))
    parts.append(s)
    parts.append(rng.integers(0, 4, rng.integers(10, 2000)).astype(np.uint8))
    if i % 7 == 0:
        parts.append(np.full(rng.integers(1, 50), 4, np.uint8))
    if i % 5 == 0:
        parts.append(np.tile(rng.integers(0, 4, rng.integers(1, 6)).astype(np.uint8), 40))
codes = np.concatenate(parts)
L = len(codes)
names, lengths = ["chrA", "chrB", "chr10"], [L // 3, L // 3, L - 2 * (L // 3)]
reads = _mk(codes, 400, 100, 5, True, seed=100 * 7 + 1)
if len(sys.argv) > 1 and sys.argv[1] == "cpu":
    import hostcore
    os.environ["GWA_TRACE_READ"] = str(READ)
    hc = hostcore.HostCore(codes, names, lengths)
    sam = hc.align(reads, k=0.1)
    open("gpurun_out/cpu_rep.sam", "w").write(sam if isinstance(sam, str) else "".join(sam))
    print("cpu done")
else:
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths, device=0)
    os.environ["GWA_TRACE_READ"] = str(READ)
    os.environ["GWA_TRACE_FILE"] = "gpurun_out/gpu_trace.bin"
    b = gwa.Batch(gi, gwa.AlignmentConfig(k=0.1), reads)
    b.run()
    sam, off = b.results()
    open('gpurun_out/gpu_rep.sam', 'w').write(sam if isinstance(sam, str) else "".join(sam))
    np.save('gpurun_out/gpu_rep_counters.npy', b.read_counters())
    print("gpu done", b.stats().tier_reads[:])
    if os.path.exists("dbg_cpu_rep.sam"):
        exp = open("dbg_cpu_rep.sam").read().splitlines()
        got = (sam if isinstance(sam, str) else "".join(sam)).splitlines()
        print("lib", os.environ.get("GWA_LIB", "libgwa.so"), "diff lines:", sum(1 for a, b in zip(exp, got) if a != b), len(exp), len(got))
