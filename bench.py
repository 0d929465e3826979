"""bench.py -- reads/s of the MI355X `align -m bsf` path (BASELINE.json metric).

One step = one pass of the hot path (fm_quickscan + bsf_search tiers) over one batch of synthetic
100 bp reads already resident in HBM.  Weak scaling: every rank holds a full index replica on its
own GPU and aligns its own shard; value = total reads of all ranks / max-over-ranks time.

  python bench.py [--gpus N --steps K --warmup W] [--genome hg19|ecoli|<Mbp>] [--reads R]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "genome-weaver-align_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

METRIC = "reads/sec (whole node), 100 bp k≤2 vs hg19, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def _pmc_traffic(kernel, workload):
    """Per-launch HBM read bytes of `kernel` from the newest committed rocprofv3 PMC summary of the
    same workload (profiles/*_profile.json, written by tools/prof_summary.py from FETCH_SIZE, see
    profiles/README.md for the correction); (None, None) when no profile of this workload exists.
    "Newest" is by round tag in the file name (r01 < r01c < r01d ...): file mtimes do not survive a
    checkout."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_profile.json")), key=os.path.basename):
        try:
            d = json.load(open(f))
            line = d.get("bench_lines", {}).get("bench.json", {})
            k = d["kernels"][kernel + "_kernel"]
        except (OSError, ValueError, KeyError):
            continue
        if line.get("config", {}).get("workload") == workload and "hbm_read_bytes_corrected" in k:
            best = (k["hbm_read_bytes_corrected"], os.path.relpath(f, REPO))
    return best if best else (None, None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--genome", default=os.environ.get("GWA_BENCH_GENOME", "hg19"))
    ap.add_argument("--reads", type=int, default=int(os.environ.get("GWA_BENCH_READS", "0")))
    ap.add_argument("--k", type=float, default=None, help="max edits (default: 2 for c2, 5 for c4)")
    ap.add_argument("--workload", default="c2", choices=["c2", "c4"],
                    help="c2: 100 bp, 0-2 substitutions (the BASELINE metric); c4: 150 bp, 0-5 edits with indels")
    ap.add_argument("--strategy", default="bsf", choices=["bsf", "sf"], help="-m (align strategy)")
    ap.add_argument("--cpu-sample", type=int, default=int(os.environ.get("GWA_CPU_SAMPLE", "20000")),
                    help="reads of the single-thread CPU baseline")
    ap.add_argument("--cpu-threads", type=int, default=min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
                                                           or (os.cpu_count() or 1)),
                    help="host threads of the multi-core CPU baseline (SURVEY.md 8(d)(ii))")
    ap.add_argument("--cpu-sample-mt", type=int, default=int(os.environ.get("GWA_CPU_SAMPLE_MT", "160000")),
                    help="reads of the multi-core CPU baseline")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--check", type=int, default=2000, help="reads of step 0 checked against the oracle")
    ap.add_argument("--no-pipeline", action="store_true", help="skip the host-pipeline (FASTQ-to-SAM) leg")
    args = ap.parse_args()

    import numpy as np
    import synth
    import gwa
    import dist as gdist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        tdist.init_process_group("gloo")
    import torch
    torch.cuda.set_device(local)

    if args.genome == "hg19":
        contigs, gname = synth.HG19_CONTIGS, "hg19-size synthetic (i.i.d. ACGT, hg19 contig lengths)"
    elif args.genome == "ecoli":
        contigs, gname = synth.ECOLI, "E. coli-size synthetic (4,641,652 bp i.i.d. ACGT)"
    else:
        mb = float(args.genome)
        contigs = [("chr%d" % (i + 1), int(mb * 1e6 / 4)) for i in range(4)]
        gname = "%g Mbp synthetic (4 contigs, i.i.d. ACGT)" % mb
    c4 = args.workload == "c4"
    if args.k is None:
        args.k = 5.0 if c4 else 2.0
    reads_per_step = args.reads or (1_000_000 if c4 else 10_000_000 if args.genome == "hg19" else 1_000_000)

    t0 = time.time()
    codes, names, lengths = synth.genome(contigs, config_id=1)
    log("genome %d bp generated in %.1fs" % (len(codes), time.time() - t0))
    t0 = time.time()
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths, device=local)
    t_index = time.time() - t0
    log("index built + resident in HBM: %.1fs, %.2f GB" % (t_index, gi.deviceBytes() / 1e9))

    cfg = gwa.AlignmentConfig(k=args.k, strategy=args.strategy)
    # synthetic reads: C2 100 bp with 0-2 substitutions; C4 150 bp with 0-5 edits,
    # 60 % substitutions / 20 % 1-bp insertions / 20 % 1-bp deletions; shard = rank
    m = 150 if c4 else 100
    t0 = time.time()
    seqs = synth.reads_codes(codes, lengths, reads_per_step, m, 2, config_id=4 if c4 else 2, shard=rank,
                             indels=c4, max_edits=5)
    seq_blob = synth.SYM[seqs].tobytes()
    seq_off = np.arange(0, m * (reads_per_step + 1), m, dtype=np.uint64)
    name_blob, name_off = synth.name_blob(reads_per_step)
    qual_blob = b"I" * (m * reads_per_step)
    log("reads generated in %.1fs" % (time.time() - t0))
    t0 = time.time()
    batch = gwa.Batch(gi, cfg, blobs=(name_blob, name_off, seq_blob, seq_off, qual_blob, seq_off))
    log("batch resident in HBM: %.1fs" % (time.time() - t0))
    nchk = min(max(args.check, max(args.cpu_sample, args.cpu_sample_mt) if not args.no_cpu else 0), reads_per_step)
    reads = [(name_blob[10 * i:10 * i + 10].decode(), seq_blob[m * i:m * i + m].decode(), "I" * m) for i in range(nchk)]

    for _ in range(args.warmup):
        batch.run()

    def barrier():
        if dist:
            tdist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kms = qms = sms = 0.0
    for _ in range(args.steps):
        batch.run()
        st = batch.stats()
        kms += st.kernel_ms
        qms += st.quickscan_ms
        sms += st.search_ms
    torch.cuda.synchronize()
    barrier()
    dt = gdist.max_over_ranks(time.perf_counter() - t0)

    # host pipeline (first bullet): the whole path for one batch outside the timed
    # region -- reads from host memory to HBM (batch create), kernels, records back to the host and SAM
    # text formatted (16 host threads) -- reported beside `value`, never as it
    pipe = None
    if rank == 0 and not args.no_pipeline:
        t0 = time.perf_counter()
        b2 = gwa.Batch(gi, cfg, blobs=(name_blob, name_off, seq_blob, seq_off, qual_blob, seq_off))
        t1 = time.perf_counter()
        b2.run()
        t2 = time.perf_counter()
        nbytes = b2.sam_size()
        t3 = time.perf_counter()
        b2.close()
        pipe = {"reads_per_s": reads_per_step / (t3 - t0), "h2d_setup_s": t1 - t0, "kernels_s": t2 - t1,
                "d2h_sam_format_s": t3 - t2, "sam_bytes": nbytes,
                "note": "one batch, host read blobs -> HBM -> kernels -> host SAM text; index load excluded"}
        log("host pipeline: %.0f reads/s (setup %.2fs, kernels %.2fs, SAM %.2fs, %.2f GB)"
            % (pipe["reads_per_s"], t1 - t0, t2 - t1, t3 - t2, nbytes / 1e9))

    nres = min(args.check, reads_per_step)
    sam, off = batch.results(0, nres)
    st = batch.stats()
    total_reads = reads_per_step * args.steps * world
    value = total_reads / dt

    # parity spot check of this rank's first reads against the oracle (checker only)
    parity = None
    if args.check and rank == 0:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle as O
        t0 = time.time()
        oi = O.Index.from_arrays(codes, names, lengths, sa_f=gi.suffixArray(0), sa_r=gi.suffixArray(1))
        t_oidx = time.time() - t0
        nchk = nres
        exp = oi.align(reads[:nchk], O.OrcConfig.default(k=args.k, strategy=gwa.STRATEGIES[args.strategy]))
        got = sam
        parity = {"reads": nchk, "identical": got == exp}
        log("parity on %d reads: %s (oracle index %.1fs)" % (nchk, got == exp, t_oidx))

    # CPU baseline: the oracle (single-thread C++ restatement of the reference path) on this host.
    # (i) 1 thread, as the reference runs (A/Align.java:174-196); (ii) T threads over contiguous read
    # ranges.  cpu_baseline reports (ii); (i) is kept in detail.
    cpu = cpu1 = None
    if rank == 0 and not args.no_cpu and args.cpu_sample > 0:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle as O
        if parity is None:
            oi = O.Index.from_arrays(codes, names, lengths, sa_f=gi.suffixArray(0), sa_r=gi.suffixArray(1))
        ns = min(args.cpu_sample, len(reads))
        t0 = time.perf_counter()
        oi.align(reads[:ns], O.OrcConfig.default(k=args.k, strategy=gwa.STRATEGIES[args.strategy]))
        ct = time.perf_counter() - t0
        model = "unknown CPU"
        try:
            with open("/proc/cpuinfo") as f:
                model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), model)
        except OSError:
            pass
        cpu1 = {"value": ns / ct, "unit": "reads/s", "cores": 1, "kind": "port",
                "sample": "first %d reads of rank 0's batch, single-thread C++ restatement of the reference "
                          "%s path (oracle/; CPU restatement, not the JVM), same index; %s"
                          % (ns, args.strategy.upper(), model)}
        log("cpu baseline (1 thread): %.0f reads/s (%d reads in %.1fs)" % (ns / ct, ns, ct))
        cpu = cpu1
        T = max(1, args.cpu_threads)
        nt = min(args.cpu_sample_mt, len(reads))
        if T > 1 and nt > 0:
            t0 = time.perf_counter()
            oi.align(reads[:nt], O.OrcConfig.default(k=args.k, strategy=gwa.STRATEGIES[args.strategy]), threads=T)
            ct = time.perf_counter() - t0
            cpu = {"value": nt / ct, "unit": "reads/s", "cores": T, "kind": "port",
                   "sample": "first %d reads of rank 0's batch on %d host threads (contiguous ranges, one "
                             "Aligner each), C++ restatement of the reference %s path (oracle/; CPU "
                             "restatement, not the JVM), same index; %s" % (nt, T, args.strategy.upper(), model)}
            log("cpu baseline (%d threads): %.0f reads/s (%d reads in %.1fs)" % (T, nt / ct, nt, ct))

    # roofline of the dominant kernel.  Algorithmic bytes = the bytes this path's algorithm must read
    # (DESIGN.md §5): 64 B per Occ block of every FM step that reads one, 8 B per k-mer interval-table
    # lookup, 3/8 B (2-bit base + N bit) per FM step answered from the text (single-row interval),
    # 4 B per suffix-array gather.  `ref_equiv_bytes` prices every reference FM step at the SURVEY.md
    # §8d lower bound of one 64-B block instead (what the reference's algorithm would read).
    steps = args.steps
    q_ms, s_ms = qms / steps, sms / steps
    q_bytes = 64.0 * st.quick_blocks + 8.0 * st.kmer_lookups + 0.375 * st.quick_short_steps + 4.0 * st.quick_sa_reads
    q_ref = 64.0 * (st.quick_blocks + st.quick_short_steps) + 4.0 * st.quick_sa_reads
    s_bytes = (64.0 * (st.blocks - st.quick_blocks) + 0.375 * st.search_short_steps
               + 4.0 * (st.sa_reads - st.quick_sa_reads))
    s_ref = 64.0 * (st.blocks - st.quick_blocks + st.search_short_steps) + 4.0 * (st.sa_reads - st.quick_sa_reads)
    if q_ms >= s_ms:
        dom, ach_bytes, dom_ms, dom_ref = "fm_quickscan", q_bytes, q_ms, q_ref
    else:
        dom, ach_bytes, dom_ms, dom_ref = args.strategy + "_search", s_bytes, s_ms, s_ref
    achieved = ach_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    workload = ("%s; %d x %d bp reads per GPU per step, %s, -k %g, -m %s, besthit"
                % (gname, reads_per_step, m, "0-5 edits (subs/1-bp indels)" if c4 else "0-2 substitutions", args.k,
                   args.strategy))
    traffic, traffic_src = _pmc_traffic(dom, workload)
    out = {
        "metric": METRIC if not c4 else "reads/sec, 150 bp k<=5 with indels vs hg19 (config C4)", "value": value, "unit": "reads/s", "n_gpus": world, "steps": steps,
        "warmup": args.warmup, "ms_per_step": dt * 1e3 / steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "config": {"workload": workload,
                   "genome_bp": int(len(codes)), "reads_per_gpu_per_step": reads_per_step,
                   "parallelism": "reads sharded, index replicated (%d GPU)" % world},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": ach_bytes, "avg_launch_ms": dom_ms,
                     "ref_equiv_bytes_per_launch": dom_ref},
        "cpu_baseline": cpu,
        "detail": {"quickscan_ms": q_ms, "search_ms": s_ms, "kernel_ms": kms / steps,
                   "fm_searches_per_read": st.fm_searches / reads_per_step,
                   "quick_steps_per_read": st.quick_steps / reads_per_step,
                   "blocks_per_read": st.blocks / reads_per_step, "tier_reads": list(st.tier_reads),
                   "tier_ms": [round(x, 3) for x in st.tier_ms],
                   "quick_short_steps_per_read": st.quick_short_steps / reads_per_step,
                   "cpu_baseline_1thread": cpu1, "host_pipeline": pipe,
                   "search_short_steps_per_read": st.search_short_steps / reads_per_step,
                   "rank_kernel": {"kernel": "fm_quickscan", "algorithmic_bytes_per_launch": q_bytes,
                                   "ref_equiv_bytes_per_launch": q_ref, "avg_launch_ms": q_ms,
                                   "achieved_GBs": q_bytes / (q_ms * 1e-3) / 1e9 if q_ms > 0 else 0.0,
                                   "frac": (q_bytes / (q_ms * 1e-3) / 1e9 if q_ms > 0 else 0.0) / HBM_PEAK_GBS,
                                   "traffic": _pmc_traffic("fm_quickscan", workload)[0]},
                   "mapped": st.n_mapped, "unmapped": st.n_unmapped, "index_build_s": t_index,
                   "index_gb": gi.deviceBytes() / 1e9, "parity": parity},
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    batch.close()
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
