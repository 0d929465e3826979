"""bench.py -- reads/s of the MI355X `align -m bsf` path (BASELINE.json metric).

One step = the whole device path over one batch of synthetic 100 bp reads whose text is already
resident in HBM: encode the read text (gwa_batch_run starts from it, as the reference's per-read
call starts from the Read's String), fm_quickscan + bsf_search tiers, and the SAM text of every read
written in HBM (gwa_batch_format; A/Align.java:187-195 -> A/SAMOutput.java:73-82).  Weak scaling:
every rank holds a full index replica on its own GPU and aligns its own shard; value = total reads
of all ranks / max-over-ranks time.  At N = 1 the default run adds detail.hg19r, the same step on the
hg19-like repetitive genome.

  python bench.py [--gpus N --steps K --warmup W] [--genome hg19|hg19r|ecoli|<Mbp>] [--reads R]

--gpus N > 1 without a torch.distributed environment re-launches this script under
`torch.distributed.run` with N ranks (before anything touches the GPU); ranks beyond the visible GPU
count share GPUs round-robin (each rank keeps its own index replica).
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


# the one JSON line goes here (main points fd 1 at stderr for everything else)
JSON_OUT = sys.stdout


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def _pmc_traffic(kernel, workload):
    """Per-launch HBM read (+ write, when measured) bytes of `kernel` from the newest committed rocprofv3 PMC summary of the
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
            # read + write fabric request bytes when the profile has a WRITE_SIZE pass (round 4 on)
            best = (k["hbm_read_bytes_corrected"] + k.get("hbm_write_bytes", 0.0), os.path.relpath(f, REPO))
    return best if best else (None, None)


def host_cores():
    """(cores this process may use, description): the CPU affinity set, capped by a cgroup v2 CPU
    quota when one is set (a GPU box grants each job a share of the host)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    n = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    return n, "affinity %d CPUs, cgroup quota %s" % (aff, "none" if quota is None else "%.1f CPUs" % quota)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            return next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "unknown CPU")
    except OSError:
        return "unknown CPU"


def spawn_ranks(args):
    """--gpus N outside torch.distributed: run N ranks of this script under torch.distributed.run and
    exit with its status (this process never initialises the GPU)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log("launching %d ranks: %s" % (args.gpus, " ".join(cmd)))
    sys.exit(subprocess.call(cmd))


# The chip's random-gather ceiling (tools/gather_roof.hip on MI355X, profiles/r02_gather_roof.json):
# independent random 64-B blocks (4 x 16-B loads) and random 8-B words over a 32 GiB buffer, the
# grid filling the chip; the rate does not change with 1-8 gathers in flight per lane.
GATHER_BLOCK64_PER_S = 19.17e9
GATHER_WORD8_PER_S = 47.96e9


def gather_ceiling(st, q_ms):
    """fm_quickscan against the random-gather roofline: the shortest time its gathers could take at
    the measured ceilings (Occ blocks at the block rate; k-mer entries, SA values and 2 words per
    text-mode run -- one 2-bit text line and one N-flag line -- at the word rate) over its time."""
    words = st.kmer_lookups + st.quick_sa_reads + 2 * st.quick_text_runs
    t_min_ms = (st.quick_blocks / GATHER_BLOCK64_PER_S + words / GATHER_WORD8_PER_S) * 1e3
    return {"source": "profiles/r02_gather_roof.json (tools/gather_roof.hip)",
            "note": "DRAM-miss ceiling: frac > 1 means part of the gathers hit L2 / MALL (62 % L2 hits in profiles/r02_hg19_profile.json)",
            "block64_per_s": GATHER_BLOCK64_PER_S, "word8_per_s": GATHER_WORD8_PER_S,
            "blocks": int(st.quick_blocks), "words": int(words), "text_runs": int(st.quick_text_runs),
            "min_ms": t_min_ms, "avg_launch_ms": q_ms, "frac": t_min_ms / q_ms if q_ms > 0 else 0.0}


def rank_kernel_entry(st, q_ms, q_ref, q_bytes, workload, gbs):
    """detail.rank_kernel: fm_quickscan (the Occ/rank kernel north_star names) against the HBM peak.
    `frac` is the counter-derived fraction -- the FETCH_SIZE + WRITE_SIZE bytes per launch of the newest
    committed profile of this workload (profiles/README.md calibration) over this run's launch time --
    because SURVEY.md 8(d)'s algorithmic bytes price every reference FM step as an Occ block read and the
    kernel answers most of them from the k-mer table and 32-base text runs: that figure is a rate of
    reference work (`reference_work_rate_vs_peak`, above 1), not a roofline fraction."""
    traffic, src = _pmc_traffic("fm_quickscan", workload)
    return {"kernel": "fm_quickscan", "definition": "rocprofv3 FETCH_SIZE + WRITE_SIZE bytes per launch / launch time",
            "frac": (gbs(traffic, q_ms) / HBM_PEAK_GBS) if traffic else None,
            "achieved_GBs": gbs(traffic, q_ms) if traffic else None, "traffic": traffic, "traffic_source": src,
            "avg_launch_ms": q_ms,
            "algorithmic_bytes_per_launch": q_ref, "algorithmic_GBs": gbs(q_ref, q_ms),
            "reference_work_rate_vs_peak": gbs(q_ref, q_ms) / HBM_PEAK_GBS,
            "kernel_bytes_per_launch": q_bytes, "kernel_bytes_GBs": gbs(q_bytes, q_ms),
            "kernel_bytes_frac": gbs(q_bytes, q_ms) / HBM_PEAK_GBS,
            "gather_ceiling": gather_ceiling(st, q_ms)}


def median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def cpu_baselines(oi, read_tuple, n_avail, strategy, k, args, O, label):
    """The oracle (C++ restatement of the reference path) on this host, each leg the median of 3
    runs: (i) 1 thread, as the reference runs (A/Align.java:174-196); (ii) every core this process
    may use, contiguous read ranges.  -> (cpu_baseline, cpu_baseline_1thread)."""
    T, tdesc = host_cores()
    if args.cpu_threads:
        T = args.cpu_threads
    model = cpu_model()
    ocfg = O.OrcConfig.default(k=k, strategy=strategy)
    ns = min(args.cpu_sample, n_avail)
    r1 = [read_tuple(i) for i in range(ns)]
    runs = []
    for _ in range(3):
        t0 = time.perf_counter()
        oi.align(r1, ocfg)
        runs.append(time.perf_counter() - t0)
    ct = median(runs)
    cpu1 = {"value": ns / ct, "unit": "reads/s", "cores": 1, "kind": "port", "seconds": ct,
            "runs_s": runs, "sample": "first %d reads of rank 0's batch, single-thread C++ restatement of the "
                                     "reference %s path (oracle/; CPU restatement, not the JVM), same index; median "
                                     "of 3 runs; %s" % (ns, label, model)}
    log("cpu baseline (1 thread): %.0f reads/s (%d reads, median of %s s)" % (ns / ct, ns, ["%.2f" % x for x in runs]))
    cpu = cpu1
    if T > 1:
        nt = int(min(n_avail, max(ns, args.cpu_seconds * cpu1["value"] * T)))
        rt = r1 + [read_tuple(i) for i in range(ns, nt)]
        runs = []
        for _ in range(3):
            t0 = time.perf_counter()
            oi.align(rt, ocfg, threads=T)
            runs.append(time.perf_counter() - t0)
        ct = median(runs)
        cpu = {"value": nt / ct, "unit": "reads/s", "cores": T, "kind": "port", "seconds": ct, "runs_s": runs,
               "sample": "first %d reads of rank 0's batch on %d host threads (%s; contiguous ranges, one Aligner "
                         "each), C++ restatement of the reference %s path (oracle/; CPU restatement, not the JVM), "
                         "same index; median of 3 runs; %s" % (nt, T, tdesc, label, model)}
        log("cpu baseline (%d threads): %.0f reads/s (%d reads, median of %s s)"
            % (T, nt / ct, nt, ["%.2f" % x for x in runs]))
    return cpu, cpu1


def timed_steps(batch, steps, warmup, barrier):
    """W untimed and K timed steps of the whole device path (gwa_batch_run = encode + fm_quickscan +
    search tiers, then gwa_batch_format = SAM text in HBM), bracketed by barrier + synchronize.
    -> (this rank's seconds, window, per-kernel ms sums, last stats)"""
    import torch
    for _ in range(warmup):
        batch.run()
        batch.format_device()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    win0 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)  # the rocprofv3 trace's clock (tools/prof_summary.py)
    acc = dict(encode=0.0, quickscan=0.0, search=0.0, format=0.0, kernel=0.0)
    sam_bytes = 0
    st = None
    for _ in range(steps):
        batch.run()
        sam_bytes = batch.format_device()
        st = batch.stats()
        acc["encode"] += st.encode_ms
        acc["quickscan"] += st.quickscan_ms
        acc["search"] += st.search_ms
        acc["format"] += st.format_ms
        acc["kernel"] += st.kernel_ms
    torch.cuda.synchronize()
    barrier()
    mine = time.perf_counter() - t0
    win1 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
    return mine, [win0, win1], {k: v / max(1, steps) for k, v in acc.items()}, st, sam_bytes


def make_reads(synth, np, codes, lengths, n, m, c4, rank):
    """Synthetic reads: C2 100 bp with 0-2 substitutions; C4 150 bp with 0-5 edits,
    60 % substitutions / 20 % 1-bp insertions / 20 % 1-bp deletions; shard = rank."""
    seqs = synth.reads_codes(codes, lengths, n, m, 2, config_id=4 if c4 else 2, shard=rank, indels=c4, max_edits=5)
    seq_blob = synth.SYM[seqs].tobytes()
    del seqs
    seq_off = np.arange(0, m * (n + 1), m, dtype=np.uint64)
    name_blob, name_off = synth.name_blob(n)
    qual_blob = b"I" * (m * n)
    return (name_blob, name_off, seq_blob, seq_off, qual_blob, seq_off)


def write_fastq(np, path, name_blob, seq_blob, n, m):
    """reads as a FASTQ file: "@r%09d\n" seq "\n+\n" qual "\n" """
    rec = np.empty((n, 12 + m + 3 + m + 1), dtype=np.uint8)
    rec[:, 0] = ord("@")
    rec[:, 1:11] = np.frombuffer(name_blob, dtype=np.uint8).reshape(n, 10)
    rec[:, 11] = ord("\n")
    rec[:, 12:12 + m] = np.frombuffer(seq_blob, dtype=np.uint8).reshape(n, m)
    rec[:, 12 + m:15 + m] = np.frombuffer(b"\n+\n", dtype=np.uint8)
    rec[:, 15 + m:15 + 2 * m] = ord("I")
    rec[:, 15 + 2 * m] = ord("\n")
    with open(path, "wb") as f:
        f.write(rec.data)


def host_ceiling_leg(args, gwa, synth, np, log, handles=4):
    """detail.host_ceiling: what the host side of gwa_pipeline_align_file (read, frame, H2D, D2H of the
    SAM text, ordered writes) sustains when the devices are not the limit: 10M exact 100 bp reads of an
    E. coli-size genome (-k 0: the quick scan ends every read, so the kernels take a few ms per batch and
    the SAM lines are C2-sized) through `handles` index replicas on this GPU, 3 workers each.  The
    C2 device rate times the GPU count a node needs is to be compared with it."""
    import tempfile
    n, m = 10_000_000, 100
    codes, names, lengths = synth.genome(synth.ECOLI, config_id=1)
    seqs = synth.reads_codes(codes, lengths, n, m, 0, config_id=11)
    seq_blob = synth.SYM[seqs].tobytes()
    del seqs
    name_blob, _ = synth.name_blob(n)
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    fq, so = os.path.join(d, "reads.fq"), os.path.join(d, "out.sam")
    write_fastq(np, fq, name_blob, seq_blob, n, m)
    del seq_blob, name_blob
    gis = [gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths) for _ in range(handles)]
    pipe = gwa.Pipeline(gis, gwa.AlignmentConfig(k=0.0), workers_per_device=3)
    legs = []
    for _ in range(2):
        with open(so, "wb") as f:
            t0 = time.perf_counter()
            got = pipe.align_file(fq, f.fileno())
            legs.append(time.perf_counter() - t0)
    pst = pipe.stats()
    sam_bytes = os.path.getsize(so)
    pipe.close()
    for g in gis:
        g.close()
    T, tdesc = host_cores()
    procs = shard_processes_leg(np, synth, codes, names, lengths, d, fq, so, got, handles, log)
    for x in (fq, so):
        os.remove(x)
    os.rmdir(d)
    out = {"reads_per_s": got / legs[1], "seconds": legs[1], "first_pass_seconds": legs[0], "reads": got,
           "handles": handles, "workers": 3 * handles, "host_cores": T, "sam_bytes": sam_bytes,
           "sam_GBps": sam_bytes / legs[1] / 1e9, "fastq_GBps": got * (2 * m + 15) / legs[1] / 1e9,
           "stages_s": {"read": pst.read_s, "frame": pst.frame_s, "setup": pst.setup_s,
                        "kernels": sum(pst.device_kernel_s[:handles]), "sam_format_d2h": pst.format_s,
                        "write": pst.write_s, "order_wait": pst.order_wait_s},
           "two_processes": procs,
           "note": "FASTQ file -> SAM file through gwa_pipeline_align_file with %d index replicas (E. coli-size, "
                   "-k 0, exact reads) on one GPU: the host side's ceiling on %s; second pass" % (handles, tdesc)}
    if isinstance(procs, dict) and "reads_per_s" in procs:
        procs["vs_one_process"] = procs["reads_per_s"] / out["reads_per_s"]
    log("host ceiling: %.1f M reads/s (%d handles, %.1f GB/s SAM out)" % (out["reads_per_s"] / 1e6, handles, out["sam_GBps"]))
    return out


def shard_processes_leg(np, synth, codes, names, lengths, d, fq, one_sam, n, handles, log, nproc=2):
    """detail.host_ceiling.two_processes: the same file through `nproc` processes at once, each running
    `gwa align --shard r/nproc` (its contiguous shard of the file, its own SAM file: DESIGN.md §6's per-rank
    sink) with handles / nproc index replicas; each process aligns its shard twice (--warm-passes 2: the
    first pass into /dev/null) and the rate is all reads over the slowest process's second pass (index load
    and the first pass excluded, as the one-process legs' second pass), and the shard files concatenated
    must equal the one-process SAM."""
    import hashlib
    import subprocess
    ref = os.path.join(d, "ref.fa")
    with open(ref, "w") as f:
        f.write(synth.fasta_text(codes, names, lengths))
    cli = os.path.join(REPO, "genome-weaver-align_amd", "gwa_cli.py")
    per = max(1, handles // nproc)
    outs, ps = [], []
    sync = os.path.join(d, "sync")
    os.makedirs(sync, exist_ok=True)
    t0 = time.perf_counter()
    for r in range(nproc):
        o = os.path.join(d, "shard%d.sam" % r)
        outs.append(o)
        with open(o, "wb") as fo:
            ps.append(subprocess.Popen([sys.executable, cli, "align", "-r", ref, "-k", "0", "--devices", ",".join(["0"] * per),
                                        "--workers", "3", "--timing", "--warm-passes", "2", "--sync", "%s:%d" % (sync, nproc),
                                        "--shard", "%d/%d" % (r, nproc), fq],
                                       stdout=fo, stderr=subprocess.PIPE, text=True))
    errs = [p.communicate()[1] for p in ps]
    wall = time.perf_counter() - t0
    align_s, spans, stages = [], [], []
    for p, e in zip(ps, errs):
        if p.returncode != 0:
            return {"error": "shard process exited %d: %s" % (p.returncode, e[-400:])}
        line = [x for x in e.splitlines() if "align (read file -> SAM" in x][-1]
        align_s.append(float(line.split("index load excluded) ")[1].split("s")[0]))
        mono = [x for x in e.splitlines() if "timed pass monotonic_ns" in x][-1].split()
        spans.append((int(mono[-2]), int(mono[-1])))
        # the process's own stage seconds (gwa_cli --timing: pipeline wall, read, frame; summed over its workers:
        # parse, set-up, kernels, SAM format + D2H, write, order wait)
        pl = [x for x in e.splitlines() if x.startswith("[gwa] pipeline ")]
        if pl:
            import re
            v = [float(x) for x in re.findall(r"([0-9]+\.[0-9]+)s", pl[-1])]
            stages.append(dict(zip(["wall", "read", "frame", "parse", "set_up", "sam_format_d2h", "write", "order_wait"],
                                   v[:3] + v[3:5] + v[-3:])))
    union_s = (max(b for _, b in spans) - min(a for a, _ in spans)) / 1e9
    overlap_s = max(0.0, (min(b for _, b in spans) - max(a for a, _ in spans)) / 1e9)

    def digest(paths):
        h = hashlib.sha256()
        for pth in paths:
            with open(pth, "rb") as f:
                for blk in iter(lambda: f.read(1 << 24), b""):
                    h.update(blk)
        return h.hexdigest()
    # the one-process SAM has no header (pipeline output); shard 0 starts with the CLI's header
    hdr = gwa_header_len(outs[0])
    with open(outs[0], "rb") as f0, open(os.path.join(d, "shard0.body"), "wb") as fb:
        f0.seek(hdr)
        for blk in iter(lambda: f0.read(1 << 24), b""):
            fb.write(blk)
    same = digest([os.path.join(d, "shard0.body")] + outs[1:]) == digest([one_sam])
    for x in outs + [os.path.join(d, "shard0.body"), ref]:
        os.remove(x)
    import shutil
    shutil.rmtree(sync, ignore_errors=True)
    out = {"processes": nproc, "handles_per_process": per, "reads_per_s": n / union_s, "align_s": align_s,
           "timed_union_s": union_s, "timed_overlap_s": overlap_s, "stages_s": stages,
           "wall_s_incl_start_and_index": wall, "concatenation_identical_to_one_process": same,
           "note": "gwa align --shard r/%d in %d processes on one GPU, each writing its own SAM shard; warm second pass "
                   "(--warm-passes 2), started together (--sync), index load excluded; reads_per_s = all reads over the "
                   "union of the timed passes (CLOCK_MONOTONIC)" % (nproc, nproc)}
    log("host ceiling, %d processes: %.1f M reads/s (align %s s), shards concatenated identical: %s"
        % (nproc, out["reads_per_s"] / 1e6, ["%.2f" % x for x in align_s], same))
    return out


def gwa_header_len(path):
    """bytes of the leading @SQ header lines of a SAM file"""
    n = 0
    with open(path, "rb") as f:
        for line in f:
            if not line.startswith(b"@"):
                break
            n += len(line)
    return n


def hg19r_leg(args, gen, gwa, synth, np, cfg, log):
    """detail.hg19r: the same C2 step on the hg19-like repetitive genome (tools/synth.genome_repeats,
    generated by a child process while the main leg ran), with its own parity block: random reads plus
    every read a search tier >= 1 ran, against the oracle on an index whose suffix arrays passed the
    complete check (the repeats send reads to the deep tiers the headline genome never reaches)."""
    import torch
    gen_proc, path = gen
    t0 = time.time()
    if gen_proc.wait() != 0:
        raise SystemExit("hg19r genome generation failed")
    codes = np.load(path)
    os.remove(path)
    names = [c[0] for c in synth.HG19_CONTIGS]
    lengths = [c[1] for c in synth.HG19_CONTIGS]
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths, device=torch.cuda.current_device())
    n = args.reads or 10_000_000
    m = 100
    blobs = make_reads(synth, np, codes, lengths, n, m, False, 0)
    batch = gwa.Batch(gi, cfg, blobs=blobs)
    dt, _, kms, st, _ = timed_steps(batch, 2, 1, lambda: None)
    out = {"value": 2 * n / dt, "unit": "reads/s", "ms_per_step": dt * 1e3 / 2, "steps": 2, "warmup": 1,
           "reads_per_step": n, "kernels_ms": kms, "tier_reads": list(st.tier_reads),
           "tier_ms": [round(x, 3) for x in st.tier_ms],
           "genome": "hg19-like synthetic (hg19 contig lengths, N gaps, interspersed repeat families, satellites, "
                     "segmental duplications; tools/synth.genome_repeats)"}
    log("hg19r leg: %.0f reads/s (%.1f ms per step; tiers %s)" % (out["value"], out["ms_per_step"], out["tier_reads"]))
    if args.check:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle as O
        T = host_cores()[0]
        t1 = time.time()
        deep = np.nonzero(batch.read_counters()[:, 12] >= 1)[0]
        sa_f, sa_r = gi.suffixArray(0), gi.suffixArray(1)
        O.check_cyclic_sa_full(codes, sa_f, threads=T)
        O.check_cyclic_sa_full(np.ascontiguousarray(codes[::-1]), sa_r, threads=T)
        oi = O.Index.from_arrays(codes, names, lengths, sa_f=sa_f, sa_r=sa_r)
        del sa_f, sa_r
        rnd = min(args.check // 4, n)
        rng = np.random.default_rng(11)
        samp = np.unique(np.concatenate([rng.choice(n, rnd, replace=False), deep])).astype(np.uint32)
        got, _ = batch.results_select(samp)
        nb, _, sb = blobs[0], blobs[1], blobs[2]
        sreads = [(nb[10 * i:10 * i + 10].decode(), sb[m * i:m * i + m].decode(), "I" * m) for i in map(int, samp)]
        exp = oi.align(sreads, O.OrcConfig.default(k=2.0), threads=T)
        del oi
        out["parity"] = {"reads": int(len(samp)), "random": int(rnd), "tier_ge1": int(len(deep)), "identical": got == exp,
                         "sa_check": "complete (every adjacent pair, both strands)", "seconds": time.time() - t1,
                         "note": "random reads + every read of search tiers >= 1 of the last timed step, GPU SAM against "
                                 "the oracle; oracle index from the GPU suffix arrays after the complete check"}
        log("hg19r parity on %d reads (%d from tiers >= 1): %s (%.0fs)" % (len(samp), len(deep), got == exp, time.time() - t1))
    out["leg_s"] = time.time() - t0
    del codes
    batch.close()
    gi.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--genome", default=os.environ.get("GWA_BENCH_GENOME", "hg19"),
                    help="hg19: hg19 contig lengths, i.i.d. ACGT with hg19-like N-gap runs (the BASELINE stand-in, "
                         "SURVEY.md 8(d)), or the FASTA file $GWA_HG19 when set; hg19r: hg19-like repeats and N gaps "
                         "(tools/synth.genome_repeats); ecoli (or the FASTA file $GWA_ECOLI); a size in Mbp; or the "
                         "path of a FASTA file")
    ap.add_argument("--reads", type=int, default=int(os.environ.get("GWA_BENCH_READS", "0")))
    ap.add_argument("--k", type=float, default=None, help="max edits (default: 2 for c2, 5 for c4)")
    ap.add_argument("--workload", default="c2", choices=["c2", "c4", "c5"],
                    help="c2: 100 bp, 0-2 substitutions (the BASELINE metric); c4: 150 bp, 0-5 edits with indels; "
                         "c5: 2x100 bp paired-end, insert ~ N(300, 30), proper pairs within [210, 390]")
    ap.add_argument("--strategy", default="bsf", choices=["bsf", "sf"], help="-m (align strategy)")
    ap.add_argument("--cpu-sample", type=int, default=int(os.environ.get("GWA_CPU_SAMPLE", "40000")),
                    help="reads of the single-thread CPU baseline (SURVEY.md 8(d)(i)), each of 3 runs")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads of the multi-core CPU baseline (default: the cores this process may use)")
    ap.add_argument("--cpu-seconds", type=float, default=5.0,
                    help="target duration of each of the 3 multi-core CPU baseline runs (sample sized from the 1-thread rate)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--check", type=int, default=20000,
                    help="random reads of step 0 checked against the oracle (plus every read a search tier >= 1 ran)")
    ap.add_argument("--no-pipeline", action="store_true", help="skip the host-pipeline (FASTQ-to-SAM) leg")
    ap.add_argument("--no-hg19r", action="store_true", help="skip the detail.hg19r leg (default C2 run at N=1 only)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        spawn_ranks(args)
    # stdout carries exactly one JSON line (rank 0): whatever else writes to fd 1 in this process or
    # its children -- torch / gloo / RCCL C++ logging such as "[Gloo] Rank 0 is connected to 1 peer
    # ranks" -- is sent to stderr
    global JSON_OUT
    sys.stdout.flush()
    JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    c4 = args.workload == "c4"
    # the hg19r leg's genome is generated by a child process (started before this process touches
    # the GPU) while the main leg runs
    gen = None
    if (world == 1 and args.workload == "c2" and args.genome == "hg19" and not args.no_hg19r and args.strategy == "bsf"
            and args.k in (None, 2.0) and not os.path.isfile(os.environ.get("GWA_HG19", ""))):
        import subprocess
        import tempfile
        import shutil
        d = "/dev/shm" if os.path.isdir("/dev/shm") and shutil.disk_usage("/dev/shm").free > (8 << 30) else tempfile.gettempdir()
        path = os.path.join(d, "gwa_bench_hg19r_%d.npy" % os.getpid())
        gen = (subprocess.Popen([sys.executable, os.path.join(REPO, "tools", "synth.py"), "hg19r", path]), path)

    import numpy as np
    import synth
    import gwa
    import dist as gdist

    dist = world > 1
    if dist:
        import torch
        import torch.distributed as tdist
        # CPU tensors (timings, barriers) over gloo; the optional SAM gather of device buffers over RCCL
        # (nccl) when every rank has a GPU of its own (torch.cuda.device_count does not initialise the GPU)
        tdist.init_process_group("cpu:gloo,cuda:nccl" if torch.cuda.device_count() >= world else "gloo")
    import torch
    dev = gdist.device_for(local, torch.cuda.device_count())
    torch.cuda.set_device(dev)

    t0 = time.time()
    # a real genome when one is given: --genome <FASTA path>, or $GWA_HG19 / $GWA_ECOLI for hg19 / ecoli
    # (SURVEY.md 8(d)); the reads stay synthetic, drawn from it
    real = None
    if os.path.isfile(args.genome):
        real = args.genome
    elif args.genome == "hg19" and os.path.isfile(os.environ.get("GWA_HG19", "")):
        real = os.environ["GWA_HG19"]
    elif args.genome == "ecoli" and os.path.isfile(os.environ.get("GWA_ECOLI", "")):
        real = os.environ["GWA_ECOLI"]
    if real:
        codes, names, lengths = synth.fasta_codes(real)
        gname = "real genome %s (%d contigs)" % (os.path.basename(real), len(names))
    elif args.genome in ("hg19", "hg19r"):
        if args.genome == "hg19":
            codes, names, lengths = synth.genome_ngaps(synth.HG19_CONTIGS, config_id=1)
            gname = "hg19-size synthetic (hg19 contig lengths, i.i.d. ACGT, hg19-like N-gap runs)"
        else:
            codes, names, lengths = synth.genome_repeats(synth.HG19_CONTIGS, config_id=1)
            gname = ("hg19-like synthetic (hg19 contig lengths, N gaps, interspersed repeat families, satellites, "
                     "segmental duplications; tools/synth.genome_repeats)")
    elif args.genome == "ecoli":
        codes, names, lengths = synth.genome(synth.ECOLI, config_id=1)
        gname = "E. coli-size synthetic (4,641,652 bp i.i.d. ACGT)"
    else:
        mb = float(args.genome)
        codes, names, lengths = synth.genome([("chr%d" % (i + 1), int(mb * 1e6 / 4)) for i in range(4)], config_id=1)
        gname = "%g Mbp synthetic (4 contigs, i.i.d. ACGT)" % mb
    data_label = ("synthetic reads from the real genome %s" % real) if real else "synthetic"
    if args.k is None:
        args.k = 5.0 if c4 else 2.0
    reads_per_step = args.reads or (1_000_000 if c4 else 10_000_000 if (args.genome.startswith("hg19") or len(codes) > 1e9)
                                    else 1_000_000)
    log("rank %d/%d on GPU %d: genome %d bp generated in %.1fs" % (rank, world, dev, len(codes), time.time() - t0))
    t0 = time.time()
    gi = gwa.FMIndexOnGenome.buildFromCodes(codes, names, lengths, device=dev)
    t_index = time.time() - t0
    index_gb = gi.deviceBytes() / 1e9
    log("index built + resident in HBM: %.1fs, %.2f GB" % (t_index, index_gb))

    cfg = gwa.AlignmentConfig(k=args.k, strategy=args.strategy)
    if args.workload == "c5":
        return bench_c5(args, gi, codes, names, lengths, gname, rank, world, dist, dev, t_index)
    m = 150 if c4 else 100
    t0 = time.time()
    blobs = make_reads(synth, np, codes, lengths, reads_per_step, m, c4, rank)
    name_blob, name_off, seq_blob, seq_off, qual_blob, _ = blobs
    log("reads generated in %.1fs" % (time.time() - t0))
    t0 = time.time()
    batch = gwa.Batch(gi, cfg, blobs=blobs)
    log("batch resident in HBM: %.1fs" % (time.time() - t0))

    def read_tuple(i):
        return (name_blob[10 * i:10 * i + 10].decode(), seq_blob[m * i:m * i + m].decode(), "I" * m)

    def barrier():
        if dist:  # a CPU all-reduce (gloo), whatever the device backend
            tdist.all_reduce(torch.zeros(1))

    mine, window, kms, st, sam_bytes = timed_steps(batch, args.steps, args.warmup, barrier)
    rank_times = gdist.all_gather_floats(mine)
    dt = max(rank_times)

    # SURVEY.md §8e's optional collective, outside the timed region: the SAM text of the last step, in
    # HBM on every rank, gathered in rank order (= input order) over RCCL / xGMI
    gather = None
    if dist and torch.cuda.device_count() >= world:
        # every rank first agrees that its text is ready (a rank that fails to copy it would leave the
        # others blocked inside the collective)
        try:
            mine_t = batch.sam_device()
            ok = 1.0
        except Exception as e:
            mine_t, ok, gather = None, 0.0, {"error": repr(e)}
        flag = torch.tensor([ok])
        tdist.all_reduce(flag, op=tdist.ReduceOp.MIN)
        if float(flag[0]) < 1.0:
            gather = gather or {"error": "another rank could not copy its SAM text"}
        else:
            torch.cuda.synchronize()
            barrier()
            t0 = time.perf_counter()
            merged = gdist.gather_sam_device(mine_t)
            torch.cuda.synchronize()
            tg = time.perf_counter() - t0
            tot = gdist.all_gather_floats(float(sam_bytes))
            gather = {"seconds": tg, "bytes_per_rank": tot, "backend": "nccl (RCCL)",
                      "merged_bytes": int(merged.numel()) if merged is not None else None,
                      "GBps_gathered": sum(tot) / tg / 1e9 if tg > 0 else None,
                      "note": "all-gather of the lengths, then each rank's text sent once, point to point, into "
                              "its slice of rank 0's merged buffer (rank order = input order)"}
            if merged is not None and int(merged.numel()) != int(sum(tot)):
                gather["error"] = "merged size differs from the sum of the ranks' SAM sizes"
            del merged, mine_t
    elif dist:
        gather = {"skipped": "ranks share a GPU (RCCL needs one GPU per rank)"}

    # host pipeline (first bullet): the whole path for one batch outside the timed
    # region -- reads from host memory to HBM (batch create), kernels, SAM text to the host -- reported
    # beside `value`, never as it
    pipe = None
    if rank == 0 and not args.no_pipeline:
        t0 = time.perf_counter()
        b2 = gwa.Batch(gi, cfg, blobs=blobs)
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

    # end to end (first bullet): this batch's reads as a FASTQ file on local disk ->
    # the library pipeline (gwa_pipeline_align_file: read, frame, H2D, parse + encode + align + SAM on
    # the GPU, D2H, write) -> a SAM file; index load excluded
    e2e = None
    if rank == 0 and not args.no_pipeline and not c4:
        import tempfile
        d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
        fq, so = os.path.join(d, "reads.fq"), os.path.join(d, "out.sam")
        t0 = time.perf_counter()
        write_fastq(np, fq, name_blob, seq_blob, reads_per_step, m)
        t_write = time.perf_counter() - t0
        # two passes over the file on one pipeline: the first also pins the pipeline's host buffers,
        # the second is the steady state
        t0 = time.perf_counter()
        pipe_ = gwa.Pipeline([gi], cfg)
        t_open = time.perf_counter() - t0
        legs = []
        for _ in range(2):
            with open(so, "wb") as f:
                t0 = time.perf_counter()
                n_e2e = pipe_.align_file(fq, f.fileno())
                legs.append(time.perf_counter() - t0)
        t_e2e = legs[1]
        pst = pipe_.stats()
        pipe_.close()
        e2e = {"reads_per_s": n_e2e / t_e2e, "seconds": t_e2e, "reads": n_e2e, "fastq_bytes": os.path.getsize(fq),
               "first_pass_reads_per_s": n_e2e / legs[0], "first_pass_seconds": legs[0], "pipeline_open_s": t_open,
               "sam_bytes": os.path.getsize(so), "fastq_write_s": t_write,
               "stages_s": {"read": pst.read_s, "frame": pst.frame_s, "setup": pst.setup_s,
                            "kernels": pst.device_kernel_s[0], "sam_format_d2h": pst.format_s, "write": pst.write_s},
               "note": "FASTQ file -> SAM file through gwa_pipeline_align_file (1 GPU, 3 worker threads), local "
                       "disk via the page cache; index load and pipeline open excluded; reads_per_s is the second "
                       "pass over the file on the same pipeline, first_pass_* the first (it also pins the host "
                       "buffers); stage times summed over threads, second pass"}
        # parity of the pipeline's output (outside all timing): the SAM file's records, byte for byte,
        # equal the SAM text the timed batch wrote in HBM for the same reads
        try:
            with open(so, "rb") as f:
                body = f.read()
            h = 0
            while h < len(body) and body[h:h + 1] == b"@":
                h = body.index(b"\n", h) + 1
            ref = batch.sam_device().cpu().numpy()
            same = len(body) - h == ref.size and np.array_equal(np.frombuffer(body, dtype=np.uint8, offset=h), ref)
            del body, ref
        except Exception as ex:  # reported, never fatal to the line
            same = False
            e2e["parity_error"] = repr(ex)
        e2e["identical_to_timed_batch"] = bool(same)
        log("end to end FASTQ -> SAM: %.0f reads/s (%d reads in %.2fs), SAM %s the timed batch's"
            % (n_e2e / t_e2e, n_e2e, t_e2e, "identical to" if same else "DIFFERS from"))
        for x in (fq, so):
            os.remove(x)
        os.rmdir(d)

    hostc = None
    if rank == 0 and world == 1 and not args.no_pipeline and not c4:
        hostc = host_ceiling_leg(args, gwa, synth, np, log)

    counters = batch.read_counters()  # also fetches the records (stats below)
    st = batch.stats()
    total_reads = reads_per_step * args.steps * world
    value = total_reads / dt
    deep = np.nonzero(counters[:, 12] >= 1)[0]

    # parity (checker only): a random sample of this rank's reads plus every read a search tier >= 1
    # ran, GPU SAM against the oracle.  The oracle index takes the GPU suffix arrays only after a
    # complete independent check of them (permutation + every adjacent pair, oracle C++).
    parity = None
    oi = None
    if rank == 0 and (args.check or (not args.no_cpu and args.cpu_sample > 0)):
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle as O
        t0 = time.time()
        sa_f, sa_r = gi.suffixArray(0), gi.suffixArray(1)
        O.check_cyclic_sa_full(codes, sa_f, threads=host_cores()[0])
        O.check_cyclic_sa_full(np.ascontiguousarray(codes[::-1]), sa_r, threads=host_cores()[0])
        t_sa = time.time() - t0
        log("GPU suffix arrays pass the complete check (every adjacent pair, both strands): %.1fs" % t_sa)
        oi = O.Index.from_arrays(codes, names, lengths, sa_f=sa_f, sa_r=sa_r)
        del sa_f, sa_r
        t_oidx = time.time() - t0 - t_sa
    if args.check and rank == 0:
        rng = np.random.default_rng(7)
        samp = np.unique(np.concatenate([rng.choice(reads_per_step, min(args.check, reads_per_step), replace=False),
                                         deep])).astype(np.uint32)
        got, _ = batch.results_select(samp)
        sreads = [read_tuple(int(i)) for i in samp]
        exp = oi.align(sreads, O.OrcConfig.default(k=args.k, strategy=gwa.STRATEGIES[args.strategy]),
                       threads=host_cores()[0])
        parity = {"reads": int(len(samp)), "random": int(min(args.check, reads_per_step)), "tier_ge1": int(len(deep)),
                  "identical": got == exp, "sa_check": "complete (every adjacent pair, both strands)",
                  "note": "random reads + every read of search tiers >= 1; oracle index from the GPU suffix arrays "
                          "after a complete independent permutation + adjacent-order check"}
        log("parity on %d reads (%d from tiers >= 1): %s (oracle index %.1fs)" % (len(samp), len(deep), got == exp, t_oidx))

    cpu = cpu1 = None
    if rank == 0 and not args.no_cpu and args.cpu_sample > 0:
        cpu, cpu1 = cpu_baselines(oi, read_tuple, reads_per_step, gwa.STRATEGIES[args.strategy], args.k, args, O,
                                  args.strategy.upper())
    oi = None

    # Roofline of the dominant kernel.  `achieved` / `frac` follow SURVEY.md §8(d): 64 B per
    # reference FM step (one Occ block, the lower bound of §8d's 1-2 blocks), 4 B per SA gather, and
    # for each DP verification ceil(2n/8) + ceil(n/8) B of reference window + 32 B of Peq per 64-base
    # block.  `kernel_bytes` re-prices what the kernels actually read: 64 B per Occ block read, 8 B per
    # k-mer table lookup, 3/8 B per FM step answered from the 2-bit text (single-row interval).
    q_ms, s_ms = kms["quickscan"], kms["search"]
    q_bytes = 64.0 * st.quick_blocks + 8.0 * st.kmer_lookups + 0.375 * st.quick_short_steps + 4.0 * st.quick_sa_reads
    q_ref = 64.0 * (st.quick_blocks + st.quick_short_steps) + 4.0 * st.quick_sa_reads
    s_bytes = (64.0 * (st.blocks - st.quick_blocks) + 0.375 * st.search_short_steps
               + 4.0 * (st.sa_reads - st.quick_sa_reads) + st.verify_bytes)
    s_ref = (64.0 * (st.blocks - st.quick_blocks + st.search_short_steps) + 4.0 * (st.sa_reads - st.quick_sa_reads)
             + st.verify_bytes)
    if q_ms >= s_ms:
        dom, k_bytes, dom_ms, dom_ref = "fm_quickscan", q_bytes, q_ms, q_ref
    else:
        dom, k_bytes, dom_ms, dom_ref = args.strategy + "_search", s_bytes, s_ms, s_ref
    gbs = (lambda b, ms: b / (ms * 1e-3) / 1e9 if ms > 0 else 0.0)
    workload = ("%s; %d x %d bp reads per GPU per step, %s, -k %g, -m %s, besthit"
                % (gname, reads_per_step, m, "0-5 edits (subs/1-bp indels)" if c4 else "0-2 substitutions", args.k,
                   args.strategy))
    traffic, traffic_src = _pmc_traffic(dom, workload)
    hg = None
    if gen is not None and rank == 0:
        batch.close()
        gi.close()
        del codes
        hg = hg19r_leg(args, gen, gwa, synth, np, cfg, log)
    out = {
        "metric": METRIC if not c4 else "reads/sec, 150 bp k<=5 with indels vs hg19 (config C4)", "value": value,
        "unit": "reads/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u64", "data": data_label,
        "config": {"workload": workload, "timed_step": "encode the read text in HBM + fm_quickscan + %s_search tiers + "
                                                      "SAM text written in HBM (gwa_batch_run + gwa_batch_format)"
                                                      % args.strategy,
                   "genome_bp": int(sum(lengths)), "reads_per_gpu_per_step": reads_per_step,
                   "parallelism": "reads sharded, index replicated (%d GPU)" % world},
        "roofline": {"bound": "hbm", "kernel": dom, "definition": "SURVEY.md 8(d) algorithmic bytes",
                     "achieved": gbs(dom_ref, dom_ms), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": gbs(dom_ref, dom_ms) / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": dom_ref, "avg_launch_ms": dom_ms,
                     "kernel_bytes_per_launch": k_bytes, "kernel_bytes_achieved": gbs(k_bytes, dom_ms),
                     "kernel_bytes_frac": gbs(k_bytes, dom_ms) / HBM_PEAK_GBS},
        "cpu_baseline": cpu,
        "detail": {"rank_seconds": rank_times, "devices": "rank r on GPU r mod %d" % torch.cuda.device_count(),
                   "timed_window_monotonic_ns": window,
                   "encode_ms": kms["encode"], "quickscan_ms": q_ms, "search_ms": s_ms, "format_ms": kms["format"],
                   "kernel_ms": kms["kernel"] + kms["format"], "sam_bytes_per_step": sam_bytes,
                   "align_kernels_reads_per_s": reads_per_step / ((q_ms + s_ms) * 1e-3) if q_ms + s_ms > 0 else None,
                   "fm_searches_per_read": st.fm_searches / reads_per_step,
                   "quick_steps_per_read": st.quick_steps / reads_per_step,
                   "blocks_per_read": st.blocks / reads_per_step, "tier_reads": list(st.tier_reads),
                   "tier_ms": [round(x, 3) for x in st.tier_ms], "dp_verifications_per_read": st.num_sw / reads_per_step,
                   "quick_short_steps_per_read": st.quick_short_steps / reads_per_step,
                   "cpu_baseline_1thread": cpu1, "host_pipeline": pipe, "end_to_end": e2e,
                   "search_short_steps_per_read": st.search_short_steps / reads_per_step,
                   "rank_kernel": rank_kernel_entry(st, q_ms, q_ref, q_bytes, workload, gbs),
                   "mapped": st.n_mapped, "unmapped": st.n_unmapped, "index_build_s": t_index,
                   "index_gb": index_gb, "parity": parity, "hg19r": hg, "host_ceiling": hostc,
                   "sam_gather": gather},
    }
    if rank == 0:
        print(json.dumps(out), file=JSON_OUT, flush=True)
    if hg is None:
        batch.close()
    if dist:
        tdist.destroy_process_group()


def bench_c5(args, gi, codes, names, lengths, gname, rank, world, dist, dev, t_index):
    """Config C5: 2x100 bp pairs (tools/synth.pairs_codes: insert ~ N(300, 30)), -k 2.  One step = the
    alignment kernels over both mates of every pair plus the pairing and SAM text written in HBM
    (gwa_batch_format), reads resident in HBM.  value = reads/s (two per pair).  The pairing rules are
    the build's own (the reference has no paired-end path); parity is against the oracle's
    restatement of them (orc_align_pairs)."""
    import numpy as np
    import synth
    import gwa
    import dist as gdist
    import torch
    if dist:
        import torch.distributed as tdist
    m = 100
    pairs = (args.reads or 10_000_000) // 2
    t0 = time.time()
    m1, m2 = synth.pairs_codes(codes, lengths, pairs, m, config_id=5, shard=rank)
    s1, s2 = synth.SYM[m1].tobytes(), synth.SYM[m2].tobytes()
    del m1, m2
    off = np.arange(0, m * (pairs + 1), m, dtype=np.uint64)
    nb, no = synth.name_blob(pairs)
    q1, q2 = b"I" * (m * pairs), b"J" * (m * pairs)
    log("pairs generated in %.1fs" % (time.time() - t0))
    cfg = gwa.AlignmentConfig(k=args.k, strategy="bsf")
    batch = gwa.Batch(gi, cfg, pair_blobs=((nb, no, s1, off, q1, off), (nb, no, s2, off, q2, off)))

    def pair_tuple(i):
        n = nb[10 * i:10 * i + 10].decode()
        return (n, s1[m * i:m * i + m].decode(), "I" * m), (n, s2[m * i:m * i + m].decode(), "J" * m)

    for _ in range(args.warmup):
        batch.run()
        batch.format_device()
    if dist:
        tdist.all_reduce(torch.zeros(1))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    win0 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
    kms = qms = sms = 0.0
    for _ in range(args.steps):
        batch.run()
        st = batch.stats()
        kms += st.kernel_ms
        qms += st.quickscan_ms
        sms += st.search_ms
        batch.format_device()
    torch.cuda.synchronize()
    if dist:
        tdist.all_reduce(torch.zeros(1))
    win1 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
    rank_times = gdist.all_gather_floats(time.perf_counter() - t0)
    dt = max(rank_times)
    value = 2 * pairs * args.steps * world / dt
    st = batch.stats()
    parity = cpu = cpu1 = None
    if rank == 0:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle as O
        T, tdesc = host_cores()
        sa_f, sa_r = gi.suffixArray(0), gi.suffixArray(1)
        O.check_cyclic_sa_full(codes, sa_f, threads=T)
        O.check_cyclic_sa_full(np.ascontiguousarray(codes[::-1]), sa_r, threads=T)
        oi = O.Index.from_arrays(codes, names, lengths, sa_f=sa_f, sa_r=sa_r)
        del sa_f, sa_r
        ocfg = O.OrcConfig.default(k=args.k)
        if args.check:
            samp = np.sort(np.random.default_rng(7).choice(pairs, min(args.check, pairs), replace=False)).astype(np.uint32)
            got, _ = batch.results_select(samp)
            tp = [pair_tuple(int(i)) for i in samp]
            exp = oi.align_pairs([a for a, b in tp], [b for a, b in tp], ocfg)
            parity = {"pairs": int(len(samp)), "identical": got == exp,
                      "note": "random pairs vs the oracle's restatement of the build's pairing rules (parity unpinned "
                              "against the reference, which has no paired-end path)"}
            log("parity on %d pairs: %s" % (len(samp), got == exp))
        if not args.no_cpu:
            from concurrent.futures import ThreadPoolExecutor
            model = cpu_model()
            ns = min(args.cpu_sample // 2, pairs)
            tp = [pair_tuple(i) for i in range(ns)]
            t1 = time.perf_counter()
            oi.align_pairs([a for a, b in tp], [b for a, b in tp], ocfg)
            ct = time.perf_counter() - t1
            cpu1 = {"value": 2 * ns / ct, "unit": "reads/s", "cores": 1, "kind": "port", "seconds": ct,
                    "sample": "first %d pairs, single-thread C++ oracle (paired-end restatement of the build's rules over "
                              "the reference BSF path; CPU restatement, not the JVM); %s" % (ns, model)}
            cpu = cpu1
            if T > 1:
                npairs = int(min(pairs, max(ns, args.cpu_seconds * cpu1["value"] / 2 * T)))
                tp = tp + [pair_tuple(i) for i in range(ns, npairs)]
                chunks = [(a * npairs // T, (a + 1) * npairs // T) for a in range(T)]
                t1 = time.perf_counter()
                with ThreadPoolExecutor(T) as ex:
                    list(ex.map(lambda c: oi.align_pairs([x for x, y in tp[c[0]:c[1]]], [y for x, y in tp[c[0]:c[1]]],
                                                         ocfg), chunks))
                ct = time.perf_counter() - t1
                cpu = {"value": 2 * npairs / ct, "unit": "reads/s", "cores": T, "kind": "port", "seconds": ct,
                       "sample": "first %d pairs on %d host threads (%s; contiguous ranges), C++ oracle; %s"
                                 % (npairs, T, tdesc, model)}
            log("cpu baseline: %.0f reads/s (%d threads)" % (cpu["value"], cpu["cores"]))
    steps = args.steps
    q_ms, s_ms = qms / steps, sms / steps
    q_ref = 64.0 * (st.quick_blocks + st.quick_short_steps) + 4.0 * st.quick_sa_reads
    s_ref = (64.0 * (st.blocks - st.quick_blocks + st.search_short_steps) + 4.0 * (st.sa_reads - st.quick_sa_reads)
             + st.verify_bytes)
    dom, dom_ref, dom_ms = ("fm_quickscan", q_ref, q_ms) if q_ms >= s_ms else ("bsf_search", s_ref, s_ms)
    ach = dom_ref / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    out = {"metric": "reads/sec, 2x100 bp paired-end k<=2 vs hg19 (config C5)", "value": value, "unit": "reads/s",
           "n_gpus": world, "steps": steps, "warmup": args.warmup, "ms_per_step": dt * 1e3 / steps,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
           "config": {"workload": "%s; %d pairs (2 x 100 bp, insert ~ N(300, 30), 0-2 substitutions per mate) per GPU "
                                  "per step, -k %g, -m bsf, proper pairs in [210, 390]" % (gname, pairs, args.k),
                      "genome_bp": int(len(codes)), "pairs_per_gpu_per_step": pairs,
                      "parallelism": "pairs sharded, index replicated (%d GPU)" % world},
           "roofline": {"bound": "hbm", "kernel": dom, "definition": "SURVEY.md 8(d) algorithmic bytes",
                        "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                        "traffic": None, "algorithmic_bytes_per_launch": dom_ref, "avg_launch_ms": dom_ms},
           "cpu_baseline": cpu,
           "detail": {"rank_seconds": rank_times, "timed_window_monotonic_ns": [win0, win1], "quickscan_ms": q_ms, "search_ms": s_ms, "kernel_ms": kms / steps,
                      "tier_reads": list(st.tier_reads), "tier_ms": [round(x, 3) for x in st.tier_ms],
                      "cpu_baseline_1thread": cpu1, "parity": parity, "index_build_s": t_index}}
    if rank == 0:
        print(json.dumps(out), file=JSON_OUT, flush=True)
    batch.close()
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
