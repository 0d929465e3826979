"""Summarise a tools/profile.sh run (rocprofv3 kernel trace + PMC passes) into one JSON file.

  python tools/prof_summary.py gpurun_out/prof_<tag> profiles/<round>_<tag>.json

Per kernel of the align path: dispatch count, average duration (kernel trace), and per-dispatch
PMC averages.  FETCH_SIZE is rocprofv3's derived memory-side read volume in KiB; per
/opt/skills/guides/MI355X_MICROARCH.md (§HBM) gfx950 reports half the bytes of 16-B-per-lane
reads.  The align kernels do not stream: they gather random 64-B Occ blocks, 8-B words and 4-B
suffix-array values.  tools/fetch_calib.hip measures FETCH_SIZE on a known count of exactly those
accesses (profiles/r01_fetch_calibration.json): one random access of 4, 8 or 64 B is tallied as
64 B per fabric request (x1.00 for 4/8-B words, x1.21 for a 64-B block read as 4 x 16 B), while the
16-B streaming control reads 1/2 as the guide says.  So `hbm_read_bytes_corrected` = 1 x 1024 x
FETCH_SIZE (requests x 64 B) for these kernels; `hbm_read_bytes_stream_x2` keeps the guide's
streaming correction as an upper bound.  Infinity-Cache hits are counted
in FETCH_SIZE (guide), so this is an upper bound on HBM traffic.
"""
import csv
import glob
import json
import os
import sys

KERNELS = ["fm_quickscan_kernel", "bsf_search_kernel", "encodeLenKernel", "encodeWriteKernel", "samLenKernel", "samWriteKernel"]


def _short(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


def _rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def _window(d, name):
    """bench.py's timed region (CLOCK_MONOTONIC ns, the clock of rocprofv3's timestamps) or None"""
    f = os.path.join(d, name)
    try:
        with open(f) as fh:
            w = json.loads(fh.read().strip().splitlines()[-1])["detail"]["timed_window_monotonic_ns"]
        return int(w[0]), int(w[1])
    except (OSError, ValueError, KeyError, IndexError):
        return None


def _timed_ids(d, sub, win):
    """Dispatch ids of the align kernels that ran inside the timed window (pass `sub`)"""
    ids = set()
    if win is None:
        return None
    for r in _rows(os.path.join(d, sub, "**", "*_kernel_trace.csv")):
        if _short(r["Kernel_Name"]) and int(r["Start_Timestamp"]) >= win[0] and int(r["End_Timestamp"]) <= win[1]:
            ids.add(r["Dispatch_Id"])
    return ids


def summarise(d):
    res = {"kernels": {}}
    # kernel trace: durations over every dispatch, and over the dispatches of bench.py's timed region
    # (the bench line's avg_launch_ms is the mean over those; the parity, pipeline and end-to-end
    # legs outside it launch the same kernels on other batches)
    win = _window(d, "bench.json")
    for r in _rows(os.path.join(d, "trace", "**", "*_kernel_trace.csv")):
        k = _short(r["Kernel_Name"])
        if not k:
            continue
        e = res["kernels"].setdefault(k, {"dispatches": 0, "durations_ns": []})
        e["dispatches"] += 1
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        e["durations_ns"].append(dur)
        if win and int(r["Start_Timestamp"]) >= win[0] and int(r["End_Timestamp"]) <= win[1]:
            e.setdefault("timed_ns", []).append(dur)
        e["vgpr"] = int(r.get("VGPR_Count") or 0)
        e["agpr"] = int(r.get("Accum_VGPR_Count") or 0)
        e["lds_bytes"] = int(r.get("LDS_Block_Size") or 0)
        e["scratch_bytes"] = int(r.get("Scratch_Size") or 0)
    for k, e in res["kernels"].items():
        ds = e.pop("durations_ns")
        e["avg_ms"] = sum(ds) / len(ds) / 1e6
        e["min_ms"] = min(ds) / 1e6
        e["max_ms"] = max(ds) / 1e6
        t = e.pop("timed_ns", None)
        if t:
            e["timed_dispatches"] = len(t)
            e["timed_avg_ms"] = sum(t) / len(t) / 1e6
    # PMC passes: average per dispatch of each counter
    # (the PMC passes run bench.py --check 0 --no-pipeline: only the timed region's dispatches are
    # kept when its window is known)
    for sub, bl in [("pmc_fetch", "bench_pmc1.json"), ("pmc_sq", "bench_pmc2.json"), ("pmc_tcc", "bench_pmc3.json"),
                    ("pmc_write", "bench_pmc4.json")]:
        acc = {}
        keep = _timed_ids(d, sub, _window(d, bl))
        for r in _rows(os.path.join(d, sub, "**", "*_counter_collection.csv")):
            k = _short(r["Kernel_Name"])
            if not k or (keep is not None and r["Dispatch_Id"] not in keep):
                continue
            key = (k, r["Dispatch_Id"], r["Counter_Name"])
            acc[key] = acc.get(key, 0.0) + float(r["Counter_Value"])
        per = {}
        for (k, disp, cn), v in acc.items():
            per.setdefault((k, cn), []).append(v)
        for (k, cn), vs in per.items():
            e = res["kernels"].setdefault(k, {})
            e.setdefault("pmc", {})[cn] = sum(vs) / len(vs)
    for k, e in res["kernels"].items():
        p = e.get("pmc", {})
        if "FETCH_SIZE" in p:
            e["hbm_read_bytes_corrected"] = 1024.0 * p["FETCH_SIZE"]
            e["hbm_read_bytes_stream_x2"] = 2.0 * 1024.0 * p["FETCH_SIZE"]
        if "WRITE_SIZE" in p:  # KiB of fabric write requests (uncalibrated for scattered 8/16-B stores)
            e["hbm_write_bytes"] = 1024.0 * p["WRITE_SIZE"]
        if "TCC_HIT_sum" in p and "TCC_MISS_sum" in p and p["TCC_HIT_sum"] + p["TCC_MISS_sum"] > 0:
            e["l2_hit_rate"] = p["TCC_HIT_sum"] / (p["TCC_HIT_sum"] + p["TCC_MISS_sum"])
        if "SQ_WAIT_ANY" in p and p.get("SQ_WAVE_CYCLES"):
            e["wait_frac"] = p["SQ_WAIT_ANY"] / p["SQ_WAVE_CYCLES"]
    for name in ["bench.json", "bench_pmc1.json"]:
        f = os.path.join(d, name)
        if os.path.exists(f) and os.path.getsize(f):
            with open(f) as fh:
                res.setdefault("bench_lines", {})[name] = json.loads(fh.read().strip().splitlines()[-1])
    stats = glob.glob(os.path.join(d, "trace", "**", "*_kernel_stats.csv"), recursive=True)
    if stats:
        with open(stats[0]) as fh:
            res["kernel_stats_csv"] = fh.read()
    return res


if __name__ == "__main__":
    out = summarise(sys.argv[1])
    txt = json.dumps(out, indent=1, sort_keys=True)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(txt + "\n")
    for k, e in out["kernels"].items():
        print(k, {x: e[x] for x in e if x != "pmc"}, e.get("pmc"))
