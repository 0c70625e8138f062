"""Summarise rocprofv3 PMC passes (tools/pmc_passes.sh) into profiles/<tag>_pmc_<workload>.json.

HBM bytes per launch of a kernel = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: FETCH_SIZE/WRITE_SIZE are KB, and on
gfx950 FETCH_SIZE tallies every L2 -> fabric read request (one whole 128-B line) as 64 B. Calibrated per access class
in round 6 (tools/probe_fetch_cal.hip, profiles/r6a_fetch_calibration.txt): the 2x holds for the 16-B/lane stream AND
for scattered 4-B reads (one 128-B request per line touched, in the full stream's time); WRITE_SIZE is exact for 4-B
stores (32-B requests), atomics (64-B requests) and streaming stores. Infinity-Cache hits are counted as requests.
Steps: the run's launches of gcc_step_mark_kernel (bench.py --step-marker, once per step; VERDICT r5 weak 7a: C3's
fold launches 5 kernels per step, so counting the dominant kernel's launches undercounted its per-step traffic 5x).
Usage: python tools/pmc_summary.py <pmc_dir> <workload> <kernel substring> <units_per_launch> <bytes_per_unit> <out.json>
(units: edges for the edge kernels; bytes_per_unit: bench.py KERNEL_BYTES)"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    d, workload, ksub, edges, per, out = (sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), float(sys.argv[5]),
                                          sys.argv[6])
    f = per_kernel(f"{d}/fetch/run_counter_collection.csv", "FETCH_SIZE")
    w = per_kernel(f"{d}/write/run_counter_collection.csv", "WRITE_SIZE")
    h = per_kernel(f"{d}/hit/run_counter_collection.csv", "TCC_HIT_sum")
    m = per_kernel(f"{d}/hit/run_counter_collection.csv", "TCC_MISS_sum")
    names = [k for k in f if ksub in k]  # every instantiation of the kernel (same units per launch)
    fv = [x for k in names for x in f[k]]
    wv = [x for k in names for x in w.get(k, [])]
    hv = [x for k in names for x in h.get(k, [])]
    mv = [x for k in names for x in m.get(k, [])]
    fetch_kb = sum(fv) / len(fv)
    write_kb = sum(wv) / len(wv)
    hit, miss = sum(hv) / len(hv), sum(mv) / len(mv)
    rec = {
        "workload": workload,
        "kernel": names[0] if len(names) == 1 else ksub,
        "instantiations": names,
        "launches_sampled": len(fv),
        "edges_per_launch": edges,
        "fetch_size_kb": fetch_kb,
        "write_size_kb": write_kb,
        "hbm_bytes_per_launch": (2 * fetch_kb + write_kb) * 1024,
        "bytes_per_unit": per,
        "algorithmic_bytes_per_launch": per * edges,
        "l2_hit_rate": hit / (hit + miss),
        "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_HIT_sum,TCC_MISS_sum (separate passes), "
                  f"bench.py --steps 5; bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 per launch",
    }
    rec["all_kernels"] = {  # every kernel of the run: HBM bytes per launch (same correction)
        k: {"launches": len(f[k]), "hbm_bytes_per_launch": (2 * sum(f[k]) / len(f[k]) + (sum(w[k]) / len(w[k]) if w.get(k) else 0)) * 1024}
        for k in f}
    # the whole step's HBM traffic: every kernel of the run except the generator, the label copies and the marker,
    # per step (steps = the marker's launches; run bench with --no-extras --step-marker so no other leg is counted)
    marks = [k for k in f if "gcc_step_mark_kernel" in k]
    if not marks:
        sys.exit("no gcc_step_mark_kernel launches in the run: run bench.py with --step-marker (tools/pmc_passes.sh)")
    steps = float(sum(len(f[k]) for k in marks))
    skip = ("gen_kernel", "__amd_rocclr_copyBuffer", "gcc_step_mark_kernel")
    per_step = sum(v["hbm_bytes_per_launch"] * v["launches"] for k, v in rec["all_kernels"].items()
                   if not any(x in k for x in skip)) / max(1.0, steps)
    # the kernel's average duration in the run's kernel-trace pass (tools/pmc_passes.sh): bench.py compares it with
    # the live duration and withholds `traffic` when the kernel changed since (the record would be stale)
    import glob
    import os
    for st in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(st)) if ksub in r["Name"]]
        if rows:
            calls = sum(int(r["Calls"]) for r in rows)
            rec["kernel_ms_at_pmc"] = sum(float(r["TotalDurationNs"]) for r in rows) / max(1, calls) / 1e6
            break
    rec["steps"] = steps
    rec["launches_per_step"] = {k: v["launches"] / steps for k, v in rec["all_kernels"].items()
                                if not any(x in k for x in skip)}
    rec["pipeline_traffic_per_step"] = per_step
    rec["pipeline_algorithmic_per_step"] = 16.0 * edges
    rec["pipeline_traffic_ratio"] = per_step / (16.0 * edges)
    import time
    rec["recorded"] = time.time()  # bench.py profile_record: the newest record wins within a session tag
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
