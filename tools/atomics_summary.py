"""Summarise tools/pmc_atomics.sh into profiles/<tag>_atomics.json: per workload and kernel, atomic requests per
launch at the L2 (TCC_ATOMIC), those that went on to the memory side (TCC_EA0_ATOMIC), their average latency in
cycles (EA0_ATOMIC_LEVEL / EA0_ATOMIC), and the achieved atomic rate (TCC_ATOMIC per launch / average duration
from the kernel-trace pass). Usage: python tools/atomics_summary.py <atom_dir> <out.json>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d, out = sys.argv[1], sys.argv[2]
    res = {}
    for wdir in sorted(glob.glob(os.path.join(d, "*"))):
        w = os.path.basename(wdir)
        pm = glob.glob(os.path.join(wdir, "pmc", "*counter_collection.csv"))
        st = glob.glob(os.path.join(wdir, "trace", "*kernel_stats.csv"))
        if not pm or not st:
            continue
        vals = defaultdict(lambda: defaultdict(list))
        for r in csv.DictReader(open(pm[0])):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur = {r["Name"]: float(r["AverageNs"]) for r in csv.DictReader(open(st[0]))}
        ks = {}
        for k, c in vals.items():
            n = max(len(v) for v in c.values())
            per = {name: sum(v) / n for name, v in c.items()}
            atom = per.get("TCC_ATOMIC_sum", 0.0)
            if atom < 1000:
                continue
            ns = dur.get(k)
            ea = per.get("TCC_EA0_ATOMIC_sum", 0.0)
            ks[k.split("(")[0]] = {
                "launches": n, "tcc_atomic_per_launch": atom, "ea_atomic_per_launch": ea,
                "ta_flat_atomic_wavefronts_per_launch": per.get("TA_FLAT_ATOMIC_WAVEFRONTS_sum"),
                "ea_atomic_latency_cycles": (per.get("TCC_EA0_ATOMIC_LEVEL_sum", 0.0) / ea) if ea else None,
                "kernel_ns_avg": ns, "atomics_per_s": (atom / (ns * 1e-9)) if ns else None}
        res[w] = ks
    json.dump({"source": "rocprofv3 --pmc TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum TCC_EA0_ATOMIC_LEVEL_sum "
                         "TA_FLAT_ATOMIC_WAVEFRONTS_sum (one pass) + --kernel-trace --stats (durations), "
                         "tools/fold_once.py <workload> 3", "workloads": res}, open(out, "w"), indent=1)
    for w, ks in res.items():
        for k, v in sorted(ks.items(), key=lambda kv: -kv[1]["tcc_atomic_per_launch"])[:5]:
            rate = v["atomics_per_s"]
            print(f"{w:10s} {k[:40]:40s} atomics/launch {v['tcc_atomic_per_launch']:.3g} ea {v['ea_atomic_per_launch']:.3g}"
                  f" {'' if rate is None else f'{rate / 1e9:.1f} G atomics/s'}")


if __name__ == "__main__":
    main()
