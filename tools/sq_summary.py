"""Summarise tools/sq_passes.sh output: per kernel (name prefix), the counters summed over its dispatches, divided by
the dispatch count; and derived ratios. Usage: python tools/sq_summary.py <dir>"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        short = k.split("(")[0].replace("void ", "")
        for key in ("bk::bucket_kernel", "bk::slice_filter_kernel<true, false", "bk::slice_filter_kernel<true, true",
                    "bk::slice_filter_kernel<false", "bk::slice_hook_kernel<true>", "bk::slice_hook_kernel<false>",
                    "compress_bits_kernel"):
            if short.startswith(key) or key in k:
                name = key
                break
        else:
            continue
        c = row.get("Counter_Name")
        v = float(row.get("Counter_Value", 0) or 0)
        acc[name][c] += v
        disp[name].add((f.split(os.sep)[-3] if False else os.path.dirname(f), row.get("Dispatch_Id")))
for name, cs in acc.items():
    n = max(1, len({x[1] for x in disp[name]}) // 3)
    print(f"== {name} (~{n} dispatches per pass)")
    for c in sorted(cs):
        print(f"  {c:28s} {cs[c] / n:.4g}")
    g = lambda c: cs.get(c, 0.0) / n
    if g("SQ_WAVE_CYCLES"):
        print(f"  waves' cycles waiting (any) {g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.2f}, issuing {g('SQ_ACTIVE_INST_ANY') / g('SQ_WAVE_CYCLES'):.2f}")
    if g("SQ_INSTS_LDS"):
        print(f"  LDS bank conflict cycles per LDS inst {g('SQ_LDS_BANK_CONFLICT') / g('SQ_INSTS_LDS'):.2f}")
