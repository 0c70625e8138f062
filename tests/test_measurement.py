"""CPU: the measurement plumbing VERDICT r5 found defective (weak 7a, 7b) — tools/pmc_summary.py counts a run's steps
from the once-per-step marker kernel (gcc_step_mark, bench.py --step-marker), not from the dominant kernel's launches,
and bench.py's PMC-record picker takes the newest session tag (r5ba after r5k), not the lexically largest name."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_record_order_is_session_order():
    names = ["r5k_pmc_c4_kron26.json", "r5ba_pmc_c4_kron26.json", "r4z2_pmc_c4_kron26.json", "r4z_pmc_c4_kron26.json",
             "r6b_pmc_c3_gnm24.json", "r5z_pmc_c4_kron26.json", "r5aa_pmc_c4_kron26.json"]
    got = sorted(names, key=bench.record_order)
    assert got == ["r4z_pmc_c4_kron26.json", "r4z2_pmc_c4_kron26.json", "r5k_pmc_c4_kron26.json",
                   "r5z_pmc_c4_kron26.json", "r5aa_pmc_c4_kron26.json", "r5ba_pmc_c4_kron26.json",
                   "r6b_pmc_c3_gnm24.json"]


def test_profile_record_picks_the_newest_session():
    rec = bench.profile_record("c4_kron26", "bucket_kernel", 1 << 30)
    assert rec is not None
    newest = max((f for f in os.listdir(os.path.join(ROOT, "profiles")) if "_pmc_c4_kron26" in f and f.endswith(".json")),
                 key=bench.record_order)
    assert rec["file"] == f"profiles/{newest}"


def _write_counters(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def test_pmc_summary_counts_steps_from_the_marker(tmp_path):
    """Three steps; the 'dominant' fold kernel launches 5 times per step (C3's sampled start), the compress once, plus a
    generator launch and the marker. Per-step traffic = (sum over kernels of 2 x FETCH + WRITE per launch x launches) /
    3 steps, the generator and the marker excluded — the hand sum the verdict asked the record to match."""
    d = tmp_path / "pmc"
    fold, comp, gen, mark = "void fold_kernel<false, true, 0, false>(...)", "compress_bits_kernel(...)", "gen_kernel(...)", \
        "gcc_step_mark_kernel()"
    launches = [(gen, 1)] + [(fold, 5), (comp, 1), (mark, 1)] * 3
    fetch, write, hit = [], [], []
    kb = {fold: (100.0, 10.0), comp: (1000.0, 500.0), gen: (0.0, 9999.0), mark: (0.0, 0.0)}
    for k, n in launches:
        for _ in range(n):
            fetch.append({"Kernel_Name": k, "Counter_Name": "FETCH_SIZE", "Counter_Value": kb[k][0]})
            write.append({"Kernel_Name": k, "Counter_Name": "WRITE_SIZE", "Counter_Value": kb[k][1]})
            hit += [{"Kernel_Name": k, "Counter_Name": "TCC_HIT_sum", "Counter_Value": 1},
                    {"Kernel_Name": k, "Counter_Name": "TCC_MISS_sum", "Counter_Value": 1}]
    _write_counters(str(d / "fetch" / "run_counter_collection.csv"), fetch)
    _write_counters(str(d / "write" / "run_counter_collection.csv"), write)
    _write_counters(str(d / "hit" / "run_counter_collection.csv"), hit)
    out = tmp_path / "rec.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), str(d), "c3_gnm24", "fold_kernel",
                    "1000", "16", str(out)], check=True, capture_output=True)
    rec = json.load(open(out))
    assert rec["steps"] == 3
    want = (5 * (2 * 100 + 10) + (2 * 1000 + 500)) * 1024  # per step: 5 folds + 1 compress
    assert abs(rec["pipeline_traffic_per_step"] - want) < 1e-6 * want
    assert rec["launches_per_step"][fold] == 5 and "recorded" in rec
