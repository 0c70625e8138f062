"""Stress of the incremental compress in the regime of the recorded stale label (VERDICT r3 "next" 1).

profiles/r3ai_gpu_tests_c3_w1M_stale_label.log: C3 (G(n, m), 2^24 ids) in 1M-edge windows, incremental compress on
(inc_div 4, in place, no inc_check), window 8 with the oracle's seen and component counts but another digest.
This folds that stream again and again, each time into a fresh forest, exactly as tests/test_gpu_windows.py does
(fold_device per window, label_digest after each), with tune post_check: a kernel after every incremental compress,
nothing added before or inside it, that counts seen ids whose label is not a root and records the first ones (is
the label marked in the compress's bloom, was it already a non-root after the previous compress). One process,
one GPU, bounded by --seconds; a progress line every few seconds.

  python tools/stress_inc.py --seconds 60 --variant default --variant inc_inplace=0
A variant is a comma-separated list of tune knobs applied on top of incremental=1, post_check=2 ("default" = none).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gelly-streaming_amd"))

import torch  # noqa: E402

from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402

DIGESTS = json.load(open(os.path.join(ROOT, "tests", "golden", "stream_digests.json")))


def parse_variant(s: str) -> dict:
    if s in ("", "default"):
        return {}
    out = {}
    for kv in s.split(","):
        k, v = kv.split("=")
        out[k.strip()] = float(v)
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", default="c3_gnm24/w1M")
    ap.add_argument("--seconds", type=float, default=60.0, help="per variant")
    ap.add_argument("--max-streams", type=int, default=100000)
    ap.add_argument("--variant", action="append", default=None)
    ap.add_argument("--post-check", type=int, default=2)
    ap.add_argument("--no-digest", action="store_true", help="skip the per-window digest (the post check still runs)")
    ap.add_argument("--out", default=None, help="JSON summary path")
    a = ap.parse_args()
    variants = a.variant or ["default"]
    fx = DIGESTS[a.fixture]
    cfg = G.CONFIGS[fx["config"]]
    E, V = cfg.info()
    starts = [0] + [w["end"] for w in fx["windows"]]
    d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
    G.generate_device(cfg, 0, E, d.data_ptr(), 0)
    torch.cuda.synchronize()
    summary = {"fixture": a.fixture, "windows": len(starts) - 1, "variants": []}
    for vs in variants:
        knobs = parse_variant(vs)
        t0 = time.time()
        last = t0
        n_streams = bad_windows = inc_checks = offenders = 0
        bad = []
        records = []
        while time.time() - t0 < a.seconds and n_streams < a.max_streams:
            ds = DisjointSet(V)
            ds.tune(incremental=1, post_check=a.post_check, **knobs)
            for w in range(len(starts) - 1):
                ds.fold_device(d.data_ptr() + 8 * starts[w], starts[w + 1] - starts[w])
                if a.no_digest:
                    ds.compress()
                    continue
                dig, seen, comps = ds.label_digest()
                want = fx["windows"][w]
                if (str(dig), seen, comps) != (want["digest"], want["seen"], want["components"]):
                    bad_windows += 1
                    bad.append({"stream": n_streams, "window": w, "seen": seen, "components": comps,
                                "seen_ok": seen == want["seen"], "components_ok": comps == want["components"]})
            c, o, recs = ds.post_check_stats()
            inc_checks += c
            offenders += o
            for r in recs:
                records.append({"stream": n_streams, "check": r[0], "v": r[1], "label": r[2], "label_of_label": r[3],
                                "root": r[4], "marked": r[5], "prev_v": r[6], "prev_label": r[7]})
            ds.close()
            n_streams += 1
            if time.time() - last > 5:
                last = time.time()
                print(f"[{vs}] {n_streams} streams, {inc_checks} incremental compresses, {bad_windows} wrong windows, "
                      f"{offenders} offenders", flush=True)
        line = {"variant": vs, "knobs": knobs, "streams": n_streams, "inc_compresses": inc_checks,
                "wrong_windows": bad_windows, "offenders": offenders, "seconds": round(time.time() - t0, 1),
                "bad": bad[:20], "records": records[:40]}
        summary["variants"].append(line)
        print(json.dumps({k: v for k, v in line.items() if k not in ("bad", "records")}), flush=True)
        for r in records[:12]:
            print("  offender", json.dumps(r), flush=True)
        for b in bad[:8]:
            print("  wrong window", json.dumps(b), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(summary, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
