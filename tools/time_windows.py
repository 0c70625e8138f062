"""A/B timing of tuning knobs on a windowed bench stream (one process, one GPU): per variant, K steps of reset + per
window a fold and an emission (compress), no synchronisation inside a step (bench.py's step); then one step with
every window's digest against tests/golden/stream_digests.json. Variants interleaved over rounds (box drift).

  python tools/time_windows.py c5_adversarial/w64K --steps 10 --rounds 3 --variant incremental=1 --variant incremental=0
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gelly-streaming_amd"))

import torch  # noqa: E402

from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402

DIGESTS = json.load(open(os.path.join(ROOT, "tests", "golden", "stream_digests.json")))


def forest_digest(parent):
    """(digest, seen, components) of a raw forest (parent[v] = UNSEEN, v for a root, or a smaller id): its labels by
    pointer jumping, then the fixtures' digest formula (bench.label_digest)."""
    import numpy as np

    sys.path.insert(0, ROOT)
    from bench import label_digest

    p = np.asarray(parent, dtype=np.uint32)
    seen = p != 0xFFFFFFFF
    lab = p.copy()
    idx = np.flatnonzero(seen)
    while True:
        nxt = lab[lab[idx]]
        if np.array_equal(nxt, lab[idx]):
            break
        lab[idx] = nxt
    comps = int(np.count_nonzero(lab[idx] == idx))
    return label_digest(lab), int(idx.size), comps


def knobs_of(s: str) -> dict:
    if s in ("", "default"):
        return {}
    return {k.strip(): float(v) for k, v in (kv.split("=") for kv in s.split(","))}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("fixture")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variant", action="append", default=None)
    ap.add_argument("--profile", action="store_true", help="also per-kernel ms per step (dispatch events)")
    ap.add_argument("--window-edges", type=int, default=0,
                    help="fixed windows over a one-window fixture (only the last window's digest is checked)")
    a = ap.parse_args()
    fx = DIGESTS[a.fixture]
    cfg = G.CONFIGS[fx.get("config", a.fixture)]
    E, V = cfg.info()
    starts = [0] + [w["end"] for w in fx["windows"]] if "windows" in fx else [0, E]
    if a.window_edges and "windows" not in fx:
        starts = list(range(0, E, a.window_edges)) + [E]
    d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
    G.generate_device(cfg, 0, E, d.data_ptr(), 0)
    torch.cuda.synchronize()
    variants = a.variant or ["default"]
    forests = {}
    for v in variants:
        ds = DisjointSet(V)
        ds.tune(**knobs_of(v))
        forests[v] = ds

    def step(ds):
        ds.reset()
        for w in range(len(starts) - 1):
            ds.fold_device(d.data_ptr() + 8 * starts[w], starts[w + 1] - starts[w])
            ds.compress()
        ds.labels_device()  # the stream's final summary materialised as labels (a lazy emission's last compress)

    times = {v: [] for v in variants}
    for r in range(a.rounds):
        for v in variants:
            ds = forests[v]
            step(ds)
            ds.sync()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step(ds)
            ds.sync()
            times[v].append((time.perf_counter() - t0) / a.steps * 1e3)
    chk = DisjointSet(V)
    for v in variants:
        ds = forests[v]
        bad = []
        ds.reset()
        for w in range(len(starts) - 1):
            ds.fold_device(d.data_ptr() + 8 * starts[w], starts[w + 1] - starts[w])
            ds.compress()  # the emission, lazy or not
            if "windows" not in fx and w < len(starts) - 2:
                continue  # (fixed windows over a one-window fixture: the last one is checked)
            # the emitted summary as it stands: the raw forest (no compress of ds, so a lazy emission's state is what
            # is checked) merged into a fresh forest on the device (CombineCC reads parent pointers), its digest there
            chk.reset()
            chk.merge(ds)
            got, seen, comps = chk.label_digest()
            want = fx["windows"][w] if "windows" in fx else fx
            if (str(got), seen, comps) != (want["digest"], want["seen"], want["components"]):
                bad.append(w)
        line = {"variant": v, "ms_per_step": [round(x, 4) for x in times[v]], "median_ms": round(statistics.median(times[v]), 4),
                "windows": len(starts) - 1, "edges_per_s": E / (statistics.median(times[v]) / 1e3),
                "parity": "bit-exact (every window)" if not bad else f"MISMATCH windows {bad[:10]}"}
        if a.profile:
            ds.enable_timing(1)
            ds.fold_profile()
            step(ds)
            prof = {}
            for name, ms, _ in ds.fold_profile():
                if name in ("begin", "fold_span", "slow_edges"):
                    continue
                prof[name] = prof.get(name, 0.0) + ms
            line["kernels_ms_per_step"] = {k: round(x, 4) for k, x in prof.items()}
            ds.enable_timing(0)
        print(json.dumps(line), flush=True)
        ds.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
