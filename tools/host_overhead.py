"""Host-side enqueue cost of a windowed step (one process, one GPU): per step, the time the host spends inside the
fold / emission calls (no synchronisation inside a step) against the step's wall time once the stream is drained; and
the host's time per window after the first (a fresh forest's first fold may wait for the device: its vote-share check
reads one word back). If the host's time per window reaches the wall's, the GPU waits for the next launch.

  python tools/host_overhead.py c2_rmat20/w1M --steps 50
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


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("fixture")
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    fx = DIGESTS[a.fixture]
    cfg = G.CONFIGS[fx["config"]]
    E, V = cfg.info()
    starts = [0] + [w["end"] for w in fx["windows"]]
    d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
    G.generate_device(cfg, 0, E, d.data_ptr(), 0)
    torch.cuda.synchronize()
    ds = DisjointSet(V)
    fold, emit = ds.fold_device, ds.compress
    ptrs = [(d.data_ptr() + 8 * starts[w], starts[w + 1] - starts[w]) for w in range(len(starts) - 1)]

    def step(acc, rest=None):
        t0 = time.perf_counter()
        ds.reset()
        t1 = None
        for w, (p, n) in enumerate(ptrs):
            fold(p, n)
            emit()
            if w == 0:
                t1 = time.perf_counter()  # (a fresh forest's first fold may wait for the device: the share check)
        ds.labels_device()
        t2 = time.perf_counter()
        acc.append(t2 - t0)
        if rest is not None and len(ptrs) > 1:
            rest.append((t2 - t1) / (len(ptrs) - 1))

    for _ in range(3):
        step([])
    ds.sync()
    host, rest = [], []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(host, rest)
    ds.sync()
    wall = (time.perf_counter() - t0) / a.steps
    h = sorted(host)[len(host) // 2]
    print(json.dumps({"fixture": a.fixture, "windows": len(ptrs), "wall_ms_per_step": round(wall * 1e3, 4),
                      "host_enqueue_ms_per_step_median": round(h * 1e3, 4),
                      "host_us_per_window": round(h * 1e6 / len(ptrs), 2),
                      "host_share_of_wall": round(h / wall, 3),
                      "host_us_per_window_after_first": round(sorted(rest)[len(rest) // 2] * 1e6, 2) if rest else None,
                      "wall_us_per_window": round(wall * 1e6 / len(ptrs), 2)}))
    ds.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
