"""Probe (not product): does edge order within a window change the plain fold's speed on C3 (uniform G(n,m),
no dominant component)? Folds the same window in its stream order and after device sorts that localise parent[]
accesses, checks the labels are identical, and times the sorts. Usage: python tools/probe_c3_order.py [wl] [reps]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3_gnm24"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    cfg = G.CONFIGS[wl]
    E, V = cfg.info()
    d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
    G.generate_device(cfg, 0, E, d.data_ptr(), 0)
    torch.cuda.synchronize()
    pr = d.view(E, 2).to(torch.int64) & 0xFFFFFFFF
    lo, hi = torch.minimum(pr[:, 0], pr[:, 1]), torch.maximum(pr[:, 0], pr[:, 1])
    canon = torch.stack([lo, hi], 1).to(torch.int32).contiguous()  # (lo, hi) per edge, stream order

    def by_key(key):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        idx = torch.sort(key, stable=True).indices
        out = canon[idx].contiguous()
        ev1.record()
        torch.cuda.synchronize()
        return out, ev0.elapsed_time(ev1)

    variants = [("stream order", d.view(E, 2), 0.0), ("canonical (lo, hi)", canon, 0.0)]
    for bits in (0, 8, 12, 16):
        out, ms = by_key(lo >> bits)
        variants.append((f"sorted by lo>>{bits}", out, ms))
    out, ms = by_key(hi)
    variants.append(("sorted by hi", out, ms))
    ref = None
    for knobs in ({"filter": 0}, {}):
        for name, arr, sort_ms in variants:
            arr = arr.contiguous()
            ds = DisjointSet(V)
            ds.tune(**knobs)
            ds.enable_timing(1)
            t = []
            for _ in range(reps):
                ds.reset()
                ds.fold_device(arr.data_ptr(), E)
                t.append(ds.last_fold_ms())
            lab = ds.labels()
            if ref is None:
                ref = lab
            ok = np.array_equal(lab, ref)
            print(f"{str(knobs):14s} {name:22s} fold {statistics.median(t):7.3f} ms (min {min(t):.3f})"
                  f"  sort {sort_ms:6.3f} ms  {'OK' if ok else 'MISMATCH'}", flush=True)
            ds.close()


if __name__ == "__main__":
    main()
