"""The delta merge's per-window cost at C5's short windows (DESIGN.md §6's predicted curve): P forests on one GPU fold
the r-th 1/P of every C5 window and merge with gcc_group_merge (one device: the delta messages through one buffer,
no transport), every window. Prints the wall time per window of the fold + merge; under rocprofv3 --kernel-trace
--stats the delta_encode_kernel / delta_absorb_kernel averages are the merge's device cost per window.
Usage: python tools/delta_probe.py [P] [windows]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import torch  # noqa: E402

from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402
from gelly_stream.distributed import group_merge  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    nwin = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    cfg = G.CONFIGS["c5_adversarial"]
    E, V = cfg.info()
    W = cfg.window_edges
    d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
    G.generate_device(cfg, 0, E, d.data_ptr(), 0)
    torch.cuda.synchronize()
    forests = [DisjointSet(V) for _ in range(P)]
    t_fold, t_merge = [], []
    for w in range(nwin):
        b = w * W
        t0 = time.perf_counter()
        for r, ds in enumerate(forests):
            lo, hi = b + W * r // P, b + W * (r + 1) // P
            ds.fold_device(d.data_ptr() + 8 * lo, hi - lo)
        for ds in forests:
            ds.sync()
        t1 = time.perf_counter()
        group_merge(forests)
        for ds in forests:
            ds.sync()
        t2 = time.perf_counter()
        if w >= 2:
            t_fold.append((t1 - t0) * 1e3)
            t_merge.append((t2 - t1) * 1e3)
    t_fold.sort()
    t_merge.sort()
    print(f"P={P} windows={nwin}: per window (median) folds of all P forests {t_fold[len(t_fold) // 2]:.3f} ms, "
          f"group merge (encode + header sync + absorb + arm of all P, serial on one GPU) {t_merge[len(t_merge) // 2]:.3f} ms",
          flush=True)
    for ds in forests:
        ds.close()


if __name__ == "__main__":
    main()
