"""One-GPU estimate of the strong-split bench's per-rank work at C4 (bench.py at N > 1): P forests each fold the
r-th 1/P of the C4 stream (fresh forests, the bucketed fold), then the one-device group merge
(gcc_group_merge: every forest encodes its compact message into one buffer, every forest absorbs the P-1 others
and compresses). The RCCL transfer is not in it; on one GPU the P absorbs run one after the other, so the merge
time per rank is the call's time / P. Usage: python tools/merge_c4.py [P ...]"""
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
    ps = [int(x) for x in sys.argv[1:]] or [2, 4, 8]
    cfg = G.CONFIGS["c4_kron26"]
    E, V = cfg.info()
    d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
    G.generate_device(cfg, 0, E, d.data_ptr(), 0)
    torch.cuda.synchronize()
    for P in ps:
        forests = [DisjointSet(V) for _ in range(P)]
        fold_ms, merge_ms = [], []
        for rep in range(3):
            per = []
            for r, ds in enumerate(forests):
                lo, hi = E * r // P, E * (r + 1) // P
                ds.reset()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ds.fold_device(d.data_ptr() + 8 * lo, hi - lo)
                ds.sync()
                per.append((time.perf_counter() - t0) * 1e3)
            fold_ms.append(max(per))
            torch.cuda.synchronize()
            if rep == 0:  # the compact message each rank would send: header + giant bitmap + (v, label) of the others
                import numpy as np
                msg = []
                for ds in forests:
                    lab = ds.labels()
                    seen = lab[lab != 0xFFFFFFFF]
                    giant = int(np.bincount(seen).max()) if seen.size else 0
                    msg.append(16 + V // 8 + 8 * (seen.size - giant))
                print(f"P={P}: message bytes per rank max {max(msg)} (bitmap {V // 8}, list {max(msg) - 16 - V // 8})",
                      flush=True)
            t0 = time.perf_counter()
            group_merge(forests)
            for ds in forests:
                ds.sync()
            merge_ms.append((time.perf_counter() - t0) * 1e3)
        n_seen = forests[0].size()
        print(f"P={P}: fold of 1/{P} of C4 per forest {min(fold_ms):.2f} ms (max over forests), one-device group "
              f"merge {min(merge_ms):.2f} ms total = {min(merge_ms) / P:.2f} ms per forest; seen {n_seen}", flush=True)
        for ds in forests:
            ds.close()


if __name__ == "__main__":
    main()
