"""Does C4's step time follow the forest (parent / spare buffers and all of its scratch)? K forests alive at once, each
folds C4 (reset + fold + emission + labels) a few times; per forest the step time and P1 / P2 / P3 from the fold
profile. Usage: python tools/forest_placement_probe.py [K] [rounds]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import torch  # noqa: E402

from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
R = int(sys.argv[2]) if len(sys.argv) > 2 else 2
cfg = G.CONFIGS["c4_kron26"]
E, V = cfg.info()
d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
G.generate_device(cfg, 0, E, d.data_ptr(), 0)
torch.cuda.synchronize()
forests = [DisjointSet(V) for _ in range(K)]


def step(ds):
    ds.reset()
    ds.fold_device(d.data_ptr(), E)
    ds.compress()
    ds.labels_device()


for ds in forests:
    step(ds)
    ds.sync()
for r in range(R):
    for i, ds in enumerate(forests):
        ds.sync()
        t0 = time.perf_counter()
        for _ in range(4):
            step(ds)
        ds.sync()
        wall = (time.perf_counter() - t0) / 4 * 1e3
        ds.enable_timing(1)
        ds.fold_profile()
        step(ds)
        prof = {}
        for name, ms, _ in ds.fold_profile():
            prof[name] = prof.get(name, 0.0) + ms
        ds.enable_timing(0)
        print(f"round {r} forest {i}: step {wall:.3f} ms  P1 {prof.get('bucket', 0):.3f}  P2 {prof.get('slice_filter', 0):.3f}"
              f"  P3 {prof.get('slice_hook', 0):.3f}  seed {prof.get('seed_filter', 0):.3f}", flush=True)
