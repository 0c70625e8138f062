"""Does C4's step time follow the placement of the bucketed fold's scratch? One forest folds C4 repeatedly; before
every trial the scratch is re-allocated (tune scratch_realloc: 1 every list, 2 the bucket storage, 3 the v-lists;
earlier buffers held so the new ones land elsewhere), and the trial's P1 / P2 / P3 / whole-fold times are printed.
Usage: python tools/placement_probe.py [mode] [trials]"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import torch  # noqa: E402

from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402

mode = int(sys.argv[1]) if len(sys.argv) > 1 else 1
trials = int(sys.argv[2]) if len(sys.argv) > 2 else 10
wl = sys.argv[3] if len(sys.argv) > 3 else "c4_kron26"
cfg = G.CONFIGS[wl]
E, V = cfg.info()
d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
G.generate_device(cfg, 0, E, d.data_ptr(), 0)
torch.cuda.synchronize()
ds = DisjointSet(V)


def step():
    ds.reset()
    ds.fold_device(d.data_ptr(), E)
    ds.compress()
    ds.labels_device()


for t in range(trials):
    if t:
        ds.tune(scratch_realloc=mode)
    step()
    ds.sync()
    t0 = time.perf_counter()
    for _ in range(5):
        step()
    ds.sync()
    wall = (time.perf_counter() - t0) / 5 * 1e3
    ds.enable_timing(1)
    ds.fold_profile()
    step()
    prof = {}
    for name, ms, _ in ds.fold_profile():
        prof[name] = prof.get(name, 0.0) + ms
    ds.enable_timing(0)
    print(f"mode {mode} trial {t}: step {wall:.3f} ms  P1 {prof.get('bucket', 0):.3f}  P2 {prof.get('slice_filter', 0):.3f}"
          f"  P3 {prof.get('slice_hook', 0):.3f}  init {prof.get('bucket_init', 0):.3f}", flush=True)
ds.close()
