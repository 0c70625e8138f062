"""P1's time per forest instance (tools/ab runs showed 3.3-4.2 ms on C4 between forests of one process): K forests
alive at once, each folds C4 a few times; prints P1 (bucket_kernel) ms per forest with its buffers' addresses
(GELLY_BUCKET_ADDR=1 prints them on stderr). Optional: a spacer allocation of S MiB between forests.
Usage: GELLY_BUCKET_ADDR=1 python tools/p1_placement.py [K] [spacer_mib] [workload]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import torch  # noqa: E402

from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
spacer = int(sys.argv[2]) if len(sys.argv) > 2 else 0
wl = sys.argv[3] if len(sys.argv) > 3 else "c4_kron26"
cfg = G.CONFIGS[wl]
E, V = cfg.info()
d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
G.generate_device(cfg, 0, E, d.data_ptr(), 0)
torch.cuda.synchronize()
forests, spacers = [], []
for i in range(K):
    ds = DisjointSet(V)
    ds.reset()
    ds.fold_device(d.data_ptr(), E)  # allocates its buffers
    ds.compress()
    ds.sync()
    forests.append(ds)
    if spacer:
        spacers.append(torch.empty(spacer << 20, dtype=torch.uint8, device="cuda:0"))
for rnd in range(2):
    for i, ds in enumerate(forests):
        ds.enable_timing(1)
        ms = []
        for _ in range(3):
            ds.fold_profile()
            ds.reset()
            ds.fold_device(d.data_ptr(), E)
            ds.compress()
            p1 = sum(m for name, m, _ in ds.fold_profile() if name == "bucket")
            ms.append(p1)
        ds.enable_timing(0)
        print(f"round {rnd} forest {i}: P1 {statistics.median(ms):.3f} ms ({', '.join(f'{x:.3f}' for x in ms)})", flush=True)
