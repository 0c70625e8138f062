"""Fold one workload a few times (fresh forest each time): a short program to run under rocprofv3 (--pmc passes or
--kernel-trace --stats) without the bench's extra legs. Usage: python tools/fold_once.py [workload] [reps] [k=v,...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import torch  # noqa: E402

from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c4_kron26"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
knobs = {k: float(v) for k, v in (kv.split("=") for kv in sys.argv[3].split(","))} if len(sys.argv) > 3 else {}
cfg = G.CONFIGS[wl]
E, V = cfg.info()
d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
G.generate_device(cfg, 0, E, d.data_ptr(), 0)
torch.cuda.synchronize()
ds = DisjointSet(V)
ds.tune(**knobs)
for _ in range(reps):
    ds.reset()
    ds.fold_device(d.data_ptr(), E)
    ds.compress()
ds.sync()
print(wl, E, V, "seen", ds.size())
