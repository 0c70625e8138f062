"""The raw forest a fold leaves behind (before the compress): the depth of every seen id (hops to its root), as a
histogram. It tells what the closing compress has to walk. Usage: python tools/probe_depth.py [workload] [k=v,...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import torch  # noqa: E402

from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c3_gnm24"
knobs = {k: float(v) for k, v in (kv.split("=") for kv in sys.argv[2].split(","))} if len(sys.argv) > 2 else {}
cfg = G.CONFIGS[wl]
E, V = cfg.info()
d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
G.generate_device(cfg, 0, E, d.data_ptr(), 0)
torch.cuda.synchronize()
ds = DisjointSet(V)
ds.tune(**knobs)
ds.fold_device(d.data_ptr(), E)
p = ds.raw_parent().astype(np.int64)
seen = p != 0xFFFFFFFF
ids = np.arange(V, dtype=np.int64)
depth = np.zeros(V, dtype=np.int64)
act = np.flatnonzero(seen & (p != ids))  # seen non-roots: walking
cur = p[act]
depth[act] = 1
while act.size:
    nxt = p[cur]
    go = nxt != cur  # cur is not a root yet
    act, cur = act[go], nxt[go]
    depth[act] += 1
h = np.bincount(depth[seen])
print(wl, "E", E, "V", V, "seen", int(seen.sum()), "roots", int((seen & (p == ids)).sum()))
print("depth histogram (0 = root):", {i: int(c) for i, c in enumerate(h)})
print("hops a per-id walk takes (sum of depths beyond 1):", int(np.maximum(depth[seen] - 1, 0).sum()))
