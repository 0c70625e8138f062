"""C3 split in P contiguous parts on one GPU, one forest per part, merged by gcc_group_merge (the compact
message exchange, repair rounds, label fallback), vs the oracle's digest of the whole stream. A probe for the
C3 N=2 path. Usage: python tools/probe_merge_c3.py [P]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle")]
import torch  # noqa: E402

import oracle as orc  # noqa: E402
from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402
from gelly_stream.distributed import group_merge  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 2
cfg = G.CONFIGS["c3_gnm24"]
E, V = cfg.info()
want = int(json.load(open(os.path.join(ROOT, "tests", "golden", "stream_digests.json")))["c3_gnm24"]["digest"])
d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
G.generate_device(cfg, 0, E, d.data_ptr(), 0)
torch.cuda.synchronize()
forests = [DisjointSet(V) for _ in range(P)]
for r, ds in enumerate(forests):
    lo, hi = E * r // P, E * (r + 1) // P
    ds.fold_device(d.data_ptr() + 8 * lo, hi - lo)
    ds.sync()
print("folded", flush=True)
group_merge(forests)
for r, ds in enumerate(forests):
    print(r, "digest ok" if orc.label_digest(ds.labels()) == want else "DIGEST MISMATCH", flush=True)
