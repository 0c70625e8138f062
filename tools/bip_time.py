"""bench.py's BipartitenessCheck legs alone (bench.bip_legs), C4's first 2^27 edges generated on the device:
python tools/bip_time.py [steps] [warmup] [k=v,...]  -> one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gelly-streaming_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from gelly_stream import generators as G  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
warmup = int(sys.argv[2]) if len(sys.argv) > 2 else 1
share = 1 << 27
d = torch.empty(2 * share, dtype=torch.int32, device="cuda:0")
G.generate_device(G.CONFIGS["c4_kron26"], 0, share, d.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
tune = dict((k, float(v)) for k, v in (kv.split("=") for kv in sys.argv[3].split(","))) if len(sys.argv) > 3 else None
out = bench.bip_legs(0, steps, warmup, d_edges=d, tune=tune)
print(json.dumps(out))
