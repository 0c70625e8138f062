"""Repro probe for the open incremental-compress observation: C3 in 4M-edge windows with inc_div = 8
(the last 1.03M-edge window takes the bloom-recording fold + incremental compress), repeated on fresh forests;
each repetition's last-window labels vs the oracle's. Variants: in place (default) and out of place. On a
mismatch: the raw forest walk of the first bad id and whether its parent chain's roots were marked... (the bloom
is internal: only the walk is shown). Usage: python tools/probe_inc_c3.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as orc  # noqa: E402
from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    cfg = G.CONFIGS["c3_gnm24"]
    E, V = cfg.info()
    W = 1 << 22
    starts = np.asarray(list(range(0, E, W)) + [E], dtype=np.uint64)
    pairs = G.generate_host(cfg)
    want = orc.cc_stream(pairs, starts, V, partitions=4, threads=4, want_labels=True)["labels"][-1]
    d = torch.from_numpy(pairs.view(np.int32).reshape(-1)).cuda()
    torch.cuda.synchronize()
    for variant, knobs in (("inplace", {"inc_div": 8}), ("spare", {"inc_div": 8, "inc_inplace": 0}),
                           ("full", {"incremental": 0})):
        bad_runs = 0
        for r in range(reps):
            with DisjointSet(V) as ds:
                ds.tune(**knobs)
                for w in range(len(starts) - 1):
                    b, e = int(starts[w]), int(starts[w + 1])
                    ds.fold_device(d.data_ptr() + 8 * b, e - b)
                    if w < len(starts) - 2:
                        ds.labels()
                raw = ds.raw_parent()
                lab = ds.labels()
                bad = np.flatnonzero(lab != want)
                if bad.size:
                    bad_runs += 1
                    v = int(bad[0])
                    walk = [v]
                    while raw[walk[-1]] < walk[-1] and len(walk) < 16:
                        walk.append(int(raw[walk[-1]]))
                    print(f"{variant} rep {r}: {bad.size} bad; first {v}: got {int(lab[v])} want {int(want[v])}; "
                          f"raw walk {walk}", flush=True)
        print(f"{variant}: {bad_runs}/{reps} runs with a mismatch", flush=True)


if __name__ == "__main__":
    main()
