"""Probe for the incremental-compress observation: C3 (G(n, m), 2^24 ids) in windows short enough that
the plain fold records its hooks in the bloom and the compress is incremental (inc_div = 8), on fresh forests, with
the library's inc_check diagnostics on: every incremental compress is compared with the roots of the forest it
started from, and every block's LDS copy of the bloom with memory-side reads of it (failures are printed by the
library to stderr). Every window's labels are also compared with the oracle's digest.
Usage: python tools/probe_inc_c3.py [reps] [window_log2 ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as orc  # noqa: E402
from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    wlogs = [int(x) for x in sys.argv[2:]] or [22, 20]
    cfg = G.CONFIGS["c3_gnm24"]
    E, V = cfg.info()
    pairs = G.generate_host(cfg)
    d = torch.from_numpy(pairs.view(np.int32).reshape(-1)).cuda()
    torch.cuda.synchronize()
    for wl in wlogs:
        W = 1 << wl
        starts = np.asarray(list(range(0, E, W)) + [E], dtype=np.uint64)
        want = orc.cc_stream(pairs, starts, V, partitions=4, threads=4)["digest"]
        for variant, knobs in (("inplace", {"inc_div": 8, "inc_check": 1}),
                               ("spare", {"inc_div": 8, "inc_inplace": 0, "inc_check": 1})):
            bad_windows = 0
            tot = [0, 0, 0]
            t0 = time.time()
            for r in range(reps):
                with DisjointSet(V) as ds:
                    ds.tune(**knobs)
                    for w in range(len(starts) - 1):
                        b, e = int(starts[w]), int(starts[w + 1])
                        ds.fold_device(d.data_ptr() + 8 * b, e - b)
                        lab = ds.labels()
                        if orc.label_digest(lab) != int(want[w]):
                            bad_windows += 1
                            print(f"W=2^{wl} {variant} rep {r} window {w}: digest mismatch vs the oracle", flush=True)
                    st = ds.inc_check_stats()
                    tot = [a + b for a, b in zip(tot, st)]
                print(f"  W=2^{wl} {variant} rep {r}: inc_check {st}", flush=True)
            print(f"W=2^{wl} {variant}: {reps} reps x {len(starts) - 1} windows: oracle mismatches {bad_windows}; "
                  f"inc_check: {tot[0]} checked compresses, {tot[1]} wrong labels, {tot[2]} lost bloom words "
                  f"({time.time() - t0:.1f} s)", flush=True)


if __name__ == "__main__":
    main()
