"""GPU diagnostic: fold a fixture stream window by window; on a mismatch report whether the fold (raw
parent partition) or the compress is wrong, and how often it happens over repeated runs."""
import json
import os
import sys

import numpy as np
from scipy.sparse import coo_matrix
from scipy.sparse.csgraph import connected_components

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle")]
import oracle as orc  # noqa: E402
from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402

U = 0xFFFFFFFF


def partition_labels(par):
    """canonical labels implied by a raw parent array (seen = parent != UNSEEN)"""
    V = par.size
    seen = np.flatnonzero(par != U)
    g = coo_matrix((np.ones(seen.size), (seen, par[seen].astype(np.int64))), shape=(V, V))
    _, comp = connected_components(g, directed=False)
    out = np.full(V, U, dtype=np.uint32)
    mins = np.full(comp.max() + 1, 1 << 62, dtype=np.int64)
    np.minimum.at(mins, comp[seen], seen)
    out[seen] = mins[comp[seen]]
    return out


def main(reps=20):
    fx = json.load(open(os.path.join(ROOT, "tests/golden/stream_adversarial_p10.json")))
    g = fx["generator"]
    cfg = G.scaled(G.CONFIGS["c5_adversarial"], scale=g["scale"], n_stars=g["n_stars"], star_size=g["star_size"], seed=g["seed"])
    pairs = G.generate_host(cfg)
    st = fx["window_starts"]
    V = fx["V"]
    want = orc.cc_stream(pairs, st, V, want_labels=True)["labels"]
    bad_fold = bad_comp = 0
    for rep in range(reps):
        ds = DisjointSet(V)
        for w in range(len(st) - 1):
            ds.fold(pairs[st[w]:st[w + 1]])
            raw = ds.raw_parent()
            inv = np.flatnonzero((raw != U) & (raw > np.arange(V)))
            impl = partition_labels(raw)
            lab = ds.labels()
            fold_ok = np.array_equal(impl, want[w])
            comp_ok = np.array_equal(lab, impl)
            if not fold_ok or not comp_ok or inv.size:
                d = np.flatnonzero(lab != want[w])
                print(f"rep {rep} window {w}: fold_ok={fold_ok} compress_ok={comp_ok} invariant_violations={inv.size} "
                      f"label_mismatches={d.size} first={[(int(i), int(lab[i]), int(want[w][i]), int(raw[i])) for i in d[:5]]}")
                bad_fold += not fold_ok
                bad_comp += not comp_ok
        ds.close()
    print(f"reps={reps} bad_fold={bad_fold} bad_compress={bad_comp}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
