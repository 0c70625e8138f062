"""Oracle digests of the full single-window streams (tools/digests.json), so GPU sweeps of the big configs do
not spend minutes of box time re-running the CPU oracle. Run here (CPU): python tools/make_digests.py [names]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle")]
import oracle as orc  # noqa: E402  (checker)
from gelly_stream import generators as G  # noqa: E402

PATH = os.path.join(ROOT, "tools", "digests.json")


def main():
    names = sys.argv[1:] or ["c2_rmat20", "c3_gnm24", "c5_adversarial", "c4_kron26", "c4_share"]
    out = json.load(open(PATH)) if os.path.exists(PATH) else {}
    for wl in names:
        cfg = G.CONFIGS[wl]
        E, V = cfg.info()
        t = time.time()
        pairs = G.generate_host(cfg)
        r = orc.cc_stream(pairs, [0, E], V, partitions=8, threads=8, want_digest=True)
        del pairs
        out[wl] = {"edges": E, "vertices": V, "digest": int(r["digest"][0]), "seen": int(r["seen"][0]),
                   "components": int(r["components"][0])}
        print(wl, out[wl], f"{time.time() - t:.0f}s", flush=True)
        json.dump(out, open(PATH, "w"), indent=1)


if __name__ == "__main__":
    main()
