"""Oracle digests of the full benchmark streams -> tests/golden/stream_digests.json (a fixture).

TEST INFRASTRUCTURE: run HERE (CPU container) with the C oracle (oracle/cc_oracle.c, the restatement of
DisjointSet / CombineCC / SummaryBulkAggregation). The GPU tests and bench.py compare the HIP path's final labels
with these digests, so no GPU run has to spend minutes of box time re-running the oracle on 1B-edge streams.

Entries: "<config>" = the whole stream of generators.CONFIGS[config] (the partition after its last window, which
is the partition of all its edges, whatever the window size); "c2_rmat20@k" = batch k of C2's generator, edges
[k*2^24, (k+1)*2^24) (bench.py rotates over batches 0..3 so that no step re-reads a batch still in the 256 MiB
Infinity Cache). digest = sum_v splitmix64((label[v] << 32) | v) mod 2^64 (oracle.label_digest).

Windowed entries "<config>/w<W>" (the parity contract is per merge window, SummaryAggregation.java:
107-119): the stream in windows of W edges; "windows" lists, per window, the end edge and the digest / seen /
component counts of the emitted summary (all edges up to that end).

Usage: python tests/golden/make_stream_digests.py [name ...]   (default: every missing entry)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle")]
import oracle as orc  # noqa: E402  (checker)
from gelly_stream import generators as G  # noqa: E402

PATH = os.path.join(ROOT, "tests", "golden", "stream_digests.json")
C2_BATCHES = 4


def entries():
    names = ["c2_rmat20", "c3_gnm24", "c5_adversarial", "c4_share", "c4_quarter", "c4_half", "c4_kron26"]
    names += [f"c2_rmat20@{k}" for k in range(1, C2_BATCHES)]
    names += list(WINDOWED)
    return names


# windowed entries: name -> (config, edges per window)
WINDOWED = {
    "c4_kron26/w8": ("c4_kron26", 1 << 27),
    "c2_rmat20/w1M": ("c2_rmat20", 1 << 20),
    "c3_gnm24/w4M": ("c3_gnm24", 1 << 22),
    "c3_gnm24/w1M": ("c3_gnm24", 1 << 20),
    "c5_adversarial/w64K": ("c5_adversarial", 1 << 16),
}


def compute_windowed(name):
    cfg_name, W = WINDOWED[name]
    cfg = G.CONFIGS[cfg_name]
    E, V = cfg.info()
    pairs = G.generate_host(cfg)
    starts = list(range(0, E, W)) + [E]
    r = orc.cc_stream(pairs, starts, V, partitions=8, threads=8, want_digest=True)
    wins = [{"end": int(starts[w + 1]), "digest": str(int(r["digest"][w])), "seen": int(r["seen"][w]),
             "components": int(r["components"][w])} for w in range(len(starts) - 1)]
    return {"config": cfg_name, "window_edges": W, "edges": E, "vertices": V, "windows": wins}


def compute(name):
    if name in WINDOWED:
        return compute_windowed(name)
    if "@" in name:
        cfg_name, k = name.split("@")
        cfg = G.CONFIGS[cfg_name]
        E, V = cfg.info()
        first = int(k) * E
        pairs = G.generate_host(cfg, first, E)
    else:
        cfg = G.CONFIGS[name]
        E, V = cfg.info()
        first = 0
        pairs = G.generate_host(cfg)
    r = orc.cc_stream(pairs, [0, E], V, partitions=8, threads=8, want_digest=True)
    return {"first": first, "edges": E, "vertices": V, "digest": str(int(r["digest"][0])), "seen": int(r["seen"][0]),
            "components": int(r["components"][0])}


def main():
    out = json.load(open(PATH)) if os.path.exists(PATH) else {}
    names = sys.argv[1:] or [n for n in entries() if n not in out]
    for name in names:
        t = time.time()
        out[name] = compute(name)
        print(name, {k: v for k, v in out[name].items() if k != "windows"}, f"{time.time() - t:.0f}s", flush=True)
        with open(PATH, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
