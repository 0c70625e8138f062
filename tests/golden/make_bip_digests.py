"""Oracle digests of BipartitenessCheck's bench streams -> tests/golden/digests_bip.json (a fixture).

TEST INFRASTRUCTURE: run HERE (CPU container) with the C oracle (oracle/bip_oracle.c, the restatement of
Candidates / BipartitenessCheck). bench.py's bip legs and tests/test_gpu_bipartite.py compare the signed forest's
final words with these digests, so no GPU run spends box time on the oracle.

Entries (one window each, the whole stream folded into a fresh summary):
  "bip_c3_gnm24"  generators.to_bipartite(C3's stream): 9.2M edges over 2^24 ids, bipartite by construction
  "bip_c4_share"  generators.to_bipartite(C4's first 2^27 edges): the kron hubs, 2^26 ids, bipartite
  "c3_gnm24"      C3's stream as it is: a random graph, an odd cycle within its first edges (success false)
digest = sum_v splitmix64((word[v] << 32) | v) mod 2^64 over the canonical words (bench.label_digest's formula);
"seen" = ids with a word; "success" = Candidates.getSuccess. A failed summary's words are not part of the contract
(its value is (false, {})), so a failed entry carries no digest.

Usage: python tests/golden/make_bip_digests.py [name ...]   (default: every missing entry)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle")]
import oracle as orc  # noqa: E402  (checker)
from gelly_stream import generators as G  # noqa: E402

PATH = os.path.join(ROOT, "tests", "golden", "digests_bip.json")
ENTRIES = {  # name -> (config, edges or None = all, bipartite mapping)
    "bip_c3_gnm24": ("c3_gnm24", None, True),
    "bip_c4_share": ("c4_kron26", 1 << 27, True),
    "c3_gnm24": ("c3_gnm24", None, False),
}


def words_digest(words):
    w = np.asarray(words, dtype=np.uint64)
    x = (w << np.uint64(32)) | np.arange(w.size, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
        return int(np.sum(x, dtype=np.uint64))


def compute(name):
    cfg_name, count, bip = ENTRIES[name]
    cfg = G.CONFIGS[cfg_name]
    E, V = cfg.info()
    pairs = G.generate_host(cfg, 0, count if count else E)
    if bip:
        pairs = G.to_bipartite(pairs)
    r = orc.bip_stream(pairs, [0, len(pairs)], V, partitions=1)
    out = {"config": cfg_name, "edges": int(len(pairs)), "vertices": V, "bipartite_mapping": bip,
           "success": bool(r["success"][0])}
    if out["success"]:
        w = r["words"][0]
        out["digest"] = str(words_digest(w))
        out["seen"] = int(np.count_nonzero(w != 0xFFFFFFFF))
        out["components"] = int(np.count_nonzero((w >> 1) == np.arange(V, dtype=np.uint32)))
    return out


def main():
    out = json.load(open(PATH)) if os.path.exists(PATH) else {}
    names = sys.argv[1:] or [n for n in ENTRIES if n not in out]
    for name in names:
        t = time.time()
        out[name] = compute(name)
        print(name, out[name], f"{time.time() - t:.0f}s", flush=True)
        with open(PATH, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
