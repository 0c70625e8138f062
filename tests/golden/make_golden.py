#!/usr/bin/env python3
"""Generate the committed golden fixtures in tests/golden/ (run in the build container; not at test time).

Independent of the C oracle and of libgelly_cc: everything here is pure Python + scipy, so the fixtures
pin both (tests/test_oracle_golden.py checks the C oracle and the C host generator against them).

  1. A pure-Python restatement of the reference's DisjointSet (…/summaries/DisjointSet.java:30-154,
     dict-based, union by rank, recursive find with path compression, merge), CombineCC
     (…/library/ConnectedComponents.java:116-125) and the SummaryBulkAggregation window topology
     (…/SummaryBulkAggregation.java:76-83 + Merger …/SummaryAggregation.java:107-119).
  2. The reference's own known-answer tests, replayed on that restatement:
       DisjointSetTest (src/test/java/org/apache/flink/graph/streaming/util/DisjointSetTest.java:36-78)
       ConnectedComponentsTest (…/example/test/ConnectedComponentsTest.java:19-21, :29-38, :73)
       ConnectedComponentsExample default data (…/example/ConnectedComponentsExample.java:78, :121-133)
  3. Every window's partition cross-checked against scipy.sparse.csgraph.connected_components.
  4. A pure-Python restatement of csrc/edge_gen.h for small streams (pins the device/host generator).

The Java reference cannot run here (no JDK/Flink), so these fixtures are the pin.
Usage: python tests/golden/make_golden.py   (rewrites tests/golden/*.json)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np
from scipy.sparse import coo_matrix
from scipy.sparse.csgraph import connected_components

HERE = os.path.dirname(os.path.abspath(__file__))
M64 = (1 << 64) - 1
UNSEEN = 0xFFFFFFFF
sys.setrecursionlimit(100000)


# --------------------------------------------------------------------------------------------------
# 1. DisjointSet restatement (pure Python)
# --------------------------------------------------------------------------------------------------
class PyDisjointSet:
    def __init__(self):
        self.matches = {}  # HashMap<R,R>  (:33)
        self.ranks = {}    # HashMap<R,Integer> (:34)

    def makeSet(self, e):  # :58-61
        self.matches[e] = e
        self.ranks[e] = 0

    def find(self, e):  # :71-85
        if e not in self.matches:
            return None
        parent = self.matches[e]
        if parent != e:
            tmp = self.find(parent)
            if parent != tmp:
                parent = tmp
                self.matches[e] = parent
        return parent

    def union(self, e1, e2):  # :97-123
        if e1 not in self.matches:
            self.makeSet(e1)
        if e2 not in self.matches:
            self.makeSet(e2)
        root1, root2 = self.find(e1), self.find(e2)
        if root1 == root2:
            return
        d1, d2 = self.ranks[root1], self.ranks[root2]
        if d1 > d2:
            self.matches[root2] = root1
        elif d1 < d2:
            self.matches[root1] = root2
        else:
            self.matches[root2] = root1
            self.ranks[root1] = d1 + 1

    def merge(self, other):  # :132-136
        for k, p in list(other.matches.items()):
            self.union(k, p)

    def labels(self, V):
        out = np.full(V, UNSEEN, dtype=np.uint32)
        mins = {}
        for k in self.matches:
            r = self.find(k)
            mins[r] = min(mins.get(r, k), k)
        for k in self.matches:
            out[k] = mins[self.find(k)]
        return out


def combine_cc(s1, s2):  # CombineCC.reduce :116-125
    if len(s1.matches) <= len(s2.matches):
        s2.merge(s1)
        return s2
    s1.merge(s2)
    return s1


def run_topology(pairs, starts, V, partitions):
    """Per emitted window: canonical labels of the running summary."""
    summary = PyDisjointSet()
    out = []
    for w in range(len(starts) - 1):
        b, e = int(starts[w]), int(starts[w + 1])
        if e == b:
            out.append(None)  # no emission
            continue
        L = e - b
        acc = None
        for p in range(partitions):
            pb, pe = b + L * p // partitions, b + L * (p + 1) // partitions
            if pe == pb:
                continue
            ds = PyDisjointSet()
            for i in range(pb, pe):
                ds.union(int(pairs[i][0]), int(pairs[i][1]))  # UpdateCC.foldEdges :83-86
            acc = ds if acc is None else combine_cc(acc, ds)
        summary = combine_cc(acc, summary)  # Merger.flatMap :110
        out.append(summary.labels(V))
    return out


def scipy_labels(pairs, V):
    """Canonical labels of the graph on `pairs` via scipy (seen = endpoints)."""
    out = np.full(V, UNSEEN, dtype=np.uint32)
    if len(pairs) == 0:
        return out
    a = np.asarray(pairs, dtype=np.int64)
    g = coo_matrix((np.ones(len(a)), (a[:, 0], a[:, 1])), shape=(V, V))
    _, comp = connected_components(g, directed=False)
    seen = np.zeros(V, dtype=bool)
    seen[a[:, 0]] = True
    seen[a[:, 1]] = True
    mins = np.full(comp.max() + 1, np.iinfo(np.int64).max, dtype=np.int64)
    idx = np.flatnonzero(seen)
    np.minimum.at(mins, comp[idx], idx)
    out[idx] = mins[comp[idx]].astype(np.uint32)
    return out


def digest(labels):
    """sum_v splitmix64((label[v] << 32) | v) mod 2^64 (same as oracle/cc_oracle.c orc_label_digest)."""
    h = 0
    for v, l in enumerate(np.asarray(labels, dtype=np.uint64).tolist()):
        h = (h + splitmix64(((l << 32) | v) & M64)) & M64
    return h


# --------------------------------------------------------------------------------------------------
# 4. generator restatement (csrc/edge_gen.h), pure Python ints
# --------------------------------------------------------------------------------------------------
def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def perm_bits(x, bits, key):
    mask = (1 << bits) - 1
    sh = (bits + 1) // 2
    for r in range(3):
        km = splitmix64((key + 2 * r) & M64) | 1
        ka = splitmix64((key + 2 * r + 1) & M64)
        x = (x * km) & mask
        x = (x + ka) & mask
        x ^= x >> sh
    return x


KEY_PERM, KEY_PATH, KEY_SHUF, KEY_DIR = 0x7065726D75746531, 0x706174687065726D, 0x73687566666C6531, 0x6469726563746E31
T_A, T_AB, T_ABC = 2448131358, 3264175144, 4080218931


def gen_rmat(scale, n_edges, seed, permute=1):
    out = []
    for i in range(n_edges):
        base = splitmix64(seed ^ splitmix64(i))
        u = v = 0
        r = 0
        for lvl in range(scale):
            if lvl % 2 == 0:
                r = splitmix64((base + lvl // 2) & M64)
            d = (r >> (32 * (lvl & 1))) & 0xFFFFFFFF
            if d < T_A:
                bu, bv = 0, 0
            elif d < T_AB:
                bu, bv = 0, 1
            elif d < T_ABC:
                bu, bv = 1, 0
            else:
                bu, bv = 1, 1
            u, v = (u << 1) | bu, (v << 1) | bv
        if permute:
            u, v = perm_bits(u, scale, seed ^ KEY_PERM), perm_bits(v, scale, seed ^ KEY_PERM)
        out.append((u, v))
    return out


def gen_gnm(n, m, seed):
    out = []
    for i in range(m):
        base = splitmix64(seed ^ splitmix64(i))
        out.append(((splitmix64(base) * n) >> 64, (splitmix64((base + 1) & M64) * n) >> 64))
    return out


def gen_adversarial(P, S, L, seed):
    E = (1 << P) - 1 + S * (L - 1)
    dbits = max(0, (E - 1).bit_length())
    out = []
    for i in range(E):
        j = perm_bits(i, dbits, seed ^ KEY_SHUF)
        while j >= E:
            j = perm_bits(j, dbits, seed ^ KEY_SHUF)
        npath = (1 << P) - 1
        if j < npath:
            u, v = perm_bits(j, P, seed ^ KEY_PATH), perm_bits(j + 1, P, seed ^ KEY_PATH)
        else:
            k = j - npath
            hub = (1 << P) + (k // (L - 1)) * L
            u, v = hub, hub + 1 + k % (L - 1)
        if splitmix64(seed ^ KEY_DIR ^ i) & 1:
            u, v = v, u
        out.append((u, v))
    return out


def pairs_sha256(pairs):
    return hashlib.sha256(np.asarray(pairs, dtype="<u4").tobytes()).hexdigest()


# --------------------------------------------------------------------------------------------------
def check_against_scipy(pairs, starts, V, windows):
    for w, lab in enumerate(windows):
        if lab is None:
            continue
        ref = scipy_labels(pairs[: int(starts[w + 1])], V)
        if not np.array_equal(ref, lab):
            raise SystemExit(f"restatement disagrees with scipy at window {w}")


def stream_fixture(name, pairs, starts, V, params, full_label_windows="last"):
    pairs = np.asarray(pairs, dtype=np.uint32).reshape(-1, 2)
    win1 = run_topology(pairs, starts, V, partitions=1)
    win4 = run_topology(pairs, starts, V, partitions=4)
    for a, b in zip(win1, win4):
        assert (a is None and b is None) or np.array_equal(a, b), "partition count changed the partition"
    check_against_scipy(pairs, starts, V, win1)
    fx = {
        "name": name,
        "generator": params,
        "V": V,
        "n_edges": int(len(pairs)),
        "edges_sha256": pairs_sha256(pairs),
        "window_starts": [int(x) for x in starts],
        "windows": [],
    }
    for w, lab in enumerate(win1):
        if lab is None:
            fx["windows"].append({"emitted": False})
            continue
        seen = lab != UNSEEN
        entry = {
            "emitted": True,
            "seen": int(seen.sum()),
            "components": int(np.unique(lab[seen]).size),
            "digest": str(digest(lab)),
        }
        if full_label_windows == "all" or (full_label_windows == "last" and w == len(win1) - 1):
            entry["labels"] = [int(x) for x in lab]
        fx["windows"].append(entry)
    return fx


def write(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", name)


def main():
    # ---- DisjointSetTest (util/DisjointSetTest.java:36-78) ----
    ds = PyDisjointSet()
    setup = [(i, i + 2) for i in range(8)]
    for a, b in setup:
        ds.union(a, b)
    assert len(ds.matches) == 10  # :45
    r0, r1 = ds.find(0), ds.find(1)
    assert r0 != r1 and all(ds.find(i) == (r0 if i % 2 == 0 else r1) for i in range(10))  # :49-57
    ds2 = PyDisjointSet()
    ds2_edges = [(i, i + 100) for i in range(8)]
    for a, b in ds2_edges:
        ds2.union(a, b)
    ds2.merge(ds)
    assert len(ds2.matches) == 18  # :69
    roots = {ds2.find(k) for k in ds2.matches}
    assert len(roots) == 2  # :77
    write("kat_disjoint_set.json", {
        "source": "src/test/java/org/apache/flink/graph/streaming/util/DisjointSetTest.java:36-78",
        "setup_edges": setup, "size": 10,
        "labels": {str(k): int(v) for k, v in enumerate(ds.labels(10).tolist())},
        "ds2_edges": ds2_edges, "merged_size": 18, "merged_roots": 2,
        "merged_labels": {str(k): int(ds2.labels(108)[k]) for k in sorted(ds2.matches)},
    })

    # ---- ConnectedComponentsTest (example/test/ConnectedComponentsTest.java:19-38, :73) ----
    edges = [(1, 2), (1, 3), (2, 3), (1, 5), (6, 7), (8, 9)]
    ds = PyDisjointSet()
    for a, b in edges:
        ds.union(a, b)
    lab = ds.labels(10)
    assert np.array_equal(lab, scipy_labels(np.array(edges), 10))
    comps = {}
    for v in sorted(ds.matches):
        comps.setdefault(int(lab[v]), []).append(v)
    assert sorted(comps.values()) == [[1, 2, 3, 5], [6, 7], [8, 9]]  # Connected_RESULT :19-21
    write("kat_connected_components.json", {
        "source": "src/test/java/org/apache/flink/graph/streaming/example/test/ConnectedComponentsTest.java:19-38,73",
        "edges": edges, "n_components": 3, "components": sorted(comps.values()),
        "labels": [int(x) for x in lab],
    })

    # ---- ConnectedComponentsExample default data, 1000 ms windows (:78, :121-133) ----
    ex = [(k, k + 2) for k in range(1, 101)]
    ts = np.array([k * 100 for k in range(1, 101)], dtype=np.int64)
    win = ts - ts % 1000
    starts = np.concatenate([[0], np.flatnonzero(np.diff(win)) + 1, [len(ts)]])
    fx = stream_fixture("c1_example", ex, starts, 103, {"kind": "EXAMPLE"}, full_label_windows="all")
    assert len(fx["windows"]) == 11
    for w, entry in enumerate(fx["windows"]):  # seen = {1..min(102, 10w+11)}, labels 1 / 2
        hi = min(102, 10 * w + 11)
        want = [UNSEEN] * 103
        for v in range(1, hi + 1):
            want[v] = 1 if v % 2 else 2
        assert entry["labels"] == want, w
    fx["source"] = "src/main/java/org/apache/flink/graph/streaming/example/ConnectedComponentsExample.java:78,121-133"
    fx["timestamps_ms"] = ts.tolist()
    write("example_default.json", fx)

    # ---- small synthetic streams (generator restatement + topology + scipy) ----
    seed2, seed3, seed5 = 0x67656C6C79000002, 0x67656C6C79000003, 0x67656C6C79000005
    rm = gen_rmat(10, 16 << 10, seed2)
    write("stream_rmat_s10.json", stream_fixture(
        "rmat_s10", rm, list(range(0, 16 << 10, 1024)) + [16 << 10], 1 << 10,
        {"kind": "RMAT", "scale": 10, "n_edges": 16 << 10, "seed": seed2, "permute": 1}))
    gn = gen_gnm(4096, 2253, seed3)
    write("stream_gnm_4096.json", stream_fixture(
        "gnm_4096", gn, list(range(0, 2253, 512)) + [2253], 4096,
        {"kind": "GNM", "n_vertices": 4096, "n_edges": 2253, "seed": seed3}))
    adv = gen_adversarial(10, 8, 128, seed5)
    write("stream_adversarial_p10.json", stream_fixture(
        "adversarial_p10", adv, list(range(0, len(adv), 256)) + [len(adv)], (1 << 10) + 8 * 128,
        {"kind": "ADVERSARIAL", "scale": 10, "n_stars": 8, "star_size": 128, "seed": seed5}))


if __name__ == "__main__":
    main()
