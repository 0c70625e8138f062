"""CPU: pin the BipartitenessCheck oracle (oracle/bip_oracle.c) against the golden fixtures.

tests/golden/bip_kat.json holds the reference's own tests (BipartitenessCheckTest / NonBipartitnessCheckTest);
tests/golden/bip_*.json the streams pinned by networkx (tests/golden/make_golden_bip.py, which also records where a
literal restatement of the reference's Candidates.merge diverges from the intended partition semantics).
"""
import glob
import os

import numpy as np
import pytest

import oracle as orc

UNSEEN = 0xFFFFFFFF
HERE = os.path.dirname(os.path.abspath(__file__))


def canonical_string(success, words):
    """Candidates.toString of the canonical summary (the minimum vertex of each component carries `true`)."""
    if not success:
        return "(false,{})"
    comps = {}
    for v in np.flatnonzero(words != UNSEEN).tolist():
        comps.setdefault(int(words[v]) >> 1, []).append((v, (int(words[v]) & 1) == 0))
    body = ", ".join(f"{c}={{" + ", ".join(f"{v}=({v},{'true' if s else 'false'})" for v, s in sorted(m)) + "}"
                     for c, m in sorted(comps.items()))
    return "(true,{" + body + "})"


def test_oracle_reference_kats(golden):
    fx = golden("bip_kat.json")
    b = fx["bipartite"]
    r = orc.bip_stream(np.array(b["edges"], dtype=np.uint32), [0, len(b["edges"])], b["V"])
    assert r["success"][0]
    assert r["words"][0].tolist() == b["words"]
    assert canonical_string(True, r["words"][0]) == b["expected"]  # the reference test's expected line
    n = fx["non_bipartite"]
    r = orc.bip_stream(np.array(n["edges"], dtype=np.uint32), [0, len(n["edges"])], n["V"])
    assert not r["success"][0]
    assert canonical_string(False, r["words"][0]) == n["expected"]


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(HERE, "golden", "bip_*.json"))))
def test_oracle_streams(path, golden):
    name = os.path.basename(path)
    if name == "bip_kat.json":
        return
    fx = golden(name)
    pairs = np.array(fx["pairs"], dtype=np.uint32)
    r = orc.bip_stream(pairs, fx["window_starts"], fx["V"], partitions=fx["partitions"])
    for w, want in enumerate(fx["windows"]):
        assert bool(r["emitted"][w]) == (want is not None)
        if want is None:
            continue
        assert bool(r["success"][w]) == want["success"], (name, w)
        if want["success"]:
            assert r["words"][w].tolist() == want["words"], (name, w)


def test_oracle_partitions_do_not_change_the_result(golden):
    """The combine topology (partitions per window) never changes the canonical summary."""
    fx = golden("bip_large_bipartite_p4.json")
    pairs = np.array(fx["pairs"], dtype=np.uint32)
    ref = orc.bip_stream(pairs, fx["window_starts"], fx["V"], partitions=1)
    for p in (2, 3, 7):
        r = orc.bip_stream(pairs, fx["window_starts"], fx["V"], partitions=p)
        assert np.array_equal(r["words"], ref["words"]) and np.array_equal(r["success"], ref["success"])


# Where the reference's own Candidates (a literal restatement, tests/golden/make_golden_bip.py) differs from the
# intended semantics this build implements (bipartite iff no odd cycle; per component its minimum vertex and a
# 2-colouring). Pinned window by window: "partition" = the literal summary's components overlap or split
# (Candidates.java:176-189 files the input under min(inputKey, selfKey) without moving the self component),
# "success" = the literal reports success where an odd cycle exists (Candidates.java:92-95 skips components with
# identical vertex sets; :128-131 drops a failed second-level merge).
DIVERGENT = {
    "bip_random_bipartite.json": {0: "partition"},
    "bip_random_bipartite_p3.json": {0: "partition"},
    "bip_closes_odd_cycle.json": {0: "partition", 2: "success"},
    "bip_large_bipartite_p4.json": {0: "partition", 1: "partition"},
    "bip_same_vertex_sets_p2.json": {0: "success"},
    "bip_random_gnm_p3.json": {0: "partition"},
    "bip_random_sparse_p2.json": {0: "partition"},
    "bip_random_sparse_p5.json": {0: "partition"},
}


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(HERE, "golden", "bip_*.json"))))
def test_reference_literal_divergence_is_pinned(path, golden):
    """The windows on which the reference's literal output differs are exactly the pinned ones, and of the pinned
    kind; every other window agrees with it (up to the sign convention of its toString)."""
    name = os.path.basename(path)
    if name == "bip_kat.json":
        return
    fx = golden(name)
    got = {}
    for w, x in enumerate(fx["windows"]):
        if x is None:
            continue
        lit = x["reference_literal"]
        if not x["reference_literal_agrees"]:
            got[w] = "success" if lit["success"] != x["success"] else "partition"
        else:
            assert lit["success"] == x["success"]
    assert got == DIVERGENT.get(name, {}), (name, got)


def test_to_bipartite_and_bench_digests(golden):
    """generators.to_bipartite (bench.py's bip legs) makes every edge join an even id to an odd one, so the oracle
    never fails on it; digests_bip.json's small-scale analogue: the same mapping of a scaled C3 folds to success and
    its words digest is bench.label_digest's formula (make_bip_digests.words_digest)."""
    import sys

    from gelly_stream import generators as G

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_bip_digests as mk
    from bench import label_digest

    cfg = G.scaled(G.CONFIGS["c3_gnm24"], n_vertices=1 << 14, n_edges=1 << 15)
    E, V = cfg.info()
    raw = G.generate_host(cfg)
    pairs = G.to_bipartite(raw)
    assert np.all(pairs[:, 0] % 2 == 0) and np.all(pairs[:, 1] % 2 == 1) and pairs.max() < V
    assert np.array_equal(raw, G.generate_host(cfg))  # a copy, not in place
    r = orc.bip_stream(pairs, [0, E], V)
    assert r["success"][0]
    assert not orc.bip_stream(raw, [0, E], V)["success"][0]  # a random graph of this density has an odd cycle
    assert mk.words_digest(r["words"][0]) == label_digest(r["words"][0])
    fx = golden("digests_bip.json")
    assert set(fx) == set(mk.ENTRIES)
    assert fx["bip_c3_gnm24"]["success"] and fx["bip_c4_share"]["success"] and not fx["c3_gnm24"]["success"]
