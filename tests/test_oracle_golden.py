"""CPU: pin the C oracle and the C host generator against the golden fixtures (reference KATs + scipy).

The fixtures (tests/golden/*.json) come from tests/golden/make_golden.py, a pure-Python restatement of
the reference cross-checked against scipy; nothing here touches the GPU.
"""
import hashlib

import numpy as np
import pytest

import oracle as orc
from gelly_stream import generators as G
from gelly_stream import native

UNSEEN = 0xFFFFFFFF


# ---- DisjointSetTest (src/test/java/org/apache/flink/graph/streaming/util/DisjointSetTest.java) ----
@pytest.fixture()
def ds_setup(golden):
    fx = golden("kat_disjoint_set.json")
    ds = orc.OracleDisjointSet()
    for a, b in fx["setup_edges"]:  # setup :36-41
        ds.union(a, b)
    return ds, fx


def test_oracle_get_matches(ds_setup):  # :43-46
    ds, fx = ds_setup
    assert ds.size() == fx["size"] == 10


def test_oracle_find(ds_setup):  # :48-57
    ds, fx = ds_setup
    root1, root2 = ds.find(0), ds.find(1)
    assert root1 != root2
    for i in range(10):
        assert ds.find(i) == (root1 if i % 2 == 0 else root2)
    assert ds.find(12345) is None  # find of an unseen key returns null (DisjointSet.java:72-74)
    lab = ds.labels(10)
    assert {str(k): int(v) for k, v in enumerate(lab)} == fx["labels"]


def test_oracle_merge(ds_setup):  # :59-78
    ds, fx = ds_setup
    ds2 = orc.OracleDisjointSet()
    for a, b in fx["ds2_edges"]:
        ds2.union(a, b)
    ds2.merge(ds)
    assert ds2.size() == fx["merged_size"] == 18
    roots = {ds2.find(k) for k in map(int, fx["merged_labels"])}
    assert len(roots) == fx["merged_roots"] == 2
    lab = ds2.labels(108)
    assert {k: int(lab[int(k)]) for k in fx["merged_labels"]} == fx["merged_labels"]


def test_oracle_union_by_rank_tie_rule():
    # DisjointSet.union :119-121: on equal ranks root2 hangs under root1 and rank1 grows
    ds = orc.OracleDisjointSet()
    ds.union(5, 3)
    assert ds.find(3) == 5 and ds.find(5) == 5
    ds.union(1, 3)  # rank(1)=0 < rank(5)=1 -> 1 hangs under 5
    assert ds.find(1) == 5


def test_oracle_self_loop_is_make_set():
    ds = orc.OracleDisjointSet()
    ds.union(7, 7)
    assert ds.size() == 1 and ds.find(7) == 7


# ---- ConnectedComponentsTest (example/test/ConnectedComponentsTest.java) ----
def test_oracle_connected_components_kat(golden):
    fx = golden("kat_connected_components.json")
    pairs = np.array(fx["edges"], dtype=np.uint32)
    out = orc.cc_stream(pairs, [0, len(pairs)], 10, want_labels=True)
    lab = out["labels"][-1]
    assert lab.tolist() == fx["labels"]
    assert int(out["components"][-1]) == fx["n_components"] == 3  # ConnectedComponentsTest :73


# ---- ConnectedComponentsExample default data: 11 event-time windows ----
def test_oracle_example_windows(golden):
    fx = golden("example_default.json")
    cfg = G.CONFIGS["c1_example"]
    pairs = G.generate_host(cfg)
    assert hashlib.sha256(pairs.astype("<u4").tobytes()).hexdigest() == fx["edges_sha256"]
    starts = G.window_starts(cfg)
    assert starts.tolist() == fx["window_starts"]
    assert G.timestamps(cfg).tolist() == fx["timestamps_ms"]
    for parts in (1, 2, 4):
        out = orc.cc_stream(pairs, starts, fx["V"], partitions=parts, want_labels=True)
        assert len(fx["windows"]) == 11
        for w, entry in enumerate(fx["windows"]):
            assert out["labels"][w].tolist() == entry["labels"], (parts, w)
            assert int(out["seen"][w]) == entry["seen"]


# ---- synthetic streams: generator bytes + per-window partitions ----
STREAMS = {
    "stream_rmat_s10.json": lambda g: G.scaled(G.CONFIGS["c2_rmat20"], scale=g["scale"], n_edges=g["n_edges"], seed=g["seed"]),
    "stream_gnm_4096.json": lambda g: G.scaled(G.CONFIGS["c3_gnm24"], n_vertices=g["n_vertices"], n_edges=g["n_edges"], seed=g["seed"]),
    "stream_adversarial_p10.json": lambda g: G.scaled(G.CONFIGS["c5_adversarial"], scale=g["scale"], n_stars=g["n_stars"],
                                                       star_size=g["star_size"], seed=g["seed"]),
}


@pytest.mark.parametrize("name", sorted(STREAMS))
def test_generator_matches_restatement(golden, name):
    fx = golden(name)
    cfg = STREAMS[name](fx["generator"])
    E, V = cfg.info()
    assert (E, V) == (fx["n_edges"], fx["V"])
    pairs = G.generate_host(cfg)
    assert hashlib.sha256(pairs.astype("<u4").tobytes()).hexdigest() == fx["edges_sha256"]
    # any slice generates the same bytes (counter-based: ranks generate their chunk independently)
    assert np.array_equal(G.generate_host(cfg, 100, 50), pairs[100:150])


@pytest.mark.parametrize("name", sorted(STREAMS))
@pytest.mark.parametrize("parts,threads", [(1, 1), (3, 3), (8, 4)])
def test_oracle_stream_windows(golden, name, parts, threads):
    fx = golden(name)
    cfg = STREAMS[name](fx["generator"])
    pairs = G.generate_host(cfg)
    out = orc.cc_stream(pairs, fx["window_starts"], fx["V"], partitions=parts, threads=threads, want_labels=True)
    for w, entry in enumerate(fx["windows"]):
        assert bool(out["emitted"][w]) == entry["emitted"]
        assert int(out["seen"][w]) == entry["seen"]
        assert int(out["components"][w]) == entry["components"]
        assert str(int(out["digest"][w])) == entry["digest"]
        assert str(orc.label_digest(out["labels"][w])) == entry["digest"]
        if "labels" in entry:
            assert out["labels"][w].tolist() == entry["labels"]


def test_oracle_empty_window_emits_nothing():
    pairs = np.array([[1, 2], [3, 4]], dtype=np.uint32)
    out = orc.cc_stream(pairs, [0, 1, 1, 2], 8, want_labels=True)
    assert out["emitted"].tolist() == [True, False, True]
    assert out["labels"][2].tolist()[:5] == [UNSEEN, 1, 1, 3, 3]


def test_oracle_rejects_ids_outside_range():
    with pytest.raises(ValueError):
        orc.cc_stream(np.array([[1, 9]], dtype=np.uint32), [0, 1], 8, want_labels=True)


def test_label_digest_numpy_matches_c():
    lab = np.array([UNSEEN, 1, 1, 3, UNSEEN, 0], dtype=np.uint32)
    assert orc.label_digest(lab) == int(orc.lib().orc_label_digest(lab.ctypes.data, lab.size))


def test_native_unseen_constant():
    assert native.UNSEEN == UNSEEN == orc.UNSEEN


def test_windowed_digest_fixtures_are_consistent(golden):
    """tests/golden/stream_digests.json's windowed entries (per-window parity at full size): the
    windows tile the stream, their seen counts never shrink (union only grows), and the last window's summary is the
    whole stream's (its own entry, computed in one window)."""
    fx = golden("stream_digests.json")
    windowed = [k for k in fx if "/w" in k]
    assert {"c4_kron26/w8", "c3_gnm24/w4M", "c3_gnm24/w1M", "c5_adversarial/w64K"} <= set(windowed)
    for k in windowed:
        e = fx[k]
        whole = fx[e["config"]]
        ends = [w["end"] for w in e["windows"]]
        assert ends == sorted(ends) and ends[-1] == e["edges"] == whole["edges"], k
        assert all(b - a <= e["window_edges"] for a, b in zip([0] + ends, ends)), k
        seen = [w["seen"] for w in e["windows"]]
        assert seen == sorted(seen), k
        last = e["windows"][-1]
        assert (last["digest"], last["seen"], last["components"]) == (whole["digest"], whole["seen"],
                                                                      whole["components"]), k
