"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle and the golden fixtures. Bit-exact labels.

Canonical form (the parity contract): after every merge window, label[v] = min id of v's
component over all edges folded so far, 0xFFFFFFFF for ids never seen. Run with: pytest -m gpu
"""
import hashlib
import os

import numpy as np
import pytest

import oracle as orc
from gelly_stream import (ConnectedComponents, DisjointSet, GellyCCError, SimpleEdgeStream, native)
from gelly_stream import generators as G

pytestmark = pytest.mark.gpu
UNSEEN = 0xFFFFFFFF
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    return torch


def device_stream(torch_cuda, cfg, first=0, count=None):
    """Generate edges straight into HBM (a torch tensor as plain device memory) and return it."""
    E, _ = cfg.info()
    count = E - first if count is None else count
    t = torch_cuda.empty(2 * max(count, 1), dtype=torch_cuda.int32, device="cuda:0")
    G.generate_device(cfg, first, count, t.data_ptr(), 0)
    torch_cuda.cuda.synchronize()
    return t


def first_mismatch(got, want):
    bad = np.flatnonzero(got != want)
    return None if bad.size == 0 else (int(bad[0]), int(got[bad[0]]), int(want[bad[0]]), int(bad.size))


def test_native_library_is_the_in_tree_build():
    native.lib()
    maps = open("/proc/self/maps").read()
    assert native.LIB_PATH in maps
    assert native.device_count() >= 1


# ---- DisjointSetTest replayed on the GPU summary (util/DisjointSetTest.java:36-78) ----
@pytest.fixture()
def gpu_ds(golden):
    fx = golden("kat_disjoint_set.json")
    ds = DisjointSet(128)
    for a, b in fx["setup_edges"]:
        ds.union(a, b)
    yield ds, fx
    ds.close()


def test_get_matches(gpu_ds):
    ds, fx = gpu_ds
    assert ds.getMatches().size() == fx["size"] == 10
    assert sorted(ds.getMatches().keySet()) == list(range(10))


def test_find(gpu_ds):
    ds, fx = gpu_ds
    root1, root2 = ds.find(0), ds.find(1)
    assert root1 != root2
    for i in range(10):
        assert ds.find(i) == (root1 if i % 2 == 0 else root2)
    assert ds.find(50) is None
    assert {str(k): int(v) for k, v in enumerate(ds.labels()[:10])} == fx["labels"]


def test_merge(gpu_ds):
    ds, fx = gpu_ds
    ds2 = DisjointSet(128)
    for a, b in fx["ds2_edges"]:
        ds2.union(a, b)
    ds2.merge(ds)
    assert ds2.getMatches().size() == 18
    roots = {ds2.find(k) for k in ds2.getMatches().keySet()}
    assert len(roots) == 2
    lab = ds2.labels()
    assert {k: int(lab[int(k)]) for k in fx["merged_labels"]} == fx["merged_labels"]
    assert ds.getMatches().size() == 10  # merge leaves `other` unchanged


def test_to_string(gpu_ds):
    ds, _ = gpu_ds
    assert str(ds) == "{0=[0, 2, 4, 6, 8], 1=[1, 3, 5, 7, 9]}"


# ---- ConnectedComponentsTest (example/test/ConnectedComponentsTest.java) ----
def test_connected_components_job(golden):
    fx = golden("kat_connected_components.json")
    cc = ConnectedComponents(mergeWindowTime=5, id_capacity=10)
    outs = [s.labels().copy() for s in SimpleEdgeStream(np.array(fx["edges"])).aggregate(cc)]
    assert outs[-1].tolist() == fx["labels"]
    comps = {}
    for v in np.flatnonzero(outs[-1] != UNSEEN):
        comps.setdefault(int(outs[-1][v]), []).append(int(v))
    assert sorted(comps.values()) == fx["components"]
    assert len(comps) == 3  # :73


# ---- ConnectedComponentsExample default data: 11 event-time windows ----
def test_example_default_windows(golden):
    fx = golden("example_default.json")
    cfg = G.CONFIGS["c1_example"]
    stream = SimpleEdgeStream(G.generate_host(cfg), timestamps=G.timestamps(cfg))
    cc = ConnectedComponents(mergeWindowTime=cfg.merge_window_ms, id_capacity=fx["V"])
    got = [s.labels().copy() for s in stream.aggregate(cc)]
    assert len(got) == 11
    for w, entry in enumerate(fx["windows"]):
        assert got[w].tolist() == entry["labels"], w


# ---- small synthetic streams vs fixtures: host-fed and device-resident paths ----
STREAMS = {
    "stream_rmat_s10.json": lambda g: G.scaled(G.CONFIGS["c2_rmat20"], scale=g["scale"], n_edges=g["n_edges"], seed=g["seed"]),
    "stream_gnm_4096.json": lambda g: G.scaled(G.CONFIGS["c3_gnm24"], n_vertices=g["n_vertices"], n_edges=g["n_edges"], seed=g["seed"]),
    "stream_adversarial_p10.json": lambda g: G.scaled(G.CONFIGS["c5_adversarial"], scale=g["scale"], n_stars=g["n_stars"],
                                                       star_size=g["star_size"], seed=g["seed"]),
}


def check_windows(summaries_iter, fx):
    n = 0
    for w, s in enumerate(summaries_iter):
        lab = s.labels()
        entry = fx["windows"][w]
        assert str(orc.label_digest(lab)) == entry["digest"], (fx["name"], w)
        assert s.getMatches().size() == entry["seen"]
        assert s.num_components() == entry["components"]
        if "labels" in entry:
            assert lab.tolist() == entry["labels"]
        n += 1
    assert n == len(fx["windows"])


@pytest.mark.parametrize("name", sorted(STREAMS))
def test_stream_fixture_host_fed(golden, name):
    fx = golden(name)
    cfg = STREAMS[name](fx["generator"])
    pairs = G.generate_host(cfg)
    starts = np.asarray(fx["window_starts"])
    stream = SimpleEdgeStream(pairs, edges_per_window=int(starts[1] - starts[0]))
    check_windows(stream.aggregate(ConnectedComponents(1000, id_capacity=fx["V"])), fx)


@pytest.mark.parametrize("name", sorted(STREAMS))
def test_stream_fixture_device_resident(golden, torch_cuda, name):
    fx = golden(name)
    cfg = STREAMS[name](fx["generator"])
    d = device_stream(torch_cuda, cfg)
    host = d.cpu().numpy().view(np.uint32).reshape(-1, 2)
    assert hashlib.sha256(host.astype("<u4").tobytes()).hexdigest() == fx["edges_sha256"]  # device generator
    stream = SimpleEdgeStream(device_ptr=d.data_ptr(), n_device_edges=fx["n_edges"],
                              device_window_starts=np.asarray(fx["window_starts"]))
    check_windows(stream.aggregate(ConnectedComponents(1000, id_capacity=fx["V"])), fx)


# ---- full-size configs vs the oracle, per window ----
def run_device_windows(torch_cuda, cfg, starts, V, knobs=None, raw=None):
    d = device_stream(torch_cuda, cfg)
    ds = DisjointSet(V)
    if knobs:
        ds.tune(**knobs)
    out = []
    for w in range(len(starts) - 1):
        b, e = int(starts[w]), int(starts[w + 1])
        ds.fold_device(d.data_ptr() + 8 * b, e - b)
        if raw is not None:  # diagnostics: the forest before the window's emission (no compress)
            raw.append(ds.raw_parent())
        out.append(ds.labels().copy())
    ds.close()
    return out


def _host_root(par, v):
    while par[v] < v:
        v = int(par[v])
    return v


@pytest.mark.parametrize("cfg_name,window", [("c2_rmat20", 1 << 20), ("c2_rmat20", 1 << 24), ("c3_gnm24", 1 << 22)])
def test_full_config_parity(torch_cuda, cfg_name, window):
    cfg = G.CONFIGS[cfg_name]
    E, V = cfg.info()
    starts = np.asarray(list(range(0, E, window)) + [E], dtype=np.uint64)
    pairs = G.generate_host(cfg)
    want = orc.cc_stream(pairs, starts, V, partitions=4, threads=4)
    raw = []
    got = run_device_windows(torch_cuda, cfg, starts, V, raw=raw)
    for w, lab in enumerate(got):
        if orc.label_digest(lab) != int(want["digest"][w]):  # diagnostics: the same windows with every
            # incremental compress off (full compresses only), to tell which stage a mismatch comes from
            ref = run_device_windows(torch_cuda, cfg, starts, V, knobs={"incremental": 0})
            bad = np.flatnonzero(lab != ref[w])
            walk = [(int(v), _host_root(raw[w], int(v)), int(raw[w][v])) for v in bad[:4]]
            prev = [(int(v), int(got[w - 1][v]) if w else -1) for v in bad[:4]]
            pytest.fail(f"{cfg_name} window {w}: digest mismatch; raw-forest walks (v, root, parent) {walk}; "
                        f"previous labels {prev}; vs the full-compress forest {bad.size} labels differ"
                        f"{'' if bad.size == 0 else f' (first at {int(bad[0])}: {int(lab[bad[0]])} vs {int(ref[w][bad[0]])})'}"
                        f", full-compress forest digest {'matches' if orc.label_digest(ref[w]) == int(want['digest'][w]) else 'differs'}")
        seen = lab != UNSEEN
        assert int(seen.sum()) == int(want["seen"][w])
        assert int(np.count_nonzero(lab[seen] == np.flatnonzero(seen))) == int(want["components"][w])


def test_adversarial_prefix_windows(torch_cuda):
    """C5's short windows (2^16 edges) over the first 2^20 edges, every window vs the oracle."""
    cfg = G.CONFIGS["c5_adversarial"]
    _, V = cfg.info()
    n = 1 << 20
    starts = np.arange(0, n + 1, cfg.window_edges, dtype=np.uint64)
    pairs = G.generate_host(cfg, 0, n)
    want = orc.cc_stream(pairs, starts, V, partitions=2, threads=2)
    got = run_device_windows(torch_cuda, cfg, starts, V)
    for w, lab in enumerate(got):
        assert orc.label_digest(lab) == int(want["digest"][w]), w


def test_adversarial_full_stream_closed_form(torch_cuda):
    """Full C5 (16.7M edges, 256 windows): the final partition is known in closed form — the whole path is one
    component labelled 0, each star is one component labelled by its hub (its smallest id)."""
    cfg = G.CONFIGS["c5_adversarial"]
    E, V = cfg.info()
    d = device_stream(torch_cuda, cfg)
    ds = DisjointSet(V)
    for b in range(0, E, cfg.window_edges):
        ds.fold_device(d.data_ptr() + 8 * b, min(cfg.window_edges, E - b))
        ds.compress()
    lab = ds.labels()
    P = 1 << cfg.scale
    assert np.all(lab[:P] == 0)
    ids = np.arange(P, V, dtype=np.int64)
    assert np.array_equal(lab[P:], (P + (ids - P) // cfg.star_size * cfg.star_size).astype(np.uint32))
    assert ds.num_components() == 1 + cfg.n_stars


def test_incremental_compress_windows(torch_cuda):
    """Short windows over a big forest: the plain folds record their mutations in a bloom filter and every window's
    compress is incremental (compress_inc_kernel). G(n, m) at the percolation threshold (n = 2^22, m = 2^21, deep
    chains), 32 windows of 2^16 edges: every window equals the oracle, a forest with the incremental compress
    off and one whose incremental compress writes a spare buffer instead of parent[] in place (inc_inplace=0).
    A CombineCC merge, the raw-pointer view and a reset in between force full compresses."""
    cfg = G.scaled(G.CONFIGS["c3_gnm24"], n_vertices=1 << 22, n_edges=1 << 21, seed=0x1234)
    E, V = cfg.info()
    W = 1 << 16
    starts = np.arange(0, E + 1, W, dtype=np.uint64)
    want = orc.cc_stream(G.generate_host(cfg), starts, V, partitions=2, threads=2)
    d = device_stream(torch_cuda, cfg)
    inc, full, spare = DisjointSet(V), DisjointSet(V), DisjointSet(V)
    inc.tune(incremental=1, emit_div=0)  # the eager emission's incremental compress (round 6's default emission is lazy)
    full.tune(incremental=0)
    spare.tune(incremental=1, inc_inplace=0, emit_div=0)
    side = DisjointSet(V)  # a partial forest merged into `inc` mid-stream (CombineCC)
    side.fold_device(d.data_ptr(), W)
    for w in range(len(starts) - 1):
        b, e = int(starts[w]), int(starts[w + 1])
        for ds in (inc, full, spare):
            ds.fold_device(d.data_ptr() + 8 * b, e - b)
        if w == 9:
            inc.merge(side)  # edges of window 0 again: the partition is unchanged, the next compress is full
        if w == 17:
            inc.device_ptr()
        got = inc.labels()
        assert np.array_equal(got, full.labels()), (w, first_mismatch(got, full.labels()))
        assert np.array_equal(spare.labels(), full.labels()), ("inc_inplace=0", w)
        assert orc.label_digest(got) == int(want["digest"][w]), w
    # reset, then the same windows again from scratch
    inc.reset()
    for w in range(4):
        inc.fold_device(d.data_ptr() + 8 * int(starts[w]), W)
        assert orc.label_digest(inc.labels()) == int(want["digest"][w]), ("after reset", w)
    for ds in (inc, full, spare, side):
        ds.close()


# ---- size-independent properties at full size ----
def test_order_invariance_and_idempotence(torch_cuda):
    cfg = G.CONFIGS["c2_rmat20"]
    E, V = cfg.info()
    d = device_stream(torch_cuda, cfg)
    a = DisjointSet(V)
    a.fold_device(d.data_ptr(), E)
    la = a.labels().copy()
    # fold the same stream again: unchanged (idempotence)
    a.fold_device(d.data_ptr(), E)
    assert np.array_equal(a.labels(), la)
    # a permuted stream gives the same partition (order invariance)
    perm = torch_cuda.randperm(E, device="cuda:0", generator=torch_cuda.Generator(device="cuda:0").manual_seed(7))
    shuffled = d.view(-1, 2)[perm].contiguous()
    b = DisjointSet(V)
    b.fold_device(shuffled.data_ptr(), E)
    assert np.array_equal(b.labels(), la)
    # split into two partitions folded separately, then CombineCC-merged: same partition
    c1, c2 = DisjointSet(V), DisjointSet(V)
    c1.fold_device(d.data_ptr(), E // 3)
    c2.fold_device(d.data_ptr() + 8 * (E // 3), E - E // 3)
    c2.merge(c1)
    assert np.array_equal(c2.labels(), la)
    # merging into an empty forest copies the partition; reset empties it
    e = DisjointSet(V)
    e.merge(a)
    assert np.array_equal(e.labels(), la)
    e.reset()
    assert e.size() == 0 and np.all(e.labels() == UNSEEN)
    for x in (a, b, c1, c2, e):
        x.close()


def test_seeded_fold_across_flag_epochs(torch_cuda):
    """The seeding marks C with flag bytes holding an epoch 1..255 (cleared once per 255 seedings) and keeps
    per-block minima: 300 reset + fold cycles of one R-MAT batch (crossing the wrap) must all give the oracle's
    labels, with the fused and the separate hub election and several BFS prefixes."""
    cfg = G.scaled(G.CONFIGS["c2_rmat20"], scale=17, n_edges=1 << 20)
    E, V = cfg.info()
    want = orc.cc_stream(G.generate_host(cfg), [0, E], V, partitions=2, threads=2)
    d = device_stream(torch_cuda, cfg)
    ds = DisjointSet(V)
    knobs = [{}, {"seed_fuse": 0}, {"seed_div": 2, "seed_div1": 4}, {"seed_passes": 1}, {"seed_passes": 3}]
    for i in range(300):
        ds.tune(**{"seed_fuse": 1, "seed_div": 3, "seed_div1": 3, "seed_passes": 2, **knobs[i % len(knobs)]})
        ds.reset()
        ds.fold_device(d.data_ptr(), E)
        if i % 7 == 0 or i >= 250:
            assert orc.label_digest(ds.labels()) == int(want["digest"][0]), i
    ds.close()


def test_edge_cases():
    ds = DisjointSet(1 << 10)
    ds.fold(np.zeros((0, 2), dtype=np.uint32))  # empty batch
    assert ds.size() == 0 and ds.num_components() == 0
    ds.union(5, 5)  # self loop = makeSet
    assert ds.find(5) == 5 and ds.size() == 1
    ds.fold(np.array([[1023, 1022], [1023, 1022], [1022, 1023]], dtype=np.uint32))  # max id, duplicates
    assert ds.find(1023) == 1022 and ds.size() == 3
    ds.makeSet(7)
    assert ds.find(7) == 7
    with pytest.raises(GellyCCError):
        ds.fold(np.array([[1, 1024]], dtype=np.uint32))  # out of range: rejected on the host, no device access
    with pytest.raises(ValueError):
        ds.union(0, 4096)
    one = DisjointSet(1)
    one.union(0, 0)
    assert one.labels().tolist() == [0]


def test_single_edge_staging_path_crosses_batches():
    """Per-edge foldEdges calls (the Java drop-in pattern) staged in pinned memory across several batches."""
    V = 1 << 12
    rng = np.random.default_rng(3)
    pairs = rng.integers(0, V, size=((1 << 20) + 17, 2), dtype=np.uint32)  # > one staging slot
    ds = DisjointSet(V)
    for u, v in pairs[:5000]:
        ds.union(int(u), int(v))
    ds.fold(pairs[5000:])
    want = orc.cc_stream(pairs, [0, len(pairs)], V, want_labels=True)["labels"][0]
    assert first_mismatch(ds.labels(), want) is None


def test_snapshot_restore_round_trip():
    cfg = G.scaled(G.CONFIGS["c2_rmat20"], scale=14, n_edges=1 << 17)
    E, V = cfg.info()
    ds = DisjointSet(V)
    ds.fold(G.generate_host(cfg))
    snap = ds.snapshot_pairs()  # Merger.snapshotState
    re = DisjointSet(V)
    re.import_pairs(snap)       # Merger.restoreState
    assert np.array_equal(re.labels(), ds.labels())


def test_hub_contention_star():
    """Every edge hits one hub (worst-case CAS contention on one parent slot)."""
    V = 1 << 20
    leaves = np.arange(1, V, dtype=np.uint32)
    pairs = np.stack([np.zeros_like(leaves), leaves], axis=1)
    pairs[::2] = pairs[::2, ::-1]
    ds = DisjointSet(V)
    ds.fold(pairs)
    assert np.all(ds.labels() == 0)


def test_descending_path_worst_case_chain():
    """A path fed from the high end hooks one root under the next smaller one: longest possible chains."""
    V = 1 << 20
    hi = np.arange(V - 1, 0, -1, dtype=np.uint32)
    ds = DisjointSet(V)
    ds.fold(np.stack([hi, hi - 1], axis=1))
    assert np.all(ds.labels() == 0)


def test_fold_timing_events():
    cfg = G.scaled(G.CONFIGS["c2_rmat20"], scale=16, n_edges=1 << 20)
    E, V = cfg.info()
    ds = DisjointSet(V)
    ds.enable_timing(1)
    ds.fold(G.generate_host(cfg))
    assert ds.last_fold_ms() > 0.0
    log = ds.fold_profile()  # per-kernel dispatch timings + one span per fold
    names = [k for k, _, _ in log]
    assert names[0] == "begin" and "fold_span" in names and "filtered" in names
    span = [ms for k, ms, _ in log if k == "fold_span"][0]
    kernels = sum(ms for k, ms, _ in log if k not in ("begin", "fold_span", "slow_edges", "compress"))
    assert 0 < kernels <= span * 1.001
    assert [n for k, _, n in log if k == "fold_span"][0] == E


# ---- cross-GPU merge message (include/gelly_cc.h): encode / absorb, the RCCL payload's two ends ----
def encode(torch_cuda, ds, cap):
    msg = torch_cuda.zeros(native.msg_bytes(ds.id_capacity, cap) + 16, dtype=torch_cuda.uint8, device="cuda:0")
    torch_cuda.cuda.synchronize()  # the zero fill runs on torch's stream, the encode on the forest's own
    ds.encode_message(msg.data_ptr(), cap)
    torch_cuda.cuda.synchronize()
    hdr = msg[:16].cpu().numpy().view("<u4")
    return msg, hdr


def test_merge_message_ranks_on_one_gpu(torch_cuda):
    """P forests on one GPU play the ranks of ForestGroup's compact all_gather: per window each folds its chunk,
    encodes, absorbs the P-1 other messages, and must hold the global partition (oracle) — every window."""
    cfg = G.scaled(G.CONFIGS["c2_rmat20"], scale=16, n_edges=1 << 20)
    E, V = cfg.info()
    starts = np.asarray([0, 1000, 1 << 17, 1 << 19, E], dtype=np.uint64)
    want = orc.cc_stream(G.generate_host(cfg), starts, V, partitions=4, threads=4, want_labels=True)["labels"]
    d = device_stream(torch_cuda, cfg)
    P, cap = 4, V
    ranks = [DisjointSet(V) for _ in range(P)]
    for w in range(len(starts) - 1):
        b, e = int(starts[w]), int(starts[w + 1])
        msgs = []
        for r, ds in enumerate(ranks):
            lo, hi = b + (e - b) * r // P, b + (e - b) * (r + 1) // P
            ds.fold_device(d.data_ptr() + 8 * lo, hi - lo)
            msg, hdr = encode(torch_cuda, ds, cap)
            lab = ds.labels()
            seen = lab != UNSEEN
            assert hdr[2] == V
            assert hdr[1] == int(np.count_nonzero(seen & (lab != hdr[0]))), (w, r)
            msgs.append(msg)
        stride = msgs[0].numel()
        packed = torch_cuda.cat(msgs)  # the all_gather receive buffer: rank p's message at p * stride
        for r, ds in enumerate(ranks):
            if r % 2:  # one fused launch over all peers (the ForestGroup path)
                ds.absorb_messages(packed.data_ptr(), stride, P, r, cap)
            else:
                for p, msg in enumerate(msgs):
                    if p != r:
                        ds.absorb_message(msg.data_ptr(), cap)
        for r, ds in enumerate(ranks):
            assert first_mismatch(ds.labels(), want[w]) is None, (w, r, first_mismatch(ds.labels(), want[w]))
    for ds in ranks:
        ds.close()


def test_merge_message_full_c2_round_trip(torch_cuda):
    """Full C2 forest -> message -> empty forest: the same partition; the message is ~1/32 of the labels."""
    cfg = G.CONFIGS["c2_rmat20"]
    E, V = cfg.info()
    d = device_stream(torch_cuda, cfg)
    a = DisjointSet(V)
    a.fold_device(d.data_ptr(), E)
    la = a.labels().copy()
    msg, hdr = encode(torch_cuda, a, cap=1)  # list too small: the header still reports the true count
    n_oth = int(hdr[1])
    assert n_oth == int(np.count_nonzero((la != UNSEEN) & (la != hdr[0])))
    assert native.msg_bytes(V, n_oth) < 4 * V // 8
    msg, hdr = encode(torch_cuda, a, cap=n_oth)
    b = DisjointSet(V)
    b.absorb_message(msg.data_ptr(), n_oth)
    assert np.array_equal(b.labels(), la)
    # absorbing into a forest that already holds part of the partition: still the union
    c = DisjointSet(V)
    c.fold_device(d.data_ptr(), E // 5)
    c.absorb_message(msg.data_ptr(), n_oth)
    assert np.array_equal(c.labels(), la)
    for x in (a, b, c):
        x.close()


# ---- DisjointSet<Long>: ids anywhere in the Long range (dense relabel at the boundary) ----
def test_long_ids_connected_components_kat(golden):
    """ConnectedComponentsTest's edges with every id mapped to a wide Long (negative and > 2^32): the same three
    components, each labelled by its minimum wide id."""
    from gelly_stream import LongDisjointSet

    fx = golden("kat_connected_components.json")
    wide = {v: (v - 5) * (1 << 40) + 3 for e in fx["edges"] for v in e}  # order-preserving, spans the sign
    ds = LongDisjointSet(64)
    ds.fold([[wide[a], wide[b]] for a, b in fx["edges"]])
    comps = {}
    for v, r in zip(*ds.seen_labels()):
        comps.setdefault(int(r), []).append(int(v))
    want = sorted(sorted(wide[v] for v in c) for c in fx["components"])
    assert sorted(sorted(m) for m in comps.values()) == want
    for c in fx["components"]:
        assert ds.find(wide[c[-1]]) == min(wide[v] for v in c)
    assert ds.find(12345) is None and ds.size() == len(wide) and ds.num_components() == 3
    ds.close()


def test_long_ids_random_stream_and_merge():
    """A random stream over random 64-bit ids, folded in two halves into two summaries and merged (CombineCC),
    against a union-find over the original ids."""
    from gelly_stream import LongDisjointSet
    from test_idmap import python_components

    rng = np.random.default_rng(11)
    universe = rng.integers(-(1 << 63), (1 << 63) - 1, size=50_000, dtype=np.int64)
    pairs = universe[rng.integers(0, universe.size, size=(40_000, 2))]
    want = python_components(pairs.tolist())
    a, b = LongDisjointSet(1 << 17), LongDisjointSet(1 << 17)
    a.fold(pairs[:20_000])
    b.fold(pairs[20_000:])
    a.merge(b)
    ids, lab = a.seen_labels()
    assert dict(zip(ids.tolist(), lab.tolist())) == want
    a.close()
    b.close()


# ---- every tuning knob leaves the result unchanged ----
# One non-default setting per key that include/gelly_cc.h lists (gcc_forest_tune), chosen so that the path it
# selects actually runs at this size (e.g. inc_min_ids low enough for the incremental compress to engage).
KNOB_CASES = {
    "filter": {"filter": 0}, "filter_min_batch": {"filter_min_batch": 1024},
    "filter_min_share": {"filter_min_share": 0}, "sample_first": {"sample_first": 1024},
    "sample_growth": {"sample_growth": 2}, "sample_div": {"sample_div": 8}, "sample_min": {"sample_min": 4096},
    "refresh_min_batch": {"refresh_min_batch": 1024}, "refresh1": {"refresh_min_batch": 1024, "refresh1": 0.1},
    "refresh2": {"refresh_min_batch": 1024, "refresh2": 0.2}, "refresh3": {"refresh_min_batch": 1024, "refresh3": 0.6},
    "depth": {"depth": 8}, "hook": {"hook": 0}, "share_async": {"share_async": 0}, "drain_at": {"drain_at": 1}, "seed": {"seed": 0},
    "seed_nt": {"seed_nt": 0}, "seed_global": {"seed_global": 1}, "seed_fuse": {"seed_fuse": 0},
    "seed_passes": {"seed_passes": 3}, "seed_div": {"seed_div": 2}, "seed_div1": {"seed_div1": 5},
    "seed_refresh": {"seed_refresh": 0.5}, "incremental": {"inc_min_ids": 1024, "incremental": 1},
    "inc_min_ids": {"inc_min_ids": 1024, "incremental": 1}, "inc_div": {"incremental": 1, "inc_min_ids": 1024, "inc_div": 1},
    "inc_inplace": {"incremental": 1, "inc_min_ids": 1024, "inc_inplace": 0},
    "refresh_labels": {"refresh_min_batch": 1024, "refresh_labels": 1},
    # the bucketed fold (bucket_fold.h) at this size only when forced by bucket_min_ids / bucket_min_batch
    "bucket": {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket": 0},
    "bucket_min_batch": {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16},
    "bucket_min_ids": {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16},
    "bucket_levels": {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_levels": 1},
    "bucket_sample": {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_sample": 1.0},
    "bucket_sample_sparse": {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_sample_sparse": 0.05},
    "pin_chunk": {"pin_chunk": 4096},
    "scratch_realloc": {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "scratch_realloc": 1},
    "bucket_p1": [{"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_p1": 0},
                  {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_p1": 3}],
    "bucket_slow2": {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_slow2": 0},
    "bucket_defer": {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_defer": 0},
    "bucket_defer_c": [{"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_defer_c": 1},
                       {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_defer_c": 2}],
    "compress_split": {"compress_split": 1},  # round 4's full compress (splitting finds): the same labels
    "fold_split": {"fold_split": 0, "filter": 0},  # the plain fold with read-only finds
    "inc_pipe": [{"incremental": 1, "inc_min_ids": 1024, "inc_pipe": 1},  # the pipelined emission (off by default)
                 {"incremental": 1, "inc_min_ids": 1024, "inc_pipe": 2}],
    "bucket_hub_sample": {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_hub_sample": 0.1},
    "lds_edges_per_word": {"lds_edges_per_word": 1e9},  # the short windows take the global-bitmap filter
    "bucket_p2_per": {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_p2_per": 8},
    "bucket_p2_vw": {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_p2_vw": 8},
    "bucket_chunk": [{"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_chunk": 64},
                     {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_chunk": 4096}],
    "bucket_items": {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_items": 1},
    "bucket_items_p3": [{"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_items_p3": 1},
                        {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16, "bucket_items_p3": 8}],
    # the later windows of this stream are short (4096 edges): bucket_min_batch 4096 lets them take the bucketed fold
    "bucket_windows": [{"bucket_min_ids": 0, "bucket_min_batch": 1 << 12, "bucket_windows": 0},
                       {"bucket_min_ids": 0, "bucket_min_batch": 1 << 12, "bucket_windows": 1}],
    "inc_check": {"incremental": 1, "inc_min_ids": 1024, "inc_div": 1, "inc_check": 1},  # diagnostics: checks every incremental compress
    "post_check": {"incremental": 1, "inc_min_ids": 1024, "post_check": 2},  # diagnostics after every incremental compress
    "fold_release": {"incremental": 1, "inc_min_ids": 1024, "fold_release": 1},
    # inc_split = 1 is refused without `experimental` (test_unsafe_setting_needs_experimental); its default here
    "inc_split": {"incremental": 1, "inc_min_ids": 1024, "inc_split": 0},
    "experimental": {"experimental": 1},
    # the lazy emission (round 6): eager, and a compress only per id_capacity folded edges in the plain regime
    "emit_div": [{"emit_div": 0}, {"emit_div": 1, "filter": 0}],
    "emit_rec": {"emit_rec": 1, "incremental": 1, "inc_min_ids": 1024, "filter": 0},
    "emit_filtered": {"emit_filtered": 1},
}


def test_unsafe_setting_needs_experimental():
    """The one setting known to give wrong results (inc_split = 1: round 3's stale label) is refused unless
    the caller sets `experimental` first: a Java or C caller cannot turn it on by accident."""
    with DisjointSet(1 << 16) as ds:
        with pytest.raises(GellyCCError, match="experimental"):
            ds.tune(inc_split=1)
        ds.tune(experimental=1)
        ds.tune(inc_split=1)  # accepted now (reproductions only)
        ds.tune(inc_split=0)


def header_tuning_keys():
    text = open(os.path.join(ROOT, "include", "gelly_cc.h")).read()
    block = text[text.index("tuning knobs"):text.index("int gcc_forest_tune")]
    block = block[block.index("Keys:") + 5:block.index("Unknown keys")]
    keys = []
    for part in block.replace("*", " ").replace("\n", " ").split(","):
        part = part.strip().rstrip(".")
        if part.startswith("refresh1..refresh"):
            keys += ["refresh1", "refresh2", "refresh3"]
        elif part:
            keys.append(part)
    return keys


def test_every_tuning_knob_is_bit_exact(torch_cuda):
    """Results never depend on the tuning (gelly_cc.h). Each key the header lists, set away from its default,
    folds an R-MAT stream (one long window, then short windows over the same forest) bit-exactly; an unknown
    key is rejected with GCC_E_INVALID."""
    keys = header_tuning_keys()
    assert sorted(keys) == sorted(KNOB_CASES), "a tuning key without a parity case (or a stale one)"
    cfg = G.scaled(G.CONFIGS["c2_rmat20"], scale=16, n_edges=1 << 20, seed=0x6B6E6F62)
    E, V = cfg.info()
    h = 1 << 19
    starts = np.array([0, h, h + 4096, h + 8192, h + 12288, E], dtype=np.uint64)
    want = orc.cc_stream(G.generate_host(cfg), starts, V, partitions=2, threads=2)["digest"]
    d = device_stream(torch_cuda, cfg)
    with DisjointSet(V) as ds:
        with pytest.raises(GellyCCError):
            ds.tune(no_such_knob=1)
    cases = [(k, c) for k, v in KNOB_CASES.items() for c in (v if isinstance(v, list) else [v])]
    for key, knobs in cases:
        print("knob case", key, knobs, flush=True)  # names the case in the report if a launch faults asynchronously
        with DisjointSet(V) as ds:
            ds.tune(**knobs)
            for w in range(len(starts) - 1):
                b, e = int(starts[w]), int(starts[w + 1])
                ds.fold_device(d.data_ptr() + 8 * b, e - b)
                ds.compress()  # the window's emission (lazy or not: the labels read below compress if it was)
                assert orc.label_digest(ds.labels()) == int(want[w]), (key, w)
