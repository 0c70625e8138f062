"""GPU parity of the bucketed fold (csrc/bucket_fold.h), the device-side id validation, the pinned host path and
the full-size north-star config C4 (Kronecker s26, 2^30 edges) against the oracle's digests.

Every test goes through the C ABI (ctypes). Bit-exact labels: label[v] = min id of v's component, UNSEEN if unseen.
"""
import json
import os

import numpy as np
import pytest

import oracle as orc
from gelly_stream import DisjointSet, GellyCCError, LongDisjointSet
from gelly_stream import generators as G

pytestmark = pytest.mark.gpu
UNSEEN = 0xFFFFFFFF
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIGESTS = json.load(open(os.path.join(ROOT, "tests", "golden", "stream_digests.json")))
FORCE = {"bucket_min_ids": 0, "bucket_min_batch": 1 << 16}  # take the bucketed path at test sizes


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    return torch


def to_device(torch_cuda, pairs):
    t = torch_cuda.from_numpy(np.ascontiguousarray(pairs, dtype=np.uint32).view(np.int32).reshape(-1)).to("cuda:0")
    torch_cuda.cuda.synchronize()
    return t


def gen_device(torch_cuda, cfg, first=0, count=None):
    E, _ = cfg.info()
    count = E - first if count is None else count
    t = torch_cuda.empty(2 * max(count, 1), dtype=torch_cuda.int32, device="cuda:0")
    G.generate_device(cfg, first, count, t.data_ptr(), 0)
    torch_cuda.cuda.synchronize()
    return t


def oracle_labels(pairs, V):
    return orc.cc_stream(pairs, [0, len(pairs)], V, partitions=4, threads=4, want_labels=True)["labels"][0]


def mismatch(got, want):
    bad = np.flatnonzero(got != want)
    return None if bad.size == 0 else (int(bad[0]), int(got[bad[0]]), int(want[bad[0]]), int(bad.size))


@pytest.mark.parametrize("knobs", [{}, {"bucket_levels": 0}, {"bucket_levels": 1, "bucket_sample": 1.0},
                                   {"bucket_sample": 0.0}, {"bucket_levels": 6, "bucket_sample": 0.05},
                                   {"bucket_slow2": 0}, {"bucket_levels": 0, "bucket_slow2": 0},
                                   {"bucket_hub_sample": 0.0}, {"bucket_levels": 3, "bucket_hub_sample": 0.15},
                                   {"bucket_defer": 0}, {"bucket_defer": 0, "bucket_slow2": 0},
                                   {"bucket_defer_c": 1}, {"bucket_defer_c": 2}, {"bucket_defer_c": 2, "bucket_slow2": 0}])
def test_bucketed_fold_rmat(torch_cuda, knobs):
    """R-MAT s20, 2^22 edges, one fresh batch through the bucketed fold (seeding knobs vary the sample and the
    level count: the result may not depend on them)."""
    cfg = G.scaled(G.CONFIGS["c2_rmat20"], n_edges=1 << 22, seed=0xB0C4)
    E, V = cfg.info()
    pairs = G.generate_host(cfg)
    want = oracle_labels(pairs, V)
    d = to_device(torch_cuda, pairs)
    with DisjointSet(V) as ds:
        ds.tune(**FORCE, **knobs)
        ds.enable_timing(1)
        ds.fold_device(d.data_ptr(), E)
        got = ds.labels()
        names = [k for k, _, _ in ds.fold_profile()]
        assert "bucket" in names and "slice_filter" in names, names  # the bucketed path ran
        assert mismatch(got, want) is None, mismatch(got, want)
        # later batches of the same forest take the filtered path against the bucketed fold's bitmap
        ds.fold_device(d.data_ptr(), E // 3)
        assert mismatch(ds.labels(), want) is None


@pytest.mark.parametrize("knobs", [{}, {"bucket_sample_sparse": 0.0}, {"bucket_sample_sparse": 1.0},
                                   {"bucket_defer_c": 2}])
def test_bucketed_fold_sparse_batch(torch_cuda, knobs):
    """A sparse batch (2 edges per id, like C4's 1/8 share): its seeding samples bucket_sample_sparse of every bucket
    (round 5); many edges reach the second level. The result may not depend on the sample."""
    cfg = G.scaled(G.CONFIGS["c2_rmat20"], n_edges=1 << 21, seed=0x5A5A)
    E, V = cfg.info()
    pairs = G.generate_host(cfg)
    want = oracle_labels(pairs, V)
    d = to_device(torch_cuda, pairs)
    with DisjointSet(V) as ds:
        ds.tune(**FORCE, **knobs)
        ds.fold_device(d.data_ptr(), E)
        assert mismatch(ds.labels(), want) is None, mismatch(ds.labels(), want)


def test_bucketed_fold_gnm_no_giant(torch_cuda):
    """G(n, m) below the threshold: no giant, the seeding's C stays small, almost every edge takes the union path."""
    cfg = G.scaled(G.CONFIGS["c3_gnm24"], n_vertices=1 << 21, n_edges=1 << 20, seed=0x77)
    E, V = cfg.info()
    pairs = G.generate_host(cfg)
    d = to_device(torch_cuda, pairs)
    with DisjointSet(V) as ds:
        ds.tune(**FORCE)
        ds.fold_device(d.data_ptr(), E)
        assert mismatch(ds.labels(), oracle_labels(pairs, V)) is None


def test_bucketed_fold_odd_length_and_self_loops(torch_cuda):
    rng = np.random.default_rng(5)
    V = 3 << 19  # 1.5 slices: a partial last slice
    pairs = rng.integers(0, V, size=((1 << 18) + 1, 2), dtype=np.uint32)  # odd: the last edge takes the overflow list
    pairs[::97, 1] = pairs[::97, 0]  # self loops
    pairs[-1] = [V - 1, V - 2]
    d = to_device(torch_cuda, pairs)
    with DisjointSet(V) as ds:
        ds.tune(**FORCE)
        ds.fold_device(d.data_ptr(), len(pairs))
        assert mismatch(ds.labels(), oracle_labels(pairs, V)) is None


@pytest.mark.parametrize("hot_share", [16, 1])
def test_bucketed_fold_overflow_and_spill(torch_cuda, hot_share):
    """The bucket capacities come from a strided sample of the batch. A batch built against that sample: every
    16th edge (the sampled positions) has its source in slice 0, the others in slice 1, so bucket 1 is
    under-estimated. hot_share=16: the rest overflows into the overflow list; hot_share=1: the overflow list
    overflows too (spill) and the whole batch is folded again. Both exact."""
    V = 1 << 20
    n = 1 << 20
    rng = np.random.default_rng(9 + hot_share)
    if hot_share == 1:  # 15/16 of the batch in slice 1, estimated empty: the overflow list overflows (spill)
        src = rng.integers(1 << 19, V, size=n, dtype=np.uint32)
        src[::16] = rng.integers(0, 1 << 19, size=n // 16, dtype=np.uint32)  # the sampled positions: slice 0
    else:  # 1/8 of the batch in slice 1 (never sampled): it overflows into the list, which holds it
        src = rng.integers(0, 1 << 19, size=n, dtype=np.uint32)
        src[5::8] = rng.integers(1 << 19, V, size=n // 8, dtype=np.uint32)
    dst = rng.integers(0, V, size=n, dtype=np.uint32)
    pairs = np.stack([src, dst], axis=1)
    d = to_device(torch_cuda, pairs)
    with DisjointSet(V) as ds:
        ds.tune(**FORCE)
        ds.fold_device(d.data_ptr(), n)
        assert mismatch(ds.labels(), oracle_labels(pairs, V)) is None


@pytest.mark.parametrize("V", [(1 << 27) + (1 << 20), 1 << 28])
def test_bucketed_fold_beyond_2_27_ids(torch_cuda, V):
    """Id ranges past 2^27 (they took the unbucketed fold): 258 / 512 buckets of 2^19 ids, P1's
    512-bucket instantiation, 28-bit targets in the 6-B entries. A giant (4096 hubs joined to each other and to 2M
    random ids) plus 2M random pairs over the whole range (the slow / union path), ids up to V - 1."""
    rng = np.random.default_rng(V & 0xFFFF)
    hubs = rng.choice(V, size=4096, replace=False).astype(np.uint32)
    n_h = 1 << 16
    hub_hub = np.stack([hubs[rng.integers(0, 4096, n_h)], hubs[rng.integers(0, 4096, n_h)]], axis=1)
    n_s = (1 << 21) - n_h
    star = np.stack([hubs[rng.integers(0, 4096, n_s)], rng.integers(0, V, n_s, dtype=np.uint32)], axis=1)
    rand = rng.integers(0, V, size=(1 << 21, 2), dtype=np.uint32)
    pairs = np.concatenate([hub_hub, star, rand])[rng.permutation(1 << 22)]
    pairs[-1] = [V - 1, hubs[0]]
    d = to_device(torch_cuda, pairs)
    with DisjointSet(V) as ds:
        ds.tune(**FORCE)
        ds.enable_timing(1)
        ds.fold_device(d.data_ptr(), len(pairs))
        names = [k for k, _, _ in ds.fold_profile()]
        assert "bucket" in names and "slice_filter" in names, names  # the bucketed path ran
        assert mismatch(ds.labels(), oracle_labels(pairs, V)) is None


@pytest.mark.parametrize("bucketed", [False, True])
def test_device_batch_id_validation(torch_cuda, bucketed):
    """An edge with an id >= id_capacity in a DEVICE batch is skipped (never dereferenced) and reported once by
    the next synchronising call; the batch's other edges are folded."""
    V = 1 << 20
    cfg = G.scaled(G.CONFIGS["c2_rmat20"], n_edges=1 << 20, seed=0xBAD)
    pairs = G.generate_host(cfg)
    bad = pairs.copy()
    bad[1000] = [V + 5, 3]
    bad[77777] = [7, 0xFFFFFFF0]
    d = to_device(torch_cuda, bad)
    good = np.delete(pairs, [1000, 77777], axis=0)
    with DisjointSet(V) as ds:
        if bucketed:
            ds.tune(**FORCE)
        ds.fold_device(d.data_ptr(), len(bad))
        with pytest.raises(GellyCCError, match="id_capacity"):
            ds.labels()
        assert mismatch(ds.labels(), oracle_labels(good, V)) is None  # reported once; state = the valid edges


def test_pinned_host_fold(torch_cuda):
    """gcc_forest_fold_pinned: chunked H2D overlapped with the folds (several chunks), ids validated on the device."""
    cfg = G.scaled(G.CONFIGS["c2_rmat20"], n_edges=(1 << 22) + 3, seed=0x9117)
    E, V = cfg.info()
    pairs = G.generate_host(cfg)
    h = torch_cuda.from_numpy(pairs.view(np.int32).reshape(-1)).pin_memory()
    with DisjointSet(V) as ds:
        ds.tune(pin_chunk=1 << 20)  # 5 chunks through the two device slots
        ds.fold_pinned(h.data_ptr(), E)
        ds.sync()
        assert mismatch(ds.labels(), oracle_labels(pairs, V)) is None


def test_long_max_value_is_a_valid_id():
    """DisjointSet<Long> keeps Long.MAX_VALUE like any other id (makeSet + find, and as a component's minimum)."""
    mx = (1 << 63) - 1
    with_max = LongDisjointSet(16)
    with_max.makeSet(mx)
    assert with_max.find(mx) == mx and with_max.size() == 1
    with_max.union(mx, mx - 1)
    assert with_max.find(mx) == mx - 1
    ids, lab = with_max.seen_labels()
    assert sorted(ids.tolist()) == [mx - 1, mx]
    with_max.close()


@pytest.mark.parametrize("name", ["c4_share", "c4_kron26"])
def test_c4_full_size_digest(torch_cuda, name):
    """The north-star config at full size on one GPU: C4's first 2^27 edges (one GPU's share at N = 8) and all of
    C4 (Kronecker s26, 2^30 edges, 64M ids), one window, against the oracle digests in
    tests/golden/stream_digests.json (tests/golden/make_stream_digests.py, computed on the CPU)."""
    cfg = G.CONFIGS[name]
    E, V = cfg.info()
    fx = DIGESTS[name]
    assert fx["edges"] == E and fx["vertices"] == V
    d = gen_device(torch_cuda, cfg)
    with DisjointSet(V) as ds:
        ds.fold_device(d.data_ptr(), E)
        lab = ds.labels()
        assert orc.label_digest(lab) == int(fx["digest"])
        assert ds.size() == fx["seen"] and ds.num_components() == fx["components"]
        # and split into two windows of the same forest (the second one is a filtered fold on the bitmap)
        ds.reset()
        ds.fold_device(d.data_ptr(), E // 2)
        ds.compress()
        ds.fold_device(d.data_ptr() + 8 * (E // 2), E - E // 2)
        assert orc.label_digest(ds.labels()) == int(fx["digest"])
    del d
    torch_cuda.cuda.empty_cache()


def test_c4_share_strong_split_and_merge(torch_cuda):
    """C4's share split into 4 contiguous partitions (bench.py's N = 4 split), folded into 4 forests and merged by
    CombineCC: the oracle digest."""
    cfg = G.CONFIGS["c4_share"]
    E, V = cfg.info()
    d = gen_device(torch_cuda, cfg)
    parts = [DisjointSet(V) for _ in range(4)]
    for r, ds in enumerate(parts):
        lo, hi = E * r // 4, E * (r + 1) // 4
        ds.fold_device(d.data_ptr() + 8 * lo, hi - lo)
    for ds in parts[1:]:
        parts[0].merge(ds)
    assert orc.label_digest(parts[0].labels()) == int(DIGESTS["c4_share"]["digest"])
    for ds in parts:
        ds.close()
    del d
    torch_cuda.cuda.empty_cache()


# ---- checkpoint / serialized summary (Merger.snapshotState / restoreState, SummaryAggregation.java:127-135) ----
@pytest.mark.parametrize("kind,cfg_args", [
    (2, ("c2_rmat20", {"scale": 18, "n_edges": 1 << 21, "seed": 0x5EED})),      # a dominant component: message
    (1, ("c3_gnm24", {"n_vertices": 1 << 19, "n_edges": 1 << 18, "seed": 0x5EED})),  # none: (v, label) pairs
])
def test_checkpoint_restore_then_keep_folding(torch_cuda, kind, cfg_args):
    """Fold windows; after every window snapshot the running summary (Merger.snapshotState -> bytes), restore it into
    a fresh summary (Merger.restoreState), and keep folding BOTH: every window of both equals the oracle."""
    from gelly_stream.aggregation import Merger
    from gelly_stream.library import CombineCC

    cfg = G.scaled(G.CONFIGS[cfg_args[0]], **cfg_args[1])
    E, V = cfg.info()
    pairs = G.generate_host(cfg)
    starts = np.linspace(0, E, 6).astype(np.uint64)
    want = orc.cc_stream(pairs, starts, V, partitions=2, threads=2)["digest"]
    d = to_device(torch_cuda, pairs)
    live = Merger(lambda: DisjointSet(V), CombineCC(), False)
    restored = None
    for w in range(len(starts) - 1):
        b, e = int(starts[w]), int(starts[w + 1])
        for m in (live, restored):
            if m is None:
                continue
            part = DisjointSet(V)
            part.fold_device(d.data_ptr() + 8 * b, e - b)
            out = m.flatMap(part)
            assert orc.label_digest(out.labels()) == int(want[w]), (w, m is restored)
        state = live.snapshotState()
        assert isinstance(state[0], bytes)
        hdr = np.frombuffer(state[0][:32], dtype="<u4")
        assert hdr[0] == 0x53434347 and hdr[1] == 1 and hdr[2] == V
        if w == len(starts) - 2:
            assert hdr[3] == kind, hdr  # the smaller form for this graph
        restored = Merger(lambda: DisjointSet(V), CombineCC(), False)
        restored.restoreState(state)
        assert np.array_equal(restored.summary.labels(), live.summary.labels()), w


def test_serialized_summary_rejects_bad_bytes():
    ds = DisjointSet(1 << 10)
    ds.fold(np.array([[1, 2], [3, 4]], dtype=np.uint32))
    blob = ds.serialize()
    with pytest.raises(GellyCCError):
        DisjointSet(1 << 10).deserialize(b"\x00" * 40)  # bad magic
    with pytest.raises(GellyCCError):
        DisjointSet(1 << 10).deserialize(blob[:-4])  # truncated
    with pytest.raises(GellyCCError):
        DisjointSet(1 << 5).deserialize(blob)  # larger id range than the target
    again = DisjointSet.from_bytes(blob)
    assert again.find(2) == 1 and again.find(4) == 3 and again.size() == 4


def test_serialized_summary_rejects_wrapped_lengths():
    """a kind-1 header whose n_seen makes 8 * n_seen wrap (2^61) with payload 0, and a payload that makes
    header + payload wrap, must be rejected before any pair is read (GCC_E_INVALID), not folded past the buffer."""
    import struct

    V = 1 << 10
    for n_seen, payload in ((1 << 61, 0), (4, (1 << 64) - 16), (3, 24 + 8)):
        blob = struct.pack("<IIIIQQ", 0x53434347, 1, V, 1, n_seen, payload) + b"\x00" * 32
        with pytest.raises(GellyCCError) as e:
            DisjointSet(V).deserialize(blob)
        assert e.value.code == -1, (n_seen, payload)


def test_absorb_ignores_bitmap_bits_past_the_id_range(torch_cuda):
    """a kind-2 (message) summary whose last bitmap word carries bits past id_capacity (untrusted bytes)
    must not index parent[] out of range: those bits are masked, the rest of the message restores exactly."""
    cfg = G.scaled(G.CONFIGS["c2_rmat20"], scale=17, n_edges=1 << 20, seed=0xB17)
    E, V = cfg.info()
    V = V - 7  # an id range that ends inside a 64-id bitmap word (and big enough for the giant filter)
    pairs = G.generate_host(cfg) % np.uint32(V)
    src = DisjointSet(V)
    src.fold(pairs)
    blob = bytearray(src.serialize())
    hdr = np.frombuffer(bytes(blob[:32]), dtype="<u4")
    assert hdr[3] == 2, "expected the message form (a dominant component)"
    nw = (V + 63) // 64
    last = 32 + 16 + 8 * (nw - 1)  # the message's last bitmap word
    word = int.from_bytes(blob[last:last + 8], "little") | (~((1 << (V % 64)) - 1) & ((1 << 64) - 1))
    blob[last:last + 8] = word.to_bytes(8, "little")
    dst = DisjointSet(V)
    dst.deserialize(bytes(blob))
    assert np.array_equal(dst.labels(), src.labels())
    src.close()
    dst.close()
