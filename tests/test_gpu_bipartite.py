"""GPU: BipartitenessCheck's signed forest (csrc/gelly_bip.hip, gcc_signed_*) and ConnectedComponentsTree's
pairwise combine, through the C ABI, against the reference's KATs, the golden fixtures and the CPU oracle.

Parity contract: per window, the success flag and per vertex the canonical word
(component min << 1) | (sign differs from the min's); the reference KATs' toString lines verbatim.
"""
import glob
import os

import numpy as np
import pytest

import oracle as orc
from gelly_stream import (BipartitenessCheck, Candidates, ConnectedComponents, ConnectedComponentsTree,
                          SimpleEdgeStream)
from gelly_stream import generators as G

pytestmark = pytest.mark.gpu
UNSEEN = 0xFFFFFFFF
HERE = os.path.dirname(os.path.abspath(__file__))


def test_reference_kats_verbatim(golden):
    """BipartitenessCheckTest / NonBipartitnessCheckTest: the emitted line, character for character."""
    fx = golden("bip_kat.json")
    for key in ("bipartite", "non_bipartite"):
        k = fx[key]
        stream = SimpleEdgeStream(np.array(k["edges"], dtype=np.uint32))
        out = [c.toString() for c in stream.aggregate(BipartitenessCheck(500, id_capacity=k["V"]))]
        assert out == [k["expected"]], key


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(HERE, "golden", "bip_*.json"))))
def test_fixture_streams(path, golden):
    name = os.path.basename(path)
    if name == "bip_kat.json":
        return
    fx = golden(name)
    pairs = np.array(fx["pairs"], dtype=np.uint32)
    starts = fx["window_starts"]
    c = Candidates(fx["V"])
    for w, want in enumerate(fx["windows"]):
        c.fold(pairs[starts[w]:starts[w + 1]])
        if want is None:
            continue
        assert c.getSuccess() == want["success"], (name, w)
        if want["success"]:
            assert c.words().tolist() == want["words"], (name, w)
        else:
            assert c.getMap() == {} and c.toString() == "(false,{})"
        lit = want["reference_literal"]
        if not want["reference_literal_agrees"]:  # a pinned deviation (tests/test_bipartite_oracle.py DIVERGENT)
            assert (c.getSuccess(), c.toString()) != (lit["success"], lit["string"]), (name, w)
        else:
            assert c.getSuccess() == lit["success"], (name, w)
    c.close()


def bipartite_stream(n_ids, n_edges, seed, odd_edge_at=None):
    rng = np.random.default_rng(seed)
    side = rng.integers(0, 2, n_ids)
    A, B = np.flatnonzero(side == 0), np.flatnonzero(side == 1)
    e = np.stack([rng.choice(A, n_edges), rng.choice(B, n_edges)], axis=1).astype(np.uint32)
    flip = rng.integers(0, 2, n_edges).astype(bool)
    e[flip] = e[flip][:, ::-1]
    if odd_edge_at is not None:  # one edge inside side A closes an odd cycle (once both ends are connected)
        e[odd_edge_at] = [A[0], A[1]]
    return e


@pytest.mark.parametrize("odd", [False, True])
def test_large_random_vs_oracle(odd):
    """1M edges over 256K ids in 4 windows, device-resident, vs the oracle every window."""
    V, E = 1 << 18, 1 << 20
    pairs = bipartite_stream(V, E, 11, odd_edge_at=(3 * E // 4) if odd else None)
    starts = [0, 1000, E // 2, 3 * E // 4 + 1, E]
    want = orc.bip_stream(pairs, starts, V, partitions=3)
    import torch

    d = torch.from_numpy(pairs.view(np.int32)).cuda()
    c = Candidates(V)
    for w in range(len(starts) - 1):
        c.fold_device(d.data_ptr() + 8 * starts[w], starts[w + 1] - starts[w])
        assert c.getSuccess() == bool(want["success"][w]), w
        if want["success"][w]:
            assert np.array_equal(c.words(), want["words"][w]), w
    c.close()


def test_merge_is_combine_function():
    """combineFunction.reduce(c1, c2) = c1.merge(c2): two partials merged equal one fold of both halves; a
    failed input fails the result (Candidates.merge :78-81)."""
    V, E = 1 << 14, 1 << 16
    pairs = bipartite_stream(V, E, 5)
    a, b, whole = Candidates(V), Candidates(V), Candidates(V)
    a.fold(pairs[: E // 3])
    b.fold(pairs[E // 3:])
    whole.fold(pairs)
    assert a.merge(b) is a
    assert a.getSuccess() and np.array_equal(a.words(), whole.words())
    bad = Candidates(V)
    bad.fold(np.array([[1, 2], [2, 3], [3, 1]], dtype=np.uint32))
    assert not bad.getSuccess()
    assert not a.merge(bad).getSuccess() and a.toString() == "(false,{})"
    for x in (a, b, whole, bad):
        x.close()


def test_self_loops_only_add_the_vertex():
    c = Candidates(16)
    c.fold(np.array([[5, 5], [7, 7], [7, 8]], dtype=np.uint32))
    assert c.getSuccess()
    assert c.toString() == "(true,{5={5=(5,true)}, 7={7=(7,true), 8=(8,false)}})"
    c.close()


def test_connected_components_tree_matches_bulk():
    """ConnectedComponentsTree (SummaryTreeReduce's pairwise combine of 8 partial forests per window) emits the
    same partition as ConnectedComponents and the oracle, every window."""
    cfg = G.scaled(G.CONFIGS["c2_rmat20"], scale=14, n_edges=1 << 18)
    pairs = G.generate_host(cfg)
    _, V = cfg.info()
    W = 1 << 16
    starts = np.arange(0, len(pairs) + 1, W, dtype=np.uint64)
    want = orc.cc_stream(pairs, starts, V, partitions=8, want_labels=True)["labels"]
    tree = SimpleEdgeStream(pairs, edges_per_window=W, parallelism=8).aggregate(
        ConnectedComponentsTree(1000, id_capacity=V, degree=8))
    bulk = SimpleEdgeStream(pairs, edges_per_window=W).aggregate(ConnectedComponents(1000, id_capacity=V))
    n = 0
    for w, (t, b) in enumerate(zip(tree, bulk)):
        assert np.array_equal(t.labels(), want[w]), w
        assert np.array_equal(b.labels(), want[w]), w
        n += 1
    assert n == len(starts) - 1


def test_bench_streams_full_size(golden):
    """bench.py's bip legs at full size, device-resident: to_bipartite(C3) against the oracle's words digest
    (tests/golden/digests_bip.json), and C3 as it is fails (the fold stops once failed; success stays false)."""
    import torch

    from bench import label_digest

    want = golden("digests_bip.json")
    cfg = G.CONFIGS["c3_gnm24"]
    E, V = cfg.info()
    d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
    G.generate_device(cfg, 0, E, d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    c = Candidates(V)
    c.fold_device(d.data_ptr(), E)
    assert c.getSuccess() == want["c3_gnm24"]["success"] is False
    c.fold_device(d.data_ptr(), E)  # a failed summary stays failed
    assert not c.getSuccess() and c.toString() == "(false,{})"
    G.to_bipartite_device(d)
    torch.cuda.synchronize()
    c.reset()
    c.fold_device(d.data_ptr(), E)
    c.compress()
    w = c.words()
    assert c.getSuccess()
    assert str(label_digest(w)) == want["bip_c3_gnm24"]["digest"]
    assert int((w != UNSEEN).sum()) == want["bip_c3_gnm24"]["seen"]
    c.close()


@pytest.mark.parametrize("giant,xcd,bucket", [(1, 1, 0), (1, 0, 0), (0, 0, 0), (1, 0, 1)])
@pytest.mark.parametrize("odd", [False, True])
def test_kron_hubs_vs_oracle(odd, giant, xcd, bucket):
    """A kron stream mapped bipartite (hubs: contended roots), 3 windows, every window's words vs the oracle. Window
    1 (6M edges over 2^18 ids) takes the giant-filtered fold (gcc_signed_tune giant = 1, the default) — over the batch
    split by source part, one part per XCD (xcd = 1, forced below its 2^25-edge default by xcd_min), bucketed by the
    ids' slices (bucket = 1, the default since round 5; one slice at 2^18 ids), or neither — or the plain one
    (giant = 0); with one odd edge between two hubs' side the summary fails in that window (inside the giant: the
    parity-bit check), and the next window's fold stops at once."""
    import torch

    cfg = G.scaled(G.CONFIGS["c4_kron26"], scale=18, n_edges=1 << 23)
    E, V = cfg.info()
    pairs = G.to_bipartite(G.generate_host(cfg))
    if odd:
        pairs[(3 * E) // 4] = [pairs[0, 0], pairs[1, 0]]  # two even ids: an even-even edge
    starts = [0, 4096, (3 * E) // 4 + 1, E]
    want = orc.bip_stream(pairs, starts, V, partitions=2)
    assert want["success"][0] and (want["success"][1] != odd)  # the odd edge closes a cycle in window 1
    d = torch.from_numpy(pairs.reshape(-1).view(np.int32)).cuda()
    c = Candidates(V).tune(giant=giant, xcd=xcd, xcd_min=0, bucket=bucket)
    for w in range(len(starts) - 1):
        c.fold_device(d.data_ptr() + 8 * starts[w], starts[w + 1] - starts[w])
        assert c.getSuccess() == bool(want["success"][w]), w
        if want["success"][w]:
            assert np.array_equal(c.words(), want["words"][w]), w
    c.close()


@pytest.mark.parametrize("spill", [False, True])
def test_bucketed_fold_overflow_and_spill(spill):
    """The bucketed signed fold's first bucketing takes its capacities from a sampled layout (64 runs of 1024 edges
    spread over the batch past the fold's sample). A batch built against that layout: the sampled runs have their
    sources in slice 0, the other edges (all of them, or 1/8) in slice 1, so bucket 1 is under-estimated. 1/8: the
    excess goes to the overflow list (the rest's rule, at level 1); all: the overflow list overflows too (spill) and
    the whole batch is folded again by the rest kernel. Both give the unbucketed fold's words; with an odd edge the
    summary fails either way."""
    import torch

    V = 1 << 20
    n = 1 << 22
    s = max(1 << 20, n >> 6)  # gelly_bip.hip signed_fold: the sample (sample_shift 6)
    rest = n - s
    stride = rest // 64  # bucket_layout_kernel: run k = [k * stride, k * stride + 1024) of the rest
    rng = np.random.default_rng(11 + spill)
    # the sample: a star of 64 even hubs over odd ids (a dominant component for the vote), sources in slice 0
    su = 2 * rng.integers(0, 64, size=s, dtype=np.uint32)
    sv = 2 * rng.integers(0, V // 2, size=s, dtype=np.uint32) + 1
    # the rest: even sources in slice 1 (all, or every 8th), slice 0 at the sampled runs; odd targets anywhere
    ru = 2 * rng.integers(0, (1 << 19) // 2, size=rest, dtype=np.uint32)
    hot = np.ones(rest, bool) if spill else (np.arange(rest) % 8 == 5)
    ru[hot] += 1 << 19
    sampled = (np.arange(rest) % stride) < 1024
    ru[sampled] = 2 * rng.integers(0, (1 << 19) // 2, size=int(sampled.sum()), dtype=np.uint32)
    rv = 2 * rng.integers(0, V // 2, size=rest, dtype=np.uint32) + 1
    pairs = np.concatenate([np.stack([su, sv], axis=1), np.stack([ru, rv], axis=1)]).astype(np.uint32)
    for odd in (False, True):
        p = pairs.copy()
        if odd:
            p[s + rest // 2] = [p[0, 0], p[s + 1, 0]]  # two even ids: an even-even edge inside the giant
        d = torch.from_numpy(p.reshape(-1).view(np.int32)).cuda()
        ref = Candidates(V).tune(bucket=0)
        ref.fold_device(d.data_ptr(), n)
        c = Candidates(V).tune(bucket_min=0)
        c.fold_device(d.data_ptr(), n)
        assert c.getSuccess() == ref.getSuccess() == (not odd)
        if not odd:
            assert np.array_equal(c.words(), ref.words())
        ref.close()
        c.close()


@pytest.mark.parametrize("odd", [False, True])
@pytest.mark.parametrize("knobs", [{}, {"bucket_levels": 1}, {"bucket_levels": 3}, {"sample_shift": 12},
                                   {"sample_shift": 12, "bucket_levels": 3}])
def test_bucketed_fold_many_slices(odd, knobs):
    """The bucketed signed fold (round 5) over 2^22 ids (8 slices of 2^19), a kron stream mapped bipartite: the same
    words as the unbucketed giant kernel and the oracle's success flag; with one odd edge (two even hub ids) placed
    late in the batch, the summary fails. A tiny sample (sample_shift 12: the snapshot holds a small part of the
    giant) sends most edges through the second level and the rest."""
    import torch

    cfg = G.scaled(G.CONFIGS["c4_kron26"], scale=22, n_edges=1 << 23)
    E, V = cfg.info()
    pairs = G.to_bipartite(G.generate_host(cfg))
    if odd:
        pairs[(7 * E) // 8] = [pairs[0, 0], pairs[1, 0]]
    d = torch.from_numpy(pairs.reshape(-1).view(np.int32)).cuda()
    ref = Candidates(V).tune(bucket=0)
    ref.fold_device(d.data_ptr(), E)
    assert ref.getSuccess() != odd
    c = Candidates(V).tune(**knobs)
    c.fold_device(d.data_ptr(), E)
    assert c.getSuccess() != odd
    if not odd:
        assert np.array_equal(c.words(), ref.words())
        # a second batch into the same forest (the bucketed fold's words are canonical: a compressed forest)
        c.fold_device(d.data_ptr(), E // 2)
        assert c.getSuccess() and np.array_equal(c.words(), ref.words())
    ref.close()
    c.close()


@pytest.mark.parametrize("extra_ids", [0, 1 << 20])
def test_bucketed_fold_largest_default_id_range(extra_ids):
    """the bucketed signed fold is the default up to 2^27 ids (256 slices: the largest shape it takes by
    default, 4-B key-only emit lists); past 2^27 the giant-filtered fold runs. A kron stream over 2^27 ids (+ 2^20
    unused ids above it) mapped bipartite, 2^25 edges: the same words and success as bucket = 0, with and without an
    odd edge between two hubs' sides."""
    import torch

    cfg = G.scaled(G.CONFIGS["c4_kron26"], scale=27, n_edges=1 << 25)
    E, V0 = cfg.info()
    V = V0 + extra_ids
    d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
    G.generate_device(cfg, 0, E, d.data_ptr(), 0)
    G.to_bipartite_device(d)
    for odd in (False, True):
        if odd:  # one edge between two even ids (the same side): an odd cycle once both sides are connected
            d[E] = d[0]
            d[E + 1] = d[2]
        torch.cuda.synchronize()  # the summaries fold on their own non-blocking streams
        ref = Candidates(V).tune(bucket=0)
        ref.fold_device(d.data_ptr(), E)
        c = Candidates(V)
        c.fold_device(d.data_ptr(), E)
        assert c.getSuccess() == ref.getSuccess()
        if not odd:
            assert ref.getSuccess()
            assert np.array_equal(c.words(), ref.words())
        ref.close()
        c.close()
    del d
    torch.cuda.empty_cache()


def test_giant_fold_knobs_and_no_dominant_component():
    """The giant-filtered fold's knobs change speed only: to_bipartite(scaled C3) (no dominant component: the
    snapshot stays empty) and a kron stream (a sample of 1/2 or 1/1024, min_share 1.0 = never filter) fold to the
    same words as the plain fold; an unknown key is GCC_E_INVALID."""
    import torch

    from gelly_stream.native import GellyCCError

    for cfg in (G.scaled(G.CONFIGS["c3_gnm24"], n_vertices=1 << 23, n_edges=1 << 22),
                G.scaled(G.CONFIGS["c4_kron26"], scale=20, n_edges=1 << 22)):
        E, V = cfg.info()
        pairs = G.to_bipartite(G.generate_host(cfg))
        d = torch.from_numpy(pairs.reshape(-1).view(np.int32)).cuda()
        ref = Candidates(V).tune(giant=0)
        ref.fold_device(d.data_ptr(), E)
        want = ref.words().copy()
        assert ref.getSuccess()
        ref.close()
        for knobs in ({}, {"sample_shift": 1}, {"sample_shift": 10}, {"min_share": 1.0}, {"min_share": 0.001},
                      {"unroll": 1}, {"unroll": 8}, {"xcd": 1, "xcd_min": 0}, {"xcd": 1, "xcd_min": 0, "min_share": 1.0},
                      {"xcd": 1, "xcd_min": 0, "sample_shift": 10}, {"xcd": 1}, {"bucket": 0}, {"bucket_levels": 1},
                      {"bucket_min": 0, "sample_shift": 10}, {"min_share": 0.001, "bucket_levels": 1},
                      {"bucket_items": 1}, {"bucket_items": 16}):
            c = Candidates(V).tune(**knobs)
            c.fold_device(d.data_ptr(), E)
            assert c.getSuccess() and np.array_equal(c.words(), want), (cfg.name, knobs)
            c.close()
    c = Candidates(16)
    with pytest.raises(GellyCCError):
        c.tune(no_such_knob=1)
    c.close()


def _bip_group_worker(rank, world, port, pairs, starts, q, extra_ids=0):
    """One rank (spawned before any GPU call): folds its contiguous 1/world of every window into a Candidates on
    cuda:0, then bipartite.merge_group over gloo; reports (success, words) per window."""
    import sys

    root = os.path.dirname(HERE)
    sys.path[:0] = [os.path.join(root, "gelly-streaming_amd")]
    import torch
    import torch.distributed as dist

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from gelly_stream.bipartite import Candidates as C
        from gelly_stream.bipartite import merge_group

        V = int(pairs.max()) + 1 + (extra_ids if rank == 1 else 0)
        d = torch.from_numpy(pairs.reshape(-1).view(np.int32)).cuda()
        c = C(V)
        out = []
        for w in range(len(starts) - 1):
            b, e = int(starts[w]), int(starts[w + 1])
            lo, hi = b + (e - b) * rank // world, b + (e - b) * (rank + 1) // world
            c.fold_device(d.data_ptr() + 8 * lo, hi - lo)
            merge_group(c)
            ok = c.getSuccess()
            out.append((ok, c.words().copy() if ok else None))
        dist.barrier()
        q.put((rank, out))
    except Exception as ex:
        q.put((rank, repr(ex)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("odd", [False, True])
def test_merge_group_two_ranks_share_one_gpu(odd):
    """combineFunction across processes (bipartite.merge_group, gcc_signed_merge_words): 2 fresh ranks over gloo
    each fold half of every window of a kron stream mapped bipartite; after each merge both hold the oracle's words
    (the union of both halves); with an odd edge in rank 1's half of window 1, both ranks report the failure."""
    import socket

    import torch.multiprocessing as mp

    cfg = G.scaled(G.CONFIGS["c4_kron26"], scale=16, n_edges=1 << 19)
    E, V = cfg.info()
    pairs = G.to_bipartite(G.generate_host(cfg))
    pairs[-1] = [V - 2, V - 1]  # id V - 1 present, so every rank sizes its forest to V
    starts = [0, 1000, E // 2, E]
    if odd:
        pairs[E // 2 - 10] = [pairs[0, 0], pairs[1, 0]]  # an even-even edge, in rank 1's half of window 1
    want = orc.bip_stream(pairs, starts, V, partitions=2)
    assert want["success"][0] and (want["success"][1] != odd)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bip_group_worker, args=(r, 2, port, pairs, starts, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        results = dict(q.get(timeout=150) for _ in range(2))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(2):
        out = results[r]
        assert isinstance(out, list), (r, out)
        for w, (ok, words) in enumerate(out):
            assert ok == bool(want["success"][w]), (r, w)
            if ok:
                assert np.array_equal(words, want["words"][w]), (r, w)


def test_merge_group_rejects_different_id_ranges():
    """the ranks' id_capacity is checked (all_reduce MAX of +cap and -cap beside the fail flag) before any
    words move: a rank with a larger id range makes merge_group raise on EVERY rank, instead of a mismatched
    all_gather."""
    import socket

    import torch.multiprocessing as mp

    pairs = np.asarray([[0, 1], [2, 3], [4, 5], [6, 7]], dtype=np.uint32)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bip_group_worker, args=(r, 2, port, pairs, [0, 4], q, 64)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        results = dict(q.get(timeout=150) for _ in range(2))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(2):
        assert isinstance(results[r], str) and "id_capacity differ" in results[r], results


def test_device_words_tensor_matches_host_words():
    """The send side of merge_group over nccl: the canonical words straight from the forest's device buffer
    (gcc_signed_device_words wrapped through __cuda_array_interface__) equal the host copy."""
    cfg = G.scaled(G.CONFIGS["c4_kron26"], scale=14, n_edges=1 << 16)
    E, V = cfg.info()
    pairs = G.to_bipartite(G.generate_host(cfg))
    c = Candidates(V)
    c.fold(pairs)
    t = c.device_words_tensor()
    assert t.device.type == "cuda" and t.dtype.itemsize == 4 and t.numel() == V
    assert np.array_equal(t.cpu().numpy().view(np.uint32), c.words())
    c.close()


def test_xcd_split_overflow_and_spill():
    """The XCD split's capacities come from a strided sample of the batch; a batch whose sampled runs (the first 1024
    edges of every 1/64) all have their sources in part 0 while the rest of it has them in part 7 leaves part 7 a
    capacity of its slack alone, so most of its edges overflow — and the overflow list too, so the whole batch is
    folded again (exact: idempotent). Bipartite and with an odd edge, every word against the oracle."""
    import torch

    V = 1 << 20
    n = 1 << 24
    rng = np.random.default_rng(0x5EED)
    u = rng.integers(0, 1 << 16, n, dtype=np.int64) * 2  # even ids: sources in part 0 (ids < 2^17)
    v = rng.integers(0, V // 2, n, dtype=np.int64) * 2 + 1  # odd ids anywhere
    s = max(1 << 20, n >> 6) & ~1                            # the signed fold's sample prefix (plain fold)
    pos = np.arange(n) - s
    m = n - s
    stride = m // 64
    far = (pos >= 0) & ((pos % stride) >= 1024)
    u[far] = (7 << 17) + rng.integers(0, 1 << 16, int(far.sum()), dtype=np.int64) * 2  # part 7, unsampled
    pairs = np.stack([u, v], axis=1).astype(np.uint32)
    for odd in (False, True):
        p = pairs.copy()
        if odd:
            p[n - 10] = [p[5, 0], p[7, 0]]  # two even ids
        want = orc.bip_stream(p, [0, n], V, partitions=1)
        d = torch.from_numpy(p.reshape(-1).view(np.int32)).cuda()
        c = Candidates(V).tune(xcd=1, xcd_min=0, min_share=0.001)
        c.fold_device(d.data_ptr(), n)
        assert c.getSuccess() == bool(want["success"][0]), odd
        if want["success"][0]:
            assert np.array_equal(c.words(), want["words"][0])
        c.close()
