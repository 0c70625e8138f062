"""The pipelined emission (round 5, tune key inc_pipe; gelly_cc.hip compress_pipe_kernel): in the incremental regime
(short windows over a big forest) the scan that emits window w runs on a second stream beside window w+1's fold.
Measured slower than the in-place incremental compress, so OFF by default; these tests turn
it on (and keep it exact while it stays in the tree).

What has to hold, window by window, against the oracle's windowed digests (tests/golden/stream_digests.json) or a
forest with the mode off (inc_pipe = 0, the in-place incremental compress of rounds 2-4):
* the emissions of a whole stream folded with compress() per window and no read between them (the overlapped
  schedule bench.py times), checked at sampled windows and at the end;
* every window read (each read waits for its window's scan);
* leaving the mode from every kind of entry point — a CombineCC merge, the raw-pointer view, a batch too long for the
  regime, a knob change, serialize, reset — with and without a fold pending since the last compress, and coming back;
* an id range that is not a multiple of 256 (the scan's partial last chunk).
Reference: the Merger emits a summary after every window (…/SummaryAggregation.java:107-119); DisjointSet.union
(…/summaries/DisjointSet.java:97-123).
"""
import json
import os

import numpy as np
import pytest

import oracle as orc
from gelly_stream import DisjointSet
from gelly_stream import generators as G

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIGESTS = json.load(open(os.path.join(ROOT, "tests", "golden", "stream_digests.json")))


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    return torch


def gen_device(torch_cuda, cfg):
    E, _ = cfg.info()
    t = torch_cuda.empty(2 * E, dtype=torch_cuda.int32, device="cuda:0")
    G.generate_device(cfg, 0, E, t.data_ptr(), 0)
    torch_cuda.cuda.synchronize()
    return t


def windows_of(name):
    fx = DIGESTS[name]
    return fx, [0] + [w["end"] for w in fx["windows"]]


def digest_ok(ds, want):
    dig, seen, comps = ds.label_digest()
    return (str(dig), seen, comps) == (want["digest"], want["seen"], want["components"])


def pipe_ran(ds):
    """The scan kernel appears in the forest's dispatch log (timing mode): the mode was on."""
    return any(name == "compress_pipe" for name, _, _ in ds.fold_profile())


@pytest.mark.parametrize("name", ["c5_adversarial/w64K", "c3_gnm24/w1M"])
def test_overlapped_stream_matches_oracle(torch_cuda, name):
    """fold + compress() per window with no read in between (the scan of window w overlaps fold w+1), reads at a few
    windows (each read waits for its window's scan, then the overlap resumes), and the last window."""
    fx, starts = windows_of(name)
    cfg = G.CONFIGS[fx["config"]]
    E, V = cfg.info()
    d = gen_device(torch_cuda, cfg)
    nw = len(starts) - 1
    sample = {3, 4, nw // 3, nw // 2 + 1, nw - 2} if nw > 8 else {2, 5}
    ds = DisjointSet(V)
    ds.tune(inc_pipe=1, emit_div=0)
    ds.enable_timing(1)
    bad = []
    for rep in range(2):  # twice into the same forest (reset between): the roots arrays restart from UNSEEN
        ds.reset()
        for w in range(nw):
            ds.fold_device(d.data_ptr() + 8 * starts[w], starts[w + 1] - starts[w])
            ds.compress()
            if w in sample and not digest_ok(ds, fx["windows"][w]):
                bad.append((rep, w))
        if not digest_ok(ds, fx["windows"][-1]):
            bad.append((rep, "last"))
        if rep == 0:
            assert pipe_ran(ds), "the pipelined emission did not engage"
    ds.close()
    del d
    torch_cuda.cuda.empty_cache()
    assert not bad, bad


def test_c5_every_window_read(torch_cuda):
    """C5 at the defaults, every window's emission read and checked (each read waits for the window's scan)."""
    fx, starts = windows_of("c5_adversarial/w64K")
    cfg = G.CONFIGS[fx["config"]]
    E, V = cfg.info()
    d = gen_device(torch_cuda, cfg)
    ds = DisjointSet(V)
    ds.tune(inc_pipe=1, emit_div=0)
    bad = []
    for w in range(len(starts) - 1):
        ds.fold_device(d.data_ptr() + 8 * starts[w], starts[w + 1] - starts[w])
        if not digest_ok(ds, fx["windows"][w]):
            bad.append(w)
    ds.close()
    del d
    torch_cuda.cuda.empty_cache()
    assert not bad, bad


def gnm_stream(torch_cuda, V, E, seed):
    cfg = G.scaled(G.CONFIGS["c3_gnm24"], n_vertices=V, n_edges=E, seed=seed)
    return cfg, gen_device(torch_cuda, cfg)


def test_leaving_and_reentering_the_mode(torch_cuda):
    """G(n, m) at the threshold (2^22 ids, 2^21 edges, 32 windows of 2^16): the default forest against one with the
    mode off, every window, while entry points that leave the mode come in between — clean (right after a compress:
    the labels become parent[]) and dirty (a fold pending: parent[] stays the live forest, the next compress is
    full) — and the mode comes back at the next window."""
    cfg, d = gnm_stream(torch_cuda, 1 << 22, 1 << 21, 0x5151)
    E, V = cfg.info()
    W = 1 << 16
    pipe, ref = DisjointSet(V), DisjointSet(V)
    pipe.tune(inc_pipe=1, emit_div=0)
    ref.tune(inc_pipe=0, emit_div=0)
    side = DisjointSet(V)
    side.fold_device(d.data_ptr(), 3 * W)
    host = d[: 2 * W].cpu().numpy().view(np.uint32).reshape(-1, 2)
    pipe.enable_timing(1)
    for w in range(E // W):
        ptr, n = d.data_ptr() + 8 * w * W, W
        if w == 11:  # 2^21 edges (x inc_div 4 > 2^22 ids: outside the regime), a repeat of the first 32 windows
            pipe.fold_device(d.data_ptr(), 1 << 21)
            ref.fold_device(d.data_ptr(), 1 << 21)
        for ds in (pipe, ref):
            ds.fold_device(ptr, n)
            ds.compress()
        if w == 4:
            pipe.merge(side)  # clean exit (after a compress); side's edges are already folded: no change
        if w == 7:
            pipe.fold_device(ptr, n)  # the same window again: a pending fold, then a dirty exit
            pipe.device_ptr()
        if w == 14:
            pipe.tune(drain_at=64)  # a knob change leaves the mode (clean); it comes back at the next window
        if w == 17:
            blob = pipe.serialize()  # clean exit; restore into the other forest and compare
            other = DisjointSet(V)
            other.deserialize(blob)
            assert np.array_equal(other.labels(), ref.labels()), ("restored", w)
            other.close()
        if w == 20:
            pipe.fold(host[:1000])  # a host-fed batch (pinned staging): stays in the mode
            ref.fold(host[:1000])
        if w in (2, 9, 23) or w % 5 == 0:
            got = pipe.labels()
            want = ref.labels()
            assert np.array_equal(got, want), (w, int(np.flatnonzero(got != want)[0]))
        elif w % 3 == 0:
            assert pipe.label_digest() == ref.label_digest(), w
    assert pipe_ran(pipe)
    assert np.array_equal(pipe.labels(), ref.labels())
    assert pipe.size() == ref.size() and pipe.num_components() == ref.num_components()
    # reset in the mode, then the first windows again
    pipe.reset()
    ref.reset()
    for w in range(6):
        for ds in (pipe, ref):
            ds.fold_device(d.data_ptr() + 8 * w * W, W)
            ds.compress()
    assert np.array_equal(pipe.labels(), ref.labels())
    for ds in (pipe, ref, side):
        ds.close()
    del d
    torch_cuda.cuda.empty_cache()


@pytest.mark.parametrize("V", [(1 << 22) + 77, (1 << 22) + 256 * 3 + 1])
def test_partial_last_chunk(torch_cuda, V):
    """An id range that is not a multiple of 256: the scan's last chunk goes id by id, its new-id words included.
    The stream's ids reach the top of the range (a shuffled path over all ids), windows of 2^16 edges (the first one
    long enough for the vote, which finds no giant: the later windows take the recording fold)."""
    rng = np.random.default_rng(V)
    perm = rng.permutation(V).astype(np.uint32)
    pairs = np.stack([perm[:-1], perm[1:]], axis=1)[: 1 << 20]
    pairs = pairs[rng.permutation(len(pairs))]
    d = torch_cuda.from_numpy(pairs.view(np.int32).reshape(-1).copy()).to("cuda:0")
    W = 1 << 16
    starts = np.arange(0, len(pairs) + 1, W, dtype=np.uint64)
    want = orc.cc_stream(pairs, starts, V, partitions=1, threads=2)
    pipe, ref = DisjointSet(V), DisjointSet(V)
    pipe.tune(inc_pipe=1, emit_div=0)
    ref.tune(inc_pipe=0, emit_div=0)
    pipe.enable_timing(1)
    for w in range(len(starts) - 1):
        for ds in (pipe, ref):
            ds.fold_device(d.data_ptr() + 8 * int(starts[w]), W)
            ds.compress()
        if w % 4 == 3:
            got = pipe.labels()
            assert np.array_equal(got, ref.labels()), w
            assert orc.label_digest(got) == int(want["digest"][w]), w
    assert pipe_ran(pipe)
    assert orc.label_digest(pipe.labels()) == int(want["digest"][-1])
    for ds in (pipe, ref):
        ds.close()
