"""CPU, multi-process: the PRODUCT's cross-GPU merge loop (csrc/gelly_group.cpp, gcc_forest_group_merge with nranks > 1)
run by world 2-4 CPU processes, every window against the oracle's global partition.

What runs: ForestGroup (gelly_stream/distributed.py) bootstraps the communicator's unique id over a gloo process group
and calls gcc_forest_group_merge — the same Python and C++ code as `bench.py --gpus N` over RCCL. Only the two ends
are stand-ins (test infrastructure, tests/cpp): the forest half of the ABI is a host union-find
(host_forest.cpp, linked with the unchanged gelly_group.cpp into libgelly_group_host.so, hipmock for the HIP calls),
and the collectives go through host shared memory (shm_rccl.cpp, loaded through the product's GELLY_RCCL_LIB seam).
The reference's topology: SummaryBulkAggregation.java:81-83 (timeWindowAll(t).reduce(CombineCC) + Merger): after every
window every rank holds the partition of all edges so far.

Covered: compact rounds with a speculative capacity that overflows (a repeat round), the label fallback when no
component dominates, an injected absorb failure on one rank (every rank returns an error: failed-status header or
agree()), a transport failure on one rank (the communicator aborts, the peers' collective errors) and a peer that
dies inside a collective (the others time out with an error, never hang).
"""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST_LIB = os.path.join(ROOT, "tests", "cpp", "build", "libgelly_group_host.so")
SHM_HOST = os.path.join(ROOT, "tests", "cpp", "build", "libshm_rccl_host.so")
UNSEEN = 0xFFFFFFFF

pytestmark = pytest.mark.skipif(not (os.path.exists(HOST_LIB) and os.path.exists(SHM_HOST)),
                                reason="build tests/cpp first (make -C tests/cpp)")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _PlainGroup:
    """ForestGroup's calls without torch.distributed (the unique id comes from the parent): most cases here, so that a
    rank process starts in a second instead of importing torch."""

    def __init__(self, world, rank, uid):
        from gelly_stream.distributed import RcclComm

        self.comm = RcclComm(0, world, rank, uid)
        self.last = {}

    def merge_forest(self, forest):
        self.comm.merge(forest)
        self.last = self.comm.last_merge()

    def close(self):
        self.comm.close()


def worker(rank, world, port, V, pairs, starts, want, q, env, uid=None):
    """One rank: fold its contiguous 1/world of every window into a host forest, merge, check. uid None: through
    ForestGroup over a gloo process group (bench.py's bootstrap); else the parent's unique id and no torch."""
    import sys

    os.environ.update(env)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GELLY_CC_LIB=HOST_LIB, GELLY_RCCL_LIB=SHM_HOST)
    sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
    import ctypes

    dist = None
    if uid is None:
        import torch.distributed as dist
    try:
        if dist is not None:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        from gelly_stream.native import GellyCCError, call

        class HostForest:  # what RcclComm.merge needs: the forest handle
            def __init__(self, h):
                self.handle = h

        h = ctypes.c_void_p()
        call("gcc_forest_create", 0, V, ctypes.byref(h))
        if env.get("FAIL_ABSORB_RANK") == str(rank):
            call("gcc_forest_tune", h, b"fail_absorb", float(env["FAIL_ABSORB_AT"]))
        if dist is not None:
            from gelly_stream.distributed import ForestGroup

            group = ForestGroup(device=0)
        else:
            group = _PlainGroup(world, rank, uid)
        f = HostForest(h)
        lasts = []
        for w in range(len(starts) - 1):
            b, e = int(starts[w]), int(starts[w + 1])
            chunk = np.ascontiguousarray(pairs[b + (e - b) * rank // world: b + (e - b) * (rank + 1) // world])
            call("gcc_forest_fold_host", h, chunk.ctypes.data, len(chunk))
            if env.get("DISARM_RANK") == str(rank) and env.get("DISARM_AT") == str(w):
                call("gcc_forest_merge_labels_device", h, np.full(1, UNSEEN, np.uint32).ctypes.data, 1)  # disarms
            try:
                group.merge_forest(f)
            except GellyCCError as ex:
                if env.get("FAIL_ABSORB_RANK") == str(rank) and w + 1 < len(starts) - 1:
                    try:  # the failing rank calls once more: its peers learn of its failure in that merge at the latest
                        group.merge_forest(f)
                    except GellyCCError:
                        pass
                q.put((rank, w, "error", str(ex), lasts))
                return
            got = np.empty(V, dtype=np.uint32)
            call("gcc_forest_labels", h, got.ctypes.data, V)
            lasts.append(dict(group.last))
            if not np.array_equal(got, want[w]):
                q.put((rank, w, "mismatch", int(np.flatnonzero(got != want[w])[0]), lasts))
                return
        group.close()
        call("gcc_forest_destroy", h)
        q.put((rank, -1, "ok", "", lasts))
    except Exception as ex:  # report instead of hanging the parent
        q.put((rank, -2, "exception", repr(ex), []))
    finally:
        if dist is not None and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass


def unique_id(tag):
    """The stand-in's unique id, made in the parent (ncclGetUniqueId of tests/cpp/build/libshm_rccl_host.so)."""
    import ctypes

    os.environ["GELLY_SHM_RCCL_TAG"] = tag
    lib = ctypes.CDLL(SHM_HOST)
    buf = ctypes.create_string_buffer(128)
    assert lib.ncclGetUniqueId(buf) == 0
    return buf.raw


def run_world(world, V, pairs, starts, want, env=None, timeout=120, torch_bootstrap=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    tag = f"t{os.getpid()}_{port}"
    env = dict(env or {}, GELLY_SHM_RCCL_TAG=tag)
    uid = None if torch_bootstrap else unique_id(tag)
    procs = [ctx.Process(target=worker, args=(r, world, port, V, pairs, starts, want, q, env, uid))
             for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time

    try:
        results, t0 = [], time.time()
        while len(results) < world and time.time() - t0 < timeout:
            try:
                results.append(q.get(timeout=1))
            except queue.Empty:
                if not any(p.is_alive() for p in procs):  # a rank that died without reporting (the dead-peer case)
                    break
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
        for f in os.listdir("/dev/shm"):  # segments are unlinked once mapped; a crash before that leaves one
            if f.startswith(f"gshm_{tag}_"):
                os.unlink(os.path.join("/dev/shm", f))
    return sorted(results, key=lambda r: r[0]), [p.exitcode for p in procs]


def rmat_case(scale=16, n_edges=1 << 17):
    import oracle as orc
    from gelly_stream import generators as G

    cfg = G.scaled(G.CONFIGS["c2_rmat20"], scale=scale, n_edges=n_edges)
    pairs = G.generate_host(cfg)
    _, V = cfg.info()
    starts = np.array([0, 700, 701, n_edges // 3, n_edges], dtype=np.uint64)
    want = orc.cc_stream(pairs, starts, V, want_labels=True)["labels"]
    return V, pairs, starts, want


def gnm_case():
    """G(n, m) just above the threshold: no dominant component, so the lists overflow until labels pay."""
    import oracle as orc
    from gelly_stream import generators as G

    cfg = G.scaled(G.CONFIGS["c3_gnm24"], n_vertices=1 << 16, n_edges=36000, seed=0x3232)
    pairs = G.generate_host(cfg)
    E, V = cfg.info()
    starts = np.array([0, 1000, 9000, 20000, E], dtype=np.uint64)
    want = orc.cc_stream(pairs, starts, V, want_labels=True)["labels"]
    return V, pairs, starts, want


@pytest.mark.parametrize("world,torch_bootstrap", [(2, True), (3, False), (4, False)])
def test_compact_rounds_every_window(world, torch_bootstrap):
    """R-MAT: one dominant component. The first windows' lists outgrow the initial capacity (max(1024, V/64)), so the
    compact exchange repeats larger; every window of every rank equals the oracle's global partition. World 2 runs
    ForestGroup itself (the unique id broadcast over gloo, as bench.py does over nccl)."""
    V, pairs, starts, want = rmat_case()
    res, _ = run_world(world, V, pairs, starts, want, torch_bootstrap=torch_bootstrap)
    assert [r[:3] for r in res] == [(r, -1, "ok") for r in range(world)], res
    lasts = res[0][4]
    assert any(last["rounds"] >= 2 and not last["labels"] for last in lasts), lasts  # a repeat round ran
    assert not lasts[-1]["labels"]  # the compact form pays at the end
    # armed after the first merge: the short windows take the delta, the last (long) one the smaller compact message
    assert lasts[0]["kind"] == "compact" and any(last["kind"] == "delta" for last in lasts), lasts


@pytest.mark.parametrize("world", [2, 4])
def test_label_fallback_every_window(world):
    """No dominant component: the compact rounds overflow until the message would not be smaller than the label
    array, then labels are all-gathered — exact after partial compact rounds (union is idempotent)."""
    V, pairs, starts, want = gnm_case()
    res, _ = run_world(world, V, pairs, starts, want)
    assert [r[:3] for r in res] == [(r, -1, "ok") for r in range(world)], res
    assert any(last["labels"] for last in res[0][4]), res[0][4]


@pytest.mark.parametrize("at", [1, 2, 3, 4, 5])
def test_absorb_failure_is_an_error_on_every_rank(at):
    """Rank 1's at-th absorb fails (tune key fail_absorb). It keeps following the protocol: a next compact round
    carries its failed-status header, or the ranks agree() before growing the buffers or before the label exchange,
    so every rank's merge returns an error in that window. If the failed absorb was the merge's last step (after its
    last collective), the peers' merges were complete; the communicator stays poisoned and the peers get the error in
    the next merge. Either way no rank hangs and no rank reports success after the failure."""
    V, pairs, starts, want = gnm_case()
    res, codes = run_world(3, V, pairs, starts, want, env={"FAIL_ABSORB_RANK": "1", "FAIL_ABSORB_AT": str(at),
                                                           "GELLY_SHM_RCCL_TIMEOUT": "5"})
    assert len(res) == 3, (res, codes)
    assert all(r[2] == "error" for r in res), res
    w1 = res[1][1]
    assert "injected failure" in res[1][3], res
    for r in res:
        if r[0] != 1:
            assert r[1] in (w1, w1 + 1) and "rank 1 failed" in r[3], res


def test_transport_failure_aborts_every_rank():
    """Rank 1's second all_gather fails in the transport: it aborts its communicator; the peers' collective ends with
    an error (no hang)."""
    V, pairs, starts, want = rmat_case(scale=12, n_edges=1 << 14)
    res, _ = run_world(2, V, pairs, starts, want, env={"GELLY_SHM_RCCL_FAIL": "1:2", "GELLY_SHM_RCCL_TIMEOUT": "20"})
    assert [r[2] for r in res] == ["error", "error"], res
    assert "ncclAllGather" in res[0][3] and "ncclAllGather" in res[1][3], res


def test_dead_peer_is_an_error_not_a_hang():
    """Rank 1's process dies inside its first all_gather: rank 0 gets an error after the stand-in's timeout."""
    V, pairs, starts, want = rmat_case(scale=12, n_edges=1 << 14)
    res, codes = run_world(2, V, pairs, starts, want, env={"GELLY_SHM_RCCL_EXIT": "1:1", "GELLY_SHM_RCCL_TIMEOUT": "5"},
                           timeout=60)
    assert codes[1] == 3, codes
    assert len(res) == 1 and res[0][0] == 0 and res[0][2] == "error", res


def short_windows_case(n_windows=24, w=2048):
    """C5's shape at a CPU-test size: a shuffled path plus stars (gcc_gen ADVERSARIAL), many short windows."""
    import oracle as orc
    from gelly_stream import generators as G

    cfg = G.scaled(G.CONFIGS["c5_adversarial"], scale=14, n_stars=16, star_size=1024)
    pairs = G.generate_host(cfg)[: n_windows * w]
    _, V = cfg.info()
    starts = np.arange(0, len(pairs) + 1, w, dtype=np.uint64)
    want = orc.cc_stream(pairs, starts, V, want_labels=True)["labels"]
    return V, pairs, starts, want


@pytest.mark.parametrize("world", [2, 3, 4])
def test_delta_merge_every_window(world):
    """The delta merge (round 6): after the first (compact) merge every rank is armed, and each later window moves only
    (x, root(x)) for the ids the rank's fold changed — at most 2 per edge, 8 B each: the all_gather is <= 16 B per edge
    of the largest rank's window + the header, once the capacity has followed the windows (it is twice the largest
    window of the last merge). Every window of every rank equals the oracle's global partition."""
    V, pairs, starts, want = short_windows_case()
    res, _ = run_world(world, V, pairs, starts, want)
    assert [r[:3] for r in res] == [(r, -1, "ok") for r in range(world)], res
    for r in res:
        lasts = r[4]
        assert lasts[0]["kind"] == "compact", lasts[0]
        assert all(last["kind"] == "delta" and last["rounds"] == 1 for last in lasts[2:]), lasts
        per_rank = [int(starts[k + 1] - starts[k] + world - 1) // world for k in range(len(starts) - 1)]
        for k, last in enumerate(lasts[2:], start=2):
            assert last["bytes"] <= 16 * per_rank[k] + 16 + 15, (k, last)


def test_delta_unarmed_rank_takes_the_compact_rounds():
    """A rank whose window took an unrecorded mutation sends an UNARMED delta (host forest: a merge_labels call
    disarms it): every rank then takes the compact rounds, exact, and is armed again after it."""
    V, pairs, starts, want = short_windows_case(n_windows=6)
    res, _ = run_world(2, V, pairs, starts, want, env={"DISARM_RANK": "1", "DISARM_AT": "3"})
    assert [r[:3] for r in res] == [(0, -1, "ok"), (1, -1, "ok")], res
    kinds = [last["kind"] for last in res[0][4]]
    assert kinds[3] == "compact" and kinds[4] == "delta", kinds
