"""GPU, multi-process: the PRODUCTION cross-GPU merge (csrc/gelly_group.cpp, gcc_forest_group_merge with nranks > 1)
driven by 2-3 fresh processes whose forests share cuda:0. ForestGroup bootstraps the communicator over a gloo process
group exactly as bench.py does over nccl; the collectives go through the shared-memory stand-in for librccl.so.1
(tests/cpp/shm_rccl.cpp, loaded through the product's GELLY_RCCL_LIB seam), because RCCL itself needs one GPU per rank
(the driver's 8-GPU run). Everything else — compact rounds, capacity repeats, agree(), failed-status headers, the
label fallback, the device forests, encode and absorb kernels — is the code bench.py --gpus N runs. Every window of
every rank is checked against the oracle (labels, or the full-size stream digests)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHM_RCCL = os.path.join(ROOT, "tests", "cpp", "build", "libshm_rccl.so")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_env(rank, port, env):
    os.environ.update(env or {})
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GELLY_RCCL_LIB=SHM_RCCL)


def worker(rank, world, port, cfg_args, starts, want, q, env):
    import sys

    _rank_env(rank, port, env)
    sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
    import torch
    import torch.distributed as dist

    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from gelly_stream import generators as G
        from gelly_stream.distributed import ForestGroup, TorchDisjointSet

        cfg = G.scaled(G.CONFIGS[cfg_args[0]], **cfg_args[1])
        E, V = cfg.info()
        d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
        G.generate_device(cfg, 0, E, d.data_ptr(), torch.cuda.current_stream().cuda_stream)
        f = TorchDisjointSet(V, 0)
        group = ForestGroup(device=0)
        lasts = []
        for w in range(len(starts) - 1):
            b, e = int(starts[w]), int(starts[w + 1])
            lo, hi = b + (e - b) * rank // world, b + (e - b) * (rank + 1) // world
            f.fold_device(d.data_ptr() + 8 * lo, hi - lo)
            group.merge_forest(f)
            lasts.append(dict(group.last))
            got = f.labels()
            if not np.array_equal(got, want[w]):
                q.put((rank, w, f"mismatch {group.last}", lasts))
                return
        group.close()
        dist.barrier()
        q.put((rank, -1, "ok", lasts))
    except Exception as ex:
        q.put((rank, -2, repr(ex), []))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_forest_group_ranks_share_one_gpu(world):
    """R-MAT, one dominant component: compact messages; the first window's list outgrows the initial capacity."""
    import oracle as orc
    from gelly_stream import generators as G

    cfg_args = ("c2_rmat20", {"scale": 16, "n_edges": 1 << 20})
    cfg = G.scaled(G.CONFIGS[cfg_args[0]], **cfg_args[1])
    E, V = cfg.info()
    starts = np.asarray([0, 777, 1 << 18, E], dtype=np.uint64)
    want = orc.cc_stream(G.generate_host(cfg), starts, V, partitions=2, threads=2, want_labels=True)["labels"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    tag = f"g{os.getpid()}_{port}"
    procs = [ctx.Process(target=worker, args=(r, world, port, cfg_args, starts, want, q, {"GELLY_SHM_RCCL_TAG": tag}))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=150) for _ in range(world)], key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=60)
    assert [r[:3] for r in res] == [(r, -1, "ok") for r in range(world)], res


def digest_worker(rank, world, port, fixture, env, q):
    """One rank of a fresh process group (spawned before any GPU call): folds its contiguous 1/world of every window
    of a full-size bench stream into a TorchDisjointSet on cuda:0, merges through ForestGroup (gcc_forest_group_merge
    over the stand-in) and checks every window's summary against the oracle's windowed digests
    (tests/golden/stream_digests.json). env FAIL_ABSORB_RANK / FAIL_ABSORB_AT: that rank's at-th absorb fails (tune key
    fail_absorb); it calls once more after its error, so its peers learn of it in-band."""
    import datetime
    import json
    import sys

    _rank_env(rank, port, env)
    sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
    import torch
    import torch.distributed as dist

    try:
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
        torch.cuda.set_device(0)
        from gelly_stream import generators as G
        from gelly_stream.distributed import ForestGroup, TorchDisjointSet
        from gelly_stream.native import GellyCCError

        fx = json.load(open(os.path.join(ROOT, "tests", "golden", "stream_digests.json")))[fixture]
        cfg = G.CONFIGS[fx["config"]]
        E, V = cfg.info()
        starts = [0] + [w["end"] for w in fx["windows"]]
        d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
        G.generate_device(cfg, 0, E, d.data_ptr(), torch.cuda.current_stream().cuda_stream)
        f = TorchDisjointSet(V, 0)
        failing = env.get("FAIL_ABSORB_RANK") == str(rank)
        if failing:
            f.ds.tune(fail_absorb=int(env["FAIL_ABSORB_AT"]))
        group = ForestGroup(device=0)
        lasts = []
        for w in range(len(starts) - 1):
            b, e = starts[w], starts[w + 1]
            lo, hi = b + (e - b) * rank // world, b + (e - b) * (rank + 1) // world
            f.fold_device(d.data_ptr() + 8 * lo, hi - lo)
            try:
                group.merge_forest(f)
            except GellyCCError as ex:
                if failing and w + 1 < len(starts) - 1:
                    try:
                        group.merge_forest(f)
                    except GellyCCError:
                        pass
                q.put((rank, w, "error: " + str(ex), lasts))
                return
            lasts.append(dict(group.last))
            dig, seen, comps = f.ds.label_digest()
            want = fx["windows"][w]
            if (str(dig), seen, comps) != (want["digest"], want["seen"], want["components"]):
                q.put((rank, w, f"window {w}: seen {seen} components {comps} digest mismatch, {group.last}", lasts))
                return
        group.close()
        dist.barrier()
        q.put((rank, -1, "ok", lasts))
    except Exception as ex:
        q.put((rank, -2, repr(ex), []))
    finally:
        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass


def _spawn(world, fixture, env=None, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    tag = f"g{os.getpid()}_{port}"
    env = dict(env or {}, GELLY_SHM_RCCL_TAG=tag)
    procs = [ctx.Process(target=digest_worker, args=(r, world, port, fixture, env, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in range(world):
            try:
                results.append(q.get(timeout=timeout))
            except Exception:
                break
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
        for f in os.listdir("/dev/shm"):
            if f.startswith(f"gshm_{tag}_"):
                os.unlink(os.path.join("/dev/shm", f))
    return sorted(results, key=lambda r: r[0])


def test_forest_group_c3_two_ranks_every_window():
    """C3 (G(n, m), 2^24 ids, 9.2M edges) split over 2 fresh ranks in 1M-edge windows, merged every
    window by the production loop, every window of both ranks against the oracle's digests. The first merge (nothing
    armed yet) takes the compact rounds, which overflow their speculative capacity (a repeat round); every later one
    the DELTA merge (round 6): at most 16 B per edge of the rank's window + the header, where rounds 4-5 all-gathered
    64 MiB label arrays per rank (C3 has no dominant component)."""
    res = _spawn(2, "c3_gnm24/w1M")
    assert [r[:3] for r in res] == [(0, -1, "ok"), (1, -1, "ok")], res
    lasts = res[0][3]
    assert lasts[0]["kind"] == "compact" and lasts[0]["rounds"] >= 2, lasts[0]  # a capacity repeat
    assert all(x["kind"] == "delta" for x in lasts[2:]), lasts
    for x in lasts[2:]:
        assert x["bytes"] <= 16 * (1 << 19) + 31, x  # 2^19 edges per rank per window


def test_forest_group_c5_delta_every_window():
    """C5 (2^24 ids, 256 windows of 2^16 edges: the short-window multi-GPU config) split over 2 fresh ranks: every
    merge after the first is the delta merge, <= 16 B per edge of the rank's window (+ header), and every window of
    both ranks matches the oracle's digests."""
    res = _spawn(2, "c5_adversarial/w64K", timeout=300)
    assert [r[:3] for r in res] == [(0, -1, "ok"), (1, -1, "ok")], res
    lasts = res[0][3]
    assert all(x["kind"] == "delta" and x["rounds"] == 1 for x in lasts[2:]), [x for x in lasts if x["kind"] != "delta"]
    assert max(x["bytes"] for x in lasts[2:]) <= 16 * (1 << 15) + 31, max(x["bytes"] for x in lasts[2:])


@pytest.mark.parametrize("at", [1, 2, 3])
def test_forest_group_absorb_failure_every_rank_errors(at):
    """Rank 1's at-th absorb fails inside the production merge (C3 x 2, 1M-edge windows: compact rounds, repeats and the
    label fallback all occur). Every rank returns an error — in the same merge (failed-status header / agree()), or,
    when the failure came after the merge's last collective, in the next one (the poisoned communicator) — and no rank
    hangs or reports success."""
    res = _spawn(2, "c3_gnm24/w1M", env={"FAIL_ABSORB_RANK": "1", "FAIL_ABSORB_AT": str(at),
                                         "GELLY_SHM_RCCL_TIMEOUT": "10"}, timeout=200)
    assert len(res) == 2 and all(r[2].startswith("error") for r in res), res
    assert "injected failure" in res[1][2], res
    assert res[0][1] in (res[1][1], res[1][1] + 1) and "rank 1 failed" in res[0][2], res


# ---- the group merge behind the C ABI (csrc/gelly_group.cpp) ----
def _windows_vs_oracle(cfg, starts, P, merge, knobs=None):
    import oracle as orc
    import torch
    from gelly_stream import DisjointSet
    from gelly_stream import generators as G

    E, V = cfg.info()
    want = orc.cc_stream(G.generate_host(cfg), starts, V, partitions=P, threads=2, want_labels=True)["labels"]
    d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
    G.generate_device(cfg, 0, E, d.data_ptr(), 0)
    torch.cuda.synchronize()
    forests = [DisjointSet(V) for _ in range(P)]
    for ds in forests:
        if knobs:
            ds.tune(**knobs)
    for w in range(len(starts) - 1):
        b, e = int(starts[w]), int(starts[w + 1])
        for r, ds in enumerate(forests):  # rank r folds its contiguous 1/P of the window (bench.py's partitioning)
            lo, hi = b + (e - b) * r // P, b + (e - b) * (r + 1) // P
            ds.fold_device(d.data_ptr() + 8 * lo, hi - lo)
        merge(forests)
        for r, ds in enumerate(forests):
            got = ds.labels()
            assert np.array_equal(got, want[w]), (w, r, int(np.flatnonzero(got != want[w])[0]))
    for ds in forests:
        ds.close()


@pytest.mark.parametrize("P", [2, 4, 8])
def test_c_abi_group_merge_one_device(P):
    """gcc_group_merge over P forests on one GPU: the compact message all-gather through one device buffer, each
    forest absorbing the others (the RCCL path's protocol without the transport). R-MAT: one dominant component."""
    from gelly_stream import generators as G
    from gelly_stream.distributed import group_merge

    cfg = G.scaled(G.CONFIGS["c2_rmat20"], scale=17, n_edges=1 << 20, seed=0x6770)
    starts = np.asarray([0, 1000, 1 << 17, 1 << 19, 1 << 20], dtype=np.uint64)
    _windows_vs_oracle(cfg, starts, P, group_merge)


def test_c_abi_group_merge_unfiltered_forests():
    """Forests without the giant filter are encoded straight from their parent pointers (msg_count_kernel<true>:
    read-only finds, no compress first) and absorb without deferred ids."""
    from gelly_stream import generators as G
    from gelly_stream.distributed import group_merge

    cfg = G.scaled(G.CONFIGS["c2_rmat20"], scale=17, n_edges=1 << 19, seed=0x6771)
    starts = np.asarray([0, 1000, 1 << 17, 1 << 19], dtype=np.uint64)
    _windows_vs_oracle(cfg, starts, 3, group_merge, knobs={"filter": 0})


def test_c_abi_group_merge_retry_and_label_fallback():
    """G(n, m) near the threshold: no dominant component, so the lists overflow the speculative capacity (a repeat
    round, exact because union is idempotent) until the compact form stops paying and labels are exchanged."""
    from gelly_stream import generators as G
    from gelly_stream.distributed import group_merge

    cfg = G.scaled(G.CONFIGS["c3_gnm24"], n_vertices=1 << 18, n_edges=1 << 17, seed=0x3131)
    starts = np.asarray([0, 1 << 10, 1 << 15, 1 << 17], dtype=np.uint64)
    _windows_vs_oracle(cfg, starts, 3, group_merge)


def test_rccl_comm_single_rank():
    """The RCCL transport loads (dlopen librccl.so.1, shared with torch's) and a 1-rank communicator merges (=
    compresses); gcc_forest_group_merge checks the forest's device against the communicator's."""
    from gelly_stream import DisjointSet
    from gelly_stream.distributed import RcclComm

    comm = RcclComm(0, 1, 0, RcclComm.unique_id())
    ds = DisjointSet(1 << 12)
    ds.fold(np.array([[5, 6], [6, 9], [100, 101]], dtype=np.uint32))
    assert ds.find(9) == 5  # caches the host labels
    comm.merge(ds)
    assert ds._labels_cache is None  # RcclComm.merge drops the pre-merge view itself
    assert ds.find(9) == 5 and ds.find(101) == 100 and ds.size() == 5
    ds.close()
    comm.close()


def test_c_abi_group_merge_two_devices():
    """Two forests on two GPUs merged through gcc_comm_init_all + gcc_group_merge (RCCL): needs >= 2 GPUs."""
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (the driver's multi-GPU node)")
    import oracle as orc
    from gelly_stream import DisjointSet
    from gelly_stream import generators as G
    from gelly_stream.distributed import RcclComm, group_merge

    cfg = G.scaled(G.CONFIGS["c2_rmat20"], scale=16, n_edges=1 << 19)
    E, V = cfg.info()
    pairs = G.generate_host(cfg)
    want = orc.cc_stream(pairs, [0, E], V, want_labels=True)["labels"][0]
    comms = RcclComm.init_all([0, 1])
    a, b = DisjointSet(V, 0), DisjointSet(V, 1)
    a.fold(pairs[: E // 2])
    b.fold(pairs[E // 2:])
    group_merge([a, b], comms)
    assert np.array_equal(a.labels(), want) and np.array_equal(b.labels(), want)
    # and DisjointSet.merge across the two devices (CombineCC with a peer copy)
    c = DisjointSet(V, 1)
    c.merge(a)
    assert np.array_equal(c.labels(), want)
    for x in (a, b, c):
        x.close()
    for x in comms:
        x.close()


def test_group_merge_deferred_new_ids():
    """The absorb defers the new ids of overlapping peer giants to its compress (gcc_forest_absorb_many). Ids that
    another peer's LONE giant or a peer's (v, label) list also touches become seen before that compress and must
    still join the tracked component. Four hand-made forests over 2^17 ids (giant filter on), every forest against
    the oracle's partition of all edges: A's giant [1000, 60000); B's [50000, 110000) overlaps it; C's
    [110000, 131000) + 70000 does not overlap A but holds one of B's ids; D's giant [200, 900) is lone everywhere and
    its small components {65000, 130500} and {100, 64000} pair ids of B's and C's giants with new ones."""
    import oracle as orc
    from gelly_stream import DisjointSet
    from gelly_stream.distributed import group_merge

    V = 1 << 17

    def path(ids):
        ids = np.asarray(ids, dtype=np.uint32)
        return np.stack([ids[:-1], ids[1:]], axis=1)

    parts = [
        path(np.arange(1000, 60000)),
        path(np.arange(50000, 110000)),
        np.concatenate([path(np.arange(110000, 131000)), np.asarray([[110000, 70000]], dtype=np.uint32)]),
        np.concatenate([path(np.arange(200, 900)), np.asarray([[65000, 130500], [100, 64000]], dtype=np.uint32)]),
    ]
    allp = np.ascontiguousarray(np.concatenate(parts))
    want = orc.cc_stream(allp, [0, len(allp)], V, partitions=1, want_labels=True)["labels"][0]
    forests = [DisjointSet(V) for _ in parts]
    try:
        for ds, p in zip(forests, parts):
            ds.fold(np.ascontiguousarray(p))
            ds.compress()  # elects and tracks each forest's giant
        group_merge(forests)
        for r, ds in enumerate(forests):
            got = ds.labels()
            assert np.array_equal(got, want), (r, int(np.flatnonzero(got != want)[0]))
    finally:
        for ds in forests:
            ds.close()


def test_merge_labels_rejects_out_of_range_labels():
    """A received label array is untrusted input (gcc_forest_merge_labels_device): a label >= id_capacity is skipped
    (never dereferenced) and reported once by the next synchronising call; the other labels are merged."""
    import torch

    from gelly_stream import DisjointSet
    from gelly_stream.native import GellyCCError

    V = 1 << 16
    lab = np.full(V, 0xFFFFFFFF, dtype=np.uint32)
    lab[10:20] = 10          # {10..19}
    lab[30] = V + 7          # out of range
    lab[31] = 0xFFFFFFF0     # out of range
    d = torch.from_numpy(lab.view(np.int32)).cuda()
    with DisjointSet(V) as ds:
        ds.merge_labels_device(d.data_ptr(), V)
        with pytest.raises(GellyCCError, match="id_capacity"):
            ds.labels()
        got = ds.labels()
        want = np.full(V, 0xFFFFFFFF, dtype=np.uint32)
        want[10:20] = 10
        assert np.array_equal(got, want)
