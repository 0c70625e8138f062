"""GPU, multi-process: ForestGroup over TorchDisjointSet (device forests, device messages, pinned header copies)
with 2-3 ranks sharing cuda:0 over gloo — the whole N>1 merge path of bench.py except the RCCL transport, which
needs one GPU per rank (the driver's 8-GPU run). Every window vs the oracle's global partition."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def worker(rank, world, port, cfg_args, starts, want, mode, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "gelly-streaming_amd")]
    import torch
    import torch.distributed as dist

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from gelly_stream import generators as G
        from gelly_stream.distributed import ForestGroup, TorchDisjointSet

        cfg = G.scaled(G.CONFIGS[cfg_args[0]], **cfg_args[1])
        E, V = cfg.info()
        d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
        G.generate_device(cfg, 0, E, d.data_ptr(), torch.cuda.current_stream().cuda_stream)
        f = TorchDisjointSet(V, 0)
        group = ForestGroup(mode=mode)
        for w in range(len(starts) - 1):
            b, e = int(starts[w]), int(starts[w + 1])
            lo, hi = b + (e - b) * rank // world, b + (e - b) * (rank + 1) // world
            f.fold_device(d.data_ptr() + 8 * lo, hi - lo)
            group.merge_forest(f)
            got = f.labels()
            if not np.array_equal(got, want[w]):
                q.put((rank, w, f"mismatch {group.last}"))
                return
        dist.barrier()
        q.put((rank, -1, "ok"))
    except Exception as ex:
        q.put((rank, -2, repr(ex)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


# mode "labels" at world 3 takes the all_gather fallback: gloo's send/recv on CUDA tensors is not ordered with
# the CUDA stream (RCCL's is), so the butterfly's P2P rounds are covered by the CPU gloo tests instead.
@pytest.mark.parametrize("mode,world", [("auto", 2), ("auto", 3), ("labels", 3)])
def test_forest_group_ranks_share_one_gpu(mode, world):
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
    procs = [ctx.Process(target=worker, args=(r, world, port, cfg_args, starts, want, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=150) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert sorted(results) == [(r, -1, "ok") for r in range(world)], results
