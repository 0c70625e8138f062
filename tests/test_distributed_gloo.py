"""CPU, multi-process: the cross-rank forest merge protocol (distributed.ForestGroup) over gloo.

Each rank folds its contiguous chunk of every window into a forest; ForestGroup.merge_forest must leave
every rank with the global partition after every window — the reference's timeWindowAll(...).reduce(CombineCC)
+ parallelism-1 Merger (SummaryBulkAggregation.java:81-83). On CPU the per-rank forest is the oracle
(test infrastructure); on GPUs the same protocol drives TorchDisjointSet over RCCL.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

UNSEEN = 0xFFFFFFFF


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class OracleForest:
    """ExchangeForest over the CPU oracle: labels travel as an int32 CPU tensor."""

    def __init__(self, V):
        import oracle as orc

        self.V = V
        self.ds = orc.OracleDisjointSet()
        self.buf = torch.empty(V, dtype=torch.int32)

    def fold(self, pairs):
        for u, v in pairs:
            self.ds.union(int(u), int(v))

    def compress(self):
        self.buf.copy_(torch.from_numpy(self.ds.labels(self.V).view(np.int32)))

    def exchange_tensor(self):
        return self.buf

    def absorb(self, labels):
        lab = labels.numpy().view(np.uint32)
        for v in np.flatnonzero(lab != UNSEEN):
            self.ds.union(int(v), int(lab[v]))

    def labels(self):
        return self.ds.labels(self.V)


def worker(rank, world, port, V, pairs, starts, want, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from gelly_stream.distributed import ForestGroup

        group = ForestGroup()
        f = OracleForest(V)
        for w in range(len(starts) - 1):
            b, e = int(starts[w]), int(starts[w + 1])
            L = e - b
            f.fold(pairs[b + L * rank // world: b + L * (rank + 1) // world])
            group.merge_forest(f)
            got = f.exchange_tensor().numpy().view(np.uint32)
            if not np.array_equal(got, want[w]):
                q.put((rank, w, "mismatch"))
                return
        dist.barrier()
        q.put((rank, -1, "ok"))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, -2, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_butterfly_merge_gives_global_partition_every_window(world):
    import oracle as orc
    from gelly_stream import generators as G

    cfg = G.scaled(G.CONFIGS["c2_rmat20"], scale=9, n_edges=3000)
    pairs = G.generate_host(cfg)
    _, V = cfg.info()
    starts = np.array([0, 700, 701, 1800, 3000], dtype=np.uint64)
    want = orc.cc_stream(pairs, starts, V, want_labels=True)["labels"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, V, pairs, starts, want, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert sorted(results) == [(r, -1, "ok") for r in range(world)], results
