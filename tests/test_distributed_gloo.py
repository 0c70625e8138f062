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
    """ExchangeForest over the CPU oracle: labels travel as an int32 CPU tensor, merge messages as uint8 CPU
    tensors in the include/gelly_cc.h layout (restated here in numpy: the device encoder's CPU twin)."""

    def __init__(self, V):
        import oracle as orc

        self.V = V
        self.id_capacity = V
        self.ds = orc.OracleDisjointSet()
        self.buf = torch.empty(V, dtype=torch.int32)

    def new_bytes(self, n):
        return torch.zeros(int(n), dtype=torch.uint8)

    def encode(self, msg, cap_others):
        self.compress()
        lab = self.buf.numpy().view(np.uint32)
        seen = lab != UNSEEN
        vals, cnt = np.unique(lab[seen], return_counts=True)
        g = int(vals[np.argmax(cnt)]) if vals.size else UNSEEN
        nw = (self.V + 63) // 64
        bits = np.zeros(nw * 64, dtype=bool)
        bits[: self.V] = seen & (lab == g)
        oth = np.flatnonzero(seen & (lab != g)).astype(np.uint32)
        m = msg.numpy()
        m[:16] = np.frombuffer(np.array([g, oth.size, self.V, 0], dtype="<u4").tobytes(), dtype=np.uint8)
        m[16:16 + nw * 8] = np.packbits(bits, bitorder="little")
        k = min(oth.size, int(cap_others))
        pairs = np.stack([oth[:k], lab[oth[:k]]], axis=1).astype("<u4").reshape(-1)
        o = 16 + nw * 8
        m[o:o + 8 * k] = np.frombuffer(pairs.tobytes(), dtype=np.uint8)

    def absorb_msgs(self, msgs, stride, count, skip, cap_others):
        for p in range(count):
            if p != skip:
                self.absorb_msg(msgs[p * stride:(p + 1) * stride], cap_others)

    def absorb_msg(self, msg, cap_others):
        m = msg.numpy()
        g, n_oth, n, _ = np.frombuffer(m[:16].tobytes(), dtype="<u4")
        assert n == self.V, "message of another id range"
        nw = (self.V + 63) // 64
        bits = np.unpackbits(m[16:16 + nw * 8], bitorder="little")[: self.V]
        for v in np.flatnonzero(bits):
            self.ds.union(int(v), int(g))
        k = min(int(n_oth), int(cap_others))
        o = 16 + nw * 8
        pairs = np.frombuffer(m[o:o + 8 * k].tobytes(), dtype="<u4").reshape(-1, 2)
        for v, l in pairs:
            self.ds.union(int(v), int(l))

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


def worker(rank, world, port, V, pairs, starts, want, q, mode="auto", cap=0, expect_compact=None):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from gelly_stream.distributed import ForestGroup

        group = ForestGroup(mode=mode)
        group._cap = cap  # 0: the default initial list capacity
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
            if expect_compact is not None and bool(group.last.get("compact")) != expect_compact:
                q.put((rank, w, f"compact={group.last.get('compact')}"))
                return
            if w == 0 and cap and expect_compact and group.last.get("rounds", 0) < 2:
                q.put((rank, w, f"no repair round with cap {cap}: {group.last}"))
                return
        dist.barrier()
        q.put((rank, -1, "ok"))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, -2, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_world(world, V, pairs, starts, want, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, V, pairs, starts, want, q), kwargs=kw)
             for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert sorted(results) == [(r, -1, "ok") for r in range(world)], results


def rmat_case():
    import oracle as orc
    from gelly_stream import generators as G

    cfg = G.scaled(G.CONFIGS["c2_rmat20"], scale=9, n_edges=3000)
    pairs = G.generate_host(cfg)
    _, V = cfg.info()
    starts = np.array([0, 700, 701, 1800, 3000], dtype=np.uint64)
    want = orc.cc_stream(pairs, starts, V, want_labels=True)["labels"]
    return V, pairs, starts, want


@pytest.mark.parametrize("world", [2, 3, 4])
def test_compact_merge_gives_global_partition_every_window(world):
    """Default protocol: compact messages (giant bitmap + others list) in one all_gather; the first window's
    list outgrows a 16-entry start capacity, so the re-encode path runs too."""
    V, pairs, starts, want = rmat_case()
    run_world(world, V, pairs, starts, want, mode="auto", cap=16, expect_compact=True)


@pytest.mark.parametrize("world", [2, 4])
def test_label_merge_fallback_when_no_component_dominates(world):
    """A stream of disjoint pairs: the compact form is larger than the label array, so labels are exchanged."""
    import oracle as orc

    V = 4096
    ids = np.random.default_rng(7).permutation(V).astype(np.uint32)
    matching = ids.reshape(-1, 2)
    pairs = np.concatenate([matching, matching, matching[:100]])  # every rank sees >= half the ids, in pairs
    starts = np.array([0, 2 * len(matching), len(pairs)], dtype=np.uint64)
    want = orc.cc_stream(pairs, starts, V, want_labels=True)["labels"]
    run_world(world, V, pairs, starts, want, mode="auto", expect_compact=False)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_label_merge_gives_global_partition_every_window(world):
    """mode "labels": butterfly of label arrays (power-of-two worlds) or all_gather (world 3)."""
    V, pairs, starts, want = rmat_case()
    run_world(world, V, pairs, starts, want, mode="labels")
