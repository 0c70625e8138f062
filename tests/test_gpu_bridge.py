"""The Java bridge's exact C-ABI call sequences, replayed through ctypes.

gelly-streaming_amd/java/.../GpuDisjointSet.java cannot be compiled here (no JDK), so `BridgeReplay` below
performs, call for call, what that class and its JNI glue (java/jni/gcc_jni.c) perform:

* direct ids: ``Gcc.staging`` (gcc_forest_staging) hands out the pinned slot, ``union`` writes (u32, u32) pairs
  into it, a full slot or any read ``Gcc.submit``s it (gcc_forest_submit; the library switches slots);
* Long ids: pairs collect in a long[]; ``Gcc.submitLong`` = gcc_forest_staging + gcc_idmap_map straight into the
  slot + gcc_forest_submit; ``find`` = gcc_idmap_lookup + gcc_forest_labels + gcc_idmap_canonical;
* reads: ``getMatches().size()`` = gcc_forest_size, labels, ``merge`` = gcc_forest_merge (direct) or the other
  dictionary's (original id, canonical id) pairs (Long ids), serialisation = gcc_forest_serialize (+ the id list
  for Long ids) and the lazy restore = gcc_forest_deserialize.

Every checkpoint is compared with the oracle (oracle/cc_oracle.c: DisjointSet.java's union-by-rank restated) over
all edges submitted so far. Reference: …/summaries/DisjointSet.java:30-154, …/library/ConnectedComponents.java:83-86.
"""
import ctypes
import struct
from ctypes import byref, c_uint64, c_void_p

import numpy as np
import pytest

import oracle as orc
from gelly_stream import DisjointSet
from gelly_stream import generators as G
from gelly_stream.longids import IdDictionary as IdMap
from gelly_stream.native import call

pytestmark = pytest.mark.gpu
UNSEEN = 0xFFFFFFFF
I64_MIN = -(1 << 63)


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    return torch


class BridgeReplay:
    """GpuDisjointSet's native call sequence (one instance = one Java object on a task thread)."""

    def __init__(self, id_capacity, long_ids=False, device=0):
        self.cap, self.long_ids = int(id_capacity), bool(long_ids)
        self.ds = DisjointSet(self.cap, device)  # gcc_forest_create (Gcc.create)
        self.idmap = IdMap(self.cap) if long_ids else None  # gcc_idmap_create (Gcc.idmapCreate)
        self.staged = 0
        self.slot = None  # (pointer, capacity in pairs) of the current staging slot
        self.pend = []    # Long ids: pending pairs (Java's long[] pend)
        self.submits = 0

    def _staging(self):
        p, n = c_void_p(), c_uint64()
        call("gcc_forest_staging", self.ds.handle, byref(p), byref(n))
        return p.value, n.value

    def union_batch(self, pairs):
        """A run of per-edge union() calls: each pair is written into the slot; a full slot is submitted."""
        pairs = np.asarray(pairs)
        i = 0
        while i < len(pairs):
            if self.long_ids:
                if self.slot is None:
                    self.slot = (None, self._staging()[1])
                room = self.slot[1] - self.staged
                take = pairs[i:i + room]
                self.pend.append(np.asarray(take, dtype=np.int64))
            else:
                if self.slot is None:
                    self.slot = self._staging()
                ptr, cap = self.slot
                room = cap - self.staged
                take = np.ascontiguousarray(pairs[i:i + room], dtype=np.uint32)
                ctypes.memmove(ptr + 8 * self.staged, take.ctypes.data, take.nbytes)  # stage.putInt x 2
            self.staged += len(take)
            i += len(take)
            if self.staged == self.slot[1]:
                self.submit()

    def submit(self):
        if self.staged == 0:
            return
        if self.long_ids:  # Gcc.submitLong: staging -> gcc_idmap_map into the slot -> submit
            ptr, cap = self._staging()
            ids = np.concatenate(self.pend).reshape(-1)
            assert ids.size == 2 * self.staged <= 2 * cap
            dense = (ctypes.c_uint32 * ids.size).from_address(ptr)
            call("gcc_idmap_map", self.idmap._h, ids.ctypes.data, ids.size, ctypes.addressof(dense))
            self.pend = []
        call("gcc_forest_submit", self.ds.handle, self.staged)
        self.staged = 0
        self.slot = None  # the library switched slots: Java re-fetches the buffer
        self.submits += 1
        self.ds._dirty()

    # ---- reads (each submits first, as in GpuDisjointSet) ----
    def size(self):
        self.submit()
        n = c_uint64()
        call("gcc_forest_size", self.ds.handle, byref(n))
        return n.value

    def labels(self):
        self.submit()
        return self.ds.labels()

    def canonical(self):
        """Long ids: (original id per dense id, canonical id per dense id) = Gcc.idmapIds, Gcc.canonical."""
        self.submit()
        ids = self.idmap.ids()
        lab = np.empty(ids.size, dtype=np.uint32)
        call("gcc_forest_labels", self.ds.handle, lab.ctypes.data, ids.size)
        return ids, self.idmap.canonical(lab, unseen=I64_MIN)

    def find(self, e):
        if self.long_ids:
            self.submit()
            d = self.idmap.lookup(e)
            return None if d is None else int(self.canonical()[1][d])
        if not 0 <= e < self.cap:
            return None
        r = int(self.labels()[e])
        return None if r == UNSEEN else r

    def merge(self, other):
        if not self.long_ids and not other.long_ids:
            other.submit()
            self.submit()
            self.ds.merge(other.ds)  # gcc_forest_merge
        elif other.long_ids:
            ids, can = other.canonical()
            self.union_batch(np.stack([ids, can], axis=1))
        else:
            lab = other.labels()
            seen = np.flatnonzero(lab != UNSEEN)
            self.union_batch(np.stack([seen, lab[seen]], axis=1))

    def state(self):
        """GpuDisjointSet.state(): the serialized summary (Long ids: [int n][n longs][summary])."""
        self.submit()
        forest = self.ds.serialize()
        if not self.long_ids:
            return forest
        ids = self.idmap.ids().astype("<i8")
        return struct.pack("<i", ids.size) + ids.tobytes() + forest

    @classmethod
    def restored(cls, data, id_capacity, long_ids=False):
        """readObject / Kryo read + the lazy h(): a fresh handle, then restore(pendingState)."""
        r = cls(id_capacity, long_ids)
        if not long_ids:
            r.ds.deserialize(data)
            return r
        (n,) = struct.unpack_from("<i", data, 0)
        ids = np.frombuffer(data, dtype="<i8", count=n, offset=4)
        r.union_batch(np.stack([ids, ids], axis=1))  # dense ids 0..n-1 in the recorded order
        r.submit()
        r.ds.deserialize(data[4 + 8 * n:])
        return r

    def close(self):
        self.ds.close()
        if self.idmap is not None:
            self.idmap.close()


def oracle_labels(pairs, cuts, V):
    """Labels after each prefix pairs[:cut] (the oracle's windows = the checkpoints)."""
    starts = np.asarray([0] + list(cuts), dtype=np.uint64)
    return orc.cc_stream(np.ascontiguousarray(pairs, dtype=np.uint32), starts, V, partitions=1,
                         want_labels=True, want_digest=False)["labels"]


def test_bridge_direct_ids_call_sequence(torch_cuda):
    """Direct ids: > 3 staging-slot switches, with size / labels / find / serialize->restore / merge interleaved
    between the submits, every checkpoint against the oracle (the restored copy keeps folding too)."""
    cfg = G.CONFIGS["c2_rmat20"]
    E, V = cfg.info()
    pairs = G.generate_host(cfg, 0, 3_700_000)
    other = G.generate_host(G.CONFIGS["c3_gnm24"], 0, 400_000) % np.uint32(V)
    cuts = [300_001, 1_100_003, 2_000_000, 2_900_017, len(pairs)]
    want = oracle_labels(pairs, cuts, V)
    b = BridgeReplay(V)
    copy = None
    lo = 0
    for k, hi in enumerate(cuts):
        b.union_batch(pairs[lo:hi])
        if copy is not None:
            copy.union_batch(pairs[lo:hi])
        lo = hi
        w = want[k]
        if k == 0:  # CombineCC reads getMatches().size() only
            assert b.size() == int(np.count_nonzero(w != UNSEEN))
        elif k == 1:  # a Kryo copy of the accumulator: serialize, restore lazily, keep folding both
            data = b.state()
            copy = BridgeReplay.restored(data, V)
            assert np.array_equal(copy.labels(), w)
        elif k == 2:  # FlattenSet: find() per key
            seen = np.flatnonzero(w != UNSEEN)[:2000]
            assert all(b.find(int(v)) == int(w[v]) for v in seen)
            assert b.find(V + 5) is None
        assert np.array_equal(b.labels(), w), k
    assert np.array_equal(copy.labels(), want[-1])
    assert b.submits >= 4
    # merge (smaller into larger, as CombineCC.reduce): a second forest over other edges
    o = BridgeReplay(V)
    o.union_batch(other)
    b.merge(o)
    both = np.concatenate([pairs, other])
    assert np.array_equal(b.labels(), oracle_labels(both, [len(both)], V)[-1])
    for r in (b, o, copy):
        r.close()


def _long_oracle(pairs_l, cuts):
    """Oracle over Long ids: dense ids in SIGNED order (np.unique sorts), so the dense minimum is the Long minimum."""
    uniq, inv = np.unique(pairs_l.reshape(-1), return_inverse=True)
    dense = inv.reshape(-1, 2).astype(np.uint32)
    return uniq, dense, oracle_labels(dense, cuts, uniq.size)


def test_bridge_long_ids_call_sequence(torch_cuda):
    """Long ids (any Long, incl. negative and the extremes): submitLong across slot switches, find, getMatches
    entries, toString-level grouping, serialize -> restore -> keep folding, and a merge of two dictionaries."""
    rng = np.random.default_rng(0x10A6)
    n_ids = 1_500_000
    pool = rng.integers(I64_MIN, (1 << 63) - 1, size=n_ids, dtype=np.int64, endpoint=True)
    pool[:4] = [I64_MIN, (1 << 63) - 1, -1, 0]
    E = 2_600_000
    # a random graph just above the percolation threshold over the pool (a giant + many small components)
    pairs_l = pool[rng.integers(0, n_ids, size=(E, 2))]
    pairs_l[:3] = [[pool[0], pool[1]], [pool[1], pool[2]], [pool[3], pool[3]]]
    cuts = [1_000_003, 1_800_000, E]
    uniq, dense, want = _long_oracle(pairs_l, cuts)
    cap = 1 << 21
    b = BridgeReplay(cap, long_ids=True)
    copy = None
    lo = 0

    def check(r, w, hi):
        ids, can = r.canonical()
        pos = np.searchsorted(uniq, ids)
        assert np.array_equal(uniq[pos], ids)
        # the oracle's canonical label is a dense (sorted) id: back to the Long it stands for
        assert np.array_equal(can, uniq[w[pos]])
        assert ids.size == np.unique(pairs_l[:hi].reshape(-1)).size == r.size()

    for k, hi in enumerate(cuts):
        b.union_batch(pairs_l[lo:hi])
        if copy is not None:
            copy.union_batch(pairs_l[lo:hi])
        lo = hi
        check(b, want[k], hi)
        if k == 0:
            copy = BridgeReplay.restored(b.state(), cap, long_ids=True)
            check(copy, want[k], hi)
            for x in pool[:4]:  # find = the minimum Long of x's component (the extremes included)
                assert b.find(int(x)) == int(uniq[want[k][np.searchsorted(uniq, x)]]), int(x)
            assert b.find(int(pool[0]) + 1) is None or int(pool[0]) + 1 in uniq  # never seen (DisjointSet.find :72-74)
    check(copy, want[-1], E)
    assert b.submits >= 3
    # CombineCC of two Long-id summaries (different dictionaries): the other's (id, canonical) pairs
    extra = pool[rng.integers(0, n_ids, size=(300_000, 2))]
    o = BridgeReplay(cap, long_ids=True)
    o.union_batch(extra)
    b.merge(o)
    allp = np.concatenate([pairs_l, extra])
    uniq2, _, want2 = _long_oracle(allp, [len(allp)])
    ids, can = b.canonical()
    pos = np.searchsorted(uniq2, ids)
    assert np.array_equal(uniq2[pos], ids) and ids.size == uniq2.size
    assert np.array_equal(can, uniq2[want2[-1][pos]])
    for r in (b, o, copy):
        r.close()
