"""BipartitenessCheck and its Candidates summary on an MI355X (mirror of …/library/BipartitenessCheck.java and
…/summaries/Candidates.java; `…/` = src/main/java/org/apache/flink/graph/streaming/).

Reference:
  BipartitenessCheck(long mergeWindowTime)   BipartitenessCheck.java:50-52
      = SummaryBulkAggregation(new updateFunction(), new combineFunction(), new Candidates(true), t, false)
  edgeToCandidate(v1, v2)                    :54-61   component min(v1,v2): {min: +, max: -}
  updateFunction.foldEdges(c, v1, v2, ev)    :93-95   c.merge(edgeToCandidate(v1, v2))
  combineFunction.reduce(c1, c2)             :128-130 c1.merge(c2)
  Candidates = (success, TreeMap<component, Map<vertex, SignedVertex>>)   Candidates.java:27-197
      merge: components that share a vertex are joined, the input side's signs reversed to match; a sign
      conflict (an odd cycle) turns the result into fail() = (false, {}) for good (:78-81, :118-121, :194-196)

Here the state is one device-resident signed forest (csrc/gelly_bip.hip): per vertex (parent, parity). The
observable output is canonical: each component keyed by its minimum vertex, every sign relative to that vertex
(the minimum is `true`). Signs in the reference depend on merge order (the input side is the one reversed), but
within a component they always agree with ours up to one flip; toString() equals the reference's output whenever
the reference's minimum vertex carries `true` (as in its own BipartitenessCheckTest). A self loop (v, v) only adds
v, as in the reference (edgeToCandidate ignores add()'s false, :58-59). Where the reference's Candidates.merge is
not a partition join, this summary keeps the intended semantics (bipartite iff no odd cycle) and differs from it:
  * _merge files the input's vertices under min(inputKey, selfKey) without moving the self component
    (Candidates.java:176-189): the reference can emit overlapping or split "components";
  * a failed second-level merge is dropped (:128-131 call fail() without returning it): an odd cycle closed across
    two merged summaries can be reported as success;
  * components with identical vertex sets are skipped (:92-95): two partitions over {1,2,3} holding the paths 1-2-3
    and 1-3-2 form a triangle, which the reference reports as bipartite.
Every such window of the fixtures is pinned (tests/test_bipartite_oracle.py DIVERGENT, checked on the GPU by
tests/test_gpu_bipartite.py); DESIGN.md §7.
"""
from __future__ import annotations

from collections.abc import Mapping
from ctypes import byref, c_int, c_uint64, c_void_p
from typing import Iterator, NamedTuple, Optional

import numpy as np

from .aggregation import EdgeBatch, EdgesFold, ReduceFunction, SummaryBulkAggregation
from .native import UNSEEN, call


class SignedVertex(NamedTuple):
    """SignedVertex = Tuple2<Long, Boolean> (…/util/SignedVertex.java:23-41)."""

    vertex: int
    sign: bool

    def getVertex(self) -> int:
        return self.vertex

    def getSign(self) -> bool:
        return self.sign

    def reverse(self) -> "SignedVertex":
        return SignedVertex(self.vertex, not self.sign)

    def __str__(self) -> str:  # Flink Tuple2.toString
        return f"({self.vertex},{'true' if self.sign else 'false'})"


class Candidates:
    """Candidates backed by a device signed forest (Candidates.java:27-197)."""

    def __init__(self, id_capacity: int, device: int = 0, success: bool = True):
        """``new Candidates(true)`` (:31-34). success=False builds the failed value (fail(), :194-196)."""
        self.id_capacity = int(id_capacity)
        self.device = int(device)
        h = c_void_p()
        call("gcc_signed_create", self.device, self.id_capacity, byref(h))
        self._h = h
        self._words: Optional[np.ndarray] = None
        self._failed_by_ctor = not success

    # ---- lifetime ----
    def close(self) -> None:
        if getattr(self, "_h", None):
            call("gcc_signed_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> c_void_p:
        if not self._h:
            raise ValueError("Candidates is closed")
        return self._h

    def _dirty(self) -> None:
        self._words = None

    # ---- Candidates.java surface ----
    def getSuccess(self) -> bool:
        """:44-46"""
        if self._failed_by_ctor:
            return False
        ok = c_int()
        call("gcc_signed_success", self.handle, byref(ok))
        return bool(ok.value)

    def getMap(self) -> dict[int, dict[int, SignedVertex]]:
        """:48-50 — TreeMap component -> (TreeMap vertex -> SignedVertex); empty once failed (fail() = (false, {}))."""
        if not self.getSuccess():
            return {}
        w = self.words()
        seen = np.flatnonzero(w != UNSEEN)
        out: dict[int, dict[int, SignedVertex]] = {}
        for v in seen.tolist():
            c, q = int(w[v]) >> 1, int(w[v]) & 1
            out.setdefault(c, {})[v] = SignedVertex(v, q == 0)
        return dict(sorted((c, dict(sorted(m.items()))) for c, m in out.items()))

    def merge(self, other: "Candidates") -> "Candidates":
        """:77-139 — self := self ∪ other (signs joined through shared vertices); returns self."""
        if other._failed_by_ctor:
            self._failed_by_ctor = True
        call("gcc_signed_merge", self.handle, other.handle)
        self._dirty()
        return self

    def toString(self) -> str:
        """Flink Tuple2.toString of (success, TreeMap): e.g. ``(true,{1={1=(1,true), 2=(2,false)}})``."""
        if not self.getSuccess():
            return "(false,{})"
        comps = ", ".join(f"{c}={{" + ", ".join(f"{v}={sv}" for v, sv in m.items()) + "}"
                          for c, m in self.getMap().items())
        return "(true,{" + comps + "})"

    def __str__(self) -> str:
        return self.toString()

    # ---- batch / device extensions ----
    def fold(self, pairs: np.ndarray) -> None:
        """Fold host edges ((n, 2) u32): updateFunction.foldEdges over a whole batch."""
        a = np.ascontiguousarray(pairs, dtype=np.uint32).reshape(-1)
        call("gcc_signed_fold_host", self.handle, a.ctypes.data, a.size // 2)
        self._dirty()

    def fold_device(self, d_pairs: int, n_edges: int) -> None:
        call("gcc_signed_fold_device", self.handle, c_void_p(d_pairs), int(n_edges))
        self._dirty()

    def reset(self) -> None:
        call("gcc_signed_reset", self.handle)
        self._failed_by_ctor = False
        self._dirty()

    def set_stream(self, hip_stream: Optional[int]) -> None:
        call("gcc_signed_set_stream", self.handle, c_void_p(hip_stream or 0), 1 if hip_stream is None else 0)

    def tune(self, **knobs) -> "Candidates":
        """Speed-only knobs of the signed fold (gcc_signed_tune): giant, sample_shift, min_share, unroll, xcd, xcd_min,
        bucket (the bucketed fold: id ranges up to 2^27), bucket_min, bucket_levels, bucket_items."""
        for k, v in knobs.items():
            call("gcc_signed_tune", self.handle, k.encode(), float(v))
        return self

    def merge_words(self, d_words: int, n: int, other_failed: bool = False) -> "Candidates":
        """self ∪= the signed partition in another forest's device words d_words[0, n) (gcc_signed_merge_words)."""
        call("gcc_signed_merge_words", self.handle, c_void_p(d_words), int(n), 1 if other_failed else 0)
        self._dirty()
        return self

    def compress(self) -> None:
        """The emission on the device (canonical words in place; asynchronous): what words() copies out."""
        call("gcc_signed_compress", self.handle)

    def device_words_tensor(self):
        """The canonical words as a torch int32 tensor on this forest's device, copied from the forest's own device
        buffer (gcc_signed_device_words after a compress; no trip through the host): the send side of merge_group."""
        import torch

        self.compress()
        p = c_void_p()
        call("gcc_signed_device_words", self.handle, byref(p))
        self.getSuccess()  # synchronises the forest's stream: the compress has written the words

        class _View:  # __cuda_array_interface__ over the forest's buffer (copied at once: valid until its next mutation)
            __cuda_array_interface__ = {"shape": (self.id_capacity,), "typestr": "<i4", "data": (p.value, False),
                                        "version": 2, "strides": None}

        with torch.cuda.device(self.device):
            return torch.as_tensor(_View(), device=f"cuda:{self.device}").clone()

    def words(self) -> np.ndarray:
        """Canonical words: (component min id << 1) | (sign differs from the minimum's), UNSEEN if unseen."""
        if self._words is None:
            out = np.empty(self.id_capacity, dtype=np.uint32)
            call("gcc_signed_words", self.handle, out.ctypes.data, self.id_capacity)
            self._words = out
        return self._words


class LiteralCandidates:
    """Candidates AS WRITTEN (reference-literal mode, csrc/gelly_literal.hip, gcc_literal_*).

    Candidates.merge (:77-192) skips components with identical vertex sets (:91-95), drops a failed second-level
    merge (:128-131) and files the input's vertices under min(inputKey, selfKey) without moving the self
    component (:176-189), so its output can hold overlapping "components" and miss odd cycles. This summary
    reproduces that output exactly — toString() is the reference's line — for a job that depends on it; the
    signed forest (Candidates above) is the intended semantics. Every fold / merge runs in the reference's order
    on one wavefront of the device.
    """

    def __init__(self, id_capacity: int, device: int = 0, entry_capacity: Optional[int] = None):
        """``new Candidates(true)`` (:31-34). entry_capacity bounds the entries (default 4 x id_capacity, >= 4096)."""
        self.id_capacity = int(id_capacity)
        self.device = int(device)
        if entry_capacity is None:  # the default, clamped to what the C ABI's u32 argument can carry
            entry_capacity = min(0xFFFFFFFF, max(4096, 4 * self.id_capacity))
        self.entry_capacity = int(entry_capacity)
        if not 0 < self.entry_capacity <= 0xFFFFFFFF:
            raise ValueError(f"entry_capacity {self.entry_capacity} does not fit the C ABI's u32 (1 .. 2^32 - 1)")
        h = c_void_p()
        call("gcc_literal_create", self.device, self.id_capacity, self.entry_capacity, byref(h))
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None):
            call("gcc_literal_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> c_void_p:
        if not self._h:
            raise ValueError("LiteralCandidates is closed")
        return self._h

    def getSuccess(self) -> bool:
        """:44-46"""
        ok = c_int()
        call("gcc_literal_success", self.handle, byref(ok))
        return bool(ok.value)

    def entries(self) -> np.ndarray:
        """The TreeMap's entries as u64 (component << 32) | (vertex << 1) | sign, sorted (component, vertex)."""
        n = c_uint64()
        call("gcc_literal_entries", self.handle, None, 0, byref(n))
        out = np.empty(n.value, dtype=np.uint64)
        if n.value:
            call("gcc_literal_entries", self.handle, out.ctypes.data, n.value, byref(n))
        return np.sort(out)

    def getMap(self) -> dict[int, dict[int, SignedVertex]]:
        """:48-50 — component -> (vertex -> SignedVertex), both in key order."""
        out: dict[int, dict[int, SignedVertex]] = {}
        for e in self.entries().tolist():
            c, v, sg = e >> 32, (e & 0xFFFFFFFF) >> 1, e & 1
            out.setdefault(c, {})[v] = SignedVertex(v, bool(sg))
        return out

    def merge(self, other: "LiteralCandidates") -> "LiteralCandidates":
        """:77-139 — this = this.merge(other), exactly as written; returns self."""
        call("gcc_literal_merge", self.handle, other.handle)
        return self

    def fold(self, pairs: np.ndarray) -> None:
        """updateFunction.foldEdges per edge, in order: this = this.merge(edgeToCandidate(v1, v2))."""
        a = np.ascontiguousarray(pairs, dtype=np.uint32).reshape(-1)
        if a.size:
            call("gcc_literal_fold_host", self.handle, a.ctypes.data, a.size // 2)

    def reset(self) -> None:
        call("gcc_literal_reset", self.handle)

    def toString(self) -> str:
        """Flink Tuple2.toString of (success, TreeMap), the reference's output line."""
        if not self.getSuccess():
            return "(false,{})"
        comps = ", ".join(f"{c}={{" + ", ".join(f"{v}={sv}" for v, sv in m.items()) + "}"
                          for c, m in self.getMap().items())
        return "(true,{" + comps + "})"

    def __str__(self) -> str:
        return self.toString()


class literalUpdateFunction(EdgesFold[LiteralCandidates]):
    """BipartitenessCheck.updateFunction (:74-96) over LiteralCandidates."""

    def foldEdges(self, candidates: LiteralCandidates, v1: int, v2: int, edgeVal=None) -> LiteralCandidates:
        candidates.fold(np.array([[v1, v2]], dtype=np.uint32))
        return candidates

    def foldEdgeBatch(self, candidates: LiteralCandidates, batch: EdgeBatch) -> LiteralCandidates:
        candidates.fold(batch.pairs())
        return candidates


class literalCombineFunction(ReduceFunction[LiteralCandidates]):
    """BipartitenessCheck.combineFunction (:108-131) over LiteralCandidates."""

    def reduce(self, c1: LiteralCandidates, c2: LiteralCandidates) -> LiteralCandidates:
        return c1.merge(c2)


class LiteralBipartitenessCheck(SummaryBulkAggregation[LiteralCandidates, LiteralCandidates]):
    """BipartitenessCheck with the reference's own Candidates semantics: the generic SummaryBulkAggregation
    topology (partials per partition, timeWindowAll reduce in order, Merger) over LiteralCandidates."""

    def __init__(self, mergeWindowTime: int, id_capacity: int, device: int = 0, entry_capacity: Optional[int] = None):
        super().__init__(literalUpdateFunction(), literalCombineFunction(),
                         lambda: LiteralCandidates(id_capacity, device, entry_capacity), mergeWindowTime, False)


class updateFunction(EdgesFold[Candidates]):
    """BipartitenessCheck.updateFunction (:74-96)."""

    def foldEdges(self, candidates: Candidates, v1: int, v2: int, edgeVal=None) -> Candidates:
        candidates.fold(np.array([[v1, v2]], dtype=np.uint32))
        return candidates

    def foldEdgeBatch(self, candidates: Candidates, batch: EdgeBatch) -> Candidates:
        if batch.host is not None:
            candidates.fold(batch.host)
        else:
            candidates.fold_device(batch.device_ptr, batch.n)
        return candidates


class combineFunction(ReduceFunction[Candidates]):
    """BipartitenessCheck.combineFunction (:108-131)."""

    def reduce(self, c1: Candidates, c2: Candidates) -> Candidates:
        return c1.merge(c2)


class BipartitenessCheck(SummaryBulkAggregation[Candidates, Candidates]):
    """BipartitenessCheck<K, EV> (BipartitenessCheck.java:39-52) on an MI355X."""

    def __init__(self, mergeWindowTime: int, id_capacity: int, device: int = 0):
        super().__init__(updateFunction(), combineFunction(), lambda: Candidates(id_capacity, device),
                         mergeWindowTime, False)
        self.id_capacity = id_capacity
        self.device = device

    @staticmethod
    def edgeToCandidate(v1: int, v2: int, id_capacity: int, device: int = 0) -> Candidates:
        """:54-61"""
        c = Candidates(id_capacity, device)
        c.fold(np.array([[v1, v2]], dtype=np.uint32))
        return c

    def run(self, edgeStream) -> Iterator[Candidates]:
        """Fused SummaryBulkAggregation.run: with transientState=false the summary after window w is the merge of
        every window's partial, whose canonical value is that of folding all edges so far into one forest."""
        summary: Optional[Candidates] = None
        for window_batches in edgeStream.windows(self.timeMillis):
            n = 0
            for batch in window_batches:
                if batch.n:
                    if summary is None:
                        summary = self.getInitialValue()
                    self.getUpdateFun().foldEdgeBatch(summary, batch)
                    n += batch.n
            if n:
                yield summary


def merge_group(c: Candidates, group=None) -> Candidates:
    """combineFunction across ranks (BipartitenessCheck.java:128-130 over torch.distributed; gloo or RCCL): every
    rank's ``c`` becomes the union of all ranks' summaries, failed if any rank's was. The words travel as one u32 per
    id (all_gather; the compressed words are the partition's constraints), the fail flags by all_reduce(MAX) together
    with the id ranges (every rank must hold the same id_capacity: checked before any words move, so a mismatch is an
    error on every rank instead of a mismatched all_gather); each rank then merges its peers' words on its device
    (gcc_signed_merge_words). Over nccl the words are gathered from device memory (device_words_tensor). The merge is
    a union, so the order of the peers does not matter and every rank ends with the same canonical words."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    failed = 0 if c.getSuccess() else 1
    on_gpu = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    cap = int(c.id_capacity)
    flag = torch.tensor([failed, cap, -cap], dtype=torch.int64, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    if int(flag[1].item()) != cap or -int(flag[2].item()) != cap:
        raise ValueError(f"merge_group: the ranks' id_capacity differ (this rank {cap}, max {int(flag[1].item())}, "
                         f"min {-int(flag[2].item())})")
    if int(flag[0].item()):
        c.merge_words(0, 0, other_failed=True)
        return c
    if world == 1:
        return c
    if on_gpu:
        mine = c.device_words_tensor().to(dev)
    else:
        mine = torch.from_numpy(c.words().view(np.int32)).to(dev)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    for r, t in enumerate(parts):
        if r == rank:
            continue
        d = t.to(torch.device("cuda", c.device)).contiguous()
        torch.cuda.synchronize(c.device)  # the copy is on torch's stream; the merge on the forest's
        c.merge_words(d.data_ptr(), c.id_capacity)
        c.getSuccess()  # synchronises the forest's stream before d is freed
    return c
