"""DisjointSet — the CC summary, resident on one MI355X (mirror of …/summaries/DisjointSet.java).

Reference (`…/` = src/main/java/org/apache/flink/graph/streaming/): DisjointSet<R> keeps
``HashMap<R,R> matches`` (vertex -> parent; key set = vertices seen) and ``HashMap<R,Integer> ranks``
(…/summaries/DisjointSet.java:33-34). Here the state is one device-resident ``u32 parent[id_capacity]``
owned by libgelly_cc (include/gelly_cc.h); every method below names the Java method it mirrors.

Differences a caller can observe (none affects the partition, which is the parity contract):
  * roots are the MINIMUM vertex id of each component (min-id hooking), not union-by-rank roots, so
    ``find`` returns the canonical label and ``toString`` groups by min id;
  * ``getMatches()`` is a lazy read-only view: ``keys()`` are the vertices seen, ``get(v)`` the root;
  * vertex ids are u32 in ``[0, id_capacity)`` (the Java K=Long ids of the benchmark fit; any other Long ids
    go through LongDisjointSet, a dense relabel on the host side of the boundary — longids.py).
"""
from __future__ import annotations

import ctypes
from collections.abc import Mapping
from ctypes import byref, c_uint32, c_uint64, c_void_p
from typing import Iterable, Iterator, Optional

import numpy as np

from .native import UNSEEN, call


class MatchesView(Mapping):
    """Read-only ``Map<K,K>`` view of ``DisjointSet.getMatches()`` (DisjointSet.java:49-51)."""

    def __init__(self, ds: "DisjointSet"):
        self._ds = ds

    def _labels(self) -> np.ndarray:
        return self._ds.labels()

    def __len__(self) -> int:
        return self._ds.size()

    def __contains__(self, v) -> bool:
        return self._ds.find(v) is not None

    def __getitem__(self, v):
        r = self._ds.find(v)
        if r is None:
            raise KeyError(v)
        return r

    def __iter__(self) -> Iterator[int]:
        return iter(np.flatnonzero(self._labels() != UNSEEN).tolist())

    def keySet(self) -> list[int]:
        return list(iter(self))

    def size(self) -> int:
        return len(self)


class DisjointSet:
    """GPU union-find forest with the method surface of DisjointSet<R> (DisjointSet.java:30-154)."""

    def __init__(self, id_capacity: int, device: int = 0, elements: Optional[Iterable[int]] = None,
                 d_buffers: Optional[tuple[int, int]] = None):
        """``new DisjointSet<>()`` (:36-39) / ``new DisjointSet<>(Set<R> elements)`` (:41-47).

        d_buffers: optional two caller-owned device buffers of id_capacity u32 each (e.g. torch tensors'
        data_ptr()); the forest and its compressed labels alternate between them (see device_ptr()).
        """
        self.id_capacity = int(id_capacity)
        self.device = int(device)
        h = c_void_p()
        if d_buffers is None:
            call("gcc_forest_create", self.device, self.id_capacity, byref(h))
        else:
            call("gcc_forest_create_ext", self.device, self.id_capacity, c_void_p(d_buffers[0]),
                 c_void_p(d_buffers[1]), byref(h))
        self._h = h
        self._labels_cache: Optional[np.ndarray] = None
        if elements is not None:
            for e in elements:
                self.makeSet(e)

    # ---- lifetime -------------------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            call("gcc_forest_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self) -> c_void_p:
        if not self._h:
            raise ValueError("DisjointSet is closed")
        return self._h

    def _dirty(self) -> None:
        self._labels_cache = None

    # ---- DisjointSet.java surface ---------------------------------------------------------------
    def getMatches(self) -> MatchesView:
        """DisjointSet.getMatches (:49-51): lazy view; key set = vertices seen."""
        return MatchesView(self)

    def makeSet(self, e: int) -> None:
        """DisjointSet.makeSet (:58-61)."""
        self._check_id(e)
        call("gcc_forest_make_set", self.handle, int(e))
        self._dirty()

    def find(self, e: int) -> Optional[int]:
        """DisjointSet.find (:71-85): the component's root (its minimum id), None if e was never seen."""
        if e < 0 or e >= self.id_capacity:
            return None
        r = int(self.labels()[e])
        return None if r == UNSEEN else r

    def union(self, e1: int, e2: int) -> None:
        """DisjointSet.union (:97-123): staged in pinned memory, folded on the GPU in batches."""
        self._check_id(e1)
        self._check_id(e2)
        call("gcc_forest_union", self.handle, int(e1), int(e2))
        self._dirty()

    def merge(self, other: "DisjointSet") -> None:
        """DisjointSet.merge (:132-136): self := self ∪ other (other unchanged; any two devices)."""
        call("gcc_forest_merge", self.handle, other.handle)
        self._dirty()

    def toString(self) -> str:
        """DisjointSet.toString (:139-153): ``{root=[members...], ...}`` (roots = min ids, sorted)."""
        lab = self.labels()
        seen = np.flatnonzero(lab != UNSEEN)
        groups: dict[int, list[int]] = {}
        for v in seen.tolist():
            groups.setdefault(int(lab[v]), []).append(v)
        return "{" + ", ".join(f"{r}={m}" for r, m in sorted(groups.items())) + "}"

    def __str__(self) -> str:
        return self.toString()

    # ---- batch / device extensions (the GPU drop-in's fast paths) -------------------------------
    def size(self) -> int:
        """getMatches().size() (:49-51) without materialising the view."""
        n = c_uint64()
        call("gcc_forest_size", self.handle, byref(n))
        return n.value

    def num_components(self) -> int:
        n = c_uint64()
        call("gcc_forest_count_components", self.handle, byref(n))
        return n.value

    def fold(self, pairs: np.ndarray) -> None:
        """Fold host edges ((n, 2) u32 or interleaved u32): UpdateCC.foldEdges over a whole batch."""
        a = np.ascontiguousarray(pairs, dtype=np.uint32).reshape(-1)
        if a.size % 2:
            raise ValueError("pairs must hold an even number of ids")
        call("gcc_forest_fold_host", self.handle, a.ctypes.data, a.size // 2)
        self._dirty()

    def fold_device(self, d_pairs: int, n_edges: int) -> None:
        """Fold n_edges interleaved u32 pairs already in HBM (async on this forest's stream)."""
        call("gcc_forest_fold_device", self.handle, c_void_p(d_pairs), int(n_edges))
        self._dirty()

    def fold_pinned(self, h_pairs: int, n_edges: int) -> None:
        """Fold n_edges interleaved u32 pairs in pinned host memory (chunked H2D overlapped with the folds; async:
        the buffer must stay valid until the next synchronising call, e.g. sync())."""
        call("gcc_forest_fold_pinned", self.handle, c_void_p(h_pairs), int(n_edges))
        self._dirty()

    def labels_device(self) -> int:
        """Compress (async) and return the device buffer of the canonical labels, read-only (valid until the next
        mutation of this forest)."""
        p = c_void_p()
        call("gcc_forest_labels_device", self.handle, byref(p))
        return p.value

    def merge_labels_device(self, d_labels: int, n: int) -> None:
        """self := self ∪ {(v, labels[v])} for a device label/parent array (the cross-GPU merge receive)."""
        call("gcc_forest_merge_labels_device", self.handle, c_void_p(d_labels), int(n))
        self._dirty()

    def encode_message(self, d_msg: int, cap_others: int) -> None:
        """Compress, then write the cross-GPU merge message (include/gelly_cc.h layout) into d_msg (async)."""
        call("gcc_forest_encode", self.handle, c_void_p(d_msg), int(cap_others))

    def absorb_message(self, d_msg: int, cap_others: int) -> None:
        """self := self ∪ the partition of a message written with the same id_capacity and cap_others."""
        call("gcc_forest_absorb", self.handle, c_void_p(d_msg), int(cap_others))
        self._dirty()

    def absorb_messages(self, d_msgs: int, stride: int, count: int, skip: int, cap_others: int) -> None:
        """Absorb `count` messages laid out every `stride` bytes from d_msgs, except number `skip` (one launch)."""
        call("gcc_forest_absorb_many", self.handle, c_void_p(d_msgs), int(stride), int(count), int(skip) & 0xFFFFFFFF,
             int(cap_others))
        self._dirty()

    def compress(self) -> None:
        """Canonicalise (async): afterwards device_ptr() holds the min-id labels."""
        call("gcc_forest_compress", self.handle)

    def labels(self) -> np.ndarray:
        """Canonical labels as a host u32 array of id_capacity (UNSEEN = 0xFFFFFFFF for unseen ids)."""
        if self._labels_cache is None:
            out = np.empty(self.id_capacity, dtype=np.uint32)
            call("gcc_forest_labels", self.handle, out.ctypes.data, self.id_capacity)
            self._labels_cache = out
        return self._labels_cache

    def raw_parent(self) -> np.ndarray:
        """The device parent array as it stands (no compress) — for forest-invariant checks."""
        out = np.empty(self.id_capacity, dtype=np.uint32)
        call("gcc_forest_raw_parent", self.handle, out.ctypes.data, self.id_capacity)
        return out

    def reset(self) -> None:
        """Back to the empty initial value (Merger transientState reset, SummaryAggregation.java:113-115)."""
        call("gcc_forest_reset", self.handle)
        self._dirty()

    def sync(self) -> None:
        call("gcc_forest_sync", self.handle)

    def set_stream(self, hip_stream: Optional[int]) -> None:
        """Order this forest's work on hip_stream (0 = the null stream); None = back to its own stream."""
        call("gcc_forest_set_stream", self.handle, c_void_p(hip_stream or 0), 1 if hip_stream is None else 0)

    def stream(self) -> int:
        s = c_void_p()
        call("gcc_forest_get_stream", self.handle, byref(s))
        return s.value or 0

    def device_ptr(self) -> int:
        """The buffer currently holding the forest (after compress(): the canonical labels)."""
        p = c_void_p()
        call("gcc_forest_device_ptr", self.handle, byref(p))
        return p.value

    def import_pairs(self, pairs: np.ndarray) -> None:
        """Restore from (key, parent) pairs (Merger.restoreState, SummaryAggregation.java:132-135)."""
        a = np.ascontiguousarray(pairs, dtype=np.uint32).reshape(-1)
        call("gcc_forest_import_pairs", self.handle, a.ctypes.data, a.size // 2)
        self._dirty()

    def serialize(self) -> bytes:
        """The summary's checkpoint / wire bytes (include/gelly_cc.h "serialized summary": (v, label) pairs, or the
        compact merge message when one component dominates). Merger.snapshotState (SummaryAggregation.java:127-130)."""
        n = c_uint64()
        call("gcc_forest_serialized_size", self.handle, byref(n))
        buf = ctypes.create_string_buffer(n.value)
        w = c_uint64()
        call("gcc_forest_serialize", self.handle, buf, n.value, byref(w))
        return buf.raw[:w.value]

    def deserialize(self, data: bytes) -> None:
        """Fold a serialized summary into this one (into a fresh or reset forest: Merger.restoreState, :132-135)."""
        call("gcc_forest_deserialize", self.handle, ctypes.c_char_p(bytes(data)), len(data))
        self._dirty()

    @classmethod
    def from_bytes(cls, data: bytes, id_capacity: Optional[int] = None, device: int = 0) -> "DisjointSet":
        """A new summary restored from serialize()'s bytes (the id range defaults to the serialized one)."""
        cap = id_capacity if id_capacity is not None else int.from_bytes(bytes(data[8:12]), "little")
        ds = cls(cap, device)
        ds.deserialize(data)
        return ds

    def snapshot_pairs(self) -> np.ndarray:
        """Serialisable state (Merger.snapshotState, SummaryAggregation.java:127-130): (v, label[v]) of seen v."""
        lab = self.labels()
        seen = np.flatnonzero(lab != UNSEEN).astype(np.uint32)
        return np.stack([seen, lab[seen]], axis=1)

    def enable_timing(self, mode: int = 1) -> None:
        """0 off; 1 HIP events around each fold and its phases; 2 also count slow-path edges."""
        call("gcc_forest_enable_timing", self.handle, int(mode))

    def last_fold_ms(self) -> float:
        ms = ctypes.c_float()
        call("gcc_forest_last_fold_ms", self.handle, byref(ms))
        return ms.value

    def fold_profile(self) -> list[tuple[str, float, int]]:
        """Drain the per-phase (name, ms, edges) log of every fold since the last call (timing mode); each fold
        starts with a ("begin", 0, 0) row (+ ("slow_edges", 0, n) rows in mode 2)."""
        buf = ctypes.create_string_buffer(1 << 20)
        call("gcc_forest_fold_profile", self.handle, buf, len(buf))
        out = []
        for line in buf.value.decode().splitlines():
            k, ms, n = line.split()
            out.append((k, float(ms), int(n)))
        return out

    def tune(self, **knobs) -> None:
        """Fold-pipeline tuning (speed only; results are independent of it)."""
        for k, v in knobs.items():
            call("gcc_forest_tune", self.handle, k.encode(), float(v))

    def label_digest(self) -> tuple:
        """(digest, seen, components) of the canonical labels, computed on the device (gcc_forest_label_digest): the
        digest of tests/golden/stream_digests.json / oracle.label_digest, without a host copy of the labels."""
        a, b, c = c_uint64(), c_uint64(), c_uint64()
        call("gcc_forest_label_digest", self.handle, byref(a), byref(b), byref(c))
        return a.value, b.value, c.value

    def inc_check_stats(self) -> tuple:
        """Diagnostics (tune(inc_check=1)): (checked incremental compresses, wrong labels, lost bloom marks)."""
        a, b, c = c_uint64(), c_uint64(), c_uint64()
        call("gcc_forest_inc_check_stats", self.handle, byref(a), byref(b), byref(c))
        return a.value, b.value, c.value

    def post_check_stats(self) -> tuple:
        """Diagnostics (tune(post_check=1 or 2)): (checks, offenders, records) of the check after every incremental
        compress; records = up to 6 tuples (check#, v, label, label's label, root, marked, prev[v], prev[label])."""
        a, b = c_uint64(), c_uint64()
        rec = (c_uint32 * 48)()
        call("gcc_forest_post_check_stats", self.handle, byref(a), byref(b), rec, 6)
        n = min(int(b.value), 6)
        return a.value, b.value, [tuple(rec[8 * k:8 * k + 8]) for k in range(n)]

    def copy(self) -> "DisjointSet":
        """A fresh forest with the same partition (Flink copies the fold's initial value per window)."""
        d = DisjointSet(self.id_capacity, self.device)
        d.merge(self)
        return d

    def _check_id(self, e: int) -> None:
        if not 0 <= int(e) < self.id_capacity:
            raise ValueError(f"vertex id {e} outside [0, {self.id_capacity})")
