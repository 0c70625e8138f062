"""DisjointSet<Long> over arbitrary Java Long vertex ids (…/summaries/DisjointSet.java:30-34 is keyed by the id).

The device forest (DisjointSet) works on dense u32 ids. IdDictionary (libgelly_cc gcc_idmap_*, host-only C++)
assigns dense ids in first-seen order; LongDisjointSet folds the relabelled edges into a device forest and
reports the reference's canonical form: find(v) = the minimum ORIGINAL id of v's component (signed Long order),
None for an id never seen. The dense relabel runs on the host side of the boundary, where the Java task thread
already holds the edge batch; the fold itself is the same HIP path.
"""
from __future__ import annotations

from collections.abc import Mapping
from ctypes import byref, c_uint32, c_uint64, c_void_p
from typing import Iterator, Optional

import numpy as np

from .native import UNSEEN, call
from .summaries import DisjointSet

_I64_MAX = np.iinfo(np.int64).max


class IdDictionary:
    """Java Long vertex id -> dense u32 id, first-seen order (gcc_idmap_*)."""

    def __init__(self, capacity: int):
        h = c_void_p()
        call("gcc_idmap_create", int(capacity), byref(h))
        self._h = h
        self.capacity = int(capacity)

    def close(self) -> None:
        if getattr(self, "_h", None):
            call("gcc_idmap_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self) -> int:
        n = c_uint64()
        call("gcc_idmap_size", self._h, byref(n))
        return n.value

    def map(self, ids) -> np.ndarray:
        """Dense ids of `ids` (any shape); ids seen for the first time take the next dense ids, in order."""
        a = np.ascontiguousarray(ids, dtype=np.int64)
        out = np.empty(a.shape, dtype=np.uint32)
        call("gcc_idmap_map", self._h, a.ctypes.data, a.size, out.ctypes.data)
        return out

    def lookup(self, v: int) -> Optional[int]:
        d = c_uint32()
        call("gcc_idmap_lookup", self._h, int(v), byref(d))
        return None if d.value == UNSEEN else d.value

    def ids(self) -> np.ndarray:
        """ids()[d] = the original id of dense id d."""
        n = len(self)
        out = np.empty(n, dtype=np.int64)
        call("gcc_idmap_ids", self._h, out.ctypes.data, n)
        return out

    def canonical(self, dense_labels: np.ndarray, unseen: int = _I64_MAX) -> np.ndarray:
        """Per dense id: the minimum original id of its component (dense_labels: a forest's labels over the
        dense range, UNSEEN for unseen), `unseen` where the forest has not seen the id."""
        lab = np.ascontiguousarray(dense_labels[:len(self)], dtype=np.uint32)
        out = np.empty(lab.size, dtype=np.int64)
        call("gcc_idmap_canonical", self._h, lab.ctypes.data, lab.size, out.ctypes.data, int(unseen))
        return out


class LongMatchesView(Mapping):
    """getMatches() (:49-51) keyed by the original ids: keys = vertices seen, value = canonical label."""

    def __init__(self, ds: "LongDisjointSet"):
        self._ds = ds

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
        ids, lab = self._ds.seen_labels()
        return iter(ids.tolist())

    def keySet(self) -> list[int]:
        return list(iter(self))

    def size(self) -> int:
        return len(self)


class LongDisjointSet:
    """DisjointSet<Long> (DisjointSet.java:30-154) for ids anywhere in the Java Long range; at most `capacity`
    distinct ids. Canonical labels are minimum original ids, so the partition output matches the reference's
    whatever the ids are."""

    def __init__(self, capacity: int, device: int = 0):
        self.dict = IdDictionary(capacity)
        self.forest = DisjointSet(capacity, device)
        self._cache = None

    def close(self) -> None:
        self.forest.close()
        self.dict.close()

    def _dirty(self) -> None:
        self._cache = None

    def fold(self, pairs) -> None:
        """UpdateCC.foldEdges over a batch of (src, trg) Long pairs ((n, 2) or interleaved)."""
        a = np.asarray(pairs, dtype=np.int64).reshape(-1)
        if a.size % 2:
            raise ValueError("pairs must hold an even number of ids")
        self.forest.fold(self.dict.map(a))
        self._dirty()

    def union(self, e1: int, e2: int) -> None:
        """DisjointSet.union (:97-123)."""
        d = self.dict.map([e1, e2])
        self.forest.union(int(d[0]), int(d[1]))
        self._dirty()

    def makeSet(self, e: int) -> None:
        """DisjointSet.makeSet (:58-61)."""
        self.forest.makeSet(int(self.dict.map([e])[0]))
        self._dirty()

    def merge(self, other: "LongDisjointSet") -> None:
        """DisjointSet.merge (:132-136): the other summary's (vertex, label) pairs, relabelled into this one."""
        ids, lab = other.seen_labels()
        if ids.size:
            self.fold(np.stack([ids, lab], axis=1))

    def _labels(self) -> tuple[np.ndarray, np.ndarray]:
        """(canonical label per dense id, seen mask per dense id). Seen-ness comes from the forest (dense label !=
        UNSEEN), never from a sentinel value: every Long, Long.MAX_VALUE included, is a valid label."""
        if self._cache is None:
            dense = self.forest.labels()
            lab = self.dict.canonical(dense)
            self._cache = (lab, dense[:lab.size] != UNSEEN)
        return self._cache

    def seen_labels(self) -> tuple[np.ndarray, np.ndarray]:
        """(original ids seen, their canonical labels)."""
        lab, seen = self._labels()
        ids = self.dict.ids()
        return ids[seen], lab[seen]

    def find(self, e: int) -> Optional[int]:
        """DisjointSet.find (:71-85): the canonical label (minimum original id), None if never seen."""
        d = self.dict.lookup(e)
        if d is None:
            return None
        lab, seen = self._labels()
        return int(lab[d]) if seen[d] else None

    def getMatches(self) -> LongMatchesView:
        return LongMatchesView(self)

    def size(self) -> int:
        return self.forest.size()

    def num_components(self) -> int:
        return self.forest.num_components()

    def toString(self) -> str:
        """DisjointSet.toString (:139-153), grouped by canonical label (sorted)."""
        ids, lab = self.seen_labels()
        groups: dict[int, list[int]] = {}
        for v, r in sorted(zip(ids.tolist(), lab.tolist())):
            groups.setdefault(r, []).append(v)
        return "{" + ", ".join(f"{r}={m}" for r, m in sorted(groups.items())) + "}"

    def __str__(self) -> str:
        return self.toString()
