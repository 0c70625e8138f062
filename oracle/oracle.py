"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU oracle (oracle/cc_oracle.c).

Importable only from tests/, __graft_entry__.smoke() (as the checker) and bench.py's cpu_baseline leg.
It restates gelly-streaming's DisjointSet / CombineCC / SummaryBulkAggregation on the CPU (file:line
citations are in cc_oracle.c). Pinned by the reference's own known-answer tests via tests/golden/.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, byref, c_double, c_int, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libcc_oracle.so")
UNSEEN = 0xFFFFFFFF

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        l = ctypes.CDLL(LIB)
        l.ods_new.restype = c_void_p
        l.ods_new.argtypes = []
        l.ods_free.argtypes = [c_void_p]
        l.ods_make_set.argtypes = [c_void_p, c_uint64]
        l.ods_find.restype = c_int
        l.ods_find.argtypes = [c_void_p, c_uint64, POINTER(c_uint64)]
        l.ods_union.argtypes = [c_void_p, c_uint64, c_uint64]
        l.ods_merge.argtypes = [c_void_p, c_void_p]
        l.ods_size.restype = c_uint64
        l.ods_size.argtypes = [c_void_p]
        l.ods_combine.restype = c_void_p
        l.ods_combine.argtypes = [c_void_p, c_void_p]
        l.ods_canonical_labels.restype = c_int
        l.ods_canonical_labels.argtypes = [c_void_p, c_uint32, c_void_p]
        l.orc_label_digest.restype = c_uint64
        l.orc_label_digest.argtypes = [c_void_p, c_uint64]
        l.orc_cc_stream.restype = c_int
        l.orc_cc_stream.argtypes = [c_void_p, c_uint64, c_void_p, c_uint32, c_uint32, c_uint32, c_uint32, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, POINTER(c_double)]
        # bip_oracle.c (BipartitenessCheck / Candidates)
        l.bo_stream.restype = c_int
        l.bo_stream.argtypes = [c_void_p, c_void_p, c_uint32, c_uint32, c_uint32, c_void_p, c_void_p, c_void_p]
        _lib = l
    return _lib


class OracleDisjointSet:
    """CPU restatement of DisjointSet<Long> (…/summaries/DisjointSet.java:30-154)."""

    def __init__(self):
        self._h = lib().ods_new()

    def __del__(self):
        if getattr(self, "_h", None):
            lib().ods_free(self._h)
            self._h = None

    def makeSet(self, e):
        lib().ods_make_set(self._h, e)

    def find(self, e):
        r = c_uint64()
        return r.value if lib().ods_find(self._h, e, byref(r)) else None

    def union(self, a, b):
        lib().ods_union(self._h, a, b)

    def merge(self, other: "OracleDisjointSet"):
        lib().ods_merge(self._h, other._h)

    def size(self) -> int:
        return lib().ods_size(self._h)

    def labels(self, V: int) -> np.ndarray:
        out = np.empty(V, dtype=np.uint32)
        if lib().ods_canonical_labels(self._h, V, out.ctypes.data):
            raise ValueError("a key is >= V")
        return out


def label_digest(labels: np.ndarray) -> int:
    """sum_v splitmix64((label[v] << 32) | v) mod 2^64 — same as orc_label_digest, vectorised."""
    lab = np.asarray(labels, dtype=np.uint64)
    x = (lab << np.uint64(32)) | np.arange(lab.size, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
        return int(np.sum(x, dtype=np.uint64))


def cc_stream(pairs: np.ndarray, window_starts, V: int, partitions: int = 1, threads: int = 1,
              want_labels: bool = False, want_digest: bool = True) -> dict:
    """Run the reference topology (SummaryBulkAggregation + CombineCC + Merger) over an edge stream.

    Returns dict with per-window arrays: emitted, seen, components, digest (and labels (W, V) if asked),
    plus fold_seconds (fold + combine wall time only).
    """
    p = np.ascontiguousarray(pairs, dtype=np.uint32).reshape(-1)
    ws = np.ascontiguousarray(window_starts, dtype=np.uint64)
    W = ws.size - 1
    emitted = np.zeros(W, dtype=np.uint8)
    seen = np.zeros(W, dtype=np.uint64)
    comps = np.zeros(W, dtype=np.uint64)
    digest = np.zeros(W, dtype=np.uint64) if want_digest else None
    labels = np.zeros((W, V), dtype=np.uint32) if want_labels else None
    secs = c_double()
    rc = lib().orc_cc_stream(p.ctypes.data, p.size // 2, ws.ctypes.data, W, partitions, threads, V,
                             emitted.ctypes.data, None if labels is None else labels.ctypes.data,
                             None if digest is None else digest.ctypes.data, seen.ctypes.data, comps.ctypes.data,
                             byref(secs))
    if rc:
        raise ValueError("oracle: a vertex id is >= V")
    out = {"emitted": emitted.astype(bool), "seen": seen, "components": comps, "fold_seconds": secs.value}
    if digest is not None:
        out["digest"] = digest
    if labels is not None:
        out["labels"] = labels
    return out


def bip_stream(pairs: np.ndarray, window_starts, V: int, partitions: int = 1) -> dict:
    """BipartitenessCheck over an edge stream (bip_oracle.c): per window emitted, success and the canonical words
    ((component min << 1) | sign differs from the min's; UNSEEN if absent), shape (W, V)."""
    p = np.ascontiguousarray(pairs, dtype=np.uint32).reshape(-1)
    ws = np.ascontiguousarray(window_starts, dtype=np.uint64)
    W = ws.size - 1
    emitted = np.zeros(W, dtype=np.uint8)
    success = np.zeros(W, dtype=np.uint8)
    words = np.zeros((W, V), dtype=np.uint32)
    rc = lib().bo_stream(p.ctypes.data, ws.ctypes.data, W, partitions, V, emitted.ctypes.data, success.ctypes.data,
                         words.ctypes.data)
    if rc:
        raise ValueError("oracle: a vertex id is >= V")
    return {"emitted": emitted.astype(bool), "success": success.astype(bool), "words": words}
