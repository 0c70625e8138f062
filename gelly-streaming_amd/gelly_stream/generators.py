"""Synthetic edge streams of the benchmark configs.

All generation runs in libgelly_cc (csrc/edge_gen.h): on the host for small parity cases, or straight
into HBM with gcc_gen_device for the benchmark, so the timed region never includes generation or PCIe.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import native
from .native import GenParams, call

SEED_BASE = 0x67656C6C79000000  # "gelly\0\0\0"


@dataclass(frozen=True)
class StreamConfig:
    """One benchmark configuration: the generator plus the merge-window model."""

    name: str
    kind: int
    scale: int = 0
    n_vertices: int = 0
    n_edges: int = 0
    seed: int = 0
    n_stars: int = 0
    star_size: int = 0
    permute: int = 1
    window_edges: int = 0  # edges per merge window (0 = the whole stream is one window)
    merge_window_ms: int = 0  # EXAMPLE only: event-time windows of this many ms

    def params(self) -> GenParams:
        return GenParams(self.kind, self.scale, self.n_vertices, self.n_edges, self.seed, self.n_stars,
                         self.star_size, self.permute, 0)

    def info(self) -> tuple[int, int]:
        """(number of edges, id range V)."""
        e, v = ctypes.c_uint64(), ctypes.c_uint64()
        call("gcc_gen_info", ctypes.byref(self.params()), ctypes.byref(e), ctypes.byref(v))
        return e.value, v.value


CONFIGS = {
    # C1: ConnectedComponentsExample default data, 1000 ms event-time windows (example/ConnectedComponentsExample.java:78,121-133)
    "c1_example": StreamConfig("c1_example", native.GCC_GEN_EXAMPLE, merge_window_ms=1000),
    # C2: R-MAT scale 20, edge factor 16, one MI355X — the N=1 bench workload
    "c2_rmat20": StreamConfig("c2_rmat20", native.GCC_GEN_RMAT, scale=20, n_edges=16 << 20, seed=SEED_BASE | 2),
    # C3: uniform G(n, m) just above the percolation threshold (mean degree ~1.1)
    "c3_gnm24": StreamConfig("c3_gnm24", native.GCC_GEN_GNM, n_vertices=1 << 24, n_edges=9_227_469, seed=SEED_BASE | 3),
    # C4: Kronecker scale 26, edge factor 16 (1 GiB-edge stream over 8 GPUs)
    "c4_kron26": StreamConfig("c4_kron26", native.GCC_GEN_RMAT, scale=26, n_edges=16 << 26, seed=SEED_BASE | 4),
    # C4's per-GPU share: the first 2^27 edges of the C4 stream (same seed, counter-based generator), all 2^26
    # ids. Weak-scaled over W ranks (bench.py) it is the first W * 2^27 edges: W = 8 is exactly C4.
    "c4_share": StreamConfig("c4_share", native.GCC_GEN_RMAT, scale=26, n_edges=2 << 26, seed=SEED_BASE | 4),
    # C4's per-rank folds at N = 4 and N = 2 (the first 2^28 / 2^29 edges): the measured inputs of DESIGN.md §6's
    # predicted 1/2/4/8 curve (bench.py config legs, round 6)
    "c4_quarter": StreamConfig("c4_quarter", native.GCC_GEN_RMAT, scale=26, n_edges=4 << 26, seed=SEED_BASE | 4),
    "c4_half": StreamConfig("c4_half", native.GCC_GEN_RMAT, scale=26, n_edges=8 << 26, seed=SEED_BASE | 4),
    # C5: adversarial path over 2^23 ids + 1024 stars of 8192 ids, windows of 2^16 edges
    "c5_adversarial": StreamConfig("c5_adversarial", native.GCC_GEN_ADVERSARIAL, scale=23, n_stars=1024,
                                   star_size=8192, seed=SEED_BASE | 5, window_edges=1 << 16),
}


def scaled(cfg: StreamConfig, **changes) -> StreamConfig:
    """A smaller (or otherwise altered) variant of a config, e.g. for CPU-oracle parity cases."""
    d = dict(cfg.__dict__)
    d.update(changes)
    return StreamConfig(**d)


def generate_host(cfg: StreamConfig, first: int = 0, count: Optional[int] = None) -> np.ndarray:
    """Edges [first, first+count) as an (count, 2) uint32 array (host generator, same bytes as the device one)."""
    n, _ = cfg.info()
    if count is None:
        count = n - first
    out = np.empty((count, 2), dtype=np.uint32)
    call("gcc_gen_host", ctypes.byref(cfg.params()), first, count, out.ctypes.data)
    return out


def generate_device(cfg: StreamConfig, first: int, count: int, d_pairs: int, hip_stream: int = 0) -> None:
    """Write edges [first, first+count) as interleaved u32 pairs to device memory d_pairs (async on hip_stream)."""
    call("gcc_gen_device", ctypes.byref(cfg.params()), first, count, ctypes.c_void_p(d_pairs),
         ctypes.c_void_p(hip_stream))


def to_bipartite(pairs: np.ndarray) -> np.ndarray:
    """The bipartite version of a stream (BipartitenessCheck's bench legs): u -> u & ~1 (even ids, one side),
    v -> v | 1 (odd ids, the other). Every edge joins the two sides, so the stream never fails; its components and
    degrees keep the source's shape (a kron stream keeps its hubs). Ids stay below an even V."""
    p = np.array(pairs, dtype=np.uint32, copy=True).reshape(-1, 2)
    p[:, 0] &= np.uint32(0xFFFFFFFE)
    p[:, 1] |= np.uint32(1)
    return p


def to_bipartite_device(t) -> None:
    """to_bipartite in place on a device tensor of interleaved int32 pairs (torch; input preparation only)."""
    v = t.view(-1, 2)
    v[:, 0].bitwise_and_(-2)
    v[:, 1].bitwise_or_(1)


def timestamps(cfg: StreamConfig, first: int = 0, count: Optional[int] = None) -> np.ndarray:
    """Event timestamps (ms) of the stream; only the EXAMPLE stream carries the reference's timestamps."""
    n, _ = cfg.info()
    if count is None:
        count = n - first
    if cfg.kind == native.GCC_GEN_EXAMPLE:
        return (np.arange(first, first + count, dtype=np.int64) + 1) * 100
    return np.zeros(count, dtype=np.int64)


def window_starts(cfg: StreamConfig) -> np.ndarray:
    """Edge offsets of the merge windows (n_windows + 1 entries; window w = edges [s[w], s[w+1])).

    EXAMPLE: tumbling event-time windows of merge_window_ms over its timestamps (Flink TimeWindow start =
    ts - ts % size), else contiguous chunks of window_edges edges (SURVEY.md §8(d) window model).
    """
    n, _ = cfg.info()
    if cfg.merge_window_ms:
        ts = timestamps(cfg)
        return time_window_starts(ts, cfg.merge_window_ms)
    w = cfg.window_edges or n
    starts = list(range(0, n, w)) + [n]
    return np.asarray(starts, dtype=np.uint64)


def time_window_starts(ts: np.ndarray, size_ms: int) -> np.ndarray:
    """Window boundaries for an ascending-timestamp stream cut into tumbling windows of size_ms."""
    ts = np.asarray(ts, dtype=np.int64)
    if ts.size and np.any(np.diff(ts) < 0):
        raise ValueError("event timestamps must be ascending (AscendingTimestampExtractor)")
    win = ts - ts % size_ms
    cut = np.flatnonzero(np.diff(win)) + 1
    return np.concatenate([[0], cut, [ts.size]]).astype(np.uint64)
