"""SimpleEdgeStream — the edge stream the CC summary is aggregated over (mirror of …/SimpleEdgeStream.java).

Reference (`…/` = src/main/java/org/apache/flink/graph/streaming/):
  SimpleEdgeStream(DataStream<Edge<K,EV>> edges, StreamExecutionEnvironment ctx)          :69-73 (IngestionTime)
  SimpleEdgeStream(edges, AscendingTimestampExtractor<Edge<K,EV>> extractor, ctx)          :86-90 (EventTime)
  aggregate(SummaryAggregation<K,EV,S,T> summaryAggregation) = summaryAggregation.run(edges) :100-102

Only the constructor + aggregate() surface of the hot path is mirrored. Windows are
tumbling event-time windows of ``timeMillis`` over the edges' timestamps; a stream without timestamps uses
the deterministic model of SURVEY.md §8(d): edge i has event time floor(i / W) * timeMillis, i.e. window k
= edges [kW, (k+1)W). Within a window the edges are split into ``parallelism`` contiguous partitions (the
reference's PartitionMapper tags each edge with its upstream subtask, SummaryBulkAggregation.java:93-106);
with rank/world set, this process owns partition ``rank`` of ``world``.
"""
from __future__ import annotations

from typing import Iterator, Optional

import numpy as np

from .aggregation import EdgeBatch
from .generators import time_window_starts


class SimpleEdgeStream:
    def __init__(self, pairs: Optional[np.ndarray] = None, timestamps: Optional[np.ndarray] = None,
                 edges_per_window: Optional[int] = None, parallelism: int = 1, rank: int = 0, world: int = 1,
                 device_ptr: int = 0, n_device_edges: int = 0, device_window_starts: Optional[np.ndarray] = None):
        """Host edges (pairs (n, 2) u32 with optional ascending event timestamps in ms) or a device-resident
        edge range (device_ptr, n_device_edges, device_window_starts = this rank's window offsets)."""
        self.pairs = None if pairs is None else np.ascontiguousarray(pairs, dtype=np.uint32).reshape(-1, 2)
        self.timestamps = None if timestamps is None else np.asarray(timestamps, dtype=np.int64)
        if self.pairs is not None and self.timestamps is not None and len(self.timestamps) != len(self.pairs):
            raise ValueError("one timestamp per edge")
        self.edges_per_window = edges_per_window
        self.parallelism = max(1, int(parallelism))
        self.rank = int(rank)
        self.world = max(1, int(world))
        self.device_ptr = int(device_ptr)
        self.n_device_edges = int(n_device_edges)
        self.device_window_starts = device_window_starts

    def aggregate(self, summaryAggregation):
        """SimpleEdgeStream.aggregate (:100-102)."""
        return summaryAggregation.run(self)

    def _window_starts(self, timeMillis: int) -> np.ndarray:
        n = len(self.pairs)
        if self.timestamps is not None:
            return time_window_starts(self.timestamps, timeMillis)
        w = self.edges_per_window or n or 1
        return np.asarray(list(range(0, n, w)) + [n], dtype=np.uint64)

    def windows(self, timeMillis: int) -> Iterator[list[EdgeBatch]]:
        """Per merge window, the EdgeBatch of each partition this process folds."""
        if self.pairs is None:
            starts = np.asarray(self.device_window_starts if self.device_window_starts is not None
                                else [0, self.n_device_edges], dtype=np.uint64)
            for w in range(len(starts) - 1):
                b, e = int(starts[w]), int(starts[w + 1])
                yield [EdgeBatch(n=e - b, device_ptr=self.device_ptr + 8 * b, window=w)]
            return
        starts = self._window_starts(timeMillis)
        parts = self.parallelism * self.world
        for w in range(len(starts) - 1):
            b, e = int(starts[w]), int(starts[w + 1])
            L = e - b
            out = []
            for p in range(self.rank * self.parallelism, (self.rank + 1) * self.parallelism):
                pb, pe = b + L * p // parts, b + L * (p + 1) // parts
                out.append(EdgeBatch(n=pe - pb, host=self.pairs[pb:pe], window=w))
            yield out
