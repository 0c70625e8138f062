"""Summary-aggregation operator surface (mirror of the reference's L2 aggregation framework).

Reference (`…/` = src/main/java/org/apache/flink/graph/streaming/):
  EdgesFold              …/EdgesFold.java:33-47      T foldEdges(T accum, K vertexID, K neighborID, EV edgeValue)
  SummaryAggregation     …/SummaryAggregation.java:50-135  (updateFun, combineFun, transform, initialValue,
                                                            transientState) + Merger running summary
  SummaryBulkAggregation …/SummaryBulkAggregation.java:51-131
        edges -> map(PartitionMapper) -> keyBy(partition) -> timeWindow(t) -> fold(initial, PartialAgg)
              -> timeWindowAll(t) -> reduce(combineFun) -> flatMap(Merger) at parallelism 1

Here a "partition" is one GPU (one rank), the window fold runs as HIP kernels on that GPU, and the
timeWindowAll reduce is the cross-GPU combine of ForestGroup (distributed.py) over RCCL/xGMI.
The generic path below keeps the reference's topology for ANY EdgesFold/ReduceFunction pair; the
ConnectedComponents library overrides run() with the equivalent fused form (library.py).
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from dataclasses import dataclass
from typing import Any, Callable, Generic, Iterator, Optional, TypeVar

import numpy as np

S = TypeVar("S")
T = TypeVar("T")


@dataclass
class EdgeBatch:
    """One partition's edges of one merge window: host pairs or a device range (interleaved u32 pairs)."""

    n: int
    host: Optional[np.ndarray] = None  # (n, 2) uint32
    device_ptr: int = 0  # address of the first pair in HBM
    values: Optional[np.ndarray] = None  # edge values (NullValue for CC: None)
    window: int = 0

    def pairs(self) -> np.ndarray:
        if self.host is None:
            raise ValueError("device-resident batch has no host view")
        return self.host


class EdgesFold(ABC, Generic[S]):
    """EdgesFold<K, EV, T> (…/EdgesFold.java:33-47)."""

    @abstractmethod
    def foldEdges(self, accum: S, vertexID: int, neighborID: int, edgeValue: Any) -> S:
        ...

    def foldEdgeBatch(self, accum: S, batch: EdgeBatch) -> S:
        """Fold a whole batch; the default applies foldEdges per edge (PartialAgg.fold :121-123)."""
        pairs = batch.pairs()
        vals = batch.values
        for i in range(batch.n):
            accum = self.foldEdges(accum, int(pairs[i, 0]), int(pairs[i, 1]), None if vals is None else vals[i])
        return accum


class ReduceFunction(ABC, Generic[S]):
    """org.apache.flink.api.common.functions.ReduceFunction<S>."""

    @abstractmethod
    def reduce(self, value1: S, value2: S) -> S:
        ...


class Merger(Generic[S]):
    """SummaryAggregation.Merger (…/SummaryAggregation.java:93-135): the parallelism-1 running summary."""

    def __init__(self, initial: Callable[[], S], combiner: Optional[ReduceFunction[S]], transientState: bool):
        self._initial = initial
        self._combiner = combiner
        self._transient = transientState
        self.summary: Optional[S] = None

    def flatMap(self, s: S) -> S:
        """:107-119 — summary = combine.reduce(s, summary); emit; reset if transientState."""
        if self._combiner is None:
            return s
        if self.summary is None:
            self.summary = self._initial()
        self.summary = self._combiner.reduce(s, self.summary)
        out = self.summary
        if self._transient:
            self.summary = None
        return out

    def snapshotState(self) -> list:
        """:127-130 — ListCheckpointed: the running summary in its serialized form (bytes) when it has one (a device
        summary: DisjointSet.serialize, include/gelly_cc.h "serialized summary"), else the object itself."""
        s = self.summary
        return [s.serialize() if hasattr(s, "serialize") else s]

    def restoreState(self, state: list) -> None:
        """:132-135 — a serialized summary is rebuilt into a fresh one from the initial-value factory."""
        s = state[0] if state else None
        if isinstance(s, (bytes, bytearray)):
            fresh = self._initial()
            fresh.deserialize(s)
            s = fresh
        self.summary = s


class SummaryAggregation(ABC, Generic[S, T]):
    """SummaryAggregation<K, EV, S, T> (…/SummaryAggregation.java:50-91)."""

    def __init__(self, updateFun: EdgesFold[S], combineFun: Optional[ReduceFunction[S]],
                 transform: Optional[Callable[[S], T]], initialValue: Callable[[], S], transientState: bool):
        # initialValue is a factory: a device summary is created lazily on the task side, never in the
        # client-side constructor (the reference Java-serialises its initial value into the job graph).
        self._updateFun = updateFun
        self._combineFun = combineFun
        self._transform = transform
        self._initial = initialValue
        self._transient = transientState

    def getUpdateFun(self) -> EdgesFold[S]:
        return self._updateFun

    def getCombineFun(self) -> Optional[ReduceFunction[S]]:
        return self._combineFun

    def getTransform(self):
        return self._transform

    def isTransientState(self) -> bool:
        return self._transient

    def getInitialValue(self) -> S:
        """A fresh copy of the initial value (Flink copies it for every (key, window) fold)."""
        return self._initial()

    def getAggregator(self) -> Merger[S]:
        """:83-85"""
        return Merger(self._initial, self._combineFun, self._transient)

    @abstractmethod
    def run(self, edgeStream) -> Iterator[T]:
        ...


class SummaryBulkAggregation(SummaryAggregation[S, T]):
    """SummaryBulkAggregation (…/SummaryBulkAggregation.java:51-131).

    run() yields one summary per non-empty merge window, like the reference's output DataStream.
    group: optional cross-rank combiner (distributed.ForestGroup-like, with ``reduce(summary, combineFun)``)
    standing in for the all-to-one ``timeWindowAll(...).reduce(combineFun)`` gather (:81-82).
    """

    def __init__(self, updateFun: EdgesFold[S], combineFun: ReduceFunction[S], initialVal: Callable[[], S],
                 timeMillis: int, transientState: bool, transformFun: Optional[Callable[[S], T]] = None,
                 group=None):
        super().__init__(updateFun, combineFun, transformFun, initialVal, transientState)
        self.timeMillis = int(timeMillis)
        self.group = group

    def run(self, edgeStream) -> Iterator[T]:
        merger = self.getAggregator()
        for window_batches in edgeStream.windows(self.timeMillis):
            # keyBy(partition).timeWindow(t).fold(initial, PartialAgg): one partial per non-empty partition
            partials = []
            for batch in window_batches:
                if batch.n == 0:
                    continue
                partials.append(self.getUpdateFun().foldEdgeBatch(self.getInitialValue(), batch))
            if not partials and self.group is None:
                continue
            # timeWindowAll(t).reduce(combineFun) — local partials, then across ranks
            acc = partials[0] if partials else self.getInitialValue()
            for p in partials[1:]:
                acc = self.getCombineFun().reduce(acc, p)
            if self.group is not None:
                acc = self.group.reduce(acc, self.getCombineFun())
            out = merger.flatMap(acc)  # flatMap(Merger).setParallelism(1)
            yield self._transform(out) if self._transform else out


class SummaryTreeReduce(SummaryBulkAggregation[S, T]):
    """SummaryTreeReduce (…/SummaryTreeReduce.java:47-160): the window's partials are combined in a pairwise tree
    instead of one all-to-one reduce. enhance() (:95-123) re-keys partition p to p // 2 and reduces each pair,
    halving the parallelism until it is <= 2; timeWindowAll(...).reduce + Merger finish (:87-90).

    degree: partitions of the window fold (-1 = the stream's parallelism, :75). On the device each partial is
    its own summary, and every level of the tree is a set of independent pairwise combines (the cross-GPU
    form of the same tree is ForestGroup's single all_gather, distributed.py).
    """

    def __init__(self, updateFun: EdgesFold[S], combineFun: ReduceFunction[S], initialVal: Callable[[], S],
                 timeMillis: int, transientState: bool, degree: int = -1,
                 transformFun: Optional[Callable[[S], T]] = None):
        super().__init__(updateFun, combineFun, initialVal, timeMillis, transientState, transformFun)
        self.degree = int(degree)

    def run(self, edgeStream) -> Iterator[T]:
        merger = self.getAggregator()
        for window_batches in edgeStream.windows(self.timeMillis):
            # map(PartitionMapper).setParallelism(degree).keyBy(0).timeWindow(t).fold(...) (:77-82)
            partials: list[tuple[int, S]] = []
            for p, batch in enumerate(window_batches):
                if batch.n:
                    partials.append((p, self.getUpdateFun().foldEdgeBatch(self.getInitialValue(), batch)))
            if not partials:
                continue
            parallelism = max(len(window_batches), 1)
            # enhance(): keyBy(f0 / 2) + AggregationWrapper reduce, while the parallelism is > 2 (:97-122)
            while parallelism > 2:
                pairs: dict[int, S] = {}
                for key, s in partials:
                    k = key // 2
                    pairs[k] = s if k not in pairs else self.getCombineFun().reduce(pairs[k], s)
                partials = sorted(pairs.items())
                parallelism //= 2
            acc = partials[0][1]
            for _, s in partials[1:]:  # timeWindowAll(...).reduce(combineFun) (:88-89)
                acc = self.getCombineFun().reduce(acc, s)
            out = merger.flatMap(acc)
            yield self._transform(out) if self._transform else out
