"""ConnectedComponents library method (mirror of …/library/ConnectedComponents.java).

Reference (`…/` = src/main/java/org/apache/flink/graph/streaming/library/):
  ConnectedComponents(long mergeWindowTime)  ConnectedComponents.java:52-54
      = SummaryBulkAggregation(new UpdateCC(), new CombineCC(), new DisjointSet<K>(), mergeWindowTime, false)
  UpdateCC.foldEdges(ds, v, v2, ev)          :83-86   ds.union(v, v2); return ds
  CombineCC.reduce(s1, s2)                   :116-125 merge the smaller forest into the larger
"""
from __future__ import annotations

from typing import Iterator, Optional

from .aggregation import EdgeBatch, EdgesFold, ReduceFunction, SummaryBulkAggregation, SummaryTreeReduce
from .summaries import DisjointSet


class UpdateCC(EdgesFold[DisjointSet]):
    """UpdateCC (ConnectedComponents.java:74-87)."""

    def foldEdges(self, ds: DisjointSet, vertex: int, vertex2: int, edgeValue=None) -> DisjointSet:
        ds.union(vertex, vertex2)
        return ds

    def foldEdgeBatch(self, ds: DisjointSet, batch: EdgeBatch) -> DisjointSet:
        """The whole batch in one HIP launch (edge values are NullValue for CC and are ignored)."""
        if batch.host is not None:
            ds.fold(batch.host)
        else:
            ds.fold_device(batch.device_ptr, batch.n)
        return ds


class CombineCC(ReduceFunction[DisjointSet]):
    """CombineCC (ConnectedComponents.java:101-126)."""

    def reduce(self, s1: DisjointSet, s2: DisjointSet) -> DisjointSet:
        count1 = s1.getMatches().size()
        count2 = s2.getMatches().size()
        if count1 <= count2:
            s2.merge(s1)
            return s2
        s1.merge(s2)
        return s1


class ConnectedComponents(SummaryBulkAggregation[DisjointSet, DisjointSet]):
    """ConnectedComponents<K, EV> (ConnectedComponents.java:41-54) on an MI355X.

    id_capacity / device: the u32 id range and GPU of the device-resident summary (no Java counterpart: the
    reference's HashMap grows on demand). group: optional distributed.ForestGroup for multi-GPU runs.
    """

    def __init__(self, mergeWindowTime: int, id_capacity: int, device: int = 0, group=None,
                 summary_factory=None):
        factory = summary_factory or (lambda: DisjointSet(id_capacity, device))
        super().__init__(UpdateCC(), CombineCC(), factory, mergeWindowTime, False, group=group)
        self.id_capacity = id_capacity
        self.device = device

    def run(self, edgeStream) -> Iterator[DisjointSet]:
        """Fused form of SummaryBulkAggregation.run for CC.

        With transientState=false the running summary after window w is CombineCC(window partials, summary),
        whose partition is that of ``summary ∪ edges(w)``. So each window's batches are folded straight into
        the running device forest (no per-window partial forest, no merge pass) and, with a group, the
        per-rank forests are combined over RCCL. The emitted object is the running summary itself (like the
        reference's Merger, which collects the same summary object every window).
        """
        summary: Optional[DisjointSet] = None
        for window_batches in edgeStream.windows(self.timeMillis):
            if summary is None:
                summary = self.getInitialValue()
            n = 0
            for batch in window_batches:
                if batch.n:
                    self.getUpdateFun().foldEdgeBatch(summary, batch)
                    n += batch.n
            if self.group is not None:
                self.group.merge_forest(summary)
            elif n == 0:
                continue
            yield summary


class ConnectedComponentsTree(SummaryTreeReduce[DisjointSet, DisjointSet]):
    """ConnectedComponentsTree<K, EV> (…/library/ConnectedComponentsTree.java:26-36): the CC summary with the
    window's partial forests combined by SummaryTreeReduce's pairwise tree (degree partitions per window).
    The emitted partition equals ConnectedComponents' (CombineCC is associative and commutative on it)."""

    def __init__(self, mergeWindowTime: int, id_capacity: int, degree: int = -1, device: int = 0):
        super().__init__(UpdateCC(), CombineCC(), lambda: DisjointSet(id_capacity, device), mergeWindowTime, False,
                         degree)
        self.id_capacity = id_capacity
        self.device = device
