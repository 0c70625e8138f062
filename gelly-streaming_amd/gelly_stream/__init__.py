"""gelly_stream — MI355X-native streaming connected components (gelly-streaming's CC hot path).

Public surface mirrors the reference's operator API (`…/` = src/main/java/org/apache/flink/graph/streaming/):
  DisjointSet              …/summaries/DisjointSet.java       (device-resident union-find forest)
  ConnectedComponents      …/library/ConnectedComponents.java (UpdateCC fold + CombineCC combine)
  SummaryBulkAggregation   …/SummaryBulkAggregation.java      (window fold -> combine -> Merger)
  EdgesFold                …/EdgesFold.java
  SimpleEdgeStream         …/SimpleEdgeStream.java            (constructor + aggregate())
  LongDisjointSet          DisjointSet<Long> for ids anywhere in the Long range (dense relabel, IdDictionary)
All device work goes through libgelly_cc.so (include/gelly_cc.h); there is no CPU fallback.
"""
from .aggregation import (EdgeBatch, EdgesFold, Merger, ReduceFunction, SummaryAggregation, SummaryBulkAggregation,
                          SummaryTreeReduce)
from .bipartite import BipartitenessCheck, Candidates, LiteralBipartitenessCheck, LiteralCandidates, SignedVertex
from .edgestream import SimpleEdgeStream
from .library import CombineCC, ConnectedComponents, ConnectedComponentsTree, UpdateCC
from .longids import IdDictionary, LongDisjointSet
from .native import UNSEEN, GellyCCError, device_count
from .summaries import DisjointSet

__all__ = [
    "BipartitenessCheck", "Candidates", "CombineCC", "ConnectedComponents", "ConnectedComponentsTree", "DisjointSet",
    "EdgeBatch", "EdgesFold", "GellyCCError", "IdDictionary", "LiteralBipartitenessCheck", "LiteralCandidates",
    "LongDisjointSet", "Merger", "ReduceFunction",
    "SignedVertex", "SimpleEdgeStream", "SummaryAggregation", "SummaryBulkAggregation", "SummaryTreeReduce", "UNSEEN",
    "UpdateCC", "device_count",
]
