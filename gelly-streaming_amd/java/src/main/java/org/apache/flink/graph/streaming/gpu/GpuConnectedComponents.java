// NOT COMPILED IN THIS IMAGE (no JDK): reference-side bridge, see gelly-streaming_amd/java/README.md
package org.apache.flink.graph.streaming.gpu;

import org.apache.flink.graph.streaming.SummaryBulkAggregation;
import org.apache.flink.graph.streaming.library.ConnectedComponents;
import org.apache.flink.graph.streaming.summaries.DisjointSet;
import org.apache.flink.types.NullValue;

/**
 * ConnectedComponents (…/library/ConnectedComponents.java:41-54) with the MI355X summary: the same UpdateCC fold and
 * CombineCC combine, the same SummaryBulkAggregation topology; only the initial value is a GpuDisjointSet. A job
 * swaps `new ConnectedComponents<>(t)` for `new GpuConnectedComponents(t, device, idCapacity)`, nothing else.
 */
public class GpuConnectedComponents extends SummaryBulkAggregation<Long, NullValue, DisjointSet<Long>, DisjointSet<Long>> {
    private static final long serialVersionUID = 1L;

    public GpuConnectedComponents(long mergeWindowTime, int device, int idCapacity) {
        this(mergeWindowTime, device, idCapacity, false);
    }

    /** longIds: vertex ids are any Long (at most idCapacity distinct ones), mapped by the id dictionary. */
    public GpuConnectedComponents(long mergeWindowTime, int device, int idCapacity, boolean longIds) {
        super(new ConnectedComponents.UpdateCC<Long>(), new ConnectedComponents.CombineCC<Long>(),
                new GpuDisjointSet(device, idCapacity, longIds), mergeWindowTime, false);
    }
}
