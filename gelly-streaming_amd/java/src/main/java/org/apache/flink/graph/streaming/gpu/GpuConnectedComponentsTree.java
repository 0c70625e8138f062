// NOT COMPILED IN THIS IMAGE (no JDK): reference-side bridge, see gelly-streaming_amd/java/README.md
package org.apache.flink.graph.streaming.gpu;

import org.apache.flink.graph.streaming.SummaryTreeReduce;
import org.apache.flink.graph.streaming.library.ConnectedComponents;
import org.apache.flink.graph.streaming.summaries.DisjointSet;
import org.apache.flink.types.NullValue;

/**
 * ConnectedComponentsTree (…/library/ConnectedComponentsTree.java:26-36) with the MI355X summary: the same UpdateCC
 * fold and CombineCC combine over SummaryTreeReduce's pairwise tree of partial forests (…/SummaryTreeReduce.java:
 * 68-123); only the initial value is a GpuDisjointSet, so every pairwise combine is a device merge
 * (gcc_forest_merge). A job swaps `new ConnectedComponentsTree<>(t[, degree])` for
 * `new GpuConnectedComponentsTree(t[, degree], device, idCapacity[, longIds])`, nothing else.
 */
public class GpuConnectedComponentsTree extends SummaryTreeReduce<Long, NullValue, DisjointSet<Long>, DisjointSet<Long>> {
    private static final long serialVersionUID = 1L;

    public GpuConnectedComponentsTree(long mergeWindowTime, int degree, int device, int idCapacity, boolean longIds) {
        super(new ConnectedComponents.UpdateCC<Long>(), new ConnectedComponents.CombineCC<Long>(),
                new GpuDisjointSet(device, idCapacity, longIds), mergeWindowTime, false, degree);
    }

    public GpuConnectedComponentsTree(long mergeWindowTime, int degree, int device, int idCapacity) {
        this(mergeWindowTime, degree, device, idCapacity, false);
    }

    public GpuConnectedComponentsTree(long mergeWindowTime, int device, int idCapacity) {
        super(new ConnectedComponents.UpdateCC<Long>(), new ConnectedComponents.CombineCC<Long>(),
                new GpuDisjointSet(device, idCapacity, false), mergeWindowTime, false);
    }
}
