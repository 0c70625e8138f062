// NOT COMPILED IN THIS IMAGE (no JDK): reference-side bridge, see gelly-streaming_amd/java/README.md
package org.apache.flink.graph.streaming.gpu;

import com.esotericsoftware.kryo.Kryo;
import com.esotericsoftware.kryo.KryoSerializable;
import com.esotericsoftware.kryo.io.Input;
import com.esotericsoftware.kryo.io.Output;
import org.apache.flink.graph.streaming.summaries.DisjointSet;

import java.io.IOException;
import java.io.ObjectInputStream;
import java.io.ObjectOutputStream;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.AbstractMap;
import java.util.AbstractSet;
import java.util.ArrayList;
import java.util.Iterator;
import java.util.List;
import java.util.Map;
import java.util.NoSuchElementException;
import java.util.Set;
import java.util.TreeMap;

/**
 * DisjointSet&lt;Long&gt; (…/summaries/DisjointSet.java:30-154) whose state is a device-resident union-find forest on
 * an MI355X (libgelly_cc, include/gelly_cc.h). Ids must lie in [0, idCapacity); wider Long ids go through the
 * id dictionary (gcc_idmap_*) first.
 *
 * <p>The native handle is transient and created lazily on the task side: the instance the client passes to the
 * SummaryBulkAggregation constructor is Java-serialised into the job graph and copied per window by Flink, so it
 * must never hold device state. Per-edge {@link #union} calls (UpdateCC.foldEdges, ConnectedComponents.java:83-86)
 * append to the library's pinned staging slot through a direct ByteBuffer (no JNI call per edge); a full slot is
 * submitted with one call. Every read (getMatches, find, merge, toString, serialisation) submits first. Roots are
 * the components' minimum ids (min-id hooking): the partition equals the reference's, the chosen roots may not.
 */
public class GpuDisjointSet extends DisjointSet<Long> implements KryoSerializable {
    private static final long serialVersionUID = 1L;

    private int device;
    private int idCapacity;
    private transient long handle;          // gcc_forest*, 0 until first use on the task side
    private transient ByteBuffer stage;     // the current pinned staging slot (little-endian u32 pairs)
    private transient int staged;           // pairs appended since the last submit
    private transient int[] labelView;      // lazy host copy of the canonical labels
    private byte[] pendingState;            // restored bytes not yet folded into a forest (lazy, like the handle)

    public GpuDisjointSet() {}  // Kryo

    public GpuDisjointSet(int device, int idCapacity) {
        this.device = device;
        this.idCapacity = idCapacity;
    }

    private long h() {
        if (handle == 0) {
            handle = Gcc.create(device, idCapacity);
            if (pendingState != null) {
                Gcc.deserialize(handle, pendingState);
                pendingState = null;
            }
        }
        return handle;
    }

    private int id(Long e) {
        final long v = e;
        if (v < 0 || v >= idCapacity) throw new GccException(-1, "vertex id " + v + " outside [0, " + idCapacity + ")");
        return (int) v;
    }

    private void append(int u, int v) {
        if (stage == null) stage = Gcc.staging(h()).order(ByteOrder.LITTLE_ENDIAN);
        stage.putInt(8 * staged, u);
        stage.putInt(8 * staged + 4, v);
        labelView = null;
        if (++staged == stage.capacity() / 8) submit();
    }

    /** Hand the staged edges to the device (async); the library switches to its other staging slot. */
    private void submit() {
        if (staged > 0) {
            Gcc.submit(h(), staged);
            staged = 0;
            stage = null;
        }
    }

    private int[] labels() {
        submit();
        if (labelView == null) {
            labelView = new int[idCapacity];
            Gcc.labels(h(), labelView);
        }
        return labelView;
    }

    /** DisjointSet.makeSet (:58-61) = union(e, e). */
    @Override
    public void makeSet(Long e) {
        final int x = id(e);
        append(x, x);
    }

    /** DisjointSet.union (:97-123), staged. */
    @Override
    public void union(Long e1, Long e2) {
        append(id(e1), id(e2));
    }

    /** DisjointSet.find (:71-85): the component's minimum id, null if e was never seen (:72-74). */
    @Override
    public Long find(Long e) {
        final long v = e;
        if (v < 0 || v >= idCapacity) return null;
        final int r = labels()[(int) v];
        return r == -1 ? null : (long) (r & 0xffffffffL);
    }

    /** DisjointSet.merge (:132-136): this := this ∪ other; CombineCC.reduce calls it smaller-into-larger. */
    @Override
    public void merge(DisjointSet<Long> other) {
        if (other instanceof GpuDisjointSet) {
            final GpuDisjointSet o = (GpuDisjointSet) other;
            o.submit();
            submit();
            Gcc.merge(h(), o.h());
            labelView = null;
        } else {  // a heap DisjointSet: its (key, parent) pairs generate its partition
            for (Map.Entry<Long, Long> kv : other.getMatches().entrySet()) union(kv.getKey(), kv.getValue());
        }
    }

    /**
     * DisjointSet.getMatches (:49-51): a read-only Map view, key set = the vertices seen, value = the canonical
     * root. size() is gcc_forest_size (no host copy), which is all CombineCC.reduce (ConnectedComponents.java:
     * 117-118) reads; FlattenSet (ConnectedComponentsExample.java:148-155) iterates keySet() and calls find().
     */
    @Override
    public Map<Long, Long> getMatches() {
        return new MatchesView();
    }

    private final class MatchesView extends AbstractMap<Long, Long> {
        @Override
        public int size() {
            submit();
            return (int) Gcc.size(h());
        }

        @Override
        public boolean containsKey(Object k) {
            return k instanceof Long && find((Long) k) != null;
        }

        @Override
        public Long get(Object k) {
            return k instanceof Long ? find((Long) k) : null;
        }

        @Override
        public Set<Map.Entry<Long, Long>> entrySet() {
            final int[] lab = labels();
            return new AbstractSet<Map.Entry<Long, Long>>() {
                @Override
                public int size() {
                    return MatchesView.this.size();
                }

                @Override
                public Iterator<Map.Entry<Long, Long>> iterator() {
                    return new Iterator<Map.Entry<Long, Long>>() {
                        int next = advance(0);

                        int advance(int i) {
                            while (i < lab.length && lab[i] == -1) ++i;
                            return i;
                        }

                        public boolean hasNext() {
                            return next < lab.length;
                        }

                        public Map.Entry<Long, Long> next() {
                            if (next >= lab.length) throw new NoSuchElementException();
                            final Map.Entry<Long, Long> e =
                                    new SimpleImmutableEntry<>((long) next, (long) (lab[next] & 0xffffffffL));
                            next = advance(next + 1);
                            return e;
                        }
                    };
                }
            };
        }
    }

    /** DisjointSet.toString (:139-153): {root=[members...], ...}, roots = minimum ids, in id order. */
    @Override
    public String toString() {
        final int[] lab = labels();
        final TreeMap<Long, List<Long>> groups = new TreeMap<>();
        for (int v = 0; v < lab.length; ++v)
            if (lab[v] != -1) groups.computeIfAbsent(lab[v] & 0xffffffffL, k -> new ArrayList<>()).add((long) v);
        return groups.toString();
    }

    /** Back to the empty initial value (Merger with transientState, SummaryAggregation.java:113-115). */
    public void reset() {
        staged = 0;
        stage = null;
        labelView = null;
        pendingState = null;
        if (handle != 0) Gcc.reset(handle);
    }

    /** Release the device forest (also done by finalize; Java 8 has no Cleaner). */
    public void close() {
        if (handle != 0) {
            Gcc.destroy(handle);
            handle = 0;
        }
    }

    @Override
    protected void finalize() throws Throwable {
        close();
        super.finalize();
    }

    // ---- serialisation: the serialized summary of include/gelly_cc.h (Merger.snapshotState / restoreState,
    // SummaryAggregation.java:127-135, and the Kryo copies Flink makes of every window's accumulator) -----------

    private byte[] state() {
        if (handle == 0) return pendingState;  // never used on this task: whatever was restored, if anything
        submit();
        return Gcc.serialize(handle);
    }

    private void writeObject(ObjectOutputStream out) throws IOException {
        out.defaultWriteObject();  // device, idCapacity (pendingState is replaced below)
        out.writeObject(state());
    }

    private void readObject(ObjectInputStream in) throws IOException, ClassNotFoundException {
        in.defaultReadObject();
        pendingState = (byte[]) in.readObject();
    }

    @Override
    public void write(Kryo kryo, Output output) {
        output.writeInt(device);
        output.writeInt(idCapacity);
        final byte[] s = state();
        output.writeInt(s == null ? -1 : s.length);
        if (s != null) output.writeBytes(s);
    }

    @Override
    public void read(Kryo kryo, Input input) {
        device = input.readInt();
        idCapacity = input.readInt();
        final int n = input.readInt();
        pendingState = n < 0 ? null : input.readBytes(n);
    }
}
