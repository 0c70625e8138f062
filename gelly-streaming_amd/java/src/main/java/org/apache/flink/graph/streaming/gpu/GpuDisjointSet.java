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
 * an MI355X (libgelly_cc, include/gelly_cc.h).
 *
 * <p>Two id modes. Direct ({@code longIds == false}): ids are the forest's own u32 ids and must lie in
 * [0, idCapacity); per-edge {@link #union} calls append to the library's pinned staging slot through a direct
 * ByteBuffer (no JNI call per edge) and a full slot is submitted with one call. Long ids ({@code longIds == true}):
 * any Long, as the reference's {@code DisjointSet<K>} takes (DisjointSet.java:30-34, ConnectedComponentsExample.java:
 * 60); edges collect in a long[] and a full batch is mapped by the id dictionary (gcc_idmap_*) straight into the
 * staging slot and submitted (Gcc.submitLong). Dense ids follow first sight, so canonical labels are taken as the
 * minimum ORIGINAL id of each component (gcc_idmap_canonical), which is the reference's min-id partition in signed
 * Long order. At most idCapacity distinct ids.
 *
 * <p>The native handles are transient and created lazily on the task side: the instance the client passes to the
 * SummaryBulkAggregation constructor is Java-serialised into the job graph and copied per window by Flink, so it
 * must never hold device state. Every read (getMatches, find, merge, toString, serialisation) submits first. Roots
 * are the components' minimum ids (min-id hooking): the partition equals the reference's, the chosen roots may not.
 */
public class GpuDisjointSet extends DisjointSet<Long> implements KryoSerializable {
    private static final long serialVersionUID = 2L;

    private int device;
    private int idCapacity;
    private boolean longIds;
    private transient long handle;          // gcc_forest*, 0 until first use on the task side
    private transient long idmap;           // gcc_idmap* (longIds only), created with the handle
    private transient ByteBuffer stage;     // direct ids: the current pinned staging slot (little-endian u32 pairs)
    private transient int staged;           // pairs appended since the last submit
    private transient int slotPairs;        // pairs per staging slot
    private transient long[] pend;          // Long ids: pairs not yet mapped and submitted
    private transient int[] labelView;      // direct ids: lazy host copy of the canonical labels
    private transient long[] canonView;     // Long ids: lazy per-dense-id canonical (min original) ids
    private transient long[] idView;        // Long ids: lazy dense -> original id
    private transient byte[] pendingState;  // restored bytes not yet folded into a forest (lazy, like the handle)

    public GpuDisjointSet() {}  // Kryo

    public GpuDisjointSet(int device, int idCapacity) {
        this(device, idCapacity, false);
    }

    /** longIds: accept any Long id (at most idCapacity distinct ones) through the id dictionary. */
    public GpuDisjointSet(int device, int idCapacity, boolean longIds) {
        this.device = device;
        this.idCapacity = idCapacity;
        this.longIds = longIds;
    }

    private long h() {
        if (handle == 0) {
            handle = Gcc.create(device, idCapacity);
            if (longIds) idmap = Gcc.idmapCreate(idCapacity);
            if (pendingState != null) {
                final byte[] s = pendingState;
                pendingState = null;
                restore(s);
            }
        }
        return handle;
    }

    private int id(Long e) {
        final long v = e;
        if (v < 0 || v >= idCapacity) throw new GccException(-1, "vertex id " + v + " outside [0, " + idCapacity + ")");
        return (int) v;
    }

    private void invalidate() {
        labelView = null;
        canonView = null;
        idView = null;
    }

    private void append(int u, int v) {
        if (stage == null) {
            stage = Gcc.staging(h()).order(ByteOrder.LITTLE_ENDIAN);
            slotPairs = stage.capacity() / 8;
        }
        stage.putInt(8 * staged, u);
        stage.putInt(8 * staged + 4, v);
        invalidate();
        if (++staged == slotPairs) submit();
    }

    private void appendLong(long u, long v) {
        if (pend == null) {
            h();
            slotPairs = Gcc.staging(handle).capacity() / 8;
            pend = new long[2 * slotPairs];
        }
        pend[2 * staged] = u;
        pend[2 * staged + 1] = v;
        invalidate();
        if (++staged == slotPairs) submit();
    }

    /** Hand the staged edges to the device (async); the library switches to its other staging slot. */
    private void submit() {
        if (staged == 0) return;
        if (longIds) Gcc.submitLong(h(), idmap, pend, staged);
        else Gcc.submit(h(), staged);
        staged = 0;
        stage = null;
    }

    private int[] labels() {
        submit();
        if (labelView == null) {
            labelView = new int[idCapacity];
            Gcc.labels(h(), labelView);
        }
        return labelView;
    }

    private long[] canon() {
        submit();
        if (canonView == null) canonView = Gcc.canonical(h(), idmap);
        return canonView;
    }

    private long[] ids() {
        submit();
        if (idView == null) idView = Gcc.idmapIds(idmap);
        return idView;
    }

    /** DisjointSet.makeSet (:58-61) = union(e, e). */
    @Override
    public void makeSet(Long e) {
        union(e, e);
    }

    /** DisjointSet.union (:97-123), staged. */
    @Override
    public void union(Long e1, Long e2) {
        if (longIds) appendLong(e1, e2);
        else append(id(e1), id(e2));
    }

    /** DisjointSet.find (:71-85): the component's minimum id, null if e was never seen (:72-74). */
    @Override
    public Long find(Long e) {
        if (longIds) {
            submit();
            h();
            final int d = Gcc.idmapLookup(idmap, e);
            return d < 0 ? null : canon()[d];
        }
        final long v = e;
        if (v < 0 || v >= idCapacity) return null;
        final int r = labels()[(int) v];
        return r == -1 ? null : (long) (r & 0xffffffffL);
    }

    /** DisjointSet.merge (:132-136): this := this ∪ other; CombineCC.reduce calls it smaller-into-larger. */
    @Override
    public void merge(DisjointSet<Long> other) {
        if (other instanceof GpuDisjointSet && !longIds && !((GpuDisjointSet) other).longIds) {
            final GpuDisjointSet o = (GpuDisjointSet) other;
            o.submit();
            submit();
            Gcc.merge(h(), o.h());  // device to device (any two GPUs)
            invalidate();
        } else if (other instanceof GpuDisjointSet && ((GpuDisjointSet) other).longIds) {
            // another dictionary: its (original id, canonical id) pairs generate its partition
            final GpuDisjointSet o = (GpuDisjointSet) other;
            final long[] oi = o.ids(), oc = o.canon();
            for (int d = 0; d < oi.length; ++d) union(oi[d], oc[d]);
        } else {  // a heap DisjointSet or a direct-id forest: its (key, parent) pairs generate its partition
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
            if (longIds) {  // every mapped id has been submitted, so every dense id is seen
                final long[] oi = ids(), oc = canon();
                return new AbstractSet<Map.Entry<Long, Long>>() {
                    @Override
                    public int size() {
                        return oi.length;
                    }

                    @Override
                    public Iterator<Map.Entry<Long, Long>> iterator() {
                        return new Iterator<Map.Entry<Long, Long>>() {
                            int next = 0;

                            public boolean hasNext() {
                                return next < oi.length;
                            }

                            public Map.Entry<Long, Long> next() {
                                if (next >= oi.length) throw new NoSuchElementException();
                                final Map.Entry<Long, Long> e = new SimpleImmutableEntry<>(oi[next], oc[next]);
                                ++next;
                                return e;
                            }
                        };
                    }
                };
            }
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
        final TreeMap<Long, List<Long>> groups = new TreeMap<>();
        if (longIds) {
            final long[] oi = ids(), oc = canon();
            final TreeMap<Long, Long> sorted = new TreeMap<>();
            for (int d = 0; d < oi.length; ++d) sorted.put(oi[d], oc[d]);
            for (Map.Entry<Long, Long> kv : sorted.entrySet())
                groups.computeIfAbsent(kv.getValue(), k -> new ArrayList<>()).add(kv.getKey());
            return groups.toString();
        }
        final int[] lab = labels();
        for (int v = 0; v < lab.length; ++v)
            if (lab[v] != -1) groups.computeIfAbsent(lab[v] & 0xffffffffL, k -> new ArrayList<>()).add((long) v);
        return groups.toString();
    }

    /** Back to the empty initial value (Merger with transientState, SummaryAggregation.java:113-115). */
    public void reset() {
        staged = 0;
        stage = null;
        invalidate();
        pendingState = null;
        if (handle != 0) Gcc.reset(handle);
        if (idmap != 0) {  // a fresh dictionary: dense ids restart at 0 with the fresh forest
            Gcc.idmapDestroy(idmap);
            idmap = Gcc.idmapCreate(idCapacity);
        }
    }

    /** Release the device forest and the dictionary (also done by finalize; Java 8 has no Cleaner). */
    public void close() {
        if (handle != 0) {
            Gcc.destroy(handle);
            handle = 0;
        }
        if (idmap != 0) {
            Gcc.idmapDestroy(idmap);
            idmap = 0;
        }
    }

    @Override
    protected void finalize() throws Throwable {
        close();
        super.finalize();
    }

    // ---- serialisation: the serialized summary of include/gelly_cc.h (Merger.snapshotState / restoreState,
    // SummaryAggregation.java:127-135, and the Kryo copies Flink makes of every window's accumulator). Long ids:
    // [int n][n x long original ids, dense order][summary bytes]; restore maps the ids in that order (the same dense
    // ids) and then folds the summary. ---------------------------------------------------------------------------

    private byte[] state() {
        if (handle == 0) return pendingState;  // never used on this task: whatever was restored, if anything
        submit();
        final byte[] forest = Gcc.serialize(handle);
        if (!longIds) return forest;
        final long[] oi = ids();
        final ByteBuffer b = ByteBuffer.allocate(4 + 8 * oi.length + forest.length).order(ByteOrder.LITTLE_ENDIAN);
        b.putInt(oi.length);
        for (long x : oi) b.putLong(x);
        b.put(forest);
        return b.array();
    }

    private void restore(byte[] s) {
        if (!longIds) {
            Gcc.deserialize(handle, s);
            return;
        }
        final ByteBuffer b = ByteBuffer.wrap(s).order(ByteOrder.LITTLE_ENDIAN);
        final int n = b.getInt();
        if (n < 0 || n > idCapacity || b.remaining() < 8L * n) throw new GccException(-1, "bad serialized Long-id summary");
        final long[] oi = new long[n];
        for (int d = 0; d < n; ++d) oi[d] = b.getLong();
        // re-create dense ids 0..n-1 in the recorded order (self pairs fold nothing but makeSet)
        for (int d = 0; d < n; ++d) appendLong(oi[d], oi[d]);
        submit();
        final byte[] forest = new byte[b.remaining()];
        b.get(forest);
        Gcc.deserialize(handle, forest);
        invalidate();
    }

    private void writeObject(ObjectOutputStream out) throws IOException {
        out.defaultWriteObject();  // device, idCapacity, longIds (the state is transient: written once, below)
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
        output.writeBoolean(longIds);
        final byte[] s = state();
        output.writeInt(s == null ? -1 : s.length);
        if (s != null) output.writeBytes(s);
    }

    @Override
    public void read(Kryo kryo, Input input) {
        device = input.readInt();
        idCapacity = input.readInt();
        longIds = input.readBoolean();
        final int n = input.readInt();
        pendingState = n < 0 ? null : input.readBytes(n);
    }
}
