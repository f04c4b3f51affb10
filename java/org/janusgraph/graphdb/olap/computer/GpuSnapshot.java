// Copyright 2026 JanusGraph Authors
// SPDX-License-Identifier: Apache-2.0
package org.janusgraph.graphdb.olap.computer;

import org.apache.tinkerpop.gremlin.structure.Direction;
import org.janusgraph.core.EdgeLabel;
import org.janusgraph.core.JanusGraphException;
import org.janusgraph.core.PropertyKey;
import org.janusgraph.core.schema.JanusGraphManagement;
import org.janusgraph.diskstorage.Entry;
import org.janusgraph.diskstorage.EntryList;
import org.janusgraph.diskstorage.StaticBuffer;
import org.janusgraph.diskstorage.keycolumnvalue.SliceQuery;
import org.janusgraph.diskstorage.keycolumnvalue.scan.ScanJob;
import org.janusgraph.diskstorage.keycolumnvalue.scan.ScanMetrics;
import org.janusgraph.diskstorage.keycolumnvalue.scan.StandardScanner;
import org.janusgraph.diskstorage.util.BufferUtil;
import org.janusgraph.graphdb.database.EdgeSerializer;
import org.janusgraph.graphdb.database.StandardJanusGraph;
import org.janusgraph.graphdb.idmanagement.IDManager;
import org.janusgraph.graphdb.internal.InternalRelationType;
import org.janusgraph.graphdb.olap.VertexJobConverter;
import org.janusgraph.graphdb.relations.RelationCache;
import org.janusgraph.graphdb.transaction.StandardJanusGraphTx;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.Collections;
import java.util.Date;
import java.util.List;
import java.util.Map;
import java.util.UUID;
import java.util.concurrent.atomic.AtomicInteger;

/**
 * The once-per-computer CSR snapshot, taken with the same edgestore scan Fulgora runs every superstep
 * (Backend.buildEdgeScanJob, janusgraph-core/.../diskstorage/Backend.java:377-396, driving
 * StandardScannerExecutor.run, diskstorage/keycolumnvalue/scan/StandardScannerExecutor.java:97-216).
 * Rows are NOT decoded here: each row key and the raw bytes of its EntryList are packed into direct
 * buffers and handed to libjanusgpu in chunks (jg_builder_add_rows), which decodes them on the GPU
 * (EdgeSerializer.parseRelation, key filter and ghost rule of VertexJobConverter.process,
 * graphdb/olap/VertexJobConverter.java:122-151,174-177) while this thread scans the next chunk.
 *
 * ShortestDistanceVertexProgram also needs the Integer edge weight, which lives in the entry's value
 * after the ids as (inline key id, value) pairs in key-id order (EdgeSerializer.writeRelation,
 * graphdb/database/EdgeSerializer.java:294-302). Where the schema allows (no edge label with signature
 * keys, the weight key in no sort key, every property key below the weight key of a type with a known
 * length) the weight is decoded on the GPU too (jg_builder_set_weight_key). Otherwise every OUT edge entry
 * of a visible row is parsed here with the graph's own EdgeSerializer and its weight sent along
 * (WeightReader). Either way an edge without an Integer weight gets JanusGpu.WEIGHT_ABSENT, which fails the
 * run only if a message crosses the edge, as Fulgora's edge function does.
 */
final class GpuSnapshot implements ScanJob {

    /** Every column of a row: the VertexExists property first, then the other relations. */
    static final SliceQuery ALL_ENTRIES = new SliceQuery(BufferUtil.zeroBuffer(1), BufferUtil.oneBuffer(4));

    // Chunk limits: direct buffers stay far below 2 GiB, and a chunk's copy and decode on the GPU
    // overlap the scan of the next one.  A single row larger than a chunk gets a chunk of its own.
    private static final int CHUNK_BYTES = 64 << 20;
    private static final int CHUNK_ENTRIES = 4 << 20;
    private static final int CHUNK_ROWS = 1 << 20;

    private static final AtomicInteger JOBS = new AtomicInteger();

    private final long builder;
    private final WeightReader weights;
    private ByteBuffer keys, rowOff, bytes, entryOff, valuePos, entryWeight;
    private int nrows, nentries, nbytes;

    private GpuSnapshot(long builder, WeightReader weights) {
        this.builder = builder;
        this.weights = weights;
        allocate(CHUNK_BYTES, CHUNK_ENTRIES, CHUNK_ROWS);
    }

    private static ByteBuffer direct(long bytes) {
        if (bytes > Integer.MAX_VALUE) throw new JanusGraphException("GPU snapshot chunk above 2 GiB");
        return ByteBuffer.allocateDirect((int) Math.max(bytes, 8)).order(ByteOrder.nativeOrder());
    }

    private void allocate(int maxBytes, int maxEntries, int maxRows) {
        keys = direct(8L * maxRows);
        rowOff = direct(8L * (maxRows + 1));
        bytes = direct(maxBytes);
        entryOff = direct(8L * (maxEntries + 1));
        valuePos = direct(4L * maxEntries);
        entryWeight = weights == null ? null : direct(4L * maxEntries);
        reset();
    }

    private void reset() {
        keys.clear();
        rowOff.clear();
        bytes.clear();
        entryOff.clear();
        valuePos.clear();
        if (entryWeight != null) entryWeight.clear();
        nrows = nentries = nbytes = 0;
        rowOff.putLong(0L);
        entryOff.putLong(0L);
    }

    @Override
    public List<SliceQuery> getQueries() {
        return Collections.singletonList(ALL_ENTRIES); // one query: no grounding slice needed (:104-116)
    }

    @Override
    public void process(StaticBuffer key, Map<SliceQuery, EntryList> entries, ScanMetrics metrics) {
        final EntryList row = entries.get(ALL_ENTRIES);
        if (row == null || row.isEmpty()) return;
        int rowBytes = 0;
        for (Entry e : row) rowBytes += e.length();
        final int rowEntries = row.size();
        if (nrows > 0 && (nbytes + rowBytes > bytes.capacity() || nentries + rowEntries > valuePos.capacity() / 4
                || nrows + 1 > keys.capacity() / 8)) {
            flush();
        }
        if (rowBytes > bytes.capacity() || rowEntries > valuePos.capacity() / 4) { // a hub row: a chunk of its own
            allocate(Math.max(rowBytes, CHUNK_BYTES), Math.max(rowEntries, CHUNK_ENTRIES), CHUNK_ROWS);
        }
        keys.putLong(key.getLong(0)); // the 8-byte big-endian row key as an unsigned value (IDManager.getKey)
        // host weights only for rows the decoder keeps: VertexJobConverter.getKeyFilter drops invisible rows
        // (olap/VertexJobConverter.java:169-171) before anything is parsed
        final boolean parseWeights = entryWeight != null && weights.visible(key);
        for (Entry e : row) {
            final byte[] b = e.as(StaticBuffer.ARRAY_FACTORY); // column then value
            bytes.put(b);
            nbytes += b.length;
            entryOff.putLong(nbytes);
            valuePos.putInt(e.getValuePosition());
            if (entryWeight != null) entryWeight.putInt(parseWeights ? weights.weight(e) : JanusGpu.WEIGHT_ABSENT);
        }
        nentries += rowEntries;
        ++nrows;
        rowOff.putLong(nentries);
    }

    /** Hands the packed rows to the library (it copies them before returning). */
    void flush() {
        if (nrows == 0) return;
        JanusGpu.check(JanusGpu.builderAddRows(builder, keys, nrows, rowOff, bytes, nbytes, entryOff, valuePos,
            entryWeight, nentries));
        if (bytes.capacity() > CHUNK_BYTES || valuePos.capacity() > 4 * CHUNK_ENTRIES) {
            allocate(CHUNK_BYTES, CHUNK_ENTRIES, CHUNK_ROWS); // back to regular chunks after a hub row
        } else {
            reset();
        }
    }

    @Override
    public GpuSnapshot clone() {
        return this; // one processor thread (setNumProcessingThreads(1)): rows arrive in key order
    }

    /** Reads the Integer weight property of the edge an entry stores (ShortestDistanceVertexProgram.java:69),
     *  on the host: the fallback when the schema rules out the GPU decode (see the class comment). */
    static final class WeightReader {
        private final StandardJanusGraphTx tx;
        private final EdgeSerializer serializer;
        private final IDManager idManager;
        private final long keyId;

        WeightReader(StandardJanusGraph graph, String weightProperty) {
            tx = VertexJobConverter.startTransaction(graph);
            serializer = graph.getEdgeSerializer();
            idManager = graph.getIDManager();
            keyId = tx.containsPropertyKey(weightProperty) ? tx.getPropertyKey(weightProperty).longId() : -1L;
        }

        boolean visible(StaticBuffer key) {
            return !IDManager.VertexIDType.Invisible.is(idManager.getKeyID(key));
        }

        int weight(Entry e) {
            if (serializer.parseDirection(e) != Direction.OUT) return JanusGpu.WEIGHT_ABSENT; // header only
            final RelationCache rc = serializer.parseRelation(e, false, tx);
            if (keyId < 0 || !tx.getExistingRelationType(rc.typeId).isEdgeLabel()) return JanusGpu.WEIGHT_ABSENT;
            final Object v = rc.get(keyId);
            if (!(v instanceof Integer)) return JanusGpu.WEIGHT_ABSENT; // absent, or not an Integer: the <Integer> cast throws when crossed
            final int w = (Integer) v;
            if (w == JanusGpu.WEIGHT_ABSENT)
                throw new JanusGraphException("GPU computer: an edge weight equals Integer.MIN_VALUE, the absent-weight marker");
            return w;
        }

        void close() {
            if (tx.isOpen()) tx.rollback();
        }
    }

    /** JG_PROP_* codes of include/janusgpu.h for a property key's data type; 0: length unknown to the GPU. */
    static byte propertyType(PropertyKey key) {
        final Class<?> t = key.dataType();
        if (t == Byte.class) return 1;
        if (t == Short.class) return 2;
        if (t == Integer.class) return 3;
        if (t == Long.class) return 4;
        if (t == Character.class) return 5;
        if (t == Boolean.class) return 6;
        if (t == Date.class) return 7;
        if (t == Float.class) return 8;
        if (t == Double.class) return 9;
        if (t == UUID.class) return 10;
        if (t == String.class) return 11;
        return 0;
    }

    /**
     * Sends the weight key and the property-key table for the GPU weight decode and returns true, or
     * returns false when the schema needs the host parse: an edge label with signature keys (their values
     * precede the inline pairs without ids), the weight key in a label's sort key (stored in the column),
     * or a key of unknown value length below the weight key.
     */
    private static boolean deviceWeights(long builder, JanusGraphManagement mgmt, List<EdgeLabel> labels,
                                         String weightProperty) {
        final PropertyKey wk = mgmt.getPropertyKey(weightProperty);
        for (EdgeLabel l : labels) {
            final InternalRelationType t = (InternalRelationType) l;
            if (t.getSignature().length > 0) return false;
            if (wk != null) for (long k : t.getSortKey()) if (k == wk.longId()) return false;
        }
        final List<PropertyKey> keys = new ArrayList<>();
        for (PropertyKey k : mgmt.getRelationTypes(PropertyKey.class)) {
            if (wk != null && k.longId() < wk.longId() && propertyType(k) == 0) return false;
            keys.add(k);
        }
        final ByteBuffer ids = direct(8L * keys.size()), types = direct(keys.size());
        for (PropertyKey k : keys) {
            ids.putLong(IDManager.stripRelationTypePadding(k.longId()));
            types.put(propertyType(k));
        }
        // no such key: inline id 0 with an empty table, every weight absent
        final long weightKey = wk == null ? 0L : IDManager.stripRelationTypePadding(wk.longId());
        JanusGpu.check(JanusGpu.builderSetWeightKey(builder, weightKey, ids, types, wk == null ? 0 : keys.size()));
        return true;
    }

    /** Multiplicity codes of include/janusgpu.h (jg_decode_edges): 0 MULTI, 1 SIMPLE, 2 ONE2MANY,
     *  3 MANY2ONE, 4 ONE2ONE (core/Multiplicity.java:35-90). */
    private static byte multiplicityCode(EdgeLabel label) {
        switch (label.multiplicity()) {
            case SIMPLE: return 1;
            case ONE2MANY: return 2;
            case MANY2ONE: return 3;
            case ONE2ONE: return 4;
            default: return 0;
        }
    }

    /**
     * Scans the edgestore into a device graph with the adjacencies `flags`. weightProperty != null
     * also gives every edge its weight (ShortestDistanceVertexProgram): decoded on the GPU, or parsed here. queryLimit > 0 builds what
     * Fulgora's programs read under its slice cap (inEntries: JanusGpu.DIR_IN or DIR_OUT, see
     * jg_builder_set_query_limit). Returns the graph handle; its vertex order is the scan's row order
     * (read it with JanusGpu.graphVertexIds).
     */
    static long scan(StandardJanusGraph graph, long ctx, int flags, String weightProperty, long queryLimit,
                     int inEntries) {
        final long[] h = new long[1];
        JanusGpu.check(JanusGpu.builderCreate(ctx, h));
        final long builder = h[0];
        WeightReader weights = null;
        try {
            // Fulgora's per-row slice cap (QueryContainer.java:42,133), reproduced in the decode
            JanusGpu.check(JanusGpu.builderSetQueryLimit(builder, queryLimit, inEntries));
            final List<EdgeLabel> labels = new ArrayList<>();
            final JanusGraphManagement mgmt = graph.openManagement();
            try {
                for (EdgeLabel l : mgmt.getRelationTypes(EdgeLabel.class)) labels.add(l);
                final ByteBuffer typeIds = direct(8L * labels.size());
                final ByteBuffer typeMult = direct(labels.size());
                for (EdgeLabel l : labels) {
                    typeIds.putLong(l.longId());
                    typeMult.put(multiplicityCode(l));
                }
                final int partitionBits = Long.numberOfTrailingZeros(graph.getIDManager().getPartitionBound());
                JanusGpu.check(JanusGpu.builderSetSchema(builder, typeIds, typeMult, labels.size(), partitionBits));
                if (weightProperty != null && !deviceWeights(builder, mgmt, labels, weightProperty))
                    weights = new WeightReader(graph, weightProperty);
            } finally {
                mgmt.rollback();
            }
            final GpuSnapshot job = new GpuSnapshot(builder, weights);
            final StandardScanner.Builder scan = graph.getBackend().buildEdgeScanJob();
            scan.setJobId("gpu-snapshot#" + JOBS.incrementAndGet());
            scan.setNumProcessingThreads(1);
            scan.setJob(job);
            final ScanMetrics metrics = scan.execute().get();
            if (metrics.get(ScanMetrics.Metric.FAILURE) > 0) {
                throw new JanusGraphException("Failed to snapshot [" + metrics.get(ScanMetrics.Metric.FAILURE)
                    + "] vertex rows for the GPU. Computer is aborting.");
            }
            job.flush(); // the scan's last partial chunk (the scan thread is done: Future.get())
            JanusGpu.check(JanusGpu.builderFinish(builder, flags, h));
            return h[0];
        } catch (JanusGraphException e) {
            throw e;
        } catch (Exception e) {
            throw new JanusGraphException("GPU snapshot scan failed. Computer is aborting.", e);
        } finally {
            if (weights != null) weights.close();
            JanusGpu.builderDestroy(builder);
        }
    }

    /** The graph's vertex ids in output order, as one long[] (n < 2^31 by the library's limit). */
    static long[] vertexIds(long graph) {
        final long[] info = new long[8];
        JanusGpu.check(JanusGpu.graphInfo(graph, info));
        final long n = info[0];
        final long[] vid = new long[(int) n];
        final int chunk = 1 << 24;
        final ByteBuffer buf = direct(8L * Math.min(n, chunk));
        for (long off = 0; off < n; off += chunk) {
            final int cnt = (int) Math.min(chunk, n - off);
            buf.clear();
            JanusGpu.check(JanusGpu.graphVertexIds(graph, off, cnt, buf));
            buf.asLongBuffer().get(vid, (int) off, cnt);
        }
        return vid;
    }
}
