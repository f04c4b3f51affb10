// Copyright 2026 JanusGraph Authors
// SPDX-License-Identifier: Apache-2.0
package org.janusgraph.graphdb.olap.computer;

import org.janusgraph.core.JanusGraphException;

import java.nio.ByteBuffer;

/**
 * JNI binding of libjanusgpu (include/janusgpu.h). Every native method returns the C status code
 * (0 = ok, &lt; 0 = error class); {@link #check(int)} turns a failure into a JanusGraphException
 * carrying jg_last_error(), in the style of FulgoraGraphComputer's "Computer is aborting" errors
 * (janusgraph-core/.../olap/computer/FulgoraGraphComputer.java:269-286).
 *
 * Arrays cross the boundary as direct ByteBuffers in native byte order (int64 ids and offsets, int32
 * weights / value positions, float64 / int64 outputs); handles are opaque longs. A direct buffer
 * holds at most 2 GiB, so snapshots go through the chunked builder (jg_builder_*) and outputs are
 * per-vertex arrays (n * 8 bytes). Java 8 target (pom.xml:112-113): JNI, not Panama.
 */
final class JanusGpu {
    /** JG_ABI_VERSION of include/janusgpu.h that these natives and their array layouts follow. */
    static final int ABI_VERSION = 3;

    static {
        System.loadLibrary("janusgpu_jni"); // links libjanusgpu.so
        if (abiVersion() != ABI_VERSION)
            throw new ExceptionInInitializerError("libjanusgpu ABI " + abiVersion() + ", GpuGraphComputer needs "
                + ABI_VERSION + ": rebuild libjanusgpu and libjanusgpu_jni");
    }

    static final int ADJ_OUT = 1, ADJ_IN = 2, ADJ_BOTH = 4;
    static final int DIR_OUT = 1, DIR_IN = 2, DIR_BOTH = 3;
    static final long DIST_ABSENT = Long.MIN_VALUE;    // JG_DIST_ABSENT
    static final int WEIGHT_ABSENT = Integer.MIN_VALUE; // JG_WEIGHT_ABSENT

    private JanusGpu() {
    }

    static native int abiVersion();
    static native String lastError();

    /** jg_ctx_create(devices, ndev, &ctx); handle written to out[0]. */
    static native int ctxCreate(int[] devices, long[] out);
    static native int ctxDestroy(long ctx);
    /** jg_ctx_trim: the device memory libjanusgpu caches for reuse goes back to the devices. */
    static native int ctxTrim(long ctx);
    /** jg_ctx_last_stats: supersteps, levels, build_ms, compute_ms, exchange_ms, kernel_ms, launches, bytes, edges. */
    static native int ctxLastStats(long ctx, double[] out9);

    /** jg_builder_create; handle written to out[0]. */
    static native int builderCreate(long ctx, long[] out);
    static native int builderDestroy(long builder);
    static native int builderAddVertices(long builder, ByteBuffer vid, long n);
    /** weight: int32 direct buffer or null (the same on every call). */
    static native int builderAddEdges(long builder, ByteBuffer src, ByteBuffer dst, ByteBuffer weight, long m);
    static native int builderSetSchema(long builder, ByteBuffer typeIds, ByteBuffer typeMult, int ntypes,
                                       int partitionBits);
    /** One scan chunk of whole rows: keys (int64), row entry offsets (int64, nrows + 1), entry bytes,
     *  entry offsets (int64, nentries + 1), value positions (int32), entry weights (int32 or null). */
    static native int builderAddRows(long builder, ByteBuffer rowKeys, long nrows, ByteBuffer rowEntryOff,
                                     ByteBuffer bytes, long nbytes, ByteBuffer entryOff, ByteBuffer valuePos,
                                     ByteBuffer entryWeight, long nentries);
    /** jg_builder_set_weight_key: the edges' Integer weight decoded on the GPU. weightKey and keyIds are inline
     *  ids (IDManager.stripRelationTypePadding), keyTypes the JG_PROP_* codes (int8). */
    static native int builderSetWeightKey(long builder, long weightKey, ByteBuffer keyIds, ByteBuffer keyTypes,
                                          int nkeys);
    /** jg_builder_set_query_limit: Fulgora's per-row slice cap (0: none); inEntries DIR_IN or DIR_OUT. */
    static native int builderSetQueryLimit(long builder, long limit, int inEntries);
    /** jg_builder_finish; graph handle written to out[0]. */
    static native int builderFinish(long builder, int flags, long[] out);

    static native int graphDestroy(long graph);
    /** jg_graph_info_get: vertices, edges, ghost edges, self loops, truncated vertices, max in, max out, bytes. */
    static native int graphInfo(long graph, long[] out8);
    /** jg_graph_vertex_ids(offset, count) into an int64 direct buffer. */
    static native int graphVertexIds(long graph, long offset, long count, ByteBuffer vidOut);

    static native int pageRank(long graph, double damping, long vertexCount, int iterations, ByteBuffer rankOut,
                               ByteBuffer edgeCountOut);
    static native int shortestDistance(long graph, long seedVid, int maxDepth, ByteBuffer distOut);
    static native int bfs(long graph, ByteBuffer sourceVids, int nsrc, int direction, int maxDepth, ByteBuffer depthOut);
    /** jg_bfs_rows: one int32 direct buffer of n depths per source (null: not wanted). */
    static native int bfsRows(long graph, ByteBuffer sourceVids, int nsrc, int direction, int maxDepth,
                              ByteBuffer[] depthRows);
    /** jg_bfs_keep: the traversal's depth rows (<= 64 sources) stay on the device for bfsKeptRow. */
    static native int bfsKeep(long graph, ByteBuffer sourceVids, int nsrc, int direction, int maxDepth);
    /** jg_bfs_kept_row: row s of the last bfsKeep into an int32 direct buffer of n depths. */
    static native int bfsKeptRow(long graph, int s, ByteBuffer depthOut);
    /** jg_bfs_kept_release: frees the kept rows before the graph goes. */
    static native int bfsKeptRelease(long graph);
    /** jg_graph_neighbors: rows (int64 output-order indices) -> offsets (int64, nrows + 1) and neighbours
     *  (int64 output-order indices; null: offsets only). */
    static native int graphNeighbors(long graph, int direction, ByteBuffer rows, long nrows, ByteBuffer offOut,
                                     ByteBuffer nbrOut);
    static native int connectedComponents(long graph, ByteBuffer componentVidOut, int[] iterationsOut);
    /** jg_combine_steps: sum/min/max MessageCombiner programs (OLAPTest.DegreeCounter family). */
    static native int combineSteps(long graph, int direction, int combiner, int int32Wrap, ByteBuffer init, int steps,
                                   ByteBuffer out, ByteBuffer receivedOut);

    static void check(int status) {
        if (status != 0) {
            throw new JanusGraphException(
                "GPU computer is aborting: libjanusgpu status " + status + ": " + lastError());
        }
    }
}
