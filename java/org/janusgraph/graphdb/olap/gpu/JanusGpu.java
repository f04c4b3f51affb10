// Copyright 2026 JanusGraph Authors
// SPDX-License-Identifier: Apache-2.0
package org.janusgraph.graphdb.olap.gpu;

import java.nio.ByteBuffer;

/**
 * JNI binding of libjanusgpu (include/janusgpu.h). Every native method returns the C status code
 * (0 = ok, &lt; 0 = error class); {@link #check(int)} turns a failure into a JanusGraphException
 * carrying jg_last_error(), in the style of FulgoraGraphComputer's "Computer is aborting" errors
 * (janusgraph-core/.../olap/computer/FulgoraGraphComputer.java:269-286).
 *
 * Arrays cross the boundary as direct ByteBuffers in native byte order (int64 ids, int32 weights,
 * float64 / int64 / int32 outputs); handles are opaque longs. Java 8 target (pom.xml:112-113):
 * JNI, not Panama.
 */
final class JanusGpu {
    static {
        System.loadLibrary("janusgpu_jni"); // links libjanusgpu.so
    }

    static final int ADJ_OUT = 1, ADJ_IN = 2, ADJ_BOTH = 4;
    static final int DIR_OUT = 1, DIR_IN = 2, DIR_BOTH = 3;

    private JanusGpu() {
    }

    static native int abiVersion();
    static native String lastError();

    /** jg_ctx_create(devices, ndev, &ctx); handle written to out[0]. */
    static native int ctxCreate(int[] devices, long[] out);
    static native int ctxDestroy(long ctx);
    /** jg_ctx_last_stats: supersteps, levels, build_ms, compute_ms, exchange_ms, kernel_ms, launches, bytes, edges. */
    static native int ctxLastStats(long ctx, double[] out9);

    /** jg_graph_build; vid/src/dst: int64 direct buffers, weight: int32 direct buffer or null. */
    static native int graphBuild(long ctx, ByteBuffer vid, long n, ByteBuffer src, ByteBuffer dst, ByteBuffer weight,
                                 long m, int flags, long[] out);
    static native int graphDestroy(long graph);
    /** jg_graph_info_get: vertices, edges, ghost edges, self loops, truncated vertices, max in, max out, bytes. */
    static native int graphInfo(long graph, long[] out8);

    static native int pageRank(long graph, double damping, long vertexCount, int iterations, ByteBuffer rankOut,
                               ByteBuffer edgeCountOut);
    static native int shortestDistance(long graph, long seedVid, int maxDepth, ByteBuffer distOut);
    static native int bfs(long graph, ByteBuffer sourceVids, int nsrc, int direction, int maxDepth, ByteBuffer depthOut);
    static native int connectedComponents(long graph, ByteBuffer componentVidOut, int[] iterationsOut);

    /** jg_graph_build_edgestore: the snapshot from the scan's raw rows (StaticBuffer keys as longs, the
     *  EntryLists' bytes, entry offsets and value positions); out2 = {graph handle, |V|}. */
    static native int graphBuildEdgestore(long ctx, ByteBuffer rowKeys, long nrows, ByteBuffer rowEntryOff,
                                          ByteBuffer bytes, long nbytes, ByteBuffer entryOff, ByteBuffer valuePos,
                                          long nentries, ByteBuffer typeIds, ByteBuffer typeMult, int ntypes,
                                          int partitionBits, int flags, ByteBuffer vidOut, long[] out2);
    /** jg_combine_steps: sum/min/max MessageCombiner programs (OLAPTest.DegreeCounter family). */
    static native int combineSteps(long graph, int direction, int combiner, int int32Wrap, ByteBuffer init, int steps,
                                   ByteBuffer out, ByteBuffer receivedOut);
    /** jg_decode_edges: EdgeSerializer.parseRelation of raw entries on the GPU. */
    static native int decodeEdges(long ctx, ByteBuffer bytes, long nbytes, ByteBuffer entryOff, ByteBuffer valuePos,
                                  long n, ByteBuffer typeIds, ByteBuffer typeMult, int ntypes, ByteBuffer typeOut,
                                  ByteBuffer dirOut, ByteBuffer otherOut, ByteBuffer relationOut);

    static void check(int status) {
        if (status != 0) {
            throw new org.janusgraph.core.JanusGraphException(
                "GPU computer is aborting: libjanusgpu status " + status + ": " + lastError());
        }
    }
}
