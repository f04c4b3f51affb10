// Copyright 2026 JanusGraph Authors
// SPDX-License-Identifier: Apache-2.0
package org.janusgraph.graphdb.olap.gpu;

import org.apache.tinkerpop.gremlin.process.computer.ComputerResult;
import org.apache.tinkerpop.gremlin.process.computer.GraphComputer;
import org.apache.tinkerpop.gremlin.process.computer.KeyValue;
import org.apache.tinkerpop.gremlin.process.computer.MapReduce;
import org.apache.tinkerpop.gremlin.process.computer.clustering.connected.ConnectedComponentVertexProgram;
import org.apache.tinkerpop.gremlin.process.computer.util.DefaultComputerResult;
import org.apache.tinkerpop.gremlin.structure.Graph;
import org.apache.tinkerpop.gremlin.structure.VertexProperty;
import org.apache.tinkerpop.gremlin.structure.util.empty.EmptyGraph;
import org.janusgraph.core.JanusGraphTransaction;
import org.janusgraph.core.JanusGraphVertex;
import org.janusgraph.graphdb.database.StandardJanusGraph;

import java.nio.ByteBuffer;
import java.util.ArrayList;
import java.util.Iterator;
import java.util.List;

/**
 * Columnar GPU outputs shaped like Fulgora's vertex memory: map-reduce emissions
 * (PageRankMapReduce / ShortestDistanceMapReduce keys) and property write-back following
 * FulgoraGraphComputer.writeMutatedPropertiesBackIntoGraph (FulgoraGraphComputer.java:359-471).
 */
final class GpuResult {
    final int iteration;
    private final String key;         // computed vertex key
    private final ByteBuffer values;  // float64 (PageRank) or int64 (distance, component vid)
    private final String key2;        // PageRank edgeCount
    private final ByteBuffer values2;
    private final int kind;           // 0 = double, 1 = long (absent when < 0), 2 = component (String)

    private GpuResult(int iteration, String key, ByteBuffer v, String key2, ByteBuffer v2, int kind) {
        this.iteration = iteration;
        this.key = key;
        this.values = v;
        this.key2 = key2;
        this.values2 = v2;
        this.kind = kind;
    }

    static GpuResult pageRank(int k, ByteBuffer rank, ByteBuffer count) {
        return new GpuResult(k, "janusgraph.pageRank.pageRank", rank, "janusgraph.pageRank.edgeCount", count, 0);
    }

    static GpuResult distance(int maxDepth, ByteBuffer dist) {
        return new GpuResult(maxDepth, "janusgraph.shortestDistanceVertexProgram.distance", dist, null, null, 1);
    }

    static GpuResult component(int iteration, ByteBuffer comp) {
        return new GpuResult(iteration, ConnectedComponentVertexProgram.COMPONENT, comp, null, null, 2);
    }

    private Object value(int i) {
        if (kind == 0) {
            final double d = values.getDouble(8 * i);
            return Double.isNaN(d) ? null : d;
        }
        final long l = values.getLong(8 * i);
        if (kind == 1) return l < 0 ? null : l;
        return Long.toString(l);
    }

    Iterator<KeyValue<Long, Object>> map(MapReduce mr, GpuGraphComputer.Snapshot s) {
        final List<KeyValue<Long, Object>> out = new ArrayList<>();
        for (int i = 0; i < s.n; i++) {
            final Object v = value(i);
            if (v != null) out.add(new KeyValue<>(s.vid.getLong(8 * i), v));
        }
        return out.iterator();
    }

    ComputerResult writeBack(StandardJanusGraph graph, GpuGraphComputer.Snapshot s, GraphComputer.ResultGraph rg,
                             GraphComputer.Persist persist, GpuMemory memory) {
        if (persist == null || persist == GraphComputer.Persist.NOTHING) {
            final Graph g = rg == GraphComputer.ResultGraph.NEW ? EmptyGraph.instance() : graph;
            return new DefaultComputerResult(g, memory);
        }
        final JanusGraphTransaction tx = graph.buildTransaction().enableBatchLoading().start();
        for (int i = 0; i < s.n; i++) {
            final Object v = value(i);
            if (v == null) continue;
            final JanusGraphVertex vertex = tx.getVertex(s.vid.getLong(8 * i));
            vertex.property(VertexProperty.Cardinality.single, key, v);
            if (key2 != null) vertex.property(VertexProperty.Cardinality.single, key2, values2.getDouble(8 * i));
        }
        tx.commit();
        return new DefaultComputerResult(graph, memory);
    }
}
