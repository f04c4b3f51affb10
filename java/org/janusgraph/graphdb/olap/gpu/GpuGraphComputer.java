// Copyright 2026 JanusGraph Authors
// SPDX-License-Identifier: Apache-2.0
package org.janusgraph.graphdb.olap.gpu;

import org.apache.commons.configuration.BaseConfiguration;
import org.apache.tinkerpop.gremlin.process.computer.ComputerResult;
import org.apache.tinkerpop.gremlin.process.computer.GraphComputer;
import org.apache.tinkerpop.gremlin.process.computer.KeyValue;
import org.apache.tinkerpop.gremlin.process.computer.MapReduce;
import org.apache.tinkerpop.gremlin.process.computer.VertexProgram;
import org.apache.tinkerpop.gremlin.process.computer.clustering.connected.ConnectedComponentVertexProgram;
import org.apache.tinkerpop.gremlin.process.traversal.Traversal;
import org.apache.tinkerpop.gremlin.structure.Direction;
import org.apache.tinkerpop.gremlin.structure.Edge;
import org.apache.tinkerpop.gremlin.structure.Vertex;
import org.janusgraph.core.JanusGraphComputer;
import org.janusgraph.core.JanusGraphEdge;
import org.janusgraph.core.JanusGraphVertex;
import org.janusgraph.diskstorage.configuration.Configuration;
import org.janusgraph.graphdb.database.StandardJanusGraph;
import org.janusgraph.graphdb.olap.computer.FulgoraGraphComputer;
import org.janusgraph.graphdb.transaction.StandardJanusGraphTx;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.Iterator;
import java.util.List;
import java.util.concurrent.CompletableFuture;
import java.util.concurrent.Future;

/**
 * Drop-in for {@link FulgoraGraphComputer} (janusgraph-core/.../olap/computer/FulgoraGraphComputer.java)
 * that runs PageRankVertexProgram, ShortestDistanceVertexProgram (janusgraph-backend-testutils olap
 * package), ConnectedComponentVertexProgram and ShortestPathVertexProgram (TinkerPop) on MI355X GPUs
 * through libjanusgpu. The edgestore is scanned ONCE into an id/edge snapshot (instead of once per
 * superstep); every other program is delegated unchanged to a FulgoraGraphComputer.
 *
 * Entry: {@code graph.compute(GpuGraphComputer.class)} once JanusGraphBlueprintsGraph.compute(Class)
 * (janusgraph-core/.../tinkerpop/JanusGraphBlueprintsGraph.java:155-161) whitelists this class.
 * Configuration: computer.gpu.devices (comma list, default "0").
 */
public class GpuGraphComputer implements JanusGraphComputer {

    private static final String PR = "org.janusgraph.olap.PageRankVertexProgram";
    private static final String SD = "org.janusgraph.olap.ShortestDistanceVertexProgram";

    private final StandardJanusGraph graph;
    private final Configuration configuration;
    private final FulgoraGraphComputer delegate;
    private VertexProgram<?> vertexProgram;
    private final List<MapReduce> mapReduces = new ArrayList<>();
    private ResultGraph resultGraph;
    private Persist persist;
    private int workers = 1;
    private boolean filtered;
    private boolean executed;

    public GpuGraphComputer(final StandardJanusGraph graph, final Configuration configuration) {
        this.graph = graph;
        this.configuration = configuration;
        this.delegate = new FulgoraGraphComputer(graph, configuration);
    }

    @Override public GraphComputer vertices(Traversal<Vertex, Vertex> f) { filtered = true; delegate.vertices(f); return this; }
    @Override public GraphComputer edges(Traversal<Vertex, Edge> f) { filtered = true; delegate.edges(f); return this; }
    @Override public GraphComputer result(ResultGraph r) { resultGraph = r; delegate.result(r); return this; }
    @Override public GraphComputer persist(Persist p) { persist = p; delegate.persist(p); return this; }
    @Override public JanusGraphComputer workers(int n) { workers = n; delegate.workers(n); return this; }
    @Override public GraphComputer mapReduce(MapReduce mr) { mapReduces.add(mr); delegate.mapReduce(mr); return this; }

    @Override
    public GraphComputer program(VertexProgram vp) {
        if (vertexProgram != null) throw new IllegalStateException("A vertex program has already been set");
        vertexProgram = vp;
        delegate.program(vp);
        return this;
    }

    private boolean runsOnGpu() {
        if (vertexProgram == null || filtered) return false;
        final String name = vertexProgram.getClass().getName();
        return name.equals(PR) || name.equals(SD) || vertexProgram instanceof ConnectedComponentVertexProgram;
    }

    @Override
    public Future<ComputerResult> submit() {
        if (!runsOnGpu()) return delegate.submit(); // SURVEY §3E: everything else stays on Fulgora
        if (executed) throw Exceptions.computerHasAlreadyBeenSubmittedAVertexProgram();
        executed = true;
        return CompletableFuture.supplyAsync(this::submitAsync);
    }

    private ComputerResult submitAsync() {
        final long t0 = System.currentTimeMillis();
        final BaseConfiguration conf = new BaseConfiguration();
        vertexProgram.storeState(conf);
        final Snapshot snap = Snapshot.scan(graph, vertexProgram.getClass().getName().equals(SD)
            ? conf.getString("janusgraph.shortestDistanceVertexProgram.weightProperty", "distance") : null);
        final long[] h = new long[1];
        JanusGpu.check(JanusGpu.ctxCreate(devices(), h));
        final long ctx = h[0];
        try {
            final GpuResult res = run(ctx, snap, conf);
            final GpuMemory memory = new GpuMemory(res.iteration, System.currentTimeMillis() - t0);
            for (MapReduce mr : allMapReduces()) memory.put(mr.getMemoryKey(), res.map(mr, snap));
            return res.writeBack(graph, snap, resultGraph, persist, memory);
        } finally {
            JanusGpu.ctxDestroy(ctx);
        }
    }

    private GpuResult run(long ctx, Snapshot s, BaseConfiguration conf) {
        final String name = vertexProgram.getClass().getName();
        final int flags = name.equals(PR) ? JanusGpu.ADJ_IN
            : name.equals(SD) ? (JanusGpu.ADJ_IN | JanusGpu.ADJ_OUT) : JanusGpu.ADJ_BOTH;
        final long[] h = new long[1];
        JanusGpu.check(JanusGpu.graphBuild(ctx, s.vid, s.n, s.src, s.dst, s.weight, s.m, flags, h));
        final long g = h[0];
        try {
            if (name.equals(PR)) {
                final int k = conf.getInt("janusgraph.pageRank.maxIterations", 10);
                final ByteBuffer rank = direct(8 * s.n), count = direct(8 * s.n);
                JanusGpu.check(JanusGpu.pageRank(g, conf.getDouble("janusgraph.pageRank.dampingFactor", 0.85),
                    conf.getLong("janusgraph.pageRank.vertexCount", 1L), k, rank, count));
                return GpuResult.pageRank(k, rank, count);
            } else if (name.equals(SD)) {
                final int maxDepth = conf.getInt("janusgraph.shortestDistanceVertexProgram.maxDepth");
                final ByteBuffer dist = direct(8 * s.n);
                JanusGpu.check(JanusGpu.shortestDistance(g,
                    conf.getLong("janusgraph.shortestDistanceVertexProgram.seedID"), maxDepth, dist));
                return GpuResult.distance(maxDepth, dist);
            } else {
                final ByteBuffer comp = direct(8 * s.n);
                final int[] it = new int[1];
                JanusGpu.check(JanusGpu.connectedComponents(g, comp, it));
                return GpuResult.component(it[0], comp);
            }
        } finally {
            JanusGpu.graphDestroy(g);
        }
    }

    private List<MapReduce> allMapReduces() {
        final List<MapReduce> all = new ArrayList<>(mapReduces);
        all.addAll(vertexProgram.getMapReducers());
        return all;
    }

    private int[] devices() {
        final String[] parts = System.getProperty("janusgraph.computer.gpu.devices", "0").split(",");
        final int[] d = new int[parts.length];
        for (int i = 0; i < parts.length; i++) d[i] = Integer.parseInt(parts[i].trim());
        return d;
    }

    static ByteBuffer direct(long bytes) {
        return ByteBuffer.allocateDirect((int) Math.max(bytes, 8)).order(ByteOrder.nativeOrder());
    }

    @Override
    public Features features() {
        return delegate.features();
    }

    /**
     * The once-per-computer edgestore snapshot: vertex ids of existing (non-ghost) vertices and the
     * OUT entries of every row (each edge once), read through a read-only transaction
     * (VertexJobConverter semantics, janusgraph-core/.../olap/VertexJobConverter.java:122-151).
     */
    static final class Snapshot {
        ByteBuffer vid, src, dst, weight;
        long n, m;

        static Snapshot scan(StandardJanusGraph graph, String weightKey) {
            final StandardJanusGraphTx tx = (StandardJanusGraphTx) graph.buildTransaction().readOnly().start();
            try {
                final List<Long> ids = new ArrayList<>();
                final List<long[]> edges = new ArrayList<>();
                final List<Integer> w = new ArrayList<>();
                for (Iterator<Vertex> it = tx.vertices(); it.hasNext(); ) {
                    final JanusGraphVertex v = (JanusGraphVertex) it.next();
                    ids.add(v.longId());
                    for (Iterator<Edge> ei = v.edges(Direction.OUT); ei.hasNext(); ) {
                        final JanusGraphEdge e = (JanusGraphEdge) ei.next();
                        edges.add(new long[]{v.longId(), e.inVertex().longId()});
                        if (weightKey != null) w.add(e.<Integer>value(weightKey));
                    }
                }
                final Snapshot s = new Snapshot();
                s.n = ids.size();
                s.m = edges.size();
                s.vid = direct(8 * s.n);
                for (long id : ids) s.vid.putLong(id);
                s.src = direct(8 * s.m);
                s.dst = direct(8 * s.m);
                for (long[] e : edges) { s.src.putLong(e[0]); s.dst.putLong(e[1]); }
                if (weightKey != null) {
                    s.weight = direct(4 * s.m);
                    for (int x : w) s.weight.putInt(x);
                }
                return s;
            } finally {
                tx.rollback();
            }
        }
    }
}
