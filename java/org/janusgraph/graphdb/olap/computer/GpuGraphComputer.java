// Copyright 2026 JanusGraph Authors
// SPDX-License-Identifier: Apache-2.0
package org.janusgraph.graphdb.olap.computer;

import org.apache.commons.configuration.BaseConfiguration;
import org.apache.tinkerpop.gremlin.process.computer.ComputerResult;
import org.apache.tinkerpop.gremlin.process.computer.GraphComputer;
import org.apache.tinkerpop.gremlin.process.computer.MapReduce;
import org.apache.tinkerpop.gremlin.process.computer.VertexComputeKey;
import org.apache.tinkerpop.gremlin.process.computer.VertexProgram;
import org.apache.tinkerpop.gremlin.process.computer.clustering.connected.ConnectedComponentVertexProgram;
import org.apache.tinkerpop.gremlin.process.computer.search.path.ShortestPathVertexProgram;
import org.apache.tinkerpop.gremlin.process.computer.util.DefaultComputerResult;
import org.apache.tinkerpop.gremlin.process.computer.util.VertexProgramHelper;
import org.apache.tinkerpop.gremlin.process.traversal.Path;
import org.apache.tinkerpop.gremlin.process.traversal.Traversal;
import org.apache.tinkerpop.gremlin.process.traversal.step.util.ImmutablePath;
import org.apache.tinkerpop.gremlin.process.traversal.util.PureTraversal;
import org.apache.tinkerpop.gremlin.process.traversal.util.TraversalUtil;
import org.apache.tinkerpop.gremlin.structure.Edge;
import org.apache.tinkerpop.gremlin.structure.Graph;
import org.apache.tinkerpop.gremlin.structure.Vertex;
import org.apache.tinkerpop.gremlin.structure.VertexProperty;
import org.apache.tinkerpop.gremlin.structure.util.empty.EmptyGraph;
import org.apache.tinkerpop.gremlin.structure.util.reference.ReferenceFactory;
import org.janusgraph.core.JanusGraphException;
import org.janusgraph.core.JanusGraphTransaction;
import org.janusgraph.core.schema.JanusGraphManagement;
import org.janusgraph.diskstorage.configuration.Configuration;
import org.janusgraph.graphdb.configuration.GraphDatabaseConfiguration;
import org.janusgraph.graphdb.database.StandardJanusGraph;
import org.janusgraph.graphdb.olap.QueryContainer;
import org.janusgraph.graphdb.util.WorkerPool;
import org.slf4j.Logger;
import org.slf4j.LoggerFactory;

import java.lang.reflect.Field;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.DoubleBuffer;
import java.nio.IntBuffer;
import java.nio.LongBuffer;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.BitSet;
import java.util.Collections;
import java.util.HashMap;
import java.util.HashSet;
import java.util.List;
import java.util.Map;
import java.util.Objects;
import java.util.Set;
import java.util.concurrent.CompletableFuture;
import java.util.concurrent.Future;
import java.util.concurrent.atomic.AtomicInteger;
import java.util.function.IntFunction;

/**
 * Drop-in for {@link FulgoraGraphComputer} that runs the superstep loop of the recognised programs on
 * MI355X GPUs through libjanusgpu, and delegates everything else to Fulgora unchanged (SURVEY §3E:
 * TraversalVertexProgram, user programs, graph filters, non-default program configurations).
 *
 * GPU programs (each exactly as Fulgora would run it):
 * <ul>
 *   <li>PageRankVertexProgram (janusgraph-backend-testutils olap; PageRankVertexProgram.java:89-110);</li>
 *   <li>ShortestDistanceVertexProgram (ShortestDistanceVertexProgram.java:112-146), settings read from the
 *       instance: storeState (:74-77) does not write the seed or the weight property;</li>
 *   <li>TinkerPop ConnectedComponentVertexProgram with its default edges and iteration cap (any
 *       component property key);</li>
 *   <li>TinkerPop ShortestPathVertexProgram with its default edge and distance traversals (any source /
 *       target filter, any maxDistance; includeEdges off): hop depths on the GPU (BOTH edges, as
 *       FulgoraGraphComputer.java:249-253 forces), paths rebuilt from the depths over the snapshot's
 *       own BOTH adjacency.</li>
 * </ul>
 * The edgestore is scanned ONCE into a device CSR (GpuSnapshot) instead of once per superstep. The
 * results then go through Fulgora's own machinery, opened to subclasses by
 * java/patches/0002-FulgoraGraphComputer-protected-phases.patch: the settings check and FulgoraMemory
 * of submit() (FulgoraGraphComputer.java:154-193), the map phase (columnar emission for
 * PageRankMapReduce / ShortestDistanceMapReduce, otherwise Fulgora's executeMapJobs VertexMapJob scan
 * over a FulgoraVertexMemory holding the results) and executeReducePhase (:331-357). The write-back
 * of the non-transient compute keys goes straight from the result columns (:359-471 semantics:
 * ORIGINAL in batch transactions, NEW in an uncommitted transaction).
 *
 * Entry: {@code graph.compute(GpuGraphComputer.class)} once JanusGraphBlueprintsGraph.compute(Class)
 * (janusgraph-core/.../tinkerpop/JanusGraphBlueprintsGraph.java:155-161) whitelists this class
 * (java/patches/0001); the transaction variant delegates to it.
 *
 * Configuration (the graph's own, registered by patch 0001 under computer.gpu next to
 * computer.result-mode, GraphDatabaseConfiguration.java:203-208; MASKABLE, so per graph):
 * <ul>
 *   <li>computer.gpu.devices (default "0"): HIP devices; several shard the snapshot 1D by vertex;</li>
 *   <li>computer.gpu.untruncated (default false): keep every entry instead of Fulgora's 100000-entry
 *       slice cap;</li>
 *   <li>computer.gpu.direct-memory (default 1 GiB): most bytes of direct result buffers held at once;</li>
 *   <li>computer.gpu.default (default false, read by patch 0001): graph.compute() returns this computer.</li>
 * </ul>
 */
public class GpuGraphComputer extends FulgoraGraphComputer {

    private static final Logger log = LoggerFactory.getLogger(GpuGraphComputer.class);

    static final String PR = "org.janusgraph.olap.PageRankVertexProgram";
    static final String SD = "org.janusgraph.olap.ShortestDistanceVertexProgram";
    static final String PR_MAP = "org.janusgraph.olap.PageRankMapReduce";
    static final String SD_MAP = "org.janusgraph.olap.ShortestDistanceMapReduce";
    static final String PAGE_RANK = "janusgraph.pageRank.pageRank";
    static final String EDGE_COUNT = "janusgraph.pageRank.edgeCount";
    static final String DISTANCE = "janusgraph.shortestDistanceVertexProgram.distance";
    static final int SOURCES_PER_BFS = 64; // jg_bfs_rows: one bit-parallel pass per 64 sources

    private final StandardJanusGraph graph;
    private final int writeBatchSize;
    private final int[] devices;
    private final long queryLimit;
    private final long directMemory;
    private VertexProgram<?> vertexProgram;
    private boolean filtered;

    public GpuGraphComputer(final StandardJanusGraph graph, final Configuration configuration) {
        super(graph, configuration);
        this.graph = graph;
        this.writeBatchSize = configuration.get(GraphDatabaseConfiguration.BUFFER_SIZE);
        this.devices = devices(configuration.get(GraphDatabaseConfiguration.COMPUTER_GPU_DEVICES));
        this.queryLimit = queryLimit(configuration.get(GraphDatabaseConfiguration.COMPUTER_GPU_UNTRUNCATED));
        this.directMemory = configuration.get(GraphDatabaseConfiguration.COMPUTER_GPU_DIRECT_MEMORY);
        if (directMemory < (64L << 20))
            throw new IllegalArgumentException("computer.gpu.direct-memory must be at least 64 MiB");
    }

    // ---- the GraphComputer builder: Fulgora records the settings; the GPU path reads them back ----

    @Override
    public GraphComputer vertices(final Traversal<Vertex, Vertex> vertexFilter) {
        filtered = true;
        return super.vertices(vertexFilter);
    }

    @Override
    public GraphComputer edges(final Traversal<Vertex, Edge> edgeFilter) {
        filtered = true;
        return super.edges(edgeFilter);
    }

    @Override
    public GraphComputer program(final VertexProgram program) {
        super.program(program);
        vertexProgram = program;
        return this;
    }

    // ---- submit ----

    @Override
    public Future<ComputerResult> submit() {
        final GpuProgram run = (vertexProgram == null || filtered) ? null : GpuProgram.recognise(vertexProgram, graph);
        if (run == null) return super.submit(); // everything else stays on Fulgora, unchanged
        // FulgoraGraphComputer.submit (:154-162) up to the superstep loop
        guardAgainstDuplicateSubmission();
        ensureSettingsAreValid();
        initializeMemory();
        return CompletableFuture.supplyAsync(() -> submitAsync(run));
    }

    private ComputerResult submitAsync(final GpuProgram run) {
        final long time = System.currentTimeMillis();
        vertexProgram.setup(memory);
        final long[] h = new long[1];
        JanusGpu.check(JanusGpu.ctxCreate(devices, h));
        final long ctx = h[0];
        final Results res;
        try {
            final long g = GpuSnapshot.scan(graph, ctx, run.adjacency(), run.weightProperty(), queryLimit,
                run.inEntries());
            try {
                final long[] vid = GpuSnapshot.vertexIds(g);
                res = run.execute(g, vid, graph, memory, directMemory);
            } finally {
                JanusGpu.graphDestroy(g);
            }
        } finally {
            JanusGpu.ctxDestroy(ctx);
        }
        // supersteps 0..K ran: Fulgora's memory counts K + 1 and complete() reports K (FulgoraMemory.java:97-101)
        memory.setIteration(res.iteration + 1);
        executeMapReduce(res);
        final Graph resultGraph = writeBack(res);
        memory.setRuntime(System.currentTimeMillis() - time);
        memory.complete();
        return new DefaultComputerResult(resultGraph, memory);
    }

    /**
     * Fulgora's hard limit on the entries of a non-fitted slice (QueryContainer.DEFAULT_HARD_QUERY_LIMIT,
     * olap/QueryContainer.java:42,133): the snapshot reproduces it, so vertices with more than 100000
     * edge entries get exactly the truncated adjacency Fulgora computes on.  computer.gpu.untruncated=true
     * computes on every entry instead.
     */
    static long queryLimit(boolean untruncated) {
        return untruncated ? 0L : QueryContainer.DEFAULT_HARD_QUERY_LIMIT;
    }

    /** computer.gpu.devices: HIP device ordinals (a String[] option: "0,1" or a list in the properties file). */
    static int[] devices(String[] parts) {
        if (parts == null || parts.length == 0) throw new IllegalArgumentException("computer.gpu.devices is empty");
        final int[] d = new int[parts.length];
        for (int i = 0; i < parts.length; i++) d[i] = Integer.parseInt(parts[i].trim());
        return d;
    }

    /** One direct buffer: at most 2 GiB (per-vertex 8-byte columns: up to 2^28 vertices). */
    static ByteBuffer direct(long bytes) {
        if (bytes > Integer.MAX_VALUE)
            throw new JanusGraphException("GPU computer: " + bytes + " bytes exceed one direct buffer (2 GiB)");
        return ByteBuffer.allocateDirect((int) Math.max(bytes, 8)).order(ByteOrder.nativeOrder());
    }

    // ---- map / reduce: Fulgora's phases (FulgoraGraphComputer.java:288-357) ----

    private void executeMapReduce(final Results res) {
        final Map<MapReduce, FulgoraMapEmitter> mapJobs = collectMapJobs();
        if (mapJobs.isEmpty()) return;
        boolean columnar = true;
        for (MapReduce mr : mapJobs.keySet()) {
            final String name = mr.getClass().getName();
            columnar &= name.equals(PR_MAP) || name.equals(SD_MAP);
        }
        if (!columnar) {
            // any other MapReduce sees what Fulgora gives it: Fulgora's VertexMapJob scan over the vertex
            // memory it would hold after the supersteps (VertexMapJob.java:107-130), then its reduce phase
            vertexMemory = res.toVertexMemory(graph, vertexProgram);
            executeMapJobs(mapJobs);
            return;
        }
        // PageRankMapReduce / ShortestDistanceMapReduce.map emit (vertex.id(), the compute key's value)
        // where it is present (PageRankMapReduce.java:62-67, ShortestDistanceMapReduce.java:59-64):
        // emitted straight from the result columns, without a second edgestore scan
        for (Map.Entry<MapReduce, FulgoraMapEmitter> job : mapJobs.entrySet()) {
            final Column col = res.column(job.getKey().getClass().getName().equals(PR_MAP) ? PAGE_RANK : DISTANCE);
            final FulgoraMapEmitter emitter = job.getValue();
            job.getKey().workerStart(MapReduce.Stage.MAP);
            for (int i = 0; i < res.vid.length; i++) {
                final Object v = col == null ? null : col.get(i);
                if (v != null) emitter.emit(res.vid[i], v);
            }
            job.getKey().workerEnd(MapReduce.Stage.MAP);
        }
        executeReducePhase(mapJobs);
        memory.attachReferenceElements(graph);
    }

    // ---- write-back (FulgoraGraphComputer.java:359-471) ----

    private Graph writeBack(final Results res) {
        if (persistMode == Persist.NOTHING) return resultGraphMode == ResultGraph.NEW ? EmptyGraph.instance() : graph;
        final List<Column> cols = new ArrayList<>();
        for (Column c : res.columns)
            if (!VertexProgramHelper.isTransientVertexComputeKey(c.key, vertexProgram.getVertexComputeKeys())) cols.add(c);
        if (cols.isEmpty() || vertexProgram.getVertexComputeKeys().isEmpty()) return graph;
        final JanusGraphManagement management = graph.openManagement();
        try {
            for (VertexComputeKey key : vertexProgram.getVertexComputeKeys()) management.getOrCreatePropertyKey(key.getKey());
            management.commit();
        } finally {
            if (management.isOpen()) management.rollback();
        }
        if (resultGraphMode == ResultGraph.NEW) { // an uncommitted transaction over the original graph
            final JanusGraphTransaction tx = graph.newTransaction();
            for (int i = 0; i < res.vid.length; i++) {
                Vertex v = null;
                for (Column c : cols) {
                    final Object value = c.get(i);
                    if (value == null) continue;
                    if (v == null) v = tx.vertices(res.vid[i]).next();
                    v.property(VertexProperty.Cardinality.single, c.key, value);
                }
            }
            return tx;
        }
        final AtomicInteger failures = new AtomicInteger();
        try (WorkerPool workers = new WorkerPool(numThreads)) {
            final int batch = Math.max(1, writeBatchSize / Math.max(1, cols.size()));
            for (int start = 0; start < res.vid.length; start += batch) {
                final int from = start, to = Math.min(res.vid.length, start + batch);
                workers.submit(() -> {
                    final JanusGraphTransaction tx = graph.buildTransaction().enableBatchLoading().start();
                    try {
                        for (int i = from; i < to; i++) {
                            Vertex v = null;
                            for (Column c : cols) {
                                final Object value = c.get(i);
                                if (value == null) continue;
                                if (v == null) v = tx.getVertex(res.vid[i]);
                                if (v == null) break;
                                v.property(VertexProperty.Cardinality.single, c.key, value);
                            }
                        }
                        tx.commit();
                    } catch (Throwable e) {
                        log.error("Encountered exception while trying to write properties: ", e);
                        failures.incrementAndGet();
                    } finally {
                        if (tx.isOpen()) tx.rollback();
                    }
                });
            }
        } catch (Exception e) {
            throw new JanusGraphException("Exception while attempting to persist result into graph", e);
        }
        if (failures.get() > 0)
            throw new JanusGraphException("Could not persist program results to graph. Check log for details.");
        return graph;
    }

    // ---- results ----

    /** One compute key over the vertices in snapshot order; get(i) == null: the property is absent. */
    abstract static class Column {
        final String key;

        Column(String key) {
            this.key = key;
        }

        abstract Object get(int i);
    }

    static final class Results {
        final long[] vid;
        final int iteration; // getIteration() of the finished run
        final List<Column> columns = new ArrayList<>();

        Results(long[] vid, int iteration) {
            this.vid = vid;
            this.iteration = iteration;
        }

        Column column(String key) {
            for (Column c : columns) if (c.key.equals(key)) return c;
            return null;
        }

        /** The vertex memory Fulgora would hold after the supersteps (for arbitrary MapReduces). */
        FulgoraVertexMemory toVertexMemory(StandardJanusGraph graph, VertexProgram<?> vp) {
            final FulgoraVertexMemory vm = new FulgoraVertexMemory(Math.max(vid.length, 16), graph.getIDManager(), vp);
            for (int i = 0; i < vid.length; i++)
                for (Column c : columns) {
                    final Object value = c.get(i);
                    if (value != null) vm.setProperty(vid[i], c.key, value);
                }
            return vm;
        }
    }

    // Columns read the output buffers through typed views: element indices, no byte offsets.

    static Column doubles(String key, ByteBuffer buf) {
        final DoubleBuffer d = buf.asDoubleBuffer();
        return new Column(key) {
            @Override
            Object get(int i) {
                final double x = d.get(i);
                return Double.isNaN(x) ? null : x; // NaN: no superstep wrote the property (K == 0)
            }
        };
    }

    static Column distances(String key, ByteBuffer buf) {
        final LongBuffer d = buf.asLongBuffer();
        return new Column(key) {
            @Override
            Object get(int i) {
                final long l = d.get(i);
                return l == JanusGpu.DIST_ABSENT ? null : l;
            }
        };
    }

    static Column components(String key, ByteBuffer buf) {
        final LongBuffer d = buf.asLongBuffer();
        return new Column(key) {
            @Override
            Object get(int i) {
                return Long.toString(d.get(i)); // the label is the id's String form
            }
        };
    }

    // ---- the programs run on the GPU ----

    /** A recognised program with its settings; null from recognise(): delegate to Fulgora. */
    abstract static class GpuProgram {
        abstract int adjacency();

        String weightProperty() {
            return null;
        }

        /** Under the slice cap: the entries a receiver reads for the IN adjacency (jg_builder_set_query_limit).
         *  PageRank's gather reads its IN entries; ShortestDistance overrides (its OUT entries). */
        int inEntries() {
            return JanusGpu.DIR_IN;
        }

        /** directMemory: computer.gpu.direct-memory, the most bytes of direct buffers held at once. */
        abstract Results execute(long g, long[] vid, StandardJanusGraph graph, FulgoraMemory memory, long directMemory);

        static GpuProgram recognise(VertexProgram<?> vp, StandardJanusGraph graph) {
            final String name = vp.getClass().getName();
            if (name.equals(PR)) return PageRank.of(vp);
            if (name.equals(SD)) return ShortestDistance.of(vp);
            if (vp instanceof ConnectedComponentVertexProgram) return Components.of(vp, graph);
            if (vp instanceof ShortestPathVertexProgram) return ShortestPaths.of(vp, graph);
            return null;
        }
    }

    static BaseConfiguration state(VertexProgram<?> vp) {
        final BaseConfiguration conf = new BaseConfiguration();
        vp.storeState(conf);
        return conf;
    }

    /** True when conf and the default configuration agree on every key outside `free`. */
    static boolean defaultsExcept(BaseConfiguration conf, BaseConfiguration defaults, Set<String> free) {
        final Set<String> keys = new HashSet<>();
        conf.getKeys().forEachRemaining(keys::add);
        defaults.getKeys().forEachRemaining(keys::add);
        for (String k : keys) {
            if (free.contains(k)) continue;
            if (!Objects.equals(String.valueOf(conf.getProperty(k)), String.valueOf(defaults.getProperty(k)))) return false;
        }
        return true;
    }

    static final class PageRank extends GpuProgram {
        final double damping;
        final long vertexCount;
        final int iterations;

        private PageRank(double damping, long vertexCount, int iterations) {
            this.damping = damping;
            this.vertexCount = vertexCount;
            this.iterations = iterations;
        }

        static PageRank of(VertexProgram<?> vp) { // storeState writes all three (PageRankVertexProgram.java:72-77)
            final BaseConfiguration c = state(vp);
            return new PageRank(c.getDouble("janusgraph.pageRank.dampingFactor", 0.85D),
                c.getLong("janusgraph.pageRank.vertexCount", 1L), c.getInt("janusgraph.pageRank.maxIterations", 10));
        }

        @Override
        int adjacency() {
            return JanusGpu.ADJ_IN;
        }

        @Override
        Results execute(long g, long[] vid, StandardJanusGraph graph, FulgoraMemory memory, long directMemory) {
            final ByteBuffer rank = direct(8L * vid.length), count = direct(8L * vid.length);
            JanusGpu.check(JanusGpu.pageRank(g, damping, vertexCount, iterations, rank, count));
            final Results r = new Results(vid, iterations);
            r.columns.add(doubles(PAGE_RANK, rank));
            r.columns.add(doubles(EDGE_COUNT, count));
            return r;
        }
    }

    static final class ShortestDistance extends GpuProgram {
        final long seed;
        final int maxDepth;
        final String weight;

        private ShortestDistance(long seed, int maxDepth, String weight) {
            this.seed = seed;
            this.maxDepth = maxDepth;
            this.weight = weight;
        }

        private static Object field(VertexProgram<?> vp, String name) throws ReflectiveOperationException {
            final Field f = vp.getClass().getDeclaredField(name);
            f.setAccessible(true);
            return f.get(vp);
        }

        /** The seed and weight key live only in the instance (storeState, :74-77, writes neither). */
        static ShortestDistance of(VertexProgram<?> vp) {
            try {
                final String w = (String) field(vp, "weightProperty");
                return new ShortestDistance((Long) field(vp, "seed"), (Integer) field(vp, "maxDepth"),
                    w == null ? "distance" : w);
            } catch (ReflectiveOperationException | ClassCastException e) {
                return null; // an incompatible program version: Fulgora runs it
            }
        }

        @Override
        int adjacency() {
            return JanusGpu.ADJ_IN | JanusGpu.ADJ_OUT;
        }

        @Override
        String weightProperty() {
            return weight;
        }

        @Override
        int inEntries() {
            return JanusGpu.DIR_OUT; // messages on Local.of(inE): the receiver reads its OUT entries
        }

        @Override
        Results execute(long g, long[] vid, StandardJanusGraph graph, FulgoraMemory memory, long directMemory) {
            final ByteBuffer dist = direct(8L * vid.length);
            JanusGpu.check(JanusGpu.shortestDistance(g, seed, maxDepth, dist));
            final Results r = new Results(vid, maxDepth);
            r.columns.add(distances(DISTANCE, dist));
            return r;
        }
    }

    static final class Components extends GpuProgram {
        final String property;

        private Components(String property) {
            this.property = property;
        }

        /** Only the default edge traversal and iteration cap; the component key may be any. */
        static Components of(VertexProgram<?> vp, StandardJanusGraph graph) {
            String property = null;
            for (VertexComputeKey k : vp.getVertexComputeKeys())
                if (!k.isTransient()) {
                    if (property != null) return null;
                    property = k.getKey();
                }
            if (property == null) return null;
            final VertexProgram<?> defaults = ConnectedComponentVertexProgram.build().create(graph);
            final BaseConfiguration conf = state(vp), def = state(defaults);
            final Set<String> free = new HashSet<>();
            final String key = property;
            conf.getKeys().forEachRemaining(k -> {
                if (key.equals(String.valueOf(conf.getProperty(k)))) free.add(k);
            });
            def.getKeys().forEachRemaining(k -> {
                if (ConnectedComponentVertexProgram.COMPONENT.equals(String.valueOf(def.getProperty(k)))) free.add(k);
            });
            return defaultsExcept(conf, def, free) ? new Components(property) : null;
        }

        @Override
        int adjacency() {
            return JanusGpu.ADJ_BOTH;
        }

        @Override
        Results execute(long g, long[] vid, StandardJanusGraph graph, FulgoraMemory memory, long directMemory) {
            final ByteBuffer comp = direct(8L * vid.length);
            final int[] it = new int[1];
            JanusGpu.check(JanusGpu.connectedComponents(g, comp, it));
            final Results r = new Results(vid, it[0]);
            r.columns.add(components(property, comp));
            return r;
        }
    }

    /**
     * ShortestPathVertexProgram with its default edge (bothE) and distance (unit) traversals and no
     * edges in the paths: every shortest path from each source to each target, as the program's
     * shortestPaths memory key. Depths come from the GPU (DIR_BOTH, the forced scope), one depth row
     * per source (jg_bfs_rows: 64 rows of n int32 do not fit one direct buffer past 2^23 vertices);
     * paths are rebuilt from each row by {@link PathDag} over the snapshot's BOTH adjacency.
     */
    static final class ShortestPaths extends GpuProgram {
        final BaseConfiguration conf;
        final Traversal.Admin<Vertex, ?> sourceFilter, targetFilter;
        final int maxDistance;

        private ShortestPaths(BaseConfiguration conf, Traversal.Admin<Vertex, ?> s, Traversal.Admin<Vertex, ?> t, int max) {
            this.conf = conf;
            this.sourceFilter = s;
            this.targetFilter = t;
            this.maxDistance = max;
        }

        static ShortestPaths of(VertexProgram<?> vp, StandardJanusGraph graph) {
            final BaseConfiguration conf = state(vp);
            final BaseConfiguration def = state(ShortestPathVertexProgram.build().create(graph));
            final Set<String> free = new HashSet<>();
            String src = null, dst = null, max = null;
            final Set<String> keys = new HashSet<>();
            conf.getKeys().forEachRemaining(keys::add);
            def.getKeys().forEachRemaining(keys::add);
            for (String k : keys) {
                if (k.endsWith("sourceVertexFilter")) src = k;
                else if (k.endsWith("targetVertexFilter")) dst = k;
                else if (k.endsWith("maxDistance")) max = k;
                else continue;
                free.add(k);
            }
            if (!defaultsExcept(conf, def, free)) return null;
            try {
                final Traversal.Admin<Vertex, ?> s = src != null && conf.containsKey(src)
                    ? PureTraversal.<Vertex, Object>loadState(conf, src, graph).get() : null;
                final Traversal.Admin<Vertex, ?> t = dst != null && conf.containsKey(dst)
                    ? PureTraversal.<Vertex, Object>loadState(conf, dst, graph).get() : null;
                final int m = max != null && conf.containsKey(max) ? ((Number) conf.getProperty(max)).intValue() : -1;
                return new ShortestPaths(conf, s, t, m);
            } catch (RuntimeException e) {
                return null; // a filter this computer cannot evaluate: Fulgora runs the program
            }
        }

        @Override
        int adjacency() {
            return JanusGpu.ADJ_BOTH;
        }

        @Override
        Results execute(long g, long[] vid, StandardJanusGraph graph, FulgoraMemory memory, long directMemory) {
            final int n = vid.length;
            final JanusGraphTransaction tx = graph.buildTransaction().readOnly().start();
            try {
                final int[] sources;
                BitSet target = null; // null: every vertex is a target
                if (sourceFilter == null && targetFilter == null) {
                    sources = new int[n];
                    for (int i = 0; i < n; i++) sources[i] = i;
                } else {
                    final PathDag.IntArray s = new PathDag.IntArray();
                    if (targetFilter != null) target = new BitSet(n);
                    for (int i = 0; i < n; i++) {
                        final Vertex v = tx.getVertex(vid[i]);
                        if (sourceFilter == null || TraversalUtil.test(v, sourceFilter.clone())) s.add(i);
                        if (target != null && TraversalUtil.test(v, targetFilter.clone())) target.set(i);
                    }
                    sources = s.toArray();
                }
                final Map<Integer, Vertex> detached = new HashMap<>(); // path elements, detached once each
                final IntFunction<Vertex> element =
                    i -> detached.computeIfAbsent(i, x -> ReferenceFactory.detach(tx.getVertex(vid[x])));
                // Direct memory: one depth row (4n bytes, reused by every source) and the walk-back's
                // neighbour batches (PathDag: at most half the budget); the batch's 64 rows stay on the
                // device (jg_bfs_keep) and come over one at a time (jg_bfs_kept_row).
                if (4L * n > directMemory / 2)
                    throw new JanusGraphException("GPU computer: a depth row of " + n + " vertices needs more than half "
                        + "of computer.gpu.direct-memory (" + directMemory + " bytes)");
                final PathDag dag = new PathDag(g, n, directMemory / 2);
                final ByteBuffer row = direct(4L * n);
                final ByteBuffer src = direct(8L * SOURCES_PER_BFS);
                final List<Path> paths = new ArrayList<>();
                int maxLevel = 0;
                try {
                    for (int b = 0; b < sources.length; b += SOURCES_PER_BFS) {
                        final int k = Math.min(SOURCES_PER_BFS, sources.length - b);
                        src.clear();
                        for (int j = 0; j < k; j++) src.putLong(vid[sources[b + j]]);
                        JanusGpu.check(JanusGpu.bfsKeep(g, src, k, JanusGpu.DIR_BOTH, maxDistance));
                        for (int j = 0; j < k; j++) {
                            JanusGpu.check(JanusGpu.bfsKeptRow(g, j, row));
                            maxLevel = Math.max(maxLevel, dag.paths(row.asIntBuffer(), sources[b + j], target, element,
                                paths));
                        }
                    }
                } finally {
                    JanusGpu.bfsKeptRelease(g);
                }
                memory.set(ShortestPathVertexProgram.SHORTEST_PATHS, paths);
                return new Results(vid, maxLevel + 1);
            } finally {
                tx.rollback();
            }
        }
    }

    /**
     * Every shortest path from one source to the targets it reaches, rebuilt from its depth row: the
     * predecessors of a vertex at depth d are its BOTH neighbours at depth d - 1. They are read level by
     * level from the device snapshot (jg_graph_neighbors), deepest targets first, so each vertex on some
     * path is expanded once and no OLTP transaction is touched; the paths are then enumerated from each
     * target (ascending) back to the source.
     */
    static final class PathDag {
        private static final int ROWS_PER_CALL = 1 << 14;
        private final long graph;
        private final int[] mark; // de-duplicates a vertex's neighbours (multi-edges, self-loops)
        private final long budget; // most bytes of the neighbour batch's direct buffers
        private int stamp;

        PathDag(long graph, int n, long budget) {
            this.graph = graph;
            this.mark = new int[n];
            this.budget = Math.min(budget, Integer.MAX_VALUE);
        }

        /** Adds the source's paths to `out`; returns the deepest target depth (0 when none). */
        int paths(IntBuffer depth, int s, BitSet target, IntFunction<Vertex> element, List<Path> out) {
            final int n = mark.length;
            final List<IntArray> level = new ArrayList<>();
            final BitSet queued = new BitSet(n);
            final IntArray targets = new IntArray();
            int deepest = -1;
            for (int t = 0; t < n; t++) {
                final int d = depth.get(t);
                if (d < 0 || (target != null && !target.get(t))) continue;
                while (level.size() <= d) level.add(new IntArray());
                level.get(d).add(t);
                queued.set(t);
                targets.add(t);
                deepest = Math.max(deepest, d);
            }
            if (deepest < 0) return 0;
            final Map<Integer, int[]> pred = new HashMap<>();
            for (int d = deepest; d >= 1; d--) {
                final int[] cur = level.get(d).toArray();
                for (int from = 0; from < cur.length; from += ROWS_PER_CALL) {
                    final int to = Math.min(cur.length, from + ROWS_PER_CALL);
                    final long[][] adj = neighbors(cur, from, to);
                    for (int i = from; i < to; i++) {
                        final IntArray p = new IntArray();
                        ++stamp;
                        for (long e = adj[0][i - from]; e < adj[0][i - from + 1]; e++) {
                            final int u = (int) adj[1][(int) e];
                            if (mark[u] == stamp || depth.get(u) != d - 1) continue;
                            mark[u] = stamp;
                            p.add(u);
                            if (!queued.get(u)) {
                                queued.set(u);
                                level.get(d - 1).add(u);
                            }
                        }
                        pred.put(cur[i], p.toArray());
                    }
                }
            }
            final IntArray suffix = new IntArray();
            for (int t : targets.toArray()) walk(pred, s, t, suffix, element, out);
            return deepest;
        }

        private static void walk(Map<Integer, int[]> pred, int s, int v, IntArray suffix, IntFunction<Vertex> element,
                                 List<Path> out) {
            suffix.add(v);
            if (v == s) {
                Path p = ImmutablePath.make();
                for (int i = suffix.size() - 1; i >= 0; i--) p = p.extend(element.apply(suffix.get(i)), Collections.emptySet());
                out.add(p);
            } else {
                for (int u : pred.get(v)) walk(pred, s, u, suffix, element, out);
            }
            suffix.pop();
        }

        /** {offsets[to - from + 1], neighbours} of rows[from, to): two jg_graph_neighbors calls (size, fill). */
        private long[][] neighbors(int[] rows, int from, int to) {
            final int k = to - from;
            final ByteBuffer r = direct(8L * k), off = direct(8L * (k + 1));
            for (int i = from; i < to; i++) r.putLong(rows[i]);
            JanusGpu.check(JanusGpu.graphNeighbors(graph, JanusGpu.DIR_BOTH, r, k, off, null));
            final long[] o = new long[k + 1];
            off.asLongBuffer().get(o);
            if (8L * o[k] + 16L * (k + 1) > budget && k > 1) { // a hub-heavy batch: split it
                final int mid = from + k / 2;
                final long[][] a = neighbors(rows, from, mid), b = neighbors(rows, mid, to);
                final long[] oo = Arrays.copyOf(a[0], k + 1);
                for (int i = 1; i < b[0].length; i++) oo[mid - from + i] = a[0][mid - from] + b[0][i];
                final long[] nn = Arrays.copyOf(a[1], a[1].length + b[1].length);
                System.arraycopy(b[1], 0, nn, a[1].length, b[1].length);
                return new long[][] {oo, nn};
            }
            final ByteBuffer nb = direct(8L * o[k]);
            JanusGpu.check(JanusGpu.graphNeighbors(graph, JanusGpu.DIR_BOTH, r, k, off, nb));
            final long[] nbr = new long[(int) o[k]];
            nb.asLongBuffer().get(nbr);
            return new long[][] {o, nbr};
        }

        /** A growable int list. */
        static final class IntArray {
            private int[] a = new int[8];
            private int size;

            void add(int v) {
                if (size == a.length) a = Arrays.copyOf(a, 2 * size);
                a[size++] = v;
            }

            int get(int i) {
                return a[i];
            }

            void pop() {
                --size;
            }

            int size() {
                return size;
            }

            int[] toArray() {
                return Arrays.copyOf(a, size);
            }
        }
    }
}
