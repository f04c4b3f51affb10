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
import org.apache.tinkerpop.gremlin.process.computer.util.GraphComputerHelper;
import org.apache.tinkerpop.gremlin.process.computer.util.VertexProgramHelper;
import org.apache.tinkerpop.gremlin.process.traversal.Path;
import org.apache.tinkerpop.gremlin.process.traversal.Traversal;
import org.apache.tinkerpop.gremlin.process.traversal.step.util.ImmutablePath;
import org.apache.tinkerpop.gremlin.process.traversal.util.PureTraversal;
import org.apache.tinkerpop.gremlin.process.traversal.util.TraversalUtil;
import org.apache.tinkerpop.gremlin.structure.Direction;
import org.apache.tinkerpop.gremlin.structure.Edge;
import org.apache.tinkerpop.gremlin.structure.Graph;
import org.apache.tinkerpop.gremlin.structure.Vertex;
import org.apache.tinkerpop.gremlin.structure.VertexProperty;
import org.apache.tinkerpop.gremlin.structure.util.empty.EmptyGraph;
import org.apache.tinkerpop.gremlin.structure.util.reference.ReferenceFactory;
import org.janusgraph.core.JanusGraphComputer;
import org.janusgraph.core.JanusGraphException;
import org.janusgraph.core.JanusGraphTransaction;
import org.janusgraph.core.schema.JanusGraphManagement;
import org.janusgraph.diskstorage.configuration.Configuration;
import org.janusgraph.diskstorage.keycolumnvalue.scan.ScanMetrics;
import org.janusgraph.diskstorage.keycolumnvalue.scan.StandardScanner;
import org.janusgraph.graphdb.configuration.GraphDatabaseConfiguration;
import org.janusgraph.graphdb.database.StandardJanusGraph;
import org.janusgraph.graphdb.olap.QueryContainer;
import org.janusgraph.graphdb.util.WorkerPool;

import java.lang.reflect.Field;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.Collections;
import java.util.HashMap;
import java.util.HashSet;
import java.util.Iterator;
import java.util.LinkedHashMap;
import java.util.List;
import java.util.Map;
import java.util.Objects;
import java.util.Optional;
import java.util.Set;
import java.util.concurrent.CompletableFuture;
import java.util.concurrent.Future;
import java.util.concurrent.atomic.AtomicInteger;

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
 *       FulgoraGraphComputer.java:249-253 forces), paths rebuilt from the depths.</li>
 * </ul>
 * The edgestore is scanned ONCE into a device CSR (GpuSnapshot) instead of once per superstep. The
 * results then go through Fulgora's own machinery where it applies: the FulgoraMemory of the run,
 * the map phase (columnar emission for PageRankMapReduce / ShortestDistanceMapReduce, otherwise
 * Fulgora's VertexMapJob scan over a FulgoraVertexMemory holding the results), the reduce phase
 * (FulgoraGraphComputer.java:331-357) and the write-back of the non-transient compute keys
 * (:359-471: ORIGINAL in batch transactions, NEW in an uncommitted transaction).
 *
 * Entry: {@code graph.compute(GpuGraphComputer.class)} once JanusGraphBlueprintsGraph.compute(Class)
 * (janusgraph-core/.../tinkerpop/JanusGraphBlueprintsGraph.java:155-161) whitelists this class
 * (java/patches/); the transaction variant delegates to it. Devices: system property
 * janusgraph.computer.gpu.devices (comma list, default "0"); several devices shard the graph 1D.
 */
public class GpuGraphComputer extends FulgoraGraphComputer {

    static final String PR = "org.janusgraph.olap.PageRankVertexProgram";
    static final String SD = "org.janusgraph.olap.ShortestDistanceVertexProgram";
    static final String PR_MAP = "org.janusgraph.olap.PageRankMapReduce";
    static final String SD_MAP = "org.janusgraph.olap.ShortestDistanceMapReduce";
    static final String PAGE_RANK = "janusgraph.pageRank.pageRank";
    static final String EDGE_COUNT = "janusgraph.pageRank.edgeCount";
    static final String DISTANCE = "janusgraph.shortestDistanceVertexProgram.distance";
    static final int SOURCES_PER_BFS = 64; // jg_bfs: one bit-parallel pass per 64 sources

    private static final AtomicInteger COMPUTERS = new AtomicInteger();

    private final StandardJanusGraph graph;
    private final int writeBatchSize;
    private VertexProgram<?> vertexProgram;
    private final Set<MapReduce> mapReduces = new HashSet<>();
    private ResultGraph resultGraphMode;
    private Persist persistMode;
    private int numThreads = 1;
    private boolean filtered;
    private boolean executed;

    public GpuGraphComputer(final StandardJanusGraph graph, final Configuration configuration) {
        super(graph, configuration);
        this.graph = graph;
        this.writeBatchSize = configuration.get(GraphDatabaseConfiguration.BUFFER_SIZE);
    }

    // ---- the GraphComputer builder: recorded here and passed on to Fulgora (the delegate path) ----

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
    public GraphComputer result(final ResultGraph resultGraph) {
        super.result(resultGraph);
        resultGraphMode = resultGraph;
        return this;
    }

    @Override
    public GraphComputer persist(final Persist persist) {
        super.persist(persist);
        persistMode = persist;
        return this;
    }

    @Override
    public JanusGraphComputer workers(final int threads) {
        super.workers(threads);
        numThreads = threads;
        return this;
    }

    @Override
    public GraphComputer program(final VertexProgram program) {
        super.program(program);
        vertexProgram = program;
        return this;
    }

    @Override
    public GraphComputer mapReduce(final MapReduce mapReduce) {
        super.mapReduce(mapReduce);
        mapReduces.add(mapReduce);
        return this;
    }

    // ---- submit ----

    @Override
    public Future<ComputerResult> submit() {
        final GpuProgram run = (vertexProgram == null || filtered) ? null : GpuProgram.recognise(vertexProgram, graph);
        if (run == null) return super.submit(); // everything else stays on Fulgora, unchanged
        if (executed) throw Exceptions.computerHasAlreadyBeenSubmittedAVertexProgram();
        executed = true;
        // FulgoraGraphComputer.ensureSettingsAreValid (:171-190)
        GraphComputerHelper.validateProgramOnComputer(this, vertexProgram);
        mapReduces.addAll(vertexProgram.getMapReducers());
        persistMode = GraphComputerHelper.getPersistState(Optional.of(vertexProgram), Optional.ofNullable(persistMode));
        resultGraphMode = GraphComputerHelper.getResultGraphState(Optional.of(vertexProgram),
            Optional.ofNullable(resultGraphMode));
        if (!features().supportsResultGraphPersistCombination(resultGraphMode, persistMode))
            throw Exceptions.resultGraphPersistCombinationNotSupported(resultGraphMode, persistMode);
        final FulgoraMemory memory = new FulgoraMemory(vertexProgram, mapReduces);
        return CompletableFuture.supplyAsync(() -> submitAsync(run, memory));
    }

    private ComputerResult submitAsync(final GpuProgram run, final FulgoraMemory memory) {
        final long time = System.currentTimeMillis();
        vertexProgram.setup(memory);
        final long[] h = new long[1];
        JanusGpu.check(JanusGpu.ctxCreate(devices(), h));
        final long ctx = h[0];
        final Results res;
        try {
            final long g = GpuSnapshot.scan(graph, ctx, run.adjacency(), run.weightProperty(), queryLimit(),
                run.inEntries());
            try {
                final long[] vid = GpuSnapshot.vertexIds(g);
                res = run.execute(g, vid, graph, memory);
            } finally {
                JanusGpu.graphDestroy(g);
            }
        } finally {
            JanusGpu.ctxDestroy(ctx);
        }
        // supersteps 0..K ran: Fulgora's memory counts K + 1 and complete() reports K (FulgoraMemory.java:97-101)
        memory.setIteration(res.iteration + 1);
        executeMapReduce(res, memory);
        final Graph resultGraph = writeBack(res);
        memory.setRuntime(System.currentTimeMillis() - time);
        memory.complete();
        return new DefaultComputerResult(resultGraph, memory);
    }

    /**
     * Fulgora's hard limit on the entries of a non-fitted slice (QueryContainer.DEFAULT_HARD_QUERY_LIMIT,
     * olap/QueryContainer.java:42,133): the snapshot reproduces it, so vertices with more than 100000
     * edge entries get exactly the truncated adjacency Fulgora computes on.  The system property
     * janusgraph.computer.gpu.untruncated=true computes on every entry instead.
     */
    private static long queryLimit() {
        return Boolean.getBoolean("janusgraph.computer.gpu.untruncated") ? 0L : QueryContainer.DEFAULT_HARD_QUERY_LIMIT;
    }

    private static int[] devices() {
        final String[] parts = System.getProperty("janusgraph.computer.gpu.devices", "0").split(",");
        final int[] d = new int[parts.length];
        for (int i = 0; i < parts.length; i++) d[i] = Integer.parseInt(parts[i].trim());
        return d;
    }

    static ByteBuffer direct(long bytes) {
        if (bytes > Integer.MAX_VALUE)
            throw new JanusGraphException("GPU computer: " + bytes + " bytes exceed one direct buffer; the graph has "
                + "more than 2^28 vertices");
        return ByteBuffer.allocateDirect((int) Math.max(bytes, 8)).order(ByteOrder.nativeOrder());
    }

    // ---- map / reduce (FulgoraGraphComputer.java:288-357) ----

    private void executeMapReduce(final Results res, final FulgoraMemory memory) {
        final Map<MapReduce, FulgoraMapEmitter> mapJobs = new LinkedHashMap<>();
        for (MapReduce mr : mapReduces)
            if (mr.doStage(MapReduce.Stage.MAP)) mapJobs.put(mr, new FulgoraMapEmitter<>(mr.doStage(MapReduce.Stage.REDUCE)));
        if (mapJobs.isEmpty()) return;
        boolean columnar = true;
        for (MapReduce mr : mapJobs.keySet()) {
            final String name = mr.getClass().getName();
            columnar &= name.equals(PR_MAP) || name.equals(SD_MAP);
        }
        if (columnar) {
            // PageRankMapReduce / ShortestDistanceMapReduce.map emit (vertex.id(), the compute key's value)
            // where it is present (PageRankMapReduce.java:62-67, ShortestDistanceMapReduce.java:59-64):
            // emitted straight from the result columns, without a second edgestore scan.
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
        } else {
            // any other MapReduce sees what Fulgora gives it: the scanned vertices with the compute keys
            // mixed in from a FulgoraVertexMemory (VertexMapJob.java:107-130)
            final FulgoraVertexMemory vertexMemory = res.toVertexMemory(graph, vertexProgram);
            try (VertexMapJob.Executor job = VertexMapJob.getVertexMapJob(graph, vertexMemory, mapJobs)) {
                final StandardScanner.Builder scan = graph.getBackend().buildEdgeScanJob();
                scan.setJobId("gpu" + COMPUTERS.incrementAndGet() + "#map");
                scan.setNumProcessingThreads(numThreads);
                scan.setWorkBlockSize(writeBatchSize * 10);
                scan.setJob(job);
                final ScanMetrics metrics = scan.execute().get();
                if (metrics.get(ScanMetrics.Metric.FAILURE) > 0)
                    throw new JanusGraphException("Failed to process [" + metrics.get(ScanMetrics.Metric.FAILURE)
                        + "] vertices in map phase. Computer is aborting.");
                if (metrics.getCustom(VertexMapJob.MAP_JOB_FAILURE) > 0)
                    throw new JanusGraphException("Failed to process [" + metrics.getCustom(VertexMapJob.MAP_JOB_FAILURE)
                        + "] individual map jobs. Computer is aborting.");
            } catch (JanusGraphException e) {
                throw e;
            } catch (Exception e) {
                throw new JanusGraphException(e);
            }
        }
        for (Map.Entry<MapReduce, FulgoraMapEmitter> mapJob : mapJobs.entrySet()) {
            final FulgoraMapEmitter<?, ?> mapEmitter = mapJob.getValue();
            final MapReduce mapReduce = mapJob.getKey();
            mapEmitter.complete(mapReduce);
            if (mapReduce.doStage(MapReduce.Stage.REDUCE)) {
                final FulgoraReduceEmitter<?, ?> reduceEmitter = new FulgoraReduceEmitter<>();
                try (WorkerPool workers = new WorkerPool(numThreads)) {
                    workers.submit(() -> mapReduce.workerStart(MapReduce.Stage.REDUCE));
                    for (final Map.Entry queueEntry : mapEmitter.reduceMap.entrySet()) {
                        if (null == queueEntry) break;
                        workers.submit(() -> mapReduce.reduce(queueEntry.getKey(),
                            ((Iterable) queueEntry.getValue()).iterator(), reduceEmitter));
                    }
                    workers.submit(() -> mapReduce.workerEnd(MapReduce.Stage.REDUCE));
                } catch (Exception e) {
                    throw new JanusGraphException("Exception while executing reduce phase", e);
                }
                reduceEmitter.complete(mapReduce);
                mapReduce.addResultToMemory(memory, reduceEmitter.reduceQueue.iterator());
            } else {
                mapReduce.addResultToMemory(memory, mapEmitter.mapQueue.iterator());
            }
        }
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

    static Column doubles(String key, ByteBuffer buf) {
        return new Column(key) {
            @Override
            Object get(int i) {
                final double d = buf.getDouble(8 * i);
                return Double.isNaN(d) ? null : d; // NaN: no superstep wrote the property (K == 0)
            }
        };
    }

    static Column distances(String key, ByteBuffer buf) {
        return new Column(key) {
            @Override
            Object get(int i) {
                final long l = buf.getLong(8 * i);
                return l == JanusGpu.DIST_ABSENT ? null : l;
            }
        };
    }

    static Column components(String key, ByteBuffer buf) {
        return new Column(key) {
            @Override
            Object get(int i) {
                return Long.toString(buf.getLong(8 * i)); // the label is the id's String form
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

        abstract Results execute(long g, long[] vid, StandardJanusGraph graph, FulgoraMemory memory);

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
        Results execute(long g, long[] vid, StandardJanusGraph graph, FulgoraMemory memory) {
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
        Results execute(long g, long[] vid, StandardJanusGraph graph, FulgoraMemory memory) {
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
            conf.getKeys().forEachRemaining(k -> {
                if (property.equals(String.valueOf(conf.getProperty(k)))) free.add(k);
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
        Results execute(long g, long[] vid, StandardJanusGraph graph, FulgoraMemory memory) {
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
     * shortestPaths memory key. Depths come from the GPU (DIR_BOTH, the forced scope); paths are
     * walked back from each target over neighbours one level closer.
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
        Results execute(long g, long[] vid, StandardJanusGraph graph, FulgoraMemory memory) {
            final JanusGraphTransaction tx = graph.buildTransaction().readOnly().start();
            try {
                final List<Integer> sources = new ArrayList<>();
                final boolean[] target = new boolean[vid.length];
                final Map<Long, Integer> index = new HashMap<>();
                for (int i = 0; i < vid.length; i++) {
                    index.put(vid[i], i);
                    final Vertex v = (sourceFilter == null && targetFilter == null) ? null : tx.getVertex(vid[i]);
                    if (sourceFilter == null || TraversalUtil.test(v, sourceFilter.clone())) sources.add(i);
                    target[i] = targetFilter == null || TraversalUtil.test(v, targetFilter.clone());
                }
                final List<Path> paths = new ArrayList<>();
                int maxLevel = 0;
                for (int b = 0; b < sources.size(); b += SOURCES_PER_BFS) {
                    final int k = Math.min(SOURCES_PER_BFS, sources.size() - b);
                    final ByteBuffer src = direct(8L * k), depth = direct(4L * k * vid.length);
                    for (int j = 0; j < k; j++) src.putLong(vid[sources.get(b + j)]);
                    JanusGpu.check(JanusGpu.bfs(g, src, k, JanusGpu.DIR_BOTH, maxDistance, depth));
                    for (int j = 0; j < k; j++) {
                        final int s = sources.get(b + j);
                        final int base = 4 * j * vid.length;
                        for (int t = 0; t < vid.length; t++) {
                            final int d = depth.getInt(base + 4 * t);
                            if (d < 0 || !target[t]) continue;
                            maxLevel = Math.max(maxLevel, d);
                            walkBack(tx, vid, index, depth, base, s, t, new ArrayList<>(), paths);
                        }
                    }
                }
                memory.set(ShortestPathVertexProgram.SHORTEST_PATHS, paths);
                return new Results(vid, maxLevel + 1);
            } finally {
                tx.rollback();
            }
        }

        /** Every shortest s..t path, walking from t to neighbours one level closer to s. */
        private static void walkBack(JanusGraphTransaction tx, long[] vid, Map<Long, Integer> index, ByteBuffer depth,
                                     int base, int s, int t, List<Integer> suffix, List<Path> out) {
            suffix.add(t);
            if (t == s) {
                Path p = ImmutablePath.make();
                for (int i = suffix.size() - 1; i >= 0; i--)
                    p = p.extend(ReferenceFactory.detach(tx.getVertex(vid[suffix.get(i)])), Collections.emptySet());
                out.add(p);
            } else {
                final int dt = depth.getInt(base + 4 * t);
                final Set<Integer> seen = new HashSet<>();
                for (Iterator<Vertex> it = tx.getVertex(vid[t]).vertices(Direction.BOTH); it.hasNext(); ) {
                    final Integer u = index.get((Long) it.next().id());
                    if (u != null && seen.add(u) && depth.getInt(base + 4 * u) == dt - 1)
                        walkBack(tx, vid, index, depth, base, s, u, suffix, out);
                }
            }
            suffix.remove(suffix.size() - 1);
        }
    }
}
