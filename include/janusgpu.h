/*
 * janusgpu.h — C-ABI of libjanusgpu, the MI355X (gfx950) OLAP graph-computer engine
 * behind GpuGraphComputer, the drop-in for JanusGraph's FulgoraGraphComputer.
 *
 * Plain C: pointers + sizes, no torch / HIP / C++ types.  Every entry point returns an int
 * status (JG_OK = 0, < 0 = error class) and never throws or aborts across the ABI; the message
 * of the last failure on the calling thread is available from jg_last_error().
 *
 * What each entry point replaces in the reference (paths relative to
 * /root/reference/janusgraph-core/src/main/java/org/janusgraph/):
 *
 *   jg_ctx_create / jg_ctx_create_rank
 *       FulgoraGraphComputer(StandardJanusGraph, Configuration) + workers(n)
 *       graphdb/olap/computer/FulgoraGraphComputer.java:101-106,134-139
 *   jg_graph_build
 *       the per-superstep edgestore scan: StandardScannerExecutor.run
 *       (diskstorage/keycolumnvalue/scan/StandardScannerExecutor.java:97-216) feeding
 *       VertexJobConverter.process (graphdb/olap/VertexJobConverter.java:122-151: ghost skip)
 *       and the canonical-id map (graphdb/olap/computer/FulgoraVertexMemory.java:74-77).
 *       Done ONCE per computer instead of once per superstep.
 *   jg_graph_build_edgestore
 *       the same, from the raw rows: the row decode of VertexJobConverter.process and
 *       EdgeSerializer.parseRelation (graphdb/database/EdgeSerializer.java:86-122) on the GPU
 *   jg_pagerank (+ begin/step/end)
 *       executeVertexProgram superstep loop (FulgoraGraphComputer.java:210-230) running
 *       janusgraph-backend-testutils/.../olap/PageRankVertexProgram.java:89-110, with the gather of
 *       VertexMemoryHandler.receiveMessages (graphdb/olap/computer/VertexMemoryHandler.java:121-151)
 *   jg_shortest_distance
 *       the same loop running ShortestDistanceVertexProgram.java:112-146 with
 *       ShortestDistanceMessageCombiner.java:29-31 (min)
 *   jg_bfs
 *       TinkerPop ShortestPathVertexProgram under Fulgora's forced {Local(bothE), Global} scopes
 *       (FulgoraGraphComputer.java:249-253): hop depth per source (paths are rebuilt host-side)
 *   jg_connected_components
 *       TinkerPop ConnectedComponentVertexProgram (String-min label over BOTH edges,
 *       VertexProgramScanJob.java:113-135 loads BOTH); pinned by OLAPTest.java:736-762
 *   jg_combine_steps
 *       the same loop for sum/min/max MessageCombiner programs (OLAPTest.DegreeCounter,
 *       janusgraph-test/.../olap/OLAPTest.java:424-503; VertexState.java:85-114)
 *   jg_graph_info_get / jg_ctx_last_stats
 *       ScanMetrics counters (StandardScanMetrics.java:28-88: ghost-vertices, truncated-results)
 *       and memory().getIteration()/getRuntime() (FulgoraMemory.java:97-101)
 *
 * Ownership: host arrays passed in are caller-owned and read only during the call; outputs are
 * caller-allocated.  Device memory is owned by the library (per jg_graph) and handed back to the
 * device by jg_graph_destroy (the library's block cache, which spares a build its ~250 device
 * synchronising frees, is emptied there and by jg_ctx_trim).  A jg_ctx is not re-entrant: one call in
 * flight per context, and a jg_graph belongs to its context's caller thread (read-only queries such as
 * jg_graph_neighbors may run from several threads: their lazily made host copies are locked).
 */
#ifndef JANUSGPU_H
#define JANUSGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: jg_graph_info.exchange_values appended; jg_bfs_rows, jg_graph_neighbors added.
 * 3: jg_bfs_keep, jg_bfs_kept_row, jg_bfs_kept_release, jg_ctx_trim added.  Callers must check
 * jg_abi_version() == JG_ABI_VERSION before passing any struct across the ABI. */
#define JG_ABI_VERSION 3

/* ---- status codes ---- */
#define JG_OK               0
#define JG_ERR_ARG         -1  /* bad argument (null pointer, size, unknown vertex id …)        */
#define JG_ERR_OOM         -2  /* device or host allocation failed                                */
#define JG_ERR_HIP         -3  /* HIP runtime error                                               */
#define JG_ERR_RCCL        -4  /* RCCL communicator / collective error                            */
#define JG_ERR_UNSUPPORTED -5  /* operation not available for this graph/context configuration  */
#define JG_ERR_STATE       -6  /* call out of order (e.g. step before begin)                      */

/* ---- adjacency requested at build time (bit flags) ---- */
#define JG_ADJ_OUT  1u  /* out-adjacency: rows = source vertex (bottom-up of IN traversals)        */
#define JG_ADJ_IN   2u  /* in-adjacency:  rows = target vertex (PageRank pull, SD push)           */
#define JG_ADJ_BOTH 4u  /* symmetrised:   rows = every vertex, a self-loop appears twice (BOTH)   */

/* ---- traversal direction (the MessageScope.Local incident traversal) ---- */
#define JG_DIR_OUT  1   /* follow u->v edges from u          */
#define JG_DIR_IN   2   /* follow u->v edges from v back to u */
#define JG_DIR_BOTH 3

/* Fulgora's hard limit on entries per non-BOTH slice (graphdb/olap/QueryContainer.java:42,133) */
#define JG_FULGORA_HARD_QUERY_LIMIT 100000

typedef struct jg_ctx jg_ctx;
typedef struct jg_graph jg_graph;

typedef struct jg_graph_info {
    int64_t num_vertices;        /* |V| handed to the build (existing, non-ghost vertices)          */
    int64_t num_edges;           /* edges kept: both endpoints in V                                  */
    int64_t ghost_edges;         /* edges dropped because an endpoint is not in V                    */
    int64_t self_loops;          /* kept edges with src == dst                                       */
    int64_t truncated_vertices;  /* without a query limit: vertices with > JG_FULGORA_HARD_QUERY_LIMIT
                                    edge entries (in+out), whose OUT/IN slices Fulgora truncates and
                                    this graph does not.  Built with jg_builder_set_query_limit: the
                                    rows whose edge slice reached the limit (Fulgora's
                                    truncated-results metric, VertexJobConverter.java:139)          */
    int64_t max_in_degree;
    int64_t max_out_degree;
    int64_t device_bytes;        /* device memory held by this graph, summed over shards             */
    int32_t num_shards;          /* 1D vertex partitions (one per device / rank)                    */
    uint32_t flags;              /* JG_ADJ_* actually built                                          */
    int64_t exchange_values;     /* vertex values this process's shards receive from peers per
                                    exchange step of the pull vector (IN adjacency if built, else
                                    BOTH): the sparse halo, or (P-1)*S each for the dense allgather;
                                    0 on one shard                                                   */
} jg_graph_info;

typedef struct jg_stats {
    int32_t supersteps;          /* memory().getIteration() of the equivalent Fulgora run           */
    int32_t levels;              /* passes actually executed on the GPU; the unit depends on the path:
                                  * BFS: levels; CC: union-find BFS levels or propagation sweeps;
                                  * shortest distance: supersteps (hop-bounded Bellman-Ford) or, on the
                                  * unbounded delta-stepping path, near-far passes      */
    double  build_ms;            /* last jg_graph_build*: snapshot -> CSR on device                 */
    double  compute_ms;          /* last program: HIP-event time of the superstep loop              */
    double  exchange_ms;         /* HIP-event time of the exchange steps (profiling on, sharded)    */
    double  kernel_ms_total;     /* sum of HIP-event durations of the dominant kernel                */
    int64_t kernel_launches;     /* number of launches of the dominant kernel that were timed       */
    double  algorithmic_bytes;   /* SURVEY §8(d) byte model for the last program, whole run         */
    double  edges_traversed;     /* adjacency entries examined (for TEPS)                           */
} jg_stats;

/* ---- library / context ---- */
int         jg_abi_version(void);
const char* jg_last_error(void);

/* One process driving `ndev` devices (the JVM case).  ndev > 1 shards the graph 1D over the listed
 * devices; distinct devices exchange through RCCL (ncclCommInitAll), a device listed more than once
 * holds several logical shards that exchange by device copies (test mode). */
int jg_ctx_create(const int* devices, int ndev, jg_ctx** out);

/* One process per GPU (torch.distributed style): this process is `rank` of `nranks`, driving
 * `device`.  `unique_id` is the JG_UNIQUE_ID_BYTES blob from jg_comm_unique_id() on rank 0,
 * broadcast out-of-band by the caller.  nranks == 1 needs no unique_id (may be NULL). */
#define JG_UNIQUE_ID_BYTES 128
int jg_comm_unique_id(void* out /* JG_UNIQUE_ID_BYTES */);
int jg_ctx_create_rank(int device, int nranks, int rank, const void* unique_id, jg_ctx** out);
/* The same rank mode over a caller-supplied host transport instead of RCCL: every exchange step is
 * staged through host memory and handed to these callbacks (synchronous, called by every rank in
 * the same order).  For tests of the multi-process control flow where RCCL cannot run (two ranks
 * on one GPU); the same code paths build, plan, pack and place the data as with RCCL.
 *   allgather: out[r * bytes .. (r + 1) * bytes) = rank r's `in`, for every rank r.
 *   exchange:  send[i] (send_bytes[i] bytes) to rank send_peer[i]; receive recv_bytes[i] bytes from
 *              rank recv_peer[i] into recv[i].  Zero-byte transfers are not listed.
 * Callbacks return 0 on success.  `t` is copied; `t->user` is passed back untouched. */
typedef struct jg_transport {
    void* user;
    int (*allgather)(void* user, const void* in, void* out, size_t bytes);
    int (*exchange)(void* user, int nsend, const int* send_peer, const void* const* send, const size_t* send_bytes,
                    int nrecv, const int* recv_peer, void* const* recv, const size_t* recv_bytes);
} jg_transport;
int jg_ctx_create_rank_transport(int device, int nranks, int rank, const jg_transport* t, jg_ctx** out);
/* Lifetime: every jg_graph and jg_builder made from a context uses its streams and communicators, so
 * destroy them before the context.  While any is alive jg_ctx_destroy changes nothing and returns
 * JG_ERR_STATE (the context stays valid: destroy the graphs/builders, then call it again). */
int jg_ctx_destroy(jg_ctx* ctx);
/* Hands the device memory the library caches for reuse (freed blocks) back to the context's devices. */
int jg_ctx_trim(jg_ctx* ctx);
int jg_ctx_last_stats(const jg_ctx* ctx, jg_stats* out);
/* Record HIP events around every launch of the dominant kernel (costs ~1 us per launch). */
int jg_ctx_set_profiling(jg_ctx* ctx, int enable);

/* ---- graph snapshot ---- */
/* vid[n]: the ids of the vertices the scan returned (unique, any order; outputs are indexed the same
 * way).  src/dst[m]: edge endpoints as vertex ids; an edge whose endpoint is not in vid is a ghost
 * edge and is dropped.  weight[m] (nullable): Integer edge property for jg_shortest_distance; NULL
 * means unit weights.  Multi-edges and self-loops are kept (JanusGraph MULTI semantics). */
int jg_graph_build(jg_ctx* ctx, const int64_t* vid, int64_t n,
                   const int64_t* src, const int64_t* dst, const int32_t* weight, int64_t m,
                   uint32_t flags, jg_graph** out);

/* The same snapshot straight from the edgestore rows the scan returns, decoded on the GPU
 * (replaces VertexJobConverter.process + EdgeSerializer.parseRelation per row and entry:
 * graphdb/olap/VertexJobConverter.java:122-151,169-181; graphdb/database/EdgeSerializer.java:86-122;
 * graphdb/idmanagement/IDManager.java:496-506).  Row r has key row_keys[r] (the 8-byte big-endian
 * StaticBuffer as an unsigned value) and entries [row_entry_off[r], row_entry_off[r+1]); entry e is
 * bytes[entry_off[e] .. entry_off[e+1]) with its value at value_pos[e] (as jg_decode_edges; the
 * type table gives edge-label multiplicities).  Rows with an odd key (schema / invisible vertices)
 * are filtered; a row whose first entry is not the VertexExists property is a ghost; the kept rows
 * are V (in row order, ids -> vid_out[nrows], count -> *num_vertices_out, both nullable) and their
 * OUT entries of visible user edges are the edges (ghost endpoints dropped as in jg_graph_build).
 * Unit weights.  Partitioned (vertex-cut) vertices are one vertex, the canonical id
 * (IDManager.java:525-551): every representative row adds its edges, only the canonical row's
 * VertexExists decides the ghost rule (VertexProgramScanJob.java:88-102).  A malformed entry on a
 * kept row or a key with no user vertex type: JG_ERR_ARG.  Stats: build_ms (whole snapshot),
 * exchange_ms (the row copies), kernel_ms_total (copies + decode kernels). */
int jg_graph_build_edgestore(jg_ctx* ctx, const uint64_t* row_keys, int64_t nrows, const int64_t* row_entry_off,
                             const uint8_t* bytes, int64_t nbytes, const int64_t* entry_off, const int32_t* value_pos,
                             int64_t nentries, const int64_t* type_ids, const int8_t* type_mult, int32_t ntypes,
                             int32_t partition_bits, uint32_t flags, int64_t* vid_out, int64_t* num_vertices_out,
                             jg_graph** out);

/* ---- chunked snapshot ----
 * The same two snapshots fed in chunks as the scan produces them (Java direct ByteBuffers hold at most
 * 2 GiB, and the scan is a stream: StandardScannerExecutor.java:141-174 hands rows to the processors
 * in key order).  Either ids (add_vertices / add_edges, any interleaving; edge weights on every
 * add_edges call or on none) or raw rows (set_schema once, then add_rows; a row never spans two
 * chunks), not both.  Each add_rows call stages its chunk and returns while the chunk is copied and
 * decoded on the GPU, so the decode overlaps the caller's scan of the next chunk.  finish builds the
 * graph exactly as jg_graph_build / jg_graph_build_edgestore would from the concatenated chunks
 * (vertex order = the order added; read it back with jg_graph_vertex_ids).  The builder is single-use;
 * destroy it after finish (or instead of it).  Stats of finish: build_ms, kernel_ms_total = copy +
 * decode time of the rows (HIP events per chunk, summed), exchange_ms = their host -> device copies
 * alone, kernel_launches = number of row chunks.  Chunks whose entries are all shorter than 256 bytes
 * cross PCIe with 1-byte lengths and value positions instead of the int64 offsets and int32 positions. */
typedef struct jg_builder jg_builder;
int jg_builder_create(jg_ctx* ctx, jg_builder** out);
int jg_builder_add_vertices(jg_builder* b, const int64_t* vid, int64_t n);
int jg_builder_add_edges(jg_builder* b, const int64_t* src, const int64_t* dst, const int32_t* weight, int64_t m);
int jg_builder_set_schema(jg_builder* b, const int64_t* type_ids, const int8_t* type_mult, int32_t ntypes,
                          int32_t partition_bits);
/* entry_weight[nentries] (nullable; on every chunk or none): the Integer weight property of each
 * entry's edge for jg_shortest_distance (JG_WEIGHT_ABSENT: the edge has none), read by the caller
 * with the edge's own serializer; ignored for entries that are not kept edges. */
int jg_builder_add_rows(jg_builder* b, const uint64_t* row_keys, int64_t nrows, const int64_t* row_entry_off,
                        const uint8_t* bytes, int64_t nbytes, const int64_t* entry_off, const int32_t* value_pos,
                        const int32_t* entry_weight, int64_t nentries);
/* Fulgora's per-row slice cap (graphdb/olap/QueryContainer.java:42,121-146): an untyped OUT or IN edge
 * scope is not a fitted query (query/vertex/BasicVertexCentricQueryBuilder.java:451-456), so the scan
 * loads each row's EDGE slice (IDHandler.getBounds(EDGE), idhandling/IDHandler.java:172-193: the visible
 * user edges of both directions, contiguous in column order) with at most `limit` entries
 * (inmemory/SinglePageEntryBuffer.java:54-77 stops there), and a program reads only the entries of its
 * direction among them.  With limit > 0 (JG_FULGORA_HARD_QUERY_LIMIT reproduces Fulgora) the graph is
 * built from what the programs would read: the OUT adjacency and out-degrees (PageRank's edgeCount)
 * from the OUT entries within their row's first `limit`; the IN adjacency, for in_entries = JG_DIR_IN,
 * from the IN entries within their row's first `limit` (PageRank's gather and a combiner over IN:
 * receivers read their own IN entries) or, for JG_DIR_OUT, as the transpose of the capped OUT entries
 * (ShortestDistance: a receiver reads its OUT entries, the IN adjacency is pushed along); BOTH is a
 * fitted query and never capped.  limit = 0 (the default) builds the untruncated graph.  Rows only
 * (jg_builder_add_rows); call before the first chunk. */
int jg_builder_set_query_limit(jg_builder* b, int64_t limit, int32_t in_entries);
/* Edge weights decoded on the GPU from the rows (ShortestDistanceVertexProgram's Integer property,
 * ShortestDistanceVertexProgram.java:69) instead of per-entry host weights: an edge's properties follow
 * its ids in its value as (inline key id, value) pairs in ascending key-id order
 * (graphdb/database/EdgeSerializer.java:294-302; inline id = IDManager.stripRelationTypePadding(key id),
 * VariableLong.writePositive, idhandling/IDHandler.java:155-158; values per StandardSerializer.writeObject:
 * a null flag byte unless String, then the attribute serializer's bytes).  weight_key = the inline id of the
 * weight key; key_ids / key_types (nkeys) = every property key an edge may carry before it, with its
 * JG_PROP_* type (an edge holding a key of unknown type before the weight: JG_ERR_UNSUPPORTED at finish).
 * The weight is JG_WEIGHT_ABSENT where the edge has no non-null Integer value for the key; a stored
 * Integer.MIN_VALUE collides with that marker and fails the build (JG_ERR_UNSUPPORTED).  The edge labels
 * must have no signature keys (their values precede the inline pairs without ids): the caller checks.
 * Rows only, before the first chunk; add_rows then takes no entry_weight. */
#define JG_PROP_BYTE   1
#define JG_PROP_SHORT  2
#define JG_PROP_INT    3
#define JG_PROP_LONG   4
#define JG_PROP_CHAR   5
#define JG_PROP_BOOL   6
#define JG_PROP_DATE   7
#define JG_PROP_FLOAT  8
#define JG_PROP_DOUBLE 9
#define JG_PROP_UUID   10
#define JG_PROP_STRING 11
int jg_builder_set_weight_key(jg_builder* b, int64_t weight_key, const int64_t* key_ids, const int8_t* key_types,
                              int32_t nkeys);
int jg_builder_finish(jg_builder* b, uint32_t flags, jg_graph** out);
int jg_builder_destroy(jg_builder* b);
/* vid_out[i] = the id of vertex offset + i in output order (the order vid[] / the kept rows were given). */
int jg_graph_vertex_ids(const jg_graph* g, int64_t offset, int64_t count, int64_t* vid_out);

/* Synthetic Graph500 Kronecker (RMAT a,b,c,d = .57,.19,.19,.05) graph generated on the device(s):
 * n = 2^scale vertices with ids 0..n-1, m = edgefactor * n directed edges, seeded and
 * bit-identical to oracle/jg_oracle.c:jo_rmat_edges. */
int jg_graph_build_rmat(jg_ctx* ctx, int scale, int edgefactor, uint64_t seed, uint32_t flags,
                        jg_graph** out);
int jg_graph_info_get(const jg_graph* g, jg_graph_info* out);
int jg_graph_destroy(jg_graph* g);

/* ---- programs ---- */
/* JanusGraph PageRankVertexProgram: `iterations` = maxIterations K (supersteps 0..K, i.e. K-1 power
 * steps), `vertex_count` = the user-supplied vertexCount N (NOT |V|).  rank_out[n] / edge_count_out[n]
 * (nullable) receive janusgraph.pageRank.pageRank / .edgeCount; with K == 0 no property is written
 * and rank_out is filled with NaN. */
int jg_pagerank(jg_graph* g, double damping, int64_t vertex_count, int32_t iterations,
                double* rank_out, double* edge_count_out);
/* The same run split for benchmarking: begin = supersteps 0 and 1, step = `nsteps` power supersteps
 * enqueued asynchronously, end = synchronise + copy results (either pointer nullable). */
int jg_pagerank_begin(jg_graph* g, double damping, int64_t vertex_count);
int jg_pagerank_step(jg_graph* g, int32_t nsteps);
int jg_pagerank_end(jg_graph* g, double* rank_out, double* edge_count_out);

/* ShortestDistanceVertexProgram: dist_out[v] = min over paths v -> ... -> seed of <= max_depth hops
 * of the summed edge weights (int64; weights may be negative), or JG_DIST_ABSENT where Fulgora leaves
 * DISTANCE absent.  A weight of JG_WEIGHT_ABSENT marks an edge without the weight property: if a
 * message crosses one, the run fails with JG_ERR_ARG (Fulgora's edge function throws there,
 * ShortestDistanceVertexProgram.java:69); untraversed ones are harmless. */
#define JG_DIST_ABSENT INT64_MIN
#define JG_WEIGHT_ABSENT INT32_MIN
int jg_shortest_distance(jg_graph* g, int64_t seed_vid, int32_t max_depth, int64_t* dist_out);

/* Hop depth from each of nsrc sources (nsrc <= 64 runs as one bit-parallel multi-source BFS);
 * depth_out[s * n + v] = hops or -1 (unreached / beyond max_depth; max_depth < 0 = unbounded).
 * depth_out may be NULL (benchmarking: results stay on the device). */
int jg_bfs(jg_graph* g, const int64_t* source_vids, int32_t nsrc, int32_t direction,
           int32_t max_depth, int32_t* depth_out);

/* The same traversal with one output row per source: depth_rows[s] (nullable, and the array itself)
 * receives n int32 depths.  A Java direct buffer holds at most 2 GiB, so the 64 rows of one
 * bit-parallel batch cannot share one buffer past 2^23 vertices (ShortestPathVertexProgram batches,
 * java/.../GpuGraphComputer.java ShortestPaths). */
int jg_bfs_rows(jg_graph* g, const int64_t* source_vids, int32_t nsrc, int32_t direction, int32_t max_depth,
                int32_t* const* depth_rows);

/* The same traversal (nsrc <= 64: one bit-parallel batch) with its depth rows kept on the device;
 * jg_bfs_kept_row(g, s, depth_out) then copies row s (n int32, caller order) into a caller buffer, so a
 * caller that consumes the rows one at a time holds one n-int32 buffer instead of nsrc of them
 * (ShortestPathVertexProgram's batches at n = 2^26: one 268 MB row instead of 17 GB of direct buffers,
 * java/.../GpuGraphComputer.java ShortestPaths).  The rows stay until the next jg_bfs_keep, until
 * jg_bfs_kept_release or until jg_graph_destroy; jg_bfs_kept_row fails with JG_ERR_ARG for s outside
 * [0, nsrc of the last jg_bfs_keep).  Replaces FulgoraVertexMemory's per-vertex path state
 * (graphdb/olap/computer/FulgoraVertexMemory.java:52-123) for the bit-parallel batch. */
int jg_bfs_keep(jg_graph* g, const int64_t* source_vids, int32_t nsrc, int32_t direction, int32_t max_depth);
int jg_bfs_kept_row(jg_graph* g, int32_t s, int32_t* depth_out);
int jg_bfs_kept_release(jg_graph* g);

/* Adjacency of vertices rows[0, nrows) (output-order indices), in output-order indices: the host copy
 * of the snapshot a path walk-back reads where Fulgora re-reads each vertex's preloaded BOTH slice
 * (graphdb/olap/computer/VertexProgramScanJob.java:113-135).  direction JG_DIR_BOTH (a self-loop
 * appears twice, multi-edges repeat), JG_DIR_OUT or JG_DIR_IN (the adjacency must have been built).
 * off_out[nrows + 1] = exclusive prefix of the rows' entry counts; nbr_out[off_out[nrows]] (nullable:
 * size first, then fill) = the neighbours.  Rank mode (jg_ctx_create_rank*): entry counts only
 * (nbr_out must be NULL, else JG_ERR_UNSUPPORTED), and rows of other ranks count 0 entries. */
int jg_graph_neighbors(const jg_graph* g, int32_t direction, const int64_t* rows, int64_t nrows, int64_t* off_out,
                       int64_t* nbr_out);

/* ConnectedComponentVertexProgram: component_vid_out[v] = the vertex id whose decimal String is the
 * component label (the String-minimum id of v's weakly connected component).  iterations_out
 * (nullable) = supersteps of the synchronous program. */
int jg_connected_components(jg_graph* g, int64_t* component_vid_out, int32_t* iterations_out);

/* Combiner vertex programs (the DegreeCounter family, janusgraph-test/.../olap/OLAPTest.java:424-503):
 * x_0 = init[v] (NULL: every vertex sends 1), then `steps` supersteps of
 *     x_t[v] = COMBINE over the entries (v, w) of v's `direction` adjacency of x_{t-1}[w]
 * (JG_DIR_OUT: v's out-edges, i.e. messages sent on Local.of(inE); one term per edge).  COMBINE is
 * JG_COMBINE_SUM (a vertex with no entries gets 0, as reduce(0, +)), _MIN or _MAX (no entries: the
 * identity, and received_out[v] = 0).  int32_wrap != 0: Java Integer values (inputs truncated to
 * int32, sums modulo 2^32).  out[n] = x_steps; received_out[n] (nullable) = v had at least one term
 * in the last superstep.  Needs the matching adjacency at build time; sharded graphs exchange the messages every superstep. */
#define JG_COMBINE_SUM 0
#define JG_COMBINE_MIN 1
#define JG_COMBINE_MAX 2
int jg_combine_steps(jg_graph* g, int32_t direction, int32_t combiner, int32_t int32_wrap, const int64_t* init,
                     int32_t steps, int64_t* out, uint8_t* received_out);

/* Decode n edgestore entries on the context's first GPU, as EdgeSerializer.parseRelation does
 * (core/graphdb/database/EdgeSerializer.java:86-122; header: IDHandler.readRelationType,
 * idhandling/IDHandler.java:130-141; varints: idhandling/VariableLong.java:44-52,193-208,276-294).
 * Entry i is bytes[entry_off[i] .. entry_off[i+1]) (column then value), value_pos[i] its value
 * position (the column length).  type_ids / type_mult (ntypes, may be 0) give the multiplicity of
 * edge labels: 0 MULTI, 1 SIMPLE, 2 ONE2MANY, 3 MANY2ONE, 4 ONE2ONE (core/core/Multiplicity.java);
 * labels absent from the table are MULTI.  Outputs per entry (each nullable): the relation type id,
 * dir_out = 0 OUT edge, 1 IN edge, 2 property, 3 system relation, -1 malformed; the other vertex id
 * and the relation id (-1 unless a user edge).  Stats: compute_ms = kernel time. */
int jg_decode_edges(jg_ctx* ctx, const uint8_t* bytes, int64_t nbytes, const int64_t* entry_off,
                    const int32_t* value_pos, int64_t n, const int64_t* type_ids, const int8_t* type_mult,
                    int32_t ntypes, int64_t* type_out, int8_t* dir_out, int64_t* other_out, int64_t* relation_out);

/* Block until all work enqueued on the graph's streams is complete. */
int jg_graph_sync(jg_graph* g);

/* Process-wide performance knobs (no effect on results).  Every key, its default and the measurement
 * behind it is in `struct Tune` (janusgraph_amd/csrc/jg_internal.h); the ranges are checked here:
 *   0/1 switches (any other value: JG_ERR_ARG): "pull_split", "halo" (read at build; sharded graphs:
 *     0 = dense allgather), "bfs_narrow", "cc_push", "cc_uf", "cc_uf_sharded", "cc_uf_search",
 *     "cc_sparse", "msbfs_sparse", "msbfs_skip", "msbfs_split", "sharded_bfs";
 *   integers: "bfs_alpha", "dobfs_alpha", "bfs_beta", "nb_alpha" [1, 1e6]; "nb_first" [4, 4096];
 *     "msbfs_td" [0, 2]; "msbfs_exit" [0, 2]; "cc_first" [1, 64]; "msbfs_td_rowapply" [0, 1024];
 *     "msbfs_td_noprobe", "msbfs_exit_live" [0, 1000]; "msbfs_scan_queue" [0, 1001];
 *     "msbfs_exit_first" [1, 256]; "bfs_td_split" [0, 2]; "bfs_td_split_levels" [0, 0xffff];
 *     "bfs_td_split_min" / "_max" [1, 2^31); "bfs_batch0" [1, 64]; "bfs_grid_mult" [1, 64];
 *     "bfs_grid" [64, 65536]; "bfs_tail_grid" [0, 65536]; "merge_temporal" [0, 2];
 *     "sd_delta" [-1, 2^30]; "sd_dist32" [0, 2]; "merge_pack" 0 | 1 | 24; "merge_stage<i>" -1 | 0 | 64 | 128 | 256 | 512;
 *     read at build: "band<i>_deg" (>= -1), "band<i>_bit" (0 or [3, 8]), "band<i>_sub" (power of two <= 256);
 *   retired (their variants were measured slower and removed; accepted and ignored): "pull_unroll",
 *     "pull_nt", "pull_lds", "light_lds", "slice_lds", "pull_short", "pull_overlap", "bfs_persistent".
 * Unknown key or value out of range: JG_ERR_ARG. */
int jg_tune_set(const char* key, int64_t value);

#ifdef __cplusplus
}
#endif
#endif /* JANUSGPU_H */
