/*
 * jg_oracle.c — CPU restatement of FulgoraGraphComputer's effective semantics.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in janusgraph_amd/ links, loads or calls this file; only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as the checker / CPU
 * baseline.  It is a "port" (restatement) — the reference is Java and cannot be built here (no JDK,
 * no jars) — pinned by the known-answer tests of the reference's OLAPTest
 * (tests/golden/, tests/test_oracle_kats.py).
 *
 * Reference paths below are relative to /root/reference/.
 *   core/ = janusgraph-core/src/main/java/org/janusgraph/
 *   tu/   = janusgraph-backend-testutils/src/main/java/org/janusgraph/
 *
 * Model of a Fulgora run (core/graphdb/olap/computer/FulgoraGraphComputer.java:210-230):
 *   memory.iteration starts at 0; superstep t is executed, then terminate(memory) is asked with
 *   iteration == t; so supersteps 0..K run when terminate is "iteration >= K", and
 *   memory().getIteration() reports K afterwards (FulgoraMemory.java:97-101 complete()).
 *   Local messages are stored on the SENDER (VertexState.java:77-83) and pulled by the receiver
 *   over the reverse incident traversal (VertexMemoryHandler.java:121-142), from the previous
 *   superstep only (VertexState.java:135-138 completeIteration).
 *   Edges count only when both endpoints exist (VertexJobConverter.java:126-129 ghost skip), so
 *   callers pass dense, ghost-free edge lists (jo_remap).
 *
 * Build: see oracle/Makefile (gcc -O2 -fopenmp -shared).  Single-source file, no dependencies.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define JO_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------------------------
 * Synthetic input: Graph500 Kronecker generator, counter-based so that a GPU
 * kernel can produce the identical edge list.  Per edge e and level l one splitmix64 hash gives
 * two 32-bit uniforms: ii = lo >= T_ab ; jj = hi >= (ii ? T_cnorm : T_anorm), as in the Graph500
 * octave reference (ab = A+B, c_norm = C/(1-(A+B)), a_norm = A/(A+B)).  Vertex labels are then
 * scrambled by a seeded bijection of [0, 2^scale).
 * ------------------------------------------------------------------------------------------ */
static inline uint64_t jo_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

typedef struct jo_rmat_params {
    uint64_t seedmix;
    uint32_t t_ab, t_anorm, t_cnorm;
    int32_t scale;
    uint64_t mask;
    uint64_t k1, c1, k2, c2, k3, c3;
    int32_t sh;
} jo_rmat_params;

JO_API void jo_rmat_params_init(int scale, uint64_t seed, jo_rmat_params* p) {
    const double A = 0.57, B = 0.19, C = 0.19;
    const double ab = A + B, c_norm = C / (1.0 - (A + B)), a_norm = A / (A + B);
    p->seedmix = jo_splitmix64(seed);
    p->t_ab = (uint32_t)(ab * 4294967296.0);
    p->t_anorm = (uint32_t)(a_norm * 4294967296.0);
    p->t_cnorm = (uint32_t)(c_norm * 4294967296.0);
    p->scale = scale;
    p->mask = (scale >= 64) ? ~0ull : ((1ull << scale) - 1ull);
    p->k1 = jo_splitmix64(seed ^ 0x1111111111111111ull) | 1ull;
    p->c1 = jo_splitmix64(seed ^ 0x2222222222222222ull);
    p->k2 = jo_splitmix64(seed ^ 0x3333333333333333ull) | 1ull;
    p->c2 = jo_splitmix64(seed ^ 0x4444444444444444ull);
    p->k3 = jo_splitmix64(seed ^ 0x5555555555555555ull) | 1ull;
    p->c3 = jo_splitmix64(seed ^ 0x6666666666666666ull);
    p->sh = scale > 1 ? (scale + 1) / 2 : 1;
}

static inline uint64_t jo_rmat_perm(const jo_rmat_params* p, uint64_t x) {
    x = (x * p->k1 + p->c1) & p->mask;
    x ^= x >> p->sh;
    x = (x * p->k2 + p->c2) & p->mask;
    x ^= x >> p->sh;
    x = (x * p->k3 + p->c3) & p->mask;
    return x;
}

/* Edges [e0, e0+count) of the RMAT(scale, seed) stream; ids are dense in [0, 2^scale). */
JO_API void jo_rmat_edges(int scale, uint64_t seed, int64_t e0, int64_t count, int64_t* src, int64_t* dst) {
    jo_rmat_params p;
    jo_rmat_params_init(scale, seed, &p);
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < count; ++k) {
        const uint64_t e = (uint64_t)(e0 + k);
        uint64_t i = 0, j = 0;
        for (int l = 0; l < scale; ++l) {
            const uint64_t h = jo_splitmix64(((e << 6) | (uint64_t)l) ^ p.seedmix);
            const uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
            const uint64_t ii = lo >= p.t_ab;
            const uint64_t jj = hi >= (ii ? p.t_cnorm : p.t_anorm);
            i |= ii << l;
            j |= jj << l;
        }
        src[k] = (int64_t)jo_rmat_perm(&p, i);
        dst[k] = (int64_t)jo_rmat_perm(&p, j);
    }
}

/* ------------------------------------------------------------------------------------------
 * Snapshot: vertex ids -> dense [0,n) in the caller's vid order; ghost edges (an endpoint not
 * in vid) dropped.  core/graphdb/olap/VertexJobConverter.java:122-151 (ghost skip),
 * core/graphdb/olap/computer/FulgoraVertexMemory.java:74-77 (canonical id map).
 * Returns the number of kept edges; out arrays hold dense ids of kept edges in input order,
 * keep_idx[k] = index of the kept edge in the input (nullable).
 * ------------------------------------------------------------------------------------------ */
typedef struct { int64_t id; int64_t pos; } jo_idpos;
static int jo_cmp_idpos(const void* a, const void* b) {
    const int64_t x = ((const jo_idpos*)a)->id, y = ((const jo_idpos*)b)->id;
    return (x > y) - (x < y);
}
static int64_t jo_lookup(const jo_idpos* t, int64_t n, int64_t id) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = lo + (hi - lo) / 2;
        if (t[mid].id < id) lo = mid + 1; else hi = mid;
    }
    return (lo < n && t[lo].id == id) ? t[lo].pos : -1;
}

JO_API int64_t jo_remap(const int64_t* vid, int64_t n, const int64_t* src, const int64_t* dst, int64_t m,
                        int32_t* dsrc, int32_t* ddst, int64_t* keep_idx) {
    jo_idpos* t = (jo_idpos*)malloc(sizeof(jo_idpos) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) { t[i].id = vid[i]; t[i].pos = i; }
    qsort(t, (size_t)n, sizeof(jo_idpos), jo_cmp_idpos);
    for (int64_t i = 1; i < n; ++i)
        if (t[i].id == t[i - 1].id) { free(t); return -1; } /* duplicate vertex id */
    int64_t k = 0;
    for (int64_t e = 0; e < m; ++e) {
        const int64_t a = jo_lookup(t, n, src[e]), b = jo_lookup(t, n, dst[e]);
        if (a < 0 || b < 0) continue;
        dsrc[k] = (int32_t)a; ddst[k] = (int32_t)b;
        if (keep_idx) keep_idx[k] = e;
        ++k;
    }
    free(t);
    return k;
}

/* ------------------------------------------------------------------------------------------
 * Adjacency: CSR over rows = key endpoint, entries = (other endpoint, edge index), sorted by other
 * endpoint then edge index — the column order of a single-label JanusGraph row (relation type +
 * direction prefix, then other vertex id, then relation id; EdgeSerializer.java:86-122), which is
 * the order Fulgora's reverse incident traversal returns messages in (VertexMemoryHandler:128-141).
 * ------------------------------------------------------------------------------------------ */
typedef struct { int64_t* ptr; int32_t* other; int64_t* eidx; } jo_csr;

static void jo_csr_build(int64_t n, int64_t m, const int32_t* key, const int32_t* other, jo_csr* c) {
    c->ptr = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    c->other = (int32_t*)malloc(sizeof(int32_t) * (size_t)(m > 0 ? m : 1));
    c->eidx = (int64_t*)malloc(sizeof(int64_t) * (size_t)(m > 0 ? m : 1));
    /* counting sort by `other` (stable in edge index), then by `key` (stable) */
    int64_t* cnt = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    int64_t* tmp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(m > 0 ? m : 1));
    for (int64_t e = 0; e < m; ++e) cnt[other[e] + 1]++;
    for (int64_t v = 0; v < n; ++v) cnt[v + 1] += cnt[v];
    for (int64_t e = 0; e < m; ++e) tmp[cnt[other[e]]++] = e;
    for (int64_t e = 0; e < m; ++e) c->ptr[key[e] + 1]++;
    for (int64_t v = 0; v < n; ++v) c->ptr[v + 1] += c->ptr[v];
    int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    memcpy(fill, c->ptr, sizeof(int64_t) * (size_t)n);
    for (int64_t k = 0; k < m; ++k) {
        const int64_t e = tmp[k];
        const int64_t pos = fill[key[e]]++;
        c->other[pos] = other[e];
        c->eidx[pos] = e;
    }
    free(cnt); free(tmp); free(fill);
}
static void jo_csr_free(jo_csr* c) { free(c->ptr); free(c->other); free(c->eidx); }

/* BOTH adjacency of v = its OUT entries then its IN entries (a self-loop is seen twice: once as
 * OUT, once as IN — StandardJanusGraph.java:617-640 stores both entries on the row). */
static void jo_csr_build_both(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, jo_csr* c) {
    int32_t* k2 = (int32_t*)malloc(sizeof(int32_t) * (size_t)(2 * m > 0 ? 2 * m : 1));
    int32_t* o2 = (int32_t*)malloc(sizeof(int32_t) * (size_t)(2 * m > 0 ? 2 * m : 1));
    for (int64_t e = 0; e < m; ++e) { k2[e] = src[e]; o2[e] = dst[e]; k2[m + e] = dst[e]; o2[m + e] = src[e]; }
    jo_csr_build(n, 2 * m, k2, o2, c);
    free(k2); free(o2);
}

/* ------------------------------------------------------------------------------------------
 * JanusGraph PageRankVertexProgram (tu/olap/PageRankVertexProgram.java:89-110):
 *   superstep 0: every vertex sends 1.0 on scope inE                                     (:90-91)
 *   superstep 1: edgeCount = sum of messages pulled over its OUT edges (reverse of inE);
 *                rank = 1/vertexCount; send rank/edgeCount on scope outE                 (:92-97)
 *   superstep t>=2: rank = d * (sum pulled over IN edges) + (1-d)/vertexCount;
 *                send rank/edgeCount                                                       (:99-103)
 *   terminate when iteration >= maxIterations                                             (:107-110)
 * receiveMessages() concatenates all previous scopes (VertexMemoryHandler.java:144-151); the scope
 * nobody sent on contributes nothing.  Sums are left folds from 0.0 in adjacency order.
 * rank/edge_count are NaN where the property is never written (K == 0).
 * ------------------------------------------------------------------------------------------ */
JO_API void jo_pagerank(int64_t n, int64_t m, const int32_t* src, const int32_t* dst,
                        double damping, int64_t vertex_count, int iterations,
                        double* rank, double* edge_count) {
    for (int64_t v = 0; v < n; ++v) { rank[v] = NAN; edge_count[v] = NAN; }
    if (iterations <= 0) return; /* only superstep 0 runs: no property is written */
    jo_csr out, in;
    jo_csr_build(n, m, src, dst, &out); /* rows = source, entries = target */
    jo_csr_build(n, m, dst, src, &in);  /* rows = target, entries = source */
    double* msg_in = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));  /* scope inE  */
    double* msg_out = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1)); /* scope outE */
    double* msg_next = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    for (int64_t v = 0; v < n; ++v) msg_in[v] = 1.0; /* superstep 0 */
    const double initial = 1.0 / (double)vertex_count;
    /* superstep 1 */
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t v = 0; v < n; ++v) {
        double s = 0.0;
        for (int64_t k = out.ptr[v]; k < out.ptr[v + 1]; ++k) s = s + msg_in[out.other[k]];
        edge_count[v] = s;
        rank[v] = initial;
        msg_out[v] = initial / s;
    }
    const double teleport = (1.0 - damping) / (double)vertex_count;
    for (int t = 2; t <= iterations; ++t) {
#pragma omp parallel for schedule(dynamic, 4096)
        for (int64_t v = 0; v < n; ++v) {
            double s = 0.0;
            for (int64_t k = in.ptr[v]; k < in.ptr[v + 1]; ++k) s = s + msg_out[in.other[k]];
            volatile double scaled = damping * s; /* no FMA contraction: Java evaluates d*s then + */
            const double r = scaled + teleport;
            rank[v] = r;
            msg_next[v] = r / edge_count[v];
        }
        double* tmp = msg_out; msg_out = msg_next; msg_next = tmp;
    }
    free(msg_in); free(msg_out); free(msg_next);
    jo_csr_free(&out); jo_csr_free(&in);
}

/* One power superstep over an in-CSR given directly (used by bench.py's bounded CPU baseline
 * on the same RMAT graph: contrib_in -> contrib_out, rank_out). */
JO_API void jo_pagerank_superstep_csr(int64_t n, const int64_t* in_ptr, const int32_t* in_src,
                                      const double* contrib_in, const double* edge_count,
                                      double damping, int64_t vertex_count,
                                      double* contrib_out, double* rank_out) {
    const double teleport = (1.0 - damping) / (double)vertex_count;
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t v = 0; v < n; ++v) {
        double s = 0.0;
        for (int64_t k = in_ptr[v]; k < in_ptr[v + 1]; ++k) s = s + contrib_in[in_src[k]];
        volatile double scaled = damping * s;
        const double r = scaled + teleport;
        if (rank_out) rank_out[v] = r;
        contrib_out[v] = r / edge_count[v];
    }
}

/* Plain in-CSR builder exported for the baseline: rows = dst, entries = src (sorted). */
JO_API void jo_build_in_csr(int64_t n, int64_t m, const int32_t* src, const int32_t* dst,
                            int64_t* ptr_out, int32_t* src_out) {
    jo_csr in;
    jo_csr_build(n, m, dst, src, &in);
    memcpy(ptr_out, in.ptr, sizeof(int64_t) * (size_t)(n + 1));
    memcpy(src_out, in.other, sizeof(int32_t) * (size_t)m);
    jo_csr_free(&in);
}

/* ------------------------------------------------------------------------------------------
 * ShortestDistanceVertexProgram (tu/olap/ShortestDistanceVertexProgram.java:112-146):
 *   superstep 0: the seed sets DISTANCE = 0 and sends 0 on scope inE with edge function
 *                msg + edge.distance (:69, :115-121)
 *   superstep t: v pulls over its OUT edges (reverse of inE) the messages its targets sent in
 *                t-1, each + weight; min-combined (ShortestDistanceMessageCombiner.java:29-31);
 *                if DISTANCE absent or larger: set it and send (:123-140)
 *   terminate at iteration >= maxDepth (:144-146)
 * weight == NULL means weight 1 on every edge.  dist[v] = INT64_MIN where DISTANCE stays absent (any
 * long is a valid distance: weights may be negative).  weight[e] == INT32_MIN marks an edge without
 * the weight property: Fulgora's edge function (:69, edge.<Integer>value(weightProperty)) throws
 * when a message crosses it, so the run returns -1 if one does (0 otherwise).
 * ------------------------------------------------------------------------------------------ */
JO_API int jo_shortest_distance(int64_t n, int64_t m, const int32_t* src, const int32_t* dst,
                                const int32_t* weight, int64_t seed, int max_depth, int64_t* dist) {
    for (int64_t v = 0; v < n; ++v) dist[v] = INT64_MIN;
    if (seed < 0 || seed >= n) return 0;
    jo_csr out;
    jo_csr_build(n, m, src, dst, &out);
    const int64_t NONE = INT64_MIN; /* absent message / absent DISTANCE */
    for (int64_t v = 0; v < n; ++v) dist[v] = NONE;
    int64_t* msg = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
    int64_t* msg_next = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
    for (int64_t v = 0; v < n; ++v) msg[v] = NONE;
    dist[seed] = 0;
    msg[seed] = 0;
    int missing = 0;
    for (int t = 1; t <= max_depth; ++t) {
        int any = 0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(| : any, missing)
        for (int64_t v = 0; v < n; ++v) {
            int64_t best = NONE;
            for (int64_t k = out.ptr[v]; k < out.ptr[v + 1]; ++k) {
                const int64_t mw = msg[out.other[k]];
                if (mw == NONE) continue;
                if (weight && weight[out.eidx[k]] == INT32_MIN) { missing = 1; continue; }
                const int64_t cand = mw + (weight ? (int64_t)weight[out.eidx[k]] : 1);
                if (best == NONE || cand < best) best = cand;
            }
            msg_next[v] = NONE;
            if (best != NONE && (dist[v] == NONE || dist[v] > best)) {
                dist[v] = best;
                msg_next[v] = best;
                any = 1;
            }
        }
        int64_t* tmp = msg; msg = msg_next; msg_next = tmp;
        if (!any) break; /* nothing sent: later supersteps change nothing */
    }
    free(msg); free(msg_next);
    jo_csr_free(&out);
    return missing ? -1 : 0;
}

/* ------------------------------------------------------------------------------------------
 * Hop depth (BFS) from one source along `direction` (1 = OUT, 2 = IN, 3 = BOTH), at most
 * max_depth hops (< 0: unbounded).  With direction BOTH this is the depth semantics of TinkerPop's
 * ShortestPathVertexProgram under Fulgora's forced {Local(bothE), Global} scopes
 * (core/graphdb/olap/computer/FulgoraGraphComputer.java:249-253); SURVEY.md Appendix A.4.
 * ------------------------------------------------------------------------------------------ */
JO_API void jo_bfs(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, int direction,
                   int64_t source, int max_depth, int32_t* depth) {
    for (int64_t v = 0; v < n; ++v) depth[v] = -1;
    if (source < 0 || source >= n) return;
    jo_csr c;
    if (direction == 1) jo_csr_build(n, m, src, dst, &c);
    else if (direction == 2) jo_csr_build(n, m, dst, src, &c);
    else jo_csr_build_both(n, m, src, dst, &c);
    int32_t* q = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
    int64_t head = 0, tail = 0;
    depth[source] = 0;
    q[tail++] = (int32_t)source;
    while (head < tail) {
        const int32_t u = q[head++];
        if (max_depth >= 0 && depth[u] >= max_depth) continue;
        for (int64_t k = c.ptr[u]; k < c.ptr[u + 1]; ++k) {
            const int32_t v = c.other[k];
            if (depth[v] < 0) { depth[v] = depth[u] + 1; q[tail++] = v; }
        }
    }
    free(q);
    jo_csr_free(&c);
}

/* ------------------------------------------------------------------------------------------
 * String order of vertex ids: ConnectedComponentVertexProgram labels are id().toString() and are
 * compared with String.compareTo (TinkerPop 3.4.6, SURVEY.md A.3 [TP-recall]; label form pinned by
 * tu/olap/OLAPTest.java:752-755).  jo_lex_rank gives every vertex its rank in that order.
 * ------------------------------------------------------------------------------------------ */
typedef struct { char s[24]; int64_t pos; } jo_strpos;
static int jo_cmp_strpos(const void* a, const void* b) {
    const int c = strcmp(((const jo_strpos*)a)->s, ((const jo_strpos*)b)->s);
    if (c) return c;
    const int64_t x = ((const jo_strpos*)a)->pos, y = ((const jo_strpos*)b)->pos;
    return (x > y) - (x < y);
}
JO_API void jo_lex_rank(const int64_t* vid, int64_t n, int32_t* rank) {
    jo_strpos* t = (jo_strpos*)malloc(sizeof(jo_strpos) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) { snprintf(t[i].s, sizeof t[i].s, "%lld", (long long)vid[i]); t[i].pos = i; }
    qsort(t, (size_t)n, sizeof(jo_strpos), jo_cmp_strpos);
    for (int64_t r = 0; r < n; ++r) rank[t[r].pos] = (int32_t)r;
    free(t);
}

/* ------------------------------------------------------------------------------------------
 * ConnectedComponentVertexProgram, synchronous restatement [TP-recall, SURVEY.md A.3]:
 *   superstep 0: component = id().toString(); a vertex with any BOTH edge sends it and votes
 *                not-to-halt
 *   superstep t: take the String-min of received messages (pulled over BOTH edges from the
 *                neighbours that sent in t-1); if smaller than the current component: set + send
 *   terminate when nobody sent in the superstep just run, or iteration >= maxIterations-1
 *   (maxIterations = 100).
 * Labels are carried as lex ranks (bijective with the strings).  Returns memory().getIteration().
 * ------------------------------------------------------------------------------------------ */
/* The superstep loop of the restatement above over a BOTH adjacency given as CSR (rows = vertices,
 * entries = neighbours, any order inside a row: the String-min fold does not depend on it) and the
 * lex rank of every vertex.  label[v] = the rank of v's component label.  Returns getIteration(). */
JO_API int jo_cc_csr(int64_t n, const int64_t* ptr, const int32_t* other, const int32_t* rank,
                     int max_iterations, int32_t* label) {
    int32_t* label_prev = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    unsigned char* sent = (unsigned char*)malloc((size_t)(n > 0 ? n : 1));
    unsigned char* sent_next = (unsigned char*)malloc((size_t)(n > 0 ? n : 1));
    int any = 0;
#pragma omp parallel for schedule(static) reduction(| : any)
    for (int64_t v = 0; v < n; ++v) {
        label[v] = rank[v];
        sent[v] = ptr[v + 1] > ptr[v];
        any |= sent[v];
    }
    int iteration = 0;
    /* terminate(iteration 0): halts iff nobody voted false */
    while (any && iteration < max_iterations - 1) {
        ++iteration;
        memcpy(label_prev, label, sizeof(int32_t) * (size_t)n);
        any = 0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(| : any)
        for (int64_t v = 0; v < n; ++v) {
            int32_t cur = label_prev[v];
            int diff = 0;
            for (int64_t k = ptr[v]; k < ptr[v + 1]; ++k) {
                const int32_t u = other[k];
                if (sent[u] && label_prev[u] < cur) { cur = label_prev[u]; diff = 1; }
            }
            sent_next[v] = (unsigned char)diff;
            if (diff) { label[v] = cur; any = 1; }
        }
        unsigned char* t = sent; sent = sent_next; sent_next = t;
    }
    free(label_prev); free(sent); free(sent_next);
    return iteration;
}

JO_API int jo_connected_components(int64_t n, int64_t m, const int32_t* src, const int32_t* dst,
                                   const int64_t* vid, int max_iterations, int64_t* comp_vid) {
    int32_t* rank = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    int64_t* vid_of_rank = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    jo_lex_rank(vid, n, rank);
    for (int64_t v = 0; v < n; ++v) vid_of_rank[rank[v]] = vid[v];
    jo_csr c;
    jo_csr_build_both(n, m, src, dst, &c);
    int32_t* label = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    const int iteration = jo_cc_csr(n, c.ptr, c.other, rank, max_iterations, label);
    for (int64_t v = 0; v < n; ++v) comp_vid[v] = vid_of_rank[label[v]];
    free(rank); free(vid_of_rank); free(label);
    jo_csr_free(&c);
    return iteration;
}

/* ------------------------------------------------------------------------------------------
 * Full-size checkers (BASELINE.json configs at RMAT scale 20-26; tests/test_gpu_configs.py).
 * The restatements above build ordered CSRs serially, which is minutes at 2^26 vertices; these
 * build the same adjacency in parallel and run the same semantics on it.
 * ------------------------------------------------------------------------------------------ */

/* CSR with rows = key[e], entries = other[e] (both = 1: also rows = other, entries = key, so a
 * self-loop appears twice, as jo_csr_build_both).  Entry order inside a row is unspecified (atomic
 * fill): use only where the result does not depend on it (BFS depth, CC labels) or where it
 * changes rounding only (PageRank sums, far below the 1e-9 bar).  ptr[n+1], out[m or 2m]. */
JO_API void jo_csr_unordered(int64_t n, int64_t m, const int32_t* key, const int32_t* other, int both,
                             int64_t* ptr, int32_t* out) {
    int64_t* fill = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
#pragma omp parallel for schedule(static)
    for (int64_t e = 0; e < m; ++e) {
        __atomic_fetch_add(&fill[key[e]], 1, __ATOMIC_RELAXED);
        if (both) __atomic_fetch_add(&fill[other[e]], 1, __ATOMIC_RELAXED);
    }
    ptr[0] = 0;
    for (int64_t v = 0; v < n; ++v) ptr[v + 1] = ptr[v] + fill[v];
#pragma omp parallel for schedule(static)
    for (int64_t v = 0; v < n; ++v) fill[v] = ptr[v];
#pragma omp parallel for schedule(static)
    for (int64_t e = 0; e < m; ++e) {
        out[__atomic_fetch_add(&fill[key[e]], 1, __ATOMIC_RELAXED)] = other[e];
        if (both) out[__atomic_fetch_add(&fill[other[e]], 1, __ATOMIC_RELAXED)] = key[e];
    }
    free(fill);
}

/* Hop depth from `source` over a CSR (jo_bfs semantics: -1 unreached or beyond max_depth, max_depth
 * < 0 unbounded), level-synchronous and parallel: the depth of a vertex is the level it is first
 * reached at, whatever thread claims it, so the result is deterministic. */
JO_API void jo_bfs_csr(int64_t n, const int64_t* ptr, const int32_t* other, int64_t source, int max_depth,
                       int32_t* depth) {
#pragma omp parallel for schedule(static)
    for (int64_t v = 0; v < n; ++v) depth[v] = -1;
    if (source < 0 || source >= n) return;
    int32_t* q = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
    int32_t* qn = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
    int64_t len = 1, len_next = 0;
    q[0] = (int32_t)source;
    depth[source] = 0;
    for (int32_t level = 0; len > 0 && (max_depth < 0 || level < max_depth); ++level) {
        len_next = 0;
#pragma omp parallel
        {
            int32_t buf[1024];
            int nb = 0;
#pragma omp for schedule(dynamic, 64)
            for (int64_t i = 0; i < len; ++i) {
                const int32_t u = q[i];
                for (int64_t k = ptr[u]; k < ptr[u + 1]; ++k) {
                    const int32_t v = other[k];
                    int32_t expect = -1;
                    if (__atomic_load_n(&depth[v], __ATOMIC_RELAXED) == -1 &&
                        __atomic_compare_exchange_n(&depth[v], &expect, level + 1, 0, __ATOMIC_RELAXED,
                                                    __ATOMIC_RELAXED)) {
                        buf[nb++] = v;
                        if (nb == 1024) {
                            const int64_t at = __atomic_fetch_add(&len_next, nb, __ATOMIC_RELAXED);
                            memcpy(qn + at, buf, sizeof(int32_t) * 1024);
                            nb = 0;
                        }
                    }
                }
            }
            if (nb) {
                const int64_t at = __atomic_fetch_add(&len_next, nb, __ATOMIC_RELAXED);
                memcpy(qn + at, buf, sizeof(int32_t) * (size_t)nb);
            }
        }
        int32_t* t = q; q = qn; qn = t;
        len = len_next;
    }
    free(q); free(qn);
}

/* Rank of every id 0..n-1 in String order (the lex rank of jo_lex_rank for vid = 0..n-1, in O(n)):
 * String order of decimal numbers is the preorder of the decimal trie ("0", "1", "10", "100", ...,
 * "101", ..., "11", ...). */
JO_API void jo_lex_rank_iota(int64_t n, int32_t* rank) {
    if (n <= 0) return;
    int32_t r = 0;
    rank[0] = r++;
    int64_t x = 1;
    while (r < n) {
        rank[x] = r++;
        if (x * 10 < n) { x *= 10; continue; }        /* first child */
        while (x % 10 == 9 || x + 1 >= n) x /= 10;    /* climb while no next sibling */
        ++x;                                          /* next sibling */
    }
}

/* Graph500-style validation of a BFS depth vector over the undirected edge list (src, dst):
 * bit 0: depth[source] != 0; bit 1: an edge with exactly one reached endpoint; bit 2: an edge whose
 * endpoint depths differ by more than one; bit 3: a reached vertex other than the source without a
 * neighbour one level up; bit 4 (comp != NULL): the reached set is not the source's component.
 * Returns the error bits (0 = valid); *edges_out = edges with a reached endpoint (Graph500 TEPS). */
JO_API int jo_bfs_validate(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, const int32_t* depth,
                           int64_t source, const int32_t* comp, int64_t* edges_out) {
    int err = 0;
    if (source < 0 || source >= n || depth[source] != 0) err |= 1;
    unsigned char* has_parent = (unsigned char*)calloc((size_t)(n > 0 ? n : 1), 1);
    int64_t edges = 0;
#pragma omp parallel for schedule(static) reduction(| : err) reduction(+ : edges)
    for (int64_t e = 0; e < m; ++e) {
        const int32_t du = depth[src[e]], dv = depth[dst[e]];
        if ((du >= 0) != (dv >= 0)) { err |= 2; continue; }
        if (du < 0) continue;
        ++edges;
        if (du - dv > 1 || dv - du > 1) err |= 4;
        if (du == dv - 1) __atomic_store_n(&has_parent[dst[e]], 1, __ATOMIC_RELAXED);
        if (dv == du - 1) __atomic_store_n(&has_parent[src[e]], 1, __ATOMIC_RELAXED);
    }
#pragma omp parallel for schedule(static) reduction(| : err)
    for (int64_t v = 0; v < n; ++v) {
        if (depth[v] > 0 && !has_parent[v]) err |= 8;
        if (comp && source >= 0 && source < n && ((depth[v] >= 0) != (comp[v] == comp[source]))) err |= 16;
    }
    free(has_parent);
    if (edges_out) *edges_out = edges;
    return err;
}

/* Hop depth from up to 64 sources at once (jo_bfs semantics per source), bit-parallel: bit k of
 * visited[v] / frontier[v] is source k.  A level either pushes from the frontier (few frontier
 * vertices: atomic OR into the neighbours' next words) or pulls over every unfinished vertex's
 * neighbours (OR of their frontier words); both give next[v] = the OR of the frontier words of v's
 * neighbours, so depth_out[k * n + v] is the level bit k first reaches v, whatever the order.
 * Duplicate sources each get their own row.  -1 = unreached or beyond max_depth (< 0: unbounded). */
JO_API void jo_msbfs_csr(int64_t n, const int64_t* ptr, const int32_t* other, const int64_t* sources, int nsrc,
                         int max_depth, int32_t* depth_out) {
    if (nsrc <= 0 || nsrc > 64) return;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)nsrc * n; ++i) depth_out[i] = -1;
    uint64_t* visited = (uint64_t*)calloc((size_t)(n > 0 ? n : 1), 8);
    uint64_t* front = (uint64_t*)calloc((size_t)(n > 0 ? n : 1), 8);
    uint64_t* next = (uint64_t*)calloc((size_t)(n > 0 ? n : 1), 8);
    const uint64_t all = nsrc == 64 ? ~0ull : ((1ull << nsrc) - 1ull);
    int64_t nfront = 0;
    for (int k = 0; k < nsrc; ++k) {
        const int64_t s = sources[k];
        if (s < 0 || s >= n) continue;
        if (!front[s]) ++nfront;
        front[s] |= 1ull << k;
        visited[s] |= 1ull << k;
        depth_out[(int64_t)k * n + s] = 0;
    }
    for (int32_t level = 0; nfront > 0 && (max_depth < 0 || level < max_depth); ++level) {
        if (nfront < n / 32) { /* push */
#pragma omp parallel for schedule(dynamic, 64)
            for (int64_t u = 0; u < n; ++u) {
                const uint64_t f = front[u];
                if (!f) continue;
                for (int64_t k = ptr[u]; k < ptr[u + 1]; ++k) {
                    const int32_t v = other[k];
                    const uint64_t add = f & ~visited[v];
                    if (add && (__atomic_load_n(&next[v], __ATOMIC_RELAXED) & add) != add)
                        __atomic_fetch_or(&next[v], add, __ATOMIC_RELAXED);
                }
            }
        } else { /* pull */
#pragma omp parallel for schedule(dynamic, 1024)
            for (int64_t v = 0; v < n; ++v) {
                if ((visited[v] & all) == all) continue;
                uint64_t acc = 0;
                for (int64_t k = ptr[v]; k < ptr[v + 1]; ++k) acc |= front[other[k]];
                next[v] = acc;
            }
        }
        nfront = 0;
#pragma omp parallel for schedule(static) reduction(+ : nfront)
        for (int64_t v = 0; v < n; ++v) {
            const uint64_t nw = next[v] & ~visited[v] & all;
            next[v] = 0;
            front[v] = nw;
            if (!nw) continue;
            visited[v] |= nw;
            ++nfront;
            for (uint64_t b = nw; b; b &= b - 1) depth_out[(int64_t)__builtin_ctzll(b) * n + v] = level + 1;
        }
    }
    free(visited); free(front); free(next);
}

/* JanusGraph PageRank (jo_pagerank's semantics) over CSRs built by jo_csr_unordered: out_ptr gives
 * the out-degree (edgeCount: one message per out-edge, a sum of 1.0s, exact), in_ptr/in_src the
 * gather.  Same superstep loop; only the summation order inside a row may differ (rounding). */
JO_API void jo_pagerank_csr(int64_t n, const int64_t* in_ptr, const int32_t* in_src, const double* edge_count,
                            double damping, int64_t vertex_count, int iterations, double* rank) {
    for (int64_t v = 0; v < n; ++v) rank[v] = NAN;
    if (iterations <= 0) return;
    double* msg = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    double* msg_next = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    const double initial = 1.0 / (double)vertex_count;
#pragma omp parallel for schedule(static)
    for (int64_t v = 0; v < n; ++v) { rank[v] = initial; msg[v] = initial / edge_count[v]; }
    for (int t = 2; t <= iterations; ++t) {
        jo_pagerank_superstep_csr(n, in_ptr, in_src, msg, edge_count, damping, vertex_count, msg_next, rank);
        double* tmp = msg; msg = msg_next; msg_next = tmp;
    }
    free(msg); free(msg_next);
}

JO_API int jo_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ------------------------------------------------------------------------------------------
 * Edgestore entry decode: one adjacency column of a vertex row, as
 * EdgeSerializer.parseRelation reads it (core/graphdb/database/EdgeSerializer.java:86-122).
 *   header: IDHandler.readRelationType (core/graphdb/database/idhandling/IDHandler.java:130-141) =
 *     VariableLong.readPositiveWithPrefix(in, 3) (idhandling/VariableLong.java:193-208): prefix bit 0 =
 *     relation type (0 property, 1 edge), prefix >> 1 == 0 = system type; value bit 0 = direction
 *     (0 OUT, 1 IN), value >> 1 = type count; type id = count << 6 | suffix (IDManager.getSchemaId,
 *     core/graphdb/idmanagement/IDManager.java:650-653; suffixes :269-294 and the property keys).
 *   edge, MULTI (unconstrained): [header][sort key][other backward][relation backward] | value, both
 *     read backward from the value position (readUnsignedBackward, VariableLong.java:276-294);
 *   edge, constrained, unique in this direction: | [other forward][relation forward] (readPositive,
 *     VariableLong.java:44-52,93-97);
 *   edge, constrained, not unique: [header][other backward] | [relation forward]
 *   (EdgeSerializer.writeRelation :264-279 is the writer of all three).
 * Multiplicity codes: 0 MULTI, 1 SIMPLE, 2 ONE2MANY (unique IN), 3 MANY2ONE (unique OUT), 4 ONE2ONE
 * (core/core/Multiplicity.java:35-90); edge labels absent from the table are MULTI.
 * dir_out: 0 OUT edge, 1 IN edge, 2 property entry, 3 system relation (ids not decoded: -1).
 * ------------------------------------------------------------------------------------------ */
static int64_t jo_read_unsigned(const uint8_t* b, int64_t* pos) {
    int64_t v = 0;
    int8_t c;
    do {
        c = (int8_t)b[(*pos)++];
        v = (v << 7) | (c & 0x7F);
    } while (c >= 0);
    return v;
}

static int64_t jo_read_unsigned_backward(const uint8_t* b, int64_t* pos) {
    int64_t v = 0;
    int n = 0;
    for (;;) {
        const int8_t c = (int8_t)b[--(*pos)];
        if (c < 0) {  /* first byte: stop marker, 3 length bits, 4 value bits */
            v |= (int64_t)(c & 0x0F) << (7 * n);
            break;
        }
        v |= (int64_t)c << (7 * n);
        ++n;
    }
    return v;
}

JO_API void jo_decode_edges(const uint8_t* bytes, const int64_t* off, const int32_t* vpos, int64_t n,
                            const int64_t* type_ids, const int8_t* type_mult, int32_t ntypes, int64_t* type_out,
                            int8_t* dir_out, int64_t* other_out, int64_t* rel_out) {
#pragma omp parallel for schedule(static)
    for (int64_t e = 0; e < n; ++e) {
        const uint8_t* b = bytes + off[e];
        /* readPositiveWithPrefix(in, 3) */
        int64_t pos = 0;
        const int first = b[pos++];
        const int64_t prefix = first >> 5;
        int64_t value = first & 0x0F;
        if ((first >> 4) & 1) {
            const int64_t p0 = pos;
            const int64_t rem = jo_read_unsigned(b, &pos);
            value = (value << (7 * (pos - p0))) + rem;
        }
        const int is_edge = (int)(prefix & 1), dirbit = (int)(value & 1), system = (prefix >> 1) == 0;
        const int64_t count = value >> 1;
        const int64_t suffix = is_edge ? (system ? 53 : 21) : (system ? 37 : 5);
        const int64_t type_id = (count << 6) | suffix;
        type_out[e] = type_id;
        if (!is_edge || system) {
            dir_out[e] = (int8_t)(is_edge ? 3 : 2);
            other_out[e] = -1;
            rel_out[e] = -1;
            continue;
        }
        dir_out[e] = (int8_t)dirbit;
        int mult = 0;
        for (int32_t t = 0; t < ntypes; ++t)
            if (type_ids[t] == type_id) { mult = type_mult[t]; break; }
        const int unique = dirbit ? (mult == 2 || mult == 4) : (mult == 3 || mult == 4);
        int64_t p = vpos[e];
        if (mult == 0) {
            rel_out[e] = jo_read_unsigned_backward(b, &p);
            other_out[e] = jo_read_unsigned_backward(b, &p);
        } else if (unique) {
            other_out[e] = jo_read_unsigned(b, &p);
            rel_out[e] = jo_read_unsigned(b, &p);
        } else {
            other_out[e] = jo_read_unsigned_backward(b, &p);
            p = vpos[e];
            rel_out[e] = jo_read_unsigned(b, &p);
        }
    }
}
