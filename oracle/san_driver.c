/* Sanitizer driver for the CPU restatement (test infrastructure, like jg_oracle.c itself): runs the
 * OpenMP checkers next to the serial restatements they are pinned to, on small RMAT graphs, so that
 * `make -C oracle asan` (gcc, -fsanitize=address,undefined) and `make -C oracle tsan` (clang + libomp,
 * -fsanitize=thread) cover every parallel loop of jg_oracle.c (race detection: the
 * reference's VertexState mutators are `synchronized`, VertexState.java:77,85,135; the restatement's
 * parallel loops must be race-free for its results to be the reference's).
 * Exit status 0 = every cross-check agreed; the sanitizers report (and, with halt_on_error, exit non-zero)
 * on any memory error or data race.  tests/test_sanitizers.py builds and runs it. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void jo_rmat_edges(int scale, uint64_t seed, int64_t e0, int64_t count, int64_t* src, int64_t* dst);
void jo_pagerank(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, double damping, int64_t vertex_count,
                 int iterations, double* rank, double* edge_count);
void jo_build_in_csr(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, int64_t* ptr_out, int32_t* src_out);
void jo_pagerank_csr(int64_t n, const int64_t* in_ptr, const int32_t* in_src, const double* edge_count, double damping,
                     int64_t vertex_count, int iterations, double* rank);
void jo_pagerank_superstep_csr(int64_t n, const int64_t* in_ptr, const int32_t* in_src, const double* contrib_in,
                               const double* edge_count, double damping, int64_t vertex_count, double* contrib_out,
                               double* rank_out);
void jo_bfs(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, int direction, int64_t source,
            int max_depth, int32_t* depth);
void jo_csr_unordered(int64_t n, int64_t m, const int32_t* key, const int32_t* other, int both, int64_t* ptr,
                      int32_t* out);
void jo_bfs_csr(int64_t n, const int64_t* ptr, const int32_t* other, int64_t source, int max_depth, int32_t* depth);
void jo_msbfs_csr(int64_t n, const int64_t* ptr, const int32_t* other, const int64_t* sources, int nsrc,
                  int max_depth, int32_t* depth_out);
int jo_bfs_validate(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, const int32_t* depth,
                    int64_t source, const int32_t* comp, int64_t* edges_out);
void jo_lex_rank_iota(int64_t n, int32_t* rank);
int jo_cc_csr(int64_t n, const int64_t* ptr, const int32_t* other, const int32_t* rank, int max_iterations,
              int32_t* label);
int jo_connected_components(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, const int64_t* vid,
                            int max_iterations, int64_t* comp_vid);

static int fails = 0;
#define CHECK(cond, ...)                       \
    do {                                       \
        if (!(cond)) {                         \
            fprintf(stderr, "FAIL: " __VA_ARGS__); \
            fprintf(stderr, "\n");             \
            ++fails;                           \
        }                                      \
    } while (0)

static void run(int scale) {
    const int64_t n = (int64_t)1 << scale, m = (int64_t)16 << scale;
    int64_t* s64 = malloc(sizeof(int64_t) * m);
    int64_t* d64 = malloc(sizeof(int64_t) * m);
    jo_rmat_edges(scale, 0x5EEDull + (uint64_t)scale, 0, m, s64, d64);
    int32_t* s = malloc(sizeof(int32_t) * m);
    int32_t* d = malloc(sizeof(int32_t) * m);
    for (int64_t e = 0; e < m; ++e) {
        s[e] = (int32_t)s64[e];
        d[e] = (int32_t)d64[e];
    }
    free(s64);
    free(d64);

    /* PageRank: the edge-list superstep loop against the parallel CSR one */
    double* rank = malloc(sizeof(double) * n);
    double* ec = malloc(sizeof(double) * n);
    double* rank2 = malloc(sizeof(double) * n);
    jo_pagerank(n, m, s, d, 0.85, n, 10, rank, ec);
    int64_t* iptr = malloc(sizeof(int64_t) * (n + 1));
    int32_t* isrc = malloc(sizeof(int32_t) * m);
    jo_build_in_csr(n, m, s, d, iptr, isrc);
    jo_pagerank_csr(n, iptr, isrc, ec, 0.85, n, 10, rank2);
    double worst = 0;
    for (int64_t v = 0; v < n; ++v)
        if (!isnan(rank[v])) worst = fmax(worst, fabs(rank[v] - rank2[v]) / fmax(fabs(rank[v]), 1e-300));
    CHECK(worst <= 1e-12, "scale %d: PageRank CSR vs edge list rel err %g", scale, worst);
    double* c0 = malloc(sizeof(double) * n);
    double* c1 = malloc(sizeof(double) * n);
    for (int64_t v = 0; v < n; ++v) c0[v] = (1.0 / (double)n) / ec[v];
    jo_pagerank_superstep_csr(n, iptr, isrc, c0, ec, 0.85, n, c1, rank2);

    /* BFS: the parallel level-synchronous CSR BFS and the bit-parallel one against the serial BFS */
    int64_t* ptr = malloc(sizeof(int64_t) * (n + 1));
    int32_t* adj = malloc(sizeof(int32_t) * 2 * m);
    jo_csr_unordered(n, m, s, d, 1, ptr, adj);
    int64_t srcs[8];
    int k = 0;
    for (int64_t v = 0; v < n && k < 8; v += n / 9 + 1)
        if (ptr[v + 1] > ptr[v]) srcs[k++] = v;
    int32_t* want = malloc(sizeof(int32_t) * n);
    int32_t* got = malloc(sizeof(int32_t) * n);
    int32_t* planes = malloc(sizeof(int32_t) * n * 8);
    jo_msbfs_csr(n, ptr, adj, srcs, k, -1, planes);
    for (int i = 0; i < k; ++i) {
        jo_bfs(n, m, s, d, 3, srcs[i], -1, want);
        jo_bfs_csr(n, ptr, adj, srcs[i], -1, got);
        CHECK(memcmp(want, got, sizeof(int32_t) * n) == 0, "scale %d: jo_bfs_csr source %lld", scale, (long long)srcs[i]);
        CHECK(memcmp(want, planes + (int64_t)i * n, sizeof(int32_t) * n) == 0, "scale %d: jo_msbfs_csr row %d", scale, i);
        int64_t edges = 0;
        CHECK(jo_bfs_validate(n, m, s, d, got, srcs[i], NULL, &edges) == 0, "scale %d: Graph500 validation", scale);
    }

    /* CC: the parallel CSR superstep loop against the edge-list one (labels as ranks of iota ids) */
    int32_t* rk = malloc(sizeof(int32_t) * n);
    int32_t* label = malloc(sizeof(int32_t) * n);
    int64_t* vid = malloc(sizeof(int64_t) * n);
    int64_t* comp = malloc(sizeof(int64_t) * n);
    for (int64_t v = 0; v < n; ++v) vid[v] = v;
    jo_lex_rank_iota(n, rk);
    const int it1 = jo_cc_csr(n, ptr, adj, rk, 100, label);
    const int it2 = jo_connected_components(n, m, s, d, vid, 100, comp);
    CHECK(it1 == it2, "scale %d: CC iterations %d vs %d", scale, it1, it2);
    int64_t* vid_of_rank = malloc(sizeof(int64_t) * n);
    for (int64_t v = 0; v < n; ++v) vid_of_rank[rk[v]] = v;
    int64_t bad = 0;
    for (int64_t v = 0; v < n; ++v) bad += vid_of_rank[label[v]] != comp[v];
    CHECK(bad == 0, "scale %d: CC labels differ on %lld vertices", scale, (long long)bad);

    free(vid_of_rank);
    free(comp);
    free(vid);
    free(label);
    free(rk);
    free(planes);
    free(got);
    free(want);
    free(adj);
    free(ptr);
    free(c1);
    free(c0);
    free(isrc);
    free(iptr);
    free(rank2);
    free(ec);
    free(rank);
    free(d);
    free(s);
}

int main(int argc, char** argv) {
    const int lo = argc > 1 ? atoi(argv[1]) : 8, hi = argc > 2 ? atoi(argv[2]) : 12;
    for (int scale = lo; scale <= hi; ++scale) run(scale);
    printf("san_driver: scales %d..%d, %d failures\n", lo, hi, fails);
    return fails ? 1 : 0;
}
