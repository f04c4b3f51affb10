// Work model of a bit-parallel direction-optimising BFS over k <= 64 sources (CPU, OpenMP), for the
// replicated-graph / partitioned-sources plan.  Counts, per level, the adjacency
// entries a top-down push examines (frontier rows with a top-down bit) and those a bottom-up pass with
// early exit examines (a row stops once it holds every needed bit).  Each source picks its own
// direction (Beamer's rule on its own frontier).  Not a checker: tools/narrow_sim.py drives it.
//   gcc -O3 -fopenmp -shared -fPIC -o tools/micro/libnarrow_sim.so tools/micro/narrow_sim.c
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned long long u64;

// ptr/adj: symmetric CSR, rows relabelled by degree (descending), each row's neighbours ascending (hubs
// first).  out[level*4 + 0..3] = td entries, bu entries, frontier rows, bu rows scanned.  Returns levels.
int narrow_sim(int64_t n, const int64_t* ptr, const int32_t* adj, const int64_t* src, int k, int alpha, int beta,
               int per_source, int64_t* out, int max_levels) {
    u64* vis = calloc((size_t)n, sizeof(u64));
    u64* F = calloc((size_t)n, sizeof(u64));
    u64* N = calloc((size_t)n, sizeof(u64));
    const u64 all = k == 64 ? ~0ull : ((1ull << k) - 1);
    for (int s = 0; s < k; ++s) {
        vis[src[s]] |= 1ull << s;
        F[src[s]] |= 1ull << s;
    }
    int64_t m = ptr[n];
    u64 bumode = 0;  // sources currently bottom-up
    int64_t explored[64] = {0};
    int level = 0;
    for (; level < max_levels; ++level) {
        int64_t nf[64] = {0}, mf[64] = {0};
        for (int64_t v = 0; v < n; ++v) {
            u64 w = F[v];
            while (w) {
                int s = __builtin_ctzll(w);
                w &= w - 1;
                nf[s]++;
                mf[s] += ptr[v + 1] - ptr[v];
            }
        }
        u64 live = 0;
        for (int s = 0; s < k; ++s)
            if (nf[s]) live |= 1ull << s;
        if (!live) break;
        // direction per source (or one direction for all: per_source 0 uses the sums)
        u64 tdm = 0, bum = 0;
        if (per_source) {
            for (int s = 0; s < k; ++s) {
                if (!(live >> s & 1)) continue;
                explored[s] += mf[s];
                const int64_t mu = m - explored[s];
                int bu = (bumode >> s) & 1;
                if (!bu && mf[s] * alpha > mu) bu = 1;
                else if (bu && nf[s] * beta < n) bu = 0;
                if (bu) bum |= 1ull << s; else tdm |= 1ull << s;
            }
        } else {
            int64_t NF = 0, MF = 0;
            for (int s = 0; s < k; ++s) { NF += nf[s]; MF += mf[s]; explored[s] += mf[s]; }
            int64_t mu = 0;
            for (int s = 0; s < k; ++s) mu += m - explored[s];
            int bu = bumode != 0;
            if (!bu && MF * alpha > mu) bu = 1;
            else if (bu && NF * beta < n * k) bu = 0;
            if (bu) bum = live; else tdm = live;
        }
        bumode = bum;
        memset(N, 0, (size_t)n * sizeof(u64));
        int64_t td_e = 0, bu_e = 0, bu_rows = 0, fr = 0;
        if (tdm) {
#pragma omp parallel for schedule(dynamic, 4096) reduction(+ : td_e)
            for (int64_t u = 0; u < n; ++u) {
                const u64 b = F[u] & tdm;
                if (!b) continue;
                td_e += ptr[u + 1] - ptr[u];
                for (int64_t e = ptr[u]; e < ptr[u + 1]; ++e) {
                    const int32_t v = adj[e];
                    const u64 g = b & ~vis[v];
                    if (g) __atomic_fetch_or(&N[v], g, __ATOMIC_RELAXED);
                }
            }
        }
        if (bum) {
#pragma omp parallel for schedule(dynamic, 4096) reduction(+ : bu_e, bu_rows)
            for (int64_t v = 0; v < n; ++v) {
                const u64 need = ~vis[v] & bum & live & all;
                if (!need || ptr[v + 1] == ptr[v]) continue;
                bu_rows++;
                u64 acc = 0;
                for (int64_t e = ptr[v]; e < ptr[v + 1]; ++e) {
                    bu_e++;
                    acc |= F[adj[e]] & need;
                    if (acc == need) break;
                }
                if (acc) __atomic_fetch_or(&N[v], acc, __ATOMIC_RELAXED);
            }
        }
#pragma omp parallel for reduction(+ : fr)
        for (int64_t v = 0; v < n; ++v) {
            const u64 nb = N[v] & ~vis[v];
            vis[v] |= nb;
            F[v] = nb;
            fr += nb != 0;
        }
        out[level * 4 + 0] = td_e;
        out[level * 4 + 1] = bu_e;
        out[level * 4 + 2] = fr;
        out[level * 4 + 3] = bu_rows;
    }
    free(vis);
    free(F);
    free(N);
    return level;
}
