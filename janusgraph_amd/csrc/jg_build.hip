// jg_build.hip — the CSR snapshot that replaces Fulgora's per-superstep edgestore scan.
//
// Reference semantics (paths under /root/reference/janusgraph-core/src/main/java/org/janusgraph/):
//   graphdb/olap/VertexJobConverter.java:122-151   ghost vertices never execute or send: an edge
//                                                  counts only if both endpoints exist
//   graphdb/olap/computer/FulgoraVertexMemory.java:74-77  canonical id per vertex
//   graphdb/database/StandardJanusGraph.java:617-640       a self-loop has an OUT and an IN entry on
//                                                  its row: once in OUT, once in IN, twice in BOTH
//   graphdb/olap/QueryContainer.java:42,133        100000-entry hard limit (reported, not applied)
//
// Pipeline per shard (device): degrees -> degree-sorted relabel (radix sort) -> padded global ids ->
// per-CSR key select (row<<cbits | col) -> stable radix sort -> row_ptr by boundary detection.
#include <algorithm>
#include <climits>

#include <cmath>

#include "jg_internal.h"
#include "jg_prim.h"

namespace jg {

namespace {

// ---------------- Graph500 Kronecker generator (bit-identical to oracle jo_rmat_edges) ----------------
struct RmatParams {
    uint64_t seedmix;
    uint32_t t_ab, t_anorm, t_cnorm;
    int32_t scale;
    uint64_t mask;
    uint64_t k1, c1, k2, c2, k3, c3;
    int32_t sh;
};

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

RmatParams rmat_params(int scale, uint64_t seed) {
    const double A = 0.57, B = 0.19, C = 0.19;
    const double ab = A + B, c_norm = C / (1.0 - (A + B)), a_norm = A / (A + B);
    RmatParams p;
    p.seedmix = splitmix64(seed);
    p.t_ab = (uint32_t)(ab * 4294967296.0);
    p.t_anorm = (uint32_t)(a_norm * 4294967296.0);
    p.t_cnorm = (uint32_t)(c_norm * 4294967296.0);
    p.scale = scale;
    p.mask = scale >= 64 ? ~0ull : ((1ull << scale) - 1ull);
    p.k1 = splitmix64(seed ^ 0x1111111111111111ull) | 1ull;
    p.c1 = splitmix64(seed ^ 0x2222222222222222ull);
    p.k2 = splitmix64(seed ^ 0x3333333333333333ull) | 1ull;
    p.c2 = splitmix64(seed ^ 0x4444444444444444ull);
    p.k3 = splitmix64(seed ^ 0x5555555555555555ull) | 1ull;
    p.c3 = splitmix64(seed ^ 0x6666666666666666ull);
    p.sh = scale > 1 ? (scale + 1) / 2 : 1;
    return p;
}

__device__ __forceinline__ uint64_t rmat_perm(const RmatParams& p, uint64_t x) {
    x = (x * p.k1 + p.c1) & p.mask;
    x ^= x >> p.sh;
    x = (x * p.k2 + p.c2) & p.mask;
    x ^= x >> p.sh;
    x = (x * p.k3 + p.c3) & p.mask;
    return x;
}

__global__ __launch_bounds__(kBlock) void rmat_kernel(RmatParams p, int64_t m, int32_t* __restrict__ src,
                                                      int32_t* __restrict__ dst) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        uint64_t i = 0, j = 0;
        for (int l = 0; l < p.scale; ++l) {
            const uint64_t h = splitmix64((((uint64_t)e << 6) | (uint64_t)l) ^ p.seedmix);
            const uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
            const uint64_t ii = lo >= p.t_ab;
            const uint64_t jj = hi >= (ii ? p.t_cnorm : p.t_anorm);
            i |= ii << l;
            j |= jj << l;
        }
        src[e] = (int32_t)rmat_perm(p, i);
        dst[e] = (int32_t)rmat_perm(p, j);
    }
}

// ---------------- id remap ----------------
// Caller vertex id -> dense index through an open-addressing hash table built on the device (16-byte
// slots: key, index), linear probing.  A lookup is one or two 16-byte loads wherever the ids come from;
// the sorted-key binary search it replaces took 24 dependent loads per endpoint (RMAT-24 from ids:
// 103 ms for 537 M endpoints).  INT64_MIN marks an empty slot; an id equal to it is rejected.
constexpr unsigned long long kIdEmpty = 0x8000000000000000ull;

__device__ __forceinline__ uint64_t id_hash(uint64_t x) {  // splitmix64 finaliser
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

__global__ void id_table_clear_kernel(IdSlot* __restrict__ t, int64_t slots) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < slots; i += (int64_t)gridDim.x * blockDim.x)
        t[i] = IdSlot{kIdEmpty, 0u, 0u};
}

// bad: bit 0 a duplicate id, bit 1 an id equal to the empty marker
__global__ void id_table_insert_kernel(const int64_t* __restrict__ vid, int64_t n, IdSlot* __restrict__ t,
                                       uint64_t mask, int32_t* __restrict__ bad) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long k = (unsigned long long)vid[i];
        if (k == kIdEmpty) {
            atomicOr(bad, 2);
            continue;
        }
        uint64_t h = id_hash(k) & mask;
        for (;;) {
            const unsigned long long prev = atomicCAS(&t[h].key, kIdEmpty, k);
            if (prev == kIdEmpty) {
                t[h].val = (uint32_t)i;  // read only by the lookup kernel, launched after this one
                break;
            }
            if (prev == k) {
                atomicOr(bad, 1);
                break;
            }
            h = (h + 1) & mask;
        }
    }
}

__device__ __forceinline__ int32_t id_lookup(const IdSlot* __restrict__ t, uint64_t mask, int64_t id) {
    const unsigned long long k = (unsigned long long)id;
    if (k == kIdEmpty) return -1;
    uint64_t h = id_hash(k) & mask;
    for (;;) {
        const IdSlot s = t[h];
        if (s.key == k) return (int32_t)s.val;
        if (s.key == kIdEmpty) return -1;  // not a caller vertex: a ghost endpoint
        h = (h + 1) & mask;
    }
}

// t == nullptr: the ids are dense indices (RMAT graphs), valid in [0, n)
__global__ void id_lookup_kernel(const IdSlot* __restrict__ t, uint64_t mask, int64_t n, const int64_t* __restrict__ q,
                                 int64_t k, const int32_t* __restrict__ padded, int64_t* __restrict__ out,
                                 int64_t* __restrict__ pout) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < k; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t d = t ? id_lookup(t, mask, q[i]) : (q[i] >= 0 && q[i] < n ? q[i] : -1);
        out[i] = d;
        if (pout) pout[i] = d >= 0 ? (int64_t)padded[d] : -1;
    }
}

__global__ void remap_kernel(const IdSlot* __restrict__ t, uint64_t mask, const int64_t* __restrict__ s,
                             const int64_t* __restrict__ d, int64_t m, int32_t* __restrict__ ds,
                             int32_t* __restrict__ dd) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = s[e], b = d[e];
        ds[e] = id_lookup(t, mask, a);
        dd[e] = id_lookup(t, mask, b);
    }
}

// ---------------- degrees & relabel ----------------
__global__ void degree_kernel(const int32_t* __restrict__ src, const int32_t* __restrict__ dst, int64_t m,
                              int32_t* __restrict__ indeg, int32_t* __restrict__ outdeg,
                              unsigned long long* __restrict__ counters /* kept, loops */) {
    unsigned long long kept = 0, loops = 0;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int32_t a = src[e], b = dst[e];
        if (a < 0 || b < 0) continue;
        atomicAdd(&outdeg[a], 1);
        atomicAdd(&indeg[b], 1);
        ++kept;
        loops += (a == b);
    }
    kept = wave_reduce_add(kept);
    loops = wave_reduce_add(loops);
    if (lane_id() == 0) {
        atomicAdd(&counters[0], kept);
        atomicAdd(&counters[1], loops);
    }
}

// key = (maxdeg - deg) << vbits | v  (ascending sort = degree descending, then id ascending)
__global__ void relabel_keys_kernel(const int32_t* __restrict__ indeg, const int32_t* __restrict__ outdeg, int64_t n,
                                    int mode, int64_t maxdeg, int vbits, uint64_t* __restrict__ keys) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        int64_t d = mode == 0 ? indeg[v] : mode == 1 ? (int64_t)indeg[v] + outdeg[v] : outdeg[v];
        keys[v] = ((uint64_t)(maxdeg - d) << vbits) | (uint64_t)v;
    }
}

// Tie-break of the degree relabel (tune relabel_ties): rank1[v] = position of v in the (degree, id)
// order; nbr_min[v] = smallest rank1 over v's pull neighbours (IN: sources of its in-edges; BOTH:
// both ends), so rows of equal degree that gather the same hot vertex become neighbours.
__global__ void rank_scatter_kernel(const uint64_t* __restrict__ sorted_keys, int64_t n, uint64_t vmask,
                                    int32_t* __restrict__ rank1) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
        rank1[sorted_keys[k] & vmask] = (int32_t)k;
}

__global__ void nbr_min_kernel(const int32_t* __restrict__ src, const int32_t* __restrict__ dst, int64_t m, int mode,
                               const int32_t* __restrict__ rank1, int32_t* __restrict__ nbr_min) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int32_t a = src[e], b = dst[e];
        if (a < 0 || b < 0) continue;
        // plain read first: the minimum only falls, so a value not below the current one is done
        // (hub rows otherwise serialise millions of atomics on one word)
        const int32_t ra = rank1[a];
        if (ra < __atomic_load_n(&nbr_min[b], __ATOMIC_RELAXED)) atomicMin(&nbr_min[b], ra);
        if (mode == 1) {
            const int32_t rb = rank1[b];
            if (rb < __atomic_load_n(&nbr_min[a], __ATOMIC_RELAXED)) atomicMin(&nbr_min[a], rb);
        }
    }
}

// pass 1 of the tie-break sort: key = nbr_min << vbits | v (vertices without neighbours last; nbr_min
// starts at 0x7F7F7F7F, above any rank).  `gather_deg` (PageRank's IN plan, tune relabel_dead_last):
// a vertex without pull neighbours (in-degree 0: all of them tie in degree) is ordered by its out-degree
// instead, descending: the rarely gathered sources among the in-degree-0 rows (~9% of the vertices,
// <1% of the gathers) sit together at the front of that class instead of spread over all of it
// (Ordering every tie by out-degree instead measured +0.9% / +0.6% at RMAT-24 / 26, round 4.)
__global__ void tie_keys_kernel(const int32_t* __restrict__ nbr_min, int64_t n, int vbits,
                                const int32_t* __restrict__ gather_deg, int64_t max_gather,
                                uint64_t* __restrict__ keys) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        int64_t t = nbr_min[v] >= n ? n : nbr_min[v];
        if (t == n && gather_deg) t = max_gather - (gather_deg[v] < max_gather ? gather_deg[v] : max_gather);
        keys[v] = ((uint64_t)t << vbits) | (uint64_t)v;
    }
}

// pass 2: key = (maxdeg - deg(v)) << 33 | dead << 32 | position in pass 1 (stable: ties keep the pass-1
// order).  dead (PageRank's IN plan, tune relabel_dead_last): v has no out-edge, so no row ever gathers
// its contribution; such rows go last in their degree class, and the gathered vector's lines hold live
// contributions only (RMAT: 20% of the in-degree > 0 rows)
__global__ void tie_deg_keys_kernel(const uint64_t* __restrict__ keys1, int64_t n, uint64_t vmask,
                                    const int32_t* __restrict__ indeg, const int32_t* __restrict__ outdeg, int mode,
                                    int64_t maxdeg, bool dead_last, uint64_t* __restrict__ keys2) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t v = (int64_t)(keys1[i] & vmask);
        const int64_t d = mode == 0 ? indeg[v] : mode == 1 ? (int64_t)indeg[v] + outdeg[v] : outdeg[v];
        const uint64_t dead = dead_last && outdeg[v] == 0 ? 1ull : 0ull;
        keys2[i] = ((uint64_t)(maxdeg - d) << 33) | (dead << 32) | (uint64_t)i;
    }
}

// back to (degree, v) keys in the final order, for padded_ids_kernel
__global__ void tie_final_kernel(const uint64_t* __restrict__ keys1, const uint64_t* __restrict__ keys2, int64_t n,
                                 uint64_t vmask, uint64_t* __restrict__ out) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
        out[k] = keys1[keys2[k] & 0xFFFFFFFFull] & vmask;
}

__global__ void stats_kernel(const int32_t* __restrict__ indeg, const int32_t* __restrict__ outdeg, int64_t n,
                             unsigned long long* __restrict__ out /* max_in, max_out, truncated */) {
    unsigned long long mi = 0, mo = 0, tr = 0;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long a = (unsigned)indeg[v], b = (unsigned)outdeg[v];
        mi = a > mi ? a : mi;
        mo = b > mo ? b : mo;
        tr += (a + b) > (unsigned long long)JG_FULGORA_HARD_QUERY_LIMIT;
    }
    atomicMax(&out[0], mi);
    atomicMax(&out[1], mo);
    tr = wave_reduce_add(tr);
    if (lane_id() == 0) atomicAdd(&out[2], tr);
}

// order[k] = dense vertex of degree rank k;  padded[v] = g(k) = (k % P) * S + k / P
__global__ void padded_ids_kernel(const uint64_t* __restrict__ sorted_keys, int64_t n, uint64_t vmask, int P,
                                  int64_t S, int32_t* __restrict__ order, int32_t* __restrict__ padded) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int32_t v = (int32_t)(sorted_keys[k] & vmask);
        order[k] = v;
        padded[v] = (int32_t)((k % P) * S + k / P);
    }
}

__global__ void local_outdeg_kernel(const int32_t* __restrict__ order, const int32_t* __restrict__ outdeg, int64_t n,
                                    int P, int r, int64_t rows, int32_t* __restrict__ out) {
    for (int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; l < rows; l += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = (int64_t)r + l * P;
        out[l] = k < n ? outdeg[order[k]] : 0;
    }
}

// ---------------- key select (stable) ----------------
// Emits, in edge order, the keys of the CSR entries owned by shard r.
//   which = 0: IN   row = dst, col = src
//           1: OUT  row = src, col = dst
//           2: BOTH both of the above (an edge contributes its OUT entry then its IN entry)
constexpr int kSelItems = 8;
constexpr int kSelTile = kBlock * kSelItems;

struct SelectArgs {
    const int32_t* src;
    const int32_t* dst;
    const int32_t* padded;
    int64_t m;
    int64_t S;
    int r;
    int which;
    int cbits;
    CompactMap cm;  // sharded pull adjacency with a halo plan: columns become compact ids
};

// The block's tile of kSelTile edges is staged through LDS with coalesced loads, so each thread's
// kSelItems consecutive edges (kept consecutive for the stable order) come from LDS instead of
// stride-kSelItems global loads.  Padded by one word per kSelItems against bank conflicts.
constexpr int kSelPad = kSelTile + kSelTile / kSelItems;
__device__ __forceinline__ int sel_slot(int i) { return i + i / kSelItems; }

__device__ __forceinline__ void stage_tile(const SelectArgs& a, int32_t* ts, int32_t* td) {
    const int64_t t0 = (int64_t)blockIdx.x * kSelTile;
#pragma unroll
    for (int u = 0; u < kSelItems; ++u) {
        const int i = threadIdx.x + u * kBlock;
        const int64_t e = t0 + i;
        ts[sel_slot(i)] = e < a.m ? a.src[e] : -1;
        td[sel_slot(i)] = e < a.m ? a.dst[e] : -1;
    }
    __syncthreads();
}

__device__ __forceinline__ int emit_count(const SelectArgs& a, int32_t s, int32_t d) {
    if (s < 0 || d < 0) return 0;
    const int32_t gs = a.padded[s], gd = a.padded[d];
    const bool own_d = (gd / a.S) == a.r, own_s = (gs / a.S) == a.r;
    if (a.which == 0) return own_d;
    if (a.which == 1) return own_s;
    return (int)own_s + (int)own_d;
}

__global__ __launch_bounds__(kBlock) void select_count_kernel(SelectArgs a, int64_t* __restrict__ block_counts) {
    __shared__ int64_t scratch[kBlock / kWave];
    __shared__ int32_t ts[kSelPad], td[kSelPad];
    stage_tile(a, ts, td);
    int64_t c = 0;
#pragma unroll
    for (int k = 0; k < kSelItems; ++k) {
        const int i = sel_slot(threadIdx.x * kSelItems + k);
        c += emit_count(a, ts[i], td[i]);
    }
    c = wave_reduce_add(c);
    if (lane_id() == 0) scratch[wave_id()] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t t = 0;
        for (int w = 0; w < kBlock / kWave; ++w) t += scratch[w];
        block_counts[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(kBlock) void select_write_kernel(SelectArgs a, const int64_t* __restrict__ block_off,
                                                              uint64_t* __restrict__ keys, uint32_t* __restrict__ eidx) {
    __shared__ int64_t scratch[kBlock / kWave];
    __shared__ int32_t ts[kSelPad], td[kSelPad];
    stage_tile(a, ts, td);
    const int64_t base = (int64_t)blockIdx.x * kSelTile + (int64_t)threadIdx.x * kSelItems;
    int64_t c = 0;
#pragma unroll
    for (int k = 0; k < kSelItems; ++k) {
        const int i = sel_slot(threadIdx.x * kSelItems + k);
        c += emit_count(a, ts[i], td[i]);
    }
    int64_t total;
    int64_t pos = block_exclusive_scan_add(c, scratch, &total) + block_off[blockIdx.x];
    for (int k = 0; k < kSelItems; ++k) {
        const int64_t e = base + k;
        if (e >= a.m) break;
        const int i = sel_slot(threadIdx.x * kSelItems + k);
        const int32_t s = ts[i], d = td[i];
        if (s < 0 || d < 0) continue;
        const int64_t gs = a.padded[s], gd = a.padded[d];
        const bool own_d = (gd / a.S) == a.r, own_s = (gs / a.S) == a.r;
        if ((a.which == 1 || a.which == 2) && own_s) {
            const int64_t c = a.cm.on() ? (int64_t)a.cm(gd) : gd;
            keys[pos] = ((uint64_t)(gs - (int64_t)a.r * a.S) << a.cbits) | (uint64_t)c;
            if (eidx) eidx[pos] = (uint32_t)e;
            ++pos;
        }
        if ((a.which == 0 || a.which == 2) && own_d) {
            const int64_t c = a.cm.on() ? (int64_t)a.cm(gs) : gs;
            keys[pos] = ((uint64_t)(gd - (int64_t)a.r * a.S) << a.cbits) | (uint64_t)c;
            if (eidx) eidx[pos] = (uint32_t)e;
            ++pos;
        }
    }
}

__global__ void fill_i64_kernel(int64_t* p, int64_t n, int64_t v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

// row_ptr[rr] = first entry of row rr; rows without entries get the next row's start.
__global__ void csr_from_sorted_kernel(const uint64_t* __restrict__ keys, int64_t nnz, int cbits, int rshift,
                                       int64_t* __restrict__ row_ptr, int32_t* __restrict__ col,
                                       const uint32_t* __restrict__ eidx, const int32_t* __restrict__ w_in,
                                       int32_t* __restrict__ w_out) {
    const uint64_t cmask = (1ull << cbits) - 1ull;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[i];
        const int64_t row = (int64_t)(k >> rshift);
        const int64_t prev = i > 0 ? (int64_t)(keys[i - 1] >> rshift) : -1;
        for (int64_t rr = prev + 1; rr <= row; ++rr) row_ptr[rr] = i;
        col[i] = (int32_t)(k & cmask);
        if (w_out) w_out[i] = w_in[eidx[i]];
    }
}

// ---------------- pull plans ----------------
__global__ void hub_flag_kernel(const int64_t* __restrict__ rp, int64_t rows, uint8_t* __restrict__ flag) {
    for (int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; l < rows; l += (int64_t)gridDim.x * blockDim.x)
        flag[l] = (rp[l + 1] - rp[l]) >= kHubDegree;
}

// degree thresholds of the lane classes 1..6 (class 7 takes the rest, class 8 the empty suffix)
__constant__ int64_t c_class_thr[kNumClasses] = {kHubDegree, 256, 128, 64, 32, 16, 8, 1, 0};
constexpr int64_t c_class_thr_host[kNumClasses] = {kHubDegree, 256, 128, 64, 32, 16, 8, 1, 0};

// first_below[c] = first row with degree < c_class_thr[c] (c = 1..6);
// first_below[kZeroClass] = 1 + last row with any entry (rows after it are all empty);
// band_below[i] = first row with degree < band_thr[i] (i < nbands).  Wave-reduced, one atomic per wave.
struct BandThresholds {
    int64_t thr[4];
    int n;
};
__global__ void class_bound_kernel(const int64_t* __restrict__ rp, int64_t rows,
                                   unsigned long long* __restrict__ first_below /* [kNumClasses] */,
                                   unsigned long long* __restrict__ last_nonempty, BandThresholds bt,
                                   unsigned long long* __restrict__ band_below /* [4] */) {
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < rows; base += (int64_t)gridDim.x * blockDim.x) {
        const int64_t l = base + threadIdx.x;
        const bool in = l < rows;
        const int64_t d = in ? rp[l + 1] - rp[l] : 0;
        const unsigned long long none = ~0ull;
#pragma unroll
        for (int c = 1; c < kNumClasses - 2; ++c) {
            const unsigned long long v = wave_reduce_min(in && d < c_class_thr[c] ? (unsigned long long)l : none);
            // a plain read first: once a low row has set the bound, later waves skip the atomic
            // (every wave's atomic on the same few words serialised at L2: 9 ms at RMAT-24)
            if (lane_id() == 0 && v != none && v < __atomic_load_n(&first_below[c], __ATOMIC_RELAXED))
                atomicMin(&first_below[c], v);
        }
        const unsigned long long ne = wave_reduce_max(in && d > 0 ? (unsigned long long)(l + 1) : 0ull);
        if (lane_id() == 0 && ne && ne > __atomic_load_n(last_nonempty, __ATOMIC_RELAXED)) atomicMax(last_nonempty, ne);
        for (int i = 0; i < bt.n; ++i) {
            const unsigned long long v = wave_reduce_min(in && d < bt.thr[i] ? (unsigned long long)l : none);
            if (lane_id() == 0 && v != none && v < __atomic_load_n(&band_below[i], __ATOMIC_RELAXED))
                atomicMin(&band_below[i], v);
        }
    }
}

// Degree runs of rows [lo, hi): st[0] = 1 if a row's degree is 0, above kRunMax or above its
// predecessor's; st[1 + d] = first row of degree d (d = 1..kRunMax), st[9 + d] = its row_ptr.
__global__ void degree_run_kernel(const int64_t* __restrict__ rp, int64_t lo, int64_t hi, int64_t* __restrict__ st) {
    for (int64_t l = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; l < hi; l += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = rp[l], d = rp[l + 1] - j;
        if (d < 1 || d > kRunMax) {
            st[0] = 1;
            continue;
        }
        const int64_t dp = l > lo ? j - rp[l - 1] : kRunMax + 1;
        if (d > dp) st[0] = 1;
        else if (d < dp) {  // a run starts here (one row per degree when the order holds)
            st[1 + d] = l;
            st[9 + d] = j;
        }
    }
}

__global__ void gather_row_bounds_kernel(const int64_t* __restrict__ rp, const int64_t* __restrict__ rows_idx,
                                         int64_t nh, int64_t* __restrict__ out /* [2*nh] */) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nh; i += (int64_t)gridDim.x * blockDim.x) {
        out[2 * i] = rp[rows_idx[i]];
        out[2 * i + 1] = rp[rows_idx[i] + 1];
    }
}

// ---------------- XCD split of the heavy rows ----------------
int64_t select_keys(const SelectArgs& a, DevBuf<uint64_t>& keys, DevBuf<uint32_t>& eidx, bool want_eidx,
                    hipStream_t s) {
    const int64_t nb = std::max<int64_t>(1, (a.m + kSelTile - 1) / kSelTile);
    DevBuf<int64_t> counts(nb), off(nb + 1);
    select_count_kernel<<<(unsigned)nb, kBlock, 0, s>>>(a, counts.get());
    JG_LAUNCH_CHECK();
    prim::exclusive_scan(counts.get(), off.get(), nb, s);
    int64_t total = 0;
    JG_HIP(hipMemcpyAsync(&total, off.get() + nb, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    JG_HIP(hipStreamSynchronize(s));
    keys.alloc(std::max<int64_t>(total, 1));
    if (want_eidx) eidx.alloc(std::max<int64_t>(total, 1));
    select_write_kernel<<<(unsigned)nb, kBlock, 0, s>>>(a, off.get(), keys.get(), want_eidx ? eidx.get() : nullptr);
    JG_LAUNCH_CHECK();
    return total;
}

}  // namespace

void generate_rmat_device(int scale, uint64_t seed, int64_t m, int32_t* src, int32_t* dst, hipStream_t s) {
    const RmatParams p = rmat_params(scale, seed);
    rmat_kernel<<<grid_for(m, kBlock, 256 * 32), kBlock, 0, s>>>(p, m, src, dst);
    JG_LAUNCH_CHECK();
}

__global__ void mask_ids_kernel(const int64_t* __restrict__ masked, const int32_t* __restrict__ dense, int64_t m,
                                int32_t* __restrict__ out) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x)
        out[e] = masked[e] < 0 ? -1 : dense[e];
}

void mask_ids_device(const int64_t* masked, const int32_t* dense, int64_t m, int32_t* out, hipStream_t s) {
    if (m <= 0) return;
    mask_ids_kernel<<<grid_for(m), kBlock, 0, s>>>(masked, dense, m, out);
    JG_LAUNCH_CHECK();
}

void remap_ids_device(const int64_t* d_vid, int64_t n, const int64_t* d_src, const int64_t* d_dst, int64_t m,
                      int32_t* dsrc, int32_t* ddst, hipStream_t s, DevBuf<IdSlot>* keep) {
    // a power of two >= 1.4 n slots (load <= 0.7; a miss probes ~6 slots, a hit ~2)
    int64_t slots = 1024;
    while (slots * 5 < 7 * n) slots *= 2;
    DevBuf<IdSlot> tmp;
    DevBuf<IdSlot>& table = keep ? *keep : tmp;
    if (table.size() != (size_t)slots) {
        table.alloc(slots);
        DevBuf<int32_t> bad(1);
        JG_HIP(hipMemsetAsync(bad.get(), 0, sizeof(int32_t), s));
        id_table_clear_kernel<<<grid_for(slots), kBlock, 0, s>>>(table.get(), slots);
        JG_LAUNCH_CHECK();
        if (n > 0) {
            id_table_insert_kernel<<<grid_for(n), kBlock, 0, s>>>(d_vid, n, table.get(), (uint64_t)(slots - 1), bad.get());
            JG_LAUNCH_CHECK();
        }
        int32_t has_bad = 0;
        JG_HIP(hipMemcpyAsync(&has_bad, bad.get(), sizeof(int32_t), hipMemcpyDeviceToHost, s));
        JG_HIP(hipStreamSynchronize(s));
        if (has_bad & 1) fail(JG_ERR_ARG, "duplicate vertex id in vid[]");
        if (has_bad & 2) fail(JG_ERR_ARG, "vertex id INT64_MIN is not supported");
    }
    if (m > 0) {
        remap_kernel<<<grid_for(m, kBlock, 256 * 64), kBlock, 0, s>>>(table.get(), (uint64_t)(slots - 1), d_src, d_dst, m,
                                                                     dsrc, ddst);
        JG_LAUNCH_CHECK();
    }
    JG_HIP(hipStreamSynchronize(s));
}

void dense_of_vids(const Graph& g, const int64_t* vids, int64_t k, int64_t* out, int64_t* padded) {
    if (k <= 0) return;
    if (g.id_table.size() == 0 && k <= 4096) {
        // no id table (vid == dense index): a few sources are looked up on the host, without the device
        // round trip (two synchronised copies and a launch: ~40 us of a 0.2 ms RMAT-20 BFS call)
        const std::vector<int32_t>* pad = padded ? &g.padded_of_dense() : nullptr;
        for (int64_t i = 0; i < k; ++i) {
            out[i] = vids[i] >= 0 && vids[i] < g.n ? vids[i] : -1;
            if (padded) padded[i] = out[i] >= 0 ? (int64_t)(*pad)[(size_t)out[i]] : -1;
        }
        return;
    }
    DeviceGuard dg(g.id_dev);
    hipStream_t s = g.shards[0]->stream;
    DevBuf<int64_t> q(k), r(k), pr(padded ? k : 0);
    copy_h2d(q.get(), vids, (size_t)k * sizeof(int64_t), s);
    const bool table = g.id_table.size() != 0;
    id_lookup_kernel<<<grid_for(k), kBlock, 0, s>>>(table ? g.id_table.get() : nullptr,
                                                   table ? (uint64_t)(g.id_table.size() - 1) : 0ull, g.n, q.get(), k,
                                                   g.padded_dev.get(), r.get(), padded ? pr.get() : nullptr);
    JG_LAUNCH_CHECK();
    copy_d2h(out, r.get(), (size_t)k * sizeof(int64_t), s);
    if (padded) copy_d2h(padded, pr.get(), (size_t)k * sizeof(int64_t), s);
}

static void build_csr(Shard& sh, const SelectArgs& a, const int32_t* weight, Csr& csr, hipStream_t s) {
    DevBuf<uint64_t> keys;
    DevBuf<uint32_t> eidx;
    const int64_t nnz = select_keys(a, keys, eidx, weight != nullptr, s);
    const int rbits = bits_for((uint64_t)std::max<int64_t>(sh.rows - 1, 0));
    if (rbits + a.cbits > 64) fail(JG_ERR_UNSUPPORTED, "CSR sort key exceeds 64 bits");
    prim::radix_sort(keys.get(), weight ? eidx.get() : nullptr, nnz, rbits + a.cbits, s);
    csr.rows = sh.rows;
    csr.nnz = nnz;
    csr.row_ptr.alloc(sh.rows + 1);
    csr.col.alloc(std::max<int64_t>(nnz, 1));
    if (weight) csr.weight.alloc(std::max<int64_t>(nnz, 1));
    fill_i64_kernel<<<grid_for(sh.rows + 1), kBlock, 0, s>>>(csr.row_ptr.get(), sh.rows + 1, nnz);
    JG_LAUNCH_CHECK();
    if (nnz > 0) {
        csr_from_sorted_kernel<<<grid_for(nnz), kBlock, 0, s>>>(keys.get(), nnz, a.cbits, a.cbits,
                                                                csr.row_ptr.get(),
                                                                csr.col.get(), weight ? eidx.get() : nullptr, weight,
                                                                weight ? csr.weight.get() : nullptr);
        JG_LAUNCH_CHECK();
    }
    JG_HIP(hipStreamSynchronize(s));
}

// ---------------- the sliced split (SliceBand) ----------------
// Sub-rows from the column-ordered CSR (round 3: the bands used to be cut from a second, sub-slice-
// ordered build of the whole CSR).  One wave per band row; a sub-row keeps its entries in the row's
// (column) order.  Wave-private LDS: the fences only keep the compiler from moving LDS accesses across
// the wave barrier (a wave executes its LDS instructions in order).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// len[h * NR + i] = entries of band row R0 + i in sub-slice h
__global__ __launch_bounds__(kBlock) void band_count_kernel(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                            int64_t R0, int64_t NR, int bits, int32_t* __restrict__ len) {
    __shared__ uint32_t cnt[kBlock / kWave][256];
    const int S = 1 << bits;
    const int wv = (int)(threadIdx.x / kWave), lane = (int)(threadIdx.x % kWave);
    const int64_t waves = (int64_t)gridDim.x * (kBlock / kWave);
    for (int64_t i = (int64_t)blockIdx.x * (kBlock / kWave) + wv; i < NR; i += waves) {
        for (int h = lane; h < S; h += kWave) cnt[wv][h] = 0u;
        wave_sync();
        const int64_t b = rp[R0 + i], e = rp[R0 + i + 1];
        for (int64_t j = b + lane; j < e; j += kWave) atomicAdd(&cnt[wv][sub_slice(col[j], bits)], 1u);
        wave_sync();
        for (int h = lane; h < S; h += kWave) len[(int64_t)h * NR + i] = (int32_t)cnt[wv][h];
        wave_sync();
    }
}

// band col[sp[h][i] + k] = the k-th entry (row order) of band row i in sub-slice h: per 64-entry chunk
// every lane finds the lanes of its sub-slice by `bits` ballots, takes its rank among them after the
// sub-row's running position, and the group's highest lane advances that position
__global__ __launch_bounds__(kBlock) void band_scatter_kernel(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                              int64_t R0, int64_t NR, int bits,
                                                              const int64_t* __restrict__ sp, int32_t* __restrict__ bcol) {
    __shared__ int64_t run[kBlock / kWave][256];
    const int S = 1 << bits;
    const int wv = (int)(threadIdx.x / kWave), lane = (int)(threadIdx.x % kWave);
    const int64_t waves = (int64_t)gridDim.x * (kBlock / kWave);
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (kWave - lane));  // lanes below this one
    for (int64_t i = (int64_t)blockIdx.x * (kBlock / kWave) + wv; i < NR; i += waves) {
        for (int h = lane; h < S; h += kWave) run[wv][h] = sp[(int64_t)h * (NR + 1) + i];
        wave_sync();
        const int64_t b = rp[R0 + i], e = rp[R0 + i + 1];
        for (int64_t j0 = b; j0 < e; j0 += kWave) {
            const int64_t j = j0 + lane;
            const bool valid = j < e;
            const int32_t c = valid ? col[j] : 0;
            const int h = valid ? sub_slice(c, bits) : 0;
            uint64_t mask = __ballot(valid);
            for (int t = 0; t < bits; ++t) {
                const uint64_t m = __ballot(valid && ((h >> t) & 1));
                mask &= ((h >> t) & 1) ? m : ~m;
            }
            const int64_t pos = run[wv][h] + (int64_t)__popcll(mask & lt);
            wave_sync();
            if (valid) {
                bcol[pos] = c;
                if ((mask >> lane) == 1ull) run[wv][h] += (int64_t)__popcll(mask);  // the group's highest lane
            }
            wave_sync();
        }
    }
}

// raw[h * NR] for h = 0..S (the sub-slice boundaries of the exclusive scan)
__global__ void band_bounds_kernel(const int64_t* __restrict__ raw, int64_t NR, int S, int64_t* __restrict__ out) {
    const int h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h <= S) out[h] = raw[(int64_t)h * NR];
}

// sp[h*(NR+1) + i] = raw[h*NR + i] - raw[h*NR] + begin[h], i in [0, NR] (raw[h*NR + NR] = its end)
__global__ void band_ptr_kernel(const int64_t* __restrict__ raw, int64_t NR, int S, const int64_t* __restrict__ begin,
                                int64_t* __restrict__ sp) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < (NR + 1) * S; x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t h = x / (NR + 1), i = x % (NR + 1);
        sp[x] = raw[h * NR + i] - raw[h * NR] + begin[h];
    }
}


__global__ void nonempty_kernel(const int32_t* __restrict__ len, int64_t n, int32_t* __restrict__ flag) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        flag[i] = len[i] > 0;
}

// Non-empty sub-rows are numbered sub-slice-major (num = exclusive scan of the flags): cstart[k] =
// first entry of sub-row k, srow[k] = its band row.
__global__ void sub_number_kernel(const int32_t* __restrict__ len, const int64_t* __restrict__ num, int64_t NR, int S,
                                  const int64_t* __restrict__ sp, int64_t* __restrict__ cstart,
                                  int32_t* __restrict__ srow) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < NR * S; x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t h = x / NR, i = x % NR;
        if (len[x] > 0) {
            cstart[num[x]] = sp[h * (NR + 1) + i];
            srow[num[x]] = (int32_t)i;
        }
    }
}

// sub_word[h][w] = (non-empty flags of band rows 32w .. 32w+31 in sub-slice h, number of the first of
// them) (SliceBand)
__global__ void sub_word_kernel(const int32_t* __restrict__ len, const int64_t* __restrict__ num, int64_t NR, int S,
                                int64_t W, uint2* __restrict__ word) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < W * S; x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t h = x / W, w = x % W, i0 = w * 32;
        uint32_t b = 0;
        for (int k = 0; k < 32 && i0 + k < NR; ++k) b |= (len[h * NR + i0 + k] > 0 ? 1u : 0u) << k;
        word[x] = make_uint2(b, (uint32_t)num[h * NR + i0]);
    }
}

// Per task: j0 = the non-empty sub-row holding its first entry, carry = it started earlier,
// heads[t][l] = row-start bits of lane l's kMergeEpl entries (bit 0 of lane 0 always set), and the
// band rows of its first and last sub-row.
__global__ void task_meta_kernel(const int64_t* __restrict__ cstart, const int32_t* __restrict__ srow,
                                 const int64_t* __restrict__ nzb, int S, const int64_t* __restrict__ begin,
                                 const int64_t* __restrict__ end, const int64_t* __restrict__ base,
                                 int32_t* __restrict__ meta, uint8_t* __restrict__ heads, int32_t* __restrict__ trows) {
    constexpr int kEpl = kMergeTask / kWave;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < base[S]; t += (int64_t)gridDim.x * blockDim.x) {
        int lo_h = 0, hi_h = S;  // sub-slice: last h with base[h] <= t
        while (hi_h - lo_h > 1) {
            const int mid = (lo_h + hi_h) >> 1;
            if (base[mid] <= t) lo_h = mid; else hi_h = mid;
        }
        const int h = lo_h;
        const int64_t e0 = begin[h] + (t - base[h]) * kMergeTask;
        const int64_t e1 = min(e0 + kMergeTask, end[h]);
        int64_t lo = nzb[h], hi = nzb[h + 1];  // first sub-row starting after e0
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (cstart[mid] <= e0) lo = mid + 1; else hi = mid;
        }
        const int64_t j0 = lo - 1;
        meta[2 * t] = (int32_t)j0;
        meta[2 * t + 1] = cstart[j0] < e0 ? 1 : 0;
        uint8_t hd[kWave];
        for (int l = 0; l < kWave; ++l) hd[l] = 0;
        hd[0] = 1;
        int64_t j = j0 + 1;
        for (; j < nzb[h + 1] && cstart[j] < e1; ++j) {
            const int pos = (int)(cstart[j] - e0);
            hd[pos / kEpl] |= (uint8_t)(1u << (pos % kEpl));
        }
        for (int l = 0; l < kWave; ++l) heads[t * kWave + l] = hd[l];
        trows[2 * t] = srow[j0];
        trows[2 * t + 1] = srow[j - 1];
    }
}

// Lane chunk x of a band (entries [8x, 8x + 8) of its col): sub-slice-local indices packed in W bits
// each, bit stream over W / 4 dwords, dwords 0..3 to pa[x], the rest to pb (SliceBand::pack_a/_b).
template <int W>
__global__ void band_pack_kernel(const int32_t* __restrict__ col, int64_t chunks, int gshift, uint4* __restrict__ pa,
                                 uint32_t* __restrict__ pb) {
    constexpr int D = W / 4, DB = D - 4;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < chunks; x += (int64_t)gridDim.x * blockDim.x) {
        uint32_t d[D];
#pragma unroll
        for (int i = 0; i < D; ++i) d[i] = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t c = (uint32_t)col[8 * x + u];
            const uint64_t loc = (uint64_t)(((c >> gshift) << 4) | (c & 15u));
            const int o = W * u, i = o >> 5, sh = o & 31;
            d[i] |= (uint32_t)(loc << sh);
            if (sh + W > 32) d[i + 1] |= (uint32_t)(loc >> (32 - sh));
        }
        pa[x] = make_uint4(d[0], d[1], d[2], d[3]);
#pragma unroll
        for (int i = 0; i < DB; ++i) pb[x * DB + i] = d[4 + i];
    }
}

// Bits of the largest sub-slice-local index of a vector of col_space entries in 2^bits sub-slices:
// the packed width 20, 24 or 32 (Tune::merge_pack = 0: always 32, 24: at least 24).
static int band_width(int64_t col_space, int bits) {
    const uint64_t cmax = (uint64_t)std::max<int64_t>(col_space - 1, 0);
    const uint64_t loc = ((cmax >> (4 + bits)) << 4) | 15u;
    int need = 1;
    while (need < 64 && (loc >> need) != 0) ++need;
    if (!tune().merge_pack) return 32;
    if (tune().merge_pack == 24) need = std::max(need, 21);  // test knob: at least 24 bits
    return need <= 20 ? 20 : need <= 24 ? 24 : 32;
}

// One band: sub-slice-major sub-CSRs of rows [R0, R1), every sub-slice's start aligned to a merge
// task (a task never spans two sub-slices and its col loads are 16-byte aligned).
static void build_band(Shard& sh, const Csr& csr, SliceBand& bd, int64_t col_space) {
    hipStream_t s = sh.stream;
    const int64_t R0 = bd.row_begin, NR = bd.rows();
    const int S = 1 << bd.bits;
    const int64_t NS = NR * S;
    DevBuf<int32_t> len(NS);
    DevBuf<int64_t> raw(NS + 1);
    band_count_kernel<<<grid_for(NR * kWave), kBlock, 0, s>>>(csr.row_ptr.get(), csr.col.get(), R0, NR, bd.bits, len.get());
    JG_LAUNCH_CHECK();
    prim::exclusive_scan(len.get(), raw.get(), NS, s);
    std::vector<int64_t> bounds(S + 1), begin(S), end(S), base(S + 1);
    {
        DevBuf<int64_t> d_b(S + 1);
        band_bounds_kernel<<<grid_for(S + 1), kBlock, 0, s>>>(raw.get(), NR, S, d_b.get());
        JG_LAUNCH_CHECK();
        copy_d2h(bounds.data(), d_b.get(), (S + 1) * sizeof(int64_t), s);
    }
    int64_t at = 0;
    base[0] = 0;
    for (int h = 0; h < S; ++h) {
        const int64_t n = bounds[h + 1] - bounds[h];
        const int64_t tasks = (n + kMergeTask - 1) / kMergeTask;
        begin[h] = at;
        end[h] = at + n;
        base[h + 1] = base[h] + tasks;
        at += tasks * kMergeTask;
    }
    bd.tasks = base[S];
    bd.sub_begin.alloc(S);
    bd.sub_end.alloc(S);
    bd.sub_base.alloc(S + 1);
    copy_h2d(bd.sub_begin.get(), begin.data(), S * sizeof(int64_t), s);
    copy_h2d(bd.sub_end.get(), end.data(), S * sizeof(int64_t), s);
    copy_h2d(bd.sub_base.get(), base.data(), (S + 1) * sizeof(int64_t), s);
    DevBuf<int64_t> sp((NR + 1) * S);
    band_ptr_kernel<<<grid_for((NR + 1) * S), kBlock, 0, s>>>(raw.get(), NR, S, bd.sub_begin.get(), sp.get());
    JG_LAUNCH_CHECK();
    bd.col.alloc(at + kMergeTask);  // one task of padding: the last task's aligned loads
    JG_HIP(hipMemsetAsync(bd.col.get(), 0, bd.col.bytes(), s));
    band_scatter_kernel<<<grid_for(NR * kWave), kBlock, 0, s>>>(csr.row_ptr.get(), csr.col.get(), R0, NR, bd.bits,
                                                                sp.get(), bd.col.get());
    JG_LAUNCH_CHECK();
    // number the non-empty sub-rows
    DevBuf<int32_t> flag(NS);
    DevBuf<int64_t> num(NS + 1);
    nonempty_kernel<<<grid_for(NS), kBlock, 0, s>>>(len.get(), NS, flag.get());
    JG_LAUNCH_CHECK();
    prim::exclusive_scan(flag.get(), num.get(), NS, s);
    DevBuf<int64_t> nzb(S + 1);
    band_bounds_kernel<<<grid_for(S + 1), kBlock, 0, s>>>(num.get(), NR, S, nzb.get());
    JG_LAUNCH_CHECK();
    copy_d2h(&bd.subrows, num.get() + NS, sizeof(int64_t), s);
    DevBuf<int64_t> cstart(std::max<int64_t>(bd.subrows, 1));
    DevBuf<int32_t> srow(std::max<int64_t>(bd.subrows, 1));
    sub_number_kernel<<<grid_for(NS), kBlock, 0, s>>>(len.get(), num.get(), NR, S, sp.get(), cstart.get(), srow.get());
    JG_LAUNCH_CHECK();
    if (bd.subrows >= (int64_t)INT32_MAX) fail(JG_ERR_UNSUPPORTED, "too many sub-rows in a split band");
    const int64_t W = (NR + 31) / 32;
    bd.sub_word.alloc(std::max<int64_t>(W * S, 1));
    if (W > 0) {
        sub_word_kernel<<<grid_for(W * S), kBlock, 0, s>>>(len.get(), num.get(), NR, S, W, bd.sub_word.get());
        JG_LAUNCH_CHECK();
    }
    bd.meta.alloc(std::max<int64_t>(2 * bd.tasks, 1));
    bd.heads.alloc(std::max<int64_t>(kWave * bd.tasks, 1));
    bd.task_rows.alloc(std::max<int64_t>(2 * bd.tasks, 1));
    if (bd.tasks > 0) {
        task_meta_kernel<<<grid_for(bd.tasks, 64), 64, 0, s>>>(cstart.get(), srow.get(), nzb.get(), S,
                                                               bd.sub_begin.get(), bd.sub_end.get(),
                                                               bd.sub_base.get(), bd.meta.get(), bd.heads.get(),
                                                               bd.task_rows.get());
        JG_LAUNCH_CHECK();
    }
    // the streamed form: packed sub-slice-local indices (the col copy is not kept)
    bd.width = band_width(col_space, bd.bits);
    const int64_t chunks = (at + kMergeTask) / 8;
    const int DB = bd.width / 4 - 4;
    bd.pack_a.alloc(std::max<int64_t>(chunks, 1));
    bd.pack_b.alloc(std::max<int64_t>(chunks * DB, 1));
    if (chunks > 0) {
        const int gshift = 4 + bd.bits;
        if (bd.width == 20)
            band_pack_kernel<20><<<grid_for(chunks), kBlock, 0, s>>>(bd.col.get(), chunks, gshift, bd.pack_a.get(), bd.pack_b.get());
        else if (bd.width == 24)
            band_pack_kernel<24><<<grid_for(chunks), kBlock, 0, s>>>(bd.col.get(), chunks, gshift, bd.pack_a.get(), bd.pack_b.get());
        else
            band_pack_kernel<32><<<grid_for(chunks), kBlock, 0, s>>>(bd.col.get(), chunks, gshift, bd.pack_a.get(), bd.pack_b.get());
        JG_LAUNCH_CHECK();
    }
    JG_HIP(hipStreamSynchronize(s));
    bd.col.reset();
}

// Sub-slices of an automatic band (band<i>_bit = 0, the default for the hub band): the LDS-resident
// share of the vector is 2^bits x one CU's image.  Measured best (tools/pr_ab.py, ms per superstep):
//   RMAT-22: 0.236 / 0.221 / 0.237 at 3 / 4 / 5 bits     RMAT-24: 0.94 / 0.98 / 1.14 at 5 / 6 / 7
//   RMAT-25: 2.18 / 2.14 / 2.36 at 5 / 6 / 7             RMAT-26: 5.29 / 5.05 / 4.88 / 5.48 at 5 / 6 / 7 / 8
// so log2(entries) - 19, within [4, 7], for the 8-byte PageRank vector (IN adjacency).  CC's 4-byte
// labels (BOTH adjacency; tools/cc_ab.py): RMAT-24 14.3 / 14.9 / 16.2 ms at 4 / 5 / 6 bits, RMAT-26
// 56.3 / 58.0 / 67.3 ms at 5 / 6 / 7, so 4 + (log2(entries) - 24) / 2.
// fp64 vectors: log2(entries) - 19, at most 6 (round 4, with rows without out-edges last in their degree
// class: RMAT-26 at 64 sub-slices 3.552 vs 3.592 ms at 128; RMAT-24 stays at 32: 0.761 vs 0.788 ms at 16;
// profiles/r04/ab/); int32 vectors: 4 + (log2 - 24) / 2, at most 7
int auto_band_bits(int64_t vec_entries, int elem_bytes) {
    const int l2 = (int)std::lround(std::log2((double)std::max<int64_t>(vec_entries, 1)));
    const int b = elem_bytes >= 8 ? l2 - 19 : 4 + (l2 - 24) / 2;
    return std::min(std::max(b, 4), elem_bytes >= 8 ? 6 : 7);
}
// Bands after the first (round 5, tools/pr_ab.py, profiles/r05/ab/).  When the whole 8-byte vector fits
// the Infinity Cache on one shard (<= 2^24 entries, 128 MB) one band of in-degree 8-95 with 4 sub-slices
// (each shared by two XCDs): half the sub-row partials where the gathers hit the cache anyway (RMAT-24
// 0.743 / 0.751 / 0.765 ms at 4 / 8 / 2 sub-slices; a third band: no gain).  A larger one-shard 8-byte
// vector: in-degree 16-95 with 8 sub-slices and 8-15 with 4 (RMAT-26 3.473-3.484 against 3.520-3.559 ms
// with one band of 8-95 at 8; 4 sub-slices for all of 8-95: 3.623).  Otherwise (sharded or 4-byte
// vectors: not re-measured) one band of 8-95 with 8.  -> (degree floor, log2 sub-slices) of band i >= 1.
struct AutoBand {
    int64_t deg;
    int bits;
};
AutoBand auto_bands(int i, int64_t vec_entries, int elem_bytes, bool sharded_vec) {
    const bool one8 = elem_bytes >= 8 && !sharded_vec;
    if (one8 && vec_entries <= (1ll << 24)) return i == 1 ? AutoBand{8, 2} : AutoBand{0, 2};
    if (one8) return i == 1 ? AutoBand{16, 3} : i == 2 ? AutoBand{8, 2} : AutoBand{0, 2};
    return i == 1 ? AutoBand{8, 3} : AutoBand{0, 3};
}

void build_pull_plan(Shard& sh, const Csr& csr, PullPlan& plan, int64_t col_space, int64_t vec_entries,
                     int elem_bytes) {
    hipStream_t s = sh.stream;
    // a segmented (sharded) vector splits every LDS image over its segments: one more sub-slice bit
    // (tools/shard_sim.py, RMAT-24 at P = 8: 0.163 vs 0.169 ms per shard superstep at 5 vs 4 bits)
    const bool sharded_vec = col_space != vec_entries && col_space != csr.rows;
    plan.lds_ok = col_space == csr.rows;  // one shard: the hot prefix of the gathered vector is [0, hot)
    plan.col_space = col_space;
    // temporal merge schedule only pays when an XCD's eighth of the vector overflows its 4 MB L2 well
    // (tools/shard_sim.py, RMAT-24 at P = 8, 41 MB vector: 0.173 vs 0.168 ms per shard superstep)
    plan.temporal = vec_entries * elem_bytes > (int64_t)64 << 20;
    const int64_t rows = csr.rows;
    // hub rows (any position) -> chunk table
    std::vector<int64_t> hubs, bounds;
    if (rows > 0) {
        DevBuf<uint8_t> flag(rows);
        DevBuf<int64_t> idx(rows);
        hub_flag_kernel<<<grid_for(rows), kBlock, 0, s>>>(csr.row_ptr.get(), rows, flag.get());
        JG_LAUNCH_CHECK();
        const int64_t nh = prim::compact_indices(flag.get(), rows, idx.get(), s);
        hubs.resize(nh);
        bounds.resize(2 * nh);
        if (nh) {
            DevBuf<int64_t> db(2 * nh);
            gather_row_bounds_kernel<<<grid_for(nh), kBlock, 0, s>>>(csr.row_ptr.get(), idx.get(), nh, db.get());
            JG_LAUNCH_CHECK();
            copy_d2h(hubs.data(), idx.get(), nh * sizeof(int64_t), s);
            copy_d2h(bounds.data(), db.get(), 2 * nh * sizeof(int64_t), s);
        }
    }
    std::vector<int64_t> crow, cbeg, cend, hptr(1, 0);
    for (size_t h = 0; h < hubs.size(); ++h) {
        const int64_t r = hubs[h], b = bounds[2 * h], e = bounds[2 * h + 1];
        for (int64_t p = b; p < e; p += kHubChunk) {
            crow.push_back(r);
            cbeg.push_back(p);
            cend.push_back(std::min(e, p + kHubChunk));
        }
        hptr.push_back((int64_t)crow.size());
    }
    plan.num_hub_rows = (int64_t)hubs.size();
    plan.max_hub_row = hubs.empty() ? -1 : *std::max_element(hubs.begin(), hubs.end());
    plan.num_chunks = (int64_t)crow.size();
    auto upload = [&](DevBuf<int64_t>& d, const std::vector<int64_t>& h) {
        d.alloc(std::max<size_t>(h.size(), 1));
        if (!h.empty()) copy_h2d(d.get(), h.data(), h.size() * sizeof(int64_t), s);
    };
    upload(plan.chunk_row, crow);
    upload(plan.chunk_begin, cbeg);
    upload(plan.chunk_end, cend);
    upload(plan.hub_chunk_ptr, hptr);
    // class boundaries: first row whose degree falls below each class threshold, and the band bounds
    unsigned long long fb[kNumClasses + 1 + 4];
    for (int c = 0; c < kNumClasses; ++c) fb[c] = (unsigned long long)rows;
    fb[kNumClasses] = 0;  // 1 + last non-empty row
    BandThresholds bt{};
    // bands only when the split is enabled at build time (cut from the column-ordered CSR by counting;
    // cutting them from a second, sub-slice-ordered build cost a select and a sort more, round 3)
    // a band's degree floor: the knob, or automatic (-1); the first unused band (0) ends the list
    auto band_floor = [&](int i) {
        return tune().band_deg[i] >= 0 ? tune().band_deg[i] : i == 0 ? 96 : auto_bands(i, vec_entries, elem_bytes, sharded_vec).deg;
    };
    if (tune().pull_split)
        for (int i = 0; i < 4 && band_floor(i) > 0; ++i) bt.thr[bt.n++] = std::max<int64_t>(band_floor(i), 1);
    for (int i = 0; i < 4; ++i) fb[kNumClasses + 1 + i] = (unsigned long long)rows;
    if (rows > 0) {
        DevBuf<unsigned long long> d_fb(kNumClasses + 1 + 4);
        copy_h2d(d_fb.get(), fb, sizeof fb, s);
        class_bound_kernel<<<grid_for(rows), kBlock, 0, s>>>(csr.row_ptr.get(), rows, d_fb.get(),
                                                             d_fb.get() + kNumClasses, bt, d_fb.get() + kNumClasses + 1);
        JG_LAUNCH_CHECK();
        copy_d2h(fb, d_fb.get(), sizeof fb, s);
    }
    // Classes are consecutive row ranges; any row may sit in a "wrong" lane class (only speed
    // changes), but the empty class starts strictly after the last non-empty row (correctness).
    const int64_t zero_begin = (int64_t)fb[kNumClasses];
    csr.empty_from = zero_begin;
    plan.bands.clear();
    int64_t row_at = 0;
    for (int i = 0; i < bt.n; ++i) {
        const int64_t end = std::min<int64_t>((int64_t)fb[kNumClasses + 1 + i], zero_begin);
        if (end <= row_at) continue;
        auto bd = std::make_unique<SliceBand>();
        bd->bits = tune().band_bits[i] >= 0 ? std::min(tune().band_bits[i], 8)
                   : i > 0 ? auto_bands(i, vec_entries, elem_bytes, sharded_vec).bits
                           : std::min(std::max(auto_band_bits(vec_entries, elem_bytes) + (sharded_vec ? 1 : 0), 3), 8);
        bd->row_begin = row_at;
        bd->row_end = end;
        row_at = end;
        plan.bands.push_back(std::move(bd));
    }
    plan.split_rows = row_at;
    auto make_classes = [&](int64_t first_row, int64_t chunks, int64_t* rb, int64_t* re, int64_t* bb) {
        int64_t begin = first_row;
        rb[0] = re[0] = 0;  // hub class is the chunk table
        bb[0] = 0;
        bb[1] = chunks;
        for (int c = 1; c < kNumClasses; ++c) {
            int64_t end = c < kZeroClass - 1 ? (int64_t)fb[c] : c == kZeroClass - 1 ? zero_begin : rows;
            end = std::min(std::max(end, begin), c < kZeroClass ? zero_begin : rows);
            end = std::max(end, begin);
            rb[c] = begin;
            re[c] = end;
            const int lanes = c == kZeroClass ? 1 : 64 >> (c - 1);
            const int64_t rows_per_block = kBlock / lanes;
            bb[c + 1] = bb[c] + (end - begin + rows_per_block - 1) / rows_per_block;
            begin = end;
        }
    };
    make_classes(0, plan.num_chunks, plan.class_row_begin, plan.class_row_end, plan.class_block_begin);
    {
        int64_t part = 0;
        for (auto& bd : plan.bands) {
            build_band(sh, csr, *bd, col_space);
            bd->part_off = part;
            bd->carry_off = part + bd->subrows;
            part += bd->subrows + bd->tasks;
        }
    }
    // light part: rows after the heavy prefix (hub rows are all heavy when rows are degree-sorted;
    // any hub beyond the prefix keeps its chunks, so chunks stay in the light table too)
    make_classes(plan.split_rows, plan.split_rows > 0 ? plan.num_chunks : plan.num_chunks, plan.light_row_begin,
                 plan.light_row_end, plan.light_block_begin);
    // degree runs of the 1-lane light rows (their class starts at the first row below 8 entries)
    plan.runs = false;
    {
        const int64_t lo = plan.light_row_begin[kZeroClass - 1], hi = plan.light_row_end[kZeroClass - 1];
        if (hi > lo && c_class_thr_host[kZeroClass - 2] == kRunMax + 1) {
            int64_t st[17];
            for (int i = 0; i < 17; ++i) st[i] = -1;
            st[0] = 0;
            DevBuf<int64_t> d_st(17);
            copy_h2d(d_st.get(), st, sizeof st, s);
            degree_run_kernel<<<grid_for(hi - lo), kBlock, 0, s>>>(csr.row_ptr.get(), lo, hi, d_st.get());
            JG_LAUNCH_CHECK();
            copy_d2h(st, d_st.get(), sizeof st, s);
            if (st[0] == 0) {
                // absent degrees get an empty run at the start of the next smaller present one
                int64_t next = hi, next_ptr = -1;
                plan.run_begin[0] = hi;
                for (int d = 1; d <= kRunMax; ++d) {
                    if (st[1 + d] >= 0) {
                        next = st[1 + d];
                        next_ptr = st[9 + d];
                    }
                    plan.run_begin[d] = next;
                    plan.run_ptr[d] = st[1 + d] >= 0 ? st[9 + d] : next_ptr;
                }
                plan.runs = plan.run_begin[kRunMax] == lo;
            }
        }
    }
    if (debug_plan()) {
        std::vector<int64_t> rp(rows + 1);
        copy_d2h(rp.data(), csr.row_ptr.get(), (rows + 1) * sizeof(int64_t), s);
        std::fprintf(stderr, "[jg plan] shard %d rows %lld nnz %lld hubs %lld chunks %lld\n", sh.index, (long long)rows,
                     (long long)csr.nnz, (long long)plan.num_hub_rows, (long long)plan.num_chunks);
        for (int c = 1; c < kNumClasses; ++c) {
            const int64_t b = plan.class_row_begin[c], e = plan.class_row_end[c];
            std::fprintf(stderr, "[jg plan]   class %d lanes %2d rows [%lld,%lld) = %lld nnz %lld blocks %lld\n", c,
                         64 >> (c - 1), (long long)b, (long long)e, (long long)(e - b), (long long)(rp[e] - rp[b]),
                         (long long)(plan.class_block_begin[c + 1] - plan.class_block_begin[c]));
        }
        for (size_t i = 0; i < plan.bands.size(); ++i) {
            const SliceBand& bd = *plan.bands[i];
            std::fprintf(stderr, "[jg plan]   band %zu bits %d rows [%lld,%lld) nnz %lld sub-rows %lld tasks %lld\n", i,
                         bd.bits, (long long)bd.row_begin, (long long)bd.row_end,
                         (long long)(rp[bd.row_end] - rp[bd.row_begin]), (long long)bd.subrows, (long long)bd.tasks);
        }
    }
}

namespace {
struct EdgeList {
    const int32_t* src;
    const int32_t* dst;
    int64_t m;
};
}  // namespace

// out[l] = order[r + l * P]: the dense vertex of owned row l of shard r
__global__ void local_dense_kernel(const int32_t* __restrict__ order, int P, int r, int64_t rows,
                                   int32_t* __restrict__ out) {
    for (int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; l < rows; l += (int64_t)gridDim.x * blockDim.x)
        out[l] = order[r + l * P];
}

void build_graph_from_dense(Graph& g, DenseEdges& e) {
    const int64_t n = g.n, m = e.m;
    const int P = g.P;
    g.S = (n + P - 1) / P;
    if (g.S < 1) g.S = 1;
    if ((int64_t)P * g.S >= (int64_t)INT32_MAX) fail(JG_ERR_UNSUPPORTED, "graph too large for int32 vertex ids");
    const int mode = (g.flags & JG_ADJ_IN) ? 0 : (g.flags & JG_ADJ_BOTH) ? 1 : 2;
    const int vbits = bits_for((uint64_t)std::max<int64_t>(n - 1, 0));
    const int cbits = std::max(1, bits_for((uint64_t)(g.padded_len() - 1)));
    bool first = true;
    for (size_t li = 0; li < g.shards.size(); ++li) {
        Shard& sh = *g.shards[li];
        DeviceGuard dg(sh);
        hipStream_t s = sh.stream;
        // The edge list of each adjacency: all of them, unless the snapshot was taken under Fulgora's
        // slice cap (then OUT: the capped OUT entries; IN: the capped IN entries or the capped OUT list).
        const EdgeList all{e.src[li], e.dst[li], m};
        const EdgeList outl = e.capped ? EdgeList{e.out_src[li], e.dst[li], m} : all;
        const EdgeList inl = !e.capped ? all : e.in_from_in ? EdgeList{e.in_src[li], e.in_dst[li], e.m_in} : outl;
        DevBuf<int32_t> indeg(std::max<int64_t>(n, 1)), outdeg(std::max<int64_t>(n, 1));
        DevBuf<unsigned long long> cnt(5);
        JG_HIP(hipMemsetAsync(indeg.get(), 0, indeg.bytes(), s));
        JG_HIP(hipMemsetAsync(outdeg.get(), 0, outdeg.bytes(), s));
        JG_HIP(hipMemsetAsync(cnt.get(), 0, cnt.bytes(), s));
        if (m > 0) {
            degree_kernel<<<grid_for(m, kBlock, 256 * 16), kBlock, 0, s>>>(e.src[li], e.dst[li], m, indeg.get(),
                                                                           outdeg.get(), cnt.get());
            JG_LAUNCH_CHECK();
        }
        if (n > 0) {
            stats_kernel<<<grid_for(n, kBlock, 1024), kBlock, 0, s>>>(indeg.get(), outdeg.get(), n, cnt.get() + 2);
            JG_LAUNCH_CHECK();
        }
        unsigned long long hc[5];
        JG_HIP(hipMemcpyAsync(hc, cnt.get(), sizeof hc, hipMemcpyDeviceToHost, s));
        JG_HIP(hipStreamSynchronize(s));
        if (first) {
            g.info.num_vertices = n;
            g.info.num_edges = (int64_t)hc[0];
            g.info.ghost_edges = m - (int64_t)hc[0];
            g.info.self_loops = (int64_t)hc[1];
            g.info.max_in_degree = (int64_t)hc[2];
            g.info.max_out_degree = (int64_t)hc[3];
            g.info.truncated_vertices = e.capped ? e.truncated_rows : (int64_t)hc[4];
        }
        // Under the cap the directed adjacencies see capped degrees: in-degree from the IN list,
        // out-degree (PageRank's edgeCount) from the OUT list.  BOTH keeps the uncapped sums.
        DevBuf<int32_t> cin, cout_;
        const int32_t *din = indeg.get(), *dout = outdeg.get();
        if (e.capped && mode != 1) {
            cin.alloc(std::max<int64_t>(n, 1));
            cout_.alloc(std::max<int64_t>(n, 1));
            DevBuf<int32_t> scratch(std::max<int64_t>(n, 1));
            DevBuf<unsigned long long> c2(5);
            JG_HIP(hipMemsetAsync(cin.get(), 0, cin.bytes(), s));
            JG_HIP(hipMemsetAsync(cout_.get(), 0, cout_.bytes(), s));
            JG_HIP(hipMemsetAsync(c2.get(), 0, c2.bytes(), s));
            if (inl.m > 0) {
                degree_kernel<<<grid_for(inl.m, kBlock, 256 * 16), kBlock, 0, s>>>(inl.src, inl.dst, inl.m, cin.get(),
                                                                                   scratch.get(), c2.get());
                JG_LAUNCH_CHECK();
            }
            if (outl.m > 0) {
                degree_kernel<<<grid_for(outl.m, kBlock, 256 * 16), kBlock, 0, s>>>(outl.src, outl.dst, outl.m,
                                                                                    scratch.get(), cout_.get(), c2.get());
                JG_LAUNCH_CHECK();
            }
            if (n > 0) {
                stats_kernel<<<grid_for(n, kBlock, 1024), kBlock, 0, s>>>(cin.get(), cout_.get(), n, c2.get() + 2);
                JG_LAUNCH_CHECK();
            }
            JG_HIP(hipMemcpyAsync(hc, c2.get(), sizeof hc, hipMemcpyDeviceToHost, s));
            JG_HIP(hipStreamSynchronize(s));
            din = cin.get();
            dout = cout_.get();
        }
        const int64_t maxdeg = mode == 0 ? (int64_t)hc[2] : mode == 1 ? (int64_t)(hc[2] + hc[3]) : (int64_t)hc[3];
        const EdgeList& pull = mode == 0 ? inl : all;  // the tie-break's pull neighbours (modes 0 and 1)
        // degree-sorted relabel
        DevBuf<uint64_t> rkeys(std::max<int64_t>(n, 1));
        DevBuf<int32_t> order(std::max<int64_t>(n, 1)), padded(std::max<int64_t>(n, 1));
        if (n > 0) {
            relabel_keys_kernel<<<grid_for(n), kBlock, 0, s>>>(din, dout, n, mode, maxdeg, vbits, rkeys.get());
            JG_LAUNCH_CHECK();
            prim::radix_sort(rkeys.get(), nullptr, n, vbits + bits_for((uint64_t)maxdeg), s);
            if (mode != 2 && pull.m > 0) {
                // equal-degree vertices ordered by their hottest pull neighbour (then id)
                const uint64_t vmask = (1ull << vbits) - 1ull;
                DevBuf<int32_t> rank1(n), nbr_min(n);
                rank_scatter_kernel<<<grid_for(n), kBlock, 0, s>>>(rkeys.get(), n, vmask, rank1.get());
                JG_LAUNCH_CHECK();
                const bool dead_last = mode == 0;  // PageRank's gathered vector
                JG_HIP(hipMemsetAsync(nbr_min.get(), 0x7F, nbr_min.bytes(), s));  // > any rank
                nbr_min_kernel<<<grid_for(pull.m, kBlock, 256 * 16), kBlock, 0, s>>>(pull.src, pull.dst, pull.m,
                                                                                      mode, rank1.get(), nbr_min.get());
                JG_LAUNCH_CHECK();
                DevBuf<uint64_t> k1(n), k2(n);
                tie_keys_kernel<<<grid_for(n), kBlock, 0, s>>>(nbr_min.get(), n, vbits, dead_last ? dout : nullptr,
                                                               std::min<int64_t>((int64_t)hc[3], n), k1.get());
                JG_LAUNCH_CHECK();
                prim::radix_sort(k1.get(), nullptr, n, vbits + bits_for((uint64_t)n), s);
                tie_deg_keys_kernel<<<grid_for(n), kBlock, 0, s>>>(k1.get(), n, vmask, din, dout, mode, maxdeg,
                                                                   dead_last, k2.get());
                JG_LAUNCH_CHECK();
                prim::radix_sort(k2.get(), nullptr, n, 33 + bits_for((uint64_t)maxdeg), s);
                tie_final_kernel<<<grid_for(n), kBlock, 0, s>>>(k1.get(), k2.get(), n, vmask, rkeys.get());
                JG_LAUNCH_CHECK();
            }
            padded_ids_kernel<<<grid_for(n), kBlock, 0, s>>>(rkeys.get(), n, (1ull << vbits) - 1ull, P, g.S,
                                                             order.get(), padded.get());
            JG_LAUNCH_CHECK();
        }
        const int r = sh.index;
        sh.rows = std::max<int64_t>(0, std::min<int64_t>(g.S, (n - r + P - 1) / P));
        // dense index of each owned row and padded id of every vertex stay on the device; their host
        // copies are made on first use (Shard::dense_of_local, Graph::padded_of_dense)
        sh.dense_rows.alloc(std::max<int64_t>(sh.rows, 1));
        sh.dense_of_local_host.clear();
        if (sh.rows > 0) {
            local_dense_kernel<<<grid_for(sh.rows), kBlock, 0, s>>>(order.get(), P, r, sh.rows, sh.dense_rows.get());
            JG_LAUNCH_CHECK();
        }
        sh.out_degree.alloc(std::max<int64_t>(sh.rows, 1));
        if (sh.rows > 0) {
            local_outdeg_kernel<<<grid_for(sh.rows), kBlock, 0, s>>>(order.get(), e.capped ? dout : outdeg.get(), n, P,
                                                                     r, sh.rows, sh.out_degree.get());
            JG_LAUNCH_CHECK();
        }
        SelectArgs a{e.src[li], e.dst[li], padded.get(), m, g.S, r, 0, cbits, CompactMap{}};
        const int32_t* w = (e.weight.size() > li) ? e.weight[li] : nullptr;
        auto use = [&](const EdgeList& l) {
            a.src = l.src;
            a.dst = l.dst;
            a.m = l.m;
        };
        // The pull adjacencies (IN: PageRank, BOTH: CC) are first built sub-slice-ordered, which the
        // split bands are cut from (separate copies), then rebuilt column-ordered: traversals scan
        // rows in column (degree-rank) order, and bottom-up BFS exits earlier that way.
        // Sharded: a halo plan first, whose compact ids the CSR columns then hold.
        auto build_pull_csr = [&](int which, const EdgeList& l, const int32_t* wt, Csr& csr, PullPlan& plan,
                                  Halo& halo) {
            use(l);
            a.which = which;
            a.cm = CompactMap{};
            int64_t col_space = g.padded_len(), vec_entries = g.padded_len();
            if (P > 1 && tune().halo) {
                build_halo(g, sh, l.src, l.dst, padded.get(), l.m, which, halo, s);
                a.cm = halo.map(g.S, r);
                col_space = halo.C;
                vec_entries = sh.rows + halo.recv_off[P];
            }
            a.cbits = std::max(cbits, bits_for((uint64_t)(col_space - 1)));  // compact ids may exceed P*S
            // round 3: one column-ordered build, the bands cut from it (band_count / band_scatter)
            build_csr(sh, a, wt, csr, s);
            // the gathered vector of the split: PageRank's fp64 contributions (IN); on BOTH the 64-source
            // BFS's uint64 frontier words on one shard (its main user since CC runs a union-find there:
            // RMAT-26 11.0 -> 10.35 ms with 64 band-0 sub-slices instead of 32, CC unchanged; round 5,
            // profiles/r05/ab/msbfs26_bands.txt), CC's int32 labels on sharded graphs (not re-measured)
            build_pull_plan(sh, csr, plan, col_space, vec_entries, which == 2 && P > 1 ? 4 : 8);
            if (halo.on) {  // segmented compact vector: every segment's hot entries are its prefix
                plan.lds_ok = true;
                plan.seg_tbits = halo.tbits;
                plan.nseg = P;
            }
            if (halo.on) release_halo_maps(halo);
            a.cm = CompactMap{};
            a.cbits = cbits;
        };
        // (the IN entries of a capped snapshot carry no weights: ShortestDistance builds IN from OUT)
        if (g.flags & JG_ADJ_IN) build_pull_csr(0, inl, e.capped && e.in_from_in ? nullptr : w, sh.in, sh.plan_in, sh.halo_in);
        if (g.flags & JG_ADJ_OUT) {
            if (P == 1) {  // one shard: OUT gets the sliced split too (combiner programs over out-edges)
                Halo none;
                build_pull_csr(1, outl, w, sh.out, sh.plan_out, none);
                sh.plan_out_built = true;
            } else {  // sharded OUT has no halo plan: global columns, class plan built on first use
                use(outl);
                a.which = 1;
                build_csr(sh, a, w, sh.out, s);
            }
        }
        if (g.flags & JG_ADJ_BOTH) build_pull_csr(2, all, nullptr, sh.both, sh.plan_both, sh.halo_both);
        JG_HIP(hipStreamSynchronize(s));
        if (first) {  // the first shard's padded ids stay with the graph (vid -> shard / row lookups)
            g.padded_dev = std::move(padded);
            g.padded_host.clear();
            if (g.id_table.size() == 0) g.id_dev = sh.device;  // RMAT graphs: no id table
        }
        first = false;
    }
    if (P > 1 && tune().halo) {
        if (g.flags & JG_ADJ_IN) check_halo_counts(g, JG_ADJ_IN);
        if (g.flags & JG_ADJ_BOTH) check_halo_counts(g, JG_ADJ_BOTH);
    }
    if (g.flags & JG_ADJ_BOTH) cc_prepare_ranks(g);  // ConnectedComponent's labels: a property of the ids
    int64_t bytes = 0;
    for (auto& sp : g.shards)
        bytes += sp->in.bytes() + sp->out.bytes() + sp->both.bytes() + sp->out_degree.bytes() + sp->cc_rank0.bytes();
    bytes += g.cc_vor.bytes();  // the String-order id of each rank (~0.5 GB at RMAT-26)
    g.info.device_bytes = bytes;
    g.info.num_shards = P;
    g.info.flags = g.flags;
}

}  // namespace jg
