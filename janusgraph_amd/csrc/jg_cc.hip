// jg_cc.hip — ConnectedComponentVertexProgram as synchronous min-label pull supersteps.
//
// Reference: TinkerPop 3.4.6 ConnectedComponentVertexProgram (not in the container; SURVEY.md A.3
// [TP-recall]) run by Fulgora with BOTH edges loaded (janusgraph-core/.../olap/computer/
// VertexProgramScanJob.java:113-135); label form pinned by janusgraph-backend-testutils/.../olap/
// OLAPTest.java:736-762 (component == id().toString(), shared by a component).
//   superstep 0: component = id().toString(); vertices with a BOTH edge send it
//   superstep t: min by String.compareTo over messages pulled over BOTH edges from neighbours that
//                sent in t-1; on improvement set + send; halt when nobody sent (or iteration >= 99)
// Labels are carried as the rank of the id's decimal string in String order (bijective), so the
// superstep is an int32 min-semiring pull: msg[g] = label if g sent in t-1, else INT32_MAX.
// String order of non-negative ids: compare x*10^(19-digits(x)) (19-digit left-aligned decimal),
// ties (a prefix such as "1" < "10") broken by fewer digits — computed with two stable radix sorts.
#include <climits>
#include <cstdio>
#include <cstdlib>

#include "jg_frontier.h"
#include "jg_pull.h"

namespace jg {

namespace {

constexpr int kCcMaxIterations = 100;  // ConnectedComponentVertexProgram default maxIterations

struct CcOp {
    using T = int32_t;
    const int32_t* __restrict__ msg;     // full length, previous superstep
    int32_t* __restrict__ msg_out;       // full length (owned slice written)
    int32_t* __restrict__ label;         // [rows]
    int32_t* __restrict__ changed;
    VecPos pos;                          // owned row -> its slot in the gathered vector
    __device__ __forceinline__ int32_t identity() const { return INT_MAX; }
    __device__ __forceinline__ int32_t combine(int32_t a, int32_t b) const { return a < b ? a : b; }
    __device__ __forceinline__ int32_t gather(int32_t c) const { return msg[c]; }
    __device__ __forceinline__ const int32_t* vec() const { return msg; }
    __device__ __forceinline__ int32_t shfl_xor(int32_t v, int o) const { return __shfl_xor(v, o, kWave); }
    __device__ __forceinline__ int32_t shfl_up(int32_t v, int d) const { return __shfl_up(v, d, kWave); }
    __device__ __forceinline__ bool active(int64_t) const { return true; }
    __device__ __forceinline__ void finalize(int64_t row, int32_t m) const {
        if (m < label[row]) {
            label[row] = m;
            msg_out[pos(row)] = m;
            *changed = 1;
        } else {
            msg_out[pos(row)] = INT_MAX;
        }
    }
};

__device__ __forceinline__ int digits_of(uint64_t x) {
    int d = 1;
    while (d < 20 && x >= 10ull) { x /= 10ull; ++d; }
    return d;
}

// pass 1 keys: digit count (tie-break, least significant)
__global__ void lex_digits_kernel(const int64_t* __restrict__ vid, int64_t n, uint64_t* __restrict__ keys,
                                  uint32_t* __restrict__ vals) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        keys[i] = (uint64_t)digits_of((uint64_t)vid[i]);
        vals[i] = (uint32_t)i;
    }
}

// pass 2 keys: left-aligned 19-digit decimal of the id (in pass-1 order)
__global__ void lex_padded_kernel(const int64_t* __restrict__ vid, const uint32_t* __restrict__ vals, int64_t n,
                                  uint64_t* __restrict__ keys) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t x = (uint64_t)vid[vals[i]];
        for (int d = digits_of(x); d < 19; ++d) x *= 10ull;
        keys[i] = x;
    }
}

__global__ void lex_rank_scatter_kernel(const uint32_t* __restrict__ vals, int64_t n, int32_t* __restrict__ rank_of) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        rank_of[vals[r]] = (int32_t)r;
}

__global__ void iota_i64_kernel(int64_t* __restrict__ p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = i;
}

// vor[r] = id of the vertex of rank r (vals: the dense vertex of each rank, after the sorts)
__global__ void vid_of_rank_kernel(const uint32_t* __restrict__ vals, const int64_t* __restrict__ vid, int64_t n,
                                   int64_t* __restrict__ vor) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        vor[r] = vid[vals[r]];
}

__global__ void gather_i32_kernel(const int32_t* __restrict__ src, const int32_t* __restrict__ idx, int64_t n,
                                  int32_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = src[idx[i]];
}

// comp[d] = vor[label[local[d]]]: each caller vertex's component id, in caller order, gathered through
// the inverse of the degree order (a coalesced store per vertex; the scatter through dense_rows it
// replaced wrote one 8-byte value per 64-byte line: ~1.5 ms at RMAT-26, round 5).  The random reads are
// avoided where the answer is known without them: a row of the giant component (one bit per row with an
// edge, `giant`: 4 MB at RMAT-26, cache-resident) takes the giant's id, and a row without an edge (from
// label_rows on) is its own component, whose id is its own (vid_is_dense: the graph's ids are its dense
// indices) or vor[its rank].  Only the other rows gather their label (round 6: 0.78 ms with every row
// gathering its label at RMAT-26, 0.388 ms with the giant bits, 0.345 ms with the loads in phases, 0.327 ms with the streams non-temporal).
__global__ void cc_giant_bits_kernel(const int32_t* __restrict__ label, int64_t label_rows, const int32_t* giant_label,
                                     unsigned long long* __restrict__ giant) {
    const int32_t gl = *giant_label;
    constexpr int R = 4;  // bitmap words per wave and trip, their label loads issued together
    const int64_t span = (int64_t)blockDim.x * R;
    for (int64_t x0 = (int64_t)blockIdx.x * span; x0 < label_rows; x0 += (int64_t)gridDim.x * span) {  // block-uniform
        int32_t lab[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int64_t l = x0 + (int64_t)k * blockDim.x + threadIdx.x;
            lab[k] = l < label_rows ? label[l] : gl ^ 1;
        }
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int64_t l = x0 + (int64_t)k * blockDim.x + threadIdx.x;
            const uint64_t w = __ballot(l < label_rows && lab[k] == gl);
            if (lane_id() == 0 && l < label_rows) giant[l >> 6] = w;
        }
    }
}
constexpr int kCcOutRun = 8;
__global__ void cc_output_kernel(const int32_t* __restrict__ label, const int32_t* __restrict__ rank,
                                 int64_t label_rows, const int32_t* __restrict__ local_of_dense,
                                 const int64_t* __restrict__ vor, int64_t n, int64_t* __restrict__ comp,
                                 const unsigned long long* __restrict__ giant, const int32_t* giant_label,
                                 int vid_is_dense) {
    const int64_t giant_id = vor[*giant_label];
    // kCcOutRun vertices per thread and trip, in phases (every local index, then every giant-bit word, then
    // the rare label gathers), so a lane keeps several random reads in flight instead of one dependent chain
    const int64_t span = (int64_t)blockDim.x * kCcOutRun;
    for (int64_t d0 = (int64_t)blockIdx.x * span + threadIdx.x; d0 < n; d0 += (int64_t)gridDim.x * span) {
        int32_t l[kCcOutRun];
        unsigned long long gw[kCcOutRun];
#pragma unroll
        for (int k = 0; k < kCcOutRun; ++k) {
            const int64_t d = d0 + (int64_t)k * blockDim.x;
            l[k] = d < n ? __builtin_nontemporal_load(&local_of_dense[d]) : -1;
        }
#pragma unroll
        for (int k = 0; k < kCcOutRun; ++k) gw[k] = l[k] >= 0 && l[k] < label_rows ? giant[l[k] >> 6] : 0ull;
#pragma unroll
        for (int k = 0; k < kCcOutRun; ++k) {
            const int64_t d = d0 + (int64_t)k * blockDim.x;
            if (l[k] < 0) continue;
            int64_t v;
            if (l[k] >= label_rows) v = vid_is_dense ? d : vor[rank[l[k]]];
            else if ((gw[k] >> (l[k] & 63)) & 1ull) v = giant_id;
            else v = vor[label[l[k]]];
            __builtin_nontemporal_store(v, &comp[d]);
        }
    }
}

__global__ void cc_init_kernel(const int32_t* __restrict__ lab0, const int64_t* __restrict__ rp, int64_t rows,
                               VecPos pos, int32_t* __restrict__ label, int32_t* __restrict__ msg) {
    for (int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; l < rows; l += (int64_t)gridDim.x * blockDim.x) {
        label[l] = lab0[l];
        msg[pos(l)] = (rp[l + 1] > rp[l]) ? lab0[l] : INT_MAX;  // only vertices with edges send
    }
}

// Sparse supersteps on one shard run push-style: only the vertices that sent a label (changed in
// the previous superstep) are visited; each takes the min into its neighbours' candidates
// (atomicMin: order-independent, so the result equals the pull superstep's), the first toucher of a
// neighbour queues it, and the apply pass keeps the improvements.  No-message cells are any value
// >= kNoMsg (INT_MAX from finalize, 0x7F7F7F7F from a memset); labels are ranks < n.
constexpr int32_t kNoMsg = 0x7F7F7F7F;

__global__ __launch_bounds__(kBlock) void cc_senders_kernel(const int32_t* __restrict__ msg, int64_t rows,
                                                            const int64_t* __restrict__ rp, int32_t* __restrict__ queue,
                                                            int64_t* __restrict__ qoff,
                                                            unsigned long long* __restrict__ packed) {
    __shared__ WaveStage ws;
    WaveApp app{ws};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x0 = (int64_t)blockIdx.x * blockDim.x; x0 < rows; x0 += stride) {  // block-uniform trips
        const int64_t v = x0 + threadIdx.x;
        const bool take = v < rows && msg[v] < kNoMsg;
        app.append(take, (int32_t)v, take ? rp[v + 1] - rp[v] : 0, queue, qoff, packed);
    }
    app.final(queue, qoff, packed);
}

struct CcPush {
    const int32_t* queue;
    const int64_t* qoff;
    int64_t nq, mf;
    const int64_t* rp;
    const int32_t* col;
    const int32_t* msg;
    int32_t* cand;  // the next superstep's message vector, preset to kNoMsg
    int32_t* touched;
    int64_t* touched_off;
    unsigned long long* tpacked;
};

__global__ __launch_bounds__(kBlock) void cc_push_kernel(CcPush a) {
    __shared__ WaveStage ws;
    WaveApp app{ws};
    const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_tile = nthreads * 4;
    const int64_t tiles = (a.mf + per_tile - 1) / per_tile;
    for (int64_t t = 0; t < tiles; ++t) {
        if ((t * nthreads + (int64_t)blockIdx.x * blockDim.x) * 4 >= a.mf) break;  // block-uniform
        const int64_t e0 = (t * nthreads + tid) * 4;
        int64_t i = 0, next_bound = 0;
        if (e0 < a.mf) {
            int64_t lo = 0, hi = a.nq - 1;
            while (lo < hi) {
                const int64_t mid = (lo + hi + 1) >> 1;
                if (a.qoff[mid] <= e0) lo = mid; else hi = mid - 1;
            }
            i = lo;
            next_bound = i + 1 < a.nq ? a.qoff[i + 1] : a.mf;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t e = e0 + k;
            bool take = false;
            int32_t v = 0;
            if (e < a.mf) {
                while (e >= next_bound) {
                    ++i;
                    next_bound = i + 1 < a.nq ? a.qoff[i + 1] : a.mf;
                }
                const int32_t u = a.queue[i];
                v = a.col[a.rp[u] + (e - a.qoff[i])];
                const int32_t m = a.msg[u];
                if (m < a.cand[v]) take = atomicMin(&a.cand[v], m) == kNoMsg;
            }
            app.append(take, v, 0, a.touched, a.touched_off, a.tpacked);
        }
    }
    app.final(a.touched, a.touched_off, a.tpacked);
}

// touched vertex v: the pull superstep's finalize with the pushed minimum
__global__ void cc_push_apply_kernel(const int32_t* __restrict__ touched, int64_t nt, CcOp op) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < nt; x += (int64_t)gridDim.x * blockDim.x) {
        const int32_t v = touched[x];
        op.finalize(v, op.msg_out[v]);  // msg_out holds the candidate; finalize rewrites it
    }
}

// ---- one shard: the fixed point by union-find, the superstep count by BFS ----
// Synchronous min-label propagation gives vertex v after t supersteps the minimum rank within t hops
// (a vertex that did not change sends nothing new, and what it sent before already arrived), so v's
// label is final exactly at t = dist(v, c(v)), c(v) the minimum-rank vertex of its component, and
// the last change anywhere is at D = max dist(v, c(v)).  The loop then stops one superstep later:
// iterations = D + 1 when any vertex has an edge (0 otherwise; cc_run's loop, jo_cc_csr), unless that
// reaches the 99-superstep cap, where the propagation itself runs (tests/test_cc_iterations.py pins
// the identity on the oracle).  So: components by union-find, each component's minimum rank, then
// one BFS started at every component's minimum-rank vertex for D.
//
// The union-find hooks the root of larger index under the smaller (rows are degree-sorted, so hubs
// become roots at once and every other vertex hooks under them without contention; hooking by rank
// instead made every link of the first round fight over the giant component's current root: 6.7 ms
// of CAS retries at RMAT-26).  Hooks are atomicCAS, performed at the memory side, so every XCD sees
// them; finds use plain loads that may be stale inside a kernel, which is safe because a parent chain
// only ever gains ancestors of strictly smaller index: a stale read yields an ancestor, a CAS against
// a stale root fails and returns the current parent.  Path compression runs in kernels of its own.
__device__ __forceinline__ int32_t uf_find(const int32_t* __restrict__ parent, int32_t x) {
    for (;;) {
        const int32_t p = parent[x];
        if (p == x) return x;
        x = p;
    }
}

__device__ __forceinline__ void uf_link(int32_t* parent, int32_t a, int32_t b) {
    a = uf_find(parent, a);
    b = uf_find(parent, b);
    while (a != b) {
        if (a > b) {  // hook the root of larger index (b) under the smaller (a)
            const int32_t t = a;
            a = b;
            b = t;
        }
        const int32_t old = atomicCAS(&parent[b], b, a);
        if (old == b) return;
        b = uf_find(parent, old);
        a = uf_find(parent, a);
    }
}

// Four rows per thread for the streaming union-find passes: 16-byte loads put four times the bytes in
// flight per lane, and the four finds walk in lock step, one dependent load per step for all four (one
// row per lane left these passes bound by load latency: 4.5 TB/s at best, RMAT-26).
constexpr int kQuad = 4;
__device__ __forceinline__ void uf_find4(const int32_t* parent, int32_t (&x)[kQuad]) {
    bool act[kQuad];
#pragma unroll
    for (int k = 0; k < kQuad; ++k) act[k] = true;
    for (;;) {
        int32_t y[kQuad];
#pragma unroll
        for (int k = 0; k < kQuad; ++k) y[k] = act[k] ? parent[x[k]] : x[k];
        bool any = false;
#pragma unroll
        for (int k = 0; k < kQuad; ++k) {
            if (y[k] == x[k]) act[k] = false;
            else {
                x[k] = y[k];
                any = true;
            }
        }
        if (!any) return;
    }
}
// the four entries of a[v0, v0 + 4) (16-byte aligned when v0 is a multiple of 4: DevBuf bases are)
__device__ __forceinline__ void load4(const int32_t* a, int64_t v0, int32_t (&x)[kQuad]) {
    const int4 q = *reinterpret_cast<const int4*>(a + v0);
    x[0] = q.x;
    x[1] = q.y;
    x[2] = q.z;
    x[3] = q.w;
}
__device__ __forceinline__ void store4(int32_t* a, int64_t v0, const int32_t (&x)[kQuad]) {
    *reinterpret_cast<int4*>(a + v0) = make_int4(x[0], x[1], x[2], x[3]);
}

__global__ void uf_init_kernel(int32_t* __restrict__ parent, int32_t* __restrict__ minr, int64_t rows) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < rows; v += (int64_t)gridDim.x * blockDim.x) {
        parent[v] = (int32_t)v;
        minr[v] = INT_MAX;
    }
}

// Afforest's first round: every vertex links to its first k neighbours.  k = 1 (the default) reads
// the dense first-column array (Csr::first_col: one coalesced load, no row_ptr pair or scattered column).
__global__ void uf_link_first_kernel(int32_t* parent, const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                     const int32_t* __restrict__ first, int64_t rows, int k) {
    if (k == 1 && first) {
        for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < rows; v += (int64_t)gridDim.x * blockDim.x) {
            const int32_t u = first[v];
            if (u >= 0 && u != (int32_t)v) uf_link(parent, (int32_t)v, u);
        }
        return;
    }
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < rows; v += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e0 = rp[v], e1 = rp[v + 1] < rp[v] + k ? rp[v + 1] : rp[v] + k;
        for (int64_t e = e0; e < e1; ++e) {
            const int32_t u = col[e];
            if (u != (int32_t)v) uf_link(parent, (int32_t)v, u);
        }
    }
}

// One shard, k = 1: the first round without atomics.  Every row hooks under its first neighbour when
// that neighbour has the smaller index (a plain store of the row's own entry: the parents then all point
// to smaller indices, a forest), the rest keep themselves; uf_link_up_compress_kernel then links the
// rows whose first neighbour has the larger index (rows are degree-sorted and the columns ascending, so
// nearly every row's first neighbour is a hub of smaller index: only the local degree maxima are left).
// The union of the two is the first round's: every row joined to its first neighbour.  Fuses uf_init.
__global__ void uf_hook_first_kernel(int32_t* __restrict__ parent, int32_t* __restrict__ minr,
                                     const int32_t* __restrict__ first, int64_t rows) {
    const int64_t quads = (rows + kQuad - 1) / kQuad;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < quads; q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t v0 = q * kQuad;
        if (v0 + kQuad <= rows) {
            int32_t u[kQuad], p[kQuad];
            load4(first, v0, u);
#pragma unroll
            for (int k = 0; k < kQuad; ++k) p[k] = u[k] >= 0 && u[k] < (int32_t)(v0 + k) ? u[k] : (int32_t)(v0 + k);
            store4(parent, v0, p);
            *reinterpret_cast<int4*>(minr + v0) = make_int4(INT_MAX, INT_MAX, INT_MAX, INT_MAX);
        } else {
            for (int64_t v = v0; v < rows; ++v) {
                const int32_t u = first[v];
                parent[v] = u >= 0 && u < (int32_t)v ? u : (int32_t)v;
                minr[v] = INT_MAX;
            }
        }
    }
}

// The rest of the first round (rows whose first neighbour has the larger index) and the compression in
// one pass.  A row's compression stores its root only when the row is no root itself: a root's entry is
// only ever written by a hook's atomicCAS, so no plain store can undo a concurrent hook, and a non-root
// stays one.  A root found here may be hooked later in the pass, so the entries end up pointing at
// ancestors, not always roots: the finds that follow (rest links, minimum ranks) walk what is left.
__global__ void uf_link_up_compress_kernel(int32_t* parent, const int32_t* __restrict__ first, int64_t rows) {
    const int64_t quads = (rows + kQuad - 1) / kQuad;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < quads; q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t v0 = q * kQuad;
        if (v0 + kQuad <= rows) {
            int32_t u[kQuad], p[kQuad], r[kQuad];
            load4(first, v0, u);
            for (int k = 0; k < kQuad; ++k)  // (rare: the local degree maxima)
                if (u[k] > (int32_t)(v0 + k)) uf_link(parent, (int32_t)(v0 + k), u[k]);
            load4(parent, v0, p);  // after the links: a row's own hook shows in its entry
#pragma unroll
            for (int k = 0; k < kQuad; ++k) r[k] = p[k];
            uf_find4(parent, r);
#pragma unroll
            for (int k = 0; k < kQuad; ++k)
                if (p[k] != (int32_t)(v0 + k) && r[k] != p[k]) parent[v0 + k] = r[k];
        } else {
            for (int64_t v = v0; v < rows; ++v) {
                const int32_t u = first[v];
                if (u > (int32_t)v) uf_link(parent, (int32_t)v, u);
                const int32_t p = parent[v];
                if (p != (int32_t)v) {
                    const int32_t r = uf_find(parent, p);
                    if (r != p) parent[v] = r;
                }
            }
        }
    }
}

// Vertices outside the sampled giant component link their remaining neighbours (an edge between the
// giant component and another vertex is linked from the other side).  Rows are degree-sorted: rows
// below `heavy` (degree >= 64) take a wave each, the others a thread.
// *linked += the entries linked (one atomic per wave; the work counter of jg_stats.algorithmic_bytes)
__global__ __launch_bounds__(kRedThreads) void uf_link_rest_kernel(int32_t* parent, const int64_t* __restrict__ rp,
                                                                    const int32_t* __restrict__ col, int64_t rows,
                                                                    int64_t heavy, int k, const int32_t* giant_p,
                                                                    unsigned long long* __restrict__ linked) {
    __shared__ unsigned long long red[kRedWaves];
    const int32_t giant = *giant_p;
    const int lane = threadIdx.x & (kWave - 1);
    unsigned long long count = 0;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) / kWave;
    for (int64_t v = wave; v < heavy; v += nwaves) {  // wave-uniform
        const int32_t p = parent[v];
        if (p == giant || uf_find(parent, p) == giant) continue;
        if (lane == 0) count += (unsigned long long)(rp[v + 1] - rp[v] - k);
        for (int64_t e = rp[v] + k + lane; e < rp[v + 1]; e += kWave) {
            const int32_t u = col[e];
            if (u != (int32_t)v) uf_link(parent, (int32_t)v, u);
        }
    }
    // light rows four per thread, from the first multiple of four at or past `heavy` (the rows between
    // take a thread each below): the giant test first, so the rows of the giant component (nearly all)
    // never read row_ptr
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (int64_t)gridDim.x * blockDim.x;
    const int64_t h4 = (heavy + kQuad - 1) / kQuad * kQuad;
    auto light = [&](int64_t v, int32_t p) {
        if (p == giant || uf_find(parent, p) == giant) return;
        const int64_t e0 = rp[v], e1 = rp[v + 1];
        if (e1 - e0 <= k) return;
        count += (unsigned long long)(e1 - e0 - k);
        for (int64_t e = e0 + k; e < e1; ++e) {
            const int32_t u = col[e];
            if (u != (int32_t)v) uf_link(parent, (int32_t)v, u);
        }
    };
    for (int64_t v = heavy + tid; v < h4 && v < rows; v += nt) light(v, parent[v]);
    const int64_t quads = (rows - h4 + kQuad - 1) / kQuad;
    for (int64_t q = tid; q < quads; q += nt) {
        const int64_t v0 = h4 + q * kQuad;
        if (v0 + kQuad <= rows) {
            int32_t p[kQuad];
            load4(parent, v0, p);
            if (p[0] == giant && p[1] == giant && p[2] == giant && p[3] == giant) continue;
#pragma unroll
            for (int j = 0; j < kQuad; ++j) light(v0 + j, p[j]);
        } else {
            for (int64_t v = v0; v < rows; ++v) light(v, parent[v]);
        }
    }
    count = block_reduce(count, AddU64{}, red);  // one atomic per block: nearly every wave links something
    if (threadIdx.x == 0 && count) atomicAdd(linked, count);
}

__global__ void uf_compress_kernel(int32_t* parent, int64_t rows) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < rows; v += (int64_t)gridDim.x * blockDim.x)
        parent[v] = uf_find(parent, (int32_t)v);
}

__global__ void uf_sample_kernel(const int32_t* __restrict__ parent, int64_t rows, int n, int32_t* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = parent[(int64_t)(((uint64_t)i * 0x9E3779B97F4A7C15ull) % (uint64_t)rows)];
}

// The giant component's root, on the device: of eight candidates (the root of row 0, the highest-degree
// row, and the first seven sampled roots) the one most frequent among kUfSamples sampled roots.  It
// replaced a read-back, a host sort of the samples and the next launch (~36 us of idle GPU per call at
// RMAT-26, round 6; an LDS bitonic sort of the samples took 79 us).  Any choice is correct (Afforest links
// an edge out of the skipped component from its other end); the most frequent skips the most work.
constexpr int kUfSamples = 1024, kUfCand = 8;
__global__ __launch_bounds__(kUfSamples) void uf_giant_kernel(const int32_t* __restrict__ parent,
                                                              const int32_t* __restrict__ sample,
                                                              int32_t* __restrict__ giant) {
    __shared__ int32_t cand[kUfCand];
    __shared__ int cnt[kUfCand];
    const int t = threadIdx.x;
    if (t < kUfCand) {
        cand[t] = t == 0 ? uf_find(parent, 0) : sample[t - 1];
        cnt[t] = 0;
    }
    const int32_t x = sample[t];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kUfCand; ++k) {
        const uint64_t b = __ballot(x == cand[k]);
        if (lane_id() == 0 && b) atomicAdd(&cnt[k], __popcll(b));
    }
    __syncthreads();
    if (t == 0) {
        int best = 0;
        for (int k = 1; k < kUfCand; ++k) best = cnt[k] > cnt[best] ? k : best;
        *giant = cand[best];
    }
}

// minr[root] = the smallest rank of the root's component: the giant component through a block
// reduction (one atomic per block), the others with an atomicMin each (small components).  The final
// path compression rides along: each row finds its root and stores it when it differs (no hook runs
// here, so a concurrent find reading a rewritten entry still meets an ancestor).
__global__ __launch_bounds__(kRedThreads) void uf_minrank_kernel(int32_t* parent, const int32_t* __restrict__ rank,
                                                                  int64_t rows, const int32_t* giant_p,
                                                                  int32_t* __restrict__ minr) {
    __shared__ int32_t red[kRedWaves];
    const int32_t giant = *giant_p;
    int32_t g = INT_MAX;
    const int64_t quads = (rows + kQuad - 1) / kQuad;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < quads; q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t v0 = q * kQuad;
        if (v0 + kQuad <= rows) {
            int32_t p[kQuad], r[kQuad], k[kQuad];
            load4(parent, v0, p);
            load4(rank, v0, k);
#pragma unroll
            for (int j = 0; j < kQuad; ++j) r[j] = p[j];
            uf_find4(parent, r);  // not `p == giant`: the rest links may have hooked it
#pragma unroll
            for (int j = 0; j < kQuad; ++j) {
                if (r[j] != p[j]) parent[v0 + j] = r[j];
                if (r[j] == giant) g = k[j] < g ? k[j] : g;
                else atomicMin(&minr[r[j]], k[j]);
            }
        } else {
            for (int64_t v = v0; v < rows; ++v) {
                const int32_t p = parent[v], k = rank[v];
                const int32_t r = uf_find(parent, p);
                if (r != p) parent[v] = r;
                if (r == giant) g = k < g ? k : g;
                else atomicMin(&minr[r], k);
            }
        }
    }
    g = block_reduce(g, MinI32{}, red);
    if (threadIdx.x == 0 && g != INT_MAX) atomicMin(&minr[giant], g);
}

// the number of rows of degree >= 64 (rows are degree-sorted: a binary search of the row offsets)
__global__ void heavy_rows_kernel(const int64_t* __restrict__ rp, int64_t rows, int32_t* __restrict__ out) {
    int64_t lo = 0, hi = rows;  // first row of degree < 64
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (rp[mid + 1] - rp[mid] >= kWave) lo = mid + 1; else hi = mid;
    }
    *out = (int32_t)lo;
}

// Union-find labels and the BFS superstep count on one shard; false (labels, label_rows untouched) if the
// count reaches the superstep cap.  On success *labels points at the labels (the parent array, rewritten),
// valid on rows [0, *label_rows) only: rows from *label_rows on (no edge) take their own rank (cc_rank0),
// and the parent array holds nothing meaningful there.
// The union-find runs over the rows that have an edge (those before Csr::empty_from): an edgeless row
// is its own component, with its own rank as label, and is never linked.
// *work_bytes: the bytes the passes need (the §8d-style model of this algorithm): per row
// with an edge 58 B (first hooks 12: the dense first column, the parent and minimum-rank initial values;
// the remaining first links with the first compression 8: the first column again and the parent;
// rest-link giant test 4; minimum rank with the second compression 8; BFS start 21: rank, parent, the
// component minimum, depth, label and seen; BFS depth and seen 5), 12 B per entry linked in the second
// round (col, both finds) and 4 B per adjacency entry of the rows the BFS reached.  k > 1 (Tune::cc_first)
// runs the atomic first round of uf_link_first_kernel instead, under the same model.
bool cc_union_find(Ctx& ctx, Shard& sh, int* iterations, const int32_t** labels, int64_t* label_rows,
                   double* work_bytes, const std::function<void(const int32_t*, int64_t)>* emit = nullptr,
                   hipEvent_t end_ev = nullptr) {
    hipStream_t s = sh.stream;
    const int64_t rows = sh.rows;
    const Csr& c = sh.both;
    const int kFirst = std::max(1, tune().cc_first);  // neighbours each vertex links in the first round
    if (rows == 0) {
        *iterations = 0;
        *labels = sh.cc_rank0.get();
        *label_rows = 0;
        return true;
    }
    const int64_t ne = c.empty_from >= 0 ? std::min(c.empty_from, rows) : rows;
    // scratch: the message vectors (re-initialised if the propagation has to run), a rows array kept
    // with the shard
    int32_t* parent = sh.cc_msg[0].get();
    int32_t* minr = sh.cc_msg[1].get();
    if ((int64_t)sh.cc_depth.size() < rows) sh.cc_depth.alloc(rows);
    DevBuf<int32_t> sample(kUfSamples + 1);  // the sampled roots, then the giant root
    if (sh.cc_linked.size() != 1) sh.cc_linked.alloc(1);
    unsigned long long* linked = sh.cc_linked.get();  // read by the caller after its timed region
    JG_HIP(hipMemsetAsync(linked, 0, sizeof(unsigned long long), s));
    // rows of degree >= 64 (a property of the graph: found once, a binary search of the degree-sorted rows)
    if (sh.cc_heavy < 0) {
        heavy_rows_kernel<<<1, 1, 0, s>>>(c.row_ptr.get(), ne, sample.get());
        JG_LAUNCH_CHECK();
        int32_t h = 0;
        copy_d2h(&h, sample.get(), sizeof h, s);
        sh.cc_heavy = h;
    }
    const int64_t heavy = sh.cc_heavy;
    const int32_t* rank = sh.cc_rank0.get();  // the initial labels are the ranks (cc_prepare_ranks)
    if (kFirst == 1 && c.first_col.get()) {
        uf_hook_first_kernel<<<grid_for((ne + kQuad - 1) / kQuad), kBlock, 0, s>>>(parent, minr, c.first_col.get(), ne);
        JG_LAUNCH_CHECK();
        uf_link_up_compress_kernel<<<grid_for((ne + kQuad - 1) / kQuad), kBlock, 0, s>>>(parent, c.first_col.get(), ne);
        JG_LAUNCH_CHECK();
    } else {
        uf_init_kernel<<<grid_for(ne), kBlock, 0, s>>>(parent, minr, ne);
        JG_LAUNCH_CHECK();
        uf_link_first_kernel<<<grid_for(ne), kBlock, 0, s>>>(parent, c.row_ptr.get(), c.col.get(), c.first_col.get(),
                                                             ne, kFirst);
        JG_LAUNCH_CHECK();
        uf_compress_kernel<<<grid_for(ne), kBlock, 0, s>>>(parent, ne);
        JG_LAUNCH_CHECK();
    }
    // the most frequent root among 1024 sampled vertices: the giant component's
    uf_sample_kernel<<<4, kBlock, 0, s>>>(parent, std::max<int64_t>(ne, 1), kUfSamples, sample.get());
    JG_LAUNCH_CHECK();
    uf_giant_kernel<<<1, kUfSamples, 0, s>>>(parent, sample.get(), sample.get() + kUfSamples);
    JG_LAUNCH_CHECK();
    const int32_t* giant = sample.get() + kUfSamples;
    uf_link_rest_kernel<<<red_grid(ne), kRedThreads, 0, s>>>(parent, c.row_ptr.get(), c.col.get(), ne, heavy, kFirst,
                                                             giant, linked);
    JG_LAUNCH_CHECK();
    uf_minrank_kernel<<<red_grid((ne + kQuad - 1) / kQuad), kRedThreads, 0, s>>>(parent, rank, ne, giant, minr);
    JG_LAUNCH_CHECK();
    // the BFS start picks the sources and rewrites parent into the labels
    double reached = 0;
    // the caller's output gathers read the labels the BFS start writes: queued between the start and the
    // levels, so the GPU does not wait for the host's read of the last level state before running them
    const std::function<void()> out_hook = [&]() { (*emit)(parent, ne); };
    const int d = cc_root_eccentricity(ctx, sh, CcRoots{parent, rank, minr, ne}, sh.cc_depth.get(), &reached,
                                       emit ? &out_hook : nullptr, emit ? end_ev : nullptr);
    const int it = c.nnz > 0 ? d + 1 : 0;
    if (it > kCcMaxIterations - 1) return false;
    // + 12 B per entry the second round linked: the caller adds them from sh.cc_linked after its timed region
    *work_bytes = 58.0 * (double)ne + 4.0 * reached;
    *iterations = it;
    *labels = parent;
    *label_rows = ne;  // an edgeless row's label is its own rank: the BFS start writes the rows before ne only
    return true;
}

void exchange_msg(Graph& g, int which) {
    std::vector<void*> bufs;
    for (auto& sp : g.shards) bufs.push_back(sp->cc_msg[which].peer());
    exchange_vec(g, JG_ADJ_BOTH, bufs, sizeof(int32_t), ncclInt32);
}

// ---- sharded (halo plans): local union-finds, tree labels over the halo, a multi-root sharded BFS ----
// Each shard runs Afforest over its own rows' BOTH entries in its compact vector space (own rows
// [0, rows), then one segment per peer), so a local tree joins own rows and halo copies of their
// neighbours.  A global component is the union of local trees that share a vertex (a copy on one
// shard, the row on its owner), and each cross edge {v on s, x on q} needs linking on ONE side only,
// because labels then flow both ways between a copy and its owner:
//  * a row outside its shard's giant tree (snapshot after the first round) links all its entries, so
//    an edge with such an endpoint is linked on that endpoint's side;
//  * an edge between two giant trees (v in s's, x in q's, `flag` bits from q by exchange_halo_bits) is
//    covered once s's giant tree holds a copy of ANY vertex of q's giant tree: a bounded search over sampled
//    entries of the hub rows links one and marks the peer found; a peer not found falls back to linking
//    every flagged entry of the giant rows into its segment;
// so the giant rows scan nothing on RMAT (one-shard Afforest skips them the same way).
// Label rounds: own labels go to the copies (forward halo exchange), every tree takes the minimum over
// its members, own rows take their tree's, copies take their tree's and send it back to the owners
// (reverse halo exchange, min); until no label changes anywhere.  The superstep count then comes from
// one sharded DO-BFS started at every component's minimum-rank vertex (cc_root_eccentricity_sharded).

constexpr int kCcSearchRows = 64, kCcSearchEntries = 2048;

// The positions of a shard's compact vector that hold something: own rows with an edge [0, ne), then
// each peer's run at the start of its segment.  Segments are 2^tbits apart, so at RMAT-26, P = 8 the
// vector spans 67 M positions for 19 M such slots; the per-slot passes walk these only.
struct SlotMap {
    int64_t ne = 0, total = 0;
    int nseg = 0;
    int64_t start[64], cum[65];  // run k: positions [start[k], start[k] + cum[k + 1] - cum[k])
    __device__ __forceinline__ int64_t pos(int64_t j) const {
        if (j < ne) return j;
        const int64_t k = j - ne;
        int s = 0;
        while (s + 1 < nseg && cum[s + 1] <= k) ++s;
        return start[s] + (k - cum[s]);
    }
};

__global__ void cc_slots_init_kernel(SlotMap m, int32_t* __restrict__ parent) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m.total; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x = m.pos(j);
        parent[x] = (int32_t)x;
    }
}

__global__ void cc_slots_compress_kernel(SlotMap m, int32_t* parent) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m.total; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x = m.pos(j);
        parent[x] = uf_find(parent, (int32_t)x);
    }
}

// every slot's own value (own rows: label, copies: the owner's) as the start of its tree minimum, so
// a root (a singleton in particular: most copies next to giant rows only) takes no atomic for itself.
// Once: later rounds start from the previous round's minima, labels of the same component that every
// member's label has already reached or passed, so the minima stay exact and only fall faster.
__global__ void cc_tree_init_kernel(SlotMap m, const int32_t* __restrict__ label, const int32_t* __restrict__ msg,
                                    int32_t* __restrict__ tmin) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m.total; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x = m.pos(j);
        tmin[x] = j < m.ne ? label[x] : msg[x];
    }
}

struct CcShardLink {
    int32_t* parent;
    const int64_t* rp;
    const int32_t* col;
    int64_t rows, ne, heavy;
    int k;
    const unsigned long long* flag;  // compact bitmap: own rows in this shard's giant tree, copies in their owner's
    int32_t* found;                  // [P] by segment: a copy of the peer's giant tree is in this shard's
    int all_found, tbits;
};

__device__ __forceinline__ bool flag_of(const unsigned long long* f, int32_t x) { return (f[x >> 6] >> (x & 63)) & 1ull; }

// own rows' bits of the flag bitmap (one wave per word): row in the giant tree after the first round
__global__ __launch_bounds__(kBlock) void cc_own_flags_kernel(const int32_t* __restrict__ parent, int64_t ne,
                                                               int64_t rows, int32_t giant, unsigned long long* flag) {
    const int64_t words = (rows + 63) / 64;
    for (int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave; w < words;
         w += ((int64_t)gridDim.x * blockDim.x) / kWave) {
        const int64_t v = w * 64 + lane_id();
        const uint64_t word = __ballot(v < ne && parent[v] == giant);
        if (lane_id() == 0) flag[w] = word;
    }
}

// send-list words for exchange_halo_bits: bit b of word w = the row at that send-list position is in
// the giant tree (a wave per word)
__global__ __launch_bounds__(kBlock) void cc_pack_flags_kernel(const int32_t* __restrict__ parent, int32_t giant,
                                                                const int32_t* __restrict__ send_src,
                                                                const int64_t* __restrict__ send_off,
                                                                const int64_t* __restrict__ woff, int P,
                                                                unsigned long long* __restrict__ sw) {
    const int64_t words = woff[P];
    for (int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave; w < words;
         w += ((int64_t)gridDim.x * blockDim.x) / kWave) {  // wave-uniform
        int q = 0;
        while (q + 1 < P && woff[q + 1] <= w) ++q;
        const int64_t x = send_off[q] + (w - woff[q]) * 64 + lane_id();
        const uint64_t word = __ballot(x < send_off[q + 1] && parent[send_src[x]] == giant);
        if (lane_id() == 0) sw[w] = word;
    }
}

// the bounded search: kCcSearchEntries entries of each of the first kCcSearchRows giant rows (kCcSearchSplit
// waves each, every lane a few entries: one wave per row walked 32 dependent col -> flag -> link steps,
// 114 us per shard at RMAT-26, P = 8) link the flagged copies they meet and mark their segments found
constexpr int kCcSearchSplit = 8;
__global__ __launch_bounds__(kBlock) void cc_giant_search_kernel(CcShardLink a) {
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
    const int64_t row = wave / kCcSearchSplit, part = wave % kCcSearchSplit;
    const int64_t nr = a.ne < kCcSearchRows ? a.ne : kCcSearchRows;
    if (row >= nr || !flag_of(a.flag, (int32_t)row)) return;
    // kCcSearchEntries entries spread evenly over the row (its columns may be ordered by segment)
    const int64_t e0 = a.rp[row], deg = a.rp[row + 1] - e0;
    const int64_t n = deg < kCcSearchEntries ? deg : kCcSearchEntries;
    for (int64_t j = part * kWave + lane_id(); j < n; j += kWave * kCcSearchSplit) {
        const int32_t u = a.col[e0 + j * deg / n];
        if (u >= a.rows && flag_of(a.flag, u)) {
            uf_link(a.parent, (int32_t)row, u);
            a.found[u >> a.tbits] = 1;
        }
    }
}

// the second round: rows outside the giant tree link their remaining entries; giant rows link the
// flagged copies of peers the search did not find (nothing when all were found).  Rows below `heavy`
// (degree >= 64) take a wave each, the others a thread.  *linked += the entries scanned.
__global__ __launch_bounds__(kRedThreads) void cc_link_rest_sharded_kernel(CcShardLink a,
                                                                            unsigned long long* __restrict__ linked) {
    __shared__ unsigned long long red[kRedWaves];
    const int lane = lane_id();
    unsigned long long count = 0;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) / kWave;
    for (int64_t v = wave; v < a.heavy; v += nwaves) {  // wave-uniform
        const bool giant = flag_of(a.flag, (int32_t)v);
        if (giant && a.all_found) continue;
        if (lane == 0) count += (unsigned long long)(a.rp[v + 1] - a.rp[v] - a.k);
        for (int64_t e = a.rp[v] + a.k + lane; e < a.rp[v + 1]; e += kWave) {
            const int32_t u = a.col[e];
            if (u == (int32_t)v) continue;
            if (!giant || (u >= a.rows && !a.found[u >> a.tbits] && flag_of(a.flag, u))) uf_link(a.parent, (int32_t)v, u);
        }
    }
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (int64_t)gridDim.x * blockDim.x;
    for (int64_t v = a.heavy + tid; v < a.ne; v += nt) {
        if (a.rp[v + 1] - a.rp[v] <= a.k) continue;
        const bool giant = flag_of(a.flag, (int32_t)v);
        if (giant && a.all_found) continue;
        count += (unsigned long long)(a.rp[v + 1] - a.rp[v] - a.k);
        for (int64_t e = a.rp[v] + a.k; e < a.rp[v + 1]; ++e) {
            const int32_t u = a.col[e];
            if (u == (int32_t)v) continue;
            if (!giant || (u >= a.rows && !a.found[u >> a.tbits] && flag_of(a.flag, u))) uf_link(a.parent, (int32_t)v, u);
        }
    }
    count = block_reduce(count, AddU64{}, red);
    if (threadIdx.x == 0 && count) atomicAdd(linked, count);
}

// T[root] = the minimum over the tree's members: own rows with an edge their labels, copies their
// owners'; the giant tree's through a block reduction (one atomic per block)
__global__ __launch_bounds__(kRedThreads) void cc_tree_min_kernel(SlotMap sm, const int32_t* __restrict__ parent,
                                                                   const int32_t* __restrict__ label,
                                                                   const int32_t* __restrict__ msg, int32_t giant,
                                                                   int32_t* __restrict__ tmin) {
    __shared__ int32_t red[kRedWaves];
    int32_t g = INT_MAX;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < sm.total; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x = sm.pos(j);
        const int32_t m = j < sm.ne ? label[x] : msg[x];
        if (m >= kNoMsg) continue;
        const int32_t r = parent[x];
        if (r == giant) g = m < g ? m : g;
        else if (m < tmin[r]) atomicMin(&tmin[r], m);
    }
    g = block_reduce(g, MinI32{}, red);
    if (threadIdx.x == 0 && g != INT_MAX && giant >= 0) atomicMin(&tmin[giant], g);
}

__device__ __forceinline__ bool bit_at(const unsigned long long* b, int64_t i) { return (b[i >> 6] >> (i & 63)) & 1ull; }

// Counters of rows whose label fell: kFellLines counters on lines of their own, a block adds its sum to
// counter (block mod kFellLines) (one counter for every wave of the grid cost ~40-100 us per launch in
// same-address atomics); the host sums them.  Every thread of the block calls this.
constexpr int kFellLines = 64, kFellStride = 16;
__device__ __forceinline__ void add_fell(unsigned long long* ctr, unsigned long long c) {
    __shared__ unsigned long long s;
    if (threadIdx.x == 0) s = 0;
    __syncthreads();
    if (c) atomicAdd(&s, c);
    __syncthreads();
    if (threadIdx.x == 0 && s) atomicAdd(&ctr[(blockIdx.x % kFellLines) * kFellStride], s);
}
__device__ __forceinline__ void set_bit_at(unsigned long long* b, int64_t i) {
    const unsigned long long m = 1ull << (i & 63);
    if (!(b[i >> 6] & m)) atomicOr(&b[i >> 6], m);
}

// own rows with an edge take their tree's minimum (labels only decrease; a row whose label fell is
// marked in `dirty` for the next round's sparse forward); copies take it too, for the reverse exchange
// (A wave's 64 consecutive slots below ne are one aligned dirty word: the wave's ballot, ORed in by one
// lane; no other wave of the launch touches that word.)  nchg += own rows whose label fell.
__global__ __launch_bounds__(kBlock) void cc_tree_apply_kernel(SlotMap sm, const int32_t* __restrict__ parent,
                                                                int32_t* __restrict__ tmin, int32_t* __restrict__ label,
                                                                int32_t* __restrict__ msg, int32_t* __restrict__ changed,
                                                                unsigned long long* __restrict__ dirty,
                                                                unsigned long long* __restrict__ nchg) {
    unsigned long long cnt = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j0 = (int64_t)blockIdx.x * blockDim.x + wave_id() * kWave; j0 < sm.total; j0 += stride) {  // wave-uniform
        const int64_t j = j0 + lane_id();
        bool fell = false;
        if (j < sm.total) {
            const int64_t x = sm.pos(j);
            const int32_t t = tmin[parent[x]];
            if (j < sm.ne) {
                if (t < label[x]) {
                    label[x] = t;
                    fell = true;
                }
            } else {
                msg[x] = t;
            }
        }
        const unsigned long long m = __ballot(fell);
        if (m && lane_id() == 0) {
            // j0 is 64-aligned and below ne wherever a bit is set; the word is zero (cleared for this
            // round, no other wave writes it, the reverse apply runs after): a plain store, no read
            dirty[j0 >> 6] = m;
            cnt += (unsigned long long)__popcll(m);
        }
    }
    if (lane_id() == 0 && cnt) *changed = 1;
    add_fell(nchg, cnt);
}

// the copies' tree minima back at the owners (element j is about own row send_src[j])
__global__ void cc_reverse_apply_kernel(const int32_t* __restrict__ rbuf, const int32_t* __restrict__ send_src, int64_t n,
                                        int32_t* __restrict__ label, int32_t* __restrict__ changed,
                                        unsigned long long* __restrict__ dirty, unsigned long long* __restrict__ nchg) {
    unsigned long long cnt = 0;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        const int32_t v = send_src[j], m = rbuf[j];
        if (m < label[v]) {  // non-returning atomics (a returning one stalls the lane on every changed row);
            atomicMin(&label[v], m);  // a row lowered by two elements is counted twice (the count only has to
            atomicOr(&dirty[v >> 6], 1ull << (v & 63));  // be non-zero exactly when something fell)
            ++cnt;
        }
    }
    if (__ballot(cnt != 0) && lane_id() == 0) *changed = 1;
    add_fell(nchg, cnt);
}

// ---- sparse label rounds (cc_sparse) ----
// After the first round a label only moves when it fell in the previous one.  Own rows whose label fell
// are marked in `dirty` (the apply and the reverse apply above and below); the next round sends only
// their send-list entries, as (offset in the run to the peer) << 32 | label pairs (forward), feeds only
// them and the received copies into the tree minima (marking each root whose minimum fell in `rootb`),
// applies only the slots of those roots, and sends back only the copies whose minimum fell (reverse
// pairs, `cb` marks them).  A direction goes dense when its pairs over all shards are at least half the
// dense run (a pair is two int32 elements).  Unchanged values change no minimum, so the rounds, their
// count and the labels are the dense rounds' exactly.
constexpr int kMaxPeersCc = 64;

// peer of send-list element j (offsets in LDS)
__device__ __forceinline__ int run_peer(const int64_t* off, int P, int64_t j) {
    int q = 0;
    while (q + 1 < P && off[q + 1] <= j) ++q;
    return q;
}
// the peer whose run sits in segment s of shard r's compact vector (inverse of Halo::seg_of)
__device__ __forceinline__ int seg_peer(int s, int r) { return s <= r ? s - 1 : s; }

// pass 1 of a forward: dirty send-list elements per peer (pcnt[q] +=)
__global__ __launch_bounds__(kBlock) void cc_fwd_count_kernel(const int32_t* __restrict__ send_src,
                                                               const int64_t* __restrict__ send_off, int P,
                                                               const unsigned long long* __restrict__ dirty,
                                                               unsigned long long* __restrict__ pcnt) {
    __shared__ int64_t so[kMaxPeersCc + 1];
    __shared__ unsigned int lc[kMaxPeersCc];
    for (int q = threadIdx.x; q <= P; q += blockDim.x) so[q] = send_off[q];
    for (int q = threadIdx.x; q < P; q += blockDim.x) lc[q] = 0u;
    __syncthreads();
    const int64_t n = so[P];
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
        if (bit_at(dirty, send_src[j])) atomicAdd(&lc[run_peer(so, P, j)], 1u);
    __syncthreads();
    for (int q = threadIdx.x; q < P; q += blockDim.x)
        if (lc[q]) atomicAdd(&pcnt[q], (unsigned long long)lc[q]);
}

// pass 2: the pairs, grouped by peer at pbase[q] (order inside a group: any)
__global__ __launch_bounds__(kBlock) void cc_fwd_pack_kernel(const int32_t* __restrict__ send_src,
                                                              const int64_t* __restrict__ send_off, int P,
                                                              const unsigned long long* __restrict__ dirty,
                                                              const int32_t* __restrict__ label,
                                                              const int64_t* __restrict__ pbase,
                                                              unsigned long long* __restrict__ cursor,
                                                              unsigned long long* __restrict__ pairs) {
    __shared__ int64_t so[kMaxPeersCc + 1];
    __shared__ unsigned int lc[kMaxPeersCc];
    __shared__ int64_t gb[kMaxPeersCc];
    for (int q = threadIdx.x; q <= P; q += blockDim.x) so[q] = send_off[q];
    __syncthreads();
    const int64_t n = so[P];
    // one tile of blockDim elements per trip (block-uniform trips): LDS counters rank the tile's pairs per
    // peer, one global add per (tile, peer) reserves their slots (a global add per pair serialised on the
    // P cursors: 1.4 ms for 126 K pairs)
    for (int64_t j0 = (int64_t)blockIdx.x * blockDim.x; j0 < n; j0 += (int64_t)gridDim.x * blockDim.x) {
        for (int q = threadIdx.x; q < P; q += blockDim.x) lc[q] = 0u;
        __syncthreads();
        const int64_t j = j0 + threadIdx.x;
        int q = -1;
        unsigned int li = 0;
        int32_t v = 0;
        if (j < n) {
            v = send_src[j];
            if (bit_at(dirty, v)) {
                q = run_peer(so, P, j);
                li = atomicAdd(&lc[q], 1u);
            }
        }
        __syncthreads();
        for (int x = threadIdx.x; x < P; x += blockDim.x)
            gb[x] = lc[x] ? pbase[x] + (int64_t)atomicAdd(&cursor[x], (unsigned long long)lc[x]) : 0;
        __syncthreads();
        if (q >= 0) pairs[gb[q] + li] = ((unsigned long long)(j - so[q]) << 32) | (uint32_t)label[v];
        __syncthreads();
    }
}

// receiver of a forward: each pair's copy slot takes the owner's label and lowers its tree's minimum
// (roff[q]: where sender q's pairs start)
__global__ __launch_bounds__(kBlock) void cc_fwd_recv_kernel(const unsigned long long* __restrict__ rpairs,
                                                              const int64_t* __restrict__ roff, int P, int r, int tbits,
                                                              const int32_t* __restrict__ parent,
                                                              int32_t* __restrict__ msg, int32_t* __restrict__ tmin,
                                                              unsigned long long* __restrict__ rootb) {
    __shared__ int64_t ro[kMaxPeersCc + 1];
    for (int q = threadIdx.x; q <= P; q += blockDim.x) ro[q] = roff[q];
    __syncthreads();
    const int64_t n = ro[P];
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int q = run_peer(ro, P, k);
        const unsigned long long p = rpairs[k];
        const int32_t val = (int32_t)(uint32_t)p;
        const int64_t x = ((int64_t)(q < r ? q + 1 : q) << tbits) + (int64_t)(p >> 32);
        msg[x] = val;
        const int32_t root = parent[x];
        if (val < tmin[root] && val < atomicMin(&tmin[root], val)) set_bit_at(rootb, root);
    }
}

// own rows whose label fell last round lower their tree's minimum
__global__ void cc_own_tree_min_kernel(const unsigned long long* __restrict__ dirty, int64_t ne,
                                       const int32_t* __restrict__ label, const int32_t* __restrict__ parent,
                                       int32_t* __restrict__ tmin, unsigned long long* __restrict__ rootb) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < ne; v += (int64_t)gridDim.x * blockDim.x) {
        if (!bit_at(dirty, v)) continue;
        const int32_t val = label[v], root = parent[v];
        if (val < tmin[root] && val < atomicMin(&tmin[root], val)) set_bit_at(rootb, root);
    }
}

// the slots of roots whose minimum fell: own rows take it (dirty), copies take it when it is lower (cb,
// counted per peer for the reverse pairs)
__global__ __launch_bounds__(kBlock) void cc_apply_sparse_kernel(SlotMap sm, const int32_t* __restrict__ parent,
                                                                  const int32_t* __restrict__ tmin,
                                                                  const unsigned long long* __restrict__ rootb,
                                                                  int32_t* __restrict__ label, int32_t* __restrict__ msg,
                                                                  unsigned long long* __restrict__ dirty,
                                                                  unsigned long long* __restrict__ cb, int r, int P,
                                                                  int tbits, unsigned long long* __restrict__ pcnt,
                                                                  int32_t* __restrict__ changed,
                                                                  unsigned long long* __restrict__ nchg) {
    __shared__ unsigned int lc[kMaxPeersCc];
    for (int q = threadIdx.x; q < P; q += blockDim.x) lc[q] = 0u;
    __syncthreads();
    unsigned long long cnt = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j0 = (int64_t)blockIdx.x * blockDim.x + wave_id() * kWave; j0 < sm.total; j0 += stride) {  // wave-uniform
        const int64_t j = j0 + lane_id();
        bool fell = false;
        if (j < sm.total) {
            const int64_t x = sm.pos(j);
            const int32_t root = parent[x];
            if (bit_at(rootb, root)) {
                const int32_t t = tmin[root];
                if (j < sm.ne) {
                    if (t < label[x]) {
                        label[x] = t;
                        fell = true;
                    }
                } else if (t < msg[x]) {
                    msg[x] = t;
                    set_bit_at(cb, x);
                    atomicAdd(&lc[seg_peer((int)(x >> tbits), r)], 1u);
                }
            }
        }
        const unsigned long long m = __ballot(fell);
        if (m && lane_id() == 0) {
            dirty[j0 >> 6] = m;  // as in cc_tree_apply_kernel
            cnt += (unsigned long long)__popcll(m);
        }
    }
    if (lane_id() == 0 && cnt) *changed = 1;
    add_fell(nchg, cnt);
    __syncthreads();
    for (int q = threadIdx.x; q < P; q += blockDim.x)
        if (lc[q]) atomicAdd(&pcnt[q], (unsigned long long)lc[q]);
}

// the reverse pairs: marked copies, grouped by owner at pbase[q]
__global__ __launch_bounds__(kBlock) void cc_rev_pack_kernel(SlotMap sm, const unsigned long long* __restrict__ cb,
                                                              const int32_t* __restrict__ msg, int r, int P, int tbits,
                                                              const int64_t* __restrict__ pbase,
                                                              unsigned long long* __restrict__ cursor,
                                                              unsigned long long* __restrict__ pairs) {
    __shared__ unsigned int lc[kMaxPeersCc];
    __shared__ int64_t gb[kMaxPeersCc];
    for (int64_t j0 = sm.ne + (int64_t)blockIdx.x * blockDim.x; j0 < sm.total; j0 += (int64_t)gridDim.x * blockDim.x) {
        for (int q = threadIdx.x; q < P; q += blockDim.x) lc[q] = 0u;
        __syncthreads();
        const int64_t j = j0 + threadIdx.x;
        int q = -1;
        unsigned int li = 0;
        int64_t x = 0;
        if (j < sm.total) {
            x = sm.pos(j);
            if (bit_at(cb, x)) {
                q = seg_peer((int)(x >> tbits), r);
                li = atomicAdd(&lc[q], 1u);
            }
        }
        __syncthreads();
        for (int y = threadIdx.x; y < P; y += blockDim.x)
            gb[y] = lc[y] ? pbase[y] + (int64_t)atomicAdd(&cursor[y], (unsigned long long)lc[y]) : 0;
        __syncthreads();
        if (q >= 0) {
            const int64_t s0 = (x >> tbits) << tbits;
            pairs[gb[q] + li] = ((unsigned long long)(x - s0) << 32) | (uint32_t)msg[x];
        }
        __syncthreads();
    }
}

// the owner's side of the reverse pairs (sender q's pairs at roff[q]; its run offset names own row
// send_src[send_off[q] + offset])
__global__ __launch_bounds__(kBlock) void cc_rev_recv_kernel(const unsigned long long* __restrict__ rpairs,
                                                              const int64_t* __restrict__ roff, int P,
                                                              const int32_t* __restrict__ send_src,
                                                              const int64_t* __restrict__ send_off,
                                                              int32_t* __restrict__ label,
                                                              unsigned long long* __restrict__ dirty,
                                                              int32_t* __restrict__ changed,
                                                              unsigned long long* __restrict__ nchg) {
    __shared__ int64_t ro[kMaxPeersCc + 1];
    for (int q = threadIdx.x; q <= P; q += blockDim.x) ro[q] = roff[q];
    __syncthreads();
    const int64_t n = ro[P];
    unsigned long long cnt = 0;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int q = run_peer(ro, P, k);
        const unsigned long long p = rpairs[k];
        const int32_t val = (int32_t)(uint32_t)p, v = send_src[send_off[q] + (int64_t)(p >> 32)];
        if (val < label[v] && val < atomicMin(&label[v], val)) {
            set_bit_at(dirty, v);
            ++cnt;
        }
    }
    if (__ballot(cnt != 0) && lane_id() == 0) *changed = 1;
    add_fell(nchg, cnt);
}

// Every shard of the process (halo plans; cc_label holds the ranks).  false (labels untouched, message
// vectors to be re-initialised) if the superstep count reaches the cap; else each shard's labels are
// in cc_label.
bool cc_union_find_sharded(Graph& g, int* iterations, int* rounds_out, double* work_bytes) {
    const size_t ns = g.shards.size();
    const int P = g.P;
    struct St {
        DevBuf<int32_t> tmin, label, rank, found, rbuf;
        DevBuf<int64_t> send_off, woff;
        DevBuf<unsigned long long> flag, sw;
        DevBuf<unsigned long long> linked;  // [1] entries scanned by the second round (on the shard's device)
        // sparse rounds: own rows whose label fell (this round's / the last round's), roots whose minimum
        // fell, copies whose value fell; per-peer pair counts [2P] (forward, reverse) and cursors [P];
        // the pair buffers and their per-peer offsets (pbase: send, roffd: receive)
        DevBuf<unsigned long long> dirty[2], rootb, cb, pcnt, cursor, spairs, rpairs;
        DevBuf<unsigned long long> nchg;  // [kFellLines * kFellStride] own rows whose label fell this round
        DevBuf<int64_t> pbase, roffd;
        int64_t ne = 0, len = 0, heavy = 0, nsend = 0;
        int32_t giant = -1;
        int giant_share = 0, all_found = 0;
        SlotMap sm;
    };
    std::vector<St> st(ns);
    const int kFirst = std::max(1, tune().cc_first);
    double bytes = 0;
    auto link_args = [&](size_t i) {
        Shard& sh = *g.shards[i];
        St& t = st[i];
        return CcShardLink{sh.cc_msg[1].get(), sh.both.row_ptr.get(), sh.both.col.get(), sh.rows, t.ne, t.heavy, kFirst,
                           t.flag.get(), t.found.get(), t.all_found, sh.halo_both.tbits};
    };
    // first round, giant sample, own flags, send-list flags
    std::vector<uint64_t*> swv, flv;
    for (size_t i = 0; i < ns; ++i) {
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        hipStream_t s = sh.stream;
        St& t = st[i];
        const Csr& c = sh.both;
        const Halo& h = sh.halo_both;
        t.ne = c.empty_from >= 0 ? std::min(c.empty_from, sh.rows) : sh.rows;
        t.len = g.vec_len(sh, JG_ADJ_BOTH);
        t.nsend = h.send_off[(size_t)P];
        t.sm.ne = t.ne;
        t.sm.cum[0] = 0;
        for (int q = 0; q < P; ++q) {
            const int64_t nr = q == sh.index ? 0 : h.recv_off[(size_t)q + 1] - h.recv_off[(size_t)q];
            if (nr == 0) continue;
            t.sm.start[t.sm.nseg] = (int64_t)h.seg_of(q, sh.index) << h.tbits;
            t.sm.cum[t.sm.nseg + 1] = t.sm.cum[t.sm.nseg] + nr;
            ++t.sm.nseg;
        }
        t.sm.total = t.ne + t.sm.cum[t.sm.nseg];
        int32_t* parent = sh.cc_msg[1].get();
        t.tmin.alloc(t.len);
        t.label.alloc(std::max<int64_t>(sh.rows, 1));
        t.rank.alloc(std::max<int64_t>(sh.rows, 1));
        t.found.alloc(P);
        t.rbuf.alloc(std::max<int64_t>(t.nsend, 1));
        t.flag.alloc((t.len + 63) / 64);
        const std::vector<int64_t> woff = halo_word_offsets(h, P);
        t.sw.alloc(std::max<int64_t>(woff[(size_t)P], 1));
        t.send_off.alloc(P + 1);
        t.woff.alloc(P + 1);
        copy_h2d(t.send_off.get(), h.send_off.data(), (P + 1) * sizeof(int64_t), s);
        copy_h2d(t.woff.get(), woff.data(), (P + 1) * sizeof(int64_t), s);
        JG_HIP(hipMemsetAsync(t.found.get(), 0, P * sizeof(int32_t), s));
        JG_HIP(hipMemsetAsync(t.flag.get(), 0, t.flag.bytes(), s));
        t.linked.alloc(1);
        JG_HIP(hipMemsetAsync(t.linked.get(), 0, sizeof(unsigned long long), s));
        if (sh.rows) {  // labels start at the ranks (cc_prepare_ranks)
            JG_HIP(hipMemcpyAsync(t.label.get(), sh.cc_rank0.get(), sh.rows * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
            JG_HIP(hipMemcpyAsync(t.rank.get(), sh.cc_rank0.get(), sh.rows * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
        }
        if (t.sm.total) {
            cc_slots_init_kernel<<<grid_for(t.sm.total), kBlock, 0, s>>>(t.sm, parent);
            JG_LAUNCH_CHECK();
        }
        if (t.ne > 0) {
            DevBuf<int32_t> sample(1025);
            uf_link_first_kernel<<<grid_for(t.ne), kBlock, 0, s>>>(parent, c.row_ptr.get(), c.col.get(),
                                                                   c.first_col.get(), t.ne, kFirst);
            JG_LAUNCH_CHECK();
            cc_slots_compress_kernel<<<grid_for(t.sm.total), kBlock, 0, s>>>(t.sm, parent);
            JG_LAUNCH_CHECK();
            // the most frequent root among 1024 sampled own rows: the giant tree's
            uf_sample_kernel<<<4, kBlock, 0, s>>>(parent, t.ne, 1024, sample.get());
            JG_LAUNCH_CHECK();
            heavy_rows_kernel<<<1, 1, 0, s>>>(c.row_ptr.get(), t.ne, sample.get() + 1024);
            JG_LAUNCH_CHECK();
            std::vector<int32_t> hs(1025);
            copy_d2h(hs.data(), sample.get(), hs.size() * sizeof(int32_t), s);
            t.heavy = hs[1024];
            hs.pop_back();
            std::sort(hs.begin(), hs.end());
            size_t best = 0;
            for (size_t a = 0; a < hs.size();) {
                size_t b = a;
                while (b < hs.size() && hs[b] == hs[a]) ++b;
                if (b - a > best) {
                    best = b - a;
                    t.giant = hs[a];
                    t.giant_share = (int)best;
                }
                a = b;
            }
            cc_own_flags_kernel<<<grid_for(((sh.rows + 63) / 64) * kWave), kBlock, 0, s>>>(parent, t.ne, sh.rows, t.giant,
                                                                                          t.flag.get());
            JG_LAUNCH_CHECK();
        }
        if (woff[(size_t)P] > 0) {
            cc_pack_flags_kernel<<<grid_for(woff[(size_t)P] * kWave), kBlock, 0, s>>>(parent, t.giant, h.send_src.get(),
                                                                              t.send_off.get(), t.woff.get(), P,
                                                                              t.sw.get());
            JG_LAUNCH_CHECK();
        }
        swv.push_back(reinterpret_cast<uint64_t*>(t.sw.get()));
        flv.push_back(reinterpret_cast<uint64_t*>(t.flag.get()));
    }
    exchange_halo_bits(g, JG_ADJ_BOTH, swv, flv, false);  // the copies' flags: in their owner's giant tree
    // the bounded search, then the second round
    for (size_t i = 0; i < ns; ++i) {
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        hipStream_t s = sh.stream;
        St& t = st[i];
        if (t.ne == 0) continue;
        if (tune().cc_uf_search) {  // 0: every peer takes the fallback (a parity-test variant)
            cc_giant_search_kernel<<<(kCcSearchRows * kCcSearchSplit * kWave + kBlock - 1) / kBlock, kBlock, 0, s>>>(
                link_args(i));
            JG_LAUNCH_CHECK();
        }
        std::vector<int32_t> found((size_t)P);
        copy_d2h(found.data(), t.found.get(), P * sizeof(int32_t), s);
        const Halo& h = sh.halo_both;
        t.all_found = 1;
        for (int q = 0; q < P; ++q)
            if (q != sh.index && h.recv_off[(size_t)q + 1] > h.recv_off[(size_t)q] && !found[(size_t)h.seg_of(q, sh.index)])
                t.all_found = 0;
        cc_link_rest_sharded_kernel<<<red_grid(t.ne), kRedThreads, 0, s>>>(link_args(i), t.linked.get());
        JG_LAUNCH_CHECK();
        cc_slots_compress_kernel<<<grid_for(t.sm.total), kBlock, 0, s>>>(t.sm, sh.cc_msg[1].get());
        JG_LAUNCH_CHECK();
    }
    // the label rounds
    std::vector<void*> mv, rv;
    for (size_t i = 0; i < ns; ++i) {
        mv.push_back(g.shards[i]->cc_msg[0].peer());
        rv.push_back(st[i].rbuf.peer());
    }
    for (size_t i = 0; i < ns; ++i) {  // the sparse rounds' marks and counters
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        St& t = st[i];
        for (int k = 0; k < 2; ++k) {
            t.dirty[k].alloc((size_t)std::max<int64_t>((sh.rows + 63) / 64, 1));
            JG_HIP(hipMemsetAsync(t.dirty[k].get(), 0, t.dirty[k].bytes(), sh.stream));
        }
        t.rootb.alloc((size_t)std::max<int64_t>((t.len + 63) / 64, 1));
        t.cb.alloc((size_t)std::max<int64_t>((t.len + 63) / 64, 1));
        JG_HIP(hipMemsetAsync(t.rootb.get(), 0, t.rootb.bytes(), sh.stream));
        JG_HIP(hipMemsetAsync(t.cb.get(), 0, t.cb.bytes(), sh.stream));
        t.pcnt.alloc(2 * (size_t)P);
        t.nchg.alloc((size_t)kFellLines * kFellStride);
        t.cursor.alloc((size_t)P);
        t.pbase.alloc((size_t)P);
        t.roffd.alloc((size_t)P + 1);
    }
    // One sparse exchange step (the pair counts are in pcnt + cofs per shard): the P x P count matrix
    // and the dense volume are summed over ranks, so every rank takes the same decision; false = dense
    // is cheaper (nothing sent).  pack(i) packs shard i's pairs, recv(i) consumes what it received.
    int64_t dense_fwd = 0;  // elements of one dense exchange over all shards
    for (size_t i = 0; i < ns; ++i) dense_fwd += st[i].nsend;
    auto sparse_step = [&](int cofs, auto&& pack, auto&& recv) -> bool {
        std::vector<std::vector<int64_t>> cnt(ns, std::vector<int64_t>((size_t)P, 0));
        std::vector<int64_t> mat((size_t)P * P + 1, 0);
        for (size_t i = 0; i < ns; ++i) {
            Shard& sh = *g.shards[i];
            DeviceGuard dg(sh);
            std::vector<unsigned long long> c((size_t)P);
            copy_d2h(c.data(), st[i].pcnt.get() + cofs, (size_t)P * sizeof(unsigned long long), sh.stream);
            for (int q = 0; q < P; ++q) mat[(size_t)sh.index * P + q] = cnt[i][(size_t)q] = (int64_t)c[(size_t)q];
        }
        mat[(size_t)P * P] = dense_fwd;
        allreduce_sum_i64(g, mat.data(), P * P + 1);
        int64_t pairs_all = 0;
        for (int64_t k = 0; k < (int64_t)P * P; ++k) pairs_all += mat[(size_t)k];
        if (2 * pairs_all >= mat[(size_t)P * P]) return false;
        std::vector<const char*> sp(ns);
        std::vector<char*> rp(ns);
        std::vector<std::vector<int64_t>> so(ns), sc(ns), ro(ns), rc(ns);
        for (size_t i = 0; i < ns; ++i) {
            Shard& sh = *g.shards[i];
            DeviceGuard dg(sh);
            St& t = st[i];
            so[i].assign((size_t)P + 1, 0);
            ro[i].assign((size_t)P + 1, 0);
            sc[i].assign((size_t)P, 0);
            rc[i].assign((size_t)P, 0);
            for (int q = 0; q < P; ++q) {
                sc[i][(size_t)q] = cnt[i][(size_t)q];
                rc[i][(size_t)q] = mat[(size_t)q * P + sh.index];
                so[i][(size_t)q + 1] = so[i][(size_t)q] + sc[i][(size_t)q];
                ro[i][(size_t)q + 1] = ro[i][(size_t)q] + rc[i][(size_t)q];
            }
            if ((int64_t)t.spairs.size() < std::max<int64_t>(so[i][(size_t)P], 1)) t.spairs.alloc(std::max<int64_t>(so[i][(size_t)P], 1));
            if ((int64_t)t.rpairs.size() < std::max<int64_t>(ro[i][(size_t)P], 1)) t.rpairs.alloc(std::max<int64_t>(ro[i][(size_t)P], 1));
            copy_h2d(t.pbase.get(), so[i].data(), (size_t)P * sizeof(int64_t), sh.stream);
            copy_h2d(t.roffd.get(), ro[i].data(), ((size_t)P + 1) * sizeof(int64_t), sh.stream);
            JG_HIP(hipMemsetAsync(t.cursor.get(), 0, (size_t)P * sizeof(unsigned long long), sh.stream));
            if (so[i][(size_t)P] > 0) pack(i);
            sp[i] = reinterpret_cast<const char*>(t.spairs.peer());
            rp[i] = reinterpret_cast<char*>(t.rpairs.peer());
        }
        exchange_runs(g, sp, so, sc, rp, ro, rc, sizeof(unsigned long long), ncclUint64);
        for (size_t i = 0; i < ns; ++i) {
            Shard& sh = *g.shards[i];
            DeviceGuard dg(sh);
            if (ro[i][(size_t)P] > 0) recv(i, ro[i][(size_t)P]);
        }
        return true;
    };
    static const bool debug_rounds = std::getenv("JG_DEBUG_CC") != nullptr;
    int64_t own_all = 0;  // own rows with an edge, all shards and ranks
    for (size_t i = 0; i < ns; ++i) own_all += st[i].ne;
    allreduce_sum_i64(g, &own_all, 1);
    int64_t dense_all = dense_fwd;
    allreduce_sum_i64(g, &dense_all, 1);
    int64_t fell = 0;         // own rows whose label fell last round, all shards and ranks
    int rounds = 0, cur = 0;  // dirty[cur]: own rows whose label fell last round
    for (bool any = true; any;) {
        ++rounds;
        const int nxt = cur ^ 1;
        bool fwd_sparse = false;
        // a sparse forward is tried when the rows that fell, at the mean send-list fan-out, would make
        // fewer pairs than half the dense run (the counts then decide; rounds 2-3 of RMAT move most labels)
        const bool try_sparse = rounds > 1 && tune().cc_sparse && P <= kMaxPeersCc &&
                                2.0 * (double)fell * (double)dense_all / (double)std::max<int64_t>(own_all, 1) <
                                    (double)dense_all;
        if (try_sparse) {
            for (size_t i = 0; i < ns; ++i) {
                Shard& sh = *g.shards[i];
                DeviceGuard dg(sh);
                St& t = st[i];
                JG_HIP(hipMemsetAsync(t.pcnt.get(), 0, 2 * (size_t)P * sizeof(unsigned long long), sh.stream));
                if (t.nsend) {
                    cc_fwd_count_kernel<<<grid_for(t.nsend), kBlock, 0, sh.stream>>>(
                        sh.halo_both.send_src.get(), t.send_off.get(), P, t.dirty[cur].get(), t.pcnt.get());
                    JG_LAUNCH_CHECK();
                }
                bytes += 4.0 * (double)t.nsend;  // send_src (the dirty bits are 1/32 of it)
            }
            fwd_sparse = sparse_step(
                0,
                [&](size_t i) {
                    Shard& sh = *g.shards[i];
                    St& t = st[i];
                    cc_fwd_pack_kernel<<<grid_for(t.nsend), kBlock, 0, sh.stream>>>(
                        sh.halo_both.send_src.get(), t.send_off.get(), P, t.dirty[cur].get(), t.label.get(), t.pbase.get(),
                        t.cursor.get(), t.spairs.get());
                    JG_LAUNCH_CHECK();
                },
                [&](size_t i, int64_t n) {
                    Shard& sh = *g.shards[i];
                    St& t = st[i];
                    cc_fwd_recv_kernel<<<grid_for(n), kBlock, 0, sh.stream>>>(t.rpairs.get(), t.roffd.get(), P, sh.index,
                                                                             sh.halo_both.tbits, sh.cc_msg[1].get(),
                                                                             sh.cc_msg[0].get(), t.tmin.get(), t.rootb.get());
                    JG_LAUNCH_CHECK();
                    bytes += 24.0 * (double)n;  // pair, parent, msg, tmin
                });
        }
        if (!fwd_sparse) {
            for (size_t i = 0; i < ns; ++i) {  // own labels into the message vector's own part
                Shard& sh = *g.shards[i];
                DeviceGuard dg(sh);
                if (st[i].ne)
                    JG_HIP(hipMemcpyAsync(sh.cc_msg[0].get(), st[i].label.get(), st[i].ne * sizeof(int32_t),
                                          hipMemcpyDeviceToDevice, sh.stream));
            }
            exchange_msg(g, 0);
        }
        for (size_t i = 0; i < ns; ++i) {
            Shard& sh = *g.shards[i];
            DeviceGuard dg(sh);
            St& t = st[i];
            JG_HIP(hipMemsetAsync(sh.cc_changed.get(), 0, sizeof(int32_t), sh.stream));
            JG_HIP(hipMemsetAsync(t.dirty[nxt].get(), 0, t.dirty[nxt].bytes(), sh.stream));
            JG_HIP(hipMemsetAsync(t.nchg.get(), 0, t.nchg.bytes(), sh.stream));
            if (!fwd_sparse) JG_HIP(hipMemsetAsync(t.pcnt.get(), 0, 2 * (size_t)P * sizeof(unsigned long long), sh.stream));
            if (t.ne == 0) continue;
            const unsigned grid = grid_for(t.sm.total);
            if (fwd_sparse) {
                cc_own_tree_min_kernel<<<grid_for(t.ne), kBlock, 0, sh.stream>>>(t.dirty[cur].get(), t.ne, t.label.get(),
                                                                                 sh.cc_msg[1].get(), t.tmin.get(),
                                                                                 t.rootb.get());
                JG_LAUNCH_CHECK();
                cc_apply_sparse_kernel<<<grid, kBlock, 0, sh.stream>>>(
                    t.sm, sh.cc_msg[1].get(), t.tmin.get(), t.rootb.get(), t.label.get(), sh.cc_msg[0].get(),
                    t.dirty[nxt].get(), t.cb.get(), sh.index, P, sh.halo_both.tbits, t.pcnt.get() + P, sh.cc_changed.get(),
                    t.nchg.get());
                JG_LAUNCH_CHECK();
                // dirty bits of own rows, parent + root bit per slot (the applied slots' tmin and values are few)
                bytes += (double)t.ne / 8.0 + 4.5 * (double)t.sm.total;
                continue;
            }
            if (rounds == 1) {
                cc_tree_init_kernel<<<grid, kBlock, 0, sh.stream>>>(t.sm, t.label.get(), sh.cc_msg[0].get(), t.tmin.get());
                JG_LAUNCH_CHECK();
            }
            cc_tree_min_kernel<<<red_grid(t.sm.total), kRedThreads, 0, sh.stream>>>(
                t.sm, sh.cc_msg[1].get(), t.label.get(), sh.cc_msg[0].get(), t.giant, t.tmin.get());
            JG_LAUNCH_CHECK();
            cc_tree_apply_kernel<<<grid, kBlock, 0, sh.stream>>>(t.sm, sh.cc_msg[1].get(), t.tmin.get(), t.label.get(),
                                                                 sh.cc_msg[0].get(), sh.cc_changed.get(), t.dirty[nxt].get(),
                                                                 t.nchg.get());
            JG_LAUNCH_CHECK();
            // per slot: init 8 B (round 1), tree minima 8 B (parent, label; the atomics of non-root
            // members), apply 12 B
            bytes += (rounds == 1 ? 28.0 : 20.0) * (double)t.sm.total;
        }
        // reverse: after a sparse apply only the marked copies moved (pairs, unless dense is cheaper);
        // after a dense one every copy holds its tree's minimum (the whole run)
        bool rev_sparse = false;
        if (fwd_sparse)
            rev_sparse = sparse_step(
                P,
                [&](size_t i) {
                    Shard& sh = *g.shards[i];
                    St& t = st[i];
                    if (t.sm.total > t.ne) {
                        cc_rev_pack_kernel<<<grid_for(t.sm.total - t.ne), kBlock, 0, sh.stream>>>(
                            t.sm, t.cb.get(), sh.cc_msg[0].get(), sh.index, P, sh.halo_both.tbits, t.pbase.get(),
                            t.cursor.get(), t.spairs.get());
                        JG_LAUNCH_CHECK();
                    }
                },
                [&](size_t i, int64_t n) {
                    Shard& sh = *g.shards[i];
                    St& t = st[i];
                    cc_rev_recv_kernel<<<grid_for(n), kBlock, 0, sh.stream>>>(t.rpairs.get(), t.roffd.get(), P,
                                                                             sh.halo_both.send_src.get(), t.send_off.get(),
                                                                             t.label.get(), t.dirty[nxt].get(),
                                                                             sh.cc_changed.get(), t.nchg.get());
                    JG_LAUNCH_CHECK();
                    bytes += 20.0 * (double)n;  // pair, send_src, label
                });
        if (!rev_sparse) {
            exchange_halo_reverse(g, JG_ADJ_BOTH, mv, rv, sizeof(int32_t), ncclInt32);
            for (size_t i = 0; i < ns; ++i) {
                Shard& sh = *g.shards[i];
                DeviceGuard dg(sh);
                St& t = st[i];
                if (t.nsend) {
                    cc_reverse_apply_kernel<<<grid_for(t.nsend), kBlock, 0, sh.stream>>>(
                        t.rbuf.get(), sh.halo_both.send_src.get(), t.nsend, t.label.get(), sh.cc_changed.get(),
                        t.dirty[nxt].get(), t.nchg.get());
                    JG_LAUNCH_CHECK();
                }
                bytes += 12.0 * (double)t.nsend;  // reverse apply per send-list element
            }
        }
        if (fwd_sparse)
            for (size_t i = 0; i < ns; ++i) {  // the marks of this round's sparse apply
                Shard& sh = *g.shards[i];
                DeviceGuard dg(sh);
                JG_HIP(hipMemsetAsync(st[i].rootb.get(), 0, st[i].rootb.bytes(), sh.stream));
                JG_HIP(hipMemsetAsync(st[i].cb.get(), 0, st[i].cb.bytes(), sh.stream));
            }
        if (debug_rounds) {
            for (size_t i = 0; i < ns; ++i) {
                Shard& sh = *g.shards[i];
                DeviceGuard dg(sh);
                std::vector<unsigned long long> c(2 * (size_t)P, 0);
                copy_d2h(c.data(), st[i].pcnt.get(), c.size() * sizeof(unsigned long long), sh.stream);
                unsigned long long f = 0, rv2 = 0;
                for (int q = 0; q < P; ++q) f += c[(size_t)q], rv2 += c[(size_t)P + q];
                std::fprintf(stderr, "[jg cc] round %d shard %d: forward %s %llu pairs, reverse %s %llu pairs (rows fell "
                             "last round, all shards: %lld)\n", rounds, sh.index, fwd_sparse ? "sparse" : "dense", f,
                             rev_sparse ? "sparse" : "dense", rv2, (long long)fell);
            }
        }
        fell = 0;  // (cc_changed is set exactly when a shard's count is non-zero)
        for (size_t i = 0; i < ns; ++i) {
            Shard& sh = *g.shards[i];
            DeviceGuard dg(sh);
            std::vector<unsigned long long> c((size_t)kFellLines * kFellStride);
            copy_d2h(c.data(), st[i].nchg.get(), c.size() * sizeof(unsigned long long), sh.stream);
            for (int k = 0; k < kFellLines; ++k) fell += (int64_t)c[(size_t)k * kFellStride];
        }
        allreduce_sum_i64(g, &fell, 1);
        any = fell > 0;
        cur = nxt;
    }
    // the superstep count: one BFS from every component's minimum-rank vertex
    std::vector<CcRoots> roots(ns);
    for (size_t i = 0; i < ns; ++i) roots[i] = CcRoots{st[i].label.peer(), st[i].rank.peer(), nullptr, st[i].ne};  // (used under shard i)
    double reached = 0;
    const int d = cc_root_eccentricity_sharded(g, roots.data(), &reached);
    const int it = d + 1;  // 0 when no vertex has an edge (d = -1)
    *rounds_out = rounds;
    static const bool debug = std::getenv("JG_DEBUG_CC") != nullptr;
    unsigned long long lk = 0;
    for (size_t i = 0; i < ns; ++i) {
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        St& t = st[i];
        unsigned long long l = 0;
        copy_d2h(&l, t.linked.get(), sizeof l, sh.stream);
        lk += l;
        if (debug)
            std::fprintf(stderr, "[jg cc] shard %d: rows %lld with edges %lld, vector %lld, entries %lld, giant root %d "
                         "(%d of 1024 sampled), all peers found %d, rest entries scanned %llu; %d label rounds, "
                         "%d supersteps\n",
                         sh.index, (long long)sh.rows, (long long)t.ne, (long long)t.len, (long long)sh.both.nnz,
                         t.giant, t.giant_share, t.all_found, l, rounds, it);
        // per slot: init 4 B, two compressions 16 B; flags 1 bit per vector position; per row with an
        // edge: first links 20 B, BFS start 17 B, depth and frontier probe 5 B
        bytes += 20.0 * (double)t.sm.total + (double)t.len / 8.0 + 42.0 * (double)t.ne;
        if (it <= kCcMaxIterations - 1 && sh.rows)
            JG_HIP(hipMemcpyAsync(sh.cc_label.get(), t.label.get(), sh.rows * sizeof(int32_t), hipMemcpyDeviceToDevice,
                                  sh.stream));
        JG_HIP(hipStreamSynchronize(sh.stream));
    }
    if (it > kCcMaxIterations - 1) return false;
    // 12 B per entry linked (col, both finds), 4 B per adjacency entry of the rows the BFS reached
    *work_bytes = bytes + 12.0 * (double)lk + 4.0 * reached;
    *iterations = it;
    return true;
}

}  // namespace

// The String-order rank of every vertex id, computed once per snapshot (build_graph_from_dense, graphs
// with the BOTH adjacency; counted in build_ms): it depends on the ids only.  g.cc_vor[r] = id of the
// vertex of rank r (on the first shard's device), sh.cc_rank0[l] = rank of own row l (each shard's
// device).  Negative ids leave them empty; cc_run then fails as before.
void cc_prepare_ranks(Graph& g) {
    const int64_t n = g.n;
    g.cc_ranks = false;
    for (int64_t d = 0; d < (int64_t)g.vid.size(); ++d)
        if (g.vid[d] < 0) return;
    Shard& shr = *g.shards[0];
    DeviceGuard dg(shr.device);  // graph-level arrays (untagged in the virtual-device check)
    hipStream_t s = shr.stream;
    DevBuf<int32_t> rk(std::max<int64_t>(n, 1));
    g.cc_vor.alloc(std::max<int64_t>(n, 1));
    g.cc_vor_host.clear();
    if (n > 0) {
        DevBuf<int64_t> vid(n);
        DevBuf<uint64_t> keys(n);
        DevBuf<uint32_t> vals(n);
        if (g.vid.empty()) {
            iota_i64_kernel<<<grid_for(n), kBlock, 0, s>>>(vid.get(), n);
            JG_LAUNCH_CHECK();
        } else {
            copy_h2d(vid.get(), g.vid.data(), n * sizeof(int64_t), s);
        }
        lex_digits_kernel<<<grid_for(n), kBlock, 0, s>>>(vid.get(), n, keys.get(), vals.get());
        JG_LAUNCH_CHECK();
        prim::radix_sort(keys.get(), vals.get(), n, 5, s);
        lex_padded_kernel<<<grid_for(n), kBlock, 0, s>>>(vid.get(), vals.get(), n, keys.get());
        JG_LAUNCH_CHECK();
        prim::radix_sort(keys.get(), vals.get(), n, 64, s);
        lex_rank_scatter_kernel<<<grid_for(n), kBlock, 0, s>>>(vals.get(), n, rk.get());
        JG_LAUNCH_CHECK();
        vid_of_rank_kernel<<<grid_for(n), kBlock, 0, s>>>(vals.get(), vid.get(), n, g.cc_vor.get());
        JG_LAUNCH_CHECK();
    }
    std::vector<int32_t> rank_of;  // host copy, for shards on other devices
    for (auto& sp : g.shards) {
        Shard& sh = *sp;
        {
            // on the shard's own device (found by the virtual-device check: round 4 allocated every shard's
            // ranks on the first device, where shards on other devices would have read them across xGMI)
            DeviceGuard dgs(sh);
            sh.cc_rank0.alloc(std::max<int64_t>(sh.rows, 1));
        }
        if (!sh.rows) continue;
        if (same_device(sh, shr.device)) {  // the rows' ranks, gathered on the device
            gather_i32_kernel<<<grid_for(sh.rows), kBlock, 0, s>>>(rk.get(), sh.dense_rows.get(), sh.rows,
                                                                   sh.cc_rank0.get());
            JG_LAUNCH_CHECK();
            continue;
        }
        if (rank_of.empty()) {
            rank_of.resize((size_t)n);
            copy_d2h(rank_of.data(), rk.get(), n * sizeof(int32_t), s);
        }
        std::vector<int32_t> lab0((size_t)sh.rows);
        const std::vector<int32_t>& dl = sh.dense_of_local();
        for (int64_t l = 0; l < sh.rows; ++l) lab0[(size_t)l] = rank_of[(size_t)dl[(size_t)l]];
        DeviceGuard dgs(sh);
        copy_h2d(sh.cc_rank0.get(), lab0.data(), sh.rows * sizeof(int32_t), sh.stream);
        JG_HIP(hipStreamSynchronize(sh.stream));
    }
    JG_HIP(hipStreamSynchronize(s));
    g.cc_ranks = true;
}

namespace {
// Superstep 0 of the propagation: labels = ranks, only vertices with an edge send (every shard), then
// the exchange step.
void cc_propagation_init(Graph& g) {
    for (auto& sp : g.shards) {
        Shard& sh = *sp;
        DeviceGuard dg(sh);
        for (auto& m : sh.cc_msg) JG_HIP(hipMemsetAsync(m.get(), 0x7F, m.bytes(), sh.stream));  // ~INT_MAX
        if (sh.rows) {
            cc_init_kernel<<<grid_for(sh.rows), kBlock, 0, sh.stream>>>(sh.cc_rank0.get(), sh.both.row_ptr.get(), sh.rows,
                                                                        g.vec_pos(sh, JG_ADJ_BOTH), sh.cc_label.get(),
                                                                        sh.cc_msg[0].get());
            JG_LAUNCH_CHECK();
        }
    }
    exchange_msg(g, 0);
}
}  // namespace

void cc_run(Graph& g, int64_t* comp_out, int32_t* iterations_out) {
    if (!(g.flags & JG_ADJ_BOTH)) fail(JG_ERR_UNSUPPORTED, "connected components need a graph built with JG_ADJ_BOTH");
    Ctx& ctx = *g.ctx;
    ctx.last = jg_stats{};
    const int64_t n = g.n;
    if (!g.cc_ranks) fail(JG_ERR_UNSUPPORTED, "connected components need non-negative vertex ids");
    // One shard keeps everything on its device (the labels become ids in caller order there); sharded
    // graphs map the labels on the host.
    Shard& sh0 = *g.shards[0];
    const bool dev_maps = g.shards.size() == 1 && sh0.rows == n;
    // buffers of the call (allocation only: every kernel of the call runs inside the timed region)
    for (auto& sp : g.shards) {
        Shard& sh = *sp;
        DeviceGuard dg(sh);
        const int64_t len = g.vec_len(sh, JG_ADJ_BOTH);
        for (int k = 0; k < 2; ++k)
            if (sh.cc_msg[k].size() != (size_t)len) sh.cc_msg[k].alloc(len);
        if ((int64_t)sh.cc_label.size() < std::max<int64_t>(sh.rows, 1)) sh.cc_label.alloc(std::max<int64_t>(sh.rows, 1));
        if ((int64_t)sh.cc_hub_partial.size() < std::max<int64_t>(sh.plan_both.num_chunks, 1))
            sh.cc_hub_partial.alloc(std::max<int64_t>(sh.plan_both.num_chunks, 1));
        if ((int64_t)sh.cc_split_partial.size() < sh.plan_both.split_partial_len())
            sh.cc_split_partial.alloc(sh.plan_both.split_partial_len());
        if (sh.cc_changed.size() == 0) sh.cc_changed.alloc(1);
    }
    // superstep 0 votes: anyone with an edge sent
    int any = 0;
    for (auto& sp : g.shards) any |= sp->both.nnz > 0;
    any = allreduce_or(g, any);

    DeviceGuard dg0(sh0.device);
    hipEvent_t t0, t1;
    JG_HIP(hipEventCreate(&t0));
    JG_HIP(hipEventCreate(&t1));
    const bool uf_one = g.shards.size() == 1 && g.P == 1 && tune().cc_uf;
    if (uf_one && sh0.rows > 0) {  // the union-find path's scratch
        if ((int64_t)sh0.cc_depth.size() < sh0.rows) sh0.cc_depth.alloc(sh0.rows);
        bfs_buffers(sh0);
        bfs_first_col(sh0, sh0.both);
    }
    if (!uf_one && g.P > 1)  // the sharded union-find's first round reads each row's first column
        for (auto& sp : g.shards)
            if (sp->both.present()) bfs_first_col(*sp, sp->both);
    for (auto& sp : g.shards) JG_HIP(hipStreamSynchronize(sp->stream));
    prof_discard_exchanges(g);  // exchange pairs count from t0 on only
    region_mark(sh0.stream, true);
    JG_HIP(hipEventRecord(t0, sh0.stream));
    int iteration = 0, cur = 0;
    // one shard: supersteps whose senders have few edges run push-style
    const bool push_ok = g.shards.size() == 1 && g.P == 1 && tune().cc_push;
    struct Push {
        DevBuf<int32_t> queue, touched;
        DevBuf<int64_t> qoff, touched_off;
        DevBuf<unsigned long long> ctr;
    } pu;
    if (push_ok) {
        const size_t r1 = (size_t)std::max<int64_t>(sh0.rows, 1);
        pu.queue.alloc(r1);
        pu.touched.alloc(r1);
        pu.qoff.alloc(r1);
        pu.touched_off.alloc(r1);
        pu.ctr.alloc(2);
    }
    // One shard: the same labels and superstep count from a union-find and one BFS (cc_union_find).
    bool solved = false;
    const int32_t* uf_labels = nullptr;  // the union-find's labels of shard 0 (when solved)
    int64_t uf_label_rows = sh0.rows;      // its rows from here on take their rank (cc_union_find)
    double uf_bytes = 0;
    // One shard: the caller-order ids are made on the device inside the timed region (VERDICT r05 item 4:
    // the edgeless rows' labels and the output are work the caller needs; only the copy to the host is
    // outside).  Sharded graphs assemble them on the host below.
    DevBuf<int64_t> out;
    DevBuf<unsigned long long> giant_bits;
    const bool dev_out = comp_out && dev_maps && n > 0;
    bool out_done = false;
    const std::function<void(const int32_t*, int64_t)> emit_output = [&](const int32_t* lab, int64_t lrows) {
        Shard& sh = *g.shards[0];  // comp[d] = id of rank label[local of d]
        DeviceGuard dg(sh);
        if (!out.size()) out.alloc(n);
        // the giant component's label: row 0's (the highest-degree row; any row would be correct)
        if (giant_bits.size() < (size_t)std::max<int64_t>((lrows + 63) / 64, 1))
            giant_bits.alloc(std::max<int64_t>((lrows + 63) / 64, 1));
        if (lrows > 0) {
            cc_giant_bits_kernel<<<grid_for((lrows + 3) / 4), kBlock, 0, sh.stream>>>(lab, lrows, lab, giant_bits.get());
            JG_LAUNCH_CHECK();
        }
        cc_output_kernel<<<grid_for((n + kCcOutRun - 1) / kCcOutRun, kBlock, 8192), kBlock, 0, sh.stream>>>(
            lab, sh.cc_rank0.get(), lrows, g.padded_dev.get(), g.cc_vor.get(), n, out.get(), giant_bits.get(),
            lrows > 0 ? lab : sh.cc_rank0.get(), g.vid.empty() ? 1 : 0);
        JG_LAUNCH_CHECK();
        out_done = true;
    };
    if (uf_one)
        solved = cc_union_find(ctx, sh0, &iteration, &uf_labels, &uf_label_rows, &uf_bytes, dev_out ? &emit_output : nullptr,
                               dev_out ? t1 : nullptr);
    // Sharded over halo plans: the same from local union-finds, tree labels over the halo and a sharded BFS
    // (cc_union_find_sharded); the sharded BFS takes at most 64 shards (jg_traverse.hip, kMaxShardsBfs).
    int uf_rounds = 0;
    if (!solved && !uf_one && g.P > 1 && g.P <= 64 && sh0.halo_both.on && tune().cc_uf && tune().cc_uf_sharded) {
        solved = cc_union_find_sharded(g, &iteration, &uf_rounds, &uf_bytes);
        if (solved) uf_labels = sh0.cc_label.get();
    }
    // the propagation (no union-find path, or the 99-superstep cap binds): from superstep 0
    if (!solved) {
        iteration = 0;
        cc_propagation_init(g);
    }
    while (!solved && any && iteration < kCcMaxIterations - 1) {
        ++iteration;
        bool pushed = false;
        if (push_ok) {
            Shard& sh = sh0;
            JG_HIP(hipMemsetAsync(pu.ctr.get(), 0, 2 * sizeof(unsigned long long), sh.stream));
            cc_senders_kernel<<<grid_for(sh.rows), kBlock, 0, sh.stream>>>(sh.cc_msg[cur].get(), sh.rows,
                                                                           sh.both.row_ptr.get(), pu.queue.get(),
                                                                           pu.qoff.get(), pu.ctr.get());
            JG_LAUNCH_CHECK();
            unsigned long long h = 0;
            copy_d2h(&h, pu.ctr.get(), sizeof h, sh.stream);
            const int64_t nq = (int64_t)(h >> kPackShift), mf = (int64_t)(h & kEdgeMask);
            if ((double)mf < (double)sh.both.nnz / (double)tune().bfs_alpha) {
                pushed = true;
                JG_HIP(hipMemsetAsync(sh.cc_changed.get(), 0, sizeof(int32_t), sh.stream));
                JG_HIP(hipMemsetAsync(sh.cc_msg[cur ^ 1].get(), 0x7F, sh.cc_msg[cur ^ 1].bytes(), sh.stream));
                if (mf > 0) {
                    CcPush a{pu.queue.get(), pu.qoff.get(), nq, mf, sh.both.row_ptr.get(), sh.both.col.get(),
                             sh.cc_msg[cur].get(), sh.cc_msg[cur ^ 1].get(), pu.touched.get(), pu.touched_off.get(),
                             pu.ctr.get() + 1};
                    cc_push_kernel<<<(unsigned)std::min<int64_t>(std::max<int64_t>((mf / 4 + kBlock - 1) / kBlock, 1),
                                                                  4096),
                                     kBlock, 0, sh.stream>>>(a);
                    JG_LAUNCH_CHECK();
                    copy_d2h(&h, pu.ctr.get() + 1, sizeof h, sh.stream);
                    const int64_t nt = (int64_t)(h >> kPackShift);
                    if (nt > 0) {
                        CcOp op;
                        op.msg = sh.cc_msg[cur].get();
                        op.msg_out = sh.cc_msg[cur ^ 1].get();
                        op.label = sh.cc_label.get();
                        op.changed = sh.cc_changed.get();
                        op.pos = g.vec_pos(sh, JG_ADJ_BOTH);
                        cc_push_apply_kernel<<<grid_for(nt), kBlock, 0, sh.stream>>>(pu.touched.get(), nt, op);
                        JG_LAUNCH_CHECK();
                    }
                }
            }
        }
        if (!pushed)
        for (auto& sp : g.shards) {
            Shard& sh = *sp;
            DeviceGuard dg(sh);
            JG_HIP(hipMemsetAsync(sh.cc_changed.get(), 0, sizeof(int32_t), sh.stream));
            CcOp op;
            op.msg = sh.cc_msg[cur].get();
            op.msg_out = sh.cc_msg[cur ^ 1].get();
            op.label = sh.cc_label.get();
            op.changed = sh.cc_changed.get();
            op.pos = g.vec_pos(sh, JG_ADJ_BOTH);
            launch_pull(sh.both, sh.plan_both, op, sh.cc_hub_partial.get(), sh.stream, ctx.profiling ? &ctx : nullptr,
                        &sh, sh.cc_split_partial.get());
        }
        exchange_msg(g, cur ^ 1);
        any = 0;
        for (auto& sp : g.shards) {
            Shard& sh = *sp;
            DeviceGuard dg(sh);
            int32_t ch = 0;
            JG_HIP(hipMemcpyAsync(&ch, sh.cc_changed.get(), sizeof ch, hipMemcpyDeviceToHost, sh.stream));
            JG_HIP(hipStreamSynchronize(sh.stream));
            any |= ch;
        }
        any = allreduce_or(g, any);
        cur ^= 1;
    }
    // the union-find queued the output behind its BFS start; the other paths (and a union-find that hit
    // the superstep cap, whose output is stale) make it here
    if (dev_out && !(solved && uf_one && out_done))
        emit_output(solved ? uf_labels : g.shards[0]->cc_label.get(), solved ? uf_label_rows : n);
    // with the output queued behind the BFS start, the BFS recorded t1 behind its last level batch (the
    // host's read of the final level state is control, as in the DO-BFS); otherwise it ends here
    if (!(dev_out && solved && uf_one && out_done)) {
        JG_HIP(hipEventRecord(t1, sh0.stream));
        region_mark(sh0.stream, false);
    }
    JG_HIP(hipEventSynchronize(t1));
    float ms = 0;
    JG_HIP(hipEventElapsedTime(&ms, t0, t1));
    JG_HIP(hipEventDestroy(t0));
    JG_HIP(hipEventDestroy(t1));
    ctx.last.compute_ms = ms;
    ctx.last.supersteps = iteration;
    ctx.last.levels = iteration;
    double nnz = 0;
    for (auto& sp : g.shards) nnz += (double)sp->both.nnz;
    ctx.last.edges_traversed = nnz * iteration;
    // the propagation: 16m + 16n per superstep; the union-find: its own pass model
    if (uf_one && solved) {  // the second round's linked entries (12 B each), read now that the region has ended
        unsigned long long rest = 0;
        DeviceGuard dg(sh0);
        copy_d2h(&rest, sh0.cc_linked.get(), sizeof rest, sh0.stream);
        uf_bytes += 12.0 * (double)rest;
    }
    ctx.last.algorithmic_bytes = solved ? uf_bytes : (8.0 * nnz + 16.0 * (double)n) * iteration;
    // the output pass: the giant bits (a 4-byte label read per row with an edge), then per vertex its local
    // index (4 B) and the id stored (8 B); the other rows' label and id gathers are not counted
    if (dev_out) ctx.last.algorithmic_bytes += 12.0 * (double)n + 4.0 * (double)(solved ? uf_label_rows : n);
    if (iterations_out) *iterations_out = iteration;
    if (dev_out) {
        Shard& sh = *g.shards[0];
        DeviceGuard dg(sh);
        copy_d2h(comp_out, out.get(), n * sizeof(int64_t), sh.stream);
    } else if (comp_out) {
        const std::vector<int64_t>& vid_of_rank = g.vid_of_rank();
        for (auto& sp : g.shards) {
            Shard& sh = *sp;
            DeviceGuard dg(sh);
            std::vector<int32_t> h(sh.rows);
            const bool uf = solved && &sh == &sh0;
            const int32_t* lab = uf ? uf_labels : sh.cc_label.get();
            const int64_t lr = uf ? std::min(uf_label_rows, sh.rows) : sh.rows;
            if (lr) copy_d2h(h.data(), lab, lr * sizeof(int32_t), sh.stream);
            if (lr < sh.rows)  // the union-find's edgeless suffix: its ranks
                copy_d2h(h.data() + lr, sh.cc_rank0.get() + lr, (sh.rows - lr) * sizeof(int32_t), sh.stream);
            for (int64_t l = 0; l < sh.rows; ++l) comp_out[sh.dense_of_local()[l]] = vid_of_rank[h[l]];
        }
    }
    prof_collect(ctx, g);
}

}  // namespace jg
