// jg_traverse.hip — hop-depth traversals and hop-bounded shortest distance.
//
// Reference semantics:
//   SPVP depth (TinkerPop ShortestPathVertexProgram under Fulgora's forced {Local(bothE), Global}
//   scopes, janusgraph-core/.../olap/computer/FulgoraGraphComputer.java:249-253): undirected hops.
//   ShortestDistanceVertexProgram (janusgraph-backend-testutils/.../olap/
//   ShortestDistanceVertexProgram.java:112-146, combiner ShortestDistanceMessageCombiner.java:29-31):
//   v pulls over its OUT edges the targets' previous-superstep messages + edge weight, keeps the
//   minimum, forwards on improvement; supersteps 0..maxDepth => min over paths of <= maxDepth hops.
//
// Kernels:
//   single source, 1 shard: direction-optimising BFS (Beamer), one kernel per level that picks its
//     direction on the device from the counters of the previous level (no host round trip per
//     level).  Top-down is edge-parallel over the frontier's edges, claims targets with atomicCAS
//     and appends them through one wave-ballot + one packed atomicAdd per wave; bottom-up gives
//     each unvisited vertex one lane that scans its pull adjacency against a 64-bit-word frontier
//     bitmap and stops at the first hit; the next bitmap word is the wave's ballot (no atomics).
//   multi-source (<= 64) or sharded: bit-parallel BFS, one uint64 frontier word per vertex, as an
//     OR-semiring pull superstep on the jg_pull.h engine, exchanged by allgather.
//   weighted SD: frontier Bellman-Ford with exact snapshot semantics (messages of superstep t-1
//     only): push over the in-CSR with 64-bit atomicMin into a scratch array, then apply.
#include <climits>
#include <initializer_list>
#include <type_traits>

#include <cstdio>

#include "jg_frontier.h"
#include "jg_pull.h"
#include "jg_scatter.h"

namespace jg {

namespace {

constexpr int kTdEdgesPerThread = 4;
constexpr int kBuBatch = 4;             // bottom-up: neighbours probed per step
constexpr int kBfsRing = 4;            // level-state ring: a level touches slots L-1, L, L+1

__device__ __forceinline__ void wave_append(bool take, int32_t v, int32_t* __restrict__ queue,
                                            unsigned long long* __restrict__ size) {
    const uint64_t mask = __ballot(take);
    if (mask == 0) return;
    const int leader = __ffsll((unsigned long long)mask) - 1;
    unsigned long long base = 0;
    if (lane_id() == leader) base = atomicAdd(size, (unsigned long long)__popcll(mask));
    base = __shfl(base, leader, kWave);
    if (take) queue[base + __popcll(mask & lanemask_lt())] = v;
}

// Append v (push degree deg) to a frontier queue whose entries also carry their first edge offset.
// One packed 64-bit atomicAdd per wave reserves both the queue slots and the edge range, so queue
// positions and edge offsets grow together (the offsets are monotone: top-down binary-searches them).
// Must be reached by all 64 lanes (wave-uniform call sites).
__device__ __forceinline__ void wave_append_frontier(bool take, int32_t v, int64_t deg, int32_t* __restrict__ queue,
                                                     int64_t* __restrict__ qoff,
                                                     unsigned long long* __restrict__ packed) {
    const uint64_t mask = __ballot(take);
    if (mask == 0) return;
    const int64_t d = take ? deg : 0;
    const int64_t dinc = wave_inclusive_scan_add(d);
    const int64_t dtot = __shfl(dinc, kWave - 1, kWave);
    const int leader = __ffsll((unsigned long long)mask) - 1;
    unsigned long long base = 0;
    if (lane_id() == leader)
        base = atomicAdd(packed, ((unsigned long long)__popcll(mask) << kPackShift) | (unsigned long long)dtot);
    base = __shfl(base, leader, kWave);
    if (take) {
        const uint64_t pos = (base >> kPackShift) + (uint64_t)__popcll(mask & lanemask_lt());
        queue[pos] = v;
        qoff[pos] = (int64_t)(base & kEdgeMask) + dinc - d;
    }
}

// Per-level device state of the single-source DO-BFS.  Level L's kernel derives its direction from
// the state and frontier counter level L-1 left behind, so the host enqueues levels in batches and
// reads the state back once per batch instead of once per level.
struct BfsState {
    long long mu;     // push edges not yet in any frontier (after this level's input frontier)
    long long edges;  // push degree summed over every frontier so far = edges of reached vertices
    int bottom_up;    // direction this level ran in
    int done;         // traversal finished: this level and all later ones do nothing
    int levels;       // levels run (valid once done)
    int pad;
};

struct BfsLevel {
    const int64_t* push_rp;  // null when there is no push adjacency
    const int32_t* push_col;
    const int64_t* pull_rp;  // null when there is no pull adjacency
    const int32_t* pull_col;
    const int32_t* pull_first;  // [rows] each pull row's first column, -1 when empty (Csr::first_col)
    const int64_t* deg_rp;   // push_rp, else pull_rp (frontier edge counts)
    int32_t* depth;
    int64_t rows;
    int64_t bu_rows;  // the bottom-up probes rows [0, bu_rows): the pull adjacency's empty suffix is never found
    const int32_t* queue_in;
    const int64_t* qoff_in;
    int32_t* queue_out;
    int64_t* qoff_out;
    const unsigned long long* bm_in;
    unsigned long long* bm_out;
    uint8_t* seen;  // seen[v] != 0: depth[v] is set (a 64 MB byte map at 2^26 vertices stays in the
                    // Infinity Cache where the 268 MB depth array does not; bytes need no atomics)
    int32_t* owner;           // [rows] split top-down levels (kTdOwner / kTdClaim)
    long long split_min, split_max;  // split: frontier entries for which the level is split (max < 2^31)
    int split;                // this launch is followed by bfs_td_claim_kernel
    unsigned long long* ctr;  // [kBfsRing] packed frontier counters, slot = level % kBfsRing
    BfsState* st;             // [kBfsRing]
    int level, max_depth;
    double alpha, beta;
};

// Direction choice (Beamer et al.): go bottom-up when the frontier's edges outweigh the unexplored
// edges / alpha, back top-down when the frontier shrinks below rows / beta.
__device__ BfsState bfs_decide(const BfsLevel& a, int64_t* nf_out, int64_t* mf_out, bool* switch_in) {
    const int pl = (a.level + kBfsRing - 1) % kBfsRing;
    const BfsState p = a.st[pl];
    const unsigned long long h = a.ctr[pl];
    BfsState c = p;
    *switch_in = false;
    *nf_out = *mf_out = 0;
    if (p.done) return c;
    const int64_t nf = (int64_t)(h >> kPackShift), mf = (int64_t)(h & kEdgeMask);
    *nf_out = nf;
    *mf_out = mf;
    c.mu = p.mu - mf;
    c.edges = p.edges + mf;
    if (nf == 0 || (a.max_depth >= 0 && a.level >= a.max_depth)) {
        c.done = 1;
        c.levels = a.level;
        return c;
    }
    // (Beamer's growth condition, bottom-up only while the frontier grows, measured RMAT-26 -0.6% and
    // RMAT-20 +2.5%, round 2: not used)
    if (!p.bottom_up && a.pull_rp && (!a.push_rp || (double)mf > (double)c.mu / a.alpha)) {
        c.bottom_up = 1;
        *switch_in = true;  // the previous frontier exists only as a queue: test depth == level instead
    } else if (p.bottom_up && a.push_rp && (double)nf < (double)a.rows / a.beta) {
        c.bottom_up = 0;  // the queue is always valid: both directions append to it
    }
    return c;
}

// Edge-parallel top-down: frontier edge e in [0, mf) belongs to the queue entry i with
// qoff[i] <= e < qoff[i+1]; each thread takes `ept` consecutive edges after one binary search (one
// edge per thread while the frontier's edges fit the grid, kTdEdgesPerThread beyond), so a hub in
// the frontier is spread over the whole grid.  A thread's edges are processed in phases (all target
// loads, then all depth probes and claims, then the degree loads) so its dependent memory round trips
// do not multiply with the edges it holds; one block-wide append per edge slot follows.
// Claims (kMode): kTdCas one CAS on the target's depth per entry; a split level runs kTdOwner (every
// entry whose target is unvisited stores its index in owner[target], a plain store) and, in a second
// launch, kTdClaim (the entry whose index survived claims the target).  Device-scope CAS runs at the
// memory side, so the ~100 entries of one level that reach the same hub target queue behind each other
// (RMAT-20 level 1: 329 K entries, 107 K targets, 64 us); plain stores to one address do not.
enum TdMode { kTdCas = 0, kTdOwner = 1, kTdClaim = 2 };

// Queue-entry search of the edge-parallel top-down: every stride-th edge offset of the input queue
// (stride = ceil(nf / kQoffSamples)) is staged in LDS by each block with work, the
// search runs there and then over at most `qs` global offsets.  The offsets were appended by every XCD
// in the previous launch, so each global probe misses the reading XCD's L2: a 22.6 K-entry queue cost
// 15 dependent probes (RMAT-20 level 4, a 24.9 K-entry top-down level: 12.4 us).
constexpr int kQoffSamples = 1024;
struct QoffIndex {
    const int64_t* lds;  // samples: lds[j] = qoff_in[j * stride]
    int64_t stride, count;
};
__device__ __forceinline__ QoffIndex stage_qoff(const BfsLevel& a, int64_t nf, int64_t mf, int ept, int64_t* s_qs) {
    QoffIndex q{s_qs, (nf + kQoffSamples - 1) / kQoffSamples, 0};
    q.count = (nf + q.stride - 1) / q.stride;
    if ((int64_t)blockIdx.x * blockDim.x * ept < mf)  // block-uniform: blocks past the frontier's edges skip it
        for (int64_t j = threadIdx.x; j < q.count; j += blockDim.x) s_qs[j] = a.qoff_in[j * q.stride];
    __syncthreads();
    return q;
}
// the queue entry i with qoff_in[i] <= e < qoff_in[i + 1] (offsets are monotone; zero-degree entries
// share their successor's offset and the search returns the last of them)
__device__ __forceinline__ int64_t find_entry(const BfsLevel& a, const QoffIndex& q, int64_t nf, int64_t e) {
    int64_t lo = 0, hi = q.count - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (q.lds[mid] <= e) lo = mid; else hi = mid - 1;
    }
    int64_t g0 = lo * q.stride, g1 = std::min(g0 + q.stride, nf) - 1;
    while (g0 < g1) {
        const int64_t mid = (g0 + g1 + 1) >> 1;
        if (a.qoff_in[mid] <= e) g0 = mid; else g1 = mid - 1;
    }
    return g0;
}

template <int kMode, class App>
__device__ __forceinline__ void bfs_top_down(const BfsLevel& a, int64_t nf, int64_t mf, unsigned long long* packed,
                                             App& app, int64_t* s_qs) {
    const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int ept = mf <= nthreads ? 1 : kTdEdgesPerThread;  // grid-uniform
    const int64_t per_tile = nthreads * ept;
    const int64_t tiles = (mf + per_tile - 1) / per_tile;  // wave-uniform
    const int32_t next_depth = a.level + 1;
    const QoffIndex qi = stage_qoff(a, nf, mf, ept, s_qs);
    for (int64_t t = 0; t < tiles; ++t) {
        // a block (a wave, with wave-staged appends) whose slice of this tile is past the frontier's
        // edges has nothing to claim or append (small frontiers leave most of the grid idle)
        if ((t * nthreads + (int64_t)blockIdx.x * blockDim.x + (App::kWaveUniform ? wave_id() * kWave : 0)) * ept >= mf)
            break;
        const int64_t e0 = (t * nthreads + tid) * ept;
        int32_t v[kTdEdgesPerThread];
        bool have[kTdEdgesPerThread], won[kTdEdgesPerThread];
        int64_t vdeg[kTdEdgesPerThread];
        if (e0 < mf) {
            int64_t i = find_entry(a, qi, nf, e0);
            int64_t next_bound = i + 1 < nf ? a.qoff_in[i + 1] : mf;
#pragma unroll
            for (int k = 0; k < kTdEdgesPerThread; ++k) {
                const int64_t e = e0 + k;
                have[k] = k < ept && e < mf;
                v[k] = 0;
                if (have[k]) {
                    while (e >= next_bound) {  // skips zero-degree frontier entries too
                        ++i;
                        next_bound = i + 1 < nf ? a.qoff_in[i + 1] : mf;
                    }
                    const int32_t u = a.queue_in[i];
                    v[k] = a.push_col[a.push_rp[u] + (e - a.qoff_in[i])];
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < kTdEdgesPerThread; ++k) have[k] = false, v[k] = 0;
        }
        uint8_t sv[kTdEdgesPerThread];
#pragma unroll
        for (int k = 0; k < kTdEdgesPerThread; ++k) sv[k] = have[k] ? a.seen[v[k]] : 1;
        if constexpr (kMode == kTdOwner) {
#pragma unroll
            for (int k = 0; k < kTdEdgesPerThread; ++k)
                if (!sv[k]) a.owner[v[k]] = (int32_t)(e0 + k);  // td_split: mf < 2^31
            continue;
        }
        if constexpr (kMode == kTdClaim) {
            // the seen bytes are the ones the owner pass read: only the claiming entry changes them
            int32_t ow[kTdEdgesPerThread];
#pragma unroll
            for (int k = 0; k < kTdEdgesPerThread; ++k) ow[k] = sv[k] ? -1 : a.owner[v[k]];
#pragma unroll
            for (int k = 0; k < kTdEdgesPerThread; ++k) {
                won[k] = !sv[k] && ow[k] == (int32_t)(e0 + k);
                if (won[k]) {
                    a.depth[v[k]] = next_depth;
                    a.seen[v[k]] = 1;
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < kTdEdgesPerThread; ++k) {
                // the byte map filters; the CAS on depth decides (a stale byte only costs a failed CAS)
                won[k] = !sv[k] && atomicCAS(&a.depth[v[k]], -1, next_depth) == -1;
                if (won[k]) a.seen[v[k]] = 1;
            }
        }
#pragma unroll
        for (int k = 0; k < kTdEdgesPerThread; ++k) vdeg[k] = won[k] ? a.deg_rp[v[k] + 1] - a.deg_rp[v[k]] : 0;
        for (int k = 0; k < ept; ++k) app.append(won[k], v[k], vdeg[k], a.queue_out, a.qoff_out, packed);
    }
}

// Bottom-up: one lane per unvisited vertex scans its pull row against the frontier and stops at the
// first hit; 64 consecutive vertices per wave so the next frontier word is the wave's ballot.
template <bool kFromDepth, class App>
__device__ __forceinline__ void bfs_bottom_up(const BfsLevel& a, unsigned long long* packed, App& app) {
    // every word of the output bitmap is written (a word past bu_rows comes out zero: a stale bit there
    // would put a row in the next level's frontier); rows from bu_rows on read nothing
    const int64_t words = (a.rows + 63) / 64;
    constexpr int kWpb = kBlock / kWave;
    const int64_t wstride = (int64_t)gridDim.x * kWpb;
    const int32_t next_depth = a.level + 1;
    // block-uniform trip count when the append is block-wide (words past the end take nothing);
    // wave-staged appends let every wave run its own words
    const int64_t wv0 = App::kWaveUniform ? wave_id() : 0;
    for (int64_t w0 = (int64_t)blockIdx.x * kWpb + wv0; w0 < words; w0 += wstride) {
        const int64_t w = App::kWaveUniform ? w0 : w0 + wave_id();
        const int64_t v = w * 64 + lane_id();
        bool found = false;
        int64_t vdeg = 0;
        if (v < a.bu_rows && !a.seen[v]) {
            // kBuBatch neighbours per step: all column loads, then all frontier probes, then the test,
            // so a row scanned to its end pays two round trips per batch instead of per neighbour
            // (which neighbour hits does not matter: the depth is level + 1 either way)
            auto probe = [&](int32_t x) -> bool {
                return kFromDepth ? a.depth[x] == a.level : ((a.bm_in[x >> 6] >> (x & 63)) & 1ull);
            };
            // the first neighbour alone, from the dense first-column array (one coalesced load per wave;
            // -1: an empty row, which a directed pull adjacency may hold before its empty suffix): columns
            // are in relabelled order, so it is the row's highest-degree neighbour, the likeliest to be in
            // the frontier (a row still unvisited at level L has no neighbour of depth < L); for most rows
            // of the big levels one probe is all, with no row_ptr or column load (round 5: probing the
            // first column alone took RMAT-26 DO-BFS 1.730 -> 1.625 ms and CC 2.97 -> 2.88 ms,
            // profiles/r05/ab/bfs_bu_first_*; the dense array: profiles/r05/ab/bfs_first_col_*)
            const int32_t u0 = a.pull_first[v];
            if (u0 >= 0) found = probe(u0);
            const int64_t j1 = found ? 0 : a.pull_rp[v + 1];
            int64_t j = found ? 0 : a.pull_rp[v] + 1;
            for (; j < j1 && !found; j += kBuBatch) {
                int32_t u[kBuBatch];
#pragma unroll
                for (int k = 0; k < kBuBatch; ++k) u[k] = a.pull_col[j + k < j1 ? j + k : j1 - 1];
                bool hit[kBuBatch];
#pragma unroll
                for (int k = 0; k < kBuBatch; ++k) hit[k] = probe(u[k]);
#pragma unroll
                for (int k = 0; k < kBuBatch; ++k) found |= hit[k];
            }
            if (found) {
                a.depth[v] = next_depth;
                a.seen[v] = 1;
                vdeg = a.deg_rp[v + 1] - a.deg_rp[v];
            }
        }
        const uint64_t word = __ballot(found);
        if (lane_id() == 0 && w < words) a.bm_out[w] = word;
        app.append(found, (int32_t)v, vdeg, a.queue_out, a.qoff_out, packed);
    }
}

// a top-down level runs split when its launch is followed by the claim launch and its input frontier's
// entries are in [split_min, split_max] (split_max < 2^31: the owner map holds int32 entry indices)
__device__ __forceinline__ bool td_split(const BfsLevel& a, long long mf) {
    return a.split && mf >= a.split_min && mf <= a.split_max;
}

// Appends are wave-staged (WaveStage: no block barrier per step; the block-wide staged append measured
// RMAT-20 0.145-0.157 -> 0.119-0.129 ms, round 2).
__global__ __launch_bounds__(kBlock) void bfs_level_kernel(BfsLevel a) {
    __shared__ BfsState s_st;
    __shared__ long long s_nf, s_mf;
    __shared__ int s_switch;
    using App = WaveApp;
    __shared__ WaveStage s_app;
    if (threadIdx.x == 0) {
        int64_t nf, mf;
        bool sw;
        const BfsState c = bfs_decide(a, &nf, &mf, &sw);
        s_st = c;
        s_nf = nf;
        s_mf = mf;
        s_switch = sw;
        if (blockIdx.x == 0) {
            a.st[a.level % kBfsRing] = c;
            if (!c.done) a.ctr[(a.level + 1) % kBfsRing] = 0ull;  // counter of the next level
        }
    }
    __syncthreads();
    if (s_st.done) return;
    unsigned long long* packed = a.ctr + a.level % kBfsRing;
    App app{s_app};
    app.init();
    if (!s_st.bottom_up) {
        __shared__ int64_t s_qs[kQoffSamples];
        if (td_split(a, s_mf)) bfs_top_down<kTdOwner>(a, s_nf, s_mf, packed, app, s_qs);  // the claim launch appends
        else bfs_top_down<kTdCas>(a, s_nf, s_mf, packed, app, s_qs);
    } else if (s_switch) {
        bfs_bottom_up<true>(a, packed, app);
    } else {
        bfs_bottom_up<false>(a, packed, app);
    }
    app.final(a.queue_out, a.qoff_out, packed);
}

// Second launch of a split top-down level: the level's state (bfs_level_kernel wrote it) and input
// frontier counter say whether the level was split; if so, every entry re-reads its target's owner.
__global__ __launch_bounds__(kBlock) void bfs_td_claim_kernel(BfsLevel a) {
    __shared__ long long s_nf, s_mf;
    __shared__ int s_run;
    using App = WaveApp;
    __shared__ WaveStage s_app;
    if (threadIdx.x == 0) {
        const BfsState c = a.st[a.level % kBfsRing];
        const unsigned long long h = a.ctr[(a.level + kBfsRing - 1) % kBfsRing];
        s_nf = (long long)(h >> kPackShift);
        s_mf = (long long)(h & kEdgeMask);
        s_run = !c.done && !c.bottom_up && td_split(a, s_mf);
    }
    __syncthreads();
    if (!s_run) return;
    App app{s_app};
    app.init();
    __shared__ int64_t s_qs[kQoffSamples];
    bfs_top_down<kTdClaim>(a, s_nf, s_mf, a.ctr + a.level % kBfsRing, app, s_qs);
    app.final(a.queue_out, a.qoff_out, a.ctr + a.level % kBfsRing);
}

__global__ void fill_i32_kernel(int32_t* p, int64_t n, int32_t v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

// depth = -1 except the source; level -1 state: nothing explored, the source is the frontier.
// A vertex with an empty pull row can never be reached: its seen byte starts set, so no bottom-up
// level looks at it again (its depth stays -1).
// empty_from >= 0: rows from there on are the empty suffix (no row_ptr reads; at RMAT-26 reading the
// 537 MB row_ptr made this kernel 158 us of a 2.1 ms traversal).
__global__ void bfs_init_kernel(int32_t* __restrict__ depth, int64_t rows, int64_t source, int32_t* queue,
                                int64_t* qoff, const int64_t* __restrict__ deg_rp, long long total,
                                unsigned long long* ctr, BfsState* st, uint8_t* __restrict__ seen,
                                const int64_t* __restrict__ pull_rp, int64_t empty_from) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += (int64_t)gridDim.x * blockDim.x) {
        depth[i] = i == source ? 0 : -1;
        const bool empty = empty_from >= 0 ? i >= empty_from : (pull_rp && pull_rp[i + 1] == pull_rp[i]);
        seen[i] = i == source || empty;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        depth[source] = 0;  // (also when the source lies past `rows`: the caller's init_rows skipped the suffix)
        seen[source] = 1;
        queue[0] = (int32_t)source;
        qoff[0] = 0;
        ctr[kBfsRing - 1] = (1ull << kPackShift) | (unsigned long long)(deg_rp[source + 1] - deg_rp[source]);
        ctr[0] = 0ull;
        BfsState s{};
        s.mu = total;
        st[kBfsRing - 1] = s;
    }
}

// Multi-source start (cc_root_eccentricity), fused with the union-find's last per-row pass: a row with
// an edge whose rank is its component's minimum is a level-0 source, and every row's label (that
// minimum) replaces its parent.  Rows from r.ne on have no edge: no row_ptr, parent or minr reads
// (their label is their own rank).  At RMAT-26 this one pass replaced three (sources, init, labels:
// 530 us).
__global__ __launch_bounds__(kBlock) void bfs_init_roots_kernel(int32_t* __restrict__ depth, int64_t rows, CcRoots r,
                                                                const int64_t* __restrict__ deg_rp, int32_t* queue,
                                                                int64_t* qoff, unsigned long long* packed,
                                                                uint8_t* __restrict__ seen, BfsState* st0, long long total) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // level -1's state: nothing explored (no host copy and sync)
        BfsState s0{};
        s0.mu = total;
        *st0 = s0;
    }
    // Four rows per thread (16-byte loads and stores: one row per lane left the pass bound by load
    // latency, 218 us at RMAT-26).  A row whose component minimum is another row has an edge, so only
    // the component minima read the row pointers: an edgeless row is its own singleton component.
    constexpr int kQ = 4;
    __shared__ WaveStage ws;
    WaveApp app{ws};
    const int64_t quads = (rows + kQ - 1) / kQ;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q0 = (int64_t)blockIdx.x * blockDim.x; q0 < quads; q0 += stride) {  // block-uniform trips
        const int64_t q = q0 + threadIdx.x, v0 = q * kQ;
        bool take[kQ] = {false, false, false, false};
        int64_t deg[kQ] = {0, 0, 0, 0};
        if (q < quads) {
            int32_t lab[kQ], par[kQ], dep[kQ];
            uint8_t sn[kQ];
            const bool full = v0 + kQ <= rows, in = v0 + kQ <= r.ne;
            if (full) {
                const int4 x = *reinterpret_cast<const int4*>(r.rank + v0);
                lab[0] = x.x, lab[1] = x.y, lab[2] = x.z, lab[3] = x.w;
            } else {
#pragma unroll
                for (int k = 0; k < kQ; ++k) lab[k] = v0 + k < rows ? r.rank[v0 + k] : 0;
            }
            if (in) {
                const int4 x = *reinterpret_cast<const int4*>(r.parent + v0);
                par[0] = x.x, par[1] = x.y, par[2] = x.z, par[3] = x.w;
            } else {
#pragma unroll
                for (int k = 0; k < kQ; ++k) par[k] = v0 + k < r.ne ? r.parent[v0 + k] : 0;
            }
#pragma unroll
            for (int k = 0; k < kQ; ++k) {
                const int64_t v = v0 + k;
                bool least = true;
                dep[k] = -1;
                if (v < r.ne) {
                    const int32_t m = r.minr[par[k]];
                    least = lab[k] == m;
                    if (least) {
                        deg[k] = deg_rp[v + 1] - deg_rp[v];
                        take[k] = deg[k] > 0;
                    }
                    lab[k] = m;
                    dep[k] = take[k] ? 0 : -1;  // only the traversal reads the depths: the edgeless rows need none
                }
                sn[k] = least;  // = take || deg == 0; BOTH: push and pull rows are the same (bfs_init_kernel)
            }
            if (full) {
                *reinterpret_cast<int4*>(r.parent + v0) = make_int4(lab[0], lab[1], lab[2], lab[3]);
                *reinterpret_cast<uint32_t*>(seen + v0) =
                    (uint32_t)sn[0] | (uint32_t)sn[1] << 8 | (uint32_t)sn[2] << 16 | (uint32_t)sn[3] << 24;
            } else {
                for (int k = 0; k < kQ && v0 + k < rows; ++k) {
                    r.parent[v0 + k] = lab[k];
                    seen[v0 + k] = sn[k];
                }
            }
            if (in) *reinterpret_cast<int4*>(depth + v0) = make_int4(dep[0], dep[1], dep[2], dep[3]);
            else
                for (int k = 0; k < kQ && v0 + k < r.ne; ++k) depth[v0 + k] = dep[k];
        }
#pragma unroll
        for (int k = 0; k < kQ; ++k) app.append(take[k], (int32_t)(v0 + k), deg[k], queue, qoff, packed);
    }
    app.final(queue, qoff, packed);
}

// ---------------- bit-parallel multi-source BFS (pull, OR semiring) ----------------
// levels 0 .. kMsLevelWords-1 record their depths as one new-bit word per own row (MsBfsOp::nwl)
constexpr int kMsLevelWords = 12;
struct MsBfsOp {
    using T = unsigned long long;
    const T* __restrict__ F;    // frontier words of the previous level, full length
    T* __restrict__ Fout;       // full length, owned slice written
    T* __restrict__ visited;    // [rows]
    int32_t* __restrict__ depth;  // [nsrc * rows] int32 planes (used when depth8 is null)
    // [nsrc * rows] byte planes, 255 = unreached: the levels 0..254 of a traversal, a quarter of the
    // scattered depth writes (RMAT-26, 64 sources: 2.1 instead of 8.6 GB); widened to int32 planes on the
    // host's request (output) or when a traversal reaches level 255 (msbfs_widen_kernel)
    uint8_t* __restrict__ depth8;
    // this level's new-bit words of the own rows ([rows], nullable): levels below kMsLevelWords record
    // their depths here, one coalesced word per finalised row instead of a scattered byte per (source,
    // row) (msbfs_levels_to_planes_kernel turns them into planes when the host asks)
    unsigned long long* __restrict__ nwl;
    int32_t* __restrict__ changed;
    int64_t rows;
    VecPos pos;                 // owned row -> its slot in the gathered vector
    int32_t lvl;
    // the sources whose bits are in some word of the gathered vector F (msbfs_live_kernel; device
    // word): no other bit can arrive this level, so a row whose unvisited bits miss them all is done
    const T* live;
    __device__ __forceinline__ T identity() const { return 0ull; }
    __device__ __forceinline__ T combine(T a, T b) const { return a | b; }
    __device__ __forceinline__ T gather(int32_t c) const { return F[c]; }
    __device__ __forceinline__ const T* vec() const { return F; }
    __device__ __forceinline__ T shfl_xor(T v, int o) const { return __shfl_xor(v, o, kWave); }
    __device__ __forceinline__ T shfl_up(T v, int d) const { return __shfl_up(v, d, kWave); }
    __device__ __forceinline__ bool active(int64_t row) const { return (~visited[row] & *live) != 0ull; }
    // masking with live also discards what a done row's skipped merge tasks left in its partials
    __device__ __forceinline__ void finalize(int64_t row, T acc) const {
        T nw = acc & ~visited[row] & *live;
        Fout[pos(row)] = nw;
        if (nwl) nwl[row] = nw;
        if (nw) {
            visited[row] |= nw;
            if (changed) *changed = 1;
            while (nw) {
                const int s = __ffsll(nw) - 1;
                if (depth8) depth8[(int64_t)s * rows + row] = (uint8_t)lvl;
                else if (depth) depth[(int64_t)s * rows + row] = lvl;
                nw &= nw - 1;
            }
        }
    }
};

// *live |= the OR of every word of F (one atomic per block)
__global__ __launch_bounds__(kRedThreads) void msbfs_live_kernel(const unsigned long long* __restrict__ F, int64_t len,
                                                                 unsigned long long* __restrict__ live) {
    __shared__ unsigned long long red[kRedWaves];
    unsigned long long m = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += (int64_t)gridDim.x * blockDim.x)
        m |= F[i];
    m = block_reduce(m, OrU64{}, red);
    if (threadIdx.x == 0 && m) atomicOr(live, m);
}

// After a pull level (one shard): the next level's live bits and its packed frontier counter
// ((vertices << kPackShift) | push-edge sum: the direction rule's input) in one read of F, without the
// top-down queue, which msbfs_frontier_kernel builds only if the next level runs top-down
// (the queue build cost 750 us at RMAT-26's first two pull levels, whose successors pull).
__global__ __launch_bounds__(kRedThreads) void msbfs_scan_kernel(const unsigned long long* __restrict__ F, int64_t rows,
                                                                 const int64_t* __restrict__ push_rp,
                                                                 unsigned long long* __restrict__ live,
                                                                 unsigned long long* __restrict__ packed) {
    __shared__ unsigned long long red_or[kRedWaves], red_n[kRedWaves];
    unsigned long long m = 0, cnt = 0;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < rows; v += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long w = F[v];
        if (w) {
            m |= w;
            cnt += (1ull << kPackShift) + (unsigned long long)(push_rp[v + 1] - push_rp[v]);
        }
    }
    m = block_reduce(m, OrU64{}, red_or);
    cnt = block_reduce(cnt, AddU64{}, red_n);
    if (threadIdx.x == 0) {
        if (m) atomicOr(live, m);
        if (cnt) atomicAdd(packed, cnt);
    }
}

// bit i of todo: band row i (row0 + i) can still gain a bit this level
__global__ __launch_bounds__(kBlock) void msbfs_todo_kernel(const unsigned long long* __restrict__ visited,
                                                            int64_t row0, int64_t nrows,
                                                            const unsigned long long* __restrict__ live,
                                                            unsigned long long* __restrict__ todo) {
    const unsigned long long lv = *live;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x0 = (int64_t)blockIdx.x * blockDim.x; x0 < nrows; x0 += stride) {  // block-uniform trips
        const int64_t i = x0 + threadIdx.x;
        const bool b = i < nrows && (~visited[row0 + i] & lv) != 0ull;
        const unsigned long long word = __ballot(b);
        if (lane_id() == 0 && i < nrows) todo[i >> 6] = word;
    }
}

// bit t of tlive (MergeArgs::live): merge task t touches a band row that can still gain a bit;
// *nlive += the live tasks (one atomic per block; the work counter of jg_stats.algorithmic_bytes)
__global__ __launch_bounds__(kRedThreads) void msbfs_task_live_kernel(const int32_t* __restrict__ task_rows, int64_t tasks,
                                                                      const unsigned long long* __restrict__ todo,
                                                                      unsigned long long* __restrict__ tlive,
                                                                      unsigned long long* __restrict__ nlive) {
    __shared__ unsigned long long red[kRedWaves];
    unsigned long long count = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x0 = (int64_t)blockIdx.x * blockDim.x; x0 < tasks; x0 += stride) {  // block-uniform trips
        const int64_t t = x0 + threadIdx.x;
        bool b = false;
        if (t < tasks) {
            const int32_t lo = task_rows[2 * t], hi = task_rows[2 * t + 1];
            for (int32_t w = lo >> 6; w <= (hi >> 6) && !b; ++w) {
                unsigned long long m = todo[w];
                if (w == (lo >> 6)) m &= ~0ull << (lo & 63);
                if (w == (hi >> 6) && (hi & 63) != 63) m &= (2ull << (hi & 63)) - 1ull;
                b = m != 0ull;
            }
        }
        const unsigned long long word = __ballot(b);
        if (lane_id() == 0 && t < tasks) {
            tlive[t >> 6] = word;
            count += (unsigned long long)__popcll(word);
        }
    }
    count = block_reduce(count, AddU64{}, red);
    if (threadIdx.x == 0 && count) atomicAdd(nlive, count);
}

// int32 planes from byte planes (255 = unreached -> -1)
__global__ void msbfs_widen_kernel(const uint8_t* __restrict__ d8, int64_t n, int32_t* __restrict__ d32) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t v = d8[i];
        d32[i] = v == 255 ? -1 : (int32_t)v;
    }
}

// Levels recorded as new-bit words ([levels][rows]) into int32 depth planes (plane s, row r = the level
// whose word holds bit s; pairs no recorded level holds keep what the planes had: a later level's
// depth, or -1)
// Rows [ne, rows) have no pull entries, so no level after 0 reaches them; pull levels do not finalise
// them (msbfs_skip_empty) and their words of levels >= 1 are never written.
__global__ void msbfs_levels_to_planes_kernel(const unsigned long long* __restrict__ nwl, int levels, unsigned word_levels,
                                              int64_t rows, int64_t ne, int nsrc, int32_t* __restrict__ depth) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x)
        for (int L = 0; L < levels; ++L) {
            if (!((word_levels >> L) & 1u)) continue;  // a top-down level: its (row, word) records instead
            if (L > 0 && r >= ne) break;
            unsigned long long w = nwl[(int64_t)L * rows + r];
            while (w) {
                const int s = __ffsll(w) - 1;
                if (s < nsrc) depth[(int64_t)s * rows + r] = L;
                w &= w - 1;
            }
        }
}

// pairs += the set bits of visited[0, rows) (sources x reached rows: the depth entries written)
__global__ __launch_bounds__(kRedThreads) void msbfs_pairs_kernel(const unsigned long long* __restrict__ visited, int64_t rows,
                                                                  unsigned long long* __restrict__ pairs) {
    __shared__ unsigned long long red[kRedWaves];
    unsigned long long c = 0;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < rows; v += (int64_t)gridDim.x * blockDim.x)
        c += (unsigned long long)__popcll(visited[v]);
    c = block_reduce(c, AddU64{}, red);
    if (threadIdx.x == 0 && c) atomicAdd(pairs, c);
}

__global__ __launch_bounds__(kWave) void msbfs_init_kernel(const int64_t* __restrict__ local_src, int nsrc,
                                                           unsigned long long* __restrict__ F,
                                                           unsigned long long* __restrict__ visited,
                                                           unsigned long long* __restrict__ nw0, int64_t rows, VecPos pos,
                                                           int32_t* __restrict__ rec_rows,
                                                           unsigned long long* __restrict__ rec_words) {
    // one wave, lane s = source s (nsrc <= 64: the caller walks the sources in batches of 64).  Several
    // sources may share a vertex: each lane ORs in the bits of every source on its row, so lanes sharing
    // a row store the same words (one thread walking the sources took ~46 us: 128 dependent round trips)
    const int s = (int)threadIdx.x;
    const int64_t l = s < nsrc ? local_src[s] : -1;
    unsigned long long word = 0;
    for (int t = 0; t < nsrc; ++t)
        if (__shfl(l, t, kWave) == l) word |= 1ull << t;
    if (l >= 0) {  // stores, not ORs: a source row past the empty suffix is not cleared first (one shard)
        F[pos(l)] = word;
        visited[l] = word;
        if (nw0) nw0[l] = word;  // level 0's new-bit word
        if (rec_rows) rec_words[s] = word;
    } else if (rec_rows && s < nsrc) {
        rec_words[s] = 0ull;
    }
    // level 0 as (row, word) records: a shared source row records the same full word twice
    if (rec_rows && s < nsrc) rec_rows[s] = (int32_t)l;
}

// A top-down level's depths as (row, new-bit word) records: the rows that gained a bit are exactly the
// next frontier's queue (msbfs_td_apply_kernel queues a touched row iff its new word is nonzero), so the
// level needs no [rows]-long word array cleared before it
__global__ void msbfs_td_record_kernel(const int32_t* __restrict__ queue, int64_t n, const unsigned long long* __restrict__ F,
                                       VecPos pos, int32_t* __restrict__ rec_rows,
                                       unsigned long long* __restrict__ rec_words) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = queue[i];
        rec_rows[i] = r;
        rec_words[i] = F[pos(r)];
    }
}

// depth planes from (row, word) records of one level (rows < 0: none)
__global__ void msbfs_records_to_planes_kernel(const int32_t* __restrict__ rec_rows,
                                               const unsigned long long* __restrict__ rec_words, int64_t n, int level,
                                               int64_t rows, int nsrc, int32_t* __restrict__ depth) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = rec_rows[i];
        if (r < 0) continue;
        unsigned long long w = rec_words[i];
        while (w) {
            const int s = __ffsll(w) - 1;
            if (s < nsrc) depth[(int64_t)s * rows + r] = level;
            w &= w - 1;
        }
    }
}

// Top-down levels of the bit-parallel BFS (one shard): the frontier is a queue of vertices with a
// nonzero word and their push-edge offsets.  Each frontier edge v -> u ORs F[v]'s unvisited bits into
// Fnext[u] (OR is order-independent: deterministic); the first toucher of u queues it; the apply pass
// turns the touched words into the next frontier.
__global__ __launch_bounds__(kBlock) void msbfs_frontier_kernel(const unsigned long long* __restrict__ F, int64_t rows,
                                                                const int64_t* __restrict__ push_rp,
                                                                int32_t* __restrict__ queue, int64_t* __restrict__ qoff,
                                                                unsigned long long* __restrict__ packed,
                                                                unsigned long long mask = ~0ull) {
    __shared__ WaveStage ws;
    WaveApp app{ws};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x0 = (int64_t)blockIdx.x * blockDim.x; x0 < rows; x0 += stride) {  // block-uniform trips
        const int64_t v = x0 + threadIdx.x;
        const bool take = v < rows && (F[v] & mask) != 0ull;
        const int64_t deg = take ? push_rp[v + 1] - push_rp[v] : 0;
        app.append(take, (int32_t)v, deg, queue, qoff, packed);
    }
    app.final(queue, qoff, packed);
}

// msbfs_frontier_kernel and msbfs_scan_kernel in one pass, after a pull level whose successor is
// expected to run top-down (its exit bands had almost no live task): the queue, the packed counter
// and the live bits (*live |= the OR of the words, one atomic per block)
__global__ __launch_bounds__(kBlock) void msbfs_frontier_live_kernel(const unsigned long long* __restrict__ F, int64_t rows,
                                                                     const int64_t* __restrict__ push_rp,
                                                                     int32_t* __restrict__ queue, int64_t* __restrict__ qoff,
                                                                     unsigned long long* __restrict__ packed,
                                                                     unsigned long long* __restrict__ live) {
    __shared__ WaveStage ws;
    __shared__ unsigned long long red[kBlock / kWave];
    WaveApp app{ws};
    unsigned long long m = 0;
    // four rows per thread and trip, their loads issued together (one per trip: 217 -> 196 us at RMAT-26,
    // round 6; the pass reads the frontier words and the row pointers of the frontier rows)
    constexpr int R = 4;
    const int64_t span = (int64_t)blockDim.x * R;
    for (int64_t x0 = (int64_t)blockIdx.x * span; x0 < rows; x0 += (int64_t)gridDim.x * span) {  // block-uniform trips
        unsigned long long w[R];
        int64_t deg[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int64_t v = x0 + (int64_t)k * blockDim.x + threadIdx.x;
            w[k] = v < rows ? F[v] : 0ull;
        }
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int64_t v = x0 + (int64_t)k * blockDim.x + threadIdx.x;
            m |= w[k];
            deg[k] = w[k] ? push_rp[v + 1] - push_rp[v] : 0;
        }
#pragma unroll
        for (int k = 0; k < R; ++k)
            app.append(w[k] != 0ull, (int32_t)(x0 + (int64_t)k * blockDim.x + threadIdx.x), deg[k], queue, qoff, packed);
    }
    app.final(queue, qoff, packed);
    m = block_reduce(m, OrU64{}, red);
    if (threadIdx.x == 0 && m) atomicOr(live, m);
}

// The first top-down queue: the distinct source rows with their push-edge offsets, and the packed
// frontier counter (one thread: at most 64 sources)
__global__ __launch_bounds__(kWave) void msbfs_source_queue_kernel(const int64_t* __restrict__ rows, int cnt,
                                                                   const int64_t* __restrict__ push_rp,
                                                                   int32_t* __restrict__ queue, int64_t* __restrict__ qoff,
                                                                   unsigned long long* __restrict__ packed) {
    // one wave, lane i = distinct source row i (cnt <= 64: one batch's distinct rows); the entry offsets are
    // the wave's exclusive scan of the row degrees
    const int i = (int)threadIdx.x;
    const int64_t v = i < cnt ? rows[i] : 0;
    const int64_t d = i < cnt ? push_rp[v + 1] - push_rp[v] : 0;
    const int64_t inc = wave_inclusive_scan_add(d);
    if (i < cnt) {
        queue[i] = (int32_t)v;
        qoff[i] = inc - d;
    }
    if (i == kWave - 1) packed[0] = ((unsigned long long)cnt << kPackShift) | (unsigned long long)inc;
}

// ---- bottom-up rows of the bit-parallel BFS with early exit (one shard) ----
// A row's gain this level is the OR of its neighbours' frontier words masked by need = ~visited & live;
// once the OR covers need, no further entry can add a bit, so the scan stops (Beamer's bottom-up
// early exit, per 64-bit word).  The result equals the merge engine's: the same OR, the same finalize.
// (Every pull level bottom-up, rows [0, ne) by workgroup / wave / lane roles, measured 2-4x slower than
// the merge engine at RMAT-22 / 26, round 3: the exit pays only on the levels after the frontier's peak.)
constexpr int kMsBuUnroll = 4;  // pass B: 4 x 64 entries in flight per wave step
struct MsBu {
    const int64_t* rp;
    const int32_t* col;
    const int32_t* first_col;         // [rows] each row's first column (Csr::first_col)
    int64_t rows;                     // rows [0, rows) take the early exit
    unsigned long long* examined;     // += the entries scanned (work counter, jg_stats.algorithmic_bytes)
    int first = 16;                   // msbfs_exit_first_kernel: entries a lane scans before pass B takes the row
};

__device__ __forceinline__ unsigned long long wave_or(unsigned long long m) {
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) m |= __shfl_xor(m, o, kWave);
    return m;
}

// ---- the split's first band with early exit, inside a merged pull level (msbfs_exit) ----
// On the level after the frontier's peak a hub row typically finds every unvisited live bit within its
// first two or three entries (RMAT-22: 2.4 on average; tools/msbfs_exit_sim.py), so a 256-entry wave
// step gathers ~100x what the row needs.  Pass A gives each row a lane
// and its first `first` entries (MsBu::first, Tune::msbfs_exit_first; 16 by default); a row still missing bits leaves its partial word in Fout and a bit
// in `rest` (one word per 64 rows, a plain store per wave), and pass B scans the remaining entries of
// those rows a wave each.  Entries scanned are summed per 1024-thread workgroup, one atomic each.

__global__ __launch_bounds__(kRedThreads) void msbfs_exit_first_kernel(MsBu a, MsBfsOp op,
                                                                        unsigned long long* __restrict__ rest) {
    __shared__ unsigned long long red[kRedWaves];
    const unsigned long long live = *op.live;
    const int64_t words = (a.rows + 63) / 64, nwaves = (int64_t)gridDim.x * kRedWaves;
    unsigned long long scanned = 0;
    for (int64_t w = (int64_t)blockIdx.x * kRedWaves + wave_id(); w < words; w += nwaves) {  // wave-uniform
        const int64_t v = w * 64 + lane_id();
        bool more = false;
        if (v < a.rows) {
            const unsigned long long need = ~op.visited[v] & live;
            unsigned long long acc = 0;
            if (need) {
                const int64_t e0 = a.rp[v], e1 = a.rp[v + 1], ek = e1 < e0 + a.first ? e1 : e0 + a.first;
                int64_t j = e0;
                // the first entry alone (the row's highest-degree neighbour: often every bit the row needs; as
                // in bfs_bottom_up): RMAT-26 64-source BFS 10.50 -> 10.04-10.17 ms (profiles/r05/ab/msbfs_first1.log)
                if (j < ek) {  // (its column from the dense array: one coalesced load)
                    acc |= op.F[a.first_col[v]] & need;
                    ++j;
                }
                for (; j < ek && acc != need; j += 4) {
                    int32_t c[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) c[u] = a.col[j + u < ek ? j + u : ek - 1];
#pragma unroll
                    for (int u = 0; u < 4; ++u) acc |= op.F[c[u]] & need;
                }
                scanned += (unsigned long long)((j < ek ? j : ek) - e0);
                more = acc != need && ek < e1;
            }
            if (more) op.Fout[op.pos(v)] = acc;  // pass B's starting word
            else op.finalize(v, acc);
        }
        const uint64_t word = __ballot(more);
        if (lane_id() == 0) rest[w] = word;
    }
    scanned = block_reduce(scanned, AddU64{}, red);
    if (threadIdx.x == 0 && scanned) atomicAdd(a.examined, scanned);
}

__global__ __launch_bounds__(kRedThreads) void msbfs_exit_rest_kernel(MsBu a, MsBfsOp op,
                                                                       const unsigned long long* __restrict__ rest) {
    __shared__ unsigned long long red[kRedWaves];
    const unsigned long long live = *op.live;
    const int lane = lane_id();
    const int64_t words = (a.rows + 63) / 64, nwaves = (int64_t)gridDim.x * kRedWaves;
    unsigned long long scanned = 0;
    for (int64_t w = (int64_t)blockIdx.x * kRedWaves + wave_id(); w < words; w += nwaves) {  // wave-uniform
        uint64_t bits = rest[w];
        while (bits) {
            const int64_t v = w * 64 + (__ffsll((unsigned long long)bits) - 1);
            bits &= bits - 1;
            const unsigned long long need = ~op.visited[v] & live;
            unsigned long long acc = op.Fout[op.pos(v)];
            const int64_t e0 = a.rp[v] + a.first, e1 = a.rp[v + 1];
            int64_t j = e0;
            for (; j < e1 && acc != need; j += kMsBuUnroll * kWave) {
                int32_t c[kMsBuUnroll];
#pragma unroll
                for (int u = 0; u < kMsBuUnroll; ++u) {
                    const int64_t e = j + u * kWave + lane;
                    c[u] = e < e1 ? a.col[e] : -1;
                }
                unsigned long long m = 0;
#pragma unroll
                for (int u = 0; u < kMsBuUnroll; ++u) m |= c[u] >= 0 ? op.F[c[u]] : 0ull;
                acc |= wave_or(m & need);
            }
            if (lane == 0) {
                scanned += (unsigned long long)((j < e1 ? j : e1) - e0);
                op.finalize(v, acc);
            }
        }
    }
    scanned = block_reduce(scanned, AddU64{}, red);
    if (threadIdx.x == 0 && scanned) atomicAdd(a.examined, scanned);
}

constexpr int kMaxPeersMs = 64;
__device__ __forceinline__ int slot_peer(int32_t u, int tbits, int r) {
    const int seg = (int)((uint32_t)u >> tbits);
    return seg <= r ? seg - 1 : seg;
}

struct MsTd {
    const int32_t* queue;
    const int64_t* qoff;
    int64_t nq, mf;
    const int64_t* push_rp;
    const int32_t* push_col;
    const unsigned long long* F;
    const unsigned long long* visited;
    unsigned long long* Fnext;
    int32_t* touched;
    int64_t* touched_off;  // scratch (the appender writes edge offsets)
    unsigned long long* tpacked;
    int tbits;             // sharded (compact BOTH columns): u >> tbits != 0 is a peer's vertex; 31 on one shard
    // sharded: the halo staging vector (compact positions; zero outside a level) and the list of its
    // slots this level set first, so they can be cleared without a pass over the whole vector
    unsigned long long* hstage;
    int32_t* hlist;
    int64_t* hlist_off;        // scratch of the appender
    unsigned long long* hpacked;
    // (unused: the per-peer counts of the sparse reverse exchange come from msbfs_slot_hist_kernel)
    unsigned long long* pcnt;
    int r, P;                  // this shard's index, the shard count
    int probe_visited;         // 0: no visited probe before the OR (the apply masks with visited anyway)
    int no_touched;            // 1: no touched list (the level's apply passes over every row instead)
};

__global__ __launch_bounds__(kBlock) void msbfs_td_kernel(MsTd a) {
    __shared__ WaveStage ws, hws;
    WaveApp app{ws}, happ{hws};
    const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_tile = nthreads * kTdEdgesPerThread;
    const int64_t tiles = (a.mf + per_tile - 1) / per_tile;
    for (int64_t t = 0; t < tiles; ++t) {
        if ((t * nthreads + (int64_t)blockIdx.x * blockDim.x) * kTdEdgesPerThread >= a.mf) break;  // block-uniform
        const int64_t e0 = (t * nthreads + tid) * kTdEdgesPerThread;
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
        for (int k = 0; k < kTdEdgesPerThread; ++k) {
            const int64_t e = e0 + k;
            bool take = false, hfirst = false;
            int32_t u = 0;
            if (e < a.mf) {
                while (e >= next_bound) {
                    ++i;
                    next_bound = i + 1 < a.nq ? a.qoff[i + 1] : a.mf;
                }
                const int32_t v = a.queue[i];
                u = a.push_col[a.push_rp[v] + (e - a.qoff[i])];
                const unsigned long long fv = a.F[v];
                if ((u >> a.tbits) == 0) {
                    const unsigned long long w = fv & ~(a.probe_visited ? a.visited[u] : 0ull);
                    // a plain read first: a hub neighbour already holding these bits takes no atomic (the
                    // atomics on one word serialise at the memory side); a stale read only costs the atomic
                    if (w && (w & ~a.Fnext[u])) take = atomicOr(&a.Fnext[u], w) == 0ull && !a.no_touched;
                } else if (fv & ~a.hstage[u]) {
                    // a peer's vertex: its halo slot collects the bits; the reverse exchange takes them to
                    // the owner, which masks them with its visited bits (msbfs_td_recv_kernel)
                    hfirst = atomicOr(&a.hstage[u], fv) == 0ull;
                }
            }
            app.append(take, u, 0, a.touched, a.touched_off, a.tpacked);
            if (a.hstage) happ.append(hfirst, u, 0, a.hlist, a.hlist_off, a.hpacked);

        }
    }
    app.final(a.touched, a.touched_off, a.tpacked);
    if (a.hstage) happ.final(a.hlist, a.hlist_off, a.hpacked);

}

// ---- sparse reverse exchange of a sharded top-down level (only the staging slots the level set) ----
// A staging slot u (compact position, segment u >> tbits >= 1) is about peer q = seg - 1 if seg <= r,
// else seg (the inverse of Halo::seg_of for shard r); it travels as (offset in the segment, word): the
// offset is the slot's position in q's send list for r, so q finds its own row as send_src[send_off[r] + o].

struct PairRuns {
    int64_t off[kMaxPeersMs + 1];       // pack: the run of peer q starts at pair off[q]; receive: from q at off[q]
    int64_t send_off[kMaxPeersMs + 1];  // receive: the owner's send-list offsets (Halo::send_off)
    int P;
};

// the (offset, word) pairs of every set staging slot, grouped by peer (order inside a run is free: the
// receiver ORs); cursor[P] zeroed by the caller
// Per-peer counts of the halo staging slots a top-down level set first (hlist[0, nh), nh the packed
// counter's vertices): block b takes the b-th of gridDim.x equal chunks, bcount[b * P + q] = its slots
// about peer q, pcnt[q] += them (at most gridDim.x atomics per peer; the top-down kernel's one atomic per
// block and peer, on grids of up to 8192 blocks, queued thousands of them on each counter).
__global__ __launch_bounds__(kRedThreads) void msbfs_slot_hist_kernel(const int32_t* __restrict__ hlist,
                                                                      const unsigned long long* __restrict__ hpacked,
                                                                      int tbits, int r, int P,
                                                                      unsigned int* __restrict__ bcount,
                                                                      unsigned long long* __restrict__ pcnt) {
    __shared__ unsigned int lc[kMaxPeersMs];
    const int64_t nh = (int64_t)(*hpacked >> kPackShift);
    const int64_t chunk = (nh + gridDim.x - 1) / gridDim.x;
    const int64_t k0 = (int64_t)blockIdx.x * chunk, k1 = k0 + chunk < nh ? k0 + chunk : nh;
    for (int q = threadIdx.x; q < P; q += blockDim.x) lc[q] = 0u;
    __syncthreads();
    for (int64_t k = k0 + threadIdx.x; k < k1; k += blockDim.x) atomicAdd(&lc[slot_peer(hlist[k], tbits, r)], 1u);
    __syncthreads();
    for (int q = threadIdx.x; q < P; q += blockDim.x) {
        bcount[(int64_t)blockIdx.x * P + q] = lc[q];
        if (lc[q]) atomicAdd(&pcnt[q], (unsigned long long)lc[q]);
    }
}

// Packs the set staging slots as (offset in the peer's segment, word) pairs, grouped by peer: block b
// takes the same chunk as msbfs_slot_hist_kernel (the same grid), its runs start after the earlier
// blocks' (an exclusive sum of bcount), and its slots take their places by LDS cursors: no global atomics.
__global__ __launch_bounds__(kRedThreads) void msbfs_pair_pack_kernel(const int32_t* __restrict__ hlist, int64_t nh,
                                                                      const unsigned long long* __restrict__ hs, int tbits,
                                                                      int r, PairRuns pr,
                                                                      const unsigned int* __restrict__ bcount,
                                                                      unsigned long long* __restrict__ pairs) {
    __shared__ unsigned int lc[kMaxPeersMs];
    __shared__ int64_t base[kMaxPeersMs];
    const int64_t chunk = (nh + gridDim.x - 1) / gridDim.x;
    const int64_t k0 = (int64_t)blockIdx.x * chunk, k1 = k0 + chunk < nh ? k0 + chunk : nh;
    if (k0 >= k1) return;  // block-uniform: an empty chunk writes nothing
    // this block's run starts: wave w sums peer q = w (+ kRedWaves ...) over the earlier blocks' counts,
    // one lane per block (a thread walking up to 511 blocks alone made every launch cost ~50 us)
    for (int q = wave_id(); q < pr.P; q += kRedWaves) {
        unsigned int s = 0;
        for (unsigned x = lane_id(); x < blockIdx.x; x += kWave) s += bcount[(int64_t)x * pr.P + q];
        s = wave_reduce_add(s);
        if (lane_id() == 0) base[q] = pr.off[q] + (int64_t)s;
    }
    __syncthreads();
    for (int64_t s0 = k0; s0 < k1; s0 += blockDim.x) {  // block-uniform trips
        for (int q = threadIdx.x; q < pr.P; q += blockDim.x) lc[q] = 0u;
        __syncthreads();
        const int64_t k = s0 + threadIdx.x;
        int q = 0;
        unsigned int p = 0;
        int32_t u = 0;
        if (k < k1) {
            u = hlist[k];
            q = slot_peer(u, tbits, r);
            p = atomicAdd(&lc[q], 1u);
        }
        __syncthreads();
        if (k < k1) {
            const int64_t j = base[q] + p;
            pairs[2 * j] = (unsigned long long)((uint32_t)u & ((1u << tbits) - 1u));
            pairs[2 * j + 1] = hs[u];
        }
        __syncthreads();
        for (int x = threadIdx.x; x < pr.P; x += blockDim.x) base[x] += lc[x];
        __syncthreads();
    }
}

// owner side of the sparse exchange: like msbfs_td_recv_kernel, over the received pairs
__global__ __launch_bounds__(kBlock) void msbfs_td_recv_pairs_kernel(const unsigned long long* __restrict__ rpairs,
                                                                     int64_t total, PairRuns pr,
                                                                     const int32_t* __restrict__ send_src,
                                                                     const unsigned long long* __restrict__ visited,
                                                                     unsigned long long* __restrict__ Fnext,
                                                                     int32_t* __restrict__ touched,
                                                                     int64_t* __restrict__ touched_off,
                                                                     unsigned long long* __restrict__ tpacked) {
    __shared__ WaveStage ws;
    WaveApp app{ws};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x0 = (int64_t)blockIdx.x * blockDim.x; x0 < total; x0 += stride) {  // block-uniform trips
        const int64_t k = x0 + threadIdx.x;
        bool take = false;
        int32_t u = 0;
        if (k < total) {
            int q = 0;
            while (q + 1 < pr.P && pr.off[q + 1] <= k) ++q;
            const unsigned long long o = rpairs[2 * k], r = rpairs[2 * k + 1];
            u = send_src[pr.send_off[q] + (int64_t)o];
            const unsigned long long w = r & ~visited[u];
            if (w && (w & ~Fnext[u])) take = atomicOr(&Fnext[u], w) == 0ull;
        }
        app.append(take, u, 0, touched, touched_off, tpacked);
    }
    app.final(touched, touched_off, tpacked);
}

// Zeroes a few small control buffers in one launch (each hipMemsetAsync is a kernel dispatch of its own:
// four per top-down level and shard were ~0.2 ms of a sharded RMAT-26 traversal)
struct ZeroList {
    uint32_t* p[6];
    int n[6];  // 32-bit words
    int k;
};
__global__ void zero_words_kernel(ZeroList z) {
    for (int j = 0; j < z.k; ++j)
        for (int i = threadIdx.x; i < z.n[j]; i += blockDim.x) z.p[j][i] = 0u;
}
inline void zero_words(std::initializer_list<std::pair<void*, size_t>> bufs, hipStream_t s) {
    ZeroList z{};
    for (const auto& b : bufs) {
        if (!b.first || !b.second) continue;
        if (z.k == 6) fail(JG_ERR_UNSUPPORTED, "zero_words: too many buffers");
        z.p[z.k] = static_cast<uint32_t*>(b.first);
        z.n[z.k] = (int)(b.second / 4);
        ++z.k;
    }
    if (!z.k) return;
    zero_words_kernel<<<1, kBlock, 0, s>>>(z);
    JG_LAUNCH_CHECK();
}

// the same with the count in a packed device counter (no host read-back)
__global__ void msbfs_zero_list_packed_kernel(unsigned long long* __restrict__ v, const int32_t* __restrict__ list,
                                              const unsigned long long* __restrict__ packed) {
    const int64_t n = (int64_t)(*packed >> kPackShift);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        v[list[i]] = 0ull;
}

// v[list[i]] = 0 for i < n: clears the words a level set (its frontier rows, or its halo staging slots)
// without a pass over the whole vector
__global__ void msbfs_zero_list_kernel(unsigned long long* __restrict__ v, const int32_t* __restrict__ list, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        v[list[i]] = 0ull;
}

// The source rows at or past from (rows without pull entries) of a frontier vector: the only such rows
// whose word can be nonzero after level 0 (one wave; n <= 64 distinct source rows)
__global__ __launch_bounds__(kWave) void msbfs_zero_tail_sources_kernel(unsigned long long* __restrict__ v,
                                                                       const int64_t* __restrict__ src, int n,
                                                                       int64_t from) {
    const int i = (int)threadIdx.x;
    if (i < n && src[i] >= from) v[src[i]] = 0ull;
}

// Sharded top-down level, owner side: the peers' halo slots for own rows, received at the send-list
// positions (rbuf[k] is about own row send_src[k]); own rows that gain a bit join the touched list
// the local top-down kernel started (the first toucher of a word appends it, as there)
__global__ __launch_bounds__(kBlock) void msbfs_td_recv_kernel(const unsigned long long* __restrict__ rbuf,
                                                               const int32_t* __restrict__ send_src, int64_t nrecv,
                                                               const unsigned long long* __restrict__ visited,
                                                               unsigned long long* __restrict__ Fnext,
                                                               int32_t* __restrict__ touched,
                                                               int64_t* __restrict__ touched_off,
                                                               unsigned long long* __restrict__ tpacked) {
    __shared__ WaveStage ws;
    WaveApp app{ws};
    // four words per thread and trip, loaded together (a sparse level's words are mostly zero: the
    // kernel is a stream of rbuf, latency-bound one word at a time)
    constexpr int kU = 4;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * kU;
    for (int64_t x0 = (int64_t)blockIdx.x * blockDim.x * kU; x0 < nrecv; x0 += stride) {  // block-uniform trips
        unsigned long long r[kU];
#pragma unroll
        for (int j = 0; j < kU; ++j) {
            const int64_t k = x0 + (int64_t)j * blockDim.x + threadIdx.x;
            r[j] = k < nrecv ? rbuf[k] : 0ull;
        }
#pragma unroll
        for (int j = 0; j < kU; ++j) {
            const int64_t k = x0 + (int64_t)j * blockDim.x + threadIdx.x;
            bool take = false;
            int32_t u = 0;
            if (r[j]) {
                u = send_src[k];
                const unsigned long long w = r[j] & ~visited[u];
                if (w && (w & ~Fnext[u])) take = atomicOr(&Fnext[u], w) == 0ull;
            }
            app.append(take, u, 0, touched, touched_off, tpacked);
        }
    }
    app.final(touched, touched_off, tpacked);
}

// touched vertex u: its new bits become its next-frontier word (and the visited / depth updates);
// *live_out |= the OR of the new words (the next pull level's live bits: untouched rows hold zero)
__global__ __launch_bounds__(kBlock) void msbfs_td_apply_kernel(const int32_t* __restrict__ touched,
                                                                const unsigned long long* __restrict__ tcount,
                                                                MsBfsOp op, const int64_t* __restrict__ push_rp,
                                                                int32_t* __restrict__ queue, int64_t* __restrict__ qoff,
                                                                unsigned long long* __restrict__ packed,
                                                                unsigned long long* __restrict__ live_out) {
    __shared__ WaveStage ws;
    __shared__ unsigned long long red[kBlock / kWave];
    WaveApp app{ws};
    unsigned long long lv = 0;
    // the touched count from the device (packed counter): the host does not wait for it
    const int64_t nt = (int64_t)(*tcount >> kPackShift);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x0 = (int64_t)blockIdx.x * blockDim.x; x0 < nt; x0 += stride) {  // block-uniform trips
        const int64_t x = x0 + threadIdx.x;
        bool take = false;
        int32_t u = 0;
        int64_t deg = 0;
        if (x < nt) {
            u = touched[x];
            const unsigned long long acc = op.Fout[u];  // the ORed words (finalize overwrites Fout[u])
            op.finalize(u, acc);
            const unsigned long long nw = op.Fout[u];
            lv |= nw;
            take = nw != 0ull;
            if (take) deg = push_rp[u + 1] - push_rp[u];
        }
        app.append(take, u, deg, queue, qoff, packed);
    }
    app.final(queue, qoff, packed);
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) lv |= __shfl_xor(lv, o, kWave);
    if (lane_id() == 0) red[wave_id()] = lv;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / kWave; ++w) lv |= red[w];
        // a plain read first: once every source is live (most levels) no block takes the atomic, which
        // serialises at the memory side (one per block was +1.5 ms over a sharded RMAT-26 traversal)
        if (lv & ~*(volatile unsigned long long*)live_out) atomicOr(live_out, lv);
    }
}

// The same over every own row in row order (msbfs_td_rowapply): a big top-down level touches a good
// part of the rows (RMAT-26 level 1: 33.6 M edges), and its touched list, in append order, made every
// word, visited and next-word access of the apply a random 8-byte one (0.48 ms); the pass reads the
// words sequentially and finalises the nonzero ones.
__global__ __launch_bounds__(kBlock) void msbfs_td_apply_rows_kernel(int64_t rows, MsBfsOp op,
                                                                     const int64_t* __restrict__ push_rp,
                                                                     int32_t* __restrict__ queue, int64_t* __restrict__ qoff,
                                                                     unsigned long long* __restrict__ packed,
                                                                     unsigned long long* __restrict__ live_out) {
    __shared__ WaveStage ws;
    __shared__ unsigned long long red[kBlock / kWave];
    WaveApp app{ws};
    unsigned long long lv = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x0 = (int64_t)blockIdx.x * blockDim.x; x0 < rows; x0 += stride) {  // block-uniform trips
        const int64_t u = x0 + threadIdx.x;
        bool take = false;
        int64_t deg = 0;
        if (u < rows) {
            const unsigned long long acc = op.Fout[op.pos(u)];
            if (acc) {
                op.finalize(u, acc);
                const unsigned long long nw = op.Fout[op.pos(u)];
                lv |= nw;
                take = nw != 0ull;
                if (take) deg = push_rp[u + 1] - push_rp[u];
            }
        }
        app.append(take, (int32_t)u, deg, queue, qoff, packed);
    }
    app.final(queue, qoff, packed);
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) lv |= __shfl_xor(lv, o, kWave);
    if (lane_id() == 0) red[wave_id()] = lv;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / kWave; ++w) lv |= red[w];
        if (lv & ~*(volatile unsigned long long*)live_out) atomicOr(live_out, lv);
    }
}

// ---------------- weighted shortest distance (frontier Bellman-Ford) ----------------
// An edge without the weight property carries kWeightAbsent: a message crossing it is an error, as
// in Fulgora; distances may be negative, so an absent DISTANCE is reported as INT64_MIN.
constexpr int32_t kWeightAbsent = INT32_MIN;

// A superstep edge-balanced: the frontier carries each row's first edge number
// (qoff), and each thread takes kTdEdgesPerThread consecutive edges of the whole frontier after one
// binary search, so a hub row's 10^5 in-entries are spread over the grid instead of holding one lane
// group for the superstep (RMAT-20, weights 1..255, unbounded: 15.8 ms with the lane groups).
//
// The supersteps are controlled on the device (round 6, as the delta-stepping steps): superstep t's push
// and apply take the frontier count from a ring the previous apply filled, and its state (done, the
// superstep count) from the push's decision; the host enqueues supersteps in batches and reads the state
// once per batch instead of twice per superstep.
constexpr int kSdRing = 4;  // decision / counter rings of the device-controlled SD loops
struct SdSuper {      // superstep t's decision, ring slot t % kSdRing
    int32_t done;     // no superstep from t on
    int32_t levels;   // the supersteps counted so far (as the host loop counted them)
};
struct SdPush {
    const int64_t* rp;
    const int32_t* col;
    const int32_t* wt;
    int32_t* frontier[2];         // superstep t reads frontier[t & 1] (+ qoff), its apply writes [(t + 1) & 1]
    int64_t* qoff[2];
    unsigned long long* fr;       // [kSdRing] superstep t's frontier, packed (rows << kPackShift) | edges
    unsigned long long* tsz;      // [kSdRing] rows superstep t touched
    SdSuper* st;                  // [kSdRing]
    long long* msg;
    long long* best;
    long long* dist;
    int32_t* touched;
    int32_t* err;
    int32_t t;
};
__device__ __forceinline__ SdSuper sd_super_decide(const SdPush& a, int64_t* nq, int64_t* mf) {
    const SdSuper p = a.st[(a.t + kSdRing - 1) % kSdRing];
    const unsigned long long h = a.fr[a.t % kSdRing];
    *nq = (int64_t)(h >> kPackShift);
    *mf = (int64_t)(h & kEdgeMask);
    SdSuper c = p;
    if (p.done) return c;
    if (*nq == 0) {
        c.done = 1;
    } else if (*mf == 0) {  // the frontier's rows have no entries: the superstep sends nothing, the run ends
        c.done = 1;
        c.levels = a.t;
    } else {
        c.levels = a.t;
    }
    return c;
}
__global__ __launch_bounds__(kBlock) void sd_push_q_kernel(SdPush a) {
    __shared__ SdSuper s_c;
    __shared__ int64_t s_nq, s_mf;
    if (threadIdx.x == 0) {
        int64_t nq, mf;
        s_c = sd_super_decide(a, &nq, &mf);
        s_nq = nq;
        s_mf = mf;
        if (blockIdx.x == 0) {
            a.st[a.t % kSdRing] = s_c;
            if (!s_c.done) {  // the apply's next frontier and the next push's touched count start at zero
                a.fr[(a.t + 1) % kSdRing] = 0ull;
                a.tsz[(a.t + 1) % kSdRing] = 0ull;
            }
        }
    }
    __syncthreads();
    if (s_c.done) return;
    const int64_t nq = s_nq, mf = s_mf;
    const int32_t* __restrict__ frontier = a.frontier[a.t & 1];
    const int64_t* __restrict__ qoff = a.qoff[a.t & 1];
    unsigned long long* tsize = a.tsz + a.t % kSdRing;
    const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_tile = nthreads * kTdEdgesPerThread;
    const int64_t tiles = (mf + per_tile - 1) / per_tile;
    for (int64_t t = 0; t < tiles; ++t) {
        if ((t * nthreads + (int64_t)blockIdx.x * blockDim.x) * kTdEdgesPerThread >= mf) break;  // block-uniform
        const int64_t e0 = (t * nthreads + tid) * kTdEdgesPerThread;
        int64_t i = 0, next_bound = 0;
        if (e0 < mf) {
            int64_t lo = 0, hi = nq - 1;
            while (lo < hi) {
                const int64_t mid = (lo + hi + 1) >> 1;
                if (qoff[mid] <= e0) lo = mid; else hi = mid - 1;
            }
            i = lo;
            next_bound = i + 1 < nq ? qoff[i + 1] : mf;
        }
#pragma unroll
        for (int k = 0; k < kTdEdgesPerThread; ++k) {
            const int64_t e = e0 + k;
            bool first = false;
            int32_t u = 0;
            if (e < mf) {
                while (e >= next_bound) {
                    ++i;
                    next_bound = i + 1 < nq ? qoff[i + 1] : mf;
                }
                const int32_t w = frontier[i];
                const int64_t j = a.rp[w] + (e - qoff[i]);
                u = a.col[j];
                const int32_t wk = a.wt ? a.wt[j] : 1;
                if (wk == kWeightAbsent) {  // the edge function would throw (ShortestDistanceVertexProgram.java:69)
                    *a.err = 1;
                } else {
                    const long long cand = a.msg[w] + (long long)wk;
                    // a read first (past L1, as in sd_near_kernel): a candidate no better than the best so far
                    // takes no atomic
                    if (cand < __hip_atomic_load(&a.best[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                        first = atomicMin(&a.best[u], cand) == LLONG_MAX;
                }
            }
            wave_append(first, u, a.touched, tsize);
        }
    }
}

// The apply of a superstep: touched rows whose candidate beats their distance take it and form the next
// frontier, with its first edge numbers (for sd_push_q_kernel)
__global__ __launch_bounds__(kBlock) void sd_apply_q_kernel(SdPush a) {
    __shared__ WaveStage ws;
    if (a.st[a.t % kSdRing].done) return;
    WaveApp app{ws};
    const int32_t* __restrict__ touched = a.touched;
    const int64_t tsize = (int64_t)a.tsz[a.t % kSdRing];
    long long* __restrict__ best = a.best;
    long long* __restrict__ dist = a.dist;
    long long* __restrict__ msg = a.msg;
    const int64_t* __restrict__ rp = a.rp;
    int32_t* next_frontier = a.frontier[(a.t + 1) & 1];
    int64_t* next_qoff = a.qoff[(a.t + 1) & 1];
    unsigned long long* packed = a.fr + (a.t + 1) % kSdRing;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x0 = (int64_t)blockIdx.x * blockDim.x; x0 < tsize; x0 += stride) {  // block-uniform trips
        const int64_t i = x0 + threadIdx.x;
        bool improved = false;
        int32_t u = 0;
        int64_t du = 0;
        if (i < tsize) {
            u = touched[i];
            const long long b = best[u];
            best[u] = LLONG_MAX;
            if (dist[u] == LLONG_MIN || dist[u] > b) {
                dist[u] = b;
                msg[u] = b;
                improved = true;
                du = rp[u + 1] - rp[u];
            }
        }
        app.append(improved, u, du, next_frontier, next_qoff, packed);
    }
    app.final(next_frontier, next_qoff, packed);
}

// ---------------- weighted shortest distance, unbounded hops (near-far delta-stepping) ----------------
// When the hop bound cannot bind (maxDepth >= rows - 1) and no weight is negative, the hop-bounded
// minimum is the plain shortest distance (a shortest path can be taken simple: <= rows - 1 hops), so
// the supersteps can be replaced by delta-stepping (Meyer & Sanders; the GPU
// near-far pile of Davidson et al.): the rows below the threshold T are relaxed pass by pass (the near
// queue), the rest wait in a far pile, and T rises by delta once the near queue is empty.  The frontier
// Bellman-Ford above re-relaxes a row every time a longer-hop path improves it; here a row is relaxed
// only while its distance is below T, so most rows are relaxed once.  The reported distances are the
// Bellman-Ford ones bit for bit (integers, a min); an absent weight on an edge out of a reached row
// fails the run as there (every reached row is relaxed at least once, at its final distance).
// Queues hold each row at most once: near entries by a pass stamp, far entries by a flag.
//
// The passes are controlled on the device (round 6): a step is sd_split_kernel (which moves the far pile
// when the near queue came out empty) and sd_near_kernel (one near pass); both take the step's decision
// from the state ring and the previous step's counters, as the DO-BFS levels do, and the host enqueues
// steps in batches and reads the state once per batch.  (A host read per pass cost ~50 us of every pass:
// RMAT-22, 10 passes, 0.5 of 3.0 ms.)
struct SdState {     // a step's decision, ring slot = step % kSdRing
    long long T;     // the threshold: the near pass relaxes rows below it
    int32_t fc;      // the far pile rows join (far[fc], its size fsz[fc])
    int32_t split;   // this step moved the far pile before its near pass
    int32_t done;
    int32_t end_step;  // done: the step that found nothing left
};

// Distances are 64-bit, or 32-bit when every distance the run can store fits (sd_delta_stepping: a row's
// first distance is a path of at most rows - 1 entries, later ones only fall): half the bytes per
// random distance read and atomicMin, so twice the rows per cached line.
template <class D> struct DistTraits;
template <> struct DistTraits<long long> { static constexpr long long kNone = LLONG_MAX; };
template <> struct DistTraits<unsigned int> { static constexpr unsigned int kNone = UINT_MAX; };

template <class D>
struct SdStep {
    const int64_t* rp;
    const int32_t* col;
    const int32_t* wt;
    D* dist;                    // DistTraits<D>::kNone: unreached
    int32_t* nq[2];             // near queues: step s relaxes nq[s & 1] (and its first-edge offsets qo),
    int64_t* qo[2];             // its near pass appends to nq[(s + 1) & 1]
    unsigned long long* nctr;   // [kSdRing] step s's near queue, packed (rows << kPackShift) | edges
    int32_t* far[2];            // far piles and their sizes
    unsigned long long* fsz;    // [2]
    int32_t* far_flag;
    int32_t* stamp;             // near-queue stamps (pass = step + 1)
    unsigned long long* fmin;   // [kSdRing] smallest distance seen in the far pile up to step s
    SdState* st;                // [kSdRing]
    unsigned long long* passes; // near passes run (a near queue with rows)
    int32_t* err;
    long long delta;
    int32_t step;
};

// Step s's decision (every block of both kernels computes it from the same completed inputs): relax the
// near queue when it has entries; else stop when the far pile is empty; else move the far pile, with the
// threshold past the previous one by delta, or to the bucket of the smallest far distance seen when that
// lies further (the host version's two split attempts; any threshold sequence gives the same distances,
// the bucket only decides how much is relaxed again)
template <class D>
__device__ SdState sd_decide(const SdStep<D>& a) {
    const int ps = (a.step + kSdRing - 1) % kSdRing;
    const SdState p = a.st[ps];
    SdState c = p;
    c.split = 0;
    if (p.done) return c;
    if ((a.nctr[a.step % kSdRing] & kEdgeMask) > 0) return c;
    if (a.fsz[p.fc] == 0) {
        c.done = 1;
        c.end_step = a.step;
        return c;
    }
    long long t2 = p.T + a.delta;
    const unsigned long long m = a.fmin[ps];
    if (m != ULLONG_MAX) {
        const long long jump = ((long long)m / a.delta + 1) * a.delta;
        t2 = jump > t2 ? jump : t2;
    }
    c.T = t2;
    c.fc = p.fc ^ 1;
    c.split = 1;
    return c;
}

// The far pile at a threshold change: rows now below T join the step's near queue, rows below the previous
// threshold were relaxed at their final distance already (dropped), the others stay (their smallest
// distance goes to fmin[step]).
template <class D>
__global__ __launch_bounds__(kBlock) void sd_split_kernel(SdStep<D> a) {
    __shared__ SdState s_st;
    __shared__ long long s_tprev;
    __shared__ WaveStage ws;
    if (threadIdx.x == 0) {
        s_st = sd_decide(a);
        s_tprev = a.st[(a.step + kSdRing - 1) % kSdRing].T;
        if (blockIdx.x == 0) a.st[a.step % kSdRing] = s_st;
    }
    __syncthreads();
    if (!s_st.split) return;
    WaveApp app{ws};
    const int from = s_st.fc ^ 1;
    const int64_t fsize = (int64_t)a.fsz[from];
    const int32_t* __restrict__ far = a.far[from];
    const long long T = s_st.T, t_prev = s_tprev;
    int32_t* nq = a.nq[a.step & 1];
    int64_t* qo = a.qo[a.step & 1];
    unsigned long long* packed = a.nctr + a.step % kSdRing;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    unsigned long long mk = ULLONG_MAX;
    for (int64_t x0 = (int64_t)blockIdx.x * blockDim.x; x0 < fsize; x0 += stride) {  // block-uniform trips
        const int64_t i = x0 + threadIdx.x;
        bool to_near = false, keep = false;
        int32_t u = 0;
        int64_t du = 0;
        if (i < fsize) {
            u = far[i];
            const long long d = (long long)a.dist[u];
            keep = d >= T;
            to_near = !keep && d >= t_prev;
            if (keep) mk = (unsigned long long)d < mk ? (unsigned long long)d : mk;
            else a.far_flag[u] = 0;
            if (to_near) du = a.rp[u + 1] - a.rp[u];
        }
        app.append(to_near, u, du, nq, qo, packed);
        wave_append(keep, u, a.far[s_st.fc], a.fsz + s_st.fc);
    }
    app.final(nq, qo, packed);
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        const unsigned long long t = __shfl_xor(mk, o, kWave);
        mk = t < mk ? t : mk;
    }
    if (lane_id() == 0 && mk != ULLONG_MAX) atomicMin(a.fmin + a.step % kSdRing, mk);
}

// One near pass, edge-balanced over the step's near queue (first-edge numbers, one binary search per 4
// edges per thread).  Block 0 also keeps the rings: the next step's output counter and far minimum start
// empty, the far minimum carries over a step without a split, and after a split the emptied pile's size
// is reset.
template <class D>
__global__ __launch_bounds__(kBlock) void sd_near_kernel(SdStep<D> a) {
    __shared__ SdState s_st;
    __shared__ long long s_nq, s_mf;
    __shared__ WaveStage ws;
    const int cs = a.step % kSdRing;
    if (threadIdx.x == 0) {
        s_st = a.st[cs];
        const unsigned long long h = a.nctr[cs];
        s_nq = (long long)(h >> kPackShift);
        s_mf = (long long)(h & kEdgeMask);
        if (blockIdx.x == 0 && !s_st.done) {
            a.nctr[(a.step + 2) % kSdRing] = 0ull;
            a.fmin[(a.step + 2) % kSdRing] = ULLONG_MAX;
            if (s_st.split) a.fsz[s_st.fc ^ 1] = 0ull;
            else atomicMin(a.fmin + cs, a.fmin[(a.step + kSdRing - 1) % kSdRing]);
            if (s_nq > 0) a.passes[0] += 1;  // (as the host-driven passes counted: a queue with rows)
        }
    }
    __syncthreads();
    if (s_st.done || s_mf == 0) return;
    WaveApp app{ws};
    const int64_t nq = s_nq, mf = s_mf;
    const long long T = s_st.T;
    const int32_t pass = a.step + 1;
    const int32_t* __restrict__ near = a.nq[a.step & 1];
    const int64_t* __restrict__ qoff = a.qo[a.step & 1];
    int32_t* near_next = a.nq[(a.step + 1) & 1];
    int64_t* qoff_next = a.qo[(a.step + 1) & 1];
    unsigned long long* packed = a.nctr + (a.step + 1) % kSdRing;
    int32_t* far = a.far[s_st.fc];
    unsigned long long* far_size = a.fsz + s_st.fc;
    unsigned long long fm = ULLONG_MAX;  // this lane's smallest distance that stays in the far pile
    const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_tile = nthreads * kTdEdgesPerThread;
    const int64_t tiles = (mf + per_tile - 1) / per_tile;
    for (int64_t t = 0; t < tiles; ++t) {
        if ((t * nthreads + (int64_t)blockIdx.x * blockDim.x) * kTdEdgesPerThread >= mf) break;  // block-uniform
        const int64_t e0 = (t * nthreads + tid) * kTdEdgesPerThread;
        int64_t i = 0, next_bound = 0;
        if (e0 < mf) {
            int64_t lo = 0, hi = nq - 1;
            while (lo < hi) {
                const int64_t mid = (lo + hi + 1) >> 1;
                if (qoff[mid] <= e0) lo = mid; else hi = mid - 1;
            }
            i = lo;
            next_bound = i + 1 < nq ? qoff[i + 1] : mf;
        }
#pragma unroll
        for (int k = 0; k < kTdEdgesPerThread; ++k) {
            const int64_t e = e0 + k;
            bool to_near = false, to_far = false;
            int32_t u = 0;
            int64_t du = 0;
            if (e < mf) {
                while (e >= next_bound) {
                    ++i;
                    next_bound = i + 1 < nq ? qoff[i + 1] : mf;
                }
                const int32_t w = near[i];
                const int64_t j = a.rp[w] + (e - qoff[i]);
                u = a.col[j];
                const int32_t wk = a.wt ? a.wt[j] : 1;
                if (wk == kWeightAbsent) {  // the edge function would throw (ShortestDistanceVertexProgram.java:69)
                    *a.err = 1;
                } else {
                    // dist[w] now: it only fell since w was queued
                    const long long nd = (long long)a.dist[w] + (long long)wk;
                    // the prefilter reads past L1 (agent scope): a hub row's entry is hit from every XCD at
                    // once, and a stale L1 copy would send each of those lanes to the atomic
                    if (nd < (long long)__hip_atomic_load(&a.dist[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &&
                        nd < (long long)atomicMin(&a.dist[u], (D)nd)) {
                        if (nd < T) {
                            to_near = atomicExch(&a.stamp[u], pass) != pass;
                            if (to_near) du = a.rp[u + 1] - a.rp[u];
                        } else {
                            to_far = atomicExch(&a.far_flag[u], 1) == 0;
                            fm = (unsigned long long)nd < fm ? (unsigned long long)nd : fm;
                        }
                    }
                }
            }
            app.append(to_near, u, du, near_next, qoff_next, packed);
            wave_append(to_far, u, far, far_size);
        }
    }
    app.final(near_next, qoff_next, packed);
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        const unsigned long long x = __shfl_xor(fm, o, kWave);
        fm = x < fm ? x : fm;
    }
    if (lane_id() == 0 && fm != ULLONG_MAX) atomicMin(a.fmin + cs, fm);
}

// The superstep start: distances absent, best empty, the seed at 0 as superstep 1's frontier.
__global__ void sd_super_init_kernel(SdPush a, int64_t rows, int32_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += (int64_t)gridDim.x * blockDim.x) {
        a.dist[i] = i == seed ? 0ll : LLONG_MIN;
        a.best[i] = LLONG_MAX;
        if (i == seed) a.msg[i] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.frontier[1][0] = seed;
        a.qoff[1][0] = 0;
        for (int k = 0; k < kSdRing; ++k) {
            a.fr[k] = 0ull;
            a.tsz[k] = 0ull;
        }
        a.fr[1 % kSdRing] = (1ull << kPackShift) | (unsigned long long)(a.rp[seed + 1] - a.rp[seed]);
        a.st[0] = SdSuper{0, 0};
        *a.err = 0;
    }
}

// The start: every row unreached, no stamps or far flags, the seed at 0 as step 0's near queue, the ring
// empty, the state before step 0: threshold delta, far pile 0.
template <class D>
__global__ void sd_init_kernel(SdStep<D> a, int64_t rows, int32_t seed, long long delta) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += (int64_t)gridDim.x * blockDim.x) {
        a.dist[i] = i == seed ? (D)0 : DistTraits<D>::kNone;
        a.stamp[i] = 0;
        a.far_flag[i] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.nq[0][0] = seed;
        a.qo[0][0] = 0;
        a.nctr[0] = (1ull << kPackShift) | (unsigned long long)(a.rp[seed + 1] - a.rp[seed]);
        for (int k = 1; k < kSdRing; ++k) a.nctr[k] = 0ull;
        for (int k = 0; k < kSdRing; ++k) a.fmin[k] = ULLONG_MAX;
        a.fsz[0] = a.fsz[1] = 0ull;
        a.passes[0] = 0ull;
        *a.err = 0;
        SdState s0{};
        s0.T = delta;
        a.st[kSdRing - 1] = s0;
    }
}

// Weight statistics of a CSR for the delta-stepping gate and its automatic delta: [0] the smallest
// weight, [1] the sum, [2] the count, [3] the largest (absent weights excluded).
__global__ void sd_weight_stats_kernel(const int32_t* __restrict__ wt, int64_t nnz, long long* __restrict__ out) {
    long long mn = LLONG_MAX, mx = LLONG_MIN, sum = 0, cnt = 0;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nnz; j += (int64_t)gridDim.x * blockDim.x) {
        const int32_t w = wt[j];
        if (w == kWeightAbsent) continue;
        mn = w < mn ? w : mn;
        mx = w > mx ? w : mx;
        sum += w;
        ++cnt;
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        const long long a = __shfl_xor(mn, o, kWave), b = __shfl_xor(mx, o, kWave);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
        sum += __shfl_xor(sum, o, kWave);
        cnt += __shfl_xor(cnt, o, kWave);
    }
    if (lane_id() == 0) {
        atomicMin(&out[0], mn);
        atomicMax(&out[3], mx);
        atomicAdd((unsigned long long*)&out[1], (unsigned long long)sum);
        atomicAdd((unsigned long long*)&out[2], (unsigned long long)cnt);
    }
}


// The peers' candidates for own rows, received at the send-list positions (send_src[k] = own row)
// Sharded supersteps, edge-balanced as sd_push_q_kernel (round 6; the 16-lane row groups of
// ssd_push_kernel held a hub row's group for the superstep): the frontier carries each row's first edge
// number, targets are compact positions, a candidate for a peer's row stays in its halo slot of best
// (the reverse exchange takes it to the owner), only own rows are listed as touched.
struct SsdPushQ {
    const int64_t* rp;
    const int32_t* col;
    const int32_t* wt;
    const int32_t* frontier;
    const int64_t* qoff;
    int64_t nq, mf;
    const long long* msg;
    long long* best;
    int tbits;
    int32_t* touched;
    unsigned long long* tsize;
    int32_t* err;
};
__global__ __launch_bounds__(kBlock) void ssd_push_q_kernel(SsdPushQ a) {
    const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_tile = nthreads * kTdEdgesPerThread;
    const int64_t tiles = (a.mf + per_tile - 1) / per_tile;
    for (int64_t t = 0; t < tiles; ++t) {
        if ((t * nthreads + (int64_t)blockIdx.x * blockDim.x) * kTdEdgesPerThread >= a.mf) break;  // block-uniform
        const int64_t e0 = (t * nthreads + tid) * kTdEdgesPerThread;
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
        for (int k = 0; k < kTdEdgesPerThread; ++k) {
            const int64_t e = e0 + k;
            bool first = false;
            int32_t u = 0;
            if (e < a.mf) {
                while (e >= next_bound) {
                    ++i;
                    next_bound = i + 1 < a.nq ? a.qoff[i + 1] : a.mf;
                }
                const int32_t w = a.frontier[i];
                const int64_t j = a.rp[w] + (e - a.qoff[i]);
                u = a.col[j];
                const int32_t wk = a.wt ? a.wt[j] : 1;
                if (wk == kWeightAbsent) {
                    *a.err = 1;
                } else {
                    const long long cand = a.msg[w] + (long long)wk;
                    if (cand < __hip_atomic_load(&a.best[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                        first = atomicMin(&a.best[u], cand) == LLONG_MAX && (u >> a.tbits) == 0;
                }
            }
            wave_append(first, u, a.touched, a.tsize);
        }
    }
}

// The halo slots of every peer's run back to "no candidate" once sent, one launch per shard (a fill per
// peer was 7 launches per superstep and shard at P = 8: 0.20 of 2.89 ms per shard at RMAT-22)
struct SlotRuns {
    long long* p[64];
    int64_t n[64];
};
__global__ __launch_bounds__(kBlock) void ssd_reset_slots_kernel(SlotRuns r) {
    long long* __restrict__ p = r.p[blockIdx.y];
    const int64_t n = r.n[blockIdx.y];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = LLONG_MAX;
}

// sd_apply_q_kernel's apply with the counts from the host (for ssd_push_q_kernel)
__global__ __launch_bounds__(kBlock) void ssd_apply_q_kernel(const int32_t* __restrict__ touched, int64_t tsize,
                                                             long long* __restrict__ best, long long* __restrict__ dist,
                                                             long long* __restrict__ msg, const int64_t* __restrict__ rp,
                                                             int32_t* next_frontier, int64_t* next_qoff,
                                                             unsigned long long* packed) {
    __shared__ WaveStage ws;
    WaveApp app{ws};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x0 = (int64_t)blockIdx.x * blockDim.x; x0 < tsize; x0 += stride) {  // block-uniform trips
        const int64_t i = x0 + threadIdx.x;
        bool improved = false;
        int32_t u = 0;
        int64_t du = 0;
        if (i < tsize) {
            u = touched[i];
            const long long b = best[u];
            best[u] = LLONG_MAX;
            if (dist[u] == LLONG_MIN || dist[u] > b) {
                dist[u] = b;
                msg[u] = b;
                improved = true;
                du = rp[u + 1] - rp[u];
            }
        }
        app.append(improved, u, du, next_frontier, next_qoff, packed);
    }
    app.final(next_frontier, next_qoff, packed);
}

__global__ void ssd_recv_kernel(const long long* __restrict__ rbuf, const int32_t* __restrict__ send_src, int64_t nrecv,
                                long long* __restrict__ best, int32_t* __restrict__ touched,
                                unsigned long long* __restrict__ tsize) {
    const int64_t iters = (nrecv + (int64_t)gridDim.x * blockDim.x - 1) / ((int64_t)gridDim.x * blockDim.x);
    for (int64_t it = 0; it < iters; ++it) {
        const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + it * (int64_t)gridDim.x * blockDim.x;
        bool first = false;
        int32_t u = 0;
        if (k < nrecv) {
            const long long v = rbuf[k];
            if (v != LLONG_MAX) {
                u = send_src[k];
                first = atomicMin(&best[u], v) == LLONG_MAX;
            }
        }
        wave_append(first, u, touched, tsize);
    }
}

__global__ void fill_ll_kernel(long long* p, int64_t n, long long v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

struct BfsCsrs {
    const Csr* push;
    const Csr* pull;
};

BfsCsrs pick_csrs(const Shard& sh, int direction) {
    if (direction == JG_DIR_BOTH) {
        if (!sh.both.present()) fail(JG_ERR_UNSUPPORTED, "BOTH traversal needs a graph built with JG_ADJ_BOTH");
        return {&sh.both, &sh.both};
    }
    // OUT traversal: push from u over out-rows; pull for v over in-rows (u -> v).  IN is the mirror.
    const Csr* push = direction == JG_DIR_OUT ? &sh.out : &sh.in;
    const Csr* pull = direction == JG_DIR_OUT ? &sh.in : &sh.out;
    if (!push->present() && !pull->present())
        fail(JG_ERR_UNSUPPORTED, "directed traversal needs JG_ADJ_OUT and/or JG_ADJ_IN");
    return {push->present() ? push : nullptr, pull->present() ? pull : nullptr};
}

// the pull adjacency of a traversal, as the key of its gathered vector's layout (Graph::vec_pos)
uint32_t adj_of(const Shard& sh, const BfsCsrs& c) { return c.pull == &sh.both ? JG_ADJ_BOTH : JG_ADJ_IN; }

// rows [0, live) of the pull adjacency have entries; from there on none (the degree-sorted empty suffix):
// no level after 0 reaches or finalises them
int64_t pull_live_rows(const Shard& sh, const BfsCsrs& c) {
    return c.pull && c.pull->empty_from >= 0 ? std::min(c.pull->empty_from, sh.rows) : sh.rows;
}

// Direction-optimising single-source BFS on one shard; depth (device, [rows]) receives the result.
// Returns levels run; *edges_out = adjacency entries of reached vertices (degree CSR).
}  // namespace

// The single-shard traversal's scratch, kept with the shard (callers allocate it before their timed
// region: a first call would otherwise time ~1 ms of allocations at RMAT-26).
// Trace markers (JG_TRACE_MARKS=1): an empty dispatch just before a program's t0 event and just after its
// t1 event, so tools/bench_trace.py cuts a rocprofv3 kernel trace of the bench process to exactly the
// event-timed regions.  Unset: no launch.
__global__ void region_begin_kernel() {}
__global__ void region_end_kernel() {}
void region_mark(hipStream_t s, bool begin) {
    static const bool on = [] {
        const char* e = std::getenv("JG_TRACE_MARKS");
        return e && std::atoi(e) != 0;
    }();
    if (!on) return;
    if (begin) region_begin_kernel<<<1, kWave, 0, s>>>();
    else region_end_kernel<<<1, kWave, 0, s>>>();
    JG_LAUNCH_CHECK();
}

__global__ void first_col_kernel(const int64_t* __restrict__ rp, const int32_t* __restrict__ col, int64_t rows,
                                 int32_t* __restrict__ first) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < rows; v += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = rp[v];
        first[v] = rp[v + 1] > j ? col[j] : -1;
    }
}

// Csr::first_col of a traversal's pull adjacency, built on first use (outside any timed region: the
// callers run it before their t0 event)
const int32_t* bfs_first_col(Shard& sh, const Csr& c) {
    if (c.first_col.size() != (size_t)std::max<int64_t>(c.rows, 1)) {
        DeviceGuard dg(sh);
        c.first_col.alloc(std::max<int64_t>(c.rows, 1));
        if (c.rows > 0) {
            first_col_kernel<<<grid_for(c.rows), kBlock, 0, sh.stream>>>(c.row_ptr.get(), c.col.get(), c.rows,
                                                                         c.first_col.get());
            JG_LAUNCH_CHECK();
        }
    }
    return c.first_col.peer();  // (the callers pass it to kernels under the shard's own guard)
}

void bfs_buffers(Shard& sh) {
    const int64_t rows = sh.rows;
    const int64_t words = (rows + 63) / 64;
    const size_t r1 = (size_t)std::max<int64_t>(rows, 1), w1 = (size_t)std::max<int64_t>(words, 1);
    for (int k = 0; k < 2; ++k) {
        if (sh.bfs_queue[k].size() != r1) sh.bfs_queue[k].alloc(r1);
        if (sh.bfs_qoff[k].size() != r1) sh.bfs_qoff[k].alloc(r1);
        if (sh.bfs_bm[k].size() != w1) sh.bfs_bm[k].alloc(w1);
    }
    if (sh.bfs_seen.size() != r1) sh.bfs_seen.alloc(r1);
    if (tune().bfs_td_split && sh.bfs_owner.size() != r1) sh.bfs_owner.alloc(r1);
    if (sh.bfs_ctr.size() != (size_t)kBfsRing) sh.bfs_ctr.alloc(kBfsRing);
    if (sh.bfs_state.size() != kBfsRing * sizeof(BfsState)) sh.bfs_state.alloc(kBfsRing * sizeof(BfsState));
}

namespace {

// end_ev (nullable) is recorded behind the last level launch, before the host reads the final state:
// the traversal's GPU span ends there (the state read-back is the host's control, not traversal work)
// tail = false: the depths of the empty suffix already hold -1 (bfs_run keeps them so: Shard::
// bfs_depth_tail_clean); on a BOTH traversal the traversal itself never reads or writes those rows, so the
// init skips them.
int dobfs_single(Ctx& ctx, Shard& sh, const BfsCsrs& c, int64_t source, int max_depth, int32_t* depth,
                 double* edges_out, const CcRoots* roots = nullptr, hipEvent_t end_ev = nullptr, bool tail = true,
                 const std::function<void()>* after_start = nullptr) {
    hipStream_t s = sh.stream;
    const int64_t rows = sh.rows;
    const Csr* push = c.push;
    const Csr* pull = c.pull;
    const Csr* degcsr = push ? push : pull;
    bfs_buffers(sh);
    BfsState* st = reinterpret_cast<BfsState*>(sh.bfs_state.get());
    if (roots) {  // every component's minimum-rank vertex with an edge starts at depth 0
        JG_HIP(hipMemsetAsync(sh.bfs_ctr.get(), 0, kBfsRing * sizeof(unsigned long long), s));
        // rows from roots->ne on (no edge) are neither read by the traversal (BOTH: no entry) nor labelled here
        // (cc_output_kernel gives them their rank)
        bfs_init_roots_kernel<<<grid_for((roots->ne + 3) / 4), kBlock, 0, s>>>(
            depth, roots->ne, *roots, degcsr->row_ptr.get(), sh.bfs_queue[0].get(), sh.bfs_qoff[0].get(),
            sh.bfs_ctr.get() + kBfsRing - 1, sh.bfs_seen.get(), st + kBfsRing - 1, (long long)degcsr->nnz);
        JG_LAUNCH_CHECK();
        if (after_start) (*after_start)();  // (CC: its output gathers, queued before the levels)
    } else {
        // BOTH (push = pull): rows from the empty suffix on have no entry at all, so no bottom-up probe or
        // top-down claim reads their depth or seen byte, only the caller's depth output does.  (Directed,
        // a row without pull entries may still be a pull neighbour whose depth a bottom-up level probes.)
        const int64_t live = pull && pull->empty_from >= 0 ? std::min(rows, pull->empty_from) : rows;
        const int64_t init_rows = tail || push != pull ? rows : live;
        bfs_init_kernel<<<grid_for(init_rows), kBlock, 0, s>>>(depth, init_rows, source, sh.bfs_queue[0].get(),
                                                          sh.bfs_qoff[0].get(), degcsr->row_ptr.get(),
                                                          (long long)degcsr->nnz, sh.bfs_ctr.get(), st,
                                                          sh.bfs_seen.get(), pull ? pull->row_ptr.get() : nullptr,
                                                          pull ? pull->empty_from : -1);
    }
    JG_LAUNCH_CHECK();
    BfsLevel a{};
    a.push_rp = push ? push->row_ptr.get() : nullptr;
    a.push_col = push ? push->col.get() : nullptr;
    a.pull_rp = pull ? pull->row_ptr.get() : nullptr;
    a.pull_col = pull ? pull->col.get() : nullptr;
    a.pull_first = pull ? bfs_first_col(sh, *pull) : nullptr;  // (the callers build it before their t0)
    a.deg_rp = degcsr->row_ptr.get();
    a.depth = depth;
    a.rows = rows;
    // rows from the pull adjacency's empty suffix on have no pull entries: no bottom-up level finds them
    // (their seen bytes are set at the start), so its probes skip them without reading their seen bytes
    // (RMAT-26 BOTH: ~34 M of 67 M rows)
    a.bu_rows = pull && pull->empty_from >= 0 ? std::min(rows, pull->empty_from) : rows;
    a.seen = sh.bfs_seen.get();
    a.ctr = sh.bfs_ctr.get();
    a.st = st;
    a.max_depth = max_depth;
    a.alpha = (double)(roots ? tune().bfs_alpha : tune().dobfs_alpha);
    a.beta = (double)tune().bfs_beta;
    a.owner = sh.bfs_owner.get();
    a.split_min = (long long)tune().bfs_td_split_min;
    a.split_max = (long long)tune().bfs_td_split_max;
    const int split_mode = tune().bfs_td_split, split_levels = tune().bfs_td_split_levels;
    // a fixed grid, both directions grid-stride: ~sqrt(rows) workgroups (tools/bfs_sweep.py, ms per
    // traversal: RMAT-20 0.164 / 0.141 / 0.140 / 0.157 at 256 / 512 / 1024 / 4096; RMAT-22 0.311 /
    // 0.310 / 0.412 at 1024 / 2048 / 8192; RMAT-26 3.46 / 2.45 / 2.19 / 2.11 / 2.14 / 2.76 at 512 / 1024
    // / 4096 / 8192 / 16384 / 65536): small levels pay less per block, big ones need the parallelism
    const int64_t sq = 1ll << ((bits_for((uint64_t)std::max<int64_t>(rows - 1, 1)) + 1) / 2);
    const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>(sq * tune().bfs_grid_mult / 4, 64), tune().bfs_grid);
    // Launches past the deepest of this shard's last few traversals are almost always no-ops that only
    // read the device state and exit (RMAT-20: 3-4 of the first batch's 10, ~4.2 us each at the full
    // grid): they go out with a small grid (bfs_tail_grid workgroups; a level that does have work there
    // still runs, grid-stride, just slower).  Single-source traversals only (the CC start is not history).
    int predicted = 0;
    if (!roots && tune().bfs_tail_grid > 0 && sh.bfs_hist_n >= 2)
        for (int k = 0; k < std::min(sh.bfs_hist_n, 4); ++k) predicted = std::max(predicted, sh.bfs_hist[k]);
    const unsigned tail_grid = (unsigned)std::min<int64_t>(std::max(tune().bfs_tail_grid, 1), grid);
    BfsState hs{};
    int level = 0;
    // (A persistent kernel running every level in one launch with a grid barrier between levels was
    // built in round 5 and measured slower: the barrier cost 6-19 us per level, profiles/r05/persistent/;
    // deleted in round 6.)
    // Levels are enqueued in batches, the host reading the device state once per batch: first
    // bfs_batch0 (RMAT traversals end within ~10 levels plus the one that finds the frontier empty),
    // then 4, 8, 16, ... (levels past the end are launched anyway and cost ~4 us each: a second batch
    // of 16 after 8 wasted ~14 of them at RMAT-26)
    int next_batch = 4;
    // (A first batch sized from the previous traversal's level count, to drop the 2-4 no-op levels of
    // ~4.6 us that end a 6-8-level RMAT-20 traversal, measured slower: 0.154 / 0.157 vs 0.140 / 0.128 ms,
    // since a deeper traversal then pays a host read and a second batch; profiles/r03/bfs/.)
    for (int batch = std::max(1, tune().bfs_batch0);; batch = next_batch, next_batch = std::min(next_batch * 2, 64)) {
        if (max_depth >= 0) batch = std::min(batch, max_depth + 1 - level);
        if (batch <= 0) fail(JG_ERR_STATE, "BFS level control did not terminate");  // level max_depth stops
        for (int k = 0; k < batch; ++k, ++level) {
            const int p = level & 1;
            a.level = level;
            a.queue_in = sh.bfs_queue[p].get();
            a.qoff_in = sh.bfs_qoff[p].get();
            a.queue_out = sh.bfs_queue[p ^ 1].get();
            a.qoff_out = sh.bfs_qoff[p ^ 1].get();
            a.bm_in = sh.bfs_bm[p].get();
            a.bm_out = sh.bfs_bm[p ^ 1].get();
            a.split = a.owner && (split_mode == 1 || (split_mode == 2 && level < 16 && ((split_levels >> level) & 1)));
            if (prof_enabled(ctx)) prof_record_start(ctx, sh);
            const unsigned lg = predicted > 0 && level >= predicted ? tail_grid : grid;
            bfs_level_kernel<<<lg, kBlock, 0, s>>>(a);
            JG_LAUNCH_CHECK();
            if (a.split) {
                bfs_td_claim_kernel<<<lg, kBlock, 0, s>>>(a);
                JG_LAUNCH_CHECK();
            }
            if (prof_enabled(ctx)) prof_record_stop(ctx, sh);
            if (debug_bfs()) {
                BfsState ds{};
                unsigned long long dc = 0;
                copy_d2h(&ds, st + level % kBfsRing, sizeof ds, s);
                copy_d2h(&dc, sh.bfs_ctr.get() + level % kBfsRing, sizeof dc, s);
                std::fprintf(stderr, "[jg bfs] level %d %s done %d next frontier %llu vertices %llu edges\n", level,
                             ds.bottom_up ? "bottom-up" : "top-down", ds.done, dc >> kPackShift, dc & kEdgeMask);
            }
        }
        if (end_ev) {
            JG_HIP(hipEventRecord(end_ev, s));
            region_mark(s, false);
        }
        copy_d2h(&hs, st + (level - 1) % kBfsRing, sizeof hs, s);
        if (hs.done) break;
    }
    if (edges_out) *edges_out = (double)hs.edges;
    if (!roots) {  // the history of level counts (bfs_tail_grid)
        for (int k = 3; k > 0; --k) sh.bfs_hist[k] = sh.bfs_hist[k - 1];
        sh.bfs_hist[0] = hs.levels;
        sh.bfs_hist_n = std::min(sh.bfs_hist_n + 1, 4);
    }
    return hs.levels;
}

// The owning shard and local row of each caller vid (local -1: not a vertex of the graph), one
// device lookup for the batch
void locals_of_vids(const Graph& g, const int64_t* vids, int64_t k, int64_t* local, int* shard) {
    std::vector<int64_t> d((size_t)k), pg((size_t)k);
    dense_of_vids(g, vids, k, d.data(), pg.data());
    for (int64_t i = 0; i < k; ++i) {
        local[i] = -1;
        shard[i] = -1;
        if (d[(size_t)i] < 0) continue;
        shard[i] = (int)(pg[(size_t)i] / g.S);
        local[i] = pg[(size_t)i] % g.S;
    }
}

int64_t local_of_vid(const Graph& g, int64_t vid, int* shard_out) {
    int64_t l = -1;
    int sh = -1;
    locals_of_vids(g, &vid, 1, &l, &sh);
    if (l >= 0) *shard_out = sh;
    return l;
}

// ---------------- sharded direction-optimising BFS (BOTH adjacency, halo plan) ----------------
// Each shard owns its rows and their depths (Shard::bfs_depth, [rows]).  Column ids of the BOTH CSR are
// compact: own rows [0, rows), then one segment per peer (its vertices this shard's rows touch).
// Frontiers cross shards as bits (a 14.7 M-vertex halo per shard at RMAT-26, P = 8, is 1.8 MB of words
// instead of 59 MB of int32 depths):
//  * bottom-up: each owner packs "depth == level" of its send lists into words (sw), the forward
//    exchange lands them in the readers' compact bitmaps (hb), and own unvisited rows probe own depths
//    and those bits;
//  * top-down: edge-parallel over the local frontier; own targets are claimed by CAS, a remote target is
//    stamped with a plain byte store (st8, zero between levels: a same-word atomicOr into a bitmap
//    queued behind the hub targets, RMAT-26 level 2 61 -> 146 us per shard), the stamps are packed into
//    the compact mark bitmap's segment words (mk) and cleared, the reverse exchange hands the marks to
//    the owners (rm), which claim the marked send-list rows.
// Level control lives on the device: one packed counter per shard and level
// ((vertices << 37) | entries) is summed over shards and ranks on the stream -- by the deciding kernels
// themselves over the shards' counter rings when the shards share a device, by a stream-ordered
// ncclAllReduce otherwise (over the host only in host-transport mode) -- and every kernel of level L takes
// Beamer's decision from level L-1's state and global counter, so the host enqueues whole batches of
// levels and reads the state once per batch (as dobfs_single does).  Both directions' words travel in
// every level's exchange (a few MB), so the host never needs the direction.  A level is four steps:
// sbfs_pre_kernel (pack the send-list bits | top-down push), sbfs_mid_kernel (- | pack the stamps), the
// exchange, sbfs_post_kernel (bottom-up probes | claim the received marks), then the counter reduction.
// Appends are wave-staged (WaveApp); the appending launches stay at ~2 K workgroups, since every
// workgroup ends with one device atomic on the level's counter (~88 per us at the memory side).
constexpr int kSRing = 4;  // level-state ring: level L reads slot L-1, writes L, zeroes L+1
// shard count the sharded traversal takes (CC checks it too before choosing its sharded path)
constexpr int kMaxShardsBfs = 64;
// bits of x at the set positions of m, packed into the low popc(m) bits (x's set bits only are visited)
__device__ __forceinline__ unsigned long long pext_u64(unsigned long long x, unsigned long long m) {
    x &= m;
    unsigned long long r = 0;
    while (x) {
        const int b = __ffsll(x) - 1;
        r |= 1ull << __popcll(m & ((1ull << b) - 1ull));
        x &= x - 1;
    }
    return r;
}

struct SBfsState {
    long long mu;     // entries of all shards not yet in any frontier (after this level's input frontier)
    long long edges;  // entries summed over every frontier so far (all shards)
    int bottom_up;    // direction this level runs in
    int done;         // traversal finished: this level and all later ones do nothing
    int levels;       // levels run (valid once done)
    int pad;
};

struct SBfsLevel {
    const int64_t* rp;
    const int32_t* col;
    const int32_t* first_col;       // [rows] each row's first column (Csr::first_col)
    int64_t rows;
    int64_t bu_rows;                // rows [bu_rows, rows) have no entry (BOTH empty suffix): never probed
    int32_t* dvec;                  // [rows] own depths
    uint8_t* seen;                  // [rows] 1: the row's depth is set (a byte probe instead of an int32 one)
    // Own frontiers as bitmaps over own rows, rotating by level: fb[L % 3] = the rows of depth L (set by
    // level L-1's claims: the bottom-up's ballot words, the top-down claims' atomicOr), fb[(L + 1) % 3]
    // receives level L's claims, fb[(L + 2) % 3] (level L-1's, read by nothing any more) is cleared by
    // level L's first kernel for level L+1.
    unsigned long long* fb[3];
    int64_t fw;                     // words per bitmap
    // Send lists as bitmaps over own rows: bit v of bq[q] = own row v is in peer q's send list (which
    // holds its rows in ascending order), bpre[q][w] = the send-list position of word w's first set bit
    const unsigned long long* bq;   // [P][fw]
    const int32_t* bpre;            // [P][fw + 1]
    unsigned long long* hb;         // compact bitmap: the peers' frontier bits, received forward (bottom-up)
    unsigned long long* mk;         // compact bitmap: this level's remote marks (top-down), packed from st8
    uint8_t* st8;                   // compact byte map: remote targets stamped by the top-down push
    uint8_t* dirty;                 // [C / 512] a stamp was set in this 512-byte chunk (zero between levels)
    unsigned long long* sw;         // send-list words: own frontier bits for the peers (bottom-up)
    const unsigned long long* rm;   // send-list words: the peers' marks of own rows, received back (top-down)
    const int32_t* queue_in;
    const int64_t* qoff_in;   // first frontier edge of each queue entry (edge-parallel top-down)
    int32_t* queue_out;
    int64_t* qoff_out;
    const int64_t* send_off;        // [P + 1] send-list element offsets per peer
    const int64_t* woff;            // [P + 1] send-list word offsets per peer
    const int64_t* rseg;            // [P] first position of each peer's segment in the compact vector
    const int64_t* rlen;            // [P] length of each peer's run in this shard's segment
    int P;
    const int32_t* send_src;        // own row of each send-list position
    unsigned long long* ctr;        // [kSRing] this shard's packed counters: slot L = level L's appends
    const unsigned long long* gsum[kMaxShardsBfs];  // counter rings whose sum is the global counter (by
    int nsum;                                       // value: the decision's loads issue together)
    SBfsState* st;                  // [kSRing] this shard's copy of the (identical) level decisions
    int64_t apply_x;                // workgroups per peer of the mark claims (the post kernel's x extent may be larger)
    int32_t level, max_depth;
    double alpha, beta;
    int64_t nrows;                  // rows of all shards (the beta rule)
};

__device__ __forceinline__ void sbfs_claim_bit(const SBfsLevel& a, int64_t v) {  // v joins level L+1's frontier
    atomicOr(&a.fb[(a.level + 1) % 3][v >> 6], 1ull << (v & 63));
}

__device__ __forceinline__ unsigned long long shfl_u64(unsigned long long v, int src) {
    const int lo = __shfl((int)(uint32_t)v, src, kWave), hi = __shfl((int)(uint32_t)(v >> 32), src, kWave);
    return ((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo;
}

// Level L's decision from level L-1's state and global counter (Beamer: bottom-up when the frontier's
// entries outweigh the unexplored ones / alpha, back top-down when the frontier falls below rows / beta);
// *nq / *mf = this shard's own input frontier.  Every shard and rank computes the same state.  Called by
// every lane of wave 0 (lane k < nsum loads counter ring k: one round trip for all the loads); the result
// is valid in lane 0.
__device__ SBfsState sbfs_decide(const SBfsLevel& a, long long* nq, long long* mf) {
    const int pl = (a.level + kSRing - 1) % kSRing;
    const int l = lane_id();
    const SBfsState p = a.st[pl];
    const unsigned long long own = a.ctr[pl];
    unsigned long long h = l < a.nsum ? a.gsum[l][pl] : 0ull;
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) h += shfl_u64(h, l ^ o);
    *nq = (long long)(own >> kPackShift);
    *mf = (long long)(own & kEdgeMask);
    if (p.done) return p;
    const long long gnf = (long long)(h >> kPackShift), gmf = (long long)(h & kEdgeMask);
    SBfsState c = p;
    c.mu = p.mu - gmf;
    c.edges = p.edges + gmf;
    if (gnf == 0 || (a.max_depth >= 0 && a.level >= a.max_depth)) {
        c.done = 1;
        c.levels = a.level;
        return c;
    }
    if (!p.bottom_up && (double)gmf > (double)c.mu / a.alpha) c.bottom_up = 1;
    else if (p.bottom_up && (double)gnf < (double)a.nrows / a.beta) c.bottom_up = 0;
    return c;
}

// The per-word passes run on a (blocks, P) grid: blockIdx.y is the peer whose run a block works on, so
// no word searches the per-peer offset tables (a scan of LDS-staged tables per word held them to 45-80 us
// per launch at RMAT-26, P = 8, round 4).  The row-parallel passes use the same grid flattened.

// bottom-up, owner side before the forward exchange: peer q's send-list words, bit b = send-list row b is
// in this level's frontier.  A thread per row word: its frontier bits at peer q's membership bits are
// extracted and ORed in at their send-list position (a send list holds its rows in ascending order), one or
// two atomics per word with a frontier row in q's list; the words start zero (the post kernel clears them
// after the exchange).  Reads 1 MB bitmaps instead of the 59 MB list of rows and their depths (RMAT-26,
// P = 8: 42 us per bottom-up level and shard through the list; a thread per send-list word that walked
// the row words it spans took 25 ms: the sparse tail of a list spans thousands of row words, round 6).
__device__ __forceinline__ void sbfs_pack_bits(const SBfsLevel& a) {
    const int q = blockIdx.y;
    unsigned long long* __restrict__ out = a.sw + a.woff[q];
    const unsigned long long* __restrict__ F = a.fb[a.level % 3];
    const unsigned long long* __restrict__ B = a.bq + (int64_t)q * a.fw;
    const int32_t* __restrict__ pre = a.bpre + (int64_t)q * (a.fw + 1);
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < a.fw; w += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long m = B[w], f = F[w] & m;
        if (!f) continue;
        const unsigned long long bits = pext_u64(f, m);
        const int64_t p = pre[w];
        const int o = (int)(p & 63);
        atomicOr(&out[p >> 6], bits << o);
        if (o && (bits >> (64 - o))) atomicOr(&out[(p >> 6) + 1], bits >> (64 - o));
    }
}

// top-down, edge-parallel over the local frontier's nq vertices and mf entries (as bfs_top_down): own
// neighbours are claimed by CAS, remote ones marked
__device__ __forceinline__ void sbfs_td_push(const SBfsLevel& a, int64_t nq, int64_t mf, WaveApp& app) {
    const int64_t bid = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    const int64_t nthreads = (int64_t)gridDim.x * gridDim.y * blockDim.x;
    const int64_t tid = bid * blockDim.x + threadIdx.x;
    const int64_t per_tile = nthreads * kTdEdgesPerThread;
    const int64_t tiles = (mf + per_tile - 1) / per_tile;
    const int32_t nd = a.level + 1;
    unsigned long long* packed = a.ctr + a.level % kSRing;
    for (int64_t t = 0; t < tiles; ++t) {
        if ((t * nthreads + bid * blockDim.x + wave_id() * kWave) * kTdEdgesPerThread >= mf) break;  // wave-uniform
        const int64_t e0 = (t * nthreads + tid) * kTdEdgesPerThread;
        int64_t i = 0, next_bound = 0;
        if (e0 < mf) {
            int64_t lo = 0, hi = nq - 1;
            while (lo < hi) {
                const int64_t mid = (lo + hi + 1) >> 1;
                if (a.qoff_in[mid] <= e0) lo = mid; else hi = mid - 1;
            }
            i = lo;
            next_bound = i + 1 < nq ? a.qoff_in[i + 1] : mf;
        }
#pragma unroll
        for (int k = 0; k < kTdEdgesPerThread; ++k) {
            const int64_t e = e0 + k;
            bool take = false;
            int32_t u = 0;
            int64_t deg = 0;
            if (e < mf) {
                while (e >= next_bound) {
                    ++i;
                    next_bound = i + 1 < nq ? a.qoff_in[i + 1] : mf;
                }
                const int32_t v = a.queue_in[i];
                u = a.col[a.rp[v] + (e - a.qoff_in[i])];
                if (u < a.rows) {
                    if (!a.seen[u] && atomicCAS(&a.dvec[u], -1, nd) == -1) {
                        a.seen[u] = 1;
                        sbfs_claim_bit(a, u);
                        take = true;
                        deg = a.rp[u + 1] - a.rp[u];
                    }
                } else {
                    a.st8[u] = 1;
                    a.dirty[u >> 9] = 1;
                }
            }
            app.append(take, u, deg, a.queue_out, a.qoff_out, packed);
        }
    }
}

// bottom-up over own rows [0, bu_rows): a neighbour is in the frontier if its depth (own) or bit (halo)
// says so; the flattened grid walks 64-row words, one per wave
__device__ __forceinline__ void sbfs_bottom_up(const SBfsLevel& a, WaveApp& app) {
    const int64_t words = (a.bu_rows + 63) / 64;
    constexpr int kWpb = kBlock / kWave;
    const int64_t bid = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    const int64_t wstride = (int64_t)gridDim.x * gridDim.y * kWpb;
    const int32_t nd = a.level + 1;
    unsigned long long* packed = a.ctr + a.level % kSRing;
    for (int64_t w = bid * kWpb + wave_id(); w < words; w += wstride) {  // wave-uniform
        const int64_t v = w * 64 + lane_id();
        bool found = false;
        int64_t deg = 0;
        if (v < a.bu_rows && !a.seen[v]) {
            const unsigned long long* __restrict__ F = a.fb[a.level % 3];
            auto in_frontier = [&](int32_t x) -> bool {
                return (bool)(((x < a.rows ? F[x >> 6] : a.hb[x >> 6]) >> (x & 63)) & 1ull);
            };
            // the first neighbour alone, from the dense first-column array (bfs_bottom_up)
            const int32_t u0 = a.first_col[v];
            if (u0 >= 0) found = in_frontier(u0);
            const int64_t j0 = a.rp[v], j1 = a.rp[v + 1];
            int64_t j = found ? j1 : j0 + 1;
            for (; j < j1 && !found; j += kBuBatch) {
                int32_t u[kBuBatch];
#pragma unroll
                for (int k = 0; k < kBuBatch; ++k) u[k] = a.col[j + k < j1 ? j + k : j1 - 1];
#pragma unroll
                for (int k = 0; k < kBuBatch; ++k) found |= in_frontier(u[k]);
            }
            if (found) {
                a.dvec[v] = nd;
                a.seen[v] = 1;
                deg = j1 - j0;
            }
        }
        const uint64_t word = __ballot(found);  // level L+1's frontier word (words past bu_rows stay zero)
        if (lane_id() == 0) a.fb[(a.level + 1) % 3][w] = word;
        app.append(found, (int32_t)v, deg, a.queue_out, a.qoff_out, packed);
    }
}

// top-down, owner side: the received words of peer q's run, kSbfsApplyChunk per wave and trip (lanes
// 0 .. 15 load); the rows of the set bits are claimed AW non-zero words at a time (lane b: the
// row of bit b).  Blocks from apply_x on leave: the claims end with one counter atomic per block.
// (64 words per wave and trip on 2048 workgroups measured 43 / 124 us per shard at RMAT-26's levels 1 and
// 2 against 21 / 100 us for this shape, round 6.)
constexpr int kSbfsApplyChunk = 16;
// Round-6 A/B at RMAT-26, P = 8 (tools/shard_sim.py, event time per shard; profiles/r06/sbfs/variants.log):
// 4 -> 8 words per trip in the claims 0.606 -> 0.601 ms (in the list-walking pack, since replaced, 0.583);
// 1024 -> 2048 / 4096 claim workgroups 0.578 / 0.573.
constexpr int kSbfsApplyWords = 8;
constexpr int64_t kSbfsApplyBlocks = 4096;
template <int AW>
__device__ __forceinline__ void sbfs_td_apply(const SBfsLevel& a, WaveApp& app) {
    const int q = blockIdx.y;
    const int64_t so = a.send_off[q], cnt = a.send_off[q + 1] - so, wo = a.woff[q], nw = a.woff[q + 1] - wo;
    const int32_t* __restrict__ src = a.send_src + so;
    const int64_t nwaves = (int64_t)a.apply_x * (kBlock / kWave);
    const int32_t nd = a.level + 1;
    unsigned long long* packed = a.ctr + a.level % kSRing;
    for (int64_t c0 = ((int64_t)blockIdx.x * (kBlock / kWave) + wave_id()) * kSbfsApplyChunk; c0 < nw;
         c0 += nwaves * kSbfsApplyChunk) {
        const unsigned long long mine =
            lane_id() < kSbfsApplyChunk && c0 + lane_id() < nw ? a.rm[wo + c0 + lane_id()] : 0ull;
        uint64_t nz = __ballot(mine != 0ull);
        while (nz) {  // wave-uniform
            unsigned long long word[AW];
            int32_t u[AW];
#pragma unroll
            for (int k = 0; k < AW; ++k) {
                const int l = nz ? __ffsll((unsigned long long)nz) - 1 : 0;
                word[k] = nz ? shfl_u64(mine, l) : 0ull;
                nz &= nz - 1;
                const int64_t x = (c0 + l) * 64 + lane_id();
                u[k] = src[x < cnt ? x : cnt - 1];  // bits past the run's end are never set
            }
#pragma unroll
            for (int k = 0; k < AW; ++k) {
                if (!word[k]) continue;  // wave-uniform
                bool take = false;
                int64_t deg = 0;
                if (((word[k] >> lane_id()) & 1ull) && !a.seen[u[k]] && atomicCAS(&a.dvec[u[k]], -1, nd) == -1) {
                    a.seen[u[k]] = 1;
                    sbfs_claim_bit(a, u[k]);
                    take = true;
                    deg = a.rp[u[k] + 1] - a.rp[u[k]];
                }
                app.append(take, u[k], deg, a.queue_out, a.qoff_out, packed);
            }
        }
    }
}

// First kernel of a level: the decision (block (0, 0) publishes it and zeroes the next level's counter),
// then this shard's send-list bits (bottom-up) or its top-down push.
__global__ __launch_bounds__(kBlock) void sbfs_pre_kernel(SBfsLevel a) {
    __shared__ SBfsState s_st;
    __shared__ long long s_nq, s_mf;
    __shared__ WaveStage ws;
    long long nq = 0, mf = 0;
    SBfsState c{};
    if (threadIdx.x < kWave) c = sbfs_decide(a, &nq, &mf);  // (wave 0: its lanes' loads issue together)
    if (threadIdx.x == 0) {
        s_st = c;
        s_nq = nq;
        s_mf = mf;
        if (blockIdx.x == 0 && blockIdx.y == 0) {
            a.st[a.level % kSRing] = c;
            if (!c.done) a.ctr[(a.level + 1) % kSRing] = 0ull;
        }
    }
    __syncthreads();
    if (s_st.done) return;
    {  // level L-1's frontier bitmap becomes level L+1's (cleared before level L+1's claims)
        unsigned long long* __restrict__ z = a.fb[(a.level + 2) % 3];
        const int64_t stride = (int64_t)gridDim.x * gridDim.y * blockDim.x;
        for (int64_t i = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x; i < a.fw; i += stride)
            z[i] = 0ull;
    }
    if (s_st.bottom_up) {
        sbfs_pack_bits(a);
    } else {
        WaveApp app{ws};
        sbfs_td_push(a, s_nq, s_mf, app);
        app.final(a.queue_out, a.qoff_out, a.ctr + a.level % kSRing);
    }
}

// Second kernel of a top-down level (a bottom-up level leaves at once): peer q's segment of stamp bytes
// into its mark words, every word written (zero or not: the words are the exchange's payload) and every
// set byte cleared for the next top-down level.  Chunks the push left clean (no dirty flag) are not read:
// the small top-down levels (a few thousand stamps) write zero words only.  Lane l loads bytes [8l, 8l + 8) of a 512-byte chunk
// (eight mark words) as one 8-byte load; word k is the byte masks of lanes 8k .. 8k + 7.  (One byte per
// lane and load ran 13-19 us per level and shard at RMAT-26, P = 8.)
__global__ __launch_bounds__(kBlock) void sbfs_mid_kernel(SBfsLevel a) {
    __shared__ int s_run;
    if (threadIdx.x == 0) {
        const SBfsState c = a.st[a.level % kSRing];
        s_run = !c.done && !c.bottom_up;
    }
    __syncthreads();
    if (!s_run) return;
    const int q = blockIdx.y;
    const int64_t len = a.rlen[q], seg = a.rseg[q], nw = (len + 63) / 64, nchunks = (nw + 7) / 8;
    uint8_t* __restrict__ stamp = a.st8 + seg;  // seg: a multiple of 2^tbits, so 8-byte aligned
    unsigned long long* __restrict__ mk = a.mk + (seg >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * (kBlock / kWave);
    const int l = lane_id();
    uint8_t* __restrict__ dirty = a.dirty + (seg >> 9);  // one flag per 512-byte chunk (segments start on one)
    for (int64_t c0 = (int64_t)blockIdx.x * (kBlock / kWave) + wave_id(); c0 < nchunks; c0 += nwaves * 2) {
        unsigned long long x[2];
        bool in[2];
        uint8_t dc[2];  // the chunk's dirty flag: a clean chunk's words are zero, its stamps are not read
#pragma unroll
        for (int k = 0; k < 2; ++k) dc[k] = c0 + k * nwaves < nchunks ? dirty[c0 + k * nwaves] : (uint8_t)0;
#pragma unroll
        for (int k = 0; k < 2; ++k) {  // two chunks per trip, both loads issued first
            const int64_t b0 = (c0 + k * nwaves) * 512 + 8 * l;  // this lane's first byte
            in[k] = dc[k] && b0 < len;
            x[k] = 0ull;
            if (in[k]) {
                if (b0 + 8 <= len) {
                    x[k] = *reinterpret_cast<const unsigned long long*>(stamp + b0);
                } else {
                    for (int64_t j = b0; j < len; ++j) x[k] |= (unsigned long long)stamp[j] << (8 * (j - b0));
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            unsigned m = 0;  // bit i: byte i of this lane's eight is set
#pragma unroll
            for (int i = 0; i < 8; ++i) m |= ((x[k] >> (8 * i)) & 0xffull) ? (1u << i) : 0u;
            unsigned long long word = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) word |= (unsigned long long)__shfl((int)m, 8 * (l & 7) + i, kWave) << (8 * i);
            const int64_t w = (c0 + k * nwaves) * 8 + l;  // lanes 0..7 write words 8c .. 8c + 7
            if (l < 8 && c0 + k * nwaves < nchunks && w < nw) mk[w] = word;
            if (l == 0 && dc[k]) dirty[c0 + k * nwaves] = 0;
            if (m) {  // clear this lane's stamps (the tail of the run byte by byte)
                const int64_t b0 = (c0 + k * nwaves) * 512 + 8 * l;
                if (b0 + 8 <= len) *reinterpret_cast<unsigned long long*>(stamp + b0) = 0ull;
                else for (int64_t j = b0; j < len; ++j) stamp[j] = 0;
            }
        }
    }
}

// Last kernel of a level (after the exchange): bottom-up probes, or the claims of the received marks.
template <int AW>
__global__ __launch_bounds__(kBlock) void sbfs_post_kernel(SBfsLevel a) {
    __shared__ SBfsState s_st;
    __shared__ WaveStage ws;
    if (threadIdx.x == 0) s_st = a.st[a.level % kSRing];
    __syncthreads();
    if (s_st.done) return;
    if (s_st.bottom_up) {  // the send-list words went out with the exchange: clear them for the next pack
        const int64_t nw = a.woff[a.P];
        const int64_t stride = (int64_t)gridDim.x * gridDim.y * blockDim.x;
        for (int64_t i = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x; i < nw; i += stride)
            a.sw[i] = 0ull;
    }
    if (!s_st.bottom_up && blockIdx.x >= a.apply_x) return;  // (block-uniform)
    WaveApp app{ws};
    if (s_st.bottom_up) sbfs_bottom_up(a, app);
    else sbfs_td_apply<AW>(a, app);
    app.final(a.queue_out, a.qoff_out, a.ctr + a.level % kSRing);
}

// Shards on one device: the exchange as one kernel that copies, for every (owner, reader) pair, the
// direction this level runs in (bottom-up: the owner's send-list words to the reader's segment; top-down:
// the reader's marks back to the owner's received words), with the decision read from the first shard.
struct SBfsCopyRun {
    const unsigned long long* fsrc;  // forward: owner's send-list words for the reader
    unsigned long long* fdst;        //          reader's bitmap segment for the owner
    const unsigned long long* rsrc;  // reverse: reader's marks about the owner's vertices
    unsigned long long* rdst;        //          owner's received words from the reader
    int64_t n;                       // words
};
__global__ __launch_bounds__(kBlock) void sbfs_copy_kernel(const SBfsCopyRun* __restrict__ runs, const SBfsState* st,
                                                           int slot) {
    const SBfsState c = st[slot];
    if (c.done) return;
    const SBfsCopyRun r = runs[blockIdx.y];
    const unsigned long long* __restrict__ s = c.bottom_up ? r.fsrc : r.rsrc;
    unsigned long long* __restrict__ d = c.bottom_up ? r.fdst : r.rdst;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < r.n; i += (int64_t)gridDim.x * blockDim.x)
        d[i] = s[i];
}

// Single-source start: depths (rows [0, init_rows): the caller keeps the empty suffix at -1), the
// level-0 queue, the counter ring (level -1's slot: the source's own frontier) and the level -1 state.
__global__ __launch_bounds__(kBlock) void sbfs_init_kernel(SBfsLevel a, int64_t init_rows, int64_t src, long long total) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x, tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t i = tid; i < init_rows; i += stride) {
        a.dvec[i] = i == src ? 0 : -1;
        a.seen[i] = i == src ? 1 : 0;  // (rows past the empty suffix are never read)
    }
    for (int64_t i = tid; i < a.fw; i += stride) {  // level 0's frontier bitmap: the source; level 1's: empty
        a.fb[0][i] = src >= 0 && i == (src >> 6) ? 1ull << (src & 63) : 0ull;
        a.fb[1][i] = 0ull;
    }
    for (int64_t i = tid; i < a.woff[a.P]; i += stride) a.sw[i] = 0ull;  // the pack ORs into zero words
    if (tid == 0) {
        const long long deg = src >= 0 ? (long long)(a.rp[src + 1] - a.rp[src]) : 0;
        if (src >= 0) {
            a.dvec[src] = 0;  // (also when the source lies in the skipped suffix: the caller refills it)
            a.seen[src] = 1;
            const_cast<int32_t*>(a.queue_in)[0] = (int32_t)src;
            const_cast<int64_t*>(a.qoff_in)[0] = 0;
        }
        for (int k = 0; k < kSRing; ++k) a.ctr[k] = 0ull;
        a.ctr[kSRing - 1] = src >= 0 ? (1ull << kPackShift) | (unsigned long long)deg : 0ull;
        SBfsState s0{};
        s0.mu = total;
        a.st[kSRing - 1] = s0;
    }
}

// Multi-root start (cc_root_eccentricity_sharded): an own row with an edge whose label is its own rank is
// its component's minimum-rank vertex, a level-0 root; appended to level -1's counter slot (zeroed by
// the caller).  Rows from r.ne on have no edge.
__global__ __launch_bounds__(kBlock) void sbfs_init_roots_kernel(SBfsLevel a, CcRoots r, long long total) {
    __shared__ WaveStage ws;
    WaveApp app{ws};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int32_t* queue = const_cast<int32_t*>(a.queue_in);
    int64_t* qoff = const_cast<int64_t*>(a.qoff_in);
    for (int64_t x0 = (int64_t)blockIdx.x * blockDim.x; x0 < a.rows; x0 += stride) {  // block-uniform trips
        const int64_t v = x0 + threadIdx.x;
        bool take = false;
        int64_t deg = 0;
        if (v < a.rows) {
            if (v < r.ne) {
                deg = a.rp[v + 1] - a.rp[v];
                take = deg > 0 && r.parent[v] == r.rank[v];
            }
            a.dvec[v] = take ? 0 : -1;
            a.seen[v] = take ? 1 : 0;
        }
        const uint64_t word = __ballot(take);  // level 0's frontier bitmap (64 consecutive rows per wave)
        if (lane_id() == 0 && v < a.rows) a.fb[0][v >> 6] = word;
        app.append(take, (int32_t)v, deg, queue, qoff, a.ctr + kSRing - 1);
    }
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.fw; i += stride) a.fb[1][i] = 0ull;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.woff[a.P]; i += stride) a.sw[i] = 0ull;
    app.final(queue, qoff, a.ctr + kSRing - 1);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        SBfsState s0{};
        s0.mu = total;
        a.st[kSRing - 1] = s0;
    }
}

// bq[q][w]: the membership bitmap of peer q's send list (grid (blocks, P))
__global__ __launch_bounds__(kBlock) void sbfs_bq_kernel(const int32_t* __restrict__ send_src,
                                                         const int64_t* __restrict__ send_off, int64_t fw,
                                                         unsigned long long* __restrict__ bq) {
    const int q = blockIdx.y;
    for (int64_t x = send_off[q] + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < send_off[q + 1];
         x += (int64_t)gridDim.x * blockDim.x) {
        const int32_t v = send_src[x];
        atomicOr(&bq[(int64_t)q * fw + (v >> 6)], 1ull << (v & 63));
    }
}

// The send lists as bitmaps (SBfsLevel::bq / bpre), built on a shard's first sharded traversal (before
// its timed region) and kept: the bitmaps on the device, the prefixes from a host pass over them.
void sbfs_send_bitmaps(Graph& g, Shard& sh) {
    const int64_t fw = std::max<int64_t>((sh.rows + 63) / 64, 1);
    const int P = g.P;
    if (sh.sbfs_bq.size() == (size_t)P * fw) return;
    const Halo& h = sh.halo_both;
    DeviceGuard dg(sh);
    sh.sbfs_bq.alloc((size_t)P * fw);
    JG_HIP(hipMemsetAsync(sh.sbfs_bq.get(), 0, sh.sbfs_bq.bytes(), sh.stream));
    {
        DevBuf<int64_t> so(P + 1);
        copy_h2d(so.get(), h.send_off.data(), (P + 1) * sizeof(int64_t), sh.stream);
        int64_t longest = 0;
        for (int q = 0; q < P; ++q) longest = std::max(longest, h.send_off[(size_t)q + 1] - h.send_off[(size_t)q]);
        if (longest > 0) {
            sbfs_bq_kernel<<<dim3(grid_for(longest, kBlock, 1024), (unsigned)P), kBlock, 0, sh.stream>>>(
                h.send_src.get(), so.get(), fw, sh.sbfs_bq.get());
            JG_LAUNCH_CHECK();
        }
        JG_HIP(hipStreamSynchronize(sh.stream));
    }
    std::vector<unsigned long long> bq((size_t)P * fw);
    copy_d2h(bq.data(), sh.sbfs_bq.get(), bq.size() * sizeof(unsigned long long), sh.stream);
    std::vector<int32_t> pre((size_t)P * (fw + 1));
    for (int q = 0; q < P; ++q) {
        const unsigned long long* b = bq.data() + (size_t)q * fw;
        int32_t* pq = pre.data() + (size_t)q * (fw + 1);
        int64_t c = 0;
        for (int64_t w = 0; w < fw; ++w) {
            pq[w] = (int32_t)c;
            c += __builtin_popcountll(b[w]);
        }
        pq[fw] = (int32_t)c;
        if (c != h.send_off[(size_t)q + 1] - h.send_off[(size_t)q])
            fail(JG_ERR_STATE, "sharded BFS: a send list repeats a row");
    }
    sh.sbfs_bpre.alloc(pre.size());
    copy_h2d(sh.sbfs_bpre.get(), pre.data(), pre.size() * sizeof(int32_t), sh.stream);
}

// The level counters of slot `slot` summed into every shard's global slot (gctr), on the streams: a
// grouped ncclAllReduce, or over the host in host-transport mode.  Shards sharing one device need no
// step (the deciding kernels sum the shards' rings).
void sbfs_reduce(Graph& g, const std::vector<unsigned long long*>& ctr, const std::vector<unsigned long long*>& gctr,
                 int slot) {
    Ctx& c = *g.ctx;
    if (c.logical) return;
    if (c.host_transport) {
        Shard& sh = *g.shards[0];
        DeviceGuard dg(sh);
        unsigned long long v = 0;
        copy_d2h(&v, ctr[0] + slot, sizeof v, sh.stream);
        int64_t s = (int64_t)v;  // packed: the fields sum independently (neither overflows)
        allreduce_sum_i64(g, &s, 1);
        v = (unsigned long long)s;
        copy_h2d(gctr[0] + slot, &v, sizeof v, sh.stream);
        return;
    }
    rccl_check(ncclGroupStart(), "ncclGroupStart");
    for (size_t i = 0; i < g.shards.size(); ++i) {
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        rccl_check(ncclAllReduce(ctr[i] + slot, gctr[i] + slot, 1, ncclUint64, ncclSum, sh.comm, sh.stream),
                   "ncclAllReduce");
    }
    rccl_check(ncclGroupEnd(), "ncclGroupEnd");
}

// Sharded DO-BFS over BOTH from one source (src_shard, src_local) or, with `roots` (one per local
// shard), from every component's minimum-rank vertex; returns levels run, *edges_out = entries of
// reached rows.  Depths go to Shard::bfs_depth (rows of the empty suffix stay -1 between calls:
// Shard::bfs_depth_tail_clean).
int dobfs_sharded(Graph& g, int64_t src_shard, int64_t src_local, int max_depth, double* edges_out, float* ms_out,
                  const CcRoots* roots = nullptr) {
    Ctx& ctx = *g.ctx;
    const size_t ns = g.shards.size();
    struct St {
        DevBuf<int32_t> queue[2];
        DevBuf<int64_t> qoff[2], send_off, woff, rseg, rlen;
        DevBuf<unsigned long long> ctr, gctr, hb, mk, sw, rm, fb;
        DevBuf<uint8_t> seen;
        DevBuf<SBfsState> st;
        int64_t hb_words = 0, sw_max = 0, rw_max = 0, live = 0, apply_x = 1;
        bool full_init = false;
    };
    std::vector<St> st(ns);
    int64_t tot[2] = {0, 0};  // entries of all shards, rows of all shards
    std::vector<unsigned long long*> ctrv, gctrv;
    std::vector<uint64_t*> swv, hbv, mkv, rmv;
    for (size_t i = 0; i < ns; ++i) {
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        const Halo& h = sh.halo_both;
        St& t = st[i];
        const std::vector<int64_t> woff = halo_word_offsets(h, g.P);
        t.hb_words = (h.C + 63) / 64;
        std::vector<int64_t> rseg((size_t)g.P, 0), rlen((size_t)g.P, 0);
        for (int q = 0; q < g.P; ++q) {
            rlen[(size_t)q] = q == sh.index ? 0 : h.recv_off[(size_t)q + 1] - h.recv_off[(size_t)q];
            rseg[(size_t)q] = (int64_t)h.seg_of(q, sh.index) << h.tbits;
            t.rw_max = std::max(t.rw_max, (rlen[(size_t)q] + 63) / 64);
            t.sw_max = std::max(t.sw_max, woff[(size_t)q + 1] - woff[(size_t)q]);
        }
        t.rseg.alloc(g.P);
        t.rlen.alloc(g.P);
        t.send_off.alloc(g.P + 1);
        t.woff.alloc(g.P + 1);
        copy_h2d(t.rseg.get(), rseg.data(), g.P * sizeof(int64_t), sh.stream);
        copy_h2d(t.rlen.get(), rlen.data(), g.P * sizeof(int64_t), sh.stream);
        copy_h2d(t.send_off.get(), h.send_off.data(), (g.P + 1) * sizeof(int64_t), sh.stream);
        copy_h2d(t.woff.get(), woff.data(), (g.P + 1) * sizeof(int64_t), sh.stream);
        const int64_t r1 = std::max<int64_t>(sh.rows, 1);
        for (int k = 0; k < 2; ++k) {
            t.queue[k].alloc(r1);
            t.qoff[k].alloc(r1);
        }
        t.hb.alloc(std::max<int64_t>(t.hb_words, 1));
        t.mk.alloc(std::max<int64_t>(t.hb_words, 1));
        // the stamp bytes stay with the shard, zero between traversals (each top-down level's mid kernel
        // clears what its push set), so the start clears them only after an allocation or a failed call
        if (sh.sbfs_stamp.size() != (size_t)std::max<int64_t>(t.hb_words * 64, 1)) {
            sh.sbfs_stamp.alloc(std::max<int64_t>(t.hb_words * 64, 1));
            sh.sbfs_dirty.alloc(std::max<int64_t>(t.hb_words / 8 + 1, 1));
            sh.sbfs_stamp_clean = false;
        }
        if (!sh.sbfs_stamp_clean) {
            JG_HIP(hipMemsetAsync(sh.sbfs_stamp.get(), 0, sh.sbfs_stamp.bytes(), sh.stream));
            JG_HIP(hipMemsetAsync(sh.sbfs_dirty.get(), 0, sh.sbfs_dirty.bytes(), sh.stream));
        }
        sh.sbfs_stamp_clean = false;  // until this traversal completes
        t.sw.alloc(std::max<int64_t>(woff[(size_t)g.P], 1));
        t.rm.alloc(std::max<int64_t>(woff[(size_t)g.P], 1));
        t.ctr.alloc(kSRing);
        t.gctr.alloc(kSRing);
        t.seen.alloc(r1);
        t.fb.alloc(3 * (size_t)((r1 + 63) / 64));
        sbfs_send_bitmaps(g, sh);
        t.st.alloc(kSRing);
        bfs_first_col(sh, sh.both);  // the bottom-up's first columns (before t0)
        // depths live in bfs_depth; the BOTH empty suffix is never reached, so it keeps -1 between calls
        if (sh.bfs_depth.size() != (size_t)r1) {
            sh.bfs_depth.alloc(r1);
            sh.bfs_depth_tail_clean = false;
        }
        t.live = sh.both.empty_from >= 0 ? std::min(sh.rows, sh.both.empty_from) : sh.rows;
        if (t.live < sh.rows && !sh.bfs_depth_tail_clean) {
            fill_i32_kernel<<<grid_for(sh.rows - t.live), kBlock, 0, sh.stream>>>(sh.bfs_depth.get() + t.live,
                                                                                  sh.rows - t.live, -1);
            JG_LAUNCH_CHECK();
        }
        t.full_init = !roots && sh.index == src_shard && src_local >= t.live;
        tot[0] += sh.both.nnz;
        tot[1] += sh.rows;
        ctrv.push_back(t.ctr.peer());  // (collected for the exchange / reduction / peers' kernels)
        gctrv.push_back(t.gctr.peer());
        swv.push_back(reinterpret_cast<uint64_t*>(t.sw.peer()));
        hbv.push_back(reinterpret_cast<uint64_t*>(t.hb.peer()));
        mkv.push_back(reinterpret_cast<uint64_t*>(t.mk.peer()));
        rmv.push_back(reinterpret_cast<uint64_t*>(t.rm.peer()));
    }
    allreduce_sum_i64(g, tot, 2);
    // shards on one device: the exchange's (owner, reader) runs for sbfs_copy_kernel
    Shard& sh0 = *g.shards[0];
    DevBuf<SBfsCopyRun> runs;
    int nruns = 0;
    int64_t run_max = 0;
    if (ctx.logical) {
        std::vector<SBfsCopyRun> rv;
        for (size_t oi = 0; oi < ns; ++oi) {
            const Halo& ho = g.shards[oi]->halo_both;
            const std::vector<int64_t> woff = halo_word_offsets(ho, g.P);
            for (size_t ri = 0; ri < ns; ++ri) {
                if (ri == oi) continue;
                const Shard& rs = *g.shards[ri];
                const Halo& hr = rs.halo_both;
                const int q = g.shards[oi]->index, r = rs.index;
                const int64_t n = (ho.send_off[(size_t)r + 1] - ho.send_off[(size_t)r] + 63) / 64;
                if (n == 0) continue;
                const int64_t seg = ((int64_t)hr.seg_of(q, r) << hr.tbits) >> 6;
                using U = unsigned long long;
                rv.push_back({reinterpret_cast<const U*>(swv[oi] + woff[(size_t)r]), reinterpret_cast<U*>(hbv[ri] + seg),
                              reinterpret_cast<const U*>(mkv[ri] + seg), reinterpret_cast<U*>(rmv[oi] + woff[(size_t)r]), n});
                run_max = std::max(run_max, n);
            }
        }
        nruns = (int)rv.size();
        DeviceGuard dg(sh0.device);
        runs.alloc(std::max<size_t>(rv.size(), 1));
        if (nruns) copy_h2d(runs.get(), rv.data(), rv.size() * sizeof(SBfsCopyRun), sh0.stream);
    }
    // the direction thresholds of dobfs_single: a single source switches to bottom-up at dobfs_alpha, the
    // multi-root start (CC) at bfs_alpha
    const double alpha = (double)(roots ? tune().bfs_alpha : tune().dobfs_alpha), beta = (double)tune().bfs_beta;
    auto level_args = [&](size_t i, int level) {
        Shard& sh = *g.shards[i];
        St& t = st[i];
        SBfsLevel a{};
        a.rp = sh.both.row_ptr.get();
        a.col = sh.both.col.get();
        a.first_col = sh.both.first_col.get();
        a.rows = sh.rows;
        a.bu_rows = t.live;
        a.dvec = sh.bfs_depth.get();
        a.seen = t.seen.get();
        a.fw = (std::max<int64_t>(sh.rows, 1) + 63) / 64;
        for (int k = 0; k < 3; ++k) a.fb[k] = t.fb.get() + k * a.fw;
        a.bq = sh.sbfs_bq.get();
        a.bpre = sh.sbfs_bpre.get();
        a.hb = t.hb.get();
        a.mk = t.mk.get();
        a.st8 = sh.sbfs_stamp.get();
        a.dirty = sh.sbfs_dirty.get();
        a.sw = t.sw.get();
        a.rm = t.rm.get();
        a.queue_in = t.queue[level & 1].get();
        a.qoff_in = t.qoff[level & 1].get();
        a.queue_out = t.queue[(level & 1) ^ 1].get();
        a.qoff_out = t.qoff[(level & 1) ^ 1].get();
        a.send_off = t.send_off.get();
        a.woff = t.woff.get();
        a.rseg = t.rseg.get();
        a.rlen = t.rlen.get();
        a.P = g.P;
        a.send_src = sh.halo_both.send_src.get();
        a.ctr = t.ctr.get();
        // the global counter: the sum of every shard's ring on one device, else this shard's reduced ring
        if (ctx.logical) {
            a.nsum = (int)ns;
            for (size_t k = 0; k < ns; ++k) a.gsum[k] = ctrv[k];
        } else {
            a.nsum = 1;
            a.gsum[0] = gctrv[i];
        }
        a.st = t.st.get();
        a.apply_x = t.apply_x;
        a.level = level;
        a.max_depth = max_depth;
        a.alpha = alpha;
        a.beta = beta;
        a.nrows = tot[1];
        return a;
    };
    // (blocks, P) grids.  The appending launches (top-down push, bottom-up probes, mark claims) keep to
    // about kSbfsAppendBlocks workgroups, grid-stride, sized from the shard alone (the frontier is on the
    // device); the per-peer word passes cover the longest run (at most 256 workgroups per peer).
    constexpr int64_t kSbfsAppendBlocks = 2048;
    std::vector<dim3> gpre(ns), gmid(ns), gpost(ns);
    for (size_t i = 0; i < ns; ++i) {
        St& t = st[i];
        const Shard& sh = *g.shards[i];
        const int64_t mid_trip = (kBlock / kWave) * 16;
        const int64_t fx = std::max<int64_t>(kSbfsAppendBlocks / g.P, 1);
        const int64_t pack_x = std::min<int64_t>((((sh.rows + 63) / 64) + kBlock - 1) / kBlock, 256);  // a row word per thread
        const int64_t mid_x = std::min<int64_t>((t.rw_max + mid_trip - 1) / mid_trip, 256);
        gpre[i] = dim3((unsigned)std::max<int64_t>({pack_x, fx, 1}), (unsigned)g.P);
        gmid[i] = dim3((unsigned)std::max<int64_t>(mid_x, 1), (unsigned)g.P);
        // the claims: kSbfsApplyChunk words per wave and trip, at most kSbfsApplyBlocks workgroups in all
        st[i].apply_x = std::max<int64_t>(std::min<int64_t>((t.sw_max + (kBlock / kWave) * kSbfsApplyChunk - 1) /
                                                                ((kBlock / kWave) * kSbfsApplyChunk),
                                                            std::max<int64_t>(kSbfsApplyBlocks / g.P, 1)),
                                          1);
        gpost[i] = dim3((unsigned)std::max(fx, st[i].apply_x), (unsigned)g.P);
    }
    hipEvent_t t0, t1;
    {
        DeviceGuard dg(sh0.device);
        JG_HIP(hipEventCreate(&t0));
        JG_HIP(hipEventCreate(&t1));
        for (auto& sp : g.shards) {
            DeviceGuard dgs(*sp);
            JG_HIP(hipStreamSynchronize(sp->stream));  // the plan copies above; t0 marks the traversal's start
        }
        region_mark(sh0.stream, true);
        JG_HIP(hipEventRecord(t0, sh0.stream));
    }
    for (size_t i = 0; i < ns; ++i) {
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        St& t = st[i];
        const SBfsLevel a = level_args(i, 0);
        if (roots) {
            JG_HIP(hipMemsetAsync(t.ctr.get(), 0, kSRing * sizeof(unsigned long long), sh.stream));
            sbfs_init_roots_kernel<<<grid_for(sh.rows), kBlock, 0, sh.stream>>>(a, roots[i], (long long)tot[0]);
        } else {
            const int64_t init_rows = t.full_init ? sh.rows : t.live;
            sbfs_init_kernel<<<grid_for(init_rows), kBlock, 0, sh.stream>>>(
                a, init_rows, sh.index == src_shard ? src_local : -1, (long long)tot[0]);
        }
        JG_LAUNCH_CHECK();
    }
    sbfs_reduce(g, ctrv, gctrv, kSRing - 1);
    // Levels in batches, the state read back once per batch: the first batch covers the deepest of the
    // last traversals plus the level that finds the frontier empty (a level enqueued past the end costs an
    // exchange and an all-reduce on N GPUs), then 4, 8, 16, ...
    int predicted = 0;
    for (int k = 0; k < std::min(sh0.bfs_hist_n, 4); ++k) predicted = std::max(predicted, sh0.bfs_hist[k]);
    int level = 0;
    SBfsState hs{};
    for (int batch = predicted > 0 ? predicted + 1 : std::max(1, tune().bfs_batch0), next_batch = 4;;
         batch = next_batch, next_batch = std::min(next_batch * 2, 64)) {
        if (max_depth >= 0) batch = std::min(batch, max_depth + 1 - level);
        if (batch <= 0) fail(JG_ERR_STATE, "sharded BFS level control did not terminate");  // level max_depth stops
        for (int k = 0; k < batch; ++k, ++level) {
            for (size_t i = 0; i < ns; ++i) {
                Shard& sh = *g.shards[i];
                DeviceGuard dg(sh);
                sbfs_pre_kernel<<<gpre[i], kBlock, 0, sh.stream>>>(level_args(i, level));
                JG_LAUNCH_CHECK();
            }
            for (size_t i = 0; i < ns; ++i) {
                Shard& sh = *g.shards[i];
                DeviceGuard dg(sh);
                sbfs_mid_kernel<<<gmid[i], kBlock, 0, sh.stream>>>(level_args(i, level));
                JG_LAUNCH_CHECK();
            }
            if (ctx.logical) {
                if (nruns) {
                    ExchTimer et(g);
                    DeviceGuard dg(sh0.device);
                    const dim3 grid((unsigned)std::min<int64_t>((run_max + kBlock - 1) / kBlock, 64), (unsigned)nruns);
                    sbfs_copy_kernel<<<grid, kBlock, 0, sh0.stream>>>(runs.get(), st[0].st.peer(), level % kSRing);
                    JG_LAUNCH_CHECK();
                }
            } else {
                exchange_halo_bits_both(g, JG_ADJ_BOTH, swv, hbv, mkv, rmv);
            }
            for (size_t i = 0; i < ns; ++i) {
                Shard& sh = *g.shards[i];
                DeviceGuard dg(sh);
                sbfs_post_kernel<kSbfsApplyWords><<<gpost[i], kBlock, 0, sh.stream>>>(level_args(i, level));
                JG_LAUNCH_CHECK();
            }
            sbfs_reduce(g, ctrv, gctrv, level % kSRing);
            if (debug_bfs()) {
                SBfsState ds{};
                unsigned long long dc = 0;
                DeviceGuard dg(sh0);
                copy_d2h(&ds, st[0].st.get() + level % kSRing, sizeof ds, sh0.stream);
                copy_d2h(&dc, st[0].ctr.get() + level % kSRing, sizeof dc, sh0.stream);
                std::fprintf(stderr, "[jg sbfs] level %d %s done %d shard-0 next frontier %llu vertices %llu entries\n",
                             level, ds.bottom_up ? "bottom-up" : "top-down", ds.done, dc >> kPackShift, dc & kEdgeMask);
            }
        }
        {
            DeviceGuard dg(sh0);
            JG_HIP(hipEventRecord(t1, sh0.stream));
            copy_d2h(&hs, st[0].st.get() + (level - 1) % kSRing, sizeof hs, sh0.stream);
        }
        if (hs.done) break;
    }
    {
        DeviceGuard dg(sh0.device);
        region_mark(sh0.stream, false);
        JG_HIP(hipEventSynchronize(t1));
        JG_HIP(hipEventElapsedTime(ms_out, t0, t1));
        JG_HIP(hipEventDestroy(t0));
        JG_HIP(hipEventDestroy(t1));
    }
    for (size_t i = 0; i < ns; ++i) {
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        JG_HIP(hipStreamSynchronize(sh.stream));
        // a source in the skipped suffix left its 0 there: the next call refills the suffix
        sh.bfs_depth_tail_clean = !st[i].full_init || st[i].live == sh.rows;
        sh.sbfs_stamp_clean = true;  // every top-down level cleared its stamps
    }
    if (!roots) {  // the level counts of the last traversals (the first batch's size)
        for (int k = 3; k > 0; --k) sh0.bfs_hist[k] = sh0.bfs_hist[k - 1];
        sh0.bfs_hist[0] = hs.levels;
        sh0.bfs_hist_n = std::min(sh0.bfs_hist_n + 1, 4);
    }
    *edges_out = (double)hs.edges;
    return hs.levels;  // levels run, as dobfs_single counts them
}

}  // namespace

int cc_root_eccentricity_sharded(Graph& g, const CcRoots* roots, double* edges_out) {
    float ms = 0;
    return dobfs_sharded(g, -1, -1, -1, edges_out, &ms, roots) - 1;
}

int cc_root_eccentricity(Ctx& ctx, Shard& sh, const CcRoots& r, int32_t* depth, double* edges_out,
                         const std::function<void()>* after_start, hipEvent_t end_ev) {
    *edges_out = 0;
    if (sh.rows == 0) return -1;
    const BfsCsrs c{&sh.both, &sh.both};
    // the traversal stops at the first level with an empty frontier, which it counts: the deepest
    // depth is the one before (no depth-max pass over the rows)
    return dobfs_single(ctx, sh, c, -1, -1, depth, edges_out, &r, end_ev, true, after_start) - 1;
}


// Clears the positions of a shard's gathered vector that hold values: its own rows and, on a segmented
// compact vector (halo plan), each peer's run at the start of its segment.  Nothing reads the rest of a
// segment (columns and exchanges address the runs only), which at RMAT-26, P = 8 is 83% of the vector's
// 134 M positions; a dense (allgather) vector is cleared whole.
namespace {
// The runs of a compact vector a shard gathers into (own rows + one segment per peer), zeroed by one
// launch: a memset per run was P + 1 fill dispatches of ~5 us each per vector (three vectors per
// 64-source traversal).  Run starts are 16-byte aligned (rows at 0, segments 2^tbits elements apart).
constexpr int kZeroRuns = 32;
struct ZeroRuns {
    char* p[kZeroRuns];
    int64_t n[kZeroRuns];  // bytes
};
__global__ __launch_bounds__(kBlock) void zero_runs_kernel(ZeroRuns z) {
    char* p = z.p[blockIdx.y];
    const int64_t n = z.n[blockIdx.y], n16 = n >> 4;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x, tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t i = tid; i < n16; i += stride) reinterpret_cast<uint4*>(p)[i] = make_uint4(0u, 0u, 0u, 0u);
    for (int64_t i = (n16 << 4) + tid; i < n; i += stride) p[i] = 0;
}
}  // namespace

void zero_gathered(const Graph& g, const Shard& sh, uint32_t adj, void* v, size_t eb) {
    const Halo& h = g.halo(sh, adj);
    char* p = static_cast<char*>(v);
    if (!h.on) {
        JG_HIP(hipMemsetAsync(p, 0, (size_t)g.vec_len(sh, adj) * eb, sh.stream));
        return;
    }
    std::vector<std::pair<char*, int64_t>> runs;
    if (sh.rows) runs.emplace_back(p, sh.rows * (int64_t)eb);
    for (int q = 0; q < g.P; ++q) {
        if (q == sh.index) continue;
        const int64_t nr = h.recv_off[(size_t)q + 1] - h.recv_off[(size_t)q];
        if (nr > 0) runs.emplace_back(p + ((size_t)h.seg_of(q, sh.index) << h.tbits) * eb, nr * (int64_t)eb);
    }
    for (size_t r0 = 0; r0 < runs.size(); r0 += kZeroRuns) {
        ZeroRuns z{};
        const size_t k = std::min<size_t>(kZeroRuns, runs.size() - r0);
        int64_t longest = 0;
        for (size_t j = 0; j < k; ++j) {
            z.p[j] = runs[r0 + j].first;
            z.n[j] = runs[r0 + j].second;
            longest = std::max(longest, z.n[j]);
        }
        const dim3 grid(grid_for((longest + 15) / 16, kBlock, 2048), (unsigned)k);
        zero_runs_kernel<<<grid, kBlock, 0, sh.stream>>>(z);
        JG_LAUNCH_CHECK();
    }
}

void bfs_kept_release(Graph& g) {
    for (auto& sp : g.shards) {
        DeviceGuard dg(*sp);
        sp->kept_depth.reset();
    }
    g.kept_nsrc = 0;
}

namespace {
// one source's depths (a single-source traversal's bfs_depth) kept as plane 0 of every shard: the buffers
// swap (no copy); the next traversal finds bfs_depth of another size or with a stale suffix and refills
// it before its timed region
void keep_depth_rows(Graph& g) {
    for (auto& sp : g.shards) {
        Shard& sh = *sp;
        DeviceGuard dg(sh);
        JG_HIP(hipStreamSynchronize(sh.stream));
        sh.kept_depth.swap(sh.bfs_depth);
        sh.bfs_depth_tail_clean = false;
    }
    g.kept_nsrc = 1;
}
}  // namespace

void bfs_kept_row(Graph& g, int s, int32_t* depth_out) {
    if (s < 0 || s >= g.kept_nsrc) fail(JG_ERR_ARG, "no kept depth row with that index (jg_bfs_keep)");
    for (auto& sp : g.shards) rows_to_dense(g, *sp, sp->kept_depth.peer() + (int64_t)s * sp->rows, depth_out);
}

void bfs_run(Graph& g, const int64_t* source_vids, int nsrc, int direction, int max_depth, int32_t* const* depth_rows,
             bool keep) {
    if (nsrc <= 0) fail(JG_ERR_ARG, "nsrc must be positive");
    if (keep && nsrc > 64) fail(JG_ERR_ARG, "jg_bfs_keep takes at most 64 sources (one bit-parallel batch)");
    if (keep) bfs_kept_release(g);
    if (direction < JG_DIR_OUT || direction > JG_DIR_BOTH) fail(JG_ERR_ARG, "bad direction");
    Ctx& ctx = *g.ctx;
    ctx.last = jg_stats{};
    prof_discard_exchanges(g);  // exchange pairs of this call only
    const bool single = nsrc == 1 && g.P == 1;
    const bool sharded_do = nsrc == 1 && g.P > 1 && g.P <= kMaxShardsBfs && direction == JG_DIR_BOTH &&
                            g.shards[0]->halo_both.on && tune().sharded_bfs;
    hipEvent_t t0, t1;
    Shard& sh0 = *g.shards[0];
    DeviceGuard dg0(sh0.device);
    JG_HIP(hipEventCreate(&t0));
    JG_HIP(hipEventCreate(&t1));
    if (sharded_do) {
        int shard = -1;
        const int64_t l = local_of_vid(g, source_vids[0], &shard);
        double edges = 0;
        float ms = 0;
        const int levels = dobfs_sharded(g, l >= 0 ? shard : -1, l, max_depth, &edges, &ms);
        ctx.last.compute_ms = ms;
        ctx.last.levels = levels;
        ctx.last.supersteps = levels;
        ctx.last.edges_traversed = l >= 0 ? edges / 2 : 0;
        if (depth_rows && depth_rows[0])
            for (auto& sp : g.shards) rows_to_dense(g, *sp, sp->bfs_depth.peer(), depth_rows[0]);
        if (keep) keep_depth_rows(g);
        prof_collect(ctx, g);
    } else if (single) {
        Shard& sh = sh0;
        const BfsCsrs c = pick_csrs(sh, direction);
        int shard = 0;
        const int64_t l = local_of_vid(g, source_vids[0], &shard);
        if (sh.bfs_depth.size() != (size_t)std::max<int64_t>(sh.rows, 1)) {
            sh.bfs_depth.alloc(std::max<int64_t>(sh.rows, 1));
            sh.bfs_depth_tail_clean = false;
        }
        DevBuf<int32_t>& depth = sh.bfs_depth;
        int levels = 0;
        double edges = 0;
        if (l < 0) {
            fill_i32_kernel<<<grid_for(sh.rows), kBlock, 0, sh.stream>>>(depth.get(), sh.rows, -1);
            JG_LAUNCH_CHECK();
            sh.bfs_depth_tail_clean = true;
            JG_HIP(hipEventRecord(t0, sh.stream));
            JG_HIP(hipEventRecord(t1, sh.stream));
        } else {
            bfs_buffers(sh);
            if (c.pull) bfs_first_col(sh, *c.pull);
            // BOTH: rows of the empty suffix (no entry) are never reached, so their depths stay -1 from one
            // traversal to the next and the init skips them, whatever the caller wants back (the
            // depth output and kept rows no longer pay a longer init than want=False).  The suffix is filled
            // once, before t0; a source inside it (an isolated vertex) takes the full init and leaves its 0
            // behind, so the next traversal refills.
            const int64_t live = c.push == c.pull && c.pull->empty_from >= 0 ? std::min(sh.rows, c.pull->empty_from)
                                                                              : sh.rows;
            if (live < sh.rows && !sh.bfs_depth_tail_clean) {
                fill_i32_kernel<<<grid_for(sh.rows - live), kBlock, 0, sh.stream>>>(depth.get() + live, sh.rows - live, -1);
                JG_LAUNCH_CHECK();
            }
            const bool full_init = l >= live;
            region_mark(sh.stream, true);
            JG_HIP(hipEventRecord(t0, sh.stream));
            levels = dobfs_single(ctx, sh, c, l, max_depth, depth.get(), &edges, nullptr, t1, full_init);
            sh.bfs_depth_tail_clean = !full_init || live == sh.rows;
        }
        JG_HIP(hipEventSynchronize(t1));
        float ms = 0;
        JG_HIP(hipEventElapsedTime(&ms, t0, t1));
        ctx.last.compute_ms = ms;
        ctx.last.levels = levels;
        ctx.last.supersteps = levels;
        ctx.last.edges_traversed = direction == JG_DIR_BOTH ? edges / 2 : edges;
        const Csr* degcsr = c.push ? c.push : c.pull;
        ctx.last.algorithmic_bytes = 4.0 * (double)degcsr->nnz + 12.0 * (double)sh.rows;
        if (depth_rows && depth_rows[0]) rows_to_dense(g, sh, depth.get(), depth_rows[0]);
        if (keep) keep_depth_rows(g);
        prof_collect(ctx, g);
    } else if (nsrc <= kNarrowMax && g.P == 1 && g.shards.size() == 1 && tune().bfs_narrow &&
               pick_csrs(sh0, direction).push && pick_csrs(sh0, direction).pull) {
        // 2..8 sources on one shard: the narrow engine (jg_narrow.hip), one frontier byte per row
        Shard& sh = sh0;
        const BfsCsrs c = pick_csrs(sh, direction);
        std::vector<int64_t> loc((size_t)nsrc);
        std::vector<int> shard((size_t)nsrc);
        locals_of_vids(g, source_vids, nsrc, loc.data(), shard.data());
        DevBuf<int32_t> planes;
        if (depth_rows || keep) planes.alloc(std::max<int64_t>((int64_t)nsrc * sh.rows, 1));
        const NarrowRun r = narrow_bfs(ctx, sh, *c.push, *c.pull, loc.data(), nsrc, max_depth,
                                       planes.size() ? planes.get() : nullptr);
        ctx.last.compute_ms = r.ms;
        ctx.last.levels = r.levels;
        ctx.last.supersteps = r.levels;
        ctx.last.edges_traversed = r.entries;
        ctx.last.algorithmic_bytes = r.bytes;
        if (depth_rows)
            for (int s = 0; s < nsrc; ++s)
                if (depth_rows[s]) rows_to_dense(g, sh, planes.get() + (size_t)s * sh.rows, depth_rows[s]);
        if (keep) {
            sh.kept_depth.swap(planes);
            g.kept_nsrc = nsrc;
        }
        prof_collect(ctx, g);
    } else {
        // bit-parallel BFS in batches of 64 sources; works sharded (frontier words allgathered)
        float total_ms = 0;
        int max_levels = 0;
        double work_bytes = 0, work_entries = 0;
        for (int b0 = 0; b0 < nsrc; b0 += 64) {
            const int ns = std::min(64, nsrc - b0);
            const unsigned long long full = ns == 64 ? ~0ull : ((1ull << ns) - 1ull);
            struct St {
                DevBuf<unsigned long long> F[2], vis;
                DevBuf<int32_t> depth, changed;  // depth: int32 planes once widened
                DevBuf<uint8_t> depth8;           // byte planes of levels kMsLevelWords .. 254 (allocated on reaching them)
                DevBuf<unsigned long long> nwl;   // [kMsLevelWords][rows] new-bit words of levels 0 .. kMsLevelWords-1
                DevBuf<unsigned long long> hub, split;
                DevBuf<unsigned long long> live;  // [0] the pull level's live bits, [1] all sources (top-down)
                DevBuf<unsigned long long> xrest;  // msbfs_exit: the rows pass B scans (a bit per row)
                MsBu bx{};                         // msbfs_exit: every row with entries (bx.rows 0: off on this shard)
                int64_t exit_tasks = 0;            // band 0's merge tasks (its live count decides an exit level)
                int64_t all_rows = 0;   // the rows a pull level finalises (those with entries)
                int exit_all_levels = 0;
                // merge tasks of the bands the exit kernels took instead (on levels that count every task, and on all)
                double exit_unskipped_tasks = 0, exit_level_tasks = 0;
                unsigned long long b0_live_merged = 0;     // msbfs_exit 1: band 0's live tasks of levels that merged it
                double xlive_permille = 1000.0;            // the last probe's live share of band 0's tasks
                std::vector<DevBuf<unsigned long long>> todo, tlive;  // per band: row and task bitmaps
                DevBuf<int64_t> dloc;             // [64] each source's own row (-1: another shard's)
                // levels recorded as (row, new word) records instead of nwl words (level 0 from the sources and
                // every top-down level below kMsLevelWords): {level, count, rows, words}
                struct Rec {
                    int level = 0;
                    int64_t n = 0;
                    DevBuf<int32_t> rows;
                    DevBuf<unsigned long long> words;
                };
                std::vector<Rec> recs;
                DevBuf<unsigned long long> work;  // [0] live merge tasks over all pull levels, [1] reached pairs,
                                                  // [2] entries the early-exit bottom-up levels scanned,
                                                  // [3] band 0's live tasks of this level (msbfs_exit 1)
                int64_t light_nnz = 0, all_tasks = 0;  // entries outside the split, merge tasks of all bands
            };
            std::vector<St> st(g.shards.size());
            const BfsCsrs c0 = pick_csrs(sh0, direction);
            const uint32_t adj0 = adj_of(sh0, c0);
            // Levels whose frontier has few edges run top-down: on one shard with a push adjacency, and
            // on a sharded BOTH traversal over the halo plan (msbfs_td 1; 2 = one shard only).  Sharded,
            // a shard pushes its own frontier rows; bits for a peer's vertex collect in its halo slot and
            // go to the owner by the reverse halo exchange (msbfs_td_recv_kernel).
            const bool td_one = g.shards.size() == 1 && g.P == 1 && c0.push != nullptr && tune().msbfs_td != 0;
            const bool td_shard = g.P > 1 && g.P <= kMaxPeersMs && direction == JG_DIR_BOTH && sh0.halo_both.on &&
                                  tune().msbfs_td == 1;
            const bool td_ok = td_one || td_shard;
            struct Td {
                DevBuf<int32_t> queue[2], touched;
                DevBuf<int64_t> qoff[2], touched_off;
                DevBuf<unsigned long long> ctr;   // [0] frontier, [1] touched, [2] halo slots set
                DevBuf<int64_t> srcs;             // the shard's distinct source rows
                DevBuf<unsigned long long> rbuf;  // sharded: the peers' halo slots for own rows (send-list order)
                DevBuf<unsigned long long> hs;    // sharded: halo staging (compact positions), zero between levels
                DevBuf<int32_t> hlist;            // sharded: the staging slots a level set
                DevBuf<int64_t> hlist_off;        // appender scratch
                DevBuf<unsigned int> bcount;      // [kRedBlocks][P] set staging slots per histogram block and peer
                DevBuf<unsigned long long> pairs, rpairs, pcnt;  // sparse reverse exchange: sent / received
                                                                 // (offset, word) pairs, per-peer counts + cursors
                std::vector<int64_t> src_rows;
                int64_t nq = 0, mf = 0;
                int64_t nrp = 0;                  // pairs received by the last sparse exchange
                PairRuns pv{};                    // their per-peer runs and this shard's send-list offsets
                int64_t nq_in = 0;                // the last top-down level's input frontier (its queue)
                bool rowapply = false;            // this level's apply passes over every row (no touched list)
            };
            std::vector<Td> tds(g.shards.size());
            std::vector<int64_t> src_local((size_t)ns);
            std::vector<int> src_shard((size_t)ns);
            locals_of_vids(g, source_vids + b0, ns, src_local.data(), src_shard.data());
            int64_t push_nnz = 0;  // entries of the push adjacency, all shards and ranks (the direction rule)
            for (size_t i = 0; i < g.shards.size(); ++i) {
                Shard& sh = *g.shards[i];
                DeviceGuard dg(sh);
                const BfsCsrs c = pick_csrs(sh, direction);
                if (!c.pull) fail(JG_ERR_UNSUPPORTED, "multi-source BFS needs the pull adjacency");
                const PullPlan& plan = (c.pull == &sh.both) ? sh.plan_both : sh.plan_in;
                if (c.pull == &sh.out) fail(JG_ERR_UNSUPPORTED, "multi-source IN traversal is not supported");
                if (c.push) push_nnz += c.push->nnz;
                St& t = st[i];
                const int64_t len = g.vec_len(sh, adj_of(sh, c));
                t.F[0].alloc(len);
                t.F[1].alloc(len);
                t.vis.alloc(std::max<int64_t>(sh.rows, 1));
                t.nwl.alloc(std::max<int64_t>(sh.rows * kMsLevelWords, 1));
                t.changed.alloc(1);
                t.hub.alloc(std::max<int64_t>(plan.num_chunks, 1));
                if (tune().msbfs_split && plan.split_rows > 0) t.split.alloc(plan.split_partial_len());
                t.live.alloc(3);  // [2]: a split level's pull live bits
                t.work.alloc(4);
                JG_HIP(hipMemsetAsync(t.work.get(), 0, 4 * sizeof(unsigned long long), sh.stream));
                if (tune().msbfs_exit > 0 && t.split.size() && !plan.bands.empty())
                    t.xrest.alloc(std::max<int64_t>((sh.rows + 63) / 64, 1));
                t.light_nnz = c.pull->nnz;
                if (t.split.size() && plan.split_rows > 0) {
                    int64_t split_nnz = 0;
                    copy_d2h(&split_nnz, c.pull->row_ptr.get() + plan.split_rows, sizeof split_nnz, sh.stream);
                    t.light_nnz -= split_nnz;
                    for (const auto& bd : plan.bands) t.all_tasks += bd->tasks;
                }
                const unsigned long long lw[2] = {full, full};
                copy_h2d(t.live.get(), lw, sizeof lw, sh.stream);
                if (t.split.size() && tune().msbfs_skip) {
                    t.todo.resize(plan.bands.size());
                    t.tlive.resize(plan.bands.size());
                    for (size_t b = 0; b < plan.bands.size(); ++b) {
                        t.todo[b].alloc(std::max<int64_t>((plan.bands[b]->rows() + 63) / 64, 1));
                        t.tlive[b].alloc(std::max<int64_t>((plan.bands[b]->tasks + 63) / 64, 1));
                    }
                }
                std::vector<int64_t> loc(ns, -1);
                for (int s = 0; s < ns; ++s)
                    if (src_local[(size_t)s] >= 0 && src_shard[(size_t)s] == sh.index) loc[s] = src_local[(size_t)s];
                // the shard's distinct source rows: its first top-down queue (msbfs_source_queue_kernel)
                for (int64_t l : loc)
                    if (l >= 0 && std::find(tds[i].src_rows.begin(), tds[i].src_rows.end(), l) == tds[i].src_rows.end())
                        tds[i].src_rows.push_back(l);
                t.dloc.alloc(ns);
                copy_h2d(t.dloc.get(), loc.data(), ns * sizeof(int64_t), sh.stream);
                JG_HIP(hipStreamSynchronize(sh.stream));
            }
            allreduce_sum_i64(g, &push_nnz, 1);
            // need_fwd: the current F's halo segments are stale.  The forward exchange runs lazily, before a
            // pull level: a top-down level reads own frontier words only (and writes own rows only)
            bool need_fwd = g.P > 1;
            int cur = 0, level = 0, qc = 0;
            int64_t g_nq = 0, g_mf = 0;  // the current frontier's vertices and push entries, all shards and ranks
            // touched (nullable): += the rows the top-down level just applied (its touched counter)
            auto read_frontier = [&](double* touched = nullptr) {
                int64_t v[2] = {0, 0};
                for (size_t i = 0; i < g.shards.size(); ++i) {
                    Shard& sh = *g.shards[i];
                    DeviceGuard dg(sh);
                    unsigned long long hh[2] = {0, 0};
                    copy_d2h(hh, tds[i].ctr.get(), (touched ? 2 : 1) * sizeof(unsigned long long), sh.stream);
                    const unsigned long long h = hh[0];
                    if (touched) *touched += (double)(hh[1] >> kPackShift);
                    tds[i].nq = (int64_t)(h >> kPackShift);
                    tds[i].mf = (int64_t)(h & kEdgeMask);
                    v[0] += tds[i].nq;
                    v[1] += tds[i].mf;
                }
                allreduce_sum_i64(g, v, 2);
                g_nq = v[0];
                g_mf = v[1];
            };
            // live bits of the next pull level from every shard's own rows (the top-down apply or the scan
            // after a pull level ORed them into live[0]): OR over the local shards and the ranks, a superset
            // of what the shard's gathered vector holds, which is all the task skip needs
            auto combine_live = [&]() {
                if (g.shards.size() == 1 && ctx.nranks == 1) return;
                uint64_t v = 0;
                for (size_t i = 0; i < g.shards.size(); ++i) {
                    Shard& sh = *g.shards[i];
                    DeviceGuard dg(sh);
                    uint64_t w = 0;
                    copy_d2h(&w, st[i].live.get(), sizeof w, sh.stream);
                    v |= w;
                }
                v = allreduce_or_u64(g, v);
                for (size_t i = 0; i < g.shards.size(); ++i) {
                    Shard& sh = *g.shards[i];
                    DeviceGuard dg(sh);
                    copy_h2d(st[i].live.get(), &v, sizeof v, sh.stream);
                }
            };
            auto build_frontier = [&](int qslot) {
                for (size_t i = 0; i < g.shards.size(); ++i) {
                    Shard& sh = *g.shards[i];
                    DeviceGuard dg(sh);
                    const BfsCsrs c = pick_csrs(sh, direction);
                    const int64_t ne = pull_live_rows(sh, c);
                    JG_HIP(hipMemsetAsync(tds[i].ctr.get(), 0, sizeof(unsigned long long), sh.stream));
                    msbfs_frontier_kernel<<<grid_for(ne), kBlock, 0, sh.stream>>>(
                        st[i].F[cur].get(), ne, c.push->row_ptr.get(), tds[i].queue[qslot].get(),
                        tds[i].qoff[qslot].get(), tds[i].ctr.get());
                    JG_LAUNCH_CHECK();
                }
                read_frontier();
            };
            if (td_ok) {  // allocated before the timed region (~2.3 GB at RMAT-26 on one shard)
                for (size_t i = 0; i < g.shards.size(); ++i) {
                    Shard& sh = *g.shards[i];
                    DeviceGuard dg(sh);
                    Td& td = tds[i];
                    const size_t r1 = (size_t)std::max<int64_t>(sh.rows, 1);
                    for (int k = 0; k < 2; ++k) {
                        td.queue[k].alloc(r1);
                        td.qoff[k].alloc(r1);
                    }
                    td.touched.alloc(r1);
                    td.touched_off.alloc(r1);
                    td.ctr.alloc(3);
                    td.srcs.alloc(std::max<size_t>(td.src_rows.size(), 1));
                    if (!td.src_rows.empty())
                        copy_h2d(td.srcs.get(), td.src_rows.data(), td.src_rows.size() * sizeof(int64_t), sh.stream);
                    if (td_shard) {
                        const Halo& h = sh.halo_both;
                        td.rbuf.alloc(std::max<int64_t>(h.send_off[g.P], 1));
                        td.hs.alloc(g.vec_len(sh, JG_ADJ_BOTH));
                        td.hlist.alloc(std::max<int64_t>(h.recv_off[g.P], 1));
                        td.hlist_off.alloc(std::max<int64_t>(h.recv_off[g.P], 1));
                        if (tune().msbfs_sparse) {
                            td.pairs.alloc(2 * std::max<int64_t>(h.recv_off[g.P], 1));
                            td.rpairs.alloc(2 * std::max<int64_t>(h.send_off[g.P], 1));
                            td.pcnt.alloc(2 * (size_t)g.P);
                            td.bcount.alloc((size_t)kRedBlocks * g.P);
                        }
                    }
                }
            }
            for (size_t i = 0; i < g.shards.size(); ++i) {  // the early exit's first columns (before t0)
                Shard& sh = *g.shards[i];
                const BfsCsrs c = pick_csrs(sh, direction);
                if (c.pull) bfs_first_col(sh, *c.pull);
            }
            prof_discard_exchanges(g);  // exchange pairs never straddle t0
            region_mark(sh0.stream, true);
            JG_HIP(hipEventRecord(t0, sh0.stream));
            // the call's state, inside the timed region: frontiers, visited bits, the halo staging, the
            // sources (and level 0's depth record)
            for (size_t i = 0; i < g.shards.size(); ++i) {
                Shard& sh = *g.shards[i];
                DeviceGuard dg(sh);
                St& t = st[i];
                const BfsCsrs c = pick_csrs(sh, direction);
                if (td_one && c.pull == c.push) {
                    // one shard, BOTH: only rows before the empty suffix are read after level 0 (no gather,
                    // push target, scan, apply or finalise reaches the rows past it, §5; a directed traversal
                    // gathers columns without pull entries of their own, so it clears everything); the source
                    // rows among them get their words stored by the init below.  RMAT-26 BOTH: 34 of 67 M rows,
                    // three 537 MB clears halved
                    const int64_t ne = pull_live_rows(sh, c), base = g.vec_pos(sh, adj_of(sh, c)).base;
                    if (std::getenv("JG_MSBFS_POISON") && ne < sh.rows) {  // (test switch: garbage past the suffix)
                        const size_t tail = (size_t)(sh.rows - ne) * sizeof(unsigned long long);
                        JG_HIP(hipMemsetAsync(t.F[0].get() + base + ne, 0xA5, tail, sh.stream));
                        JG_HIP(hipMemsetAsync(t.F[1].get() + base + ne, 0x5A, tail, sh.stream));
                        JG_HIP(hipMemsetAsync(t.vis.get() + ne, 0xC3, tail, sh.stream));
                    }
                    JG_HIP(hipMemsetAsync(t.F[0].get() + base, 0, (size_t)ne * sizeof(unsigned long long), sh.stream));
                    JG_HIP(hipMemsetAsync(t.F[1].get() + base, 0, (size_t)ne * sizeof(unsigned long long), sh.stream));
                    JG_HIP(hipMemsetAsync(t.vis.get(), 0, (size_t)ne * sizeof(unsigned long long), sh.stream));
                } else {
                    zero_gathered(g, sh, adj_of(sh, c), t.F[0].get(), sizeof(unsigned long long));
                    zero_gathered(g, sh, adj_of(sh, c), t.F[1].get(), sizeof(unsigned long long));
                    JG_HIP(hipMemsetAsync(t.vis.get(), 0, t.vis.bytes(), sh.stream));
                }
                if (tds[i].hs.size()) zero_gathered(g, sh, JG_ADJ_BOTH, tds[i].hs.get(), sizeof(unsigned long long));
                St::Rec* r0 = nullptr;
                if (td_ok) {  // level 0 as records of the source rows
                    t.recs.emplace_back();
                    r0 = &t.recs.back();
                    r0->level = 0;
                    r0->n = ns;
                    r0->rows.alloc(ns);
                    r0->words.alloc(ns);
                } else {  // level 0's words
                    JG_HIP(hipMemsetAsync(t.nwl.get(), 0, (size_t)sh.rows * sizeof(unsigned long long), sh.stream));
                }
                msbfs_init_kernel<<<1, kWave, 0, sh.stream>>>(t.dloc.get(), ns, t.F[0].get(), t.vis.get(),
                                                          r0 ? nullptr : t.nwl.get(), sh.rows, g.vec_pos(sh, adj_of(sh, c)),
                                                          r0 ? r0->rows.get() : nullptr, r0 ? r0->words.get() : nullptr);
                JG_LAUNCH_CHECK();
            }
            if (!td_ok) {
                std::vector<void*> bufs;
                for (auto& t : st) bufs.push_back(t.F[0].peer());
                exchange_vec(g, adj0, bufs, sizeof(unsigned long long), ncclUint64);
                need_fwd = false;
            }
            if (td_ok) {  // the level-0 frontier is the source rows: queued directly, no scan of F
                for (size_t i = 0; i < g.shards.size(); ++i) {
                    Shard& sh = *g.shards[i];
                    DeviceGuard dg(sh);
                    const BfsCsrs c = pick_csrs(sh, direction);
                    msbfs_source_queue_kernel<<<1, kWave, 0, sh.stream>>>(tds[i].srcs.get(), (int)tds[i].src_rows.size(),
                                                                       c.push->row_ptr.get(), tds[i].queue[0].get(),
                                                                       tds[i].qoff[0].get(), tds[i].ctr.get());
                    JG_LAUNCH_CHECK();
                }
                read_frontier();
            }
            // queued: tds[i].queue[qc] holds the current frontier; live_ready: live[0] holds its live bits
            // (both from the previous level's end)
            // Depths: levels 0 .. kMsLevelWords-1 as new-bit words (nwl), levels up to 254 as byte planes
            // (allocated, all 255 = unreached, when the traversal reaches them), beyond as int32 planes (a
            // traversal about to write level 255 widens the byte planes first)
            auto ensure_depth8 = [&]() {
                for (size_t i = 0; i < g.shards.size(); ++i) {
                    Shard& sh = *g.shards[i];
                    St& t = st[i];
                    if (t.depth8.size() || t.depth.size()) continue;
                    DeviceGuard dg(sh);
                    t.depth8.alloc(std::max<int64_t>(sh.rows * ns, 1));
                    JG_HIP(hipMemsetAsync(t.depth8.get(), 0xFF, t.depth8.bytes(), sh.stream));
                }
            };
            auto widen = [&]() {
                for (size_t i = 0; i < g.shards.size(); ++i) {
                    Shard& sh = *g.shards[i];
                    St& t = st[i];
                    if (t.depth.size()) continue;
                    DeviceGuard dg(sh);
                    const int64_t total = std::max<int64_t>(sh.rows * ns, 1);
                    t.depth.alloc(total);
                    if (t.depth8.size()) {
                        msbfs_widen_kernel<<<grid_for(total), kBlock, 0, sh.stream>>>(t.depth8.get(), total, t.depth.get());
                        JG_LAUNCH_CHECK();
                    } else {
                        fill_i32_kernel<<<grid_for(total), kBlock, 0, sh.stream>>>(t.depth.get(), total, -1);
                        JG_LAUNCH_CHECK();
                    }
                    JG_HIP(hipStreamSynchronize(sh.stream));
                    t.depth8.reset();
                }
            };
            // levels whose depths are nwl words (bit L): a pull level finalises every own row (its word is
            // written, zero or not); a top-down level records (row, word) pairs of the rows it reached
            unsigned word_levels = td_ok ? 0u : 1u;
            // the caller's int32 planes: the widened byte / int32 planes, then the word-recorded levels
            auto materialize = [&](int levels_run) {
                widen();
                for (size_t i = 0; i < g.shards.size(); ++i) {
                    Shard& sh = *g.shards[i];
                    St& t = st[i];
                    DeviceGuard dg(sh);
                    const int lw = std::min(levels_run + 1, kMsLevelWords);
                    if (sh.rows > 0) {
                        const Csr* pc = pick_csrs(sh, direction).pull;
                        const int64_t ne = pc->empty_from >= 0 ? std::min(pc->empty_from, sh.rows) : sh.rows;
                        msbfs_levels_to_planes_kernel<<<grid_for(sh.rows), kBlock, 0, sh.stream>>>(
                            t.nwl.get(), lw, word_levels, sh.rows, ne, ns, t.depth.get());
                        JG_LAUNCH_CHECK();
                    }
                    for (const auto& r : t.recs)
                        if (r.n > 0 && r.level < lw) {
                            msbfs_records_to_planes_kernel<<<grid_for(r.n), kBlock, 0, sh.stream>>>(
                                r.rows.get(), r.words.get(), r.n, r.level, sh.rows, ns, t.depth.get());
                            JG_LAUNCH_CHECK();
                        }
                    JG_HIP(hipStreamSynchronize(sh.stream));
                }
            };
            // msbfs_exit: every row with entries scans its row with early exit (msbfs_exit_first_kernel /
            // msbfs_exit_rest_kernel) on pull levels where few of band 0's merge tasks are live, and such a
            // level runs no merge launch at all.  On the level after the frontier's peak a hub row finds all
            // its unvisited live bits within its first entries: RMAT-22, band 0 examines 0.1% instead of
            // 27.3% of the entries (tools/msbfs_exit_sim.py).  Band 0's live tasks alone decide
            // (every exit band's bitmaps took the same decisions, round 4); each shard decides for its own
            // rows.  (Only the exit bands through the exit, the light rows merged: RMAT-26 11.42 vs 11.20 ms.)
            for (size_t i = 0; i < g.shards.size(); ++i) {
                Shard& sh = *g.shards[i];
                DeviceGuard dg(sh);
                const BfsCsrs c = pick_csrs(sh, direction);
                const PullPlan& plan = (c.pull == &sh.both) ? sh.plan_both : sh.plan_in;
                St& t = st[i];
                if (tune().msbfs_exit > 0 && tune().pull_split && plan.split_rows > 0 && !plan.bands.empty() &&
                    t.xrest.size() > 0 && plan.bands[0]->row_begin == 0 && plan.bands[0]->row_end > 0) {
                    t.bx.rp = c.pull->row_ptr.get();
                    t.bx.col = c.pull->col.get();
                    t.bx.first_col = bfs_first_col(sh, *c.pull);
                    t.all_rows = c.pull->empty_from >= 0 ? std::min(c.pull->empty_from, sh.rows) : sh.rows;
                    t.bx.rows = t.all_rows;
                    t.bx.examined = t.work.get() + 2;
                    t.bx.first = tune().msbfs_exit_first;
                    t.exit_tasks = plan.bands[0]->tasks;
                }
            }
            bool queued = td_ok, live_ready = false;
            bool prev_td = false;  // the previous level ran top-down: F[cur ^ 1]'s nonzero own words are
                                   // exactly its input queue (tds[i].queue[qc ^ 1][0, nq_in))
            // work of the levels (jg_stats.algorithmic_bytes): pull levels (per shard: the live merge tasks
            // counted on the device, or every task when the skip is off) and top-down frontier entries
            int pull_levels = 0;
            int unskipped_levels = 0;  // pull levels that ran every merge task (msbfs_skip_first)
            double td_entries = 0, td_touched = 0, td_queued = 0;
            double td_row_passes = 0;  // rows the row-order applies read (8 B each)
            while (max_depth < 0 || level < max_depth) {
                if (level + 1 >= kMsLevelWords) ensure_depth8();
                if (level + 1 >= 255) widen();
                const bool td_level = td_ok && (double)g_mf < (double)push_nnz / (double)tune().bfs_alpha;
                // a pull level (merge engine or the exit kernels) finalises every own row: its words need no clearing
                if (!td_level && level + 1 < kMsLevelWords) word_levels |= 1u << (level + 1);
                if (td_level && !queued) {
                    build_frontier(qc ^ 1);
                    qc ^= 1;
                }
                const bool have_live = live_ready;
                queued = live_ready = false;
                bool queued_next = false;  // this pull level built the next level's top-down queue
                if (td_level) {
                    std::vector<void*> fv, rv;
                    for (size_t i = 0; i < g.shards.size(); ++i) {
                        Shard& sh = *g.shards[i];
                        DeviceGuard dg(sh);
                        const BfsCsrs c = pick_csrs(sh, direction);
                        St& t = st[i];
                        Td& td = tds[i];
                        // changed, the frontier / touched / staging counters, the live bits the apply ORs and the
                        // sparse exchange's per-peer counts and cursors
                        zero_words({{t.changed.get(), sizeof(int32_t)},
                                    {td.ctr.get(), 3 * sizeof(unsigned long long)},
                                    {t.live.get(), sizeof(unsigned long long)},
                                    {td.pcnt.get(), td.pcnt.bytes()}},
                                   sh.stream);
                        // the output's own words start at zero (the first toucher of a word queues it): after a
                        // top-down level only its input queue's words are set, otherwise clear every own row
                        if (prev_td) {
                            if (td.nq_in > 0) {
                                msbfs_zero_list_kernel<<<grid_for(td.nq_in), kBlock, 0, sh.stream>>>(
                                    t.F[cur ^ 1].get(), td.queue[qc ^ 1].get(), td.nq_in);
                                JG_LAUNCH_CHECK();
                            }
                        } else if (level > 0) {  // level 0: F[1] is as the init zeroed it
                            // rows without pull entries are never written after level 0: their words are zero
                            // except an isolated source's level-0 word, cleared apart (RMAT-26: 215 of 537 MB
                            // cleared)
                            const int64_t ne = c.pull && c.pull->empty_from >= 0 ? std::min(c.pull->empty_from, sh.rows)
                                                                                 : sh.rows;
                            JG_HIP(hipMemsetAsync(t.F[cur ^ 1].get(), 0, (size_t)ne * sizeof(unsigned long long), sh.stream));
                            if (ne < sh.rows && !td.src_rows.empty()) {
                                msbfs_zero_tail_sources_kernel<<<1, kWave, 0, sh.stream>>>(
                                    t.F[cur ^ 1].get(), td.srcs.get(), (int)td.src_rows.size(), ne);
                                JG_LAUNCH_CHECK();
                            }
                        }
                        td.nq_in = td.nq;
                        // a big level (one shard): the apply passes over every row instead of a touched list
                        td.rowapply = !td_shard && tune().msbfs_td_rowapply > 0 &&
                                      td.mf * tune().msbfs_td_rowapply >= sh.rows;
                        if (td.mf > 0) {
                            MsTd a{td.queue[qc].get(), td.qoff[qc].get(), td.nq, td.mf, c.push->row_ptr.get(),
                                   c.push->col.get(), t.F[cur].get(), t.vis.get(), t.F[cur ^ 1].get(), td.touched.get(),
                                   td.touched_off.get(), td.ctr.get() + 1, td_shard ? sh.halo_both.tbits : 31,
                                   td_shard ? td.hs.get() : nullptr, td.hlist.get(), td.hlist_off.get(), td.ctr.get() + 2,
                                   td_shard && td.pcnt.size() ? td.pcnt.get() : nullptr, sh.index, g.P,
                                   // the first top-down levels skip the visited probe: next to nothing is visited
                                   // yet, and it is a random 8-byte read per edge (RMAT-26 level 1: 33.6 M)
                                   level >= tune().msbfs_td_noprobe ? 1 : 0, td.rowapply ? 1 : 0};
                            msbfs_td_kernel<<<(unsigned)std::min<int64_t>(std::max<int64_t>(
                                                  (td.mf / kTdEdgesPerThread + kBlock - 1) / kBlock, 1), tune().bfs_grid),
                                              kBlock, 0, sh.stream>>>(a);
                            JG_LAUNCH_CHECK();
                            if (td_shard && td.pcnt.size()) {  // the set slots per peer (the sparse exchange's sizes)
                                msbfs_slot_hist_kernel<<<(unsigned)kRedBlocks, kRedThreads, 0, sh.stream>>>(
                                    td.hlist.get(), td.ctr.get() + 2, sh.halo_both.tbits, sh.index, g.P, td.bcount.get(),
                                    td.pcnt.get());
                                JG_LAUNCH_CHECK();
                            }
                        }
                        fv.push_back(td.hs.peer());
                        rv.push_back(td.rbuf.peer());
                    }
                    // sparse: only the set staging slots travel, as (offset, word) pairs, when they are fewer
                    // than half the halo slots over all shards (the tail levels and the first levels from
                    // the sources set a few thousand)
                    bool sparse_done = false;
                    if (td_shard && tune().msbfs_sparse) {
                        const int P = g.P;
                        std::vector<std::vector<int64_t>> cnt(g.shards.size(), std::vector<int64_t>((size_t)P, 0));
                        std::vector<int64_t> mat((size_t)P * P + 1, 0);
                        for (size_t i = 0; i < g.shards.size(); ++i) {
                            Shard& sh = *g.shards[i];
                            DeviceGuard dg(sh);
                            // per-peer slot counts: the top-down kernel counted the slots it set first
                            std::vector<unsigned long long> c((size_t)P);
                            copy_d2h(c.data(), tds[i].pcnt.get(), (size_t)P * sizeof(unsigned long long), sh.stream);
                            for (int q = 0; q < P; ++q) {
                                cnt[i][(size_t)q] = (int64_t)c[(size_t)q];
                                mat[(size_t)sh.index * P + q] = (int64_t)c[(size_t)q];
                            }
                            mat[(size_t)P * P] += sh.halo_both.recv_off[(size_t)P];  // the dense exchange's words
                        }
                        allreduce_sum_i64(g, mat.data(), P * P + 1);
                        int64_t pairs_all = 0;
                        for (int64_t k = 0; k < (int64_t)P * P; ++k) pairs_all += mat[(size_t)k];
                        if (2 * pairs_all < mat[(size_t)P * P]) {
                            const size_t ns_ = g.shards.size();
                            std::vector<const char*> sp(ns_);
                            std::vector<char*> rp(ns_);
                            std::vector<std::vector<int64_t>> so(ns_), sc(ns_), ro(ns_), rc(ns_);
                            for (size_t i = 0; i < ns_; ++i) {
                                Shard& sh = *g.shards[i];
                                DeviceGuard dg(sh);
                                so[i].assign((size_t)P + 1, 0);
                                ro[i].assign((size_t)P + 1, 0);
                                sc[i].assign((size_t)P, 0);
                                rc[i].assign((size_t)P, 0);
                                PairRuns pk{}, pv{};
                                pk.P = pv.P = P;
                                for (int q = 0; q < P; ++q) {
                                    so[i][(size_t)q + 1] = so[i][(size_t)q] + cnt[i][(size_t)q];
                                    const int64_t from_q = mat[(size_t)q * P + sh.index];
                                    ro[i][(size_t)q + 1] = ro[i][(size_t)q] + from_q;
                                    sc[i][(size_t)q] = 2 * cnt[i][(size_t)q];  // uint64 elements: two per pair
                                    rc[i][(size_t)q] = 2 * from_q;
                                }
                                for (int q = 0; q <= P; ++q) {
                                    pk.off[q] = so[i][(size_t)q];
                                    pv.off[q] = ro[i][(size_t)q];
                                    pv.send_off[q] = sh.halo_both.send_off[(size_t)q];
                                }
                                const int64_t nh = so[i][(size_t)P];
                                if (nh > 0) {
                                    msbfs_pair_pack_kernel<<<(unsigned)kRedBlocks, kRedThreads, 0, sh.stream>>>(
                                        tds[i].hlist.get(), nh, tds[i].hs.get(), sh.halo_both.tbits, sh.index, pk,
                                        tds[i].bcount.get(), tds[i].pairs.get());
                                    JG_LAUNCH_CHECK();
                                }
                                for (int q = 0; q <= P; ++q) {
                                    so[i][(size_t)q] *= 2;
                                    ro[i][(size_t)q] *= 2;
                                }
                                sp[i] = reinterpret_cast<const char*>(tds[i].pairs.get());
                                rp[i] = reinterpret_cast<char*>(tds[i].rpairs.get());
                                tds[i].nrp = ro[i][(size_t)P] / 2;
                                tds[i].pv = pv;
                            }
                            exchange_runs(g, sp, so, sc, rp, ro, rc, sizeof(unsigned long long), ncclUint64);
                            for (size_t i = 0; i < ns_; ++i) {
                                Shard& sh = *g.shards[i];
                                DeviceGuard dg(sh);
                                if (tds[i].nrp > 0) {
                                    msbfs_td_recv_pairs_kernel<<<grid_for(tds[i].nrp), kBlock, 0, sh.stream>>>(
                                        tds[i].rpairs.get(), tds[i].nrp, tds[i].pv, sh.halo_both.send_src.get(),
                                        st[i].vis.get(), st[i].F[cur ^ 1].get(), tds[i].touched.get(),
                                        tds[i].touched_off.get(), tds[i].ctr.get() + 1);
                                    JG_LAUNCH_CHECK();
                                }
                            }
                            sparse_done = true;
                            if (std::getenv("JG_DEBUG_BFS"))
                                std::fprintf(stderr, "[jg msbfs] level %d top-down, sparse reverse exchange: %lld pairs (dense: %lld words)\n",
                                             level, (long long)pairs_all, (long long)mat[(size_t)P * P]);
                        }
                    }
                    if (td_shard && !sparse_done) {
                        exchange_halo_reverse(g, JG_ADJ_BOTH, fv, rv, sizeof(unsigned long long), ncclUint64);
                        for (size_t i = 0; i < g.shards.size(); ++i) {
                            Shard& sh = *g.shards[i];
                            DeviceGuard dg(sh);
                            const int64_t nrecv = sh.halo_both.send_off[g.P];
                            if (nrecv > 0) {
                                msbfs_td_recv_kernel<<<grid_for(nrecv, kBlock, 256 * 8), kBlock, 0, sh.stream>>>(
                                    tds[i].rbuf.get(), sh.halo_both.send_src.get(), nrecv, st[i].vis.get(),
                                    st[i].F[cur ^ 1].get(), tds[i].touched.get(), tds[i].touched_off.get(),
                                    tds[i].ctr.get() + 1);
                                JG_LAUNCH_CHECK();
                            }
                        }
                    }
                    for (size_t i = 0; i < g.shards.size(); ++i) {
                        Shard& sh = *g.shards[i];
                        DeviceGuard dg(sh);
                        const BfsCsrs c = pick_csrs(sh, direction);
                        St& t = st[i];
                        Td& td = tds[i];
                        // counts stay on the device (the apply and the clearing read them there): one host
                        // read-back per level, read_frontier's
                        if (td_shard) {  // the staging slots went out with the reverse exchange: back to zero
                            msbfs_zero_list_packed_kernel<<<grid_for(sh.halo_both.recv_off[(size_t)g.P]), kBlock, 0, sh.stream>>>(
                                td.hs.get(), td.hlist.get(), td.ctr.get() + 2);
                            JG_LAUNCH_CHECK();
                        }
                        td_entries += (double)td.mf;
                        if (debug_bfs())
                            std::fprintf(stderr, "[jg msbfs] level %d top-down (shard %d): %lld frontier rows, %lld push entries\n",
                                         level, sh.index, (long long)td.nq, (long long)td.mf);
                        td_queued += (double)td.nq;
                        if (td.rowapply) td_row_passes += (double)pull_live_rows(sh, c);
                        {
                            MsBfsOp op;
                            op.F = t.F[cur].get();
                            op.Fout = t.F[cur ^ 1].get();
                            op.visited = t.vis.get();
                            op.depth = t.depth.get();
                            op.depth8 = t.depth8.get();
                            op.nwl = nullptr;  // recorded from the next queue below (msbfs_td_record_kernel)
                            op.changed = t.changed.get();
                            op.rows = sh.rows;
                            op.pos = g.vec_pos(sh, adj_of(sh, c));
                            op.lvl = level + 1;
                            op.live = t.live.get() + 1;
                            // (the row-order apply stops at the pull adjacency's empty suffix: a push target has a
                            // pull entry, so no row past it gains a bit after level 0; RMAT-26 BOTH: 34 of 67 M rows)
                            if (td.rowapply)
                                msbfs_td_apply_rows_kernel<<<grid_for(pull_live_rows(sh, c)), kBlock, 0, sh.stream>>>(
                                    pull_live_rows(sh, c), op, c.push->row_ptr.get(), td.queue[qc ^ 1].get(),
                                    td.qoff[qc ^ 1].get(), td.ctr.get(), t.live.get());
                            else
                                msbfs_td_apply_kernel<<<grid_for(sh.rows), kBlock, 0, sh.stream>>>(
                                    td.touched.get(), td.ctr.get() + 1, op, c.push->row_ptr.get(), td.queue[qc ^ 1].get(),
                                    td.qoff[qc ^ 1].get(), td.ctr.get(), t.live.get());
                            JG_LAUNCH_CHECK();
                        }
                    }
                    read_frontier(&td_touched);
                    if (level + 1 < kMsLevelWords)
                        for (size_t i = 0; i < g.shards.size(); ++i) {  // the level's depths: its new queue
                            Shard& sh = *g.shards[i];
                            DeviceGuard dg(sh);
                            St& t = st[i];
                            const int64_t nq = tds[i].nq;
                            t.recs.emplace_back();
                            St::Rec& r = t.recs.back();
                            r.level = level + 1;
                            r.n = nq;
                            r.rows.alloc(std::max<int64_t>(nq, 1));
                            r.words.alloc(std::max<int64_t>(nq, 1));
                            if (nq > 0) {
                                msbfs_td_record_kernel<<<grid_for(nq), kBlock, 0, sh.stream>>>(
                                    tds[i].queue[qc ^ 1].get(), nq, t.F[cur ^ 1].get(),
                                    g.vec_pos(sh, adj_of(sh, pick_csrs(sh, direction))), r.rows.get(), r.words.get());
                                JG_LAUNCH_CHECK();
                            }
                        }
                    combine_live();
                    qc ^= 1;
                    queued = live_ready = true;
                    need_fwd = td_shard;
                    prev_td = true;
                } else {
                    prev_td = false;
                    if (need_fwd) {  // stale halo segments: the lazy forward exchange
                        std::vector<void*> bufs;
                        for (auto& t : st) bufs.push_back(t.F[cur].peer());
                        exchange_vec(g, adj0, bufs, sizeof(unsigned long long), ncclUint64);
                        need_fwd = false;
                    }
                    for (size_t i = 0; i < g.shards.size(); ++i) {
                        Shard& sh = *g.shards[i];
                        DeviceGuard dg(sh);
                        const BfsCsrs c = pick_csrs(sh, direction);
                        const PullPlan& plan = (c.pull == &sh.both) ? sh.plan_both : sh.plan_in;
                        St& t = st[i];
                        // (with the top-down path the frontier count ends the traversal: no changed flag, whose
                        // one-word store every gaining row's wave would repeat)
                        if (!td_ok) JG_HIP(hipMemsetAsync(t.changed.get(), 0, sizeof(int32_t), sh.stream));
                        // rows without pull entries are not written by a pull level: a source among them keeps
                        // its level-0 word in this output vector unless cleared here, and the frontier scan would
                        // count it (one extra level)
                        if (td_ok && c.pull->empty_from >= 0 &&
                            c.pull->empty_from < sh.rows && !tds[i].src_rows.empty()) {
                            msbfs_zero_tail_sources_kernel<<<1, kWave, 0, sh.stream>>>(
                                t.F[cur ^ 1].get(), tds[i].srcs.get(), (int)tds[i].src_rows.size(), c.pull->empty_from);
                            JG_LAUNCH_CHECK();
                        }
                        MsBfsOp op;
                        op.F = t.F[cur].get();
                        op.Fout = t.F[cur ^ 1].get();
                        op.visited = t.vis.get();
                        op.depth = t.depth.get();
                        op.depth8 = t.depth8.get();
                        op.nwl = level + 1 < kMsLevelWords ? t.nwl.get() + (int64_t)(level + 1) * sh.rows : nullptr;
                        op.changed = td_ok ? nullptr : t.changed.get();
                        op.rows = sh.rows;
                        op.pos = g.vec_pos(sh, adj_of(sh, c));
                        op.lvl = level + 1;
                        // Live bits: the sources present in some word of this level's gathered vector.  A row
                        // none of whose unvisited bits is live gains nothing, so the light rows skip it
                        // (MsBfsOp::active) and the split skips every merge task whose rows are all such
                        // (their partials are then stale, and finalize's live mask discards them).  At
                        // RMAT-26 the last pull level has ~all rows done and the one before ~40% of band 0.
                        unsigned long long* lw = t.live.get();
                        if (!have_live) {
                            const int64_t vlen = g.vec_len(sh, adj_of(sh, c));
                            JG_HIP(hipMemsetAsync(lw, 0, sizeof(unsigned long long), sh.stream));
                            msbfs_live_kernel<<<red_grid(vlen), kRedThreads, 0, sh.stream>>>(t.F[cur].get(), vlen, lw);
                            JG_LAUNCH_CHECK();
                        }
                        op.live = lw;
                        // msbfs_skip_first: no task bitmaps on the traversal's first pull level (few rows can be
                        // done there; every task runs, the finalize's live mask keeps it exact)
                        const bool no_bitmaps = pull_levels == 0;
                        // msbfs_exit 1: every row with entries exits early on pull levels where fewer than
                        // msbfs_exit_live permille of band 0's merge tasks hold a row that can still gain a bit
                        // (their live count is read back once); 2: on every pull level
                        const MsBu& bx = t.bx;
                        int64_t exit_rows = bx.rows > 0 && tune().msbfs_exit == 2 ? bx.rows : 0;
                        const bool exit_probe = bx.rows > 0 && tune().msbfs_exit == 1 && !no_bitmaps && !t.todo.empty();
                        std::vector<const uint32_t*> tl;
                        for (size_t b = 0; b < t.todo.size() && !no_bitmaps && !exit_rows; ++b) {
                            const SliceBand& bd = *plan.bands[b];
                            if (bd.tasks == 0 || bd.rows() == 0) {
                                tl.push_back(nullptr);
                                continue;
                            }
                            msbfs_todo_kernel<<<grid_for(bd.rows()), kBlock, 0, sh.stream>>>(
                                t.vis.get(), bd.row_begin, bd.rows(), lw, t.todo[b].get());
                            JG_LAUNCH_CHECK();
                            // band 0 counts its live tasks apart (work[3]), and the count decides: an exit level
                            // builds no bitmaps for the other bands
                            const bool probe = exit_probe && b == 0;
                            if (probe) JG_HIP(hipMemsetAsync(t.work.get() + 3, 0, sizeof(unsigned long long), sh.stream));
                            msbfs_task_live_kernel<<<red_grid(bd.tasks), kRedThreads, 0, sh.stream>>>(
                                bd.task_rows.get(), bd.tasks, t.todo[b].get(), t.tlive[b].get(),
                                t.work.get() + (probe ? 3 : 0));
                            JG_LAUNCH_CHECK();
                            if (probe) {
                                unsigned long long xlive = 0;
                                copy_d2h(&xlive, t.work.get() + 3, sizeof xlive, sh.stream);
                                const bool go = (double)xlive * 1000.0 < (double)t.exit_tasks * (double)tune().msbfs_exit_live;
                                t.xlive_permille = t.exit_tasks ? (double)xlive * 1000.0 / (double)t.exit_tasks : 1000.0;
                                if (debug_bfs())
                                    std::fprintf(stderr, "[jg msbfs] level %d band 0: %llu of %lld merge tasks live -> %s\n",
                                                 level, xlive, (long long)t.exit_tasks, go ? "early exit" : "merge");
                                if (go) {
                                    exit_rows = bx.rows;
                                    break;
                                }
                                t.b0_live_merged += xlive;  // (work[0] holds the other bands' live tasks)
                            }
                            tl.push_back(reinterpret_cast<const uint32_t*>(t.tlive[b].get()));
                        }
                        if (no_bitmaps && i == 0) ++unskipped_levels;
                        if (exit_rows) {  // every row with entries through the exit kernels, no merge launch
                            t.exit_level_tasks += (double)t.all_tasks;
                            if (no_bitmaps) t.exit_unskipped_tasks += (double)t.all_tasks;
                            unsigned long long before = 0, after = 0;
                            if (debug_bfs()) copy_d2h(&before, bx.examined, sizeof before, sh.stream);
                            const unsigned xg = red_grid((bx.rows + 63) / 64 * kWave);
                            msbfs_exit_first_kernel<<<xg, kRedThreads, 0, sh.stream>>>(bx, op, t.xrest.get());
                            JG_LAUNCH_CHECK();
                            msbfs_exit_rest_kernel<<<xg, kRedThreads, 0, sh.stream>>>(bx, op, t.xrest.get());
                            JG_LAUNCH_CHECK();
                            ++t.exit_all_levels;
                            if (debug_bfs()) {
                                copy_d2h(&after, bx.examined, sizeof after, sh.stream);
                                std::fprintf(stderr, "[jg msbfs] level %d exit rows [0, %lld): %llu entries examined\n",
                                             level, (long long)bx.rows, after - before);
                            }
                        } else {
                            // rows without pull entries are not finalised: they gain nothing, their words are zero
                            // on every output vector, and their new-bit words are masked at output
                            // (msbfs_levels_to_planes_kernel)
                            launch_pull(*c.pull, plan, op, t.hub.get(), sh.stream, ctx.profiling ? &ctx : nullptr, &sh,
                                        t.split.size() ? t.split.get() : (unsigned long long*)nullptr, true,
                                        tl.empty() ? nullptr : tl.data());
                        }
                        if (td_ok) {  // the next level's frontier counter (its direction) and, on one shard, live bits
                            zero_words({{tds[i].ctr.get(), sizeof(unsigned long long)}, {lw, sizeof(unsigned long long)}},
                                       sh.stream);
                            // a level whose exit bands had (almost) no live task leaves a small frontier, which
                            // the next level pushes top-down: its queue is built here, in the same pass
                            const bool qnext = td_one && !t.todo.empty() && t.xlive_permille < (double)tune().msbfs_scan_queue;
                            t.xlive_permille = 1000.0;
                            // rows without pull entries gained nothing (a pull level does not finalise them):
                            // the scans stop at the empty suffix (RMAT-26 BOTH: 34 M of 67 M rows)
                            const int64_t ne = pull_live_rows(sh, c);
                            if (qnext) {
                                msbfs_frontier_live_kernel<<<grid_for((ne + 3) / 4), kBlock, 0, sh.stream>>>(
                                    t.F[cur ^ 1].get(), ne, c.push->row_ptr.get(), tds[i].queue[qc ^ 1].get(),
                                    tds[i].qoff[qc ^ 1].get(), tds[i].ctr.get(), lw);
                                queued_next = true;
                            } else {
                                msbfs_scan_kernel<<<red_grid(ne), kRedThreads, 0, sh.stream>>>(
                                    t.F[cur ^ 1].get(), ne, c.push->row_ptr.get(), lw, tds[i].ctr.get());
                            }
                            JG_LAUNCH_CHECK();
                        }
                    }
                    if (td_ok) {
                        read_frontier();
                        combine_live();
                        live_ready = true;
                        if (queued_next) {  // the queue is in slot qc ^ 1 (one shard): the next top-down level's
                            qc ^= 1;
                            queued = true;
                        }
                    }
                    ++pull_levels;
                    need_fwd = g.P > 1;
                }
                int32_t any = 0;
                if (td_ok) {
                    // the level's new frontier (counted over all shards and ranks by read_frontier) is
                    // exactly the rows that gained a bit: no read-back of the changed flags
                    any = g_nq > 0;
                } else {
                    for (size_t i = 0; i < g.shards.size(); ++i) {
                        Shard& sh = *g.shards[i];
                        DeviceGuard dg(sh);
                        int32_t ch = 0;
                        JG_HIP(hipMemcpyAsync(&ch, st[i].changed.get(), sizeof ch, hipMemcpyDeviceToHost, sh.stream));
                        JG_HIP(hipStreamSynchronize(sh.stream));
                        any |= ch;
                    }
                    any = allreduce_or(g, any);
                }
                cur ^= 1;
                ++level;
                if (!any) break;
            }
            JG_HIP(hipEventRecord(t1, sh0.stream));
            region_mark(sh0.stream, false);
            JG_HIP(hipEventSynchronize(t1));
            float ms = 0;
            JG_HIP(hipEventElapsedTime(&ms, t0, t1));
            total_ms += ms;
            max_levels = std::max(max_levels, level);
            // the work of this batch, counted after its timed region: per pull level 12 B per entry of a
            // live merge task (col + gathered frontier word; a task streams its 512 slots) and of the light
            // rows, 32 B per row (visited, the new frontier word, the level's new-bit word, the next
            // level's live scan); per top-down level 12 B per frontier entry, 24 B per touched word and 8 B
            // per queued vertex; past kMsLevelWords levels 4 B per reached (source, row) pair (a plane entry)
            for (size_t i = 0; i < g.shards.size(); ++i) {
                Shard& sh = *g.shards[i];
                DeviceGuard dg(sh);
                St& t = st[i];
                // one shard, BOTH: the visited words past the empty suffix were not cleared (the init); there only
                // the source rows hold bits, one per source
                const BfsCsrs cp = pick_csrs(sh, direction);
                const int64_t prow = td_one && cp.pull == cp.push ? pull_live_rows(sh, cp) : sh.rows;
                if (level >= kMsLevelWords) {  // the plane entries are counted only when planes were written
                    msbfs_pairs_kernel<<<red_grid(prow), kRedThreads, 0, sh.stream>>>(t.vis.get(), prow,
                                                                                       t.work.get() + 1);
                    JG_LAUNCH_CHECK();
                }
                unsigned long long w[3] = {0, 0, 0};
                copy_d2h(w, t.work.get(), sizeof w, sh.stream);
                if (level >= kMsLevelWords && prow < sh.rows)
                    for (int q = 0; q < ns; ++q)
                        if (src_local[(size_t)q] >= prow && src_shard[(size_t)q] == sh.index) ++w[1];
                const double live_tasks = t.todo.empty() ? (double)t.all_tasks * pull_levels - t.exit_level_tasks
                                                          : (double)w[0] +
                                                                (double)t.b0_live_merged +
                                                                (double)t.all_tasks * unskipped_levels -
                                                                t.exit_unskipped_tasks;
                const double entries = live_tasks * kMergeTask + (double)t.light_nnz * (pull_levels - t.exit_all_levels) + (double)w[2];
                work_entries += entries;
                work_bytes += 12.0 * entries + 32.0 * (double)sh.rows * pull_levels +
                              (level >= kMsLevelWords ? 4.0 * (double)w[1] : 0.0);
            }
            work_entries += td_entries;
            work_bytes += 12.0 * td_entries + 24.0 * td_touched + 8.0 * td_queued + 8.0 * td_row_passes;
            if (depth_rows || keep) {
                materialize(level);  // the caller's int32 rows
                if (depth_rows)
                    for (size_t i = 0; i < g.shards.size(); ++i)
                        for (int s = 0; s < ns; ++s)
                            if (depth_rows[b0 + s])
                                rows_to_dense(g, *g.shards[i], st[i].depth.peer() + (size_t)s * g.shards[i]->rows,
                                              depth_rows[b0 + s]);
                if (keep)  // the planes stay with their shards (jg_bfs_kept_row)
                    for (size_t i = 0; i < g.shards.size(); ++i) g.shards[i]->kept_depth.swap(st[i].depth);
            }
        }
        if (keep) g.kept_nsrc = nsrc;
        ctx.last.compute_ms = total_ms;
        ctx.last.levels = max_levels;
        ctx.last.supersteps = max_levels;
        ctx.last.algorithmic_bytes = work_bytes;
        ctx.last.edges_traversed = work_entries;  // adjacency entries the levels examined
        prof_collect(ctx, g);
    }
    JG_HIP(hipEventDestroy(t0));
    JG_HIP(hipEventDestroy(t1));
}

// Sharded ShortestDistanceVertexProgram (weighted or unit): the same exact supersteps as the single
// shard (push from the rows whose distance fell last superstep, min into `best`, apply), over the IN
// adjacency's halo plan.  Candidates for remote vertices collect in their halo slots and go to the
// owners by the reverse halo exchange (the transpose of the PageRank/CC exchange), which take their
// min; frontier sizes are summed over shards and ranks every superstep.
static const char* const kMissingWeight =
    "a message crossed an edge without the weight property (ShortestDistanceVertexProgram.java:69 "
    "edge.value(weightProperty) throws)";

static void shortest_distance_sharded(Graph& g, int64_t seed_vid, int max_depth, int64_t* dist_out) {
    Ctx& ctx = *g.ctx;
    const size_t ns = g.shards.size();
    for (auto& sp : g.shards)
        if (!sp->halo_in.on)
            fail(JG_ERR_UNSUPPORTED, "sharded shortest distance needs the halo plan (tune \"halo\" = 1 at build)");
    int seed_shard = -1;
    const int64_t seed_local = local_of_vid(g, seed_vid, &seed_shard);
    struct St {
        DevBuf<long long> best, dist, msg, rbuf;
        DevBuf<int32_t> fa, fb, touched;
        DevBuf<int64_t> qa, qb;  // the frontier's first edge numbers
        DevBuf<unsigned long long> sizes;
        DevBuf<int32_t> err;
        int64_t fsize = 0, fedges = 0;
    };
    std::vector<St> st(ns);
    std::vector<void*> bv, rv;
    for (size_t i = 0; i < ns; ++i) {
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        const Halo& h = sh.halo_in;
        St& t = st[i];
        const int64_t rows = std::max<int64_t>(sh.rows, 1);
        t.best.alloc(std::max<int64_t>(h.C, 1));
        t.dist.alloc(rows);
        t.msg.alloc(rows);
        t.fa.alloc(rows);
        t.fb.alloc(rows);
        t.qa.alloc(rows);
        t.qb.alloc(rows);
        t.touched.alloc(rows);
        t.rbuf.alloc(std::max<int64_t>(h.send_off[g.P], 1));
        t.sizes.alloc(2);
        t.err.alloc(1);
        JG_HIP(hipMemsetAsync(t.err.get(), 0, sizeof(int32_t), sh.stream));
        fill_ll_kernel<<<grid_for(h.C), kBlock, 0, sh.stream>>>(t.best.get(), h.C, LLONG_MAX);
        fill_ll_kernel<<<grid_for(sh.rows), kBlock, 0, sh.stream>>>(t.dist.get(), sh.rows, LLONG_MIN);  // absent
        JG_LAUNCH_CHECK();
        if (seed_local >= 0 && sh.index == seed_shard) {
            const long long zero = 0;
            const int32_t seed32 = (int32_t)seed_local;
            copy_h2d(t.dist.get() + seed_local, &zero, sizeof zero, sh.stream);
            copy_h2d(t.msg.get() + seed_local, &zero, sizeof zero, sh.stream);
            copy_h2d(t.fa.get(), &seed32, sizeof seed32, sh.stream);
            const int64_t zero64 = 0;
            copy_h2d(t.qa.get(), &zero64, sizeof zero64, sh.stream);
            int64_t srp[2];
            copy_d2h(srp, sh.in.row_ptr.get() + seed_local, sizeof srp, sh.stream);
            t.fsize = 1;
            t.fedges = srp[1] - srp[0];
        }
        bv.push_back(t.best.peer());
        rv.push_back(t.rbuf.peer());
    }
    int64_t total = seed_local >= 0 ? 1 : 0;
    allreduce_sum_i64(g, &total, 1);
    Shard& sh0 = *g.shards[0];
    hipEvent_t t0, t1;
    {
        DeviceGuard dg(sh0.device);
        JG_HIP(hipEventCreate(&t0));
        JG_HIP(hipEventCreate(&t1));
        region_mark(sh0.stream, true);
        JG_HIP(hipEventRecord(t0, sh0.stream));
    }
    int levels = 0;
    for (int lv = 1; lv <= max_depth && total > 0; ++lv) {
        for (size_t i = 0; i < ns; ++i) {
            Shard& sh = *g.shards[i];
            DeviceGuard dg(sh);
            St& t = st[i];
            JG_HIP(hipMemsetAsync(t.sizes.get(), 0, 2 * sizeof(unsigned long long), sh.stream));
            if (t.fsize > 0 && t.fedges > 0) {
                SsdPushQ a{sh.in.row_ptr.get(), sh.in.col.get(), g.has_weights ? sh.in.weight.get() : nullptr, t.fa.get(),
                           t.qa.get(), t.fsize, t.fedges, t.msg.get(), t.best.get(), sh.halo_in.tbits, t.touched.get(),
                           t.sizes.get(), t.err.get()};
                const unsigned grid = (unsigned)std::min<int64_t>(
                    std::max<int64_t>((t.fedges + (int64_t)kBlock * kTdEdgesPerThread - 1) / ((int64_t)kBlock * kTdEdgesPerThread), 1),
                    8192);
                ssd_push_q_kernel<<<grid, kBlock, 0, sh.stream>>>(a);
                JG_LAUNCH_CHECK();
            }
        }
        exchange_halo_reverse(g, JG_ADJ_IN, bv, rv, sizeof(long long), ncclInt64);
        int64_t next = 0;
        for (size_t i = 0; i < ns; ++i) {
            Shard& sh = *g.shards[i];
            DeviceGuard dg(sh);
            St& t = st[i];
            const Halo& h = sh.halo_in;
            const int64_t nrecv = h.send_off[g.P];
            if (nrecv > 0) {
                ssd_recv_kernel<<<grid_for(nrecv, kBlock, 256 * 8), kBlock, 0, sh.stream>>>(
                    t.rbuf.get(), h.send_src.get(), nrecv, t.best.get(), t.touched.get(), t.sizes.get());
                JG_LAUNCH_CHECK();
            }
            {  // the halo slots are sent: back to "no candidate"
                SlotRuns r{};
                int nr_runs = 0;
                int64_t nmax = 0;
                for (int q = 0; q < g.P; ++q) {
                    const int64_t nr = h.recv_off[q + 1] - h.recv_off[q];
                    if (q == sh.index || nr == 0) continue;
                    if (nr_runs == 64) {  // (more than 65 shards: the runs so far in one launch, then on)
                        ssd_reset_slots_kernel<<<dim3(grid_for(nmax, kBlock, 1024), 64u), kBlock, 0, sh.stream>>>(r);
                        JG_LAUNCH_CHECK();
                        nr_runs = 0;
                        nmax = 0;
                    }
                    r.p[nr_runs] = t.best.get() + ((int64_t)h.seg_of(q, sh.index) << h.tbits);
                    r.n[nr_runs++] = nr;
                    nmax = std::max(nmax, nr);
                }
                if (nr_runs > 0) {
                    ssd_reset_slots_kernel<<<dim3(grid_for(nmax, kBlock, 1024), (unsigned)nr_runs), kBlock, 0, sh.stream>>>(r);
                    JG_LAUNCH_CHECK();
                }
            }
            unsigned long long ts = 0;
            copy_d2h(&ts, t.sizes.get(), sizeof ts, sh.stream);
            if (ts > 0) {
                ssd_apply_q_kernel<<<grid_for((int64_t)ts, kBlock, 256 * 8), kBlock, 0, sh.stream>>>(
                    t.touched.get(), (int64_t)ts, t.best.get(), t.dist.get(), t.msg.get(), sh.in.row_ptr.get(), t.fb.get(),
                    t.qb.get(), t.sizes.get() + 1);
                JG_LAUNCH_CHECK();
            }
            unsigned long long nn = 0;
            copy_d2h(&nn, t.sizes.get() + 1, sizeof nn, sh.stream);
            t.fsize = (int64_t)(nn >> kPackShift);
            t.fedges = (int64_t)(nn & kEdgeMask);
            t.fa.swap(t.fb);
            t.qa.swap(t.qb);
            next += t.fsize;
        }
        allreduce_sum_i64(g, &next, 1);
        total = next;
        levels = lv;
    }
    float ms = 0;
    {
        DeviceGuard dg(sh0.device);
        JG_HIP(hipEventRecord(t1, sh0.stream));
        region_mark(sh0.stream, false);
        JG_HIP(hipEventSynchronize(t1));
        JG_HIP(hipEventElapsedTime(&ms, t0, t1));
        (void)hipEventDestroy(t0);
        (void)hipEventDestroy(t1);
    }
    int missing = 0;
    for (size_t i = 0; i < ns; ++i) {
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        int32_t e = 0;
        copy_d2h(&e, st[i].err.get(), sizeof e, sh.stream);
        missing |= e;
        rows_to_dense(g, sh, st[i].dist.get(), reinterpret_cast<long long*>(dist_out));  // LLONG_MIN: absent
    }
    if (allreduce_or(g, missing)) fail(JG_ERR_ARG, kMissingWeight);
    ctx.last.compute_ms = ms;
    ctx.last.levels = levels;
    ctx.last.supersteps = max_depth;
}

// The weight statistics of c (sd_weight_stats_kernel), cached on the CSR.
const long long* sd_weight_stats(Shard& sh, const Csr& c) {
    if (!c.wstat_ok) {
        hipStream_t s = sh.stream;
        DevBuf<long long> out(4);
        const long long init[4] = {LLONG_MAX, 0, 0, LLONG_MIN};
        copy_h2d(out.get(), init, sizeof init, s);
        if (c.nnz > 0 && c.weight.get()) {
            sd_weight_stats_kernel<<<grid_for(c.nnz), kBlock, 0, s>>>(c.weight.get(), c.nnz, out.get());
            JG_LAUNCH_CHECK();
        }
        copy_d2h(c.wstat, out.get(), sizeof c.wstat, s);
        c.wstat_ok = true;
    }
    return c.wstat;
}

// delta: Tune::sd_delta when set, else kSdDeltaScale x the mean weight / the mean in-degree, at least 1
// (the near-far rule of thumb, delta ~ c w / d; RMAT-20 / 22 with weights 1..255 and c = 32, 128: 1.50 /
// 3.40 and 1.23 / 3.05 ms, c = 512 equal to 128: profiles/r05/sssp/)
constexpr double kSdDeltaScale = 128.0;
long long sd_auto_delta(const long long* ws, int64_t nnz, int64_t rows) {
    if (tune().sd_delta > 0) return tune().sd_delta;
    const double mean_w = ws[2] > 0 ? (double)ws[1] / (double)ws[2] : 1.0;
    const double mean_deg = std::max(1.0, (double)nnz / (double)std::max<int64_t>(rows, 1));
    return std::max<long long>(1, (long long)std::llround(kSdDeltaScale * mean_w / mean_deg));
}

// Near-far delta-stepping from `seed` over sh.in (see sd_near_kernel); host[] gets the distances
// (INT64_MIN: absent); end_ev is recorded once the distances are final, before they are copied out.
// Returns the near passes run.
template <class D>
int sd_delta_stepping_t(Shard& sh, int64_t seed, long long delta, int64_t* host, hipEvent_t end_ev) {
    hipStream_t s = sh.stream;
    const int64_t rows = sh.rows, cap = std::max<int64_t>(rows, 1);
    const Csr& c = sh.in;
    DevBuf<D> dist(cap);
    DevBuf<int32_t> nq[2] = {DevBuf<int32_t>(cap), DevBuf<int32_t>(cap)};
    DevBuf<int64_t> qo[2] = {DevBuf<int64_t>(cap), DevBuf<int64_t>(cap)};
    DevBuf<int32_t> far[2] = {DevBuf<int32_t>(cap), DevBuf<int32_t>(cap)};
    DevBuf<int32_t> stamp(cap), far_flag(cap), err(1);
    DevBuf<unsigned long long> ring(2 * kSdRing + 3);  // nctr[kSdRing], fmin[kSdRing], fsz[2], passes
    DevBuf<SdState> st(kSdRing);
    SdStep<D> a{};
    a.rp = c.row_ptr.get();
    a.col = c.col.get();
    a.wt = c.weight.get();
    a.dist = dist.get();
    for (int k = 0; k < 2; ++k) {
        a.nq[k] = nq[k].get();
        a.qo[k] = qo[k].get();
        a.far[k] = far[k].get();
    }
    a.nctr = ring.get();
    a.fmin = ring.get() + kSdRing;
    a.fsz = ring.get() + 2 * kSdRing;
    a.passes = ring.get() + 2 * kSdRing + 2;
    a.far_flag = far_flag.get();
    a.stamp = stamp.get();
    a.st = st.get();
    a.err = err.get();
    a.delta = delta;
    sd_init_kernel<D><<<grid_for(rows), kBlock, 0, s>>>(a, rows, (int32_t)seed, delta);
    JG_LAUNCH_CHECK();
    // Fixed grids (the host does not know a pass's size): the near pass grid-strides over its edges, a
    // workgroup whose slice of a tile is past the end leaves at once.  tools/sd_bench.py, weights 1..255,
    // median ms at a cap of 4096 / 8192 / 16384 / 32768 / 65536 near workgroups: RMAT-24 10.25 / 9.94 / 9.68 /
    // 9.95 / 10.41, RMAT-22 2.84 / 2.74 / 2.72 (its entries / 4096 = 16384); split 1024 -> 256: equal
    // (profiles/r06/sssp_ctl/)
    const unsigned near_grid = (unsigned)std::min<int64_t>(std::max<int64_t>(c.nnz / ((int64_t)kBlock * kTdEdgesPerThread * 4), 64), 16384);
    const unsigned split_grid = (unsigned)std::min<int64_t>(std::max<int64_t>(rows / ((int64_t)kBlock * 8), 16), 256);
    // Steps in batches, the state read once per batch: the first sized from the last calls' step counts
    int step = 0, predicted = 0;
    for (int k = 0; k < std::min(sh.sd_hist_n, 4); ++k) predicted = std::max(predicted, sh.sd_hist[k]);
    SdState hs{};
    for (int batch = predicted > 0 ? predicted + 1 : 16, next_batch = 8;; batch = next_batch, next_batch = std::min(next_batch * 2, 64)) {
        if (step > (1 << 26)) fail(JG_ERR_STATE, "delta-stepping control did not terminate");
        for (int k = 0; k < batch; ++k, ++step) {
            a.step = step;
            sd_split_kernel<D><<<split_grid, kBlock, 0, s>>>(a);
            JG_LAUNCH_CHECK();
            sd_near_kernel<D><<<near_grid, kBlock, 0, s>>>(a);
            JG_LAUNCH_CHECK();
        }
        copy_d2h(&hs, st.get() + (step - 1) % kSdRing, sizeof hs, s);
        if (hs.done) break;
    }
    JG_HIP(hipEventRecord(end_ev, s));  // the distances are final: their copy-out is the caller's
    region_mark(s, false);
    unsigned long long passes = 0;
    copy_d2h(&passes, a.passes, sizeof passes, s);
    // the steps this call needed: up to the one that found nothing left (the next call's first batch)
    for (int k = 3; k > 0; --k) sh.sd_hist[k] = sh.sd_hist[k - 1];
    sh.sd_hist[0] = hs.end_step + 1;
    sh.sd_hist_n = std::min(sh.sd_hist_n + 1, 4);
    std::vector<D> hd(rows);
    if (rows) copy_d2h(hd.data(), dist.get(), rows * sizeof(D), s);
    for (int64_t l = 0; l < rows; ++l) host[l] = hd[l] == DistTraits<D>::kNone ? LLONG_MIN : (int64_t)hd[l];
    int32_t e = 0;
    copy_d2h(&e, err.get(), sizeof e, s);
    if (e) fail(JG_ERR_ARG, kMissingWeight);
    return (int)passes;
}

// 32-bit distances when no stored distance can reach UINT_MAX: a row's first distance is the length of a
// path of at most rows - 1 entries (the first-touch tree has no cycle), every later one is smaller, and a
// candidate adds one more weight (ws: sd_weight_stats).  Tune::sd_dist32: 0 keeps 64 bits, 2 takes 32 when
// safe, 1 (default) when safe and rows >= 2^23: weights 1..255, tools/sd_bench.py, median ms 64 / 32 bits,
// RMAT-20 1.197 / 1.249, RMAT-22 3.036 / 3.130, RMAT-24 10.715 / 10.228 (fabric reads -18% at RMAT-22, but
// the near pass is bound by its random round trips and atomics more than by the lines they move;
// profiles/r06/sssp32/)
int sd_delta_stepping(Shard& sh, int64_t seed, long long delta, int64_t* host, hipEvent_t end_ev, const long long* ws) {
    const unsigned long long wmax = ws[3] > 0 ? (unsigned long long)ws[3] : 0ull;
    const unsigned long long bound = (unsigned long long)std::max<int64_t>(sh.rows, 1) * wmax;  // rows * wmax
    const bool want32 = tune().sd_dist32 == 2 || (tune().sd_dist32 == 1 && sh.rows >= (1ll << 23));
    if (want32 && wmax < (1ull << 31) && (uint64_t)sh.rows < (1ull << 32) && bound < (unsigned long long)UINT_MAX)
        return sd_delta_stepping_t<unsigned int>(sh, seed, delta, host, end_ev);
    return sd_delta_stepping_t<long long>(sh, seed, delta, host, end_ev);
}

void shortest_distance_run(Graph& g, int64_t seed_vid, int max_depth, int64_t* dist_out) {
    Ctx& ctx = *g.ctx;
    ctx.last = jg_stats{};
    prof_discard_exchanges(g);  // exchange pairs of this call only
    if (!(g.flags & JG_ADJ_IN)) fail(JG_ERR_UNSUPPORTED, "shortest distance needs a graph built with JG_ADJ_IN");
    if (g.P != 1) {
        shortest_distance_sharded(g, seed_vid, max_depth, dist_out);
        return;
    }
    Shard& sh = *g.shards[0];
    DeviceGuard dg(sh);
    hipStream_t s = sh.stream;
    const int64_t rows = sh.rows;
    int shard = 0;
    const int64_t seed = local_of_vid(g, seed_vid, &shard);
    std::vector<int64_t> host(rows, LLONG_MIN);  // absent
    hipEvent_t t0, t1;
    JG_HIP(hipEventCreate(&t0));
    JG_HIP(hipEventCreate(&t1));
    if (seed >= 0 && !g.has_weights) {
        bfs_buffers(sh);
        if (sh.out.present()) bfs_first_col(sh, sh.out);  // the traversal's pull adjacency
    }
    // weighted with an unbounded hop count and no negative weight: delta-stepping (the weight
    // statistics are taken once per graph, outside the timed region)
    long long delta = 0;
    if (seed >= 0 && g.has_weights && tune().sd_delta != 0 && (int64_t)max_depth >= rows - 1) {
        const long long* ws = sd_weight_stats(sh, sh.in);
        if (ws[0] >= 0) delta = sd_auto_delta(ws, sh.in.nnz, rows);
    }
    region_mark(s, true);
    JG_HIP(hipEventRecord(t0, s));
    int levels = 0;
    bool timed_end = false;  // t1 recorded by the branch (before its output copy)
    if (seed >= 0 && !g.has_weights) {
        // unit weights: min over <= maxDepth-hop paths == BFS depth along IN edges, capped
        DevBuf<int32_t> depth(std::max<int64_t>(rows, 1));
        BfsCsrs c{&sh.in, sh.out.present() ? &sh.out : nullptr};
        levels = dobfs_single(ctx, sh, c, seed, max_depth, depth.get(), nullptr, nullptr, t1);
        timed_end = true;
        std::vector<int32_t> h(rows);
        if (rows) copy_d2h(h.data(), depth.get(), rows * sizeof(int32_t), s);
        for (int64_t l = 0; l < rows; ++l) host[l] = h[l] >= 0 ? h[l] : LLONG_MIN;
    } else if (seed >= 0 && delta > 0) {
        levels = sd_delta_stepping(sh, seed, delta, host.data(), t1, sd_weight_stats(sh, sh.in));
        timed_end = true;
    } else if (seed >= 0) {
        const int64_t cap = std::max<int64_t>(rows, 1);
        DevBuf<long long> dist(cap), msg(cap), best(cap);
        DevBuf<int32_t> fa(cap), fb(cap), touched(cap);
        DevBuf<int64_t> qa(cap), qb(cap);
        DevBuf<unsigned long long> ring(2 * kSdRing);  // frontier counts, touched counts
        DevBuf<SdSuper> sst(kSdRing);
        DevBuf<int32_t> err(1);
        SdPush a{};
        a.rp = sh.in.row_ptr.get();
        a.col = sh.in.col.get();
        a.wt = sh.in.weight.get();
        a.frontier[0] = fa.get();
        a.frontier[1] = fb.get();
        a.qoff[0] = qa.get();
        a.qoff[1] = qb.get();
        a.fr = ring.get();
        a.tsz = ring.get() + kSdRing;
        a.st = sst.get();
        a.msg = msg.get();
        a.best = best.get();
        a.dist = dist.get();
        a.touched = touched.get();
        a.err = err.get();
        sd_super_init_kernel<<<grid_for(rows), kBlock, 0, s>>>(a, rows, (int32_t)seed);
        JG_LAUNCH_CHECK();
        // fixed grids (the host does not know a superstep's size): the push grid-strides over its edges
        const unsigned push_grid = (unsigned)std::min<int64_t>(
            std::max<int64_t>(sh.in.nnz / ((int64_t)kBlock * kTdEdgesPerThread * 4), 64), 16384);
        const unsigned apply_grid = grid_for(rows, kBlock, 4096);
        SdSuper hs{};
        int t = 1;
        for (int batch = std::min(max_depth, 16), next_batch = 8; t <= max_depth;
             batch = std::min(next_batch, max_depth - t + 1), next_batch = std::min(next_batch * 2, 64)) {
            for (int k = 0; k < batch; ++k, ++t) {
                a.t = t;
                sd_push_q_kernel<<<push_grid, kBlock, 0, s>>>(a);
                JG_LAUNCH_CHECK();
                sd_apply_q_kernel<<<apply_grid, kBlock, 0, s>>>(a);
                JG_LAUNCH_CHECK();
            }
            copy_d2h(&hs, sst.get() + (t - 1) % kSdRing, sizeof hs, s);
            if (hs.done) break;
        }
        levels = hs.levels;
        JG_HIP(hipEventRecord(t1, s));  // the distances are final: the copy-out is outside the timed region
        region_mark(s, false);
        timed_end = true;
        std::vector<long long> h(rows);
        if (rows) copy_d2h(h.data(), dist.get(), rows * sizeof(long long), s);
        for (int64_t l = 0; l < rows; ++l) host[l] = h[l];
        int32_t e = 0;
        copy_d2h(&e, err.get(), sizeof e, s);
        if (e) fail(JG_ERR_ARG, kMissingWeight);
    }
    if (!timed_end) {
        JG_HIP(hipEventRecord(t1, s));
        region_mark(s, false);
    }
    JG_HIP(hipEventSynchronize(t1));
    float ms = 0;
    JG_HIP(hipEventElapsedTime(&ms, t0, t1));
    JG_HIP(hipEventDestroy(t0));
    JG_HIP(hipEventDestroy(t1));
    ctx.last.compute_ms = ms;
    ctx.last.levels = levels;
    ctx.last.supersteps = max_depth;  // Fulgora always runs supersteps 0..maxDepth
    for (int64_t l = 0; l < rows; ++l) dist_out[sh.dense_of_local()[l]] = host[l];
    prof_collect(ctx, g);
}

}  // namespace jg
