// jg_narrow.hip — narrow bit-parallel direction-optimising BFS: 2..8 sources on one shard.
//
// Reference semantics: TinkerPop ShortestPathVertexProgram's hop depths under Fulgora's forced
// {Local(bothE), Global} scopes (janusgraph-core/.../olap/computer/FulgoraGraphComputer.java:249-253),
// the same depths jg_traverse.hip computes; only the engine differs.
//
// Why a second bit-parallel engine: the 64-source engine's pull levels
// gather an 8-byte word per adjacency entry through the merge engine and cannot stop a row early, so 8
// sources cost as much as 64 there (RMAT-26: 9.2-13.5 ms for 8 against 11.1 ms for 64; profiles/r05/groups).
// Here a frontier is one byte per row (8 sources), so a level's frontier vector (67 MB at RMAT-26) stays
// in the 256 MiB Infinity Cache, and every source runs Beamer's direction rule on its own frontier:
//   * bottom-up sources (large frontiers): every row with an unvisited bottom-up bit scans its pull row
//     until it holds all of them (pass A: a lane per row, its first `first` entries; pass B: a wave per
//     unfinished row, 256 entries per step);
//   * top-down sources (small frontiers): edge-parallel push over a queue of the frontier rows holding a
//     top-down bit, a 32-bit atomicOr of the byte into the next frontier, first toucher queued.
// A level's launches read their decisions from device state the level's first kernel derives from the
// previous level's counters (per-source frontier rows and push entries), so the host reads the state
// once per batch of levels, as the single-source DO-BFS does.  Level L's frontier array F_L holds the
// bits that reached each row at level L, so the arrays are the depths (nb_planes_kernel).
#include <climits>

#include "jg_frontier.h"
#include "jg_internal.h"

namespace jg {

namespace {

constexpr int kNbRing = 4;         // per-level state / counters: a level touches slots L-1, L, L+1
constexpr int kNbStep = 256;       // pass B: entries a wave scans per step (4 per lane)
constexpr int kNbEpt = 4;          // top-down: edges per thread beyond the grid
constexpr int kNbSamples = 1024;   // top-down: LDS samples of the queue's edge offsets

// Counters of the frontier a level produces (zeroed two levels ahead by the first kernel's block 0)
struct NbCtr {
    unsigned long long nf[kNarrowMax];  // rows that gained source s's bit
    unsigned long long mf[kNarrowMax];  // their push entries
    unsigned long long q;               // packed (rows << kPackShift | entries) of the next level's queue
    unsigned long long scanq;           // packed counter of a queue this level built by a scan
    unsigned long long examined;        // adjacency entries this level examined
    unsigned long long pad;
};
constexpr int kNbCtrWords = sizeof(NbCtr) / sizeof(unsigned long long);
constexpr int kNbSums = 2 * kNarrowMax + 1;  // nf, mf, examined: what a kernel adds up

struct NbState {
    long long explored[kNarrowMax];  // push entries of every frontier of s so far (Beamer's unexplored)
    unsigned tdm, bum;               // sources pushed top-down / pulled bottom-up at this level
    unsigned bumode;                 // sources in bottom-up mode (sticky until the frontier shrinks)
    unsigned qmask;                  // the level's queue (for the next level) holds rows with these bits
    int scan;                        // this level's queue must be built by a scan of its frontier
    int done, levels, pad;
};

struct NbLevel {
    const int64_t* push_rp;
    const int32_t* push_col;
    const int64_t* pull_rp;
    const int32_t* pull_col;
    const int32_t* pull_first;  // [rows] each pull row's first column (Csr::first_col)
    const uint8_t* Fc;  // F_L: this level's frontier (rows [0, ne) defined; level 0: every row)
    uint8_t* Fn;        // F_{L+1}
    uint8_t* vis;
    unsigned long long* rest;  // [ceil(ne / 64)]
    int32_t* queue_in;  // the level's top-down queue (slot L & 1)
    int64_t* qoff_in;
    int32_t* queue_out;  // the next level's (slot (L + 1) & 1)
    int64_t* qoff_out;
    NbCtr* ctr;
    NbState* st;
    unsigned long long* tot;  // [2] examined entries, reached pairs (whole traversal)
    int64_t rows, ne, push_nnz;
    int level, max_depth, ns, first;
    double alpha, beta;
};

// Beamer per source: top-down -> bottom-up when the frontier's push entries exceed the entries not yet
// in any of its frontiers / alpha, back when its frontier holds fewer than rows / beta rows.
__device__ NbState nb_decide(const NbLevel& a) {
    const int pl = (a.level + kNbRing - 1) % kNbRing;
    const NbState p = a.st[pl];
    const NbCtr& h = a.ctr[pl];
    NbState c = p;
    c.tdm = c.bum = 0;
    c.scan = 0;
    if (p.done) return c;
    unsigned live = 0, bumode = 0;
    for (int s = 0; s < a.ns; ++s) {
        const long long mf = (long long)h.mf[s], nf = (long long)h.nf[s];
        c.explored[s] = p.explored[s] + mf;
        if (nf == 0) continue;
        live |= 1u << s;
        bool bu = (p.bumode >> s) & 1u;
        const double mu = (double)(a.push_nnz - c.explored[s]);
        if (!bu && (double)mf > mu / a.alpha) bu = true;
        else if (bu && (double)nf < (double)a.rows / a.beta) bu = false;
        if (bu) bumode |= 1u << s;
    }
    if (!live || (a.max_depth >= 0 && a.level >= a.max_depth)) {
        c.done = 1;
        c.levels = a.level;
        return c;
    }
    c.bumode = bumode;
    c.bum = bumode;
    c.tdm = live & ~bumode;
    // the previous level queued the rows that gained one of its top-down sources' bits: exactly this
    // level's queue when the top-down sources are the same (those still live)
    c.scan = c.tdm != 0 && c.tdm != (p.qmask & live);
    c.qmask = c.tdm;
    return c;
}

// per-lane sums: rows gaining each bit and their push entries, entries examined
struct NbSums {
    unsigned nf[kNarrowMax];
    unsigned long long mf[kNarrowMax];
    unsigned long long ex;
    __device__ void zero() {
#pragma unroll
        for (int s = 0; s < kNarrowMax; ++s) nf[s] = 0, mf[s] = 0;
        ex = 0;
    }
    __device__ void add(unsigned bits, long long deg) {
#pragma unroll
        for (int s = 0; s < kNarrowMax; ++s) {
            const unsigned b = (bits >> s) & 1u;
            nf[s] += b;
            mf[s] += b ? (unsigned long long)deg : 0ull;
        }
    }
};
// every thread of the block calls once at its end: wave sums, LDS, one atomic per counter per block;
// tot[0] / tot[1]: the traversal's examined entries and reached (source, row) pairs
__device__ void nb_flush(const NbSums& t, NbCtr* out, unsigned long long* tot, unsigned long long* s_sum) {
    if (threadIdx.x < kNbSums) s_sum[threadIdx.x] = 0;
    __syncthreads();
    unsigned long long v[kNbSums];
#pragma unroll
    for (int s = 0; s < kNarrowMax; ++s) {
        v[s] = t.nf[s];
        v[kNarrowMax + s] = t.mf[s];
    }
    v[kNbSums - 1] = t.ex;
#pragma unroll
    for (int k = 0; k < kNbSums; ++k) {
        const unsigned long long w = wave_reduce_add(v[k]);
        if (lane_id() == 0 && w) atomicAdd(&s_sum[k], w);
    }
    __syncthreads();
    if (threadIdx.x < kNbSums && s_sum[threadIdx.x]) {
        const int k = (int)threadIdx.x;
        unsigned long long* dst = k < kNarrowMax ? &out->nf[k] : k < 2 * kNarrowMax ? &out->mf[k - kNarrowMax] : &out->examined;
        atomicAdd(dst, s_sum[k]);
    }
    if (threadIdx.x == kWave) {  // another wave than the counters' threads
        unsigned long long pairs = 0;
        for (int k = 0; k < kNarrowMax; ++k) pairs += s_sum[k];
        if (s_sum[kNbSums - 1]) atomicAdd(&tot[0], s_sum[kNbSums - 1]);
        if (pairs) atomicAdd(&tot[1], pairs);
    }
}

__device__ __forceinline__ long long nb_push_deg(const NbLevel& a, int64_t v, int64_t j0, int64_t j1) {
    return a.push_rp == a.pull_rp ? (long long)(j1 - j0) : (long long)(a.push_rp[v + 1] - a.push_rp[v]);
}

// First kernel of a level: the decision; bottom-up pass A over rows [0, ne) (a lane per row, 64
// consecutive rows per wave); without bottom-up sources, F_{L+1} is zeroed for the top-down atomics.
__global__ __launch_bounds__(kBlock) void nb_bu_kernel(NbLevel a) {
    __shared__ NbState s_st;
    __shared__ unsigned long long s_sum[kNbSums];
    if (threadIdx.x == 0) {
        s_st = nb_decide(a);
        if (blockIdx.x == 0) a.st[a.level % kNbRing] = s_st;
    }
    if (blockIdx.x == 0 && threadIdx.x < kNbCtrWords)  // the counters of level L + 1's output
        reinterpret_cast<unsigned long long*>(a.ctr + (a.level + 1) % kNbRing)[threadIdx.x] = 0ull;
    __syncthreads();
    if (s_st.done) return;
    const unsigned bum = s_st.bum;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    if (!bum) {
        // 16-byte stores; the tail of the last partial 16 bytes byte by byte
        const int64_t n16 = a.ne / 16;
        uint4* f4 = reinterpret_cast<uint4*>(a.Fn);
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) f4[i] = make_uint4(0, 0, 0, 0);
        for (int64_t i = n16 * 16 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.ne; i += stride) a.Fn[i] = 0;
        return;
    }
    NbSums sum;
    sum.zero();
    // F_L is defined on rows [0, ne) (level 0: every row); a directed traversal's pull rows can name rows
    // past ne (no pull entries of their own, so never reached after level 0): they hold no bit
    const int64_t fdef = a.level == 0 ? a.rows : a.ne;
    for (int64_t base = ((int64_t)blockIdx.x * blockDim.x) + wave_id() * kWave; base < a.ne; base += stride) {
        const int64_t v = base + lane_id();
        const bool in = v < a.ne;
        const unsigned vis = in ? a.vis[v] : 0xFFu;
        const unsigned need = ~vis & bum & 0xFFu;
        unsigned acc = 0;
        bool rest = false;
        if (need) {
            const int64_t j0 = a.pull_rp[v], j1 = a.pull_rp[v + 1];
            const int64_t je = j0 + a.first < j1 ? j0 + a.first : j1;
            int64_t j = j0;
            if (j < je) {  // the first (highest-degree) neighbour alone, as in bfs_bottom_up
                const int32_t u0 = a.pull_first[v];  // (the dense array: one coalesced load)
                ++j;
                acc |= (u0 < fdef ? a.Fc[u0] : 0u) & need;
            }
            for (; j < je && acc != need; j += 4) {
                int32_t u[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) u[k] = a.pull_col[j + k < je ? j + k : je - 1];
                unsigned f = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) f |= u[k] < fdef ? a.Fc[u[k]] : 0u;
                acc |= f & need;
            }
            sum.ex += (unsigned long long)((j < je ? j : je) - j0);
            rest = acc != need && je < j1;
            if (!rest && acc) {
                a.vis[v] = (uint8_t)(vis | acc);
                sum.add(acc, nb_push_deg(a, v, j0, j1));
            }
        }
        if (in) a.Fn[v] = (uint8_t)acc;  // final, or pass B's start
        const uint64_t word = __ballot(rest);
        if (lane_id() == 0) a.rest[base >> 6] = word;
    }
    nb_flush(sum, a.ctr + a.level % kNbRing, a.tot, s_sum);
}

// Bottom-up pass B: a wave per row pass A left unfinished, kNbStep entries per step, until the row holds
// every needed bit
__global__ __launch_bounds__(kBlock) void nb_rest_kernel(NbLevel a) {
    __shared__ unsigned long long s_sum[kNbSums];
    const NbState st = a.st[a.level % kNbRing];
    if (st.done || !st.bum) return;
    NbSums sum;
    sum.zero();
    const int64_t words = (a.ne + 63) / 64;
    const int64_t fdef = a.level == 0 ? a.rows : a.ne;  // (nb_bu_kernel)
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / kWave);
    for (int64_t w = (int64_t)blockIdx.x * (blockDim.x / kWave) + wave_id(); w < words; w += nw) {
        unsigned long long word = a.rest[w];
        while (word) {
            const int b = __ffsll((unsigned long long)word) - 1;
            word &= word - 1;
            const int64_t v = w * 64 + b;
            const unsigned vis = a.vis[v];
            const unsigned need = ~vis & st.bum & 0xFFu;
            unsigned acc = a.Fn[v];
            const int64_t j0 = a.pull_rp[v], j1 = a.pull_rp[v + 1];
            int64_t j = j0 + a.first;
            while (j < j1 && acc != need) {
                int32_t u[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int64_t e = j + k * kWave + lane_id();
                    u[k] = a.pull_col[e < j1 ? e : j1 - 1];
                }
                unsigned f = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) f |= u[k] < fdef ? a.Fc[u[k]] : 0u;
#pragma unroll
                for (int o = kWave / 2; o > 0; o >>= 1) f |= (unsigned)__shfl_xor((int)f, o, kWave);
                acc |= f & need;
                const int64_t step = j1 - j < kNbStep ? j1 - j : kNbStep;
                if (lane_id() == 0) sum.ex += (unsigned long long)step;
                j += kNbStep;
            }
            if (lane_id() == 0) {
                a.Fn[v] = (uint8_t)acc;
                if (acc) {
                    a.vis[v] = (uint8_t)(vis | acc);
                    sum.add(acc, nb_push_deg(a, v, j0, j1));
                }
            }
        }
    }
    nb_flush(sum, a.ctr + a.level % kNbRing, a.tot, s_sum);
}

// The level's top-down queue when the previous level's does not fit (a source changed direction): every
// frontier row holding a top-down bit, with its push degree (wave-staged appends)
__global__ __launch_bounds__(kBlock) void nb_scan_kernel(NbLevel a) {
    __shared__ WaveStage s_app;
    const NbState st = a.st[a.level % kNbRing];
    if (st.done || !st.scan) return;
    WaveApp app{s_app};
    app.init();
    const int64_t lim = a.level == 0 ? a.rows : a.ne;
    unsigned long long* packed = &a.ctr[a.level % kNbRing].scanq;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = ((int64_t)blockIdx.x * blockDim.x) + wave_id() * kWave; base < lim; base += stride) {
        const int64_t v = base + lane_id();
        const bool take = v < lim && (a.Fc[v] & st.tdm) != 0;
        const long long d = take ? (long long)(a.push_rp[v + 1] - a.push_rp[v]) : 0;
        app.append(take, (int32_t)v, d, a.queue_in, a.qoff_in, packed);
    }
    app.final(a.queue_in, a.qoff_in, packed);
}

// Top-down: edge-parallel over the queue's push entries (entry e belongs to queue row i with
// qoff[i] <= e < qoff[i + 1]; the search runs over LDS samples first).  A target that lacks some of the
// row's top-down bits gets them by a 32-bit atomicOr on the word holding its byte (after plain reads of
// its visited and next bytes, so a target that has them takes no atomic); the first to set a top-down bit
// in a byte queues the row for the next level.
__global__ __launch_bounds__(kBlock) void nb_td_kernel(NbLevel a) {
    __shared__ WaveStage s_app;
    __shared__ int64_t s_qs[kNbSamples];
    __shared__ unsigned long long s_sum[kNbSums];
    const NbState st = a.st[a.level % kNbRing];
    if (st.done || !st.tdm) return;
    const unsigned long long h = st.scan ? a.ctr[a.level % kNbRing].scanq : a.ctr[(a.level + kNbRing - 1) % kNbRing].q;
    const int64_t nq = (int64_t)(h >> kPackShift), mf = (int64_t)(h & kEdgeMask);
    const unsigned tdm = st.tdm;
    WaveApp app{s_app};
    app.init();
    unsigned long long* packed = &a.ctr[a.level % kNbRing].q;
    NbSums sum;
    sum.zero();
    const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int ept = mf <= nthreads ? 1 : kNbEpt;
    const int64_t per_tile = nthreads * ept;
    const int64_t tiles = (mf + per_tile - 1) / per_tile;
    // samples of the queue's edge offsets
    const int64_t qstride = (nq + kNbSamples - 1) / kNbSamples > 0 ? (nq + kNbSamples - 1) / kNbSamples : 1;
    const int64_t qcount = (nq + qstride - 1) / qstride;
    if ((int64_t)blockIdx.x * blockDim.x * ept < mf)
        for (int64_t j = threadIdx.x; j < qcount; j += blockDim.x) s_qs[j] = a.qoff_in[j * qstride];
    __syncthreads();
    for (int64_t t = 0; t < tiles; ++t) {
        if ((t * nthreads + (int64_t)blockIdx.x * blockDim.x + wave_id() * kWave) * ept >= mf) break;
        const int64_t e0 = (t * nthreads + tid) * ept;
        int32_t v[kNbEpt];
        unsigned bits[kNbEpt];
#pragma unroll
        for (int k = 0; k < kNbEpt; ++k) v[k] = 0, bits[k] = 0;
        if (e0 < mf) {
            int64_t lo = 0, hi = qcount - 1;
            while (lo < hi) {
                const int64_t mid = (lo + hi + 1) >> 1;
                if (s_qs[mid] <= e0) lo = mid; else hi = mid - 1;
            }
            int64_t g0 = lo * qstride, g1 = (g0 + qstride < nq ? g0 + qstride : nq) - 1;
            while (g0 < g1) {
                const int64_t mid = (g0 + g1 + 1) >> 1;
                if (a.qoff_in[mid] <= e0) g0 = mid; else g1 = mid - 1;
            }
            int64_t i = g0;
            int64_t next_bound = i + 1 < nq ? a.qoff_in[i + 1] : mf;
#pragma unroll
            for (int k = 0; k < kNbEpt; ++k) {
                const int64_t e = e0 + k;
                if (k < ept && e < mf) {
                    while (e >= next_bound) {  // zero-degree queue rows too
                        ++i;
                        next_bound = i + 1 < nq ? a.qoff_in[i + 1] : mf;
                    }
                    const int32_t u = a.queue_in[i];
                    v[k] = a.push_col[a.push_rp[u] + (e - a.qoff_in[i])];
                    bits[k] = a.Fc[u] & tdm;
                    sum.ex += 1;
                }
            }
        }
        bool won[kNbEpt];
        long long dg[kNbEpt];
#pragma unroll
        for (int k = 0; k < kNbEpt; ++k) {
            won[k] = false;
            dg[k] = 0;
            if (bits[k]) {
                const unsigned g = bits[k] & ~(unsigned)a.vis[v[k]] & ~(unsigned)a.Fn[v[k]];
                if (g) {
                    const int sh = (v[k] & 3) * 8;
                    const unsigned old = atomicOr(reinterpret_cast<unsigned*>(a.Fn + (v[k] & ~3)), g << sh);
                    won[k] = ((old >> sh) & tdm) == 0;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < kNbEpt; ++k)
            if (won[k]) dg[k] = (long long)(a.push_rp[v[k] + 1] - a.push_rp[v[k]]);
        for (int k = 0; k < ept; ++k) app.append(won[k], v[k], dg[k], a.queue_out, a.qoff_out, packed);
    }
    app.final(a.queue_out, a.qoff_out, packed);
    nb_flush(sum, a.ctr + a.level % kNbRing, a.tot, s_sum);
}

// Top-down apply: every row the level queued (its first toucher) takes its new top-down bits into its
// visited bits and the level's counters
__global__ __launch_bounds__(kBlock) void nb_td_apply_kernel(NbLevel a) {
    __shared__ unsigned long long s_sum[kNbSums];
    const NbState st = a.st[a.level % kNbRing];
    if (st.done || !st.tdm) return;
    const unsigned long long h = a.ctr[a.level % kNbRing].q;
    const int64_t n = (int64_t)(h >> kPackShift), tot = (int64_t)(h & kEdgeMask);
    NbSums sum;
    sum.zero();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t v = a.queue_out[i];
        const unsigned w = a.Fn[v] & st.tdm;
        a.vis[v] = (uint8_t)(a.vis[v] | w);
        const int64_t o1 = i + 1 < n ? a.qoff_out[i + 1] : tot;
        sum.add(w, (long long)(o1 - a.qoff_out[i]));
    }
    // (sum.ex stays 0: the push counted its entries)
    nb_flush(sum, a.ctr + a.level % kNbRing, a.tot, s_sum);
}

// Level -1: F_0 and the visited bits of the sources, the first queue (distinct source rows) and its
// counters; one wave, lane s = source s
__global__ __launch_bounds__(kWave) void nb_init_kernel(const int64_t* __restrict__ src, int ns, const int64_t* push_rp,
                                                        uint8_t* F0, uint8_t* vis, int32_t* queue, int64_t* qoff,
                                                        NbCtr* ctr, NbState* st) {
    const int s = lane_id();
    const int64_t r = s < ns ? src[s] : -1;
    unsigned mine = 0;  // the sources on my row (the first lane of a row writes it)
    bool first = r >= 0;
    for (int t = 0; t < ns; ++t) {
        const int64_t rt = __shfl(r, t, kWave);
        if (rt == r && r >= 0) {
            mine |= 1u << t;
            if (t < s) first = false;
        }
    }
    const long long deg = r >= 0 ? (long long)(push_rp[r + 1] - push_rp[r]) : 0;
    if (first) {
        F0[r] = (uint8_t)mine;
        vis[r] = (uint8_t)mine;
    }
    const uint64_t m = __ballot(first);
    const long long dd = first ? deg : 0;
    const long long inc = wave_inclusive_scan_add(dd);
    const long long tot = __shfl(inc, kWave - 1, kWave);
    if (first) {
        const int pos = __popcll(m & lanemask_lt());
        queue[pos] = (int32_t)r;
        qoff[pos] = inc - dd;
    }
    NbCtr* c = ctr + kNbRing - 1;
    if (s < kNarrowMax) {
        c->nf[s] = r >= 0 ? 1ull : 0ull;
        c->mf[s] = r >= 0 ? (unsigned long long)deg : 0ull;
    }
    if (s == 0) {
        c->q = ((unsigned long long)__popcll(m) << kPackShift) | (unsigned long long)tot;
        NbState z{};
        z.qmask = ns >= 32 ? ~0u : ((1u << ns) - 1u);
        *(st + kNbRing - 1) = z;
    }
}

// Depths: plane s of row v = the level whose frontier array holds bit s (-1 unreached); levels >= 1 hold
// rows [0, ne) only
__global__ void nb_planes_kernel(const uint8_t* const* __restrict__ F, int levels, int64_t rows, int64_t ne, int ns,
                                 int32_t* __restrict__ planes) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < rows; v += (int64_t)gridDim.x * blockDim.x) {
        int32_t d[kNarrowMax];
#pragma unroll
        for (int s = 0; s < kNarrowMax; ++s) d[s] = -1;
        for (int L = 0; L < levels; ++L) {
            if (L > 0 && v >= ne) break;
            const unsigned w = F[L][v];
#pragma unroll
            for (int s = 0; s < kNarrowMax; ++s)
                if ((w >> s) & 1u) d[s] = L;
        }
        for (int s = 0; s < ns; ++s) planes[(int64_t)s * rows + v] = d[s];
    }
}

}  // namespace

NarrowRun narrow_bfs(Ctx& ctx, Shard& sh, const Csr& push, const Csr& pull, const int64_t* src, int ns, int max_depth,
                     int32_t* planes) {
    if (ns < 1 || ns > kNarrowMax) fail(JG_ERR_ARG, "narrow BFS takes 1..8 sources");
    hipStream_t s = sh.stream;
    const int64_t rows = sh.rows;
    const int64_t ne = pull.empty_from >= 0 ? std::min(pull.empty_from, rows) : rows;
    const size_t r1 = (size_t)std::max<int64_t>(rows, 1);
    const size_t lvl_bytes = ((size_t)rows + 64) / 64 * 64;  // the top-down atomics touch 4-byte words
    // scratch before the timed region (kept with the shard)
    if (sh.nb_vis.size() != r1) sh.nb_vis.alloc(r1);
    if (sh.nb_rest.size() != (size_t)std::max<int64_t>((ne + 63) / 64, 1)) sh.nb_rest.alloc(std::max<int64_t>((ne + 63) / 64, 1));
    for (int k = 0; k < 2; ++k) {
        if (sh.nb_queue[k].size() != r1) sh.nb_queue[k].alloc(r1);
        if (sh.nb_qoff[k].size() != r1) sh.nb_qoff[k].alloc(r1);
    }
    const size_t ctr_words = (size_t)kNbRing * kNbCtrWords + 2;  // + the traversal's totals
    if (sh.nb_ctr.size() != ctr_words) sh.nb_ctr.alloc(ctr_words);
    if (sh.nb_state.size() != kNbRing * sizeof(NbState)) sh.nb_state.alloc(kNbRing * sizeof(NbState));
    auto ensure_levels = [&](int n) {
        for (auto& b : sh.nb_level)
            if (b.size() != lvl_bytes) b.alloc(lvl_bytes);
        while ((int)sh.nb_level.size() < n) {
            sh.nb_level.emplace_back();
            sh.nb_level.back().alloc(lvl_bytes);
        }
    };
    ensure_levels(16);
    DevBuf<int64_t> dsrc(ns);
    copy_h2d(dsrc.get(), src, (size_t)ns * sizeof(int64_t), s);
    NbCtr* ctr = reinterpret_cast<NbCtr*>(sh.nb_ctr.get());
    NbState* st = reinterpret_cast<NbState*>(sh.nb_state.get());

    hipEvent_t t0, t1;
    JG_HIP(hipEventCreate(&t0));
    JG_HIP(hipEventCreate(&t1));
    JG_HIP(hipEventRecord(t0, s));
    if (prof_enabled(ctx)) prof_record_start(ctx, sh);
    JG_HIP(hipMemsetAsync(sh.nb_vis.get(), 0, (size_t)rows, s));
    JG_HIP(hipMemsetAsync(sh.nb_level[0].get(), 0, (size_t)rows, s));
    JG_HIP(hipMemsetAsync(sh.nb_ctr.get(), 0, sh.nb_ctr.bytes(), s));
    nb_init_kernel<<<1, kWave, 0, s>>>(dsrc.get(), ns, push.row_ptr.get(), sh.nb_level[0].get(), sh.nb_vis.get(),
                                      sh.nb_queue[0].get(), sh.nb_qoff[0].get(), ctr, st);
    JG_LAUNCH_CHECK();

    NbLevel a{};
    a.push_rp = push.row_ptr.get();
    a.push_col = push.col.get();
    a.pull_rp = pull.row_ptr.get();
    a.pull_col = pull.col.get();
    a.pull_first = bfs_first_col(sh, pull);
    a.vis = sh.nb_vis.get();
    a.rest = sh.nb_rest.get();
    a.ctr = ctr;
    a.st = st;
    a.tot = sh.nb_ctr.get() + (size_t)kNbRing * kNbCtrWords;
    a.rows = rows;
    a.ne = ne;
    a.push_nnz = push.nnz;
    a.max_depth = max_depth;
    a.ns = ns;
    a.first = std::max(4, tune().nb_first);
    a.alpha = (double)tune().nb_alpha;
    a.beta = (double)tune().bfs_beta;
    // grids: rows passes at most 4096 workgroups (grid-stride); the push ~sqrt(rows) like the DO-BFS
    const unsigned rgrid = grid_for(std::max<int64_t>(ne, 1), kBlock, 4096);
    const int64_t sq = 1ll << ((bits_for((uint64_t)std::max<int64_t>(rows - 1, 1)) + 1) / 2);
    const unsigned tgrid = (unsigned)std::min<int64_t>(std::max<int64_t>(sq, 64), tune().bfs_grid);
    const unsigned bgrid = (unsigned)std::min<int64_t>(std::max<int64_t>((ne + 63) / 64 / 16, 1), 2048);
    const unsigned agrid = 1024;
    int level = 0;
    NbState hs{};
    int next_batch = 4;
    for (int batch = std::max(1, tune().bfs_batch0);; batch = next_batch, next_batch = std::min(next_batch * 2, 64)) {
        if (max_depth >= 0) batch = std::min(batch, max_depth + 1 - level);
        if (batch <= 0) fail(JG_ERR_STATE, "narrow BFS level control did not terminate");
        ensure_levels(level + batch + 1);
        for (int k = 0; k < batch; ++k, ++level) {
            a.level = level;
            a.Fc = sh.nb_level[(size_t)level].get();
            a.Fn = sh.nb_level[(size_t)level + 1].get();
            a.queue_in = sh.nb_queue[level & 1].get();
            a.qoff_in = sh.nb_qoff[level & 1].get();
            a.queue_out = sh.nb_queue[(level + 1) & 1].get();
            a.qoff_out = sh.nb_qoff[(level + 1) & 1].get();
            nb_bu_kernel<<<rgrid, kBlock, 0, s>>>(a);
            nb_rest_kernel<<<bgrid, kBlock, 0, s>>>(a);
            nb_scan_kernel<<<rgrid, kBlock, 0, s>>>(a);
            nb_td_kernel<<<tgrid, kBlock, 0, s>>>(a);
            nb_td_apply_kernel<<<agrid, kBlock, 0, s>>>(a);
            JG_LAUNCH_CHECK();
            if (debug_bfs()) {
                NbState ds{};
                NbCtr dc{};
                copy_d2h(&ds, st + level % kNbRing, sizeof ds, s);
                copy_d2h(&dc, ctr + level % kNbRing, sizeof dc, s);
                unsigned long long nf = 0;
                for (int q = 0; q < ns; ++q) nf += dc.nf[q];
                std::fprintf(stderr, "[jg narrow] level %d done %d td %02x bu %02x scan %d: new pairs %llu, examined %llu\n",
                             level, ds.done, ds.tdm, ds.bum, ds.scan, nf, dc.examined);
            }
        }
        copy_d2h(&hs, st + (level - 1) % kNbRing, sizeof hs, s);
        if (hs.done) break;
    }
    if (prof_enabled(ctx)) prof_record_stop(ctx, sh);
    JG_HIP(hipEventRecord(t1, s));
    JG_HIP(hipEventSynchronize(t1));
    NarrowRun out;
    JG_HIP(hipEventElapsedTime(&out.ms, t0, t1));
    JG_HIP(hipEventDestroy(t0));
    JG_HIP(hipEventDestroy(t1));
    out.levels = hs.levels;
    // work: the examined entries of every level and the reached (source, row) pairs; the sources'
    // own pairs (level 0) are not counted by the kernels
    unsigned long long tot[2] = {0, 0};
    copy_d2h(tot, a.tot, sizeof tot, s);
    out.entries = (double)tot[0];
    out.reached = (double)tot[1];
    // 5 B per examined entry (4-byte column + the 1-byte frontier gather), and per level 2 B per row with
    // entries (visited byte read, next frontier byte written)
    out.bytes = 5.0 * out.entries + 2.0 * (double)ne * (double)(out.levels + 1);
    if (planes) {
        std::vector<const uint8_t*> tab((size_t)out.levels + 1);
        for (int L = 0; L <= out.levels; ++L) tab[(size_t)L] = sh.nb_level[(size_t)L].get();
        if (sh.nb_table.size() < tab.size()) sh.nb_table.alloc(tab.size());
        copy_h2d(sh.nb_table.get(), tab.data(), tab.size() * sizeof(const uint8_t*), s);
        nb_planes_kernel<<<grid_for(rows), kBlock, 0, s>>>(sh.nb_table.get(), out.levels + 1, rows, ne, ns, planes);
        JG_LAUNCH_CHECK();
        JG_HIP(hipStreamSynchronize(s));
    }
    return out;
}

}  // namespace jg
