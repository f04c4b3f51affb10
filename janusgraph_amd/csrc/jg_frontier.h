// jg_frontier.h — frontier queues shared by the traversals (jg_traverse.hip) and CC (jg_cc.hip).
#pragma once

#include "jg_prim.h"

namespace jg {

constexpr int kPackShift = 37;  // packed frontier counter: (vertices << 37) | push edges
constexpr unsigned long long kEdgeMask = (1ull << kPackShift) - 1ull;

// Counters reduced by many workgroups (MS-BFS live bits, frontier counters, live-task and pair counts,
// CC's linked entries and giant-component minima): one device atomic per 1024-thread workgroup on a
// grid of at most kRedBlocks (two per CU: 32 waves).  A device-scope atomic on one word executes at
// the memory side, ~88 per us (MI355X_MICROARCH.md, dequeue row); one per wave on a 4096-block grid
// queued 16 K of them, ~0.2 ms, behind kernels of ~20-60 us of work (msbfs_task_live_kernel,
// msbfs_pairs_kernel in the round-3 8-shard trace).
constexpr int kRedThreads = 1024, kRedWaves = kRedThreads / kWave;
constexpr int64_t kRedBlocks = 512;
inline unsigned red_grid(int64_t work) { return grid_for(work, kRedThreads, kRedBlocks); }

// v reduced over the block (every thread calls; `red` holds blockDim.x / kWave elements); valid in thread 0
template <class T, class F>
__device__ __forceinline__ T block_reduce(T v, F op, T* red) {
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) v = op(v, (T)__shfl_xor(v, o, kWave));
    if (lane_id() == 0) red[wave_id()] = v;
    __syncthreads();
    if (threadIdx.x == 0)
        for (int w = 1; w < (int)(blockDim.x / kWave); ++w) v = op(v, red[w]);
    return v;
}
struct OrU64 {
    __device__ unsigned long long operator()(unsigned long long a, unsigned long long b) const { return a | b; }
};
struct AddU64 {
    __device__ unsigned long long operator()(unsigned long long a, unsigned long long b) const { return a + b; }
};
struct MinI32 {
    __device__ int32_t operator()(int32_t a, int32_t b) const { return a < b ? a : b; }
};

// Wave-staged frontier append: every wave collects its appends in its own LDS region and keeps its
// count in registers, so appending needs no block barrier and the waves of a block run their loops
// independently (a block-wide append made every wave wait, every iteration, for the block's slowest
// lane scan).  Global queue space is still reserved with one atomic per block at the end
// (wave_stage_final, block-uniform); a wave whose region fills up reserves for itself.
struct WaveStage {
    static constexpr int kCap = 512;  // entries per wave
    int32_t v[kBlock / kWave][kCap];
    int64_t off[kBlock / kWave][kCap];  // edge offset inside the wave's staged run
    unsigned long long cnt[kBlock / kWave], dsum[kBlock / kWave];
    unsigned long long base;
};
struct WaveRun {  // a wave's staged run (wave-uniform registers)
    unsigned long long n = 0, ds = 0;
};
__device__ __forceinline__ void wave_stage_flush(WaveStage& sa, WaveRun& run, int32_t* __restrict__ queue,
                                                 int64_t* __restrict__ qoff, unsigned long long* __restrict__ packed) {
    if (run.n == 0) return;
    const int wv = wave_id();
    unsigned long long base = 0;
    if (lane_id() == 0) base = atomicAdd(packed, (run.n << kPackShift) | run.ds);
    base = __shfl(base, 0, kWave);
    const unsigned long long qb = base >> kPackShift, eb = base & kEdgeMask;
    for (unsigned long long i = lane_id(); i < run.n; i += kWave) {
        queue[qb + i] = sa.v[wv][i];
        qoff[qb + i] = (int64_t)eb + sa.off[wv][i];
    }
    run.n = run.ds = 0;
}
// Wave-uniform call: lanes with `take` append v (push degree deg).
__device__ __forceinline__ void wave_stage_append(bool take, int32_t v, int64_t deg, WaveStage& sa, WaveRun& run,
                                                  int32_t* __restrict__ queue, int64_t* __restrict__ qoff,
                                                  unsigned long long* __restrict__ packed) {
    const uint64_t mask = __ballot(take);
    if (mask == 0) return;
    const int64_t d = take ? deg : 0;
    const int64_t dinc = wave_inclusive_scan_add(d);
    const int64_t tot = __shfl(dinc, kWave - 1, kWave);
    const int wv = wave_id();
    if (take) {
        const unsigned long long p = run.n + (unsigned long long)__popcll(mask & lanemask_lt());
        sa.v[wv][p] = v;
        sa.off[wv][p] = (int64_t)run.ds + dinc - d;
    }
    run.n += (unsigned long long)__popcll(mask);
    run.ds += (unsigned long long)tot;
    if (run.n > (unsigned long long)(WaveStage::kCap - kWave)) wave_stage_flush(sa, run, queue, qoff, packed);
}
// Block-uniform: the block's remaining runs reserve their space with one atomic and are written out.
__device__ __forceinline__ void wave_stage_final(WaveStage& sa, WaveRun& run, int32_t* __restrict__ queue,
                                                 int64_t* __restrict__ qoff, unsigned long long* __restrict__ packed) {
    const int wv = wave_id();
    if (lane_id() == 0) {
        sa.cnt[wv] = run.n;
        sa.dsum[wv] = run.ds;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long c = 0, e = 0;
        for (int k = 0; k < kBlock / kWave; ++k) {
            const unsigned long long ck = sa.cnt[k], ek = sa.dsum[k];
            sa.cnt[k] = c;  // exclusive prefixes
            sa.dsum[k] = e;
            c += ck;
            e += ek;
        }
        sa.base = c ? atomicAdd(packed, (c << kPackShift) | e) : 0ull;
    }
    __syncthreads();
    const unsigned long long qb = (sa.base >> kPackShift) + sa.cnt[wv], eb = (sa.base & kEdgeMask) + sa.dsum[wv];
    for (unsigned long long i = lane_id(); i < run.n; i += kWave) {
        queue[qb + i] = sa.v[wv][i];
        qoff[qb + i] = (int64_t)eb + sa.off[wv][i];
    }
    run.n = run.ds = 0;
}

// The wave-staged appender behind the interface the traversal kernels use (init / append / final).
// (A block-wide staged append, one LDS flush per block, made every wave wait each step for the block's
// slowest lane scan: RMAT-20 DO-BFS 0.145-0.157 -> 0.119-0.129 ms with per-wave runs, round 2.)
struct WaveApp {
    static constexpr bool kWaveUniform = true;
    WaveStage& sa;
    WaveRun run;
    __device__ void init() {}
    __device__ void append(bool take, int32_t v, int64_t deg, int32_t* q, int64_t* qo, unsigned long long* packed) {
        wave_stage_append(take, v, deg, sa, run, q, qo, packed);
    }
    __device__ void final(int32_t* q, int64_t* qo, unsigned long long* packed) { wave_stage_final(sa, run, q, qo, packed); }
};

}  // namespace jg
