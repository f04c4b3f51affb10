// jg_frontier.h — frontier queues shared by the traversals (jg_traverse.hip) and CC (jg_cc.hip).
#pragma once

#include "jg_prim.h"

namespace jg {

constexpr int kPackShift = 37;  // packed frontier counter: (vertices << 37) | push edges
constexpr unsigned long long kEdgeMask = (1ull << kPackShift) - 1ull;

// Block-aggregated frontier append: the block's waves combine their counts in LDS and
// one thread reserves the block's range with a single atomic (a level that finds most of the graph
// would otherwise put one atomic per wave on one address).  Must be reached by every thread of the
// block (block-uniform call sites); queue positions and edge offsets stay monotone.
struct AppendScratch {
    unsigned long long cnt[kBlock / kWave], deg[kBlock / kWave];
    unsigned long long base;
};
__device__ __forceinline__ void block_append_frontier(bool take, int32_t v, int64_t deg, int32_t* __restrict__ queue,
                                                      int64_t* __restrict__ qoff, unsigned long long* __restrict__ packed,
                                                      AppendScratch& sc) {
    const uint64_t mask = __ballot(take);
    const int64_t d = take ? deg : 0;
    const int64_t dinc = wave_inclusive_scan_add(d);
    const int wv = wave_id();
    if (lane_id() == kWave - 1) {
        sc.cnt[wv] = (unsigned long long)__popcll(mask);
        sc.deg[wv] = (unsigned long long)dinc;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long c = 0, e = 0;
        for (int k = 0; k < kBlock / kWave; ++k) {
            const unsigned long long ck = sc.cnt[k], ek = sc.deg[k];
            sc.cnt[k] = c;  // exclusive prefixes
            sc.deg[k] = e;
            c += ck;
            e += ek;
        }
        sc.base = c ? atomicAdd(packed, (c << kPackShift) | e) : 0ull;
    }
    __syncthreads();
    if (take) {
        const unsigned long long base = sc.base;
        const uint64_t pos = (base >> kPackShift) + sc.cnt[wv] + (uint64_t)__popcll(mask & lanemask_lt());
        queue[pos] = v;
        qoff[pos] = (int64_t)(base & kEdgeMask) + (int64_t)sc.deg[wv] + dinc - d;
    }
    __syncthreads();  // the scratch is reused by the next call
}

}  // namespace jg
