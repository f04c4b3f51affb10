// jg_pull.h — the pull superstep engine: one launch streams a CSR's col[] once and folds the
// gathered source values per row.  This is Fulgora's message gather
// (graphdb/olap/computer/VertexMemoryHandler.java:121-151: for each reverse-incident edge, read the
// neighbour's previous-superstep message) as a segmented reduction.
//
// Work decomposition (rows are degree-sorted, PullPlan classes are contiguous row ranges):
//   class 0  hub rows (degree >= kHubDegree): one workgroup per kHubChunk entries, partial folds
//            written to hub_partial[], combined in chunk order by pull_hub_finalize_kernel
//   class c  (c = 1..7) L = 64 >> (c-1) lanes per row, 256/L rows per workgroup; lanes stride the
//            row, fold, then a width-L xor-shuffle tree; lane 0 finalises the row
//   class 8  the suffix of rows without entries: finalised with the identity, row_ptr not read
// Every row is folded in a fixed order that does not depend on timing (bit-reproducible runs).
// An Op supplies: T, identity(), combine(a,b), gather(col), vec(), shfl_xor(v,o),
// shfl_up(v,d), active(row) (false: the row is not folded but still finalised with identity()),
// finalize(row, acc).
#pragma once

#include "jg_internal.h"
#include "jg_prim.h"

namespace jg {

struct PullArgs {
    const int64_t* __restrict__ row_ptr;
    const int32_t* __restrict__ col;
    const int64_t* __restrict__ chunk_row;
    const int64_t* __restrict__ chunk_begin;
    const int64_t* __restrict__ chunk_end;
    const int64_t* __restrict__ hub_chunk_ptr;
    int64_t num_chunks;
    int64_t num_hub_rows;
    int64_t class_row_begin[kNumClasses];
    int64_t class_row_end[kNumClasses];
    int64_t class_block_begin[kNumClasses + 1];
    int64_t block_offset;  // diagnostic split launches (JG_PULL_SPLIT=1): first block of this launch
    int64_t skip_rows;     // rows [0, skip_rows) are folded by the XCD split: their hub chunks are skipped
    int runs;              // 1-lane rows from run_begin[kRunMax] on are addressed by degree run (PullPlan::runs)
    int64_t run_begin[kRunMax + 1];
    int64_t run_ptr[kRunMax + 1];
};

inline PullArgs make_pull_args(const Csr& csr, const PullPlan& p, bool light = false) {
    PullArgs a;
    a.row_ptr = csr.row_ptr.get();
    a.col = csr.col.get();
    a.chunk_row = p.chunk_row.get();
    a.chunk_begin = p.chunk_begin.get();
    a.chunk_end = p.chunk_end.get();
    a.hub_chunk_ptr = p.hub_chunk_ptr.get();
    a.num_chunks = p.num_chunks;
    a.num_hub_rows = p.num_hub_rows;
    for (int c = 0; c < kNumClasses; ++c) {
        a.class_row_begin[c] = light ? p.light_row_begin[c] : p.class_row_begin[c];
        a.class_row_end[c] = light ? p.light_row_end[c] : p.class_row_end[c];
    }
    for (int c = 0; c <= kNumClasses; ++c) a.class_block_begin[c] = light ? p.light_block_begin[c] : p.class_block_begin[c];
    a.block_offset = 0;
    a.skip_rows = light ? p.split_rows : 0;
    a.runs = p.runs;
    for (int d = 0; d <= kRunMax; ++d) {
        a.run_begin[d] = p.run_begin[d];
        a.run_ptr[d] = p.run_ptr[d];
    }
    return a;
}

// How a fold reads the gathered vector (the class rows: straight from global memory).
template <class Op>
struct GlobalGather {
    const Op& op;
    __device__ __forceinline__ typename Op::T operator()(int32_t c) const { return op.gather(c); }
};
// LDS pointers keep address space 3: through a generic pointer the compiler emits flat loads, which
// go through the TA/TD like global loads and defeat the point of staging.
template <class T>
using lds_ptr = __attribute__((address_space(3))) T*;

// Fold col[j..j1) with stride `stride`; U gathers in flight per lane, folded in index order.
// Software-pipelined: the col batch of iteration i+1 is loaded while the gathers of iteration i are
// in flight, so a long row pays one round trip per batch instead of two.  The last, partial batch is
// not walked one entry at a time: its out-of-range slots re-read the row's last entry (a cache hit)
// and are dropped from the fold by a select, so every batch is branch-free.
template <class Op, int U>
__device__ __forceinline__ void load_cols(const int32_t* __restrict__ col, int64_t j, int64_t j1, int stride,
                                          int32_t (&c)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t k = j + u * (int64_t)stride;
        c[u] = col[k < j1 ? k : j1 - 1];
    }
}

template <class Op, int U, class G>
__device__ __forceinline__ typename Op::T fold_strided(const Op& op, const G& gather, const int32_t* __restrict__ col,
                                                       int64_t j, int64_t j1, int stride) {
    using T = typename Op::T;
    T acc = op.identity();
    if (j >= j1) return acc;
    int32_t c[U];
    load_cols<Op, U>(col, j, j1, stride, c);
    for (;;) {
        T v[U];
        const int64_t jn = j + U * (int64_t)stride;
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = gather(c[u]);
        load_cols<Op, U>(col, jn, j1, stride, c);  // clamped: unconditional keeps vmcnt counting exact
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const T t = op.combine(acc, v[u]);
            acc = (j + u * (int64_t)stride < j1) ? t : acc;
        }
        j = jn;
        if (j >= j1) break;
    }
    return acc;
}

// Short rows (one lane per row, < 8 entries): all entries in one masked batch of 8.  Out-of-range
// slots issue no load at all (exec-masked), instead of re-reading the last entry: a duplicate lane
// still costs the TA/TD its cycles (tools/micro/td_mask.hip: cost scales with active lanes).
template <class Op, class G>
__device__ __forceinline__ typename Op::T fold_short(const Op& op, const G& gather, const int32_t* __restrict__ col,
                                                     int64_t j, int64_t j1) {
    using T = typename Op::T;
    constexpr int kMax = 8;
    const int n = (int)(j1 - j);
    int32_t c[kMax];
#pragma unroll
    for (int u = 0; u < kMax; ++u) {
        c[u] = 0;
        if (u < n) c[u] = col[j + u];
    }
    T v[kMax];
#pragma unroll
    for (int u = 0; u < kMax; ++u) {
        v[u] = op.identity();
        if (u < n) v[u] = gather(c[u]);
    }
    T acc = op.identity();
#pragma unroll
    for (int u = 0; u < kMax; ++u)
        if (u < n) acc = op.combine(acc, v[u]);
    return acc;
}

template <class Op, int U>
__device__ __forceinline__ typename Op::T fold_strided(const Op& op, const int32_t* __restrict__ col, int64_t j,
                                                       int64_t j1, int stride) {
    return fold_strided<Op, U>(op, GlobalGather<Op>{op}, col, j, j1, stride);
}

// `tid` is the thread's index inside its (virtual) 256-thread block.
template <class Op, int L, int U, class G>
__device__ __forceinline__ void pull_rows_class(const PullArgs& a, const Op& op, const G& gather, int c,
                                                int64_t local_block, int tid) {
    using T = typename Op::T;
    constexpr int kRowsPerBlock = kBlock / L;
    const int sub = tid % L;
    const int64_t row = a.class_row_begin[c] + local_block * kRowsPerBlock + tid / L;
    const bool valid = row < a.class_row_end[c];
    T acc = op.identity();
    bool hub = false;
    if (L == 1 && valid && a.runs && row >= a.run_begin[kRunMax]) {
        // degree run: rows of degree d are consecutive, so the entries follow from the row number
        int64_t d = kRunMax, j0 = a.run_ptr[kRunMax] + (row - a.run_begin[kRunMax]) * kRunMax;
#pragma unroll
        for (int k = kRunMax - 1; k >= 1; --k)
            if (row >= a.run_begin[k]) {
                d = k;
                j0 = a.run_ptr[k] + (row - a.run_begin[k]) * k;
            }
        if (op.active(row)) acc = fold_short<Op>(op, gather, a.col, j0, j0 + d);
        op.finalize(row, acc);
        return;
    }
    if (valid) {
        const int64_t j0 = a.row_ptr[row], j1 = a.row_ptr[row + 1];
        hub = (j1 - j0) >= kHubDegree;  // folded by the chunk path
        if (!hub && op.active(row)) {
            if (L == 1 && j1 - j0 <= 8) acc = fold_short<Op>(op, gather, a.col, j0, j1);
            else acc = fold_strided<Op, U>(op, gather, a.col, j0 + sub, j1, L);
        }
    }
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) acc = op.combine(acc, op.shfl_xor(acc, o));
    if (valid && !hub && sub == 0) op.finalize(row, acc);
}

// Rows known to have no entries (the degree-sorted suffix): finalise with the identity, no row_ptr.
template <class Op>
__device__ __forceinline__ void pull_rows_empty(const PullArgs& a, const Op& op, int64_t local_block, int tid) {
    const int64_t row = a.class_row_begin[kZeroClass] + local_block * kBlock + tid;
    if (row < a.class_row_end[kZeroClass]) op.finalize(row, op.identity());
}

// Class dispatch of (virtual) block b >= num_chunks.
template <class Op, int U, class G>
__device__ __forceinline__ void pull_block_rows(const PullArgs& a, const Op& op, const G& gather, int64_t b, int tid) {
    int c = 1;
#pragma unroll
    for (int k = 1; k < kNumClasses; ++k)
        if (b >= a.class_block_begin[k + 1]) c = k + 1;
    const int64_t lb = b - a.class_block_begin[c];
    switch (c) {
        case 1: pull_rows_class<Op, 64, U>(a, op, gather, c, lb, tid); break;
        case 2: pull_rows_class<Op, 32, U>(a, op, gather, c, lb, tid); break;
        case 3: pull_rows_class<Op, 16, U>(a, op, gather, c, lb, tid); break;
        case 4: pull_rows_class<Op, 8, U>(a, op, gather, c, lb, tid); break;
        case 5: pull_rows_class<Op, 4, U>(a, op, gather, c, lb, tid); break;
        case 6: pull_rows_class<Op, 2, U>(a, op, gather, c, lb, tid); break;
        case 7: pull_rows_class<Op, 1, U>(a, op, gather, c, lb, tid); break;
        default: pull_rows_empty<Op>(a, op, lb, tid); break;
    }
}

template <class Op, int U>
__device__ __forceinline__ void pull_block(const PullArgs& a, const Op& op, typename Op::T* __restrict__ hub_partial,
                                           int64_t b) {
    using T = typename Op::T;
    if (b < a.num_chunks) {
        __shared__ T red[kBlock / kWave];
        const int64_t j0 = a.chunk_begin[b], j1 = a.chunk_end[b];
        const int64_t crow = a.chunk_row[b];
        T acc = (crow >= a.skip_rows && op.active(crow)) ? fold_strided<Op, U>(op, a.col, j0 + threadIdx.x, j1, kBlock)
                                                         : op.identity();
#pragma unroll
        for (int o = kWave / 2; o > 0; o >>= 1) acc = op.combine(acc, op.shfl_xor(acc, o));
        if (lane_id() == 0) red[wave_id()] = acc;
        __syncthreads();
        if (threadIdx.x == 0) {
            T t = red[0];
#pragma unroll
            for (int w = 1; w < kBlock / kWave; ++w) t = op.combine(t, red[w]);
            hub_partial[b] = t;
        }
        return;
    }
    pull_block_rows<Op, U>(a, op, GlobalGather<Op>{op}, b, (int)threadIdx.x);
}

template <class Op, int U>
__global__ __launch_bounds__(kBlock) void pull_kernel(PullArgs a, Op op, typename Op::T* __restrict__ hub_partial) {
    pull_block<Op, U>(a, op, hub_partial, (int64_t)blockIdx.x + a.block_offset);
}

template <class Op>
__global__ void pull_hub_finalize_kernel(PullArgs a, Op op, const typename Op::T* __restrict__ hub_partial) {
    using T = typename Op::T;
    for (int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; h < a.num_hub_rows;
         h += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c0 = a.hub_chunk_ptr[h], c1 = a.hub_chunk_ptr[h + 1];
        if (a.chunk_row[c0] < a.skip_rows) continue;  // finalised by the XCD split
        T acc = op.identity();
        for (int64_t k = c0; k < c1; ++k) acc = op.combine(acc, hub_partial[k]);
        op.finalize(a.chunk_row[c0], acc);
    }
}

// ---------------- XCD-sliced split of the heavy rows (PullPlan::bands) ----------------
// A band's entries are kept sub-slice-major: sub-slice h (2^bits of them, sub_slice(): each aligned
// group of 2^bits lines of the gathered vector gives one line to every sub-slice) is a sub-CSR over
// the band's rows.  Each sub-slice is folded merge-path style (CSR-stream): a wave task is kMergeTask
// consecutive entries of one sub-slice, kMergeEpl per lane, whatever the row boundaries, so col loads
// are whole 2 KiB spans and no lane idles on short rows.  Workgroup b runs sub-slice
// h = (b mod 8) | ((b / 8) mod 2^bits/8) << 3, so h's workgroups share the dispatcher's XCD b mod 8
// (speed only: any placement gives the same result) and an XCD's L2 only ever holds its eighth of
// the vector.  On one shard every workgroup also stages the hottest lines of its sub-slice in LDS:
// with 2^bits sub-slices the CUs of one XCD hold different images, so the LDS-resident share of the
// vector grows with bits.  The superstep is bound by TCP->L2 requests in flight (PMC: TA/TD ~90%
// busy, TCP pending-stalled), so every gather served from LDS is one request fewer.
// Row boundaries come from build-time task metadata, so a task's only dependent loads are its
// gathers: heads[t][l] holds the row-start bits of lane l's entries (entry 0 of a task is always a
// head), meta[t] = (j0, carry): head h of the task is non-empty sub-row j0 + h, and with carry = 1
// head 0 continues sub-row j0 from the previous task.  Sums are a deterministic segmented reduction:
// sequential inside a lane, a fixed Hillis-Steele segmented scan across lanes.  A segment that starts
// in the task goes to partial[j]; a continuation goes to carry[t], and pull_merge_fixup_kernel adds a
// sub-row's carries in task order.  pull_slice_finalize_kernel folds every row's sub-slices in order.
constexpr int kMergeThreads = 1024;                    // one workgroup per CU
constexpr int kMergeWaves = kMergeThreads / kWave;
constexpr int kMergeEpl = kMergeTask / kWave;          // entries per lane
constexpr int kMergeLdsBytes = 160 * 1024;

struct MergeArgs {
    const uint4* __restrict__ pack_a;       // band entries, packed (SliceBand::pack_a/_b)
    const uint32_t* __restrict__ pack_b;
    const uint8_t* __restrict__ heads;      // [tasks][64]
    const int32_t* __restrict__ meta;       // [tasks][2]
    const int64_t* __restrict__ sub_begin;  // [S]
    const int64_t* __restrict__ sub_end;    // [S]
    const int64_t* __restrict__ sub_base;   // [S+1]
    int64_t tasks;
    int bits;
    int stage;         // LDS staging slots per wave for a task's partials (0: direct stores)
    // nullable: bit t (of the band's tasks) clear = task t is skipped, its partials and carry left as
    // they are.  A program passes it only when every row the task touches would discard what the task
    // folds (the multi-source BFS: rows that can gain no bit; see msbfs_task_live_kernel).
    const uint32_t* __restrict__ live;
};

// The hot entries of a gathered vector: the first `hs` entries of each of its `nseg` segments
// (stride 2^tbits; one segment of stride 2^31 on a single shard, a shard's own rows + one per peer
// on a sharded compact vector).
struct HotSegs {
    int32_t hs = 0;
    int tbits = 31;
    int nseg = 1;
};

// Gathers of sub-slice h of a 2^bits band from the entries' sub-slice-local indices
// (SliceBand::pack_a/_b): loc = g << 4 | lane16, g = the line group (c >> (4 + bits)).  Hot ids come
// from the LDS image of the sub-slice's lines in the hot entries (segment s = g >> (tbits - gshift),
// its group j = the rest; hot when j < hg, at LDS line s * hg + j), the rest from global memory at
// the column restored from loc: line = g << bits | (h ^ the hash bits of the group's first line).
template <class Op>
struct SliceGather {
    using T = typename Op::T;
    const Op& op;
    lds_ptr<const T> lds;
    uint32_t hg;        // hot line groups per segment
    int sb;             // tbits - gshift: group bits inside a segment
    int bits;
    uint32_t hmask, h;  // 2^bits - 1, the sub-slice
    uint32_t idcell;    // the identity cell just past the staged lines
    __device__ __forceinline__ bool is_hot(uint32_t loc) const { return ((loc >> 4) & ((1u << sb) - 1u)) < hg; }
    // Cold and invalid lanes read the identity cell: no select, so the read cannot become a branch.
    __device__ __forceinline__ T hot(uint32_t loc, bool valid) const {
        const uint32_t g = loc >> 4, j = g & ((1u << sb) - 1u), seg = g >> sb;
        return lds[valid && j < hg ? (((seg * hg + j) << 4) | (loc & 15u)) : idcell];
    }
    __device__ __forceinline__ int32_t col(uint32_t loc) const {
        const uint32_t x = (loc >> 4) << bits;  // the group's first line
        const uint32_t hx = (x ^ (x >> 8) ^ (x >> 16) ^ (x >> 24)) & hmask;
        return (int32_t)(((x | (h ^ hx)) << 4) | (loc & 15u));
    }
    // Only valid cold lanes load (exec-masked); the others keep identity().
    __device__ __forceinline__ T cold(uint32_t loc, bool valid, bool lds_on) const {
        T v = op.identity();
        if (valid && !(lds_on && is_hot(loc))) v = op.gather(col(loc));
        return v;
    }
};

// Entry u of a lane chunk packed in W bits (bit stream over the chunk's dwords).
template <int W>
__device__ __forceinline__ uint32_t unpack_entry(const uint32_t (&d)[W / 4], int u) {
    const int o = W * u, i = o >> 5, sh = o & 31;
    uint32_t v = d[i] >> sh;
    if (sh + W > 32) v |= d[i + 1] << (32 - sh);
    if constexpr (W < 32) v &= (1u << W) - 1u;
    return v;
}

// Bands of fewer than 8 sub-slices (2^bits < 8) share each sub-slice among 8 / 2^bits XCDs.
// (Non-temporal band loads / partial stores measured no gain at RMAT-24/26 in round 2: 4.12-4.25 vs
// 4.12 ms.)
template <class Op, bool LDS, int PW>
__global__ __launch_bounds__(kMergeThreads) void pull_merge_kernel(MergeArgs a, Op op, typename Op::T* __restrict__ partial,
                                                                   typename Op::T* __restrict__ carry, HotSegs hs,
                                                                   int temporal) {
    using T = typename Op::T;
    extern __shared__ __align__(16) unsigned char merge_lds[];
    const int S = 1 << a.bits;
    const int xs = S < kXcds ? S : kXcds;  // sub-slice residues: h mod xs is fixed by the XCD
    const int rep = kXcds / xs;            // XCDs sharing each sub-slice
    const int per = S / xs;                // sub-slices per XCD
    const int w = (int)(blockIdx.x >> 3), W = (int)(gridDim.x >> 3);
    const int xcd = (int)(blockIdx.x & (kXcds - 1));
    const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    lds_ptr<T> hotv = (lds_ptr<T>)merge_lds;
    const int gshift = 4 + a.bits;
    const int hg = hs.hs >> gshift;  // hot line groups per segment
    const int nl = hs.nseg * hg;     // LDS lines
    lds_ptr<T> stg = hotv + (nl * 16 + 1) + wave * a.stage;  // this wave's partial window (after the image)
    // the block's task counter (dynamic assignment), after every wave's window
    lds_ptr<uint32_t> tctr = (lds_ptr<uint32_t>)(hotv + (nl * 16 + 1) + kMergeWaves * a.stage);
    // Static: block w of an XCD folds sub-slice (w mod per) with the XCD's other W / per blocks of it.
    // Temporal: every block of an XCD sweeps the XCD's per sub-slices in the same order, all W blocks
    // on one sub-slice at a time, so the XCD's L2 holds one sub-slice's part of the vector instead
    // of all of them at once (one image restaged per round).
    const int rounds = temporal ? per : 1;
    const uint32_t hmask = (1u << a.bits) - 1u;
    // the vector line held by LDS line j of segment seg in sub-slice hh's image
    auto image_line = [&](int seg, int j, int hh) {
        const int64_t grp = ((int64_t)seg << (hs.tbits - gshift)) + j;
        return (grp << a.bits) + (int64_t)(hh ^ (sub_hash(grp << gshift) & hmask));
    };
    for (int rd = 0; rd < rounds; ++rd) {
    const int h = (xcd % xs) | ((temporal ? rd : w % per) << 3);
    // this block's rank among h's blocks
    const int64_t g = (int64_t)(temporal ? w : w / per) * rep + xcd / xs;
    const int64_t G = (int64_t)(temporal ? W : W / per) * rep;
    if constexpr (LDS) {
        if (rd > 0) __syncthreads();  // every wave is done with the previous round's image
        // LDS line i = the line of sub-slice h in hot line group i (a permutation of each aligned group).
        // 16-byte units (16 / sizeof(T) elements of one line), kStage loads in flight per thread: with
        // 2^bits sub-slices the image lines are scattered over 2^bits x the image span, so a
        // load-store-load loop would pay one memory round trip each.
        constexpr int kStage = 8;
        constexpr int kUnit = 16 / (int)sizeof(T);
        static_assert(16 % sizeof(T) == 0 && kUnit <= 16, "16-byte staging units");
        const unsigned char* src = reinterpret_cast<const unsigned char*>(op.vec());
        const int units = nl * 16 / kUnit;
        using u4 = uint32_t __attribute__((ext_vector_type(4)));
        lds_ptr<u4> hv4 = (lds_ptr<u4>)merge_lds;
        for (int q0 = 0; q0 < units; q0 += kStage * kMergeThreads) {
            u4 buf[kStage];
#pragma unroll
            for (int u = 0; u < kStage; ++u) {
                const int q = q0 + u * kMergeThreads + (int)threadIdx.x;
                const int i = q * kUnit, sg = i >> 4;
                int seg = 0, j = sg;
                if (hs.nseg > 1) {
                    seg = sg / hg;
                    j = sg - seg * hg;
                }
                buf[u] = u4{0, 0, 0, 0};
                if (q < units)
                    buf[u] = *reinterpret_cast<const u4*>(src + (image_line(seg, j, h) * 16 + (i & 15)) * (int64_t)sizeof(T));
            }
#pragma unroll
            for (int u = 0; u < kStage; ++u) {
                const int q = q0 + u * kMergeThreads + (int)threadIdx.x;
                if (q < units) hv4[q] = buf[u];
            }
        }
        if (threadIdx.x == 0) {
            hotv[nl * 16] = op.identity();  // the cold lanes' cell
            *tctr = 0u;                     // this round's task counter (dynamic)
        }
        __syncthreads();
    }
    const SliceGather<Op> lg{op,       hotv, (uint32_t)hg, hs.tbits - gshift, a.bits, (1u << a.bits) - 1u, (uint32_t)h,
                             (uint32_t)nl * 16u};
    const int64_t base = a.sub_base[h];
    const int64_t ntask = a.sub_base[h + 1] - base;
    const int64_t hbegin = a.sub_begin[h], hend = a.sub_end[h];
    // The block's j-th task, j = 0, 1, ...: interleaved, k = j * G + (g + rd) mod G, so the G blocks of
    // a sub-slice differ by at most one task per round and the rotation spreads the extra tasks over
    // the blocks round by round (chunks of 16 per block gave the low blocks up to one more chunk in
    // every round, ~4% more work by the kernel's end).  Without an LDS image, wave w takes j = w, w +
    // 16, ...; the LDS image kernels' waves take j from the block's LDS counter, so a wave that drew
    // cheaper tasks takes more and the round's barrier waits less for the slowest wave (RMAT-24 0.848
    // -> 0.800 ms).  Any order gives the same result (tasks are independent).
    constexpr bool dyn = LDS;
    const int64_t grot = (g + rd) % G;
    auto task_of = [&](int64_t j) { return j * G + grot; };
    auto grab = [&]() -> int64_t {
        uint32_t j = 0;
        if (lane == 0) j = __hip_atomic_fetch_add(tctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return task_of((int64_t)__builtin_amdgcn_readfirstlane(j));
    };
    int64_t jstat = wave;
    auto advance = [&]() -> int64_t {
        if (dyn) return grab();
        jstat += kMergeWaves;
        return task_of(jstat);
    };
    // a skipped task (a.live): a scalar load of its bit (waiting on it does not wait for the vector
    // gathers in flight), then the next task
    auto dead = [&](int64_t kk) -> bool {
        if (a.live == nullptr || kk >= ntask) return false;
        const uint64_t tt = (uint64_t)(base + kk);
        const uint32_t wd = __builtin_amdgcn_readfirstlane(a.live[tt >> 5]);
        return ((wd >> (tt & 31)) & 1u) == 0;
    };
    int64_t k = dyn ? grab() : task_of(jstat);
    while (dead(k)) k = advance();
    if (k >= ntask) continue;
    // The next task's entries and metadata are loaded while this task's gathers are in flight.  The
    // loop carries the raw load registers (the packed lane chunk, head byte, meta word) and unpacks
    // them at the top, so a prefetch writes straight into them and nothing waits on it until the next
    // task.  Metadata are vector loads (lane 0: j0, lane 1: carry flag; one head byte per lane): a
    // scalar prefetch would hold up every LDS wait (lgkmcnt does not count SMEM in order).
    static_assert(kMergeEpl == 8, "a lane chunk is 8 entries");
    constexpr int DB = PW / 4 - 4;  // dwords of a chunk in pack_b
    auto chunk = [&](int64_t kk) { return (hbegin >> 3) + kk * kWave + lane; };
    auto meta_idx = [&](int64_t kk) { return 2 * (base + kk) + (lane & 1); };
    auto head_idx = [&](int64_t kk) { return (base + kk) * kWave + lane; };
    auto ld = [](const auto* p) { return *p; };
    using v4u = uint32_t __attribute__((ext_vector_type(4)));
    using v2u = uint32_t __attribute__((ext_vector_type(2)));
    auto load_chunk = [&](int64_t kk, uint32_t (&d)[PW / 4]) {
        const int64_t x = chunk(kk);
        const v4u va = ld(reinterpret_cast<const v4u*>(a.pack_a) + x);
        d[0] = va.x, d[1] = va.y, d[2] = va.z, d[3] = va.w;
        if constexpr (DB == 1) {
            d[4] = ld(a.pack_b + x);
        } else if constexpr (DB == 2) {
            const v2u vb = ld(reinterpret_cast<const v2u*>(a.pack_b) + x);
            d[4] = vb.x, d[5] = vb.y;
        } else {
            const v4u vb = ld(reinterpret_cast<const v4u*>(a.pack_b) + x);
            d[4] = vb.x, d[5] = vb.y, d[6] = vb.z, d[7] = vb.w;
        }
    };
    uint32_t cd[PW / 4];
    load_chunk(k, cd);
    uint32_t hb = ld(a.heads + head_idx(k));
    int32_t mw = ld(a.meta + meta_idx(k));
    for (;;) {
        const int64_t t = base + k;
        const int64_t e0 = hbegin + k * kMergeTask;
        const int n = (int)min((int64_t)kMergeTask, hend - e0);
        uint32_t loc[kMergeEpl];
#pragma unroll
        for (int u = 0; u < kMergeEpl; ++u) loc[u] = unpack_entry<PW>(cd, u);
        const int32_t j0 = __builtin_amdgcn_readlane(mw, 0);
        const bool carry_in = __builtin_amdgcn_readlane(mw, 1) != 0;
        const uint32_t hbc = hb;
        T v[kMergeEpl];
        if constexpr (LDS) {
            T vg[kMergeEpl], vl[kMergeEpl];
#pragma unroll
            for (int u = 0; u < kMergeEpl; ++u) vl[u] = lg.hot(loc[u], kMergeEpl * lane + u < n);
#pragma unroll
            for (int u = 0; u < kMergeEpl; ++u) vg[u] = lg.cold(loc[u], kMergeEpl * lane + u < n, true);
#pragma unroll
            for (int u = 0; u < kMergeEpl; ++u) v[u] = op.combine(vl[u], vg[u]);
        } else {
#pragma unroll
            for (int u = 0; u < kMergeEpl; ++u) v[u] = lg.cold(loc[u], kMergeEpl * lane + u < n, false);
        }
        int64_t kn = advance();
        while (dead(kn)) kn = advance();
        if (kn < ntask) {
            load_chunk(kn, cd);
            hb = ld(a.heads + head_idx(kn));
            mw = ld(a.meta + meta_idx(kn));
        }
        // head numbers: exclusive wave scan of the per-lane head counts
        const int cnt = __builtin_popcount(hbc);
        int incl = cnt;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const int o = __shfl_up(incl, d, kWave);
            if (lane >= d) incl += o;
        }
        const int hbase = incl - cnt;  // head number of this lane's first head
        const bool valid_lane = kMergeEpl * lane < n;
        // A task's partials are consecutive slots: with at most `stage` heads they are collected in the
        // wave's LDS window and written by one coalesced store per 64, instead of up to 10 exec-masked
        // scattered stores per lane (the stores cost ~20% of the merge kernel, round 2).
        const int H = __builtin_amdgcn_readlane(incl, kWave - 1);
        const bool staged = LDS && H <= a.stage;
        // (Folding band 0 into one accumulator per (row, XCD), read-modified-written round by round, was
        // measured 7-9% slower than these partials: profiles/r06/abfold/.)
        auto store_partial = [&](int64_t j, T val) { partial[j] = val; };
        auto emit = [&](int hh, T val) {  // segment of head hh
            if (staged) {
                stg[hh] = val;
                return;
            }
            if (hh == 0 && carry_in) carry[t] = val;
            else store_partial(j0 + hh, val);
        };
        // lane-local: the part before the first head (continues the segment on the left), inner
        // segments (emitted here) and the segment of the last head (continues to the right)
        const int fh = hbc ? __builtin_ctz(hbc) : kMergeEpl;
        T pre = op.identity(), run = op.identity();
        int run_h = hbase - 1;
#pragma unroll
        for (int u = 0; u < kMergeEpl; ++u) {
            if (u < fh) {
                pre = u == 0 ? v[u] : op.combine(pre, v[u]);
            } else if ((hbc >> u) & 1u) {
                if (u > fh) emit(run_h, run);  // the previous head's segment ends here
                run = v[u];
                ++run_h;
            } else {
                run = op.combine(run, v[u]);
            }
        }
        // segmented inclusive scan across lanes of (lane_out, has_head, head number)
        T x = fh < kMergeEpl ? run : pre;
        int f = fh < kMergeEpl ? 1 : 0;
        int xh = run_h;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const T xu = op.shfl_up(x, d);
            const int fu = __shfl_up(f, d, kWave);
            const int hu = __shfl_up(xh, d, kWave);
            if (lane >= d) {
                if (!f) {
                    x = op.combine(xu, x);
                    xh = hu;
                }
                f |= fu;
            }
        }
        const T in_x = op.shfl_up(x, 1);
        const int in_h = __shfl_up(xh, 1, kWave);
        if (valid_lane) {
            if (lane > 0 && fh < kMergeEpl) emit(in_h, fh > 0 ? op.combine(in_x, pre) : in_x);
            if (kMergeEpl * (lane + 1) >= n) {  // the task's last segment ends here
                if (fh < kMergeEpl) emit(run_h, run);
                else emit(in_h, lane > 0 ? op.combine(in_x, pre) : pre);
            }
        }
        if (staged) {
            // the window is wave-private and LDS runs a wave's instructions in order: the fences only
            // keep the compiler from moving these reads above the writes (or the next task's writes
            // above these reads)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (int i = lane; i < H; i += kWave) {
                const T val = stg[i];
                if (i == 0 && carry_in) carry[t] = val;
                else store_partial(j0 + i, val);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (kn >= ntask) break;
        k = kn;
    }
    }  // rounds
}

// Sub-rows that span tasks: the sub-row's first task wrote partial[j]; every later task it covers left
// its segment in carry[t] (meta[t] = (j, 1)).  The first carry of each run adds the run in task order.
// (The first task of a sub-slice is never a carry: sub-slices start at a sub-row start.)
// Carries of every band in one launch: thread x of [0, sum of tasks) takes task x - task_begin[b] of
// band b.
constexpr int kMaxBands = 4;
struct FixupBands {
    const int32_t* meta[kMaxBands];
    int64_t task_begin[kMaxBands + 1];
    int64_t part_off[kMaxBands], carry_off[kMaxBands];
    int n;
};
template <class Op>
__global__ void pull_merge_fixup_kernel(FixupBands fb, Op op, typename Op::T* __restrict__ split_partial) {
    using T = typename Op::T;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < fb.task_begin[fb.n];
         x += (int64_t)gridDim.x * blockDim.x) {
        int b = 0;
        while (x >= fb.task_begin[b + 1]) ++b;
        const int64_t t = x - fb.task_begin[b], tasks = fb.task_begin[b + 1] - fb.task_begin[b];
        const int32_t* __restrict__ meta = fb.meta[b];
        T* __restrict__ partial = split_partial + fb.part_off[b];
        const T* __restrict__ carry = split_partial + fb.carry_off[b];
        // one round trip for this task, its predecessor and its successor (most runs are one task
        // long), then the sub-row's partial
        const int64_t tp = t > 0 ? t - 1 : 0, tn = t + 1 < tasks ? t + 1 : t;
        const int32_t f = meta[2 * t + 1], j = meta[2 * t];
        const int32_t pf = meta[2 * tp + 1], pj = meta[2 * tp];
        const int32_t nf = meta[2 * tn + 1], nj = meta[2 * tn];
        const T c = carry[t], cn = carry[tn];
        if (!f || (t > 0 && pf && pj == j)) continue;  // no carry, or not the first carry of the run
        T acc = op.combine(partial[j], c);
        if (tn != t && nf && nj == j) {
            acc = op.combine(acc, cn);
            for (int64_t u = t + 2; u < tasks && meta[2 * u + 1] && meta[2 * u] == j; ++u) acc = op.combine(acc, carry[u]);
        }
        partial[j] = acc;
    }
}

// Row r of the split: fold its non-empty sub-slices in h order.  One lane per row, so a wave reads
// sub-slice h's partials of 64 consecutive rows (consecutive numbers: coalesced); several lanes per
// row were measured slower (their partials of different sub-slices sit far apart).
struct FinalizeBands {
    const uint2* sub_word[kMaxBands];
    int64_t row_begin[kMaxBands];
    int64_t row_end[kMaxBands];
    int64_t part_off[kMaxBands];
    int bits[kMaxBands];
    int n;
};
template <class Op>
__device__ __forceinline__ void slice_finalize_row(int64_t r, const Op& op, const FinalizeBands& fb,
                                                   const typename Op::T* __restrict__ partial) {
    using T = typename Op::T;
    int b = 0;
    while (b < fb.n - 1 && r >= fb.row_end[b]) ++b;
    const int64_t NR = fb.row_end[b] - fb.row_begin[b], i = r - fb.row_begin[b];
    const int64_t W = (NR + 31) / 32, wi = i >> 5;
    const uint32_t below = (1u << (i & 31)) - 1u, me = 1u << (i & 31);
    const int S = 1 << fb.bits[b];
    const uint2* __restrict__ sw = fb.sub_word[b];
    const T* __restrict__ part = partial + fb.part_off[b];
    T acc = op.identity();
    bool first = true;
    // batches of 8 sub-slices: all index loads, then all partial loads, then the fold in h order, and
    // the next batch's index words are loaded with this batch's partials, so a hub row's 128 sub-slices
    // cost 17 round trips instead of 128 dependent pairs (the unpipelined batches: RMAT-26 light+finalize
    // 858 -> 771 us).  The index words are shared by 32 rows (1/16 of the bytes of an int32 index per
    // sub-row).
    uint2 wc[8], wn[8];
    auto load_words = [&](int h0, uint2 (&wd)[8]) {
#pragma unroll
        for (int u = 0; u < 8; ++u)  // bands of fewer than 8 sub-slices: empty words
            wd[u] = h0 + u < S ? sw[(int64_t)(h0 + u) * W + wi] : make_uint2(0u, 0u);
    };
    load_words(0, wc);
    for (int h0 = 0; h0 < S; h0 += 8) {
        int32_t j[8];
        T v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) j[u] = (wc[u].x & me) ? (int32_t)wc[u].y + __popc(wc[u].x & below) : -1;
        if (h0 + 8 < S) load_words(h0 + 8, wn);
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = j[u] >= 0 ? part[j[u]] : op.identity();
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (j[u] >= 0) {
                acc = first ? v[u] : op.combine(acc, v[u]);
                first = false;
            }
#pragma unroll
        for (int u = 0; u < 8; ++u) wc[u] = wn[u];
    }
    op.finalize(r, acc);
}

template <class Op>
__global__ void pull_slice_finalize_kernel(int64_t row0, int64_t rows, Op op, FinalizeBands fb,
                                           const typename Op::T* __restrict__ partial) {
    for (int64_t r = row0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x)
        slice_finalize_row(r, op, fb, partial);
}

// The light rows and the split's finalize in one launch: blocks [0, fin_blocks) finalise split rows
// (one per thread), the rest run light-row blocks.  Both are latency-bound and independent, so
// interleaving their blocks hides one's stalls behind the other's (the order of the two block ranges
// measured equal at RMAT-24 and 26, round 1).
template <class Op, int U>
__global__ __launch_bounds__(kBlock) void pull_light_finalize_kernel(PullArgs a, Op op,
                                                                     typename Op::T* __restrict__ hub_partial,
                                                                     FinalizeBands fb,
                                                                     const typename Op::T* __restrict__ partial,
                                                                     int64_t split_rows, int64_t fin_blocks,
                                                                     int64_t fin_row0) {
    const int64_t b = blockIdx.x;
    if (b < fin_blocks) {
        const int64_t r = fin_row0 + b * kBlock + threadIdx.x;
        if (r < split_rows) slice_finalize_row<Op>(r, op, fb, partial);
        return;
    }
    pull_block<Op, U>(a, op, hub_partial, b - fin_blocks + a.block_offset);
}

// Enqueue one pull superstep on `s`.
// `split_partial` ([8 * plan.split_rows], nullable) enables the XCD split of the heavy rows.

// `skip_empty`: the rows without entries (the degree-sorted suffix, class kZeroClass) are not
// finalised, for programs whose value there no longer changes (PageRank after two power steps).
// `task_live` (nullable): per band, the MergeArgs::live bitmap of its tasks.
// `caller_rows`: the split rows [0, caller_rows) are the caller's this superstep (it gathers and
// finalises them itself: the bit-parallel BFS's early-exit rows); it must end a prefix of the bands,
// which are then neither merged, fixed up nor finalised here.
template <class Op>
void launch_pull(const Csr& csr, const PullPlan& plan, const Op& op, typename Op::T* hub_partial, hipStream_t s,
                 Ctx* prof_ctx = nullptr, Shard* prof_shard = nullptr, typename Op::T* split_partial = nullptr,
                 bool skip_empty = false, const uint32_t* const* task_live = nullptr, int64_t caller_rows = 0) {
    using T = typename Op::T;
    const bool split = tune().pull_split && plan.split_rows > 0 && split_partial != nullptr;
    size_t band0 = 0;  // the first band this call merges
    if (caller_rows > 0) {
        while (band0 < plan.bands.size() && plan.bands[band0]->row_end <= caller_rows) ++band0;
        if (!split || band0 == 0 || plan.bands[band0 - 1]->row_end != caller_rows)
            fail(JG_ERR_UNSUPPORTED, "launch_pull: caller rows must end a prefix of the split bands");
    }
    PullArgs a = make_pull_args(csr, plan, split);
    if (skip_empty) a.class_block_begin[kNumClasses] = a.class_block_begin[kZeroClass];
    const int64_t blocks = a.class_block_begin[kNumClasses];
    if (prof_ctx) prof_record_start(*prof_ctx, *prof_shard);
    // (Measured and removed: the light rows on a side stream beside the merge kernels, band 1's merge on
    // a side stream beside band 0's, two merge workgroups per CU with half the LDS image each, the light
    // rows through a persistent LDS-prefix kernel: no gain or slower at RMAT-24 and 26)
    if (split) {
        static bool attr = false;
        if (!attr) {
            JG_HIP(hipFuncSetAttribute((const void*)pull_merge_kernel<Op, true, 20>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kMergeLdsBytes));
            JG_HIP(hipFuncSetAttribute((const void*)pull_merge_kernel<Op, true, 24>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kMergeLdsBytes));
            JG_HIP(hipFuncSetAttribute((const void*)pull_merge_kernel<Op, true, 32>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kMergeLdsBytes));
            attr = true;
        }
        for (size_t bi = band0; bi < plan.bands.size(); ++bi) {
            const SliceBand& bd = *plan.bands[bi];
            if (bd.tasks == 0) continue;
            // staging window: -1 = automatic, the power of two >= 4x the band's mean heads per task,
            // within [128, 256] (RMAT-24 band 0 ~21 heads: 128; RMAT-26 band 0 ~73 and band 1 ~110:
            // 256).  Heads per task are heavy-tailed (tasks of short sub-rows near the band's degree
            // floor), and a task over the window stores directly: at RMAT-24 a 64-slot window was
            // 1.6% slower than 128 although the mean is 21.
            int stage = tune().merge_stage[std::min<size_t>(bi, 3)];
            if (stage < 0) {
                const double heads = (double)bd.subrows / (double)std::max<int64_t>(bd.tasks, 1);
                stage = 128;
                while (stage < 4.0 * heads && stage < 256) stage *= 2;
            }
            MergeArgs ma{bd.pack_a.get(), bd.pack_b.get(), bd.heads.get(), bd.meta.get(), bd.sub_begin.get(),
                         bd.sub_end.get(), bd.sub_base.get(), bd.tasks, bd.bits, stage,
                         task_live ? task_live[bi] : nullptr};
            T* part = split_partial + bd.part_off;
            T* carry = split_partial + bd.carry_off;
            // LDS image: kMergeLdsBytes / sizeof(T) - 16 elements (1 identity line) per sub-slice
            const int64_t S = 1ll << bd.bits, gsz = 16 * S;
            // one workgroup per CU, a multiple of S: every sub-slice gets grid / S of them
            const unsigned grid = (unsigned)std::max<int64_t>(S, (int64_t)device_cu_count() / S * S);
            // shared equally by the segments; a segment's hot part stays below its stride
            const int64_t stage_bytes = (int64_t)kMergeWaves * stage * (int64_t)sizeof(T);
            const int64_t hot_max = (int64_t)((kMergeLdsBytes - stage_bytes - 16) / (int64_t)sizeof(T) - 16) * S;
            HotSegs hs;
            hs.tbits = plan.seg_tbits;
            hs.nseg = plan.nseg;
            const int64_t seg_cap = plan.nseg == 1 ? plan.col_space : (1ll << plan.seg_tbits) - gsz;
            hs.hs = plan.lds_ok ? (int32_t)(std::min<int64_t>(hot_max / plan.nseg, seg_cap) / gsz * gsz) : 0;
            const int temporal = tune().merge_temporal == 2 || (tune().merge_temporal == 1 && plan.temporal);
            const size_t lds = hs.hs > 0 ? (size_t)(hs.nseg * (hs.hs / S) + 1) * sizeof(T) + (size_t)stage_bytes + 16 : 0;
            auto go = [&](auto kern) { kern<<<grid, kMergeThreads, lds, s>>>(ma, op, part, carry, hs, temporal); };
            if (hs.hs > 0) {
                if (bd.width == 20) go(pull_merge_kernel<Op, true, 20>);
                else if (bd.width == 24) go(pull_merge_kernel<Op, true, 24>);
                else go(pull_merge_kernel<Op, true, 32>);
            } else {
                if (bd.width == 20) go(pull_merge_kernel<Op, false, 20>);
                else if (bd.width == 24) go(pull_merge_kernel<Op, false, 24>);
                else go(pull_merge_kernel<Op, false, 32>);
            }
            JG_LAUNCH_CHECK();
        }
        FixupBands fx{};
        for (size_t bi = band0; bi < plan.bands.size(); ++bi) {
            const auto& bp = plan.bands[bi];
            if (fx.n == kMaxBands) fail(JG_ERR_UNSUPPORTED, "too many split bands");
            fx.meta[fx.n] = bp->meta.get();
            fx.part_off[fx.n] = bp->part_off;
            fx.carry_off[fx.n] = bp->carry_off;
            fx.task_begin[fx.n + 1] = fx.task_begin[fx.n] + bp->tasks;
            ++fx.n;
        }
        if (fx.task_begin[fx.n] > 0) {
            pull_merge_fixup_kernel<Op><<<grid_for(fx.task_begin[fx.n], kBlock, 0), kBlock, 0, s>>>(fx, op, split_partial);
            JG_LAUNCH_CHECK();
        }
    }
    // 4 gathers in flight per lane (8 measured no faster: RMAT-26 4.36 vs 4.32 ms, round 1)
    auto launch = [&](unsigned grid) {
        pull_kernel<Op, 4><<<grid, kBlock, 0, s>>>(a, op, hub_partial);
        JG_LAUNCH_CHECK();
    };
    FinalizeBands fb{};
    if (split) {
        for (const auto& bp : plan.bands) {
            if (fb.n == kMaxBands) fail(JG_ERR_UNSUPPORTED, "too many split bands");
            fb.sub_word[fb.n] = bp->sub_word.get();
            fb.row_begin[fb.n] = bp->row_begin;
            fb.row_end[fb.n] = bp->row_end;
            fb.part_off[fb.n] = bp->part_off;
            fb.bits[fb.n] = bp->bits;
            ++fb.n;
        }
    }
    const bool fuse = split && !pull_split_launches();
    if (fuse) {
        const int64_t fin_blocks = (plan.split_rows - caller_rows + kBlock - 1) / kBlock;
        const unsigned grid = (unsigned)(fin_blocks + blocks);
        pull_light_finalize_kernel<Op, 4><<<grid, kBlock, 0, s>>>(a, op, hub_partial, fb, split_partial, plan.split_rows,
                                                                  fin_blocks, caller_rows);
        JG_LAUNCH_CHECK();
    } else if (pull_split_launches()) {  // diagnostic: one launch per degree class (per-class rocprof times)
        for (int c = 0; c < kNumClasses; ++c) {
            const int64_t b0 = a.class_block_begin[c], b1 = a.class_block_begin[c + 1];
            if (b1 <= b0) continue;
            a.block_offset = b0;
            launch((unsigned)(b1 - b0));
        }
    } else if (blocks > 0) {
        launch((unsigned)blocks);
    }
    // with the split, hub rows inside it are finalised by it (skip the launch when that is all of them)
    if (plan.num_hub_rows > 0 && !(split && plan.max_hub_row < plan.split_rows)) {
        pull_hub_finalize_kernel<Op><<<grid_for(plan.num_hub_rows), kBlock, 0, s>>>(a, op, hub_partial);
        JG_LAUNCH_CHECK();
    }
    if (split && !fuse) {
        if (plan.split_rows > caller_rows)
            pull_slice_finalize_kernel<Op><<<grid_for(plan.split_rows - caller_rows), kBlock, 0, s>>>(
                caller_rows, plan.split_rows, op, fb, split_partial);
        JG_LAUNCH_CHECK();
    }
    if (prof_ctx) prof_record_stop(*prof_ctx, *prof_shard);  // the whole superstep: every launch above
}

}  // namespace jg
