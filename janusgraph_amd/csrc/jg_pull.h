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
// An Op supplies: T, identity(), combine(a,b), gather(col), shfl_xor(v,o), active(row) (false: the
// row is not folded but still finalised with identity()), finalize(row, acc).
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
    return a;
}

template <bool NT>
__device__ __forceinline__ int32_t load_col(const int32_t* __restrict__ col, int64_t j) {
    if constexpr (NT) return __builtin_nontemporal_load(col + j);  // streamed once: don't keep it in cache
    else return col[j];
}

// How a fold reads the gathered vector: straight from global memory, or from an LDS copy of its
// hottest prefix (the degree-sorted first `hot` ids) with global memory for the rest.
template <class Op>
struct GlobalGather {
    const Op& op;
    __device__ __forceinline__ typename Op::T operator()(int32_t c) const { return op.gather(c); }
};
// LDS pointers keep address space 3: through a generic pointer the compiler emits flat loads, which
// go through the TA/TD like global loads and defeat the point of staging.
template <class T>
using lds_ptr = __attribute__((address_space(3))) T*;

template <class Op>
struct LdsGather {
    const Op& op;
    lds_ptr<const typename Op::T> lds;
    int32_t hot;
    __device__ __forceinline__ typename Op::T operator()(int32_t c) const { return c < hot ? lds[c] : op.gather(c); }
};

// Fold col[j..j1) with stride `stride`; U gathers in flight per lane, folded in index order.
// Software-pipelined: the col batch of iteration i+1 is loaded while the gathers of iteration i are
// in flight, so a long row pays one round trip per batch instead of two.  The last, partial batch is
// not walked one entry at a time: its out-of-range slots re-read the row's last entry (a cache hit)
// and are dropped from the fold by a select, so every batch is branch-free.
template <class Op, int U, bool NT>
__device__ __forceinline__ void load_cols(const int32_t* __restrict__ col, int64_t j, int64_t j1, int stride,
                                          int32_t (&c)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t k = j + u * (int64_t)stride;
        c[u] = load_col<NT>(col, k < j1 ? k : j1 - 1);
    }
}

template <class G, class = void>
struct is_split_gather { static constexpr bool value = false; };
template <class G>
struct is_split_gather<G, decltype((void)G::kSplit)> { static constexpr bool value = G::kSplit; };

template <class Op, int U, bool NT, class G>
__device__ __forceinline__ typename Op::T fold_strided(const Op& op, const G& gather, const int32_t* __restrict__ col,
                                                       int64_t j, int64_t j1, int stride) {
    using T = typename Op::T;
    T acc = op.identity();
    if (j >= j1) return acc;
    int32_t c[U];
    load_cols<Op, U, NT>(col, j, j1, stride, c);
    for (;;) {
        T v[U];
        const int64_t jn = j + U * (int64_t)stride;
        if constexpr (is_split_gather<G>::value) {
            // Wait for the whole col batch once (the empty asm needs every c[u] in a register), so
            // the masked global loads below issue back to back: exec-masked, a hot lane costs the
            // TA/TD nothing (an out-of-range buffer lane still costs a TD cycle).  The LDS reads are
            // unconditional (cold lanes read the identity cell) and land in their own registers.
            static_assert(U == 4, "split gathers are written for U == 4");
            asm volatile("" : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]));
            T vg[U], vl[U];
#pragma unroll
            for (int u = 0; u < U; ++u) vl[u] = gather.hot(c[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) vg[u] = gather.cold(c[u]);
            load_cols<Op, U, NT>(col, jn, j1, stride, c);
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = op.combine(vl[u], vg[u]);
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = gather(c[u]);
            load_cols<Op, U, NT>(col, jn, j1, stride, c);  // clamped: unconditional keeps vmcnt counting exact
        }
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

template <class Op, int U, bool NT>
__device__ __forceinline__ typename Op::T fold_strided(const Op& op, const int32_t* __restrict__ col, int64_t j,
                                                       int64_t j1, int stride) {
    return fold_strided<Op, U, NT>(op, GlobalGather<Op>{op}, col, j, j1, stride);
}

// `tid` is the thread's index inside its (virtual) 256-thread block.
template <class Op, int L, int U, bool NT, class G>
__device__ __forceinline__ void pull_rows_class(const PullArgs& a, const Op& op, const G& gather, int c,
                                                int64_t local_block, int tid) {
    using T = typename Op::T;
    constexpr int kRowsPerBlock = kBlock / L;
    const int sub = tid % L;
    const int64_t row = a.class_row_begin[c] + local_block * kRowsPerBlock + tid / L;
    const bool valid = row < a.class_row_end[c];
    T acc = op.identity();
    bool hub = false;
    if (valid) {
        const int64_t j0 = a.row_ptr[row], j1 = a.row_ptr[row + 1];
        hub = (j1 - j0) >= kHubDegree;  // folded by the chunk path
        if (!hub && op.active(row)) acc = fold_strided<Op, U, NT>(op, gather, a.col, j0 + sub, j1, L);
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
template <class Op, int U, bool NT, class G>
__device__ __forceinline__ void pull_block_rows(const PullArgs& a, const Op& op, const G& gather, int64_t b, int tid) {
    int c = 1;
#pragma unroll
    for (int k = 1; k < kNumClasses; ++k)
        if (b >= a.class_block_begin[k + 1]) c = k + 1;
    const int64_t lb = b - a.class_block_begin[c];
    switch (c) {
        case 1: pull_rows_class<Op, 64, U, NT>(a, op, gather, c, lb, tid); break;
        case 2: pull_rows_class<Op, 32, U, NT>(a, op, gather, c, lb, tid); break;
        case 3: pull_rows_class<Op, 16, U, NT>(a, op, gather, c, lb, tid); break;
        case 4: pull_rows_class<Op, 8, U, NT>(a, op, gather, c, lb, tid); break;
        case 5: pull_rows_class<Op, 4, U, NT>(a, op, gather, c, lb, tid); break;
        case 6: pull_rows_class<Op, 2, U, NT>(a, op, gather, c, lb, tid); break;
        case 7: pull_rows_class<Op, 1, U, NT>(a, op, gather, c, lb, tid); break;
        default: pull_rows_empty<Op>(a, op, lb, tid); break;
    }
}

template <class Op, int U, bool NT>
__global__ __launch_bounds__(kBlock) void pull_kernel(PullArgs a, Op op, typename Op::T* __restrict__ hub_partial) {
    using T = typename Op::T;
    const int64_t b = (int64_t)blockIdx.x + a.block_offset;
    if (b < a.num_chunks) {
        __shared__ T red[kBlock / kWave];
        const int64_t j0 = a.chunk_begin[b], j1 = a.chunk_end[b];
        const int64_t crow = a.chunk_row[b];
        T acc = (crow >= a.skip_rows && op.active(crow)) ? fold_strided<Op, U, NT>(op, a.col, j0 + threadIdx.x, j1, kBlock)
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
    pull_block_rows<Op, U, NT>(a, op, GlobalGather<Op>{op}, b, (int)threadIdx.x);
}

// LDS-cached variant (persistent, 1024 threads = 4 virtual 256-thread blocks, one workgroup per
// CU): the gathered vector's hottest prefix [0, hot) — the highest-degree vertices after the
// degree-sorted relabel — is staged once per superstep into LDS (up to 160 KiB), so those gathers
// never become L2 requests (the pull superstep is bound by L2 request rate, not bytes:
// tools/pr_locality.py).  Virtual blocks >= num_chunks are dealt round-robin; hub chunks stay with
// pull_kernel.  No block-wide barrier after the staging one, so the four virtual blocks run freely.
constexpr int kLdsThreads = 1024;
template <class Op, int U, bool NT>
__global__ __launch_bounds__(kLdsThreads) void pull_lds_kernel(PullArgs a, Op op, int32_t hot) {
    using T = typename Op::T;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    lds_ptr<T> lds = (lds_ptr<T>)lds_raw;
    const T* src = op.vec();
    for (int i = threadIdx.x; i < hot; i += kLdsThreads) lds[i] = src[i];
    __syncthreads();
    const LdsGather<Op> gather{op, lds, hot};
    constexpr int kVirt = kLdsThreads / kBlock;
    const int tid = threadIdx.x % kBlock;
    const int64_t last = a.class_block_begin[kNumClasses];
    for (int64_t b = a.class_block_begin[1] + (int64_t)blockIdx.x * kVirt + threadIdx.x / kBlock; b < last;
         b += (int64_t)gridDim.x * kVirt)
        pull_block_rows<Op, U, NT>(a, op, gather, b, tid);
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

// ---------------- XCD-sliced split of the heavy rows (PullPlan::split_*) ----------------
// The entries of every heavy row of a sliced CSR are grouped by col_slice (mode 1: each aligned
// group of 8 lines of the gathered vector gives one line to every slice).  A wave item is (task t,
// slice q); every item of slice q runs in a workgroup b with b mod 8 == q, which the dispatcher
// deals to one XCD (speed only: any placement gives the same result), so each XCD's L2 only ever
// holds its own eighth of the vector.  On one shard the workgroup also stages the hottest lines of
// its slice (the first kSliceLdsLines line groups, i.e. ids < 16 * 8 * kSliceLdsLines) in LDS, and
// those gathers never leave the CU: the superstep is bound by TCP->L2 requests in flight
// (PMC: TA/TD ~95% busy stalled on the TCP), not by bytes.
//   task kind R (meta & 0xff = L lanes per row, meta >> 8 = rows): 64/L consecutive rows, sub-row
//             (r, q) folded by L lanes, written to partial[q * split_rows + r]
//   task kind C (meta & 0xff = 0, meta >> 8 = k | K << 12): chunk k of K of sub-row (r, q), folded by
//             the wave, written to chunk_partial[t * 8 + q]; the chunked rows are the prefix
//             [0, chunk_rows) and their tasks the prefix of the task list (chunk_ptr[r] = first task)
// pull_slice_finalize_kernel folds the 8 slices (and the chunks of chunked rows) in fixed order.
constexpr int kSliceThreads = 1024;                   // one workgroup per CU
constexpr int kSliceLdsBytes = 160 * 1024;            // all of the CU's LDS

struct SliceArgs {
    const int64_t* __restrict__ slice_ptr;  // [8 * rows + 1], slice-major
    const int32_t* __restrict__ col;        // slice_col
    const int32_t* __restrict__ task_row;
    const int32_t* __restrict__ task_meta;
    int64_t ntasks;
    int64_t rows;       // split (heavy) rows
    uint32_t vec_bytes;  // bytes of the gathered vector (buffer resource range)
};

// Sub-row (r, q): [j0, j1) of col.
__device__ __forceinline__ void slice_segment(const SliceArgs& a, int64_t r, int q, int64_t& j0, int64_t& j1) {
    const int64_t i = (int64_t)q * a.rows + r;
    j0 = a.slice_ptr[i];
    j1 = a.slice_ptr[i + 1];
}

// Gathers of slice q: ids below `hot` come from the LDS image of the slice's first lines (line group
// c >> 7 holds one line of this slice; it sits at LDS line c >> 7), the rest from global memory.
// Split form for fold_strided: hot(c) / cold(c) each return identity() for the other kind, and
// combine(hot, cold) is the gathered value (exact: combine(x, identity) == x).
template <class Op>
struct SliceLdsGather {
    static constexpr bool kSplit = true;
    using T = typename Op::T;
    const Op& op;
    lds_ptr<const T> lds;
    int32_t hot_ids;
    // Cold lanes read the identity cell just past the staged lines: no select, so the compiler
    // cannot turn the read into a branch.
    __device__ __forceinline__ T hot(int32_t c) const {
        return lds[c < hot_ids ? (((c >> 7) << 4) | (c & 15)) : (hot_ids >> 3)];
    }
    // Only cold lanes load (exec-masked); the others keep identity().
    __device__ __forceinline__ T cold(int32_t c) const {
        T v = op.identity();
        if (c >= hot_ids) v = op.gather(c);
        return v;
    }
};

template <class Op, int L, int U, class G>
__device__ __forceinline__ void slice_rows_item(const SliceArgs& a, const Op& op, const G& gather, int q, int64_t row0,
                                                int nrows, int lane, typename Op::T* __restrict__ partial) {
    using T = typename Op::T;
    const int sub = lane % L;
    const int local = lane / L;
    const int64_t r = row0 + local;
    const bool valid = local < nrows;
    T acc = op.identity();
    if (valid && op.active(r)) {
        int64_t j0, j1;
        slice_segment(a, r, q, j0, j1);
        acc = fold_strided<Op, U, false>(op, gather, a.col, j0 + sub, j1, L);
    }
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) acc = op.combine(acc, op.shfl_xor(acc, o));
    if (valid && sub == 0) partial[(int64_t)q * a.rows + r] = acc;
}

template <class Op, int U, bool LDS>
__global__ __launch_bounds__(kSliceThreads) void pull_slice_kernel(SliceArgs a, Op op, typename Op::T* __restrict__ partial,
                                                                   typename Op::T* __restrict__ chunk_partial,
                                                                   int32_t hot) {
    using T = typename Op::T;
    extern __shared__ __align__(16) unsigned char slice_lds_raw[];
    lds_ptr<T> lds = (lds_ptr<T>)slice_lds_raw;
    const int q = (int)(blockIdx.x & (kXcds - 1));
    const int64_t g = blockIdx.x >> 3, G = gridDim.x >> 3;
    if constexpr (LDS) {
        // LDS line i = the line of slice q in line group i (mode-1 slices permute each aligned group)
        const T* src = op.vec();
        const int nl = hot >> 7;  // line groups staged
        for (int i = threadIdx.x; i < nl * 16; i += kSliceThreads) {
            const int grp = i >> 4;
            const int line = grp * 8 + (q ^ col_slice((int64_t)grp * 128, 1));
            lds[i] = src[line * 16 + (i & 15)];
        }
        if (threadIdx.x == 0) lds[nl * 16] = op.identity();  // the cold lanes' cell (SliceLdsGather::hot)
        __syncthreads();
    }
    const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    constexpr int kWaves = kSliceThreads / kWave;
    for (int64_t t = g * kWaves + wave; t < a.ntasks; t += G * kWaves) {
        const int64_t row0 = a.task_row[t];
        const int meta = a.task_meta[t];
        const int L = meta & 0xff;
        const int arg = meta >> 8;
        auto run = [&](const auto& gather) {
            switch (L) {
                case 0: {  // chunk k of K of sub-row (row0, q)
                    const int k = arg & 0xfff, K = arg >> 12;
                    int64_t j0, j1;
                    slice_segment(a, row0, q, j0, j1);
                    const int64_t len = j1 - j0;
                    const int64_t c0 = j0 + len * k / K, c1 = j0 + len * (k + 1) / K;
                    T acc = op.active(row0) ? fold_strided<Op, U, false>(op, gather, a.col, c0 + lane, c1, kWave)
                                            : op.identity();
#pragma unroll
                    for (int o = kWave / 2; o > 0; o >>= 1) acc = op.combine(acc, op.shfl_xor(acc, o));
                    if (lane == 0) chunk_partial[t * kXcds + q] = acc;
                    break;
                }
                case 64: slice_rows_item<Op, 64, U>(a, op, gather, q, row0, arg, lane, partial); break;
                case 32: slice_rows_item<Op, 32, U>(a, op, gather, q, row0, arg, lane, partial); break;
                case 16: slice_rows_item<Op, 16, U>(a, op, gather, q, row0, arg, lane, partial); break;
                case 8: slice_rows_item<Op, 8, U>(a, op, gather, q, row0, arg, lane, partial); break;
                case 4: slice_rows_item<Op, 4, U>(a, op, gather, q, row0, arg, lane, partial); break;
                case 2: slice_rows_item<Op, 2, U>(a, op, gather, q, row0, arg, lane, partial); break;
                default: slice_rows_item<Op, 1, U>(a, op, gather, q, row0, arg, lane, partial); break;
            }
        };
        if constexpr (LDS) run(SliceLdsGather<Op>{op, lds, hot});
        else run(GlobalGather<Op>{op});
    }
}

// Row r: fold the 8 slices in q order; a chunked row folds each slice's chunks in k order first.
template <class Op>
__global__ void pull_slice_finalize_kernel(int64_t rows, int64_t chunk_rows, const int32_t* __restrict__ chunk_ptr,
                                           Op op, const typename Op::T* __restrict__ partial,
                                           const typename Op::T* __restrict__ chunk_partial) {
    using T = typename Op::T;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
        T acc = op.identity();
        if (r < chunk_rows) {
            const int t0 = chunk_ptr[r], t1 = chunk_ptr[r + 1];
            for (int q = 0; q < kXcds; ++q) {
                T sq = op.identity();
                for (int t = t0; t < t1; ++t) sq = op.combine(sq, chunk_partial[(int64_t)t * kXcds + q]);
                acc = op.combine(acc, sq);
            }
        } else {
#pragma unroll
            for (int q = 0; q < kXcds; ++q) acc = op.combine(acc, partial[(int64_t)q * rows + r]);
        }
        op.finalize(r, acc);
    }
}

// Enqueue one pull superstep on `s`.
// `split_partial` ([8 * plan.split_rows], nullable) enables the XCD split of the heavy rows.
constexpr int64_t kMaxLdsBytes = 160 * 1024;

template <class Op>
void launch_pull(const Csr& csr, const PullPlan& plan, const Op& op, typename Op::T* hub_partial, hipStream_t s,
                 Ctx* prof_ctx = nullptr, Shard* prof_shard = nullptr, typename Op::T* split_partial = nullptr) {
    using T = typename Op::T;
    const bool split = tune().pull_split && plan.split_rows > 0 && split_partial != nullptr;
    PullArgs a = make_pull_args(csr, plan, split);
    const int64_t blocks = split ? plan.light_block_begin[kNumClasses] : plan.total_blocks();
    if (prof_ctx) prof_record_start(*prof_ctx, *prof_shard);
    if (split) {
        SliceArgs sa{plan.slice_ptr.get(), plan.slice_col.get(), plan.task_row.get(), plan.task_meta.get(),
                     plan.split_tasks, plan.split_rows,
                     (uint32_t)std::min<int64_t>(plan.col_space * (int64_t)sizeof(T), 0xffffffffll)};
        T* chunk_partial = split_partial + kXcds * plan.split_rows;
        const unsigned grid = (unsigned)(device_cu_count() / kXcds * kXcds);
        const int64_t hot_max = (int64_t)(kSliceLdsBytes / sizeof(T) - 16) * kXcds;  // full LDS, 1 identity line
        const bool lds_ok = plan.lds_ok && tune().slice_lds && plan.col_space * (int64_t)sizeof(T) < (1ll << 32);
        const int32_t hot = lds_ok ? (int32_t)(std::min<int64_t>(hot_max, plan.col_space) >> 7 << 7) : 0;
        bool launched = false;
        if constexpr (Op::kZeroIdentity) {
            if (hot > 0) {
                static bool attr = false;
                if (!attr) {
                    JG_HIP(hipFuncSetAttribute((const void*)pull_slice_kernel<Op, 4, true>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, kSliceLdsBytes));
                    attr = true;
                }
                const size_t bytes = (size_t)(hot / kXcds + 1) * sizeof(T);
                pull_slice_kernel<Op, 4, true><<<grid, kSliceThreads, bytes, s>>>(sa, op, split_partial, chunk_partial,
                                                                                 hot);
                launched = true;
            }
        }
        if (!launched)
            pull_slice_kernel<Op, 4, false><<<grid, kSliceThreads, 0, s>>>(sa, op, split_partial, chunk_partial, 0);
        JG_LAUNCH_CHECK();
    }
    auto launch = [&](unsigned grid) {
        const int u = tune().pull_unroll;
        const bool nt = tune().pull_nt != 0;
        if (u >= 8) {
            if (nt) pull_kernel<Op, 8, true><<<grid, kBlock, 0, s>>>(a, op, hub_partial);
            else pull_kernel<Op, 8, false><<<grid, kBlock, 0, s>>>(a, op, hub_partial);
        } else {
            if (nt) pull_kernel<Op, 4, true><<<grid, kBlock, 0, s>>>(a, op, hub_partial);
            else pull_kernel<Op, 4, false><<<grid, kBlock, 0, s>>>(a, op, hub_partial);
        }
        JG_LAUNCH_CHECK();
    };
    if (!split && tune().pull_lds > 0 && plan.lds_ok) {  // LDS-cached hot prefix (single shard, unsliced)
        const int32_t hot = (int32_t)std::min<int64_t>(tune().pull_lds, kMaxLdsBytes / (int64_t)sizeof(T));
        if (plan.num_chunks > 0) launch((unsigned)plan.num_chunks);  // hub chunks: blocks [0, num_chunks)
        const size_t bytes = (size_t)hot * sizeof(T);
        const unsigned grid = (unsigned)device_cu_count();
        static bool attr = false;
        if (!attr) {
            JG_HIP(hipFuncSetAttribute((const void*)pull_lds_kernel<Op, 4, false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLdsBytes));
            attr = true;
        }
        pull_lds_kernel<Op, 4, false><<<grid, kLdsThreads, bytes, s>>>(a, op, hot);
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
    if (prof_ctx) prof_record_stop(*prof_ctx, *prof_shard);
    if (plan.num_hub_rows > 0) {
        pull_hub_finalize_kernel<Op><<<grid_for(plan.num_hub_rows), kBlock, 0, s>>>(a, op, hub_partial);
        JG_LAUNCH_CHECK();
    }
    if (split) {
        pull_slice_finalize_kernel<Op><<<grid_for(plan.split_rows), kBlock, 0, s>>>(
            plan.split_rows, plan.chunk_rows, plan.chunk_ptr.get(), op, split_partial,
            split_partial + kXcds * plan.split_rows);
        JG_LAUNCH_CHECK();
    }
}

}  // namespace jg
