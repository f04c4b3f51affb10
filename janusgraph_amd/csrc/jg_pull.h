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
template <class Op>
struct LdsGather {
    const Op& op;
    const typename Op::T* lds;
    int32_t hot;
    __device__ __forceinline__ typename Op::T operator()(int32_t c) const { return c < hot ? lds[c] : op.gather(c); }
};

// Fold col[j..j1) with stride `stride`; U gathers in flight per lane, folded in index order.
template <class Op, int U, bool NT, class G>
__device__ __forceinline__ typename Op::T fold_strided(const Op& op, const G& gather, const int32_t* __restrict__ col,
                                                       int64_t j, int64_t j1, int stride) {
    using T = typename Op::T;
    T acc = op.identity();
    for (; j + (U - 1) * (int64_t)stride < j1; j += U * (int64_t)stride) {
        int32_t c[U];
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = load_col<NT>(col, j + u * (int64_t)stride);
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = gather(c[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) acc = op.combine(acc, v[u]);
    }
    for (; j < j1; j += stride) acc = op.combine(acc, gather(load_col<NT>(col, j)));
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
    T* lds = reinterpret_cast<T*>(lds_raw);
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

// ---------------- XCD column split of the heavy rows (PullPlan::split_*) ----------------
struct SplitArgs {
    const int64_t* __restrict__ row_ptr;
    const int32_t* __restrict__ col;
    const int32_t* __restrict__ task_row;
    const int32_t* __restrict__ task_meta;
    const uint32_t* __restrict__ split_off;
    unsigned long long* __restrict__ heads;
    int64_t ntasks;
    int64_t rows;  // heavy rows
    unsigned long long* __restrict__ dbg;  // JG_DEBUG_SPLIT: [8 xcc][8 ranges] task counts (nullable)
};

// XCD (0..7) the calling workgroup runs on.  Placement is only a speed hint: any XCD may take any
// range (stealing), results do not depend on it.
__device__ __forceinline__ int xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return (int)(v & 7u);
}

__device__ __forceinline__ void split_segment(const SplitArgs& a, int64_t r, int q, int64_t& j0, int64_t& j1) {
    const int64_t base = a.row_ptr[r];
    j0 = base + a.split_off[r * kXcds + q];
    j1 = q == kXcds - 1 ? a.row_ptr[r + 1] : base + a.split_off[r * kXcds + q + 1];
}

template <class Op, int L, bool NT>
__device__ __forceinline__ void split_rows_task(const SplitArgs& a, const Op& op, int q, int64_t row0, int nrows,
                                                typename Op::T* __restrict__ partial) {
    using T = typename Op::T;
    const int sub = threadIdx.x % L;
    const int local = threadIdx.x / L;
    const int64_t r = row0 + local;
    const bool valid = local < nrows;
    T acc = op.identity();
    if (valid && op.active(r)) {
        int64_t j0, j1;
        split_segment(a, r, q, j0, j1);
        acc = fold_strided<Op, 4, NT>(op, a.col, j0 + sub, j1, L);
    }
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) acc = op.combine(acc, op.shfl_xor(acc, o));
    if (valid && sub == 0) partial[(int64_t)q * a.rows + r] = acc;
}

template <class Op, bool NT>
__device__ __forceinline__ void split_hub_task(const SplitArgs& a, const Op& op, int q, int64_t r,
                                               typename Op::T* __restrict__ partial, typename Op::T* red) {
    using T = typename Op::T;
    T acc = op.identity();
    if (op.active(r)) {
        int64_t j0, j1;
        split_segment(a, r, q, j0, j1);
        acc = fold_strided<Op, 4, NT>(op, a.col, j0 + threadIdx.x, j1, kBlock);
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) acc = op.combine(acc, op.shfl_xor(acc, o));
    if (lane_id() == 0) red[wave_id()] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        T t = red[0];
#pragma unroll
        for (int w = 1; w < kBlock / kWave; ++w) t = op.combine(t, red[w]);
        partial[(int64_t)q * a.rows + r] = t;
    }
}

// Workgroups loop over (task, range) items: their own XCD's queue first, then the others'.  Every
// item is processed exactly once and written to its own partial slot, so the result is independent
// of placement and timing.  Every workgroup exits once all eight queues are drained.
template <class Op, bool NT>
__global__ __launch_bounds__(kBlock) void pull_split_kernel(SplitArgs a, Op op, typename Op::T* __restrict__ partial) {
    using T = typename Op::T;
    __shared__ long long s_task;
    __shared__ int s_q;
    __shared__ T red[kBlock / kWave];
    int q = xcc_id(), tried = 0;  // thread 0's dequeue state
    for (;;) {
        if (threadIdx.x == 0) {
            long long t = -1;
            while (tried < kXcds) {
                const unsigned long long k = atomicAdd(&a.heads[q], 1ull);
                if ((long long)k < a.ntasks) { t = (long long)k; break; }
                ++tried;
                q = (q + 1) & (kXcds - 1);
            }
            s_task = t;
            s_q = q;
        }
        __syncthreads();
        const long long t = s_task;
        const int qq = s_q;
        __syncthreads();
        if (t < 0) break;
        if (a.dbg && threadIdx.x == 0) atomicAdd(&a.dbg[xcc_id() * kXcds + qq], 1ull);
        const int64_t row0 = a.task_row[t];
        const int meta = a.task_meta[t];
        const int nrows = meta >> 8;
        switch (meta & 0xff) {
            case 0: split_hub_task<Op, NT>(a, op, qq, row0, partial, red); __syncthreads(); break;
            case 64: split_rows_task<Op, 64, NT>(a, op, qq, row0, nrows, partial); break;
            case 32: split_rows_task<Op, 32, NT>(a, op, qq, row0, nrows, partial); break;
            case 16: split_rows_task<Op, 16, NT>(a, op, qq, row0, nrows, partial); break;
            case 8: split_rows_task<Op, 8, NT>(a, op, qq, row0, nrows, partial); break;
            case 4: split_rows_task<Op, 4, NT>(a, op, qq, row0, nrows, partial); break;
            default: split_rows_task<Op, 2, NT>(a, op, qq, row0, nrows, partial); break;
        }
    }
}

// Static variant: block b folds range (b mod 8) of task (b div 8).  The dispatcher deals blocks
// round-robin over the XCDs, so the blocks of one range share an XCD (speed only; any placement gives
// the same result).  No queue atomics.
template <class Op, bool NT>
__global__ __launch_bounds__(kBlock) void pull_split_static_kernel(SplitArgs a, Op op,
                                                                   typename Op::T* __restrict__ partial) {
    using T = typename Op::T;
    __shared__ T red[kBlock / kWave];
    const int64_t b = blockIdx.x;
    const int qq = (int)(b & (kXcds - 1));
    const int64_t t = b >> 3;
    if (a.dbg && threadIdx.x == 0) atomicAdd(&a.dbg[xcc_id() * kXcds + qq], 1ull);
    const int64_t row0 = a.task_row[t];
    const int meta = a.task_meta[t];
    const int nrows = meta >> 8;
    switch (meta & 0xff) {
        case 0: split_hub_task<Op, NT>(a, op, qq, row0, partial, red); break;
        case 64: split_rows_task<Op, 64, NT>(a, op, qq, row0, nrows, partial); break;
        case 32: split_rows_task<Op, 32, NT>(a, op, qq, row0, nrows, partial); break;
        case 16: split_rows_task<Op, 16, NT>(a, op, qq, row0, nrows, partial); break;
        case 8: split_rows_task<Op, 8, NT>(a, op, qq, row0, nrows, partial); break;
        case 4: split_rows_task<Op, 4, NT>(a, op, qq, row0, nrows, partial); break;
        default: split_rows_task<Op, 2, NT>(a, op, qq, row0, nrows, partial); break;
    }
}

template <class Op>
__global__ void pull_split_finalize_kernel(int64_t rows, Op op, const typename Op::T* __restrict__ partial) {
    using T = typename Op::T;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
        T acc = partial[r];
#pragma unroll
        for (int q = 1; q < kXcds; ++q) acc = op.combine(acc, partial[(int64_t)q * rows + r]);
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
    const bool split = tune().pull_split && tune().pull_lds == 0 && plan.split_rows > 0 && split_partial != nullptr;
    PullArgs a = make_pull_args(csr, plan, split);
    const int64_t blocks = split ? plan.light_block_begin[kNumClasses] : plan.total_blocks();
    if (prof_ctx) prof_record_start(*prof_ctx, *prof_shard);
    if (split) {
        SplitArgs sa{csr.row_ptr.get(), csr.col.get(), plan.task_row.get(), plan.task_meta.get(),
                     plan.split_off.get(), plan.heads.get(), plan.split_tasks, plan.split_rows,
                     split_debug_counters()};
        if (tune().pull_split == 2) {  // static blockIdx -> range mapping
            const unsigned grid = (unsigned)(plan.split_tasks * kXcds);
            if (tune().pull_nt) pull_split_static_kernel<Op, true><<<grid, kBlock, 0, s>>>(sa, op, split_partial);
            else pull_split_static_kernel<Op, false><<<grid, kBlock, 0, s>>>(sa, op, split_partial);
        } else {  // per-XCD dynamic queues
            JG_HIP(hipMemsetAsync(plan.heads.get(), 0, kXcds * sizeof(unsigned long long), s));
            const unsigned grid = (unsigned)std::min<int64_t>(plan.split_tasks * kXcds, 256 * 8);
            if (tune().pull_nt) pull_split_kernel<Op, true><<<grid, kBlock, 0, s>>>(sa, op, split_partial);
            else pull_split_kernel<Op, false><<<grid, kBlock, 0, s>>>(sa, op, split_partial);
        }
        JG_LAUNCH_CHECK();
    }
    if (!split && tune().pull_lds > 0 && plan.lds_ok) {  // LDS-cached hot prefix (single shard)
        const int32_t hot = (int32_t)std::min<int64_t>(tune().pull_lds, kMaxLdsBytes / (int64_t)sizeof(T));
        if (plan.num_chunks > 0) {  // hub chunks keep the 256-thread kernel (block-wide reductions)
            if (tune().pull_nt) pull_kernel<Op, 4, true><<<(unsigned)plan.num_chunks, kBlock, 0, s>>>(a, op, hub_partial);
            else pull_kernel<Op, 4, false><<<(unsigned)plan.num_chunks, kBlock, 0, s>>>(a, op, hub_partial);
            JG_LAUNCH_CHECK();
        }
        const size_t bytes = (size_t)hot * sizeof(T);
        const unsigned grid = (unsigned)device_cu_count();
        if (tune().pull_nt) {
            static bool attr = false;
            if (!attr) {
                JG_HIP(hipFuncSetAttribute((const void*)pull_lds_kernel<Op, 4, true>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLdsBytes));
                attr = true;
            }
            pull_lds_kernel<Op, 4, true><<<grid, kLdsThreads, bytes, s>>>(a, op, hot);
        } else {
            static bool attr = false;
            if (!attr) {
                JG_HIP(hipFuncSetAttribute((const void*)pull_lds_kernel<Op, 4, false>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLdsBytes));
                attr = true;
            }
            pull_lds_kernel<Op, 4, false><<<grid, kLdsThreads, bytes, s>>>(a, op, hot);
        }
        JG_LAUNCH_CHECK();
        if (prof_ctx) prof_record_stop(*prof_ctx, *prof_shard);
        if (plan.num_hub_rows > 0) {
            pull_hub_finalize_kernel<Op><<<grid_for(plan.num_hub_rows), kBlock, 0, s>>>(a, op, hub_partial);
            JG_LAUNCH_CHECK();
        }
        return;
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
    if (pull_split_launches()) {  // diagnostic: one launch per degree class (per-class rocprof times)
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
        pull_split_finalize_kernel<Op><<<grid_for(plan.split_rows), kBlock, 0, s>>>(plan.split_rows, op, split_partial);
        JG_LAUNCH_CHECK();
    }
}

}  // namespace jg
