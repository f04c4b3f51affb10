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
__global__ void vid_keys_kernel(const int64_t* __restrict__ vid, int64_t n, uint64_t* __restrict__ keys,
                                uint32_t* __restrict__ vals) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        keys[i] = (uint64_t)vid[i] ^ 0x8000000000000000ull;  // order-preserving for signed ids
        vals[i] = (uint32_t)i;
    }
}

__global__ void dup_check_kernel(const uint64_t* __restrict__ keys, int64_t n, int32_t* __restrict__ dup) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (keys[i] == keys[i - 1]) *dup = 1;
}

__device__ __forceinline__ int32_t lookup_dense(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                int64_t n, int64_t id) {
    const uint64_t k = (uint64_t)id ^ 0x8000000000000000ull;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (keys[mid] < k) lo = mid + 1; else hi = mid;
    }
    return (lo < n && keys[lo] == k) ? (int32_t)vals[lo] : -1;
}

__global__ void remap_kernel(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals, int64_t n,
                             const int64_t* __restrict__ s, const int64_t* __restrict__ d, int64_t m,
                             int32_t* __restrict__ ds, int32_t* __restrict__ dd) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        ds[e] = lookup_dense(keys, vals, n, s[e]);
        dd[e] = lookup_dense(keys, vals, n, d[e]);
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
    int sbits;  // 0, or kSliceBits: entries of a row grouped by XCD slice of their column (then by column)
    int smode;  // col_slice mode
};

__device__ __forceinline__ int emit_count(const SelectArgs& a, int64_t e) {
    const int32_t s = a.src[e], d = a.dst[e];
    if (s < 0 || d < 0) return 0;
    const int32_t gs = a.padded[s], gd = a.padded[d];
    const bool own_d = (gd / a.S) == a.r, own_s = (gs / a.S) == a.r;
    if (a.which == 0) return own_d;
    if (a.which == 1) return own_s;
    return (int)own_s + (int)own_d;
}

__global__ __launch_bounds__(kBlock) void select_count_kernel(SelectArgs a, int64_t* __restrict__ block_counts) {
    __shared__ int64_t scratch[kBlock / kWave];
    const int64_t base = (int64_t)blockIdx.x * kSelTile + (int64_t)threadIdx.x * kSelItems;
    int64_t c = 0;
#pragma unroll
    for (int k = 0; k < kSelItems; ++k)
        if (base + k < a.m) c += emit_count(a, base + k);
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
    const int64_t base = (int64_t)blockIdx.x * kSelTile + (int64_t)threadIdx.x * kSelItems;
    int64_t c = 0;
#pragma unroll
    for (int k = 0; k < kSelItems; ++k)
        if (base + k < a.m) c += emit_count(a, base + k);
    int64_t total;
    int64_t pos = block_exclusive_scan_add(c, scratch, &total) + block_off[blockIdx.x];
    for (int k = 0; k < kSelItems; ++k) {
        const int64_t e = base + k;
        if (e >= a.m) break;
        const int32_t s = a.src[e], d = a.dst[e];
        if (s < 0 || d < 0) continue;
        const int64_t gs = a.padded[s], gd = a.padded[d];
        const bool own_d = (gd / a.S) == a.r, own_s = (gs / a.S) == a.r;
        if ((a.which == 1 || a.which == 2) && own_s) {
            keys[pos] = ((uint64_t)(gs - (int64_t)a.r * a.S) << (a.cbits + a.sbits)) |
                        ((uint64_t)(a.sbits ? col_slice(gd, a.smode) : 0) << a.cbits) | (uint64_t)gd;
            if (eidx) eidx[pos] = (uint32_t)e;
            ++pos;
        }
        if ((a.which == 0 || a.which == 2) && own_d) {
            keys[pos] = ((uint64_t)(gd - (int64_t)a.r * a.S) << (a.cbits + a.sbits)) |
                        ((uint64_t)(a.sbits ? col_slice(gs, a.smode) : 0) << a.cbits) | (uint64_t)gs;
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

// first_below[c] = first row with degree < c_class_thr[c] (c = 1..6);
// first_below[kZeroClass] = 1 + last row with any entry (rows after it are all empty)
__global__ void class_bound_kernel(const int64_t* __restrict__ rp, int64_t rows,
                                   unsigned long long* __restrict__ first_below /* [kNumClasses] */,
                                   unsigned long long* __restrict__ last_nonempty, int64_t split_thr,
                                   unsigned long long* __restrict__ first_below_split) {
    for (int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; l < rows; l += (int64_t)gridDim.x * blockDim.x) {
        const int64_t d = rp[l + 1] - rp[l];
#pragma unroll
        for (int c = 1; c < kNumClasses - 2; ++c)
            if (d < c_class_thr[c]) atomicMin(&first_below[c], (unsigned long long)l);
        if (d > 0) atomicMax(last_nonempty, (unsigned long long)(l + 1));
        if (d < split_thr) atomicMin(first_below_split, (unsigned long long)l);
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
// split_off[r*8+q] = first entry of row r in XCD slice q, relative to row_ptr[r].  Entries of a row
// of a sliced CSR are ordered by (col_slice(col), col), so the slice is non-decreasing along the row.
__global__ void split_off_kernel(const int64_t* __restrict__ rp, const int32_t* __restrict__ col, int64_t heavy,
                                 int smode, uint32_t* __restrict__ split_off) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < heavy * kXcds;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / kXcds;
        const int q = (int)(i % kXcds);
        const int64_t b = rp[r], e = rp[r + 1];
        int64_t lo = b, hi = e;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (col_slice(col[mid], smode) < q) lo = mid + 1; else hi = mid;
        }
        split_off[i] = (uint32_t)(lo - b);
    }
}

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

void remap_ids_device(const int64_t* d_vid, int64_t n, const int64_t* d_src, const int64_t* d_dst, int64_t m,
                      int32_t* dsrc, int32_t* ddst, hipStream_t s) {
    DevBuf<uint64_t> keys(std::max<int64_t>(n, 1));
    DevBuf<uint32_t> vals(std::max<int64_t>(n, 1));
    DevBuf<int32_t> dup(1);
    JG_HIP(hipMemsetAsync(dup.get(), 0, sizeof(int32_t), s));
    if (n > 0) {
        vid_keys_kernel<<<grid_for(n), kBlock, 0, s>>>(d_vid, n, keys.get(), vals.get());
        JG_LAUNCH_CHECK();
        prim::radix_sort(keys.get(), vals.get(), n, 64, s);
        dup_check_kernel<<<grid_for(n), kBlock, 0, s>>>(keys.get(), n, dup.get());
        JG_LAUNCH_CHECK();
    }
    int32_t has_dup = 0;
    JG_HIP(hipMemcpyAsync(&has_dup, dup.get(), sizeof(int32_t), hipMemcpyDeviceToHost, s));
    JG_HIP(hipStreamSynchronize(s));
    if (has_dup) fail(JG_ERR_ARG, "duplicate vertex id in vid[]");
    if (m > 0) {
        remap_kernel<<<grid_for(m), kBlock, 0, s>>>(keys.get(), vals.get(), n, d_src, d_dst, m, dsrc, ddst);
        JG_LAUNCH_CHECK();
    }
    JG_HIP(hipStreamSynchronize(s));
}

static void build_csr(Shard& sh, const SelectArgs& a, const int32_t* weight, Csr& csr, hipStream_t s) {
    DevBuf<uint64_t> keys;
    DevBuf<uint32_t> eidx;
    const int64_t nnz = select_keys(a, keys, eidx, weight != nullptr, s);
    const int rbits = bits_for((uint64_t)std::max<int64_t>(sh.rows - 1, 0));
    prim::radix_sort(keys.get(), weight ? eidx.get() : nullptr, nnz, rbits + a.cbits + a.sbits, s);
    csr.rows = sh.rows;
    csr.nnz = nnz;
    csr.sliced = a.sbits != 0;
    csr.slice_mode = a.smode;
    csr.row_ptr.alloc(sh.rows + 1);
    csr.col.alloc(std::max<int64_t>(nnz, 1));
    if (weight) csr.weight.alloc(std::max<int64_t>(nnz, 1));
    fill_i64_kernel<<<grid_for(sh.rows + 1), kBlock, 0, s>>>(csr.row_ptr.get(), sh.rows + 1, nnz);
    JG_LAUNCH_CHECK();
    if (nnz > 0) {
        csr_from_sorted_kernel<<<grid_for(nnz), kBlock, 0, s>>>(keys.get(), nnz, a.cbits, a.cbits + a.sbits,
                                                                csr.row_ptr.get(),
                                                                csr.col.get(), weight ? eidx.get() : nullptr, weight,
                                                                weight ? csr.weight.get() : nullptr);
        JG_LAUNCH_CHECK();
    }
    JG_HIP(hipStreamSynchronize(s));
}

// Sub-row lengths in slice-major order: len[q * H + r] = entries of row r in slice q.
__global__ void slice_len_kernel(const int64_t* __restrict__ rp, const uint32_t* __restrict__ off, int64_t H,
                                 int32_t* __restrict__ len) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < H * kXcds; i += (int64_t)gridDim.x * blockDim.x) {
        const int q = (int)(i / H);
        const int64_t r = i % H;
        const int64_t b = off[r * kXcds + q];
        const int64_t e = q == kXcds - 1 ? rp[r + 1] - rp[r] : (int64_t)off[r * kXcds + q + 1];
        len[i] = (int32_t)(e - b);
    }
}

struct SliceBases {
    int64_t begin[kXcds];     // aligned first entry of each slice
    int64_t end[kXcds];       // end entry of each slice
    int64_t base[kXcds + 1];  // first task of each slice
};

// sp[q*(H+1) + r] = raw[q*H + r] - raw[q*H] + begin[q], r in [0, H] (raw[q*H + H] is slice q's end).
__global__ void slice_ptr_kernel(const int64_t* __restrict__ raw, int64_t H, SliceBases b, int64_t* __restrict__ sp) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (H + 1) * kXcds;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int q = (int)(i / (H + 1));
        const int64_t r = i % (H + 1);
        sp[i] = raw[(int64_t)q * H + r] - raw[(int64_t)q * H] + b.begin[q];
    }
}

// slice_col[sp[q][r] ...] = the slice-q entries of row r (one wave per sub-row).
__global__ void slice_copy_kernel(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                  const uint32_t* __restrict__ off, int64_t H, const int64_t* __restrict__ sp,
                                  int32_t* __restrict__ scol) {
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
    for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave; i < H * kXcds; i += waves) {
        const int q = (int)(i / H);
        const int64_t r = i % H;
        const int64_t src = rp[r] + off[r * kXcds + q];
        const int64_t* p = sp + (int64_t)q * (H + 1) + r;
        const int64_t dst = p[0], n = p[1] - p[0];
        for (int64_t k = lane_id(); k < n; k += kWave) scol[dst + k] = col[src + k];
    }
}

__global__ void nonempty_kernel(const int32_t* __restrict__ len, int64_t n, int32_t* __restrict__ flag) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        flag[i] = len[i] > 0;
}

// Number the non-empty sub-rows slice-major: sub_index[q*H + r] = k (or -1), cstart[k] = first entry.
__global__ void sub_number_kernel(const int32_t* __restrict__ len, const int64_t* __restrict__ num, int64_t H,
                                  const int64_t* __restrict__ sp, int32_t* __restrict__ sub_index,
                                  int64_t* __restrict__ cstart) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < H * kXcds; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t q = i / H, r = i % H;
        if (len[i] > 0) {
            sub_index[i] = (int32_t)num[i];
            cstart[num[i]] = sp[q * (H + 1) + r];
        } else {
            sub_index[i] = -1;
        }
    }
}

// Per task: j0 = the non-empty sub-row holding its first entry, carry = it started earlier, and
// heads[t][l] = row-start bits of lane l's kMergeEpl entries (bit 0 of lane 0 always set).
__global__ void task_meta_kernel(const int64_t* __restrict__ cstart, const int64_t* __restrict__ nzb, SliceBases b,
                                 int32_t* __restrict__ meta, uint8_t* __restrict__ heads) {
    constexpr int kEpl = kMergeTask / kWave;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < b.base[kXcds];
         t += (int64_t)gridDim.x * blockDim.x) {
        int q = 0;
        while (q < kXcds - 1 && t >= b.base[q + 1]) ++q;
        const int64_t e0 = b.begin[q] + (t - b.base[q]) * kMergeTask;
        const int64_t e1 = min(e0 + kMergeTask, b.end[q]);
        int64_t lo = nzb[q], hi = nzb[q + 1];  // first sub-row starting after e0
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (cstart[mid] <= e0) lo = mid + 1; else hi = mid;
        }
        const int64_t j0 = lo - 1;
        meta[2 * t] = (int32_t)j0;
        meta[2 * t + 1] = cstart[j0] < e0 ? 1 : 0;
        uint8_t h[kWave];
        for (int l = 0; l < kWave; ++l) h[l] = 0;
        h[0] = 1;
        for (int64_t j = j0 + 1; j < nzb[q + 1] && cstart[j] < e1; ++j) {
            const int pos = (int)(cstart[j] - e0);
            h[pos / kEpl] |= (uint8_t)(1u << (pos % kEpl));
        }
        for (int l = 0; l < kWave; ++l) heads[t * kWave + l] = h[l];
    }
}

// The sliced split of the heavy rows [0, H): slice-major sub-CSRs, each slice's start aligned to a
// merge task, so a task never spans two slices and its col loads are 16-byte aligned.
static void build_slice_plan(Shard& sh, const Csr& csr, PullPlan& plan, int64_t H) {
    hipStream_t s = sh.stream;
    plan.split_rows = plan.split_tasks = plan.split_subrows = 0;
    if (H <= 0) return;
    plan.split_rows = H;
    const int64_t NS = H * kXcds;
    DevBuf<uint32_t> off(NS);
    DevBuf<int32_t> len(NS);
    DevBuf<int64_t> raw(NS + 1);
    split_off_kernel<<<grid_for(NS), kBlock, 0, s>>>(csr.row_ptr.get(), csr.col.get(), H, csr.slice_mode, off.get());
    JG_LAUNCH_CHECK();
    slice_len_kernel<<<grid_for(NS), kBlock, 0, s>>>(csr.row_ptr.get(), off.get(), H, len.get());
    JG_LAUNCH_CHECK();
    prim::exclusive_scan(len.get(), raw.get(), NS, s);
    int64_t bounds[kXcds + 1];
    for (int q = 0; q <= kXcds; ++q) copy_d2h(&bounds[q], raw.get() + (int64_t)q * H, sizeof(int64_t), s);
    SliceBases b{};
    int64_t at = 0;
    b.base[0] = 0;
    for (int q = 0; q < kXcds; ++q) {
        const int64_t n = bounds[q + 1] - bounds[q];
        const int64_t tasks = (n + kMergeTask - 1) / kMergeTask;
        b.begin[q] = plan.slice_begin[q] = at;
        b.end[q] = plan.slice_end[q] = at + n;
        b.base[q + 1] = b.base[q] + tasks;
        at += tasks * kMergeTask;
    }
    for (int q = 0; q <= kXcds; ++q) plan.slice_task_base[q] = b.base[q];
    plan.split_tasks = b.base[kXcds];
    DevBuf<int64_t> sp((H + 1) * kXcds);
    slice_ptr_kernel<<<grid_for((H + 1) * kXcds), kBlock, 0, s>>>(raw.get(), H, b, sp.get());
    JG_LAUNCH_CHECK();
    plan.slice_col.alloc(at + kMergeTask);  // one task of padding: the last task's aligned loads
    JG_HIP(hipMemsetAsync(plan.slice_col.get(), 0, plan.slice_col.bytes(), s));
    slice_copy_kernel<<<grid_for(NS * kWave), kBlock, 0, s>>>(csr.row_ptr.get(), csr.col.get(), off.get(), H, sp.get(),
                                                              plan.slice_col.get());
    JG_LAUNCH_CHECK();
    // number the non-empty sub-rows
    DevBuf<int32_t> flag(NS);
    DevBuf<int64_t> num(NS + 1);
    nonempty_kernel<<<grid_for(NS), kBlock, 0, s>>>(len.get(), NS, flag.get());
    JG_LAUNCH_CHECK();
    prim::exclusive_scan(flag.get(), num.get(), NS, s);
    int64_t nzb[kXcds + 1];
    for (int q = 0; q <= kXcds; ++q) copy_d2h(&nzb[q], num.get() + (int64_t)q * H, sizeof(int64_t), s);
    plan.split_subrows = nzb[kXcds];
    DevBuf<int64_t> cstart(std::max<int64_t>(plan.split_subrows, 1)), d_nzb(kXcds + 1);
    copy_h2d(d_nzb.get(), nzb, sizeof nzb, s);
    plan.sub_index.alloc(NS);
    sub_number_kernel<<<grid_for(NS), kBlock, 0, s>>>(len.get(), num.get(), H, sp.get(), plan.sub_index.get(),
                                                      cstart.get());
    JG_LAUNCH_CHECK();
    plan.task_meta.alloc(std::max<int64_t>(2 * plan.split_tasks, 1));
    plan.task_heads.alloc(std::max<int64_t>(kWave * plan.split_tasks, 1));
    if (plan.split_tasks > 0) {
        task_meta_kernel<<<grid_for(plan.split_tasks, 64), 64, 0, s>>>(cstart.get(), d_nzb.get(), b, plan.task_meta.get(),
                                                                       plan.task_heads.get());
        JG_LAUNCH_CHECK();
    }
    JG_HIP(hipStreamSynchronize(s));
}

void build_pull_plan(Shard& sh, const Csr& csr, PullPlan& plan, int64_t col_space) {
    hipStream_t s = sh.stream;
    plan.lds_ok = col_space == csr.rows;  // one shard: the hot prefix of the gathered vector is [0, hot)
    plan.col_space = col_space;
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
    plan.num_chunks = (int64_t)crow.size();
    auto upload = [&](DevBuf<int64_t>& d, const std::vector<int64_t>& h) {
        d.alloc(std::max<size_t>(h.size(), 1));
        if (!h.empty()) copy_h2d(d.get(), h.data(), h.size() * sizeof(int64_t), s);
    };
    upload(plan.chunk_row, crow);
    upload(plan.chunk_begin, cbeg);
    upload(plan.chunk_end, cend);
    upload(plan.hub_chunk_ptr, hptr);
    // class boundaries: first row whose degree falls below each class threshold
    unsigned long long fb[kNumClasses + 2];
    for (int c = 0; c < kNumClasses; ++c) fb[c] = (unsigned long long)rows;
    fb[kNumClasses] = 0;                                 // 1 + last non-empty row
    fb[kNumClasses + 1] = (unsigned long long)rows;      // first row below the split threshold
    const int64_t split_thr = std::max<int64_t>(tune().split_min_degree, kXcds);
    if (rows > 0) {
        DevBuf<unsigned long long> d_fb(kNumClasses + 2);
        copy_h2d(d_fb.get(), fb, sizeof fb, s);
        class_bound_kernel<<<grid_for(rows), kBlock, 0, s>>>(csr.row_ptr.get(), rows, d_fb.get(),
                                                             d_fb.get() + kNumClasses, split_thr,
                                                             d_fb.get() + kNumClasses + 1);
        JG_LAUNCH_CHECK();
        copy_d2h(fb, d_fb.get(), sizeof fb, s);
    }
    // Classes are consecutive row ranges; any row may sit in a "wrong" lane class (only speed
    // changes), but the empty class starts strictly after the last non-empty row (correctness).
    const int64_t zero_begin = (int64_t)fb[kNumClasses];
    // the heavy prefix split by XCD slice: rows before the first row of degree < split_min_degree
    // (only on a sliced CSR, and only when the split is enabled at build time)
    const int64_t heavy = (tune().pull_split && csr.sliced && csr.slice_mode == 1)
                              ? std::min<int64_t>((int64_t)fb[kNumClasses + 1], zero_begin) : 0;
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
    build_slice_plan(sh, csr, plan, heavy);
    // light part: rows after the heavy prefix (hub rows are all heavy when rows are degree-sorted;
    // any hub beyond the prefix keeps its chunks, so chunks stay in the light table too)
    make_classes(plan.split_rows, plan.split_rows > 0 ? plan.num_chunks : plan.num_chunks, plan.light_row_begin,
                 plan.light_row_end, plan.light_block_begin);
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
    }
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
        DeviceGuard dg(sh.device);
        hipStream_t s = sh.stream;
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
        const int64_t maxdeg = mode == 0 ? (int64_t)hc[2] : mode == 1 ? (int64_t)(hc[2] + hc[3]) : (int64_t)hc[3];
        if (first) {
            g.info.num_vertices = n;
            g.info.num_edges = (int64_t)hc[0];
            g.info.ghost_edges = m - (int64_t)hc[0];
            g.info.self_loops = (int64_t)hc[1];
            g.info.max_in_degree = (int64_t)hc[2];
            g.info.max_out_degree = (int64_t)hc[3];
            g.info.truncated_vertices = (int64_t)hc[4];
        }
        // degree-sorted relabel
        DevBuf<uint64_t> rkeys(std::max<int64_t>(n, 1));
        DevBuf<int32_t> order(std::max<int64_t>(n, 1)), padded(std::max<int64_t>(n, 1));
        if (n > 0) {
            relabel_keys_kernel<<<grid_for(n), kBlock, 0, s>>>(indeg.get(), outdeg.get(), n, mode, maxdeg, vbits,
                                                               rkeys.get());
            JG_LAUNCH_CHECK();
            prim::radix_sort(rkeys.get(), nullptr, n, vbits + bits_for((uint64_t)maxdeg), s);
            padded_ids_kernel<<<grid_for(n), kBlock, 0, s>>>(rkeys.get(), n, (1ull << vbits) - 1ull, P, g.S,
                                                             order.get(), padded.get());
            JG_LAUNCH_CHECK();
        }
        const int r = sh.index;
        sh.rows = std::max<int64_t>(0, std::min<int64_t>(g.S, (n - r + P - 1) / P));
        // host copies: dense index of each owned row, padded id of every vertex (once)
        std::vector<int32_t> h_order(n);
        if (n) copy_d2h(h_order.data(), order.get(), n * sizeof(int32_t), s);
        sh.dense_of_local.resize(sh.rows);
        for (int64_t l = 0; l < sh.rows; ++l) sh.dense_of_local[l] = h_order[(size_t)(r + l * P)];
        if (first) {
            g.padded_of_dense.resize(n);
            for (int64_t k = 0; k < n; ++k) g.padded_of_dense[h_order[k]] = (k % P) * g.S + k / P;
        }
        sh.out_degree.alloc(std::max<int64_t>(sh.rows, 1));
        if (sh.rows > 0) {
            local_outdeg_kernel<<<grid_for(sh.rows), kBlock, 0, s>>>(order.get(), outdeg.get(), n, P, r, sh.rows,
                                                                     sh.out_degree.get());
            JG_LAUNCH_CHECK();
        }
        SelectArgs a{e.src[li], e.dst[li], padded.get(), m, g.S, r, 0, cbits, 0, tune().slice_mode};
        const int32_t* w = (e.weight.size() > li) ? e.weight[li] : nullptr;
        if (g.flags & JG_ADJ_IN) {
            a.which = 0;
            a.sbits = tune().pull_split ? kSliceBits : 0;  // PageRank's pull adjacency: XCD-sliced rows
            build_csr(sh, a, w, sh.in, s);
            a.sbits = 0;
            build_pull_plan(sh, sh.in, sh.plan_in, g.padded_len());
        }
        if (g.flags & JG_ADJ_OUT) {
            a.which = 1;
            build_csr(sh, a, w, sh.out, s);
        }
        if (g.flags & JG_ADJ_BOTH) {
            a.which = 2;
            build_csr(sh, a, nullptr, sh.both, s);
            build_pull_plan(sh, sh.both, sh.plan_both, g.padded_len());
        }
        JG_HIP(hipStreamSynchronize(s));
        first = false;
    }
    int64_t bytes = 0;
    for (auto& sp : g.shards) bytes += sp->in.bytes() + sp->out.bytes() + sp->both.bytes() + sp->out_degree.bytes();
    g.info.device_bytes = bytes;
    g.info.num_shards = P;
    g.info.flags = g.flags;
}

}  // namespace jg
