// jg_prim.h — device-wide primitives written for gfx950 (scan, stable LSD radix sort).
#pragma once

#include "jg_common.h"

namespace jg {

// ---- wave / block helpers (wave64, 256-thread blocks) ----
__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }
__device__ __forceinline__ uint64_t lanemask_lt() {
    const int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

template <typename T>
__device__ __forceinline__ T wave_inclusive_scan_add(T v) {
    const int l = lane_id();
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        T u = __shfl_up(v, o, kWave);
        if (l >= o) v += u;
    }
    return v;
}

template <typename T>
__device__ __forceinline__ T wave_reduce_add(T v) {
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

template <typename T>
__device__ __forceinline__ T wave_reduce_min(T v) {
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        const T u = __shfl_xor(v, o, kWave);
        v = u < v ? u : v;
    }
    return v;
}

template <typename T>
__device__ __forceinline__ T wave_reduce_max(T v) {
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        const T u = __shfl_xor(v, o, kWave);
        v = u > v ? u : v;
    }
    return v;
}

// Exclusive scan across a 256-thread block. `scratch` holds >= 4 elements. Returns the exclusive
// prefix of the calling thread; *total receives the block sum.
template <typename T>
__device__ __forceinline__ T block_exclusive_scan_add(T v, T* scratch, T* total) {
    T inc = wave_inclusive_scan_add(v);
    if (lane_id() == kWave - 1) scratch[wave_id()] = inc;
    __syncthreads();
    T wave_off = 0, sum = 0;
#pragma unroll
    for (int w = 0; w < kBlock / kWave; ++w) {
        T s = scratch[w];
        if (w < wave_id()) wave_off += s;
        sum += s;
    }
    __syncthreads();
    *total = sum;
    return wave_off + inc - v;
}

namespace prim {

// out[0..n] = exclusive scan of in[0..n) with out[n] = total.  in/out must not alias.
void exclusive_scan(const int32_t* in, int64_t* out, int64_t n, hipStream_t s);
void exclusive_scan(const int64_t* in, int64_t* out, int64_t n, hipStream_t s);
void exclusive_scan(const uint32_t* in, int64_t* out, int64_t n, hipStream_t s);
// The same, queued on s without synchronising: scratch holds scan_scratch_size(n) elements and must
// outlive the stream's work.
int64_t scan_scratch_size(int64_t n);
void exclusive_scan_async(const uint8_t* in, int64_t* out, int64_t n, int64_t* scratch, hipStream_t s);
void exclusive_scan_async(const uint32_t* in, int64_t* out, int64_t n, int64_t* scratch, hipStream_t s);

// Stable LSD radix sort of keys[0..n) on bits [0, bits), carrying vals (nullable).  Sorted data is
// returned in keys/vals (temporaries are allocated internally).
void radix_sort(uint64_t* keys, uint32_t* vals, int64_t n, int bits, hipStream_t s);

// Count elements of flags[0..n) that are nonzero, and write their indices (stable) into idx_out.
// Returns the count (synchronises the stream).
int64_t compact_indices(const uint8_t* flags, int64_t n, int64_t* idx_out, hipStream_t s);
// The same with reusable scratch (grown on demand, no allocation after that); flags must be 0 or 1.
int64_t compact_indices(const uint8_t* flags, int64_t n, int64_t* idx_out, DevBuf<int64_t>& pos,
                        DevBuf<int64_t>& scan, hipStream_t s);

}  // namespace prim
}  // namespace jg
