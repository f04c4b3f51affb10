// jg_prim.hip — device-wide scan and stable LSD radix sort for the CSR build (gfx950, wave64).
//
// Radix sort: 8-bit digits, tiles of 4096 keys per 256-thread workgroup (1024 keys per wave).
//   upsweep   per-tile digit histogram in LDS -> counts[digit][tile]
//   scan      exclusive scan of the digit-major count table -> global offset of (digit, tile)
//   downsweep each wave ranks its keys with the wave-ballot multisplit (8 ballots give the lanes
//             sharing a digit), a per-wave running base per digit in LDS keeps the order stable,
//             keys are written straight to their final slot.
#include "jg_prim.h"

namespace jg {
namespace prim {

namespace {

constexpr int kScanItems = 8;                          // elements per thread in scan kernels
constexpr int kScanTile = kBlock * kScanItems;         // 2048
constexpr int kRadixBits = 8;
constexpr int kRadixBins = 1 << kRadixBits;            // 256
constexpr int kRadixRounds = 16;                       // 64-key rounds per wave
constexpr int kRadixWaveKeys = kWave * kRadixRounds;   // 1024
constexpr int kRadixTile = kRadixWaveKeys * (kBlock / kWave);  // 4096

template <typename Tin>
__global__ __launch_bounds__(kBlock) void scan_reduce_kernel(const Tin* __restrict__ in, int64_t n,
                                                             int64_t* __restrict__ block_sums) {
    __shared__ int64_t scratch[kBlock / kWave];
    const int64_t base = (int64_t)blockIdx.x * kScanTile;
    int64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int64_t i = base + (int64_t)k * kBlock + threadIdx.x;
        if (i < n) s += (int64_t)in[i];
    }
    s = wave_reduce_add(s);
    if (lane_id() == 0) scratch[wave_id()] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t t = 0;
        for (int w = 0; w < kBlock / kWave; ++w) t += scratch[w];
        block_sums[blockIdx.x] = t;
    }
}

// Each thread owns kScanItems CONSECUTIVE elements (so the per-thread serial part keeps order).
template <typename Tin>
__global__ __launch_bounds__(kBlock) void scan_apply_kernel(const Tin* __restrict__ in, int64_t* __restrict__ out,
                                                            int64_t n, const int64_t* __restrict__ block_off) {
    __shared__ int64_t scratch[kBlock / kWave];
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
    int64_t v[kScanItems];
    int64_t local = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int64_t i = base + k;
        v[k] = i < n ? (int64_t)in[i] : 0;
        local += v[k];
    }
    int64_t total;
    int64_t pre = block_exclusive_scan_add(local, scratch, &total) + block_off[blockIdx.x];
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int64_t i = base + k;
        if (i < n) out[i] = pre;
        pre += v[k];
    }
    // the very last element writes the grand total at out[n]
    if (base <= n - 1 && n - 1 < base + kScanItems) out[n] = pre;
}

__global__ void scan_single_total_kernel(int64_t* out, int64_t n) {
    if (n == 0) out[0] = 0;
}

template <typename Tin>
void exclusive_scan_impl(const Tin* in, int64_t* out, int64_t n, hipStream_t s) {
    if (n <= 0) {
        scan_single_total_kernel<<<1, 1, 0, s>>>(out, 0);
        JG_LAUNCH_CHECK();
        return;
    }
    const int64_t nb = (n + kScanTile - 1) / kScanTile;
    DevBuf<int64_t> sums(nb), offs(nb + 1);
    scan_reduce_kernel<Tin><<<(unsigned)nb, kBlock, 0, s>>>(in, n, sums.get());
    JG_LAUNCH_CHECK();
    if (nb == 1) {
        JG_HIP(hipMemsetAsync(offs.get(), 0, sizeof(int64_t), s));
    } else {
        exclusive_scan_impl<int64_t>(sums.get(), offs.get(), nb, s);
    }
    scan_apply_kernel<Tin><<<(unsigned)nb, kBlock, 0, s>>>(in, out, n, offs.get());
    JG_LAUNCH_CHECK();
    JG_HIP(hipStreamSynchronize(s));  // temporaries are freed on return
}

// ------------------------------------------------------------------------------------------
// radix sort
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void radix_upsweep_kernel(const uint64_t* __restrict__ keys, int64_t n,
                                                               int shift, int64_t ntiles,
                                                               uint32_t* __restrict__ counts) {
    __shared__ uint32_t hist[kRadixBins];
    hist[threadIdx.x] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kRadixTile;
#pragma unroll 4
    for (int k = 0; k < kRadixTile / kBlock; ++k) {
        const int64_t i = base + (int64_t)k * kBlock + threadIdx.x;
        if (i < n) atomicAdd(&hist[(keys[i] >> shift) & (kRadixBins - 1)], 1u);
    }
    __syncthreads();
    counts[(int64_t)threadIdx.x * ntiles + blockIdx.x] = hist[threadIdx.x];
}

// Lanes of the calling wave whose digit equals this lane's digit (only lanes with `valid`).
__device__ __forceinline__ uint64_t match_digit(uint32_t digit, bool valid) {
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < kRadixBits; ++b) {
        const bool bit = (digit >> b) & 1u;
        const uint64_t ball = __ballot(bit);
        peers &= bit ? ball : ~ball;
    }
    return peers;
}

template <bool kVals>
__global__ __launch_bounds__(kBlock) void radix_downsweep_kernel(const uint64_t* __restrict__ keys_in,
                                                                 const uint32_t* __restrict__ vals_in,
                                                                 uint64_t* __restrict__ keys_out,
                                                                 uint32_t* __restrict__ vals_out, int64_t n,
                                                                 int shift, int64_t ntiles,
                                                                 const int64_t* __restrict__ offsets) {
    __shared__ int64_t base[kBlock / kWave][kRadixBins];
    __shared__ uint32_t cnt[kBlock / kWave][kRadixBins];
    const int w = wave_id(), l = lane_id();
    for (int i = threadIdx.x; i < (kBlock / kWave) * kRadixBins; i += kBlock) (&cnt[0][0])[i] = 0;
    __syncthreads();

    const int64_t wbase = (int64_t)blockIdx.x * kRadixTile + (int64_t)w * kRadixWaveKeys;
    uint64_t k[kRadixRounds];
    uint32_t v[kRadixRounds];
#pragma unroll
    for (int r = 0; r < kRadixRounds; ++r) {
        const int64_t i = wbase + r * kWave + l;
        k[r] = i < n ? keys_in[i] : 0;
        if constexpr (kVals) v[r] = i < n ? vals_in[i] : 0;
    }
    // per-wave digit histogram
#pragma unroll
    for (int r = 0; r < kRadixRounds; ++r) {
        const int64_t i = wbase + r * kWave + l;
        const bool valid = i < n;
        const uint32_t d = (uint32_t)(k[r] >> shift) & (kRadixBins - 1);
        const uint64_t peers = match_digit(d, valid);
        if (valid && (peers & lanemask_lt()) == 0) cnt[w][d] += (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    {   // digit d = threadIdx.x: bases of the 4 waves
        const int d = threadIdx.x;
        int64_t off = offsets[(int64_t)d * ntiles + blockIdx.x];
#pragma unroll
        for (int ww = 0; ww < kBlock / kWave; ++ww) {
            base[ww][d] = off;
            off += cnt[ww][d];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRadixRounds; ++r) {
        const int64_t i = wbase + r * kWave + l;
        const bool valid = i < n;
        const uint32_t d = (uint32_t)(k[r] >> shift) & (kRadixBins - 1);
        const uint64_t peers = match_digit(d, valid);
        const int64_t pos = base[w][d] + __popcll(peers & lanemask_lt());
        __builtin_amdgcn_wave_barrier();
        if (valid) {
            keys_out[pos] = k[r];
            if constexpr (kVals) vals_out[pos] = v[r];
            if ((peers & lanemask_lt()) == 0) base[w][d] += __popcll(peers);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

__global__ void flag_scan_kernel(const uint8_t* __restrict__ flags, int64_t n, int64_t* __restrict__ idx_out,
                                 const int64_t* __restrict__ pos) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (flags[i]) idx_out[pos[i]] = i;
}

__global__ void u8_to_u32_kernel(const uint8_t* __restrict__ f, uint32_t* __restrict__ o, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        o[i] = f[i] ? 1u : 0u;
}

// The same scan without a synchronisation: block sums and offsets of every level live in `scratch`.
template <typename Tin>
void exclusive_scan_async_impl(const Tin* in, int64_t* out, int64_t n, int64_t* scratch, hipStream_t s) {
    if (n <= 0) {
        scan_single_total_kernel<<<1, 1, 0, s>>>(out, 0);
        JG_LAUNCH_CHECK();
        return;
    }
    const int64_t nb = (n + kScanTile - 1) / kScanTile;
    int64_t *sums = scratch, *offs = scratch + nb;
    scan_reduce_kernel<Tin><<<(unsigned)nb, kBlock, 0, s>>>(in, n, sums);
    JG_LAUNCH_CHECK();
    if (nb == 1) {
        JG_HIP(hipMemsetAsync(offs, 0, sizeof(int64_t), s));
    } else {
        exclusive_scan_async_impl<int64_t>(sums, offs, nb, scratch + 2 * nb + 1, s);
    }
    scan_apply_kernel<Tin><<<(unsigned)nb, kBlock, 0, s>>>(in, out, n, offs);
    JG_LAUNCH_CHECK();
}

}  // namespace

int64_t scan_scratch_size(int64_t n) {
    if (n <= 0) return 1;
    const int64_t nb = (n + kScanTile - 1) / kScanTile;
    return 2 * nb + 1 + (nb > 1 ? scan_scratch_size(nb) : 0);
}
void exclusive_scan_async(const uint8_t* in, int64_t* out, int64_t n, int64_t* scratch, hipStream_t s) {
    exclusive_scan_async_impl(in, out, n, scratch, s);
}
void exclusive_scan_async(const uint32_t* in, int64_t* out, int64_t n, int64_t* scratch, hipStream_t s) {
    exclusive_scan_async_impl(in, out, n, scratch, s);
}

void exclusive_scan(const int32_t* in, int64_t* out, int64_t n, hipStream_t s) { exclusive_scan_impl(in, out, n, s); }
void exclusive_scan(const int64_t* in, int64_t* out, int64_t n, hipStream_t s) { exclusive_scan_impl(in, out, n, s); }
void exclusive_scan(const uint32_t* in, int64_t* out, int64_t n, hipStream_t s) { exclusive_scan_impl(in, out, n, s); }

void radix_sort(uint64_t* keys, uint32_t* vals, int64_t n, int bits, hipStream_t s) {
    if (n <= 1 || bits <= 0) return;
    const int64_t ntiles = (n + kRadixTile - 1) / kRadixTile;
    DevBuf<uint64_t> kalt(n);
    DevBuf<uint32_t> valt(vals ? n : 0);
    DevBuf<uint32_t> counts(ntiles * kRadixBins);
    DevBuf<int64_t> offsets(ntiles * kRadixBins + 1);
    uint64_t *kin = keys, *kout = kalt.get();
    uint32_t *vin = vals, *vout = vals ? valt.get() : nullptr;
    int passes = 0;
    for (int shift = 0; shift < bits; shift += kRadixBits, ++passes) {
        radix_upsweep_kernel<<<(unsigned)ntiles, kBlock, 0, s>>>(kin, n, shift, ntiles, counts.get());
        JG_LAUNCH_CHECK();
        exclusive_scan_impl<uint32_t>(counts.get(), offsets.get(), ntiles * kRadixBins, s);
        if (vals)
            radix_downsweep_kernel<true><<<(unsigned)ntiles, kBlock, 0, s>>>(kin, vin, kout, vout, n, shift, ntiles,
                                                                             offsets.get());
        else
            radix_downsweep_kernel<false><<<(unsigned)ntiles, kBlock, 0, s>>>(kin, nullptr, kout, nullptr, n, shift,
                                                                              ntiles, offsets.get());
        JG_LAUNCH_CHECK();
        std::swap(kin, kout);
        std::swap(vin, vout);
    }
    if (passes & 1) {  // result sits in the temporaries
        JG_HIP(hipMemcpyAsync(keys, kin, n * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
        if (vals) JG_HIP(hipMemcpyAsync(vals, vin, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    }
    JG_HIP(hipStreamSynchronize(s));
}

int64_t compact_indices(const uint8_t* flags, int64_t n, int64_t* idx_out, DevBuf<int64_t>& pos,
                        DevBuf<int64_t>& scan, hipStream_t s) {
    if (n <= 0) return 0;
    if ((int64_t)pos.size() < n + 1) pos.alloc(n + 1);
    if ((int64_t)scan.size() < scan_scratch_size(n)) scan.alloc(scan_scratch_size(n));
    exclusive_scan_async_impl<uint8_t>(flags, pos.get(), n, scan.get(), s);  // flags are 0 / 1
    flag_scan_kernel<<<grid_for(n), kBlock, 0, s>>>(flags, n, idx_out, pos.get());
    JG_LAUNCH_CHECK();
    int64_t total = 0;
    JG_HIP(hipMemcpyAsync(&total, pos.get() + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    JG_HIP(hipStreamSynchronize(s));
    return total;
}

int64_t compact_indices(const uint8_t* flags, int64_t n, int64_t* idx_out, hipStream_t s) {
    if (n <= 0) return 0;
    DevBuf<uint32_t> f32(n);
    DevBuf<int64_t> pos(n + 1);
    u8_to_u32_kernel<<<grid_for(n), kBlock, 0, s>>>(flags, f32.get(), n);
    JG_LAUNCH_CHECK();
    exclusive_scan_impl<uint32_t>(f32.get(), pos.get(), n, s);
    flag_scan_kernel<<<grid_for(n), kBlock, 0, s>>>(flags, n, idx_out, pos.get());
    JG_LAUNCH_CHECK();
    int64_t total = 0;
    JG_HIP(hipMemcpyAsync(&total, pos.get() + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    JG_HIP(hipStreamSynchronize(s));
    return total;
}

}  // namespace prim
}  // namespace jg
