// Microbenchmark: can scalar-path gathers add concurrency to the merge kernel's cold gathers?
// The merge kernel's cold (non-LDS) 8-byte gathers are bound by the vector memory path's requests in
// flight per CU (Little's law on L2 latency).  Scalar loads (uniform address, read
// through the scalar cache) have their own path to L2.  Each of 1024 threads per block (one block per
// CU, as the merge kernel) streams 8 int32 indices per iteration; an index >= 0 is a cold gather from its
// XCD's region of the table (block b gathers from region b mod 8), -1 is a hot entry (no load).
// Slots [0, SS) are gathered through scalar loads (a wave loops over its active lanes, four lanes
// per batch: readlane of the index, load, select into the lane), slots [SS, 8) through exec-masked
// vector loads.  Prints G gathers/s for SS = 0..8 at two cold fractions and two region sizes.
// Build: hipcc -O3 --offload-arch=gfx950 sgather.hip -o sgather
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 64;
constexpr int kThreads = 1024;

__global__ void gen_kernel(int32_t* idx, int64_t total, uint32_t region, uint32_t cold_per_65536, uint32_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
        h ^= h >> 31; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 29;
        const bool cold = (uint32_t)(h & 0xFFFF) < cold_per_65536;
        idx[i] = cold ? (int32_t)((h >> 20) % region) : -1;
    }
}

template <int SS>
__global__ __launch_bounds__(kThreads) void gather_kernel(const double* __restrict__ x, const int32_t* __restrict__ idx,
                                                          double* __restrict__ out, uint32_t region) {
    const int lane = threadIdx.x & 63;
    const int64_t tid = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const int64_t nthr = (int64_t)gridDim.x * kThreads;
    const double* __restrict__ xr = x + (int64_t)(blockIdx.x & 7) * region;
    double acc = 0;
    for (int it = 0; it < kIters; ++it) {
        int32_t c[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) c[u] = idx[((int64_t)it * 8 + u) * nthr + tid];
        double v[8];
#pragma unroll
        for (int u = SS; u < 8; ++u) {
            v[u] = 0;
            if (c[u] >= 0) v[u] = xr[c[u]];
        }
#pragma unroll
        for (int u = 0; u < SS; ++u) {
            v[u] = 0;
            uint64_t m = __ballot(c[u] >= 0);
            while (m) {
                int l[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    l[k] = m ? __builtin_ctzll(m) : l[0];
                    m &= m ? m - 1 : 0;
                }
                double s[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int32_t a = __builtin_amdgcn_readlane(c[u], l[k]);
                    s[k] = xr[a];
                }
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (lane == l[k]) v[u] = s[k];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    out[tid] = acc;
}

template <int SS>
float run(const double* x, const int32_t* idx, double* out, uint32_t region, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        gather_kernel<SS><<<blocks, kThreads>>>(x, idx, out, region);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    hipEventDestroy(a);
    hipEventDestroy(b);
    return best;
}

int main() {
    int dev_cus = 0;
    hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = dev_cus;
    const int64_t total = (int64_t)blocks * kThreads * kIters * 8;
    int32_t* idx;
    double* x;
    double* out;
    const uint32_t regions[2] = {1u << 19, 1u << 23};  // doubles per XCD: 4 MiB (L2), 64 MiB
    hipMalloc(&idx, total * 4);
    hipMalloc(&x, (size_t)8 * regions[1] * 8);
    hipMalloc(&out, (size_t)blocks * kThreads * 8);
    hipMemset(x, 0, (size_t)8 * regions[1] * 8);
    for (uint32_t region : regions) {
        for (uint32_t cold : {12452u /*0.19*/, 24248u /*0.37*/}) {
            gen_kernel<<<4096, 256>>>(idx, total, region, cold, 12345u);
            hipDeviceSynchronize();
            const double gathers = (double)total * cold / 65536.0;
            float t[9];
            t[0] = run<0>(x, idx, out, region, blocks);
            t[1] = run<1>(x, idx, out, region, blocks);
            t[2] = run<2>(x, idx, out, region, blocks);
            t[3] = run<3>(x, idx, out, region, blocks);
            t[4] = run<4>(x, idx, out, region, blocks);
            t[5] = run<5>(x, idx, out, region, blocks);
            t[6] = run<6>(x, idx, out, region, blocks);
            t[7] = run<7>(x, idx, out, region, blocks);
            t[8] = run<8>(x, idx, out, region, blocks);
            for (int s = 0; s <= 8; ++s)
                printf("{\"region_mib\": %u, \"cold\": %.3f, \"scalar_slots\": %d, \"ms\": %.4f, \"g_gathers_per_s\": %.1f}\n",
                       region * 8u >> 20, cold / 65536.0, s, t[s], gathers / (t[s] * 1e-3) * 1e-9);
        }
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        printf("error %s\n", hipGetErrorString(e));
        return 1;
    }
    return 0;
}
