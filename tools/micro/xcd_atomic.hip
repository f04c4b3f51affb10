// Microbenchmark: band-0 sub-row partials of the sliced PageRank merge at RMAT-26 scale, written the
// current way (one fp64 per sub-row, consecutive slots per task: 1 GB) against accumulated with fp64
// atomics into one slot per (XCD, row) (64 MB, XCD-local lines, so the atomics resolve in that XCD's
// L2).  Also reads HW_REG_XCC_ID to check the workgroup -> XCD mapping.
// Build: hipcc -O3 --offload-arch=gfx950 xcd_atomic.hip -o xcd_atomic
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int kRowsPerTask = 85;      // ~512 entries / 6 per sub-row
constexpr long kRows = 1 << 20;       // band-0 rows
constexpr long kTasks = 1536 * 1024;  // ~780 M entries / 512
constexpr int kSlices = 128;

__device__ __forceinline__ int xcc_id() {
    return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15;  // HW_REG_XCC_ID, bits [3:0]
}

__global__ void store_kernel(double* __restrict__ part, long tasks) {
    const int lane = threadIdx.x & 63;
    const long w = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((long)gridDim.x * blockDim.x) >> 6;
    for (long t = w; t < tasks; t += nw) {
        for (int i = lane; i < kRowsPerTask; i += 64) part[t * kRowsPerTask + i] = (double)(t + i) * 1e-9;
    }
}

__global__ void atomic_kernel(double* __restrict__ slots, long tasks, unsigned* __restrict__ xcc_hist) {
    const int lane = threadIdx.x & 63;
    const int x = xcc_id();
    if (threadIdx.x == 0) atomicAdd(&xcc_hist[(blockIdx.x & 7) * 16 + x], 1u);
    const long w = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((long)gridDim.x * blockDim.x) >> 6;
    double* mine = slots + (long)x * kRows;
    for (long t = w; t < tasks; t += nw) {
        const long row0 = ((t / kSlices) * kRowsPerTask) % (kRows - kRowsPerTask);
        for (int i = lane; i < kRowsPerTask; i += 64) unsafeAtomicAdd(&mine[row0 + i], (double)(t + i) * 1e-9);
    }
}

__global__ void read_kernel(const double* __restrict__ a, long n, double* out) {
    double s = 0;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) s += a[i];
    if (s == 12345.0) out[0] = s;
}

int main() {
    double *part, *slots, *out;
    unsigned* hist;
    hipMalloc(&part, kTasks * kRowsPerTask * 8);
    hipMalloc(&slots, 16 * kRows * 8);
    hipMalloc(&out, 8);
    hipMalloc(&hist, 8 * 16 * 4);
    hipMemset(slots, 0, 16 * kRows * 8);
    hipMemset(hist, 0, 8 * 16 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timeit = [&](auto f) {
        f();
        hipDeviceSynchronize();
        float best = 1e9;
        for (int r = 0; r < 5; ++r) {
            hipEventRecord(a);
            f();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
        }
        return best;
    };
    const int grid = 256 * 8 * 4;
    float ts = timeit([&] { store_kernel<<<grid, 256>>>(part, kTasks); });
    float tr = timeit([&] { read_kernel<<<grid, 256>>>(part, kTasks * kRowsPerTask, out); });
    float ta = timeit([&] { atomic_kernel<<<grid, 256>>>(slots, kTasks, hist); });
    float tr2 = timeit([&] { read_kernel<<<grid, 256>>>(slots, 8 * kRows, out); });
    const double n = (double)kTasks * kRowsPerTask;
    printf("partials %.0f M: store %.3f ms (%.0f GB/s) + finalize read %.3f ms | xcd atomics %.3f ms (%.1f G/s) + read %.3f ms\n",
           n / 1e6, ts, n * 8 / ts / 1e6, tr, ta, n / ta / 1e6, tr2);
    std::vector<unsigned> h(128);
    hipMemcpy(h.data(), hist, 128 * 4, hipMemcpyDeviceToHost);
    printf("blockIdx%%8 -> xcc histogram (rows: blockIdx%%8, cols: xcc 0..7):\n");
    for (int r = 0; r < 8; ++r) {
        for (int c = 0; c < 8; ++c) printf(" %6u", h[r * 16 + c]);
        printf("\n");
    }
    return 0;
}
