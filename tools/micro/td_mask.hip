// Microbenchmark: cost of exec-masked 8-byte gathers on gfx950 (does a masked-off lane save TA/TD
// time?).  Each thread issues kIters rounds of 8 independent gathers from a 2 MiB table (L2-resident);
// a fraction `p` of lanes is active (lane-pattern masked, or a contiguous prefix of lanes).
// Prints ns per wave-instruction for p = 1, 1/2, 1/4, 1/8, 1/64 and for dense loads of the same
// count of active lanes.  Build: hipcc -O3 --offload-arch=gfx950 td_mask.hip -o td_mask
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int kIters = 64;
constexpr int kTable = 1 << 18;  // doubles (2 MiB)

__global__ void gather_kernel(const double* __restrict__ x, const int* __restrict__ idx, double* out, int active_mod,
                              int prefix) {
    const int lane = threadIdx.x & 63;
    const bool act = prefix ? lane < active_mod : (lane % active_mod) == 0;
    int base = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
    double acc = 0;
    for (int it = 0; it < kIters; ++it) {
        int c[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) c[u] = idx[(base + it * 8 + u) & (kTable - 1)];
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            v[u] = 0;
            if (act) v[u] = x[c[u]];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    std::vector<int> hidx(kTable);
    unsigned s = 1;
    for (auto& v : hidx) { s = s * 1664525u + 1013904223u; v = (int)(s >> 8) & (kTable - 1); }
    double* x; int* idx; double* out;
    hipMalloc(&x, kTable * 8); hipMalloc(&idx, kTable * 4);
    const int blocks = 256 * 8, threads = 256;
    hipMalloc(&out, blocks * threads * 8);
    hipMemset(x, 0, kTable * 8);
    hipMemcpy(idx, hidx.data(), kTable * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    struct Case { const char* name; int mod; int prefix; };
    Case cases[] = {{"all lanes", 1, 0}, {"1/2 lanes (every 2nd)", 2, 0}, {"1/4 (every 4th)", 4, 0},
                    {"1/8 (every 8th)", 8, 0}, {"1/64 (lane 0)", 64, 0}, {"prefix 32 lanes", 32, 1},
                    {"prefix 16 lanes", 16, 1}, {"prefix 8 lanes", 8, 1}};
    for (auto& c : cases) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            gather_kernel<<<blocks, threads>>>(x, idx, out, c.mod, c.prefix);
            hipEventRecord(b);
            hipEventSynchronize(b);
        }
        float ms; hipEventElapsedTime(&ms, a, b);
        const double instr = (double)blocks * threads / 64 * kIters * 8;  // gather wave-instructions
        printf("%-24s %.3f ms  %.2f ns per gather wave-instruction (chip)\n", c.name, ms, ms * 1e6 / instr);
    }
    return 0;
}
