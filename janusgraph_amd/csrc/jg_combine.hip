// jg_combine.hip — combiner vertex programs: the DegreeCounter family.
//
// Reference (paths under /root/reference/janusgraph-test/src/main/java/org/janusgraph/olap/ and
// janusgraph-core/src/main/java/org/janusgraph/graphdb/olap/computer/):
//   OLAPTest.DegreeCounter (OLAPTest.java:424-503): superstep 0 sends 1 on Local.of(inE); superstep t
//   sets degree = sum of the received messages (reduce(0, +): 0 when nothing arrives) and, while
//   t < length, sends it on; terminates at iteration >= length.  Messages go along inE, so a vertex
//   receives from its out-neighbours: VertexMemoryHandler.receiveMessages pulls over the reverse of
//   the scope (VertexMemoryHandler.java:121-151), combined by the program's MessageCombiner
//   (VertexState.java:85-114).  Java int arithmetic: sums wrap modulo 2^32.
// So superstep t is x_t[v] = (+)_{w in N(v)} x_{t-1}[w] with N = the out-neighbours (one term per
// edge: multi-edges count, a self-loop once), x_0 = the initial message.  The same loop with a min or
// max combiner, or over IN / BOTH adjacency, is the generic semiring program behind
// jg_combine_steps.
//
// Kernels: the degree-class pull engine of PageRank and CC (jg_pull.h: lanes per row by degree
// class, chunked hubs) with a combiner Op over int64 values; the OUT adjacency gets its class plan
// on first use.  HBM-bound: 4 B column + 8 B gathered value per entry, 8 B row_ptr + 8 B write per
// row.
#include <climits>
#include <vector>

#include "jg_internal.h"
#include "jg_prim.h"
#include "jg_pull.h"

namespace jg {

namespace {

template <int OP>
struct Combine {
    __device__ static __forceinline__ int64_t identity() {
        return OP == JG_COMBINE_SUM ? 0 : OP == JG_COMBINE_MIN ? LLONG_MAX : LLONG_MIN;
    }
    __device__ static __forceinline__ int64_t apply(int64_t a, int64_t b) {
        if (OP == JG_COMBINE_SUM) return (int64_t)((uint64_t)a + (uint64_t)b);  // wrapping
        if (OP == JG_COMBINE_MIN) return b < a ? b : a;
        return b > a ? b : a;
    }
};

// Java Integer: the sum is taken modulo 2^32 (min/max of int32 inputs stay int32, and a row without
// entries keeps the identity)
template <int OP>
__device__ __forceinline__ int64_t finish(int64_t acc, int wrap32) {
    return (OP == JG_COMBINE_SUM && wrap32) ? (int64_t)(int32_t)(uint32_t)acc : acc;
}

template <int OP>
struct CombOp {
    using T = long long;
    const long long* __restrict__ x;  // previous superstep, gathered vector (compact or full length)
    long long* __restrict__ x_out;    // next superstep's gathered vector (owned slots written)
    VecPos pos;                       // owned row -> its slot
    int wrap32;
    __device__ __forceinline__ long long identity() const { return Combine<OP>::identity(); }
    __device__ __forceinline__ long long combine(long long a, long long b) const { return Combine<OP>::apply(a, b); }
    __device__ __forceinline__ long long gather(int32_t c) const { return x[c]; }
    __device__ __forceinline__ const long long* vec() const { return x; }
    __device__ __forceinline__ long long shfl_xor(long long v, int o) const { return __shfl_xor(v, o, kWave); }
    __device__ __forceinline__ long long shfl_up(long long v, int d) const { return __shfl_up(v, d, kWave); }
    __device__ __forceinline__ bool active(int64_t) const { return true; }
    __device__ __forceinline__ void finalize(int64_t row, long long acc) const {
        x_out[pos(row)] = finish<OP>(acc, wrap32);
    }
};

// received = the row has at least one entry (static over the supersteps)
__global__ void has_entries_kernel(const int64_t* __restrict__ row_ptr, int64_t rows, uint8_t* __restrict__ f) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x)
        f[r] = row_ptr[r + 1] > row_ptr[r];
}

// split_partial (nullable): the IN / BOTH plans' XCD-sliced merge bands, as PageRank and CC use them
template <int OP>
void launch_step(const Csr& c, const PullPlan& plan, long long* hub_partial, long long* split_partial,
                 const int64_t* x_in, int64_t* x_out, VecPos pos, int wrap32, hipStream_t s) {
    const CombOp<OP> op{reinterpret_cast<const long long*>(x_in), reinterpret_cast<long long*>(x_out), pos, wrap32};
    launch_pull(c, plan, op, hub_partial, s, nullptr, nullptr, split_partial);
}

}  // namespace

// Sharded graphs: the gathered vector is the adjacency's own layout: IN / BOTH use their halo plans
// (compact vectors, refreshed by the sparse halo exchange, or full length under "halo" = 0); OUT has
// no halo plan and its columns are global padded ids, so its vector is full length and refreshed by
// the dense allgather of the owned slices.
void combine_run(Graph& g, int direction, int combiner, int wrap32, const int64_t* init, int steps, int64_t* out,
                 uint8_t* received_out) {
    if (direction < JG_DIR_OUT || direction > JG_DIR_BOTH) fail(JG_ERR_ARG, "direction must be JG_DIR_OUT/IN/BOTH");
    if (combiner < JG_COMBINE_SUM || combiner > JG_COMBINE_MAX) fail(JG_ERR_ARG, "unknown combiner");
    if (steps < 0) fail(JG_ERR_ARG, "negative step count");
    const uint32_t adj = direction == JG_DIR_OUT ? JG_ADJ_OUT : direction == JG_DIR_IN ? JG_ADJ_IN : JG_ADJ_BOTH;
    if (!(g.flags & adj))
        fail(JG_ERR_UNSUPPORTED, std::string("graph was built without the ") +
                                     (direction == JG_DIR_OUT ? "OUT" : direction == JG_DIR_IN ? "IN" : "BOTH") +
                                     " adjacency");
    const size_t ns = g.shards.size();
    struct St {
        DevBuf<int64_t> x[2];
        DevBuf<uint8_t> recv;
        DevBuf<long long> hub_partial, split_partial;
        int64_t len = 0;
        VecPos pos;
    };
    std::vector<St> st(ns);
    for (size_t i = 0; i < ns; ++i) {
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        hipStream_t s = sh.stream;
        St& t = st[i];
        const Csr& c = adj == JG_ADJ_OUT ? sh.out : adj == JG_ADJ_IN ? sh.in : sh.both;
        if (adj == JG_ADJ_OUT) {
            t.len = g.padded_len();
            t.pos.base = (int64_t)sh.index * g.S;
            if (!sh.plan_out_built) {
                build_pull_plan(sh, sh.out, sh.plan_out, g.padded_len(), g.padded_len(), 8);
                sh.plan_out_built = true;
            }
        } else {
            t.len = g.vec_len(sh, adj);
            t.pos = g.vec_pos(sh, adj);
        }
        const PullPlan& plan = adj == JG_ADJ_OUT ? sh.plan_out : adj == JG_ADJ_IN ? sh.plan_in : sh.plan_both;
        const int64_t n = sh.rows;
        t.x[0].alloc(std::max<int64_t>(t.len, 1));
        t.x[1].alloc(std::max<int64_t>(t.len, 1));
        t.recv.alloc(std::max<int64_t>(n, 1));
        t.hub_partial.alloc(std::max<int64_t>(plan.num_chunks, 1));
        if (plan.split_rows > 0) t.split_partial.alloc(plan.split_partial_len());
        // owned rows' initial messages at their slots (vertex order: sh.dense_of_local)
        std::vector<int64_t> h(std::max<int64_t>(n, 1));
        for (int64_t l = 0; l < n; ++l) {
            const int64_t v = init ? init[sh.dense_of_local()[l]] : 1;
            h[l] = wrap32 ? (int64_t)(int32_t)v : v;
        }
        if (n) {
            copy_h2d(t.x[0].get() + t.pos.base, h.data(), n * sizeof(int64_t), s);
            has_entries_kernel<<<grid_for(n), kBlock, 0, s>>>(c.row_ptr.get(), n, t.recv.get());
            JG_LAUNCH_CHECK();
        }
    }
    auto exchange = [&](int which) {
        std::vector<void*> bufs;
        for (auto& t : st) bufs.push_back(t.x[which].peer());
        if (adj == JG_ADJ_OUT)
            exchange_allgather(g, bufs, sizeof(int64_t), ncclInt64);
        else
            exchange_vec(g, adj, bufs, sizeof(int64_t), ncclInt64);
    };
    Shard& sh0 = *g.shards[0];
    hipEvent_t t0, t1;
    {
        DeviceGuard dg(sh0.device);
        JG_HIP(hipEventCreate(&t0));
        JG_HIP(hipEventCreate(&t1));
        JG_HIP(hipEventRecord(t0, sh0.stream));
    }
    int cur = 0;
    for (int t = 0; t < steps; ++t) {
        exchange(cur);  // the senders' previous-superstep messages reach every reader
        for (size_t i = 0; i < ns; ++i) {
            Shard& sh = *g.shards[i];
            if (sh.rows == 0) continue;
            DeviceGuard dg(sh);
            St& s_ = st[i];
            const Csr& c = adj == JG_ADJ_OUT ? sh.out : adj == JG_ADJ_IN ? sh.in : sh.both;
            const PullPlan& plan = adj == JG_ADJ_OUT ? sh.plan_out : adj == JG_ADJ_IN ? sh.plan_in : sh.plan_both;
            const int64_t* xi = s_.x[cur].get();
            int64_t* xo = s_.x[cur ^ 1].get();
            if (combiner == JG_COMBINE_SUM)
                launch_step<JG_COMBINE_SUM>(c, plan, s_.hub_partial.get(), s_.split_partial.get(), xi, xo, s_.pos, wrap32,
                                            sh.stream);
            else if (combiner == JG_COMBINE_MIN)
                launch_step<JG_COMBINE_MIN>(c, plan, s_.hub_partial.get(), s_.split_partial.get(), xi, xo, s_.pos, wrap32,
                                            sh.stream);
            else
                launch_step<JG_COMBINE_MAX>(c, plan, s_.hub_partial.get(), s_.split_partial.get(), xi, xo, s_.pos, wrap32,
                                            sh.stream);
        }
        cur ^= 1;
    }
    float ms = 0;
    {
        DeviceGuard dg(sh0.device);
        JG_HIP(hipEventRecord(t1, sh0.stream));
        JG_HIP(hipEventSynchronize(t1));
        JG_HIP(hipEventElapsedTime(&ms, t0, t1));
        (void)hipEventDestroy(t0);
        (void)hipEventDestroy(t1);
    }
    Ctx& cx = *g.ctx;
    cx.last = jg_stats{};
    cx.last.supersteps = steps;
    cx.last.levels = steps;
    cx.last.compute_ms = ms;
    cx.last.kernel_ms_total = ms;
    cx.last.kernel_launches = steps;
    double nnz = 0, rows = 0;
    for (size_t i = 0; i < ns; ++i) {
        Shard& sh = *g.shards[i];
        const Csr& c = adj == JG_ADJ_OUT ? sh.out : adj == JG_ADJ_IN ? sh.in : sh.both;
        nnz += (double)c.nnz;
        rows += (double)sh.rows;
    }
    cx.last.algorithmic_bytes = (double)steps * (12.0 * nnz + 16.0 * rows);
    cx.last.edges_traversed = (double)steps * nnz;
    for (size_t i = 0; i < ns; ++i) {
        Shard& sh = *g.shards[i];
        const int64_t n = sh.rows;
        if (n == 0) continue;
        DeviceGuard dg(sh);
        St& t = st[i];
        std::vector<int64_t> h((size_t)n);
        copy_d2h(h.data(), t.x[cur].get() + t.pos.base, n * sizeof(int64_t), sh.stream);
        for (int64_t l = 0; l < n; ++l) out[sh.dense_of_local()[l]] = h[l];
        if (received_out) {
            std::vector<uint8_t> rc((size_t)n);
            copy_d2h(rc.data(), t.recv.get(), n, sh.stream);
            for (int64_t l = 0; l < n; ++l) received_out[sh.dense_of_local()[l]] = steps > 0 ? rc[l] : 0;
        }
    }
}

}  // namespace jg
