// jg_pagerank.hip — JanusGraph PageRankVertexProgram as fp64 pull SpMV supersteps.
//
// Reference: janusgraph-backend-testutils/src/main/java/org/janusgraph/olap/PageRankVertexProgram.java
//   :90-91   superstep 0 sends 1.0 on inE        -> edgeCount = out-degree (both endpoints existing)
//   :92-97   superstep 1: rank = 1/N, send rank/edgeCount on outE
//   :99-103  superstep t>=2: rank = d * sum_{u->v} msg(u) + (1-d)/N, send rank/edgeCount
//   :107-110 terminate at iteration >= maxIterations (supersteps 0..K: K-1 power steps)
// Fulgora's gather is VertexMemoryHandler.receiveMessages (core/.../olap/computer/
// VertexMemoryHandler.java:121-151); pulling over the in-CSR is the same reverse-adjacency read.
//
// Per power superstep and shard: contrib_out[g] = rank/edgeCount for owned rows, gathered from the
// contrib_in at col[] (full length, or the shard's compact vector); then the exchange step
// (allgather or halo exchange, RCCL) refreshes every shard's copy.
// Algorithmic bytes per superstep: 12*m + 32*n.
#include <cstdlib>

#include "jg_pull.h"
#include "jg_scatter.h"

namespace jg {

namespace {

struct PrOp {
    using T = double;
    const double* __restrict__ x;      // contrib of the previous superstep, full length
    double* __restrict__ contrib_out;  // full length (owned slice written)
    double* __restrict__ rank;         // [rows]
    const int32_t* __restrict__ outdeg;
    VecPos pos;                        // owned row -> its slot in the gathered vector
    double damping, teleport;
    bool write_rank;                   // the rank vector is stored on the last superstep of a call only
    __device__ __forceinline__ double identity() const { return 0.0; }
    __device__ __forceinline__ double combine(double a, double b) const { return __dadd_rn(a, b); }
    __device__ __forceinline__ double gather(int32_t c) const { return x[c]; }
    __device__ __forceinline__ const double* vec() const { return x; }
    __device__ __forceinline__ double shfl_xor(double v, int o) const { return __shfl_xor(v, o, kWave); }
    __device__ __forceinline__ double shfl_up(double v, int d) const { return __shfl_up(v, d, kWave); }
    __device__ __forceinline__ bool active(int64_t) const { return true; }
    __device__ __forceinline__ void finalize(int64_t row, double s) const {
        // (dampingFactor * newPageRank) + ((1D - dampingFactor) / vertexCount), no contraction
        const double r = __dadd_rn(__dmul_rn(damping, s), teleport);
        if (write_rank) rank[row] = r;
        contrib_out[pos(row)] = r / (double)outdeg[row];
    }
};

// superstep 1: rank = 1/N, contrib = rank / edgeCount (edgeCount = out-degree as a double)
__global__ void pr_init_kernel(const int32_t* __restrict__ outdeg, int64_t rows, VecPos pos, double initial,
                               double* __restrict__ contrib, double* __restrict__ rank) {
    for (int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; l < rows; l += (int64_t)gridDim.x * blockDim.x) {
        rank[l] = initial;
        contrib[pos(l)] = initial / (double)outdeg[l];
    }
}

void exchange_contrib(Graph& g, int which) {
    std::vector<void*> bufs;
    for (auto& sp : g.shards) bufs.push_back(sp->pr_contrib[which].peer());
    exchange_vec(g, JG_ADJ_IN, bufs, sizeof(double), ncclFloat64);
}

}  // namespace

void pagerank_begin(Graph& g, double damping, int64_t vertex_count) {
    if (!(g.flags & JG_ADJ_IN)) fail(JG_ERR_UNSUPPORTED, "PageRank needs a graph built with JG_ADJ_IN");
    if (vertex_count == 0) fail(JG_ERR_ARG, "vertexCount must be non-zero");
    for (auto& sp : g.shards) {
        Shard& sh = *sp;
        DeviceGuard dg(sh);
        const int64_t len = g.vec_len(sh, JG_ADJ_IN);
        for (int k = 0; k < 2; ++k) {
            if (sh.pr_contrib[k].size() != (size_t)len) sh.pr_contrib[k].alloc(len);
            JG_HIP(hipMemsetAsync(sh.pr_contrib[k].get(), 0, sh.pr_contrib[k].bytes(), sh.stream));
        }
        if (sh.pr_rank.size() != (size_t)std::max<int64_t>(sh.rows, 1)) {
            // JG_VDEV_FAULT=1 (tests/test_gpu_vdev.py): the rank vector of shards > 0 allocated under the first
            // shard's guard, the misplacement the virtual-device check must report (ADVICE r03's bug class)
            const char* f = std::getenv("JG_VDEV_FAULT");
            if (f && *f && *f != '0' && sh.index > 0) {
                DeviceGuard d0(*g.shards[0]);
                sh.pr_rank.alloc(std::max<int64_t>(sh.rows, 1));
            } else {
                sh.pr_rank.alloc(std::max<int64_t>(sh.rows, 1));
            }
        }
        if (sh.pr_hub_partial.size() != (size_t)std::max<int64_t>(sh.plan_in.num_chunks, 1))
            sh.pr_hub_partial.alloc(std::max<int64_t>(sh.plan_in.num_chunks, 1));
        if (sh.pr_split_partial.size() != (size_t)sh.plan_in.split_partial_len()) {
            sh.pr_split_partial.alloc(sh.plan_in.split_partial_len());
        }
        const double initial = 1.0 / (double)vertex_count;
        if (sh.rows > 0) {
            pr_init_kernel<<<grid_for(sh.rows), kBlock, 0, sh.stream>>>(sh.out_degree.get(), sh.rows,
                                                                        g.vec_pos(sh, JG_ADJ_IN), initial,
                                                                        sh.pr_contrib[0].get(), sh.pr_rank.get());
            JG_LAUNCH_CHECK();
        }
    }
    exchange_contrib(g, 0);
    g.pr_cur = 0;
    g.pr_begun = true;
    g.pr_damping = damping;
    g.pr_vertex_count = vertex_count;
    g.pr_steps = 0;
}

void pagerank_steps(Graph& g, int nsteps) {
    if (!g.pr_begun) fail(JG_ERR_STATE, "jg_pagerank_step before jg_pagerank_begin");
    const double teleport = (1.0 - g.pr_damping) / (double)g.pr_vertex_count;
    Ctx* pc = g.ctx->profiling ? g.ctx : nullptr;
    // One shard: one event pair around all nsteps supersteps.  A timing event between supersteps
    // costs the stream ~10 us of idle plus a cold-L2 start of the next superstep (rocprofv3 kernel
    // trace, profiles/r01/rerun); with shards the pairs stay per superstep (the exchange sits between).
    Shard* whole = (pc && g.shards.size() == 1 && g.ctx->total_shards() == 1 && nsteps > 0) ? g.shards[0].get() : nullptr;
    if (whole) {
        DeviceGuard dg(whole->device);
        prof_record_start(*pc, *whole);
        pc = nullptr;
    }
    for (int t = 0; t < nsteps; ++t) {
        const int cur = g.pr_cur, nxt = cur ^ 1;
        for (auto& sp : g.shards) {
            Shard& sh = *sp;
            DeviceGuard dg(sh);
            PrOp op;
            op.x = sh.pr_contrib[cur].get();
            op.contrib_out = sh.pr_contrib[nxt].get();
            op.rank = sh.pr_rank.get();
            op.outdeg = sh.out_degree.get();
            op.pos = g.vec_pos(sh, JG_ADJ_IN);
            op.damping = g.pr_damping;
            op.teleport = teleport;
            // the rank property is read only after the call (jg_pagerank_end): earlier supersteps' ranks
            // are dead stores, except on steps 0 and 1, which also write the rows later steps skip
            op.write_rank = t == nsteps - 1 || g.pr_steps < 2;
            // Rows without in-edges: rank = (1-d)/N and contrib = rank/edgeCount from the first power step
            // on.  Steps 0 and 1 write that constant into both contrib buffers (step 0 must still gather
            // the initial values), later steps leave those rows alone.
            const bool skip_empty = g.pr_steps >= 2;
            launch_pull(sh.in, sh.plan_in, op, sh.pr_hub_partial.get(), sh.stream, pc, &sh, sh.pr_split_partial.get(),
                        skip_empty);
        }
        exchange_contrib(g, nxt);  // timed by the exchange itself (ExchTimer) when profiling
        g.pr_cur = nxt;
        ++g.pr_steps;
    }
    if (whole) {
        DeviceGuard dg(whole->device);
        prof_record_stop(*g.ctx, *whole, nsteps);
    }
}

void pagerank_end(Graph& g, double* rank_out, double* edge_count_out) {
    if (!g.pr_begun) fail(JG_ERR_STATE, "jg_pagerank_end before jg_pagerank_begin");
    for (auto& sp : g.shards) {
        Shard& sh = *sp;
        DeviceGuard dg(sh);
        JG_HIP(hipStreamSynchronize(sh.stream));
        if (sh.rows == 0) continue;
        if (rank_out) rows_to_dense(g, sh, sh.pr_rank.get(), rank_out);
        if (edge_count_out) rows_to_dense(g, sh, sh.out_degree.get(), edge_count_out);  // int32 -> double
    }
    prof_collect(*g.ctx, g);
}

}  // namespace jg
