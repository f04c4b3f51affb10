// jg_neighbors.hip — adjacency rows of the snapshot handed back in the caller's vertex order
// (jg_graph_neighbors).
//
// The reference rebuilds shortest paths from the preloaded BOTH slice of each vertex
// (VertexProgramScanJob.java:113-135 loads it for ShortestPathVertexProgram); the drop-in walks its
// paths back over the same adjacency, read from the device CSR instead of an OLTP transaction.
// A row is copied on the device (one block per row), then its column ids are mapped on the host:
// global padded ids (OUT, or unsharded pull adjacencies) through dense_of_local, compact halo ids
// (sharded IN / BOTH) through the owning peer's send list (segment s of shard r holds, in order, the
// rows peer p sends to r: jg_halo.hip).
#include "jg_internal.h"

namespace jg {
namespace {

__global__ void row_bounds_kernel(const int64_t* __restrict__ rp, const int64_t* __restrict__ rows, int64_t k,
                                  int64_t* __restrict__ len) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < k; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = rows[i];
        len[i] = rp[r + 1] - rp[r];
    }
}

// one block per requested row (grid-stride), coalesced copy of its entries to their packed slots
__global__ __launch_bounds__(kBlock) void gather_rows_kernel(const int64_t* __restrict__ rp,
                                                             const int32_t* __restrict__ col,
                                                             const int64_t* __restrict__ rows,
                                                             const int64_t* __restrict__ off, int64_t k,
                                                             int32_t* __restrict__ out) {
    for (int64_t i = blockIdx.x; i < k; i += gridDim.x) {
        const int64_t b = rp[rows[i]], o = off[i], len = off[i + 1] - o;
        for (int64_t j = threadIdx.x; j < len; j += kBlock) out[o + j] = col[b + j];
    }
}

const Csr& pick(const Shard& sh, int direction) {
    return direction == JG_DIR_BOTH ? sh.both : direction == JG_DIR_OUT ? sh.out : sh.in;
}

}  // namespace

void graph_neighbors(const Graph& g, int direction, const int64_t* rows, int64_t nrows, int64_t* off_out,
                     int64_t* nbr_out) {
    if (direction < JG_DIR_OUT || direction > JG_DIR_BOTH) fail(JG_ERR_ARG, "bad direction");
    if (nrows < 0 || (nrows > 0 && !rows) || !off_out) fail(JG_ERR_ARG, "bad arguments");
    // rank mode: only this process's rows are here; their entry counts can be read (the others count 0),
    // their neighbours cannot (a compact id maps back through a peer's send list)
    const bool all_local = (int)g.shards.size() == g.P;
    if (!all_local && nbr_out)
        fail(JG_ERR_UNSUPPORTED, "jg_graph_neighbors in rank mode: entry counts only (nbr_out must be NULL)");
    std::vector<const Shard*> local((size_t)g.P, nullptr);
    for (const auto& sp : g.shards) local[(size_t)sp->index] = sp.get();
    const uint32_t adj = direction == JG_DIR_BOTH ? JG_ADJ_BOTH : direction == JG_DIR_OUT ? JG_ADJ_OUT : JG_ADJ_IN;
    if (!(g.flags & adj)) fail(JG_ERR_UNSUPPORTED, "the graph was built without this adjacency");
    // rows grouped by owning shard, keeping their request position
    std::vector<std::vector<int64_t>> loc((size_t)g.P), pos((size_t)g.P);
    for (int64_t k = 0; k < nrows; ++k) {
        const int64_t d = rows[k];
        if (d < 0 || d >= g.n) fail(JG_ERR_ARG, "row outside [0, num_vertices)");
        const int64_t pg = g.padded_of_dense()[(size_t)d];
        const int q = (int)(pg / g.S);
        if (!local[q]) continue;  // another rank's row: no entries here
        loc[q].push_back(pg - (int64_t)q * g.S);
        pos[q].push_back(k);
    }
    std::vector<int64_t> len((size_t)nrows, 0);
    std::vector<std::vector<int32_t>> raw((size_t)g.P);
    std::vector<std::vector<int64_t>> roff((size_t)g.P);
    for (int q = 0; q < g.P; ++q) {
        const int64_t k = (int64_t)loc[q].size();
        if (!k) continue;
        const Shard& sh = *local[q];
        const Csr& c = pick(sh, direction);
        DeviceGuard dg(sh);
        DevBuf<int64_t> drows(k), dlen(k);
        copy_h2d(drows.get(), loc[q].data(), (size_t)k * sizeof(int64_t), sh.stream);
        row_bounds_kernel<<<grid_for(k), kBlock, 0, sh.stream>>>(c.row_ptr.get(), drows.get(), k, dlen.get());
        JG_LAUNCH_CHECK();
        std::vector<int64_t> l((size_t)k);
        copy_d2h(l.data(), dlen.get(), (size_t)k * sizeof(int64_t), sh.stream);
        roff[q].assign((size_t)k + 1, 0);
        for (int64_t i = 0; i < k; ++i) {
            len[(size_t)pos[q][i]] = l[i];
            roff[q][i + 1] = roff[q][i] + l[i];
        }
        if (!nbr_out || roff[q][k] == 0) continue;
        DevBuf<int64_t> doff(k + 1);
        DevBuf<int32_t> dout(roff[q][k]);
        copy_h2d(doff.get(), roff[q].data(), (size_t)(k + 1) * sizeof(int64_t), sh.stream);
        gather_rows_kernel<<<(unsigned)std::min<int64_t>(k, 65536), kBlock, 0, sh.stream>>>(
            c.row_ptr.get(), c.col.get(), drows.get(), doff.get(), k, dout.get());
        JG_LAUNCH_CHECK();
        raw[q].resize((size_t)roff[q][k]);
        copy_d2h(raw[q].data(), dout.get(), raw[q].size() * sizeof(int32_t), sh.stream);
    }
    off_out[0] = 0;
    for (int64_t k = 0; k < nrows; ++k) off_out[k + 1] = off_out[k] + len[(size_t)k];
    if (!nbr_out) return;
    // compact (halo) column ids need the peers' send lists on the host
    const bool compact = direction != JG_DIR_OUT && g.P > 1 && g.halo(*g.shards[0], adj).on;
    std::vector<std::vector<int32_t>> send((size_t)g.P);
    if (compact)
        for (int p = 0; p < g.P; ++p) {
            const Shard& sh = *g.shards[p];
            const Halo& h = g.halo(sh, adj);
            DeviceGuard dg(sh);
            send[p].resize((size_t)h.send_off[g.P]);
            if (!send[p].empty())
                copy_d2h(send[p].data(), h.send_src.get(), send[p].size() * sizeof(int32_t), sh.stream);
        }
    for (int q = 0; q < g.P; ++q) {
        const Halo& hq = g.halo(*g.shards[q], adj);
        const int64_t mask = (int64_t(1) << hq.tbits) - 1;
        for (size_t i = 0; i < loc[q].size(); ++i) {
            int64_t* o = nbr_out + off_out[pos[q][i]];
            for (int64_t j = roff[q][i]; j < roff[q][i + 1]; ++j) {
                const int64_t c = raw[q][(size_t)j];
                int p;
                int64_t l;
                if (compact) {
                    const int64_t seg = c >> hq.tbits, rk = c & mask;
                    if (seg == 0) {
                        p = q;
                        l = rk;
                    } else {
                        p = seg <= q ? (int)seg - 1 : (int)seg;  // inverse of s(p) = p < q ? p + 1 : p
                        l = send[p][(size_t)(g.halo(*g.shards[p], adj).send_off[q] + rk)];
                    }
                } else {
                    p = (int)(c / g.S);
                    l = c - (int64_t)p * g.S;
                }
                *o++ = g.shards[p]->dense_of_local()[(size_t)l];
            }
        }
    }
}

}  // namespace jg
