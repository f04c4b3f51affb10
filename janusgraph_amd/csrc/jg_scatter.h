// jg_scatter.h — per-row results back into the caller's vertex order.
//
// Rows are relabelled by degree, so row l of a shard is caller vertex dense_of_local[l].  One shard
// holding every vertex permutes on the device (a scatter into a dense-order buffer, then one
// contiguous copy): a host loop of n random writes costs ~0.1 s at 2^24 vertices and more at 2^26.
// Sharded graphs scatter each shard's rows on the host.
#pragma once

#include <vector>

#include "jg_internal.h"

namespace jg {

template <class Td, class Th>
__global__ void rows_to_dense_kernel(const Td* __restrict__ in, const int32_t* __restrict__ dense, int64_t rows,
                                     Th* __restrict__ out) {
    for (int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; l < rows; l += (int64_t)gridDim.x * blockDim.x)
        out[dense[l]] = (Th)in[l];
}

// out[dense_of_local[l]] = (Th)dev[l] for the shard's rows (dev on the shard's device)
template <class Td, class Th>
void rows_to_dense(const Graph& g, Shard& sh, const Td* dev, Th* out) {
    if (sh.rows == 0) return;
    DeviceGuard dg(sh);
    if (g.shards.size() == 1 && sh.rows == g.n && sh.dense_rows.size() >= (size_t)sh.rows) {
        DevBuf<Th> tmp(sh.rows);
        rows_to_dense_kernel<Td, Th><<<grid_for(sh.rows), kBlock, 0, sh.stream>>>(dev, sh.dense_rows.get(), sh.rows,
                                                                                  tmp.get());
        JG_LAUNCH_CHECK();
        copy_d2h(out, tmp.get(), (size_t)sh.rows * sizeof(Th), sh.stream);
        return;
    }
    std::vector<Td> h((size_t)sh.rows);
    copy_d2h(h.data(), dev, (size_t)sh.rows * sizeof(Td), sh.stream);
    for (int64_t l = 0; l < sh.rows; ++l) out[sh.dense_of_local()[l]] = (Th)h[l];
}

}  // namespace jg
