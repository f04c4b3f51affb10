// jg_halo.hip — compact gathered vectors and the sparse halo exchange of sharded graphs.
//
// FulgoraGraphComputer has no shards: every vertex's messages sit in one JVM heap
// (core/.../olap/computer/FulgoraVertexMemory.java:52-123) and the superstep reads them in place.
// Sharded across GPUs (BASELINE north star: 1D vertex partition, exchange over xGMI), a shard's
// rows read the previous superstep's values of their in-neighbours (VertexMemoryHandler.java:
// 121-151).  A dense allgather ships every vertex's value to every shard; for RMAT at P = 8 a shard
// reads only ~23% of the remote values (most vertices have few out-neighbours, so they reach few
// shards).  The halo plan ships just those, by static per-peer lists built once from the edge list:
//   build: mark needed columns (bitmaps), number them segment by segment (the compact ids the CSR
//          holds: own rows, then per peer the vertices read, in the peer's order), extract the
//          per-peer send lists;
//   superstep: pack own values into per-peer runs -> RCCL send/recv (device copies for logical
//          shards of one device) straight into the receiving shard's segment for that peer.
#include <algorithm>
#include <cstdio>

#include "jg_internal.h"
#include "jg_prim.h"

namespace jg {

namespace {

__device__ __forceinline__ void set_bit(uint32_t* bits, int64_t i) { atomicOr(bits + (i >> 5), 1u << (i & 31)); }

// Entry (row, col) of shard r's pull adjacency, both global padded ids:
//   row owned by r, col remote -> r reads col:  need[col]
//   col owned by r, row remote -> shard row/S reads col: send[(row/S) * S + col % S]
struct MarkArgs {
    const int32_t* src;
    const int32_t* dst;
    const int32_t* padded;
    int64_t m, S;
    int r, which;
    uint32_t *need, *send;
};

__device__ __forceinline__ void mark_entry(const MarkArgs& a, int64_t row, int64_t col) {
    const int64_t rq = row / a.S, cq = col / a.S;
    if (rq == a.r && cq != a.r)
        set_bit(a.need, col);
    else if (cq == a.r && rq != a.r)
        set_bit(a.send, rq * a.S + (col - cq * a.S));
}

__global__ void halo_mark_kernel(MarkArgs a) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < a.m; e += (int64_t)gridDim.x * blockDim.x) {
        const int32_t s = a.src[e], d = a.dst[e];
        if (s < 0 || d < 0) continue;
        const int64_t gs = a.padded[s], gd = a.padded[d];
        mark_entry(a, gd, gs);                    // IN: row = target, col = source
        if (a.which == 2) mark_entry(a, gs, gd);  // BOTH: and the reverse entry
    }
}

__global__ void popc_words_kernel(const uint32_t* __restrict__ bits, int64_t words, uint32_t* __restrict__ cnt) {
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words; w += (int64_t)gridDim.x * blockDim.x)
        cnt[w] = (uint32_t)__popc(bits[w]);
}

// sorted list of the set bit indices of a bitmap (off = exclusive popcount prefix of its words)
__global__ void bits_to_list_kernel(const uint32_t* __restrict__ bits, const int64_t* __restrict__ off, int64_t words,
                                    int32_t* __restrict__ list) {
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words; w += (int64_t)gridDim.x * blockDim.x) {
        uint32_t x = bits[w];
        int64_t p = off[w];
        while (x) {
            const int b = __ffs(x) - 1;
            list[p++] = (int32_t)(w * 32 + b);
            x &= x - 1u;
        }
    }
}

// qbase[q] = set bits of the bitmap below bit q * S (q = 0..P)
__global__ void peer_base_kernel(const uint32_t* __restrict__ bits, const int64_t* __restrict__ off, int64_t S, int P,
                                 int64_t* __restrict__ qbase) {
    const int q = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (q > P) return;
    const int64_t i = (int64_t)q * S;
    qbase[q] = off[i >> 5] + ((i & 31) ? __popc(bits[i >> 5] & ((1u << (i & 31)) - 1u)) : 0);
}

// send list entries q * S + l -> own row l
__global__ void list_local_kernel(int32_t* __restrict__ list, int64_t n, int64_t S) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        list[i] = (int32_t)(list[i] % S);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void halo_pack_kernel(const T* __restrict__ vec, const int32_t* __restrict__ src,
                                                           int64_t n, T* __restrict__ out) {
    // four gathers in flight per thread and trip (one per trip left the pack latency-bound: ~60 us for
    // 14.7 M words at RMAT-26, P = 8)
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        int32_t s[4];
        T v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) s[k] = src[i + k * stride];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = vec[s[k]];
#pragma unroll
        for (int k = 0; k < 4; ++k) out[i + k * stride] = v[k];
    }
    for (; i < n; i += stride) out[i] = vec[src[i]];
}

// Exclusive popcount prefix (words + 1 entries) and per-peer bases of a peer-major bitmap over
// [0, P*S); returns the per-peer counts' offsets on the host.
void peer_prefix(const uint32_t* bits, int64_t words, int64_t S, int P, DevBuf<int64_t>& off, DevBuf<int64_t>& qbase,
                 std::vector<int64_t>& peer_off, hipStream_t s) {
    DevBuf<uint32_t> cnt(std::max<int64_t>(words, 1));
    off.alloc(words + 1);
    if (words > 0) {
        popc_words_kernel<<<grid_for(words), kBlock, 0, s>>>(bits, words, cnt.get());
        JG_LAUNCH_CHECK();
    }
    prim::exclusive_scan(cnt.get(), off.get(), words, s);
    qbase.alloc(P + 1);
    peer_base_kernel<<<1, 256, 0, s>>>(bits, off.get(), S, P, qbase.get());
    JG_LAUNCH_CHECK();
    peer_off.assign(P + 1, 0);
    copy_d2h(peer_off.data(), qbase.get(), (P + 1) * sizeof(int64_t), s);
}

}  // namespace

void build_halo(Graph& g, Shard& sh, const int32_t* src, const int32_t* dst, const int32_t* padded, int64_t m,
                int which, Halo& h, hipStream_t s) {
    const int P = g.P, r = sh.index;
    const int64_t S = g.S, N = (int64_t)P * S, words = (N + 31) / 32;
    DevBuf<uint32_t> send(std::max<int64_t>(words, 1));
    h.bits.alloc(std::max<int64_t>(words, 1));
    JG_HIP(hipMemsetAsync(h.bits.get(), 0, h.bits.bytes(), s));
    JG_HIP(hipMemsetAsync(send.get(), 0, send.bytes(), s));
    MarkArgs a{src, dst, padded, m, S, r, which, h.bits.get(), send.get()};
    if (m > 0) {
        halo_mark_kernel<<<grid_for(m, kBlock, 256 * 16), kBlock, 0, s>>>(a);
        JG_LAUNCH_CHECK();
    }
    // recv side: counts per peer; segment stride T covers the own rows and every peer's run, and is a
    // multiple of the 4096-entry line groups of the sub-slice hash (any band width)
    peer_prefix(h.bits.get(), words, S, P, h.off, h.qbase, h.recv_off, s);
    int64_t seg = std::max<int64_t>(sh.rows, 8192);
    for (int q = 0; q < P; ++q) seg = std::max(seg, h.recv_off[q + 1] - h.recv_off[q]);
    h.tbits = 13;
    while ((1ll << h.tbits) < seg) ++h.tbits;
    h.C = (int64_t)P << h.tbits;
    if (h.C >= (int64_t)INT32_MAX) fail(JG_ERR_UNSUPPORTED, "sharded vector segments exceed int32 ids");
    h.on = true;
    // send side: own rows each peer reads, by peer, ascending
    DevBuf<int64_t> soff, sbase;
    peer_prefix(send.get(), words, S, P, soff, sbase, h.send_off, s);
    const int64_t ns = h.send_off[P];
    h.send_src.alloc(std::max<int64_t>(ns, 1));
    if (words > 0) {
        bits_to_list_kernel<<<grid_for(words), kBlock, 0, s>>>(send.get(), soff.get(), words, h.send_src.get());
        JG_LAUNCH_CHECK();
    }
    if (ns > 0) {
        list_local_kernel<<<grid_for(ns), kBlock, 0, s>>>(h.send_src.get(), ns, S);
        JG_LAUNCH_CHECK();
    }
    h.send_buf.alloc(std::max<int64_t>(ns, 1));
    JG_HIP(hipStreamSynchronize(s));
    if (debug_plan())
        std::fprintf(stderr, "[jg] halo shard %d adj %d: segments %d x 2^%d (own %lld) recv %lld send %lld of dense %lld\n",
                     r, which, P, h.tbits, (long long)sh.rows, (long long)h.recv_off[P], (long long)ns,
                     (long long)(N - S));
}

void release_halo_maps(Halo& h) {
    h.bits.reset();
    h.off.reset();
    h.qbase.reset();
}

void check_halo_counts(Graph& g, uint32_t adj) {
    const int P = g.P;
    Ctx& c = *g.ctx;
    // counts[q][p] = elements shard q sends to p, gathered from every shard
    std::vector<int64_t> counts((size_t)P * P, -1);
    if (c.nranks == 1) {
        for (auto& sp : g.shards) {
            const Halo& h = g.halo(*sp, adj);
            for (int p = 0; p < P; ++p) counts[(size_t)sp->index * P + p] = h.send_off[p + 1] - h.send_off[p];
        }
    } else {
        Shard& sh0 = *g.shards[0];
        DeviceGuard dg(sh0.device);
        const size_t per = (size_t)P * g.shards.size();
        std::vector<int64_t> mine(per);
        for (size_t i = 0; i < g.shards.size(); ++i) {
            const Halo& h = g.halo(*g.shards[i], adj);
            for (int p = 0; p < P; ++p) mine[i * P + p] = h.send_off[p + 1] - h.send_off[p];
        }
        if (c.host_transport) {
            host_allgather(c, mine.data(), counts.data(), per * sizeof(int64_t));
        } else {
        DevBuf<int64_t> d(per * c.nranks);
        copy_h2d(d.get() + (size_t)c.rank * per, mine.data(), per * sizeof(int64_t), sh0.stream);
        rccl_check(ncclAllGather(d.get() + (size_t)c.rank * per, d.get(), per, ncclInt64, sh0.comm, sh0.stream),
                   "ncclAllGather(halo counts)");
        copy_d2h(counts.data(), d.get(), counts.size() * sizeof(int64_t), sh0.stream);
        }
    }
    for (auto& sp : g.shards) {
        const Halo& h = g.halo(*sp, adj);
        for (int q = 0; q < P; ++q) {
            const int64_t want = h.recv_off[q + 1] - h.recv_off[q];
            const int64_t got = counts[(size_t)q * P + sp->index];
            if (want != got)
                fail(JG_ERR_RCCL, "halo plan mismatch: shard " + std::to_string(sp->index) + " expects " +
                                          std::to_string(want) + " values from shard " + std::to_string(q) +
                                          ", which sends " + std::to_string(got));
        }
    }
}

void exchange_halo(Graph& g, uint32_t adj, std::vector<void*>& bufs, size_t elem_bytes, ncclDataType_t type) {
    ExchTimer et(g);
    if (elem_bytes != 4 && elem_bytes != 8) fail(JG_ERR_UNSUPPORTED, "halo exchange of unsupported element size");
    Ctx& c = *g.ctx;
    for (size_t i = 0; i < g.shards.size(); ++i) {  // pack the runs of own values each peer reads
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        const Halo& h = g.halo(sh, adj);
        const int64_t n = h.send_off[g.P];
        if (n == 0) continue;
        if (elem_bytes == 8)
            halo_pack_kernel<uint64_t><<<grid_for(n), kBlock, 0, sh.stream>>>(
                static_cast<const uint64_t*>(bufs[i]), h.send_src.get(), n, h.send_buf.get());
        else
            halo_pack_kernel<uint32_t><<<grid_for(n), kBlock, 0, sh.stream>>>(
                static_cast<const uint32_t*>(bufs[i]), h.send_src.get(), n,
                reinterpret_cast<uint32_t*>(h.send_buf.get()));
        JG_LAUNCH_CHECK();
    }
    // receiving shard r takes peer q's run at its segment seg_of(q, r)
    auto seg_ptr = [&](size_t i, int q) {
        const Shard& sh = *g.shards[i];
        const Halo& h = g.halo(sh, adj);
        return static_cast<char*>(bufs[i]) + ((size_t)h.seg_of(q, sh.index) << h.tbits) * elem_bytes;
    };
    if (c.logical) {  // every shard on one device and stream: copy each run directly
        Shard& s0 = *g.shards[0];
        DeviceGuard dg(s0.device);
        for (size_t di = 0; di < g.shards.size(); ++di) {
            const Halo& hd = g.halo(*g.shards[di], adj);
            for (size_t si = 0; si < g.shards.size(); ++si) {
                if (si == di) continue;
                const Halo& hs = g.halo(*g.shards[si], adj);
                const int q = g.shards[si]->index, r = g.shards[di]->index;
                const int64_t n = hd.recv_off[q + 1] - hd.recv_off[q];
                if (n == 0) continue;
                JG_HIP(hipMemcpyAsync(seg_ptr(di, q),
                                      reinterpret_cast<const char*>(hs.send_buf.peer()) + hs.send_off[r] * elem_bytes,
                                      n * elem_bytes, hipMemcpyDeviceToDevice, s0.stream));
            }
        }
        return;
    }
    if (c.host_transport) {  // rank mode over host callbacks (one shard per process): staged runs
        Shard& sh = *g.shards[0];
        const Halo& h = g.halo(sh, adj);
        DeviceGuard dg(sh);
        std::vector<char> sbuf((size_t)h.send_off[g.P] * elem_bytes);
        copy_d2h(sbuf.data(), h.send_buf.get(), sbuf.size(), sh.stream);  // after the pack kernel
        std::vector<int> sp, rp;
        std::vector<const void*> sv;
        std::vector<void*> rv;
        std::vector<size_t> sb, rb;
        std::vector<std::vector<char>> rbufs;
        for (int q = 0; q < g.P; ++q) {
            if (q == sh.index) continue;
            const int64_t ns = h.send_off[q + 1] - h.send_off[q];
            const int64_t nr = h.recv_off[q + 1] - h.recv_off[q];
            if (ns > 0) {
                sp.push_back(q);
                sv.push_back(sbuf.data() + h.send_off[q] * elem_bytes);
                sb.push_back((size_t)ns * elem_bytes);
            }
            if (nr > 0) {
                rp.push_back(q);
                rbufs.emplace_back((size_t)nr * elem_bytes);
                rb.push_back((size_t)nr * elem_bytes);
            }
        }
        for (auto& b : rbufs) rv.push_back(b.data());
        host_exchange(c, sp, sv, sb, rp, rv, rb);
        for (size_t k = 0; k < rp.size(); ++k) copy_h2d(seg_ptr(0, rp[k]), rv[k], rb[k], sh.stream);
        return;
    }
    rccl_check(ncclGroupStart(), "ncclGroupStart");
    for (size_t i = 0; i < g.shards.size(); ++i) {
        Shard& sh = *g.shards[i];
        const Halo& h = g.halo(sh, adj);
        DeviceGuard dg(sh);
        for (int q = 0; q < g.P; ++q) {
            if (q == sh.index) continue;
            const int64_t ns = h.send_off[q + 1] - h.send_off[q];
            const int64_t nr = h.recv_off[q + 1] - h.recv_off[q];
            if (ns > 0)
                rccl_check(ncclSend(reinterpret_cast<const char*>(h.send_buf.get()) + h.send_off[q] * elem_bytes,
                                    (size_t)ns, type, q, sh.comm, sh.stream),
                           "ncclSend");
            if (nr > 0) rccl_check(ncclRecv(seg_ptr(i, q), (size_t)nr, type, q, sh.comm, sh.stream), "ncclRecv");
        }
    }
    rccl_check(ncclGroupEnd(), "ncclGroupEnd");
}

void exchange_halo_reverse(Graph& g, uint32_t adj, std::vector<void*>& vecs, std::vector<void*>& rbufs,
                           size_t elem_bytes, ncclDataType_t type) {
    if (g.P == 1) return;
    ExchTimer et(g);
    Ctx& c = *g.ctx;
    // shard r's segment for peer q (the run q sent it) goes back to q, landing at q's send-list
    // position for r
    auto seg_ptr = [&](size_t i, int q) {
        const Shard& sh = *g.shards[i];
        const Halo& h = g.halo(sh, adj);
        return static_cast<char*>(vecs[i]) + ((size_t)h.seg_of(q, sh.index) << h.tbits) * elem_bytes;
    };
    if (c.logical) {
        Shard& s0 = *g.shards[0];
        DeviceGuard dg(s0.device);
        for (size_t di = 0; di < g.shards.size(); ++di) {  // receiver: the owner
            const Halo& hd = g.halo(*g.shards[di], adj);
            for (size_t si = 0; si < g.shards.size(); ++si) {
                if (si == di) continue;
                const Halo& hs = g.halo(*g.shards[si], adj);
                const int q = g.shards[si]->index, r = g.shards[di]->index;
                const int64_t n = hs.recv_off[r + 1] - hs.recv_off[r];
                if (n == 0) continue;
                JG_HIP(hipMemcpyAsync(static_cast<char*>(rbufs[di]) + hd.send_off[q] * elem_bytes, seg_ptr(si, r),
                                      n * elem_bytes, hipMemcpyDeviceToDevice, s0.stream));
            }
        }
        return;
    }
    if (c.host_transport) {  // rank mode over host callbacks (one shard per process)
        Shard& sh = *g.shards[0];
        const Halo& h = g.halo(sh, adj);
        DeviceGuard dg(sh);
        std::vector<int> sp, rp;
        std::vector<const void*> sv;
        std::vector<void*> rv;
        std::vector<size_t> sb, rb;
        std::vector<std::vector<char>> sbufs, hrecv;
        for (int q = 0; q < g.P; ++q) {
            if (q == sh.index) continue;
            const int64_t ns = h.recv_off[q + 1] - h.recv_off[q];  // my segment for q goes back to q
            const int64_t nr = h.send_off[q + 1] - h.send_off[q];  // q's segment for me comes back
            if (ns > 0) {
                sp.push_back(q);
                sbufs.emplace_back((size_t)ns * elem_bytes);
                copy_d2h(sbufs.back().data(), seg_ptr(0, q), sbufs.back().size(), sh.stream);
                sb.push_back(sbufs.back().size());
            }
            if (nr > 0) {
                rp.push_back(q);
                hrecv.emplace_back((size_t)nr * elem_bytes);
                rb.push_back((size_t)nr * elem_bytes);
            }
        }
        for (auto& b : sbufs) sv.push_back(b.data());
        for (auto& b : hrecv) rv.push_back(b.data());
        host_exchange(c, sp, sv, sb, rp, rv, rb);
        for (size_t k = 0; k < rp.size(); ++k)
            copy_h2d(static_cast<char*>(rbufs[0]) + h.send_off[rp[k]] * elem_bytes, rv[k], rb[k], sh.stream);
        return;
    }
    rccl_check(ncclGroupStart(), "ncclGroupStart");
    for (size_t i = 0; i < g.shards.size(); ++i) {
        Shard& sh = *g.shards[i];
        const Halo& h = g.halo(sh, adj);
        DeviceGuard dg(sh);
        for (int q = 0; q < g.P; ++q) {
            if (q == sh.index) continue;
            const int64_t ns = h.recv_off[q + 1] - h.recv_off[q];  // my segment for q goes back to q
            const int64_t nr = h.send_off[q + 1] - h.send_off[q];  // q's segment for me comes back
            if (ns > 0) rccl_check(ncclSend(seg_ptr(i, q), (size_t)ns, type, q, sh.comm, sh.stream), "ncclSend");
            if (nr > 0)
                rccl_check(ncclRecv(static_cast<char*>(rbufs[i]) + h.send_off[q] * elem_bytes, (size_t)nr, type, q,
                                    sh.comm, sh.stream),
                           "ncclRecv");
        }
    }
    rccl_check(ncclGroupEnd(), "ncclGroupEnd");
}

std::vector<int64_t> halo_word_offsets(const Halo& h, int P) {
    std::vector<int64_t> w((size_t)P + 1, 0);
    for (int q = 0; q < P; ++q) w[(size_t)q + 1] = w[(size_t)q] + (h.send_off[(size_t)q + 1] - h.send_off[(size_t)q] + 63) / 64;
    return w;
}

void exchange_halo_bits(Graph& g, uint32_t adj, std::vector<uint64_t*>& sends, std::vector<uint64_t*>& bitmaps,
                        bool reverse) {
    if (g.P == 1) return;
    ExchTimer et(g);
    Ctx& c = *g.ctx;
    constexpr size_t W = sizeof(uint64_t);
    // shard i's words about peer q's vertices: its segment for q (receiver side of the forward run)
    auto seg_words = [&](size_t i, int q) {
        const Shard& sh = *g.shards[i];
        const Halo& h = g.halo(sh, adj);
        return bitmaps[i] + (((int64_t)h.seg_of(q, sh.index) << h.tbits) >> 6);
    };
    auto nwords = [](int64_t bits) { return (bits + 63) / 64; };
    if (c.logical) {
        Shard& s0 = *g.shards[0];
        DeviceGuard dg(s0.device);
        for (size_t oi = 0; oi < g.shards.size(); ++oi) {  // the owner of the vertices
            const Halo& ho = g.halo(*g.shards[oi], adj);
            const std::vector<int64_t> woff = halo_word_offsets(ho, g.P);
            for (size_t ri = 0; ri < g.shards.size(); ++ri) {  // the shard that reads them
                if (ri == oi) continue;
                const int q = g.shards[oi]->index, r = g.shards[ri]->index;
                const int64_t n = nwords(ho.send_off[(size_t)r + 1] - ho.send_off[(size_t)r]);
                if (n == 0) continue;
                uint64_t* own = sends[oi] + woff[(size_t)r];
                uint64_t* seg = seg_words(ri, q);
                JG_HIP(hipMemcpyAsync(reverse ? own : seg, reverse ? seg : own, (size_t)n * W, hipMemcpyDeviceToDevice,
                                      s0.stream));
            }
        }
        return;
    }
    if (c.host_transport) {  // rank mode over host callbacks (one shard per process)
        Shard& sh = *g.shards[0];
        const Halo& h = g.halo(sh, adj);
        DeviceGuard dg(sh);
        const std::vector<int64_t> woff = halo_word_offsets(h, g.P);
        std::vector<int> sp, rp;
        std::vector<const void*> sv;
        std::vector<void*> rv;
        std::vector<size_t> sb, rb;
        std::vector<std::vector<uint64_t>> out, in;
        std::vector<uint64_t*> dst;
        for (int q = 0; q < g.P; ++q) {
            if (q == sh.index) continue;
            const int64_t mine = nwords(h.send_off[(size_t)q + 1] - h.send_off[(size_t)q]);  // my vertices q reads
            const int64_t theirs = nwords(h.recv_off[(size_t)q + 1] - h.recv_off[(size_t)q]);  // q's vertices I read
            const int64_t ns = reverse ? theirs : mine, nr = reverse ? mine : theirs;
            if (ns > 0) {
                sp.push_back(q);
                out.emplace_back((size_t)ns);
                copy_d2h(out.back().data(), reverse ? seg_words(0, q) : sends[0] + woff[(size_t)q], (size_t)ns * W,
                         sh.stream);
                sb.push_back((size_t)ns * W);
            }
            if (nr > 0) {
                rp.push_back(q);
                in.emplace_back((size_t)nr);
                rb.push_back((size_t)nr * W);
                dst.push_back(reverse ? sends[0] + woff[(size_t)q] : seg_words(0, q));
            }
        }
        for (auto& b : out) sv.push_back(b.data());
        for (auto& b : in) rv.push_back(b.data());
        host_exchange(c, sp, sv, sb, rp, rv, rb);
        for (size_t k = 0; k < rp.size(); ++k) copy_h2d(dst[k], rv[k], rb[k], sh.stream);
        return;
    }
    rccl_check(ncclGroupStart(), "ncclGroupStart");
    for (size_t i = 0; i < g.shards.size(); ++i) {
        Shard& sh = *g.shards[i];
        const Halo& h = g.halo(sh, adj);
        DeviceGuard dg(sh);
        const std::vector<int64_t> woff = halo_word_offsets(h, g.P);
        for (int q = 0; q < g.P; ++q) {
            if (q == sh.index) continue;
            const int64_t mine = nwords(h.send_off[(size_t)q + 1] - h.send_off[(size_t)q]);
            const int64_t theirs = nwords(h.recv_off[(size_t)q + 1] - h.recv_off[(size_t)q]);
            uint64_t* own = sends[i] + woff[(size_t)q];
            uint64_t* seg = seg_words(i, q);
            if (!reverse) {
                if (mine > 0) rccl_check(ncclSend(own, (size_t)mine, ncclUint64, q, sh.comm, sh.stream), "ncclSend");
                if (theirs > 0) rccl_check(ncclRecv(seg, (size_t)theirs, ncclUint64, q, sh.comm, sh.stream), "ncclRecv");
            } else {
                if (theirs > 0) rccl_check(ncclSend(seg, (size_t)theirs, ncclUint64, q, sh.comm, sh.stream), "ncclSend");
                if (mine > 0) rccl_check(ncclRecv(own, (size_t)mine, ncclUint64, q, sh.comm, sh.stream), "ncclRecv");
            }
        }
    }
    rccl_check(ncclGroupEnd(), "ncclGroupEnd");
}

void exchange_halo_bits_both(Graph& g, uint32_t adj, std::vector<uint64_t*>& fsend, std::vector<uint64_t*>& fbitmap,
                             std::vector<uint64_t*>& rbitmap, std::vector<uint64_t*>& rsend) {
    if (g.P == 1) return;
    Ctx& c = *g.ctx;
    if (c.logical) {  // (the sharded DO-BFS copies the level's one direction by kernel on one device)
        exchange_halo_bits(g, adj, fsend, fbitmap, false);
        exchange_halo_bits(g, adj, rsend, rbitmap, true);
        return;
    }
    ExchTimer et(g);
    // The transfers of every local shard, in the order RCCL matches them: two each way per peer pair,
    // both sides sending [forward, reverse] and receiving [forward, reverse].  My forward send (my send
    // list for q: `mine` words) is q's forward receive (its segment for me); my reverse send (my marks
    // about q's vertices: `theirs` words) is q's reverse receive (its send-list words from me).  The
    // host-transport mode hands the same ordered lists to the transport, whose point-to-point messages
    // also match in issue order per peer pair (gloo), so the rank-mode tests check this plan.
    struct Op {
        int peer;
        uint64_t* p;
        int64_t words;
    };
    std::vector<std::vector<Op>> sends(g.shards.size()), recvs(g.shards.size());
    for (size_t i = 0; i < g.shards.size(); ++i) {
        const Shard& sh = *g.shards[i];
        const Halo& h = g.halo(sh, adj);
        const std::vector<int64_t> woff = halo_word_offsets(h, g.P);
        for (int q = 0; q < g.P; ++q) {
            if (q == sh.index) continue;
            const int64_t mine = (h.send_off[(size_t)q + 1] - h.send_off[(size_t)q] + 63) / 64;    // my vertices q reads
            const int64_t theirs = (h.recv_off[(size_t)q + 1] - h.recv_off[(size_t)q] + 63) / 64;  // q's vertices I read
            const int64_t seg = (((int64_t)h.seg_of(q, sh.index) << h.tbits) >> 6);
            if (mine > 0) sends[i].push_back({q, fsend[i] + woff[(size_t)q], mine});
            if (theirs > 0) sends[i].push_back({q, rbitmap[i] + seg, theirs});
            if (theirs > 0) recvs[i].push_back({q, fbitmap[i] + seg, theirs});
            if (mine > 0) recvs[i].push_back({q, rsend[i] + woff[(size_t)q], mine});
        }
    }
    constexpr size_t W = sizeof(uint64_t);
    if (c.host_transport) {  // rank mode over host callbacks (one shard per process)
        Shard& sh = *g.shards[0];
        DeviceGuard dg(sh);
        std::vector<int> sp, rp;
        std::vector<std::vector<uint64_t>> out, in;
        std::vector<const void*> sv;
        std::vector<void*> rv;
        std::vector<size_t> sb, rb;
        for (const Op& o : sends[0]) {
            sp.push_back(o.peer);
            out.emplace_back((size_t)o.words);
            copy_d2h(out.back().data(), o.p, (size_t)o.words * W, sh.stream);
            sb.push_back((size_t)o.words * W);
        }
        for (const Op& o : recvs[0]) {
            rp.push_back(o.peer);
            in.emplace_back((size_t)o.words);
            rb.push_back((size_t)o.words * W);
        }
        for (auto& v : out) sv.push_back(v.data());
        for (auto& v : in) rv.push_back(v.data());
        host_exchange(c, sp, sv, sb, rp, rv, rb);
        for (size_t k = 0; k < recvs[0].size(); ++k) copy_h2d(recvs[0][k].p, rv[k], rb[k], sh.stream);
        return;
    }
    rccl_check(ncclGroupStart(), "ncclGroupStart");
    for (size_t i = 0; i < g.shards.size(); ++i) {
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        for (const Op& o : sends[i]) rccl_check(ncclSend(o.p, (size_t)o.words, ncclUint64, o.peer, sh.comm, sh.stream), "ncclSend");
        for (const Op& o : recvs[i]) rccl_check(ncclRecv(o.p, (size_t)o.words, ncclUint64, o.peer, sh.comm, sh.stream), "ncclRecv");
    }
    rccl_check(ncclGroupEnd(), "ncclGroupEnd");
}

void exchange_runs(Graph& g, const std::vector<const char*>& send, const std::vector<std::vector<int64_t>>& soff,
                   const std::vector<std::vector<int64_t>>& scount, const std::vector<char*>& recv,
                   const std::vector<std::vector<int64_t>>& roff, const std::vector<std::vector<int64_t>>& rcount,
                   size_t eb, ncclDataType_t type) {
    if (g.P == 1) return;
    ExchTimer et(g);
    Ctx& c = *g.ctx;
    const size_t ns = g.shards.size();
    if (c.logical) {  // every shard here, one device and stream: device copies
        Shard& s0 = *g.shards[0];
        DeviceGuard dg(s0.device);
        for (size_t i = 0; i < ns; ++i)
            for (size_t j = 0; j < ns; ++j) {
                if (i == j) continue;
                const int qi = g.shards[i]->index, qj = g.shards[j]->index;
                const int64_t n = scount[i][(size_t)qj];
                if (n != rcount[j][(size_t)qi]) fail(JG_ERR_HIP, "exchange_runs: send and receive counts differ");
                if (n > 0)
                    JG_HIP(hipMemcpyAsync(recv[j] + (size_t)roff[j][(size_t)qi] * eb, send[i] + (size_t)soff[i][(size_t)qj] * eb,
                                          (size_t)n * eb, hipMemcpyDeviceToDevice, s0.stream));
            }
        return;
    }
    if (c.host_transport) {  // rank mode over host callbacks (one shard per process)
        Shard& sh = *g.shards[0];
        DeviceGuard dg(sh);
        std::vector<int> sp, rp;
        std::vector<const void*> sv;
        std::vector<void*> rv;
        std::vector<size_t> sb, rb;
        std::vector<std::vector<char>> out, in;
        for (int q = 0; q < g.P; ++q) {
            if (q == sh.index) continue;
            const int64_t n_s = scount[0][(size_t)q], n_r = rcount[0][(size_t)q];
            if (n_s > 0) {
                sp.push_back(q);
                out.emplace_back((size_t)n_s * eb);
                copy_d2h(out.back().data(), send[0] + (size_t)soff[0][(size_t)q] * eb, out.back().size(), sh.stream);
                sb.push_back(out.back().size());
            }
            if (n_r > 0) {
                rp.push_back(q);
                in.emplace_back((size_t)n_r * eb);
                rb.push_back(in.back().size());
            }
        }
        for (auto& b : out) sv.push_back(b.data());
        for (auto& b : in) rv.push_back(b.data());
        host_exchange(c, sp, sv, sb, rp, rv, rb);
        for (size_t k = 0; k < rp.size(); ++k)
            copy_h2d(recv[0] + (size_t)roff[0][(size_t)rp[k]] * eb, rv[k], rb[k], sh.stream);
        return;
    }
    rccl_check(ncclGroupStart(), "ncclGroupStart");
    for (size_t i = 0; i < ns; ++i) {
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        for (int q = 0; q < g.P; ++q) {
            if (q == sh.index) continue;
            const int64_t n_s = scount[i][(size_t)q], n_r = rcount[i][(size_t)q];
            if (n_s > 0)
                rccl_check(ncclSend(send[i] + (size_t)soff[i][(size_t)q] * eb, (size_t)n_s, type, q, sh.comm, sh.stream),
                           "ncclSend");
            if (n_r > 0)
                rccl_check(ncclRecv(recv[i] + (size_t)roff[i][(size_t)q] * eb, (size_t)n_r, type, q, sh.comm, sh.stream),
                           "ncclRecv");
        }
    }
    rccl_check(ncclGroupEnd(), "ncclGroupEnd");
}

void exchange_vec(Graph& g, uint32_t adj, std::vector<void*>& bufs, size_t elem_bytes, ncclDataType_t type) {
    if (g.P == 1) return;
    if (g.halo(*g.shards[0], adj).on)
        exchange_halo(g, adj, bufs, elem_bytes, type);
    else
        exchange_allgather(g, bufs, elem_bytes, type);
}

}  // namespace jg
