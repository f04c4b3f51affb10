// jg_decode.hip — GPU decode of JanusGraph edgestore entries.
//
// The CSR snapshot's input, as the edgestore holds it: every adjacency entry of a vertex row is a
// column (relation-type header, optional sort key, vertex / relation ids) followed by a value.
// EdgeSerializer.parseRelation (core/graphdb/database/EdgeSerializer.java:86-122) decodes one entry:
//   header  IDHandler.readRelationType (idhandling/IDHandler.java:130-141) = readPositiveWithPrefix(3)
//           (idhandling/VariableLong.java:193-208): prefix bit 0 edge/property, prefix >> 1 == 0 system,
//           value bit 0 direction, value >> 1 the type count; type id = count << 6 | suffix
//           (idmanagement/IDManager.java:650-653).
//   MULTI edge:      other vertex and relation id written backward before the value position,
//                    read backward from it (VariableLong.java:276-294);
//   unique in dir:   both written forward from the value position (VariableLong.java:44-52);
//   constrained, not unique: other backward before, relation forward after the value position.
// Multiplicity per edge label (core/core/Multiplicity.java:35-90) comes from a small caller table;
// absent labels are MULTI.  One thread per entry, every entry independent: byte-level work bound by
// HBM (a few loads per entry; neighbouring threads read neighbouring entries).
#include <algorithm>
#include <vector>

#include "jg_internal.h"

namespace jg {

namespace {

// Reads stay inside the entry [0, len): a varint that runs off it sets bad (the entry is reported as
// malformed, dir = -1) instead of reading a neighbour's bytes or past the buffer.
__device__ __forceinline__ int64_t read_unsigned(const uint8_t* __restrict__ b, int64_t& pos, int64_t len, bool& bad) {
    int64_t v = 0;
    for (;;) {
        if (pos >= len) {
            bad = true;
            return 0;
        }
        const int c = b[pos++];
        v = (v << 7) | (c & 0x7F);
        if (c & 0x80) return v;
    }
}

__device__ __forceinline__ int64_t read_unsigned_backward(const uint8_t* __restrict__ b, int64_t& pos, bool& bad) {
    int64_t v = 0;
    int n = 0;
    for (;;) {
        if (pos <= 0) {
            bad = true;
            return 0;
        }
        const int c = b[--pos];
        if (c & 0x80) {  // first byte: stop marker, 3 length bits, 4 value bits
            v |= (int64_t)(c & 0x0F) << (7 * n);
            return v;
        }
        v |= (int64_t)c << (7 * n);
        ++n;
    }
}

struct DecodeArgs {
    const uint8_t* bytes;
    const int64_t* off;
    const int32_t* vpos;
    int64_t n;
    const int64_t* type_ids;  // sorted
    const int8_t* type_mult;
    int32_t ntypes;
    int64_t* type_out;
    int8_t* dir_out;
    int64_t* other_out;
    int64_t* rel_out;
};

__global__ __launch_bounds__(kBlock) void decode_edges_kernel(DecodeArgs a) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < a.n; e += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t* __restrict__ b = a.bytes + a.off[e];
        const int64_t len = a.off[e + 1] - a.off[e];
        bool bad = false;
        int64_t pos = 0;
        const int first = b[pos++];
        const int prefix = first >> 5;
        int64_t value = first & 0x0F;
        if ((first >> 4) & 1) {
            const int64_t p0 = pos;
            const int64_t rem = read_unsigned(b, pos, len, bad);
            value = (value << (7 * (pos - p0))) + rem;
        }
        const bool is_edge = prefix & 1, system = (prefix >> 1) == 0;
        const int dirbit = (int)(value & 1);
        const int64_t suffix = is_edge ? (system ? 53 : 21) : (system ? 37 : 5);
        const int64_t type_id = ((value >> 1) << 6) | suffix;
        int64_t other = -1, rel = -1;
        int8_t dir = (int8_t)(is_edge ? 3 : 2);
        if (is_edge && !system) {
            dir = (int8_t)dirbit;
            int mult = 0;
            int lo = 0, hi = a.ntypes;  // lower bound of type_id
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (a.type_ids[mid] < type_id) lo = mid + 1; else hi = mid;
            }
            if (lo < a.ntypes && a.type_ids[lo] == type_id) mult = a.type_mult[lo];
            const bool unique = dirbit ? (mult == 2 || mult == 4) : (mult == 3 || mult == 4);
            int64_t p = a.vpos[e];
            if (mult == 0) {
                rel = read_unsigned_backward(b, p, bad);
                other = read_unsigned_backward(b, p, bad);
            } else if (unique) {
                other = read_unsigned(b, p, len, bad);
                rel = read_unsigned(b, p, len, bad);
            } else {
                other = read_unsigned_backward(b, p, bad);
                p = a.vpos[e];
                rel = read_unsigned(b, p, len, bad);
            }
        }
        if (bad) {
            dir = -1;
            other = rel = -1;
        }
        if (a.type_out) a.type_out[e] = type_id;
        if (a.dir_out) a.dir_out[e] = dir;
        if (a.other_out) a.other_out[e] = other;
        if (a.rel_out) a.rel_out[e] = rel;
    }
}

}  // namespace

void decode_edges(Ctx& c, const uint8_t* bytes, int64_t nbytes, const int64_t* off, const int32_t* vpos, int64_t n,
                  const int64_t* type_ids, const int8_t* type_mult, int32_t ntypes, int64_t* type_out,
                  int8_t* dir_out, int64_t* other_out, int64_t* rel_out) {
    if (n < 0 || nbytes < 0 || ntypes < 0) fail(JG_ERR_ARG, "negative size");
    if (n > 0 && (!bytes || !off || !vpos)) fail(JG_ERR_ARG, "null entry arrays");
    if (ntypes > 0 && (!type_ids || !type_mult)) fail(JG_ERR_ARG, "null type table");
    // every entry must lie inside the byte array, with its value position inside the entry
    for (int64_t e = 0; e < n; ++e) {
        const int64_t len = off[e + 1] - off[e];
        if (off[e] < 0 || len < 1 || off[e + 1] > nbytes || vpos[e] < 1 || vpos[e] > len)
            fail(JG_ERR_ARG, "entry " + std::to_string(e) + " out of range");
    }
    std::vector<std::pair<int64_t, int8_t>> tt((size_t)ntypes);
    for (int32_t t = 0; t < ntypes; ++t) {
        if (type_mult[t] < 0 || type_mult[t] > 4) fail(JG_ERR_ARG, "multiplicity code must be in [0, 4]");
        tt[(size_t)t] = {type_ids[t], type_mult[t]};
    }
    std::sort(tt.begin(), tt.end());
    std::vector<int64_t> tid(tt.size());
    std::vector<int8_t> tm(tt.size());
    for (size_t t = 0; t < tt.size(); ++t) {
        tid[t] = tt[t].first;
        tm[t] = tt[t].second;
    }
    const int dev = c.devices.empty() ? 0 : c.devices[0];
    DeviceGuard dg(dev);
    hipStream_t s = c.streams.empty() ? nullptr : c.streams[0];
    DevBuf<uint8_t> d_bytes(std::max<int64_t>(nbytes, 1));
    DevBuf<int64_t> d_off(n + 1), d_type(std::max<int64_t>(n, 1)), d_other(std::max<int64_t>(n, 1)),
        d_rel(std::max<int64_t>(n, 1)), d_tid(std::max<int32_t>(ntypes, 1));
    DevBuf<int32_t> d_vpos(std::max<int64_t>(n, 1));
    DevBuf<int8_t> d_dir(std::max<int64_t>(n, 1)), d_tm(std::max<int32_t>(ntypes, 1));
    if (nbytes) copy_h2d(d_bytes.get(), bytes, (size_t)nbytes, s);
    if (n) {
        copy_h2d(d_off.get(), off, (size_t)(n + 1) * sizeof(int64_t), s);
        copy_h2d(d_vpos.get(), vpos, (size_t)n * sizeof(int32_t), s);
    }
    if (ntypes) {
        copy_h2d(d_tid.get(), tid.data(), tid.size() * sizeof(int64_t), s);
        copy_h2d(d_tm.get(), tm.data(), tm.size(), s);
    }
    DecodeArgs a{d_bytes.get(), d_off.get(), d_vpos.get(), n, d_tid.get(), d_tm.get(), ntypes,
                 type_out ? d_type.get() : nullptr, dir_out ? d_dir.get() : nullptr,
                 other_out ? d_other.get() : nullptr, rel_out ? d_rel.get() : nullptr};
    hipEvent_t t0, t1;
    JG_HIP(hipEventCreate(&t0));
    JG_HIP(hipEventCreate(&t1));
    JG_HIP(hipEventRecord(t0, s));
    if (n > 0) {
        decode_edges_kernel<<<grid_for(n, kBlock, 256 * 64), kBlock, 0, s>>>(a);
        JG_LAUNCH_CHECK();
    }
    JG_HIP(hipEventRecord(t1, s));
    JG_HIP(hipEventSynchronize(t1));
    float ms = 0;
    JG_HIP(hipEventElapsedTime(&ms, t0, t1));
    JG_HIP(hipEventDestroy(t0));
    JG_HIP(hipEventDestroy(t1));
    c.last = jg_stats{};
    c.last.compute_ms = ms;
    c.last.kernel_ms_total = ms;
    c.last.kernel_launches = n > 0 ? 1 : 0;
    // bytes the decode must move: the entries, offsets and value positions in, the outputs out
    c.last.algorithmic_bytes = (double)nbytes + 12.0 * (double)n +
                               (double)n * ((type_out ? 8 : 0) + (dir_out ? 1 : 0) + (other_out ? 8 : 0) + (rel_out ? 8 : 0));
    if (n && type_out) copy_d2h(type_out, d_type.get(), (size_t)n * sizeof(int64_t), s);
    if (n && dir_out) copy_d2h(dir_out, d_dir.get(), (size_t)n, s);
    if (n && other_out) copy_d2h(other_out, d_other.get(), (size_t)n * sizeof(int64_t), s);
    if (n && rel_out) copy_d2h(rel_out, d_rel.get(), (size_t)n * sizeof(int64_t), s);
}

}  // namespace jg
