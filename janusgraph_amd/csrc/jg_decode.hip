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
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "jg_internal.h"
#include "jg_prim.h"

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

// The entry stream: entry e is bytes[off[e] .. off[e+1]), its value at vpos[e]; edge-label
// multiplicities from a sorted (type id, code) table.
struct EntryView {
    const uint8_t* bytes;
    const int64_t* off;
    const int32_t* vpos;
    const int64_t* type_ids;  // sorted
    const int8_t* type_mult;
    int32_t ntypes;
};

struct Decoded {
    int64_t type_id, other, rel;
    int64_t vstart;  // user edges: first byte after the ids (signature values, then inline properties)
    int8_t dir;    // 0 OUT edge, 1 IN edge, 2 property, 3 system relation, -1 malformed
    bool visible;  // a user relation (header prefix >> 1 == 1), not system, not invisible
};

// EdgeSerializer.parseRelation (EdgeSerializer.java:86-122) of one entry, header and ids only.
// b = the entry's bytes (global memory or the block's LDS stage), len its length, vpos its value
// position.
__device__ __forceinline__ Decoded decode_entry(const EntryView& a, const uint8_t* __restrict__ b, int64_t len,
                                                int64_t vpos) {
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
    Decoded d;
    d.type_id = ((value >> 1) << 6) | suffix;
    d.other = d.rel = -1;
    d.vstart = vpos;
    d.dir = (int8_t)(is_edge ? 3 : 2);
    d.visible = (prefix >> 1) == 1;
    if (is_edge && !system) {
        d.dir = (int8_t)dirbit;
        int mult = 0;
        int lo = 0, hi = a.ntypes;  // lower bound of type_id
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (a.type_ids[mid] < d.type_id) lo = mid + 1; else hi = mid;
        }
        if (lo < a.ntypes && a.type_ids[lo] == d.type_id) mult = a.type_mult[lo];
        const bool unique = dirbit ? (mult == 2 || mult == 4) : (mult == 3 || mult == 4);
        int64_t p = vpos;
        if (mult == 0) {
            d.rel = read_unsigned_backward(b, p, bad);
            d.other = read_unsigned_backward(b, p, bad);
        } else if (unique) {
            d.other = read_unsigned(b, p, len, bad);
            d.rel = read_unsigned(b, p, len, bad);
            d.vstart = p;
        } else {
            d.other = read_unsigned_backward(b, p, bad);
            p = vpos;
            d.rel = read_unsigned(b, p, len, bad);
            d.vstart = p;
        }
    }
    if (bad) {
        d.dir = -1;
        d.other = d.rel = -1;
    }
    return d;
}

// ---- the Integer weight property of an edge, read from its value (ShortestDistanceVertexProgram.java:69)
// EdgeSerializer.writeRelation (:294-302) stores an edge's properties after its ids: the label's
// signature values (none: the caller checks), then each other property as its inline key id
// (IDHandler.writeInlineRelationType: VariableLong.writePositive of the id without its 4 padding bits)
// and its value (StandardSerializer.writeObject: a null flag byte 0 / -1 unless the serializer takes
// nulls itself, then the serializer's bytes), in ascending key-id order.  Key types (JG_PROP_*):
// the fixed widths of ByteSerializer 1, ShortSerializer 2, LongSerializer 8, CharacterSerializer 2,
// BooleanSerializer 1, DateSerializer 8, FloatSerializer 4, DoubleSerializer 8, UUIDSerializer 16;
// IntegerSerializer a signed VariableLong; StringSerializer (no flag byte) its own length header.
// Error bits of the snapshot (any set bit fails the build before the CSR is cut)
enum : int32_t { kErrBadKey = 1, kErrPartitioned = 2, kErrMalformed = 4, kErrWeightType = 8, kErrWeightValue = 16 };

// VariableLong.read: the zig-zag-free sign encoding |v| << 1 | sign (VariableLong.java:133-152)
__device__ __forceinline__ int64_t read_signed(const uint8_t* __restrict__ b, int64_t& pos, int64_t len, bool& bad) {
    const uint64_t u = (uint64_t)read_unsigned(b, pos, len, bad);
    return (u & 1) ? -(int64_t)(u >> 1) : (int64_t)(u >> 1);
}

// StringSerializer.read (StringSerializer.java:98-151), skipping the characters
__device__ __forceinline__ void skip_string(const uint8_t* __restrict__ b, int64_t& pos, int64_t len, bool& bad) {
    const int64_t h = read_unsigned(b, pos, len, bad);
    if (bad || h == 0) return;  // 0: null
    int64_t l = h >> 3;
    if ((h & 7) != 0) {  // compressed: l bytes
        pos += l;
    } else if ((l & 1) == 0) {  // ASCII: one byte per character, the last one marked
        l >>= 1;
        if (l == 2) {
            for (;;) {
                if (pos >= len) { bad = true; return; }
                if (b[pos++] & 0x80) break;
            }
        } else if (l != 1) {
            bad = true;
        }
    } else {  // full UTF: l >> 1 characters of 1 to 3 bytes (lead nibble 12/13: 2, 14: 3, any other: 1,
              // as StringSerializer.java:126-145 consumes them)
        for (int64_t i = 0, nc = l >> 1; i < nc; ++i) {
            if (pos >= len) { bad = true; return; }
            const int hi = b[pos] >> 4;
            pos += hi == 14 ? 3 : (hi == 12 || hi == 13) ? 2 : 1;
        }
    }
    if (pos > len) bad = true;
}

// The weight of one entry: JG_WEIGHT_ABSENT when the edge has no (non-null Integer) weight; *err gets
// kErrWeightType when a property of an unknown type precedes the weight key (its length is unknown).
__device__ __forceinline__ int32_t decode_weight(const uint8_t* __restrict__ b, int64_t pos, int64_t len,
                                                 const WeightSchema& w, int32_t* err) {
    bool bad = false;
    while (pos < len) {
        const int64_t kid = read_unsigned(b, pos, len, bad);
        if (bad || kid > w.key) break;  // ascending ids: the weight key is not on this edge
        int lo = 0, hi = w.n;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (w.ids[mid] < kid) lo = mid + 1; else hi = mid;
        }
        const int type = lo < w.n && w.ids[lo] == kid ? w.types[lo] : 0;
        if (type == JG_PROP_STRING) {
            skip_string(b, pos, len, bad);
            continue;
        }
        if (type <= 0 || type > JG_PROP_UUID) {
            atomicOr(err, kErrWeightType);
            return JG_WEIGHT_ABSENT;
        }
        if (pos >= len) { bad = true; break; }
        const uint8_t flag = b[pos++];
        if (flag == 0xFF) {  // a null value
            if (kid == w.key) return JG_WEIGHT_ABSENT;
            continue;
        }
        if (flag != 0) { bad = true; break; }
        if (type == JG_PROP_INT) {
            const int64_t v = read_signed(b, pos, len, bad);
            if (kid == w.key) {
                if (bad || v < INT32_MIN || v > INT32_MAX) break;
                if (v == INT32_MIN) {  // the absent marker itself: refuse rather than drop the weight
                    atomicOr(err, kErrWeightValue);
                    return JG_WEIGHT_ABSENT;
                }
                return (int32_t)v;
            }
            continue;
        }
        if (kid == w.key) return JG_WEIGHT_ABSENT;  // not an Integer: Fulgora's <Integer> cast throws
        constexpr int8_t kWidth[JG_PROP_UUID + 1] = {0, 1, 2, 0, 8, 2, 1, 8, 4, 8, 16};  // by JG_PROP_*
        pos += kWidth[type];
    }
    if (bad || pos > len) atomicOr(err, kErrMalformed);
    return JG_WEIGHT_ABSENT;
}

// One thread per entry: the weight of every OUT user edge (the kept entries' weights are compacted
// with the edges, as host-given weights are).
__global__ __launch_bounds__(kBlock) void edgestore_weight_kernel(EntryView a, int64_t nentries, WeightSchema w,
                                                                  int32_t* __restrict__ weight,
                                                                  int32_t* __restrict__ err) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nentries; e += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t* b = a.bytes + a.off[e];
        const int64_t len = a.off[e + 1] - a.off[e];
        const Decoded d = decode_entry(a, b, len, a.vpos[e]);
        weight[e] = d.dir == 0 && d.visible ? decode_weight(b, d.vstart, len, w, err) : JG_WEIGHT_ABSENT;
    }
}

struct DecodeOut {
    int64_t* type_out;
    int8_t* dir_out;
    int64_t* other_out;
    int64_t* rel_out;
};

// Block-staged entries: a block decodes kBlock consecutive entries, whose bytes are one contiguous
// range; it is streamed into LDS with coalesced dword loads, then every thread parses its entry
// there (the varint walks are dependent byte loads: from HBM they serialise on memory latency).
// A block whose range exceeds the stage (entries with long property values) reads global memory.
// The byte array is allocated with kBytePad slack, so the dword loads may run past its end.
constexpr int kStageWords = 4096;  // 16 KB of LDS per block (a 1024-entry chunk of ~10-byte entries)
constexpr int64_t kBytePad = 64;

struct Stage {
    const uint8_t* base;  // where entry bytes are read from
    int64_t origin;       // byte offset of base[0] in the array
};

__device__ __forceinline__ Stage stage_entries(const EntryView& a, int64_t e0, int64_t e_end, uint32_t* lds) {
    const int64_t b0 = a.off[e0] & ~(int64_t)3, b1 = a.off[e_end];
    const int64_t words = (b1 - b0 + 3) >> 2;
    if (words > kStageWords) return Stage{a.bytes, 0};
    const uint32_t* __restrict__ src = reinterpret_cast<const uint32_t*>(a.bytes + b0);
    for (int64_t w = threadIdx.x; w < words; w += kBlock) lds[w] = __builtin_nontemporal_load(src + w);
    __syncthreads();
    return Stage{reinterpret_cast<const uint8_t*>(lds), b0};
}

__global__ __launch_bounds__(kBlock) void decode_edges_kernel(EntryView a, int64_t n, DecodeOut o) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kStageWords];
    for (int64_t e0 = (int64_t)blockIdx.x * kBlock; e0 < n; e0 += (int64_t)gridDim.x * kBlock) {
        const int64_t e_end = e0 + kBlock < n ? e0 + kBlock : n;
        const Stage st = stage_entries(a, e0, e_end, lds);
        const int64_t e = e0 + threadIdx.x;
        if (e < e_end) {
            const int64_t o0 = a.off[e];
            const Decoded d = decode_entry(a, st.base + (o0 - st.origin), a.off[e + 1] - o0, a.vpos[e]);
            if (o.type_out) o.type_out[e] = d.type_id;
            if (o.dir_out) o.dir_out[e] = d.dir;
            if (o.other_out) o.other_out[e] = d.other;
            if (o.rel_out) o.rel_out[e] = d.rel;
        }
        __syncthreads();  // the stage is reused by the next block-iteration
    }
}

// ---------------- CSR snapshot straight from edgestore rows ----------------
// IDManager.getKeyID (idmanagement/IDManager.java:496-506) of a user row key: partition in the top
// pbits, count above the 3-bit type suffix; id = (count << pbits | partition) << 3 | suffix.
// Returns -1 for an odd key (schema / invisible row: VertexJobConverter.getKeyFilter, :174-177
// drops it) and -2 for a suffix that is no user vertex type (getUserVertexIDType throws).
__device__ __forceinline__ int64_t key_to_vertex_id(uint64_t key, int pbits) {
    if (key & 1) return -1;
    const uint64_t suffix = key & 7;
    if (suffix == 6) return -2;
    const int poff = 64 - pbits;
    const uint64_t partition = poff < 64 ? key >> poff : 0;
    const uint64_t count = (key >> 3) & ((1ull << (poff - 3)) - 1ull);
    return (int64_t)((((count << pbits) + partition) << 3) | suffix);
}

constexpr int64_t kVertexExistsId = (1 << 6) | 37;  // BaseKey.VertexExists: SystemPropertyKey count 1


// IDManager.getCanonicalVertexId (idmanagement/IDManager.java:525-547): a partitioned (vertex-cut)
// vertex's representatives share its count; the canonical one sits in the partition hashed from it.
__device__ __forceinline__ int64_t canonical_vertex_id(int64_t vid, int pbits) {
    const uint64_t count = (uint64_t)vid >> (pbits + 3);
    uint64_t h = 0;
    for (int off = 0; off < 64; off += pbits) h ^= (count >> off) & ((1ull << pbits) - 1ull);
    return (int64_t)((((count << pbits) + h) << 3) | 2u);
}

__device__ __forceinline__ bool is_partitioned(int64_t vid, int pbits) {
    return vid > 0 && (vid & 7) == 2 && ((uint64_t)vid >> (pbits + 3)) > 0;
}

// One thread per row: vertex id, key filter, ghost rule (VertexJobConverter.process / isGhostVertex,
// olap/VertexJobConverter.java:122-151: the row's first entry must be the VertexExists property;
// system properties sort first, so it is entry 0 of the row when present).  Partitioned vertices
// (VertexProgramScanJob.java:88-102; FulgoraVertexMemory.getCanonicalId): every representative row
// contributes its edges to the canonical vertex; a non-canonical representative is never a ghost
// and adds no vertex of its own.
//   keep_edges[r]: the row's OUT entries are edges; keep_vertex[r]: the row is a vertex of V.
__global__ __launch_bounds__(kBlock) void edgestore_rows_kernel(EntryView a, const uint64_t* __restrict__ keys,
                                                                 const int64_t* __restrict__ row_off, int64_t nrows,
                                                                 int pbits, uint8_t* __restrict__ keep_edges,
                                                                 uint8_t* __restrict__ keep_vertex,
                                                                 int64_t* __restrict__ row_vid, int32_t* __restrict__ err) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x) {
        int64_t vid = key_to_vertex_id(keys[r], pbits);
        uint8_t ke = 0, kv = 0;
        if (vid == -2) {
            atomicOr(err, kErrBadKey);
        } else if (vid >= 0) {
            bool canonical = true;
            if ((vid & 7) == 2) {
                if (pbits == 0) {  // getPartitionHashForId: "no partition bits"
                    atomicOr(err, kErrPartitioned);
                } else {
                    const int64_t c = canonical_vertex_id(vid, pbits);
                    canonical = c == vid;
                    vid = c;
                }
            }
            if (!canonical) {
                ke = 1;
            } else if (row_off[r + 1] > row_off[r]) {
                const int64_t e = row_off[r];
                const Decoded d = decode_entry(a, a.bytes + a.off[e], a.off[e + 1] - a.off[e], a.vpos[e]);
                if (d.dir < 0) atomicOr(err, kErrMalformed);
                ke = kv = (d.dir == 2 && d.type_id == kVertexExistsId) ? 1 : 0;
            }
        }
        keep_edges[r] = ke;
        keep_vertex[r] = kv;
        row_vid[r] = vid;
    }
}

// One thread per entry: the row (binary search of row_off), then the entry's OUT edge.  Every edge
// is stored twice, OUT on its source row and IN on its target row (a self-loop: both on one row,
// StandardJanusGraph.java:617-640), so the OUT entries of the kept rows are the edge list exactly
// once.  Visible user edges only (bothE() of a PreloadedVertex sees no system or invisible type).
__device__ __forceinline__ int64_t row_of_entry(const int64_t* __restrict__ row_off, int64_t lo, int64_t hi, int64_t e) {
    while (hi - lo > 1) {  // last row r in [lo, hi) with row_off[r] <= e
        const int64_t mid = (lo + hi) >> 1;
        if (row_off[mid] <= e) lo = mid; else hi = mid;
    }
    return lo;
}

// The snapshot kernel takes kChunk consecutive entries per block iteration (kEpt per thread, strided
// for coalescing): one staged byte range, one staged window of row offsets and keep flags, so the
// dependent global round trips (row lookup, keep, varint bytes) are paid once per chunk.
constexpr int kEpt = 4;
constexpr int64_t kChunk = (int64_t)kEpt * kBlock;
constexpr int kRowWin = 1024;

// block_row[k] = the row holding entry k * kChunk (one thread per row writes the boundaries inside it)
__global__ void block_rows_kernel(const int64_t* __restrict__ row_off, int64_t nrows, int64_t* __restrict__ block_row) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t hi = row_off[r + 1];
        for (int64_t b = (row_off[r] + kChunk - 1) / kChunk * kChunk; b < hi; b += kChunk) block_row[b / kChunk] = r;
    }
}

__global__ __launch_bounds__(kBlock) void edgestore_edges_kernel(EntryView a, const int64_t* __restrict__ row_off,
                                                                  const int64_t* __restrict__ block_row,
                                                                  int64_t nrows, int64_t nent,
                                                                  const uint8_t* __restrict__ keep,
                                                                  const int64_t* __restrict__ row_vid, int pbits,
                                                                  bool with_in, uint8_t* __restrict__ take,
                                                                  int64_t* __restrict__ src, int64_t* __restrict__ dst,
                                                                  int32_t* __restrict__ err) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kStageWords];
    __shared__ int64_t win_off[kRowWin + 1];
    __shared__ uint8_t win_keep[kRowWin];
    for (int64_t e0 = (int64_t)blockIdx.x * kChunk; e0 < nent; e0 += (int64_t)gridDim.x * kChunk) {
        const int64_t e_end = e0 + kChunk < nent ? e0 + kChunk : nent;
        const int64_t k = e0 / kChunk;
        const int64_t r0 = block_row[k], r1 = e_end < nent ? block_row[k + 1] + 1 : nrows;  // rows [r0, r1)
        const bool win = r1 - r0 <= kRowWin;
        if (win) {
            constexpr int kW = kRowWin / kBlock + 1;
            int64_t ro[kW];
            uint8_t kk[kW];
#pragma unroll
            for (int u = 0; u < kW; ++u) {
                const int64_t i = threadIdx.x + (int64_t)u * kBlock;
                if (i <= r1 - r0) ro[u] = row_off[r0 + i];
                if (i < r1 - r0) kk[u] = keep[r0 + i];
            }
#pragma unroll
            for (int u = 0; u < kW; ++u) {
                const int64_t i = threadIdx.x + (int64_t)u * kBlock;
                if (i <= r1 - r0) win_off[i] = ro[u];
                if (i < r1 - r0) win_keep[i] = kk[u];
            }
        }
        int64_t o[kEpt], o_next[kEpt];
        int32_t vp[kEpt];
#pragma unroll
        for (int j = 0; j < kEpt; ++j) {
            const int64_t e = e0 + threadIdx.x + (int64_t)j * kBlock;
            o[j] = e < e_end ? a.off[e] : 0;
            o_next[j] = e < e_end ? a.off[e + 1] : 0;
            vp[j] = e < e_end ? a.vpos[e] : 0;
        }
        const Stage st = stage_entries(a, e0, e_end, lds);  // synchronises the block when it stages
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kEpt; ++j) {  // unrolled: four decodes' loads in flight (measured 534 vs 614 us)
            const int64_t e = e0 + threadIdx.x + (int64_t)j * kBlock;
            if (e >= e_end) continue;
            int64_t r;
            uint8_t kp;
            if (win) {
                int64_t lo = 0, hi = r1 - r0;  // last window row with win_off[i] <= e
                while (hi - lo > 1) {
                    const int64_t mid = (lo + hi) >> 1;
                    if (win_off[mid] <= e) lo = mid; else hi = mid;
                }
                r = r0 + lo;
                kp = win_keep[lo];
            } else {
                r = row_of_entry(row_off, r0, r1, e);
                kp = keep[r];
            }
            uint8_t t = 0;
            if (kp) {
                const Decoded d = decode_entry(a, st.base + (o[j] - st.origin), o_next[j] - o[j], vp[j]);
                if (d.dir < 0) atomicOr(err, kErrMalformed);
                const int64_t other = pbits > 0 && d.dir >= 0 && is_partitioned(d.other, pbits)
                                          ? canonical_vertex_id(d.other, pbits) : d.other;
                if (d.dir == 0 && d.visible) {
                    t = 1;
                    src[e] = row_vid[r];
                    dst[e] = other;
                } else if (with_in && d.dir == 1 && d.visible) {  // the IN entry of edge other -> row
                    t = 2;
                    src[e] = other;
                    dst[e] = row_vid[r];
                }
            }
            take[e] = t;
        }
        __syncthreads();
    }
}

// ---- Fulgora's slice cap (jg_builder_set_query_limit) ----
// take[e] != 0 exactly for the entries of the EDGE slice on processed rows (visible user edges, both
// directions: the slice IDHandler.getBounds(EDGE) delimits).  pre = exclusive scan of that flag; an
// entry's rank in its row's slice is pre[e] - pre[row start].  A row whose slice holds more than
// `limit` entries marks the ones of rank >= limit (bit 2): the scan never returned them
// (SinglePageEntryBuffer.getSlice stops at the limit).  Rows reaching the limit are counted, as
// VertexJobConverter.process counts truncated-results (:139: entryList.size() >= limit).
__global__ void slice_flag_kernel(const uint8_t* __restrict__ take, int64_t n, uint32_t* __restrict__ f) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        f[i] = take[i] ? 1u : 0u;
}

__global__ __launch_bounds__(kBlock) void slice_cap_kernel(const int64_t* __restrict__ row_off, int64_t nrows,
                                                            const int64_t* __restrict__ pre, int64_t limit,
                                                            uint8_t* __restrict__ take,
                                                            unsigned long long* __restrict__ truncated) {
    for (int64_t r = blockIdx.x; r < nrows; r += gridDim.x) {  // block-uniform: one row per iteration
        const int64_t e0 = row_off[r], e1 = row_off[r + 1];
        const int64_t base = pre[e0], cnt = pre[e1] - base;
        if (cnt >= limit && threadIdx.x == 0) atomicAdd(truncated, 1ull);
        if (cnt <= limit) continue;
        for (int64_t e = e0 + threadIdx.x; e < e1; e += kBlock)
            if (take[e] && pre[e] - base >= limit) take[e] |= 4;
    }
}

// out_flag: OUT entries (every one: the uncapped list BOTH is built from); in_flag: IN entries within
// the cap
__global__ void split_flags_kernel(const uint8_t* __restrict__ take, int64_t n, uint8_t* __restrict__ out_flag,
                                   uint8_t* __restrict__ in_flag) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t t = take[i];
        out_flag[i] = t & 1;
        in_flag[i] = (t & 6) == 2 ? 1 : 0;
    }
}

// Narrow staging: off[i] += base (i <= n: off[n] is the scan's total), vpos[i] = the u8 position
__global__ void widen_entries_kernel(const uint8_t* __restrict__ vp8, int64_t n, int64_t base,
                                     int64_t* __restrict__ off, int32_t* __restrict__ vpos) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x) {
        if (base) off[i] += base;
        if (i < n) vpos[i] = vp8[i];
    }
}

// out[i] = in[idx[i]], or -1 where that OUT entry is beyond its row's cap
__global__ void capped_gather_kernel(const int64_t* __restrict__ in, const uint8_t* __restrict__ take,
                                     const int64_t* __restrict__ idx, int64_t n, int64_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = idx[i];
        out[i] = (take[e] & 4) ? -1 : in[e];
    }
}

template <typename T>
__global__ void gather_kernel(const T* __restrict__ in, const int64_t* __restrict__ idx, int64_t n, T* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = in[idx[i]];
}

}  // namespace

// Every entry inside the byte array, its value position inside the entry (checked before any launch).
static void check_entries(const uint8_t* bytes, int64_t nbytes, const int64_t* off, const int32_t* vpos, int64_t n) {
    if (n < 0 || nbytes < 0) fail(JG_ERR_ARG, "negative size");
    if (n > 0 && (!bytes || !off || !vpos)) fail(JG_ERR_ARG, "null entry arrays");
    for (int64_t e = 0; e < n; ++e) {
        const int64_t len = off[e + 1] - off[e];
        if (off[e] < 0 || len < 1 || off[e + 1] > nbytes || vpos[e] < 1 || vpos[e] > len)
            fail(JG_ERR_ARG, "entry " + std::to_string(e) + " out of range");
    }
}

// The multiplicity table sorted by type id, on the device.
struct TypeTable {
    DevBuf<int64_t> ids;
    DevBuf<int8_t> mult;
    int32_t n = 0;
    TypeTable(const int64_t* type_ids, const int8_t* type_mult, int32_t ntypes, hipStream_t s)
        : ids(std::max<int32_t>(ntypes, 1)), mult(std::max<int32_t>(ntypes, 1)), n(ntypes) {
        if (ntypes < 0) fail(JG_ERR_ARG, "negative size");
        if (ntypes > 0 && (!type_ids || !type_mult)) fail(JG_ERR_ARG, "null type table");
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
        if (ntypes) {
            copy_h2d(ids.get(), tid.data(), tid.size() * sizeof(int64_t), s);
            copy_h2d(mult.get(), tm.data(), tm.size(), s);
        }
    }
};

void decode_edges(Ctx& c, const uint8_t* bytes, int64_t nbytes, const int64_t* off, const int32_t* vpos, int64_t n,
                  const int64_t* type_ids, const int8_t* type_mult, int32_t ntypes, int64_t* type_out,
                  int8_t* dir_out, int64_t* other_out, int64_t* rel_out) {
    check_entries(bytes, nbytes, off, vpos, n);
    const int dev = c.devices.empty() ? 0 : c.devices[0];
    DeviceGuard dg(dev);
    hipStream_t s = c.streams.empty() ? nullptr : c.streams[0];
    TypeTable tt(type_ids, type_mult, ntypes, s);
    DevBuf<uint8_t> d_bytes(nbytes + kBytePad);
    DevBuf<int64_t> d_off(n + 1), d_type(std::max<int64_t>(n, 1)), d_other(std::max<int64_t>(n, 1)),
        d_rel(std::max<int64_t>(n, 1));
    DevBuf<int32_t> d_vpos(std::max<int64_t>(n, 1));
    DevBuf<int8_t> d_dir(std::max<int64_t>(n, 1));
    if (nbytes) copy_h2d(d_bytes.get(), bytes, (size_t)nbytes, s);
    if (n) {
        copy_h2d(d_off.get(), off, (size_t)(n + 1) * sizeof(int64_t), s);
        copy_h2d(d_vpos.get(), vpos, (size_t)n * sizeof(int32_t), s);
    }
    const EntryView a{d_bytes.get(), d_off.get(), d_vpos.get(), tt.ids.get(), tt.mult.get(), ntypes};
    const DecodeOut o{type_out ? d_type.get() : nullptr, dir_out ? d_dir.get() : nullptr,
                      other_out ? d_other.get() : nullptr, rel_out ? d_rel.get() : nullptr};
    hipEvent_t t0, t1;
    JG_HIP(hipEventCreate(&t0));
    JG_HIP(hipEventCreate(&t1));
    JG_HIP(hipEventRecord(t0, s));
    if (n > 0) {
        decode_edges_kernel<<<grid_for(n, kBlock, 256 * 64), kBlock, 0, s>>>(a, n, o);
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

// Host work over n items split into up to kHostThreads ranges: f(lo, hi, t) on threads of its own
// (the caller's thread takes range 0).  Staging a chunk is a few passes over memory the caller just
// wrote; one thread streams them at a fraction of the socket's bandwidth.
constexpr int kHostThreads = 8;
template <class F>
void parallel_ranges(int64_t n, int64_t grain, F f) {
    const int nt = (int)std::min<int64_t>(kHostThreads, std::max<int64_t>(1, n / std::max<int64_t>(grain, 1)));
    if (nt <= 1) {
        f((int64_t)0, n, 0);
        return;
    }
    std::vector<std::thread> ts;
    ts.reserve(nt - 1);
    for (int t = 1; t < nt; ++t) ts.emplace_back(f, n * t / nt, n * (t + 1) / nt, t);
    f((int64_t)0, n / nt, 0);
    for (auto& th : ts) th.join();
}

void copy_parallel(void* dst, const void* src, size_t bytes) {
    parallel_ranges((int64_t)bytes, (int64_t)4 << 20, [&](int64_t lo, int64_t hi, int) {
        std::memcpy((char*)dst + lo, (const char*)src + lo, (size_t)(hi - lo));
    });
}

// dst[i] = src[i] - base (offsets of a chunk cut out of larger arrays)
void copy_rebased(int64_t* dst, const int64_t* src, int64_t n, int64_t base) {
    if (base == 0) {
        copy_parallel(dst, src, (size_t)n * sizeof(int64_t));
        return;
    }
    parallel_ranges(n, (int64_t)1 << 18, [&](int64_t lo, int64_t hi, int) {
        for (int64_t i = lo; i < hi; ++i) dst[i] = src[i] - base;
    });
}

// The row arrays (the entries are validated while they are staged, EdgestoreDecoder::add).
static void check_rows(const EdgestoreRows& r) {
    if (r.nrows < 0 || r.nentries < 0 || r.nbytes < 0) fail(JG_ERR_ARG, "negative size");
    if (r.pbits < 0 || r.pbits > 16) fail(JG_ERR_ARG, "partition bits must be in [0, 16]");
    if (r.nrows > 0 && (!r.keys || !r.row_off)) fail(JG_ERR_ARG, "null row arrays");
    if (r.nentries > 0 && (!r.bytes || !r.entry_off || !r.vpos)) fail(JG_ERR_ARG, "null entry arrays");
    if (r.nrows == 0 ? r.nentries != 0
                     : (r.row_off[0] != r.entry_base || r.row_off[r.nrows] - r.entry_base != r.nentries))
        fail(JG_ERR_ARG, "row offsets must run from 0 to the entry count");
    for (int64_t i = 0; i < r.nrows; ++i)
        if (r.row_off[i + 1] < r.row_off[i]) fail(JG_ERR_ARG, "row offsets must be non-decreasing");
}

void edgestore_check(const EdgestoreRows& r) {
    check_rows(r);
    check_entries(r.bytes, r.nbytes, r.entry_off, r.vpos, r.nentries);
}

// ---- the snapshot decoder: chunks of rows, two in flight ----
// A chunk's arrays are staged in pinned host memory, so the call that adds it returns once they are
// copied there; the H2D copy and the two decode kernels then run on the chunk's stream while the caller
// scans the next chunk.  Completing a chunk (at the next add, or at finish) checks its error flags,
// compacts the kept rows and edges and appends them to the device accumulators.
struct EdgestoreChunk {
    int64_t R = 0, E = 0, nbytes = 0;
    PinnedBuf staging;
    DevBuf<uint8_t> d_bytes, keep, keep_v, take, out_flag, in_flag;
    DevBuf<int64_t> d_off, d_roff, row_vid, esrc, edst, block_row, pre;
    DevBuf<uint32_t> slice;
    DevBuf<unsigned long long> truncated;
    DevBuf<uint8_t> d_meta8;   // narrow staging: entry lengths then value positions
    DevBuf<int64_t> scan_tmp;  // scratch of the stream-ordered scans
    bool narrow = false;
    hipEvent_t tc = nullptr;   // after the chunk's copies
    DevBuf<uint64_t> d_keys;
    DevBuf<int32_t> d_vpos, err, d_w;
    bool weighted = false;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    bool pending = false;
};

namespace {
template <class T>
void grow_append(DevBuf<T>& acc, int64_t& len, const T* src, int64_t k, hipStream_t s) {
    if (k <= 0) return;
    if ((int64_t)acc.size() < len + k) {
        DevBuf<T> bigger(std::max<int64_t>(len + k, 2 * (int64_t)acc.size()));
        if (len) JG_HIP(hipMemcpyAsync(bigger.get(), acc.get(), (size_t)len * sizeof(T), hipMemcpyDeviceToDevice, s));
        acc.swap(bigger);
        JG_HIP(hipStreamSynchronize(s));  // the old buffer is freed on return
    }
    JG_HIP(hipMemcpyAsync(acc.get() + len, src, (size_t)k * sizeof(T), hipMemcpyDeviceToDevice, s));
    len += k;
}
}  // namespace

// Pinning host memory costs ~10 ms per 50 MB, more than staging a chunk.  Released staging buffers
// stay pinned in a small process-wide pool, so the next snapshot (the next computer run in the same
// JVM, the next build) reuses them.  The pool keeps only buffers of a regular chunk's size (a hub-row
// chunk's staging is freed) and at most kPoolTotalBytes together: a JVM that ran one GPU computer keeps
// ~2 chunk buffers page-locked, not gigabytes.  It is never torn down: the HIP runtime may be gone at exit.
namespace {
struct PinnedPool {
    std::mutex mu;
    std::vector<std::pair<void*, size_t>> free;
    size_t bytes = 0;
};
PinnedPool& pinned_pool() {
    static PinnedPool* pool = new PinnedPool();
    return *pool;
}
constexpr size_t kPoolMaxBytes = (size_t)160 << 20;    // one regular chunk's staging (64 MB bytes + metadata, +25%)
constexpr size_t kPoolTotalBytes = (size_t)320 << 20;  // the two chunks the decoder keeps in flight
void pinned_release(void* p, size_t cap) {
    if (!p) return;
    PinnedPool& pool = pinned_pool();
    {
        std::lock_guard<std::mutex> lk(pool.mu);
        if (cap <= kPoolMaxBytes && pool.bytes + cap <= kPoolTotalBytes) {
            pool.free.emplace_back(p, cap);
            pool.bytes += cap;
            return;
        }
    }
    (void)hipHostFree(p);
}
}  // namespace

PinnedBuf::~PinnedBuf() { pinned_release(p, cap); }

void PinnedBuf::reserve(size_t n) {
    if (n <= cap) return;
    pinned_release(p, cap);
    p = nullptr;
    cap = 0;
    {  // the smallest pooled buffer that fits
        PinnedPool& pool = pinned_pool();
        std::lock_guard<std::mutex> lk(pool.mu);
        size_t best = pool.free.size();
        for (size_t i = 0; i < pool.free.size(); ++i)
            if (pool.free[i].second >= n && (best == pool.free.size() || pool.free[i].second < pool.free[best].second))
                best = i;
        if (best < pool.free.size()) {
            p = pool.free[best].first;
            cap = pool.free[best].second;
            pool.bytes -= cap;
            pool.free.erase(pool.free.begin() + (std::ptrdiff_t)best);
            return;
        }
    }
    n = std::max<size_t>(n + n / 4, (size_t)1 << 20);  // headroom: chunks vary a little in size
    if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        p = nullptr;
        fail(JG_ERR_OOM, "pinned host allocation of " + std::to_string(n) + " bytes failed");
    }
    cap = n;
}

EdgestoreDecoder::EdgestoreDecoder(const int64_t* type_ids, const int8_t* type_mult, int32_t ntypes, int pbits,
                                   int device)
    : pbits_(pbits), device_(device) {
    if (pbits < 0 || pbits > 16) fail(JG_ERR_ARG, "partition bits must be in [0, 16]");
    DeviceGuard dg(device_);
    for (int i = 0; i < 2; ++i) {
        JG_HIP(hipStreamCreateWithFlags(&streams_[i], hipStreamNonBlocking));
        chunks_[i] = std::make_unique<EdgestoreChunk>();
        JG_HIP(hipEventCreate(&chunks_[i]->t0));
        JG_HIP(hipEventCreate(&chunks_[i]->t1));
        JG_HIP(hipEventCreate(&chunks_[i]->tc));
    }
    types_ = std::make_unique<TypeTable>(type_ids, type_mult, ntypes, streams_[0]);
}

void EdgestoreDecoder::set_weight_key(int64_t key, const int64_t* ids, const int8_t* types, int32_t n) {
    if (chunks_added_) fail(JG_ERR_STATE, "the weight key must be set before the first chunk");
    if (key < 0 || n < 0 || (n && (!ids || !types))) fail(JG_ERR_ARG, "bad weight key arguments");
    std::vector<std::pair<int64_t, int8_t>> t((size_t)n);
    for (int32_t i = 0; i < n; ++i) t[i] = {ids[i], types[i]};
    std::sort(t.begin(), t.end());
    std::vector<int64_t> hid((size_t)std::max(n, 1));
    std::vector<int8_t> hty((size_t)std::max(n, 1));
    wschema_ = WeightSchema{};
    wschema_.key = key;
    for (int32_t i = 0; i < n; ++i) {
        if (i && t[i].first == t[i - 1].first) fail(JG_ERR_ARG, "duplicate property key id");
        hid[i] = t[i].first;
        hty[i] = t[i].second;
        if (t[i].first == key) wschema_.key_type = t[i].second;
    }
    if (wschema_.key_type != JG_PROP_INT) wschema_.key = -1;  // no Integer weight on any edge: all absent
    wschema_.n = n;
    DeviceGuard dg(device_);
    wkeys_.alloc(std::max(n, 1));
    wtypes_.alloc(std::max(n, 1));
    copy_h2d(wkeys_.get(), hid.data(), hid.size() * sizeof(int64_t), streams_[0]);
    copy_h2d(wtypes_.get(), hty.data(), hty.size() * sizeof(int8_t), streams_[0]);
    weight_key_set_ = true;
}

EdgestoreDecoder::~EdgestoreDecoder() {
    DeviceGuard dg(device_);
    for (int i = 0; i < 2; ++i) {
        if (streams_[i]) (void)hipStreamSynchronize(streams_[i]);
        if (chunks_[i]) {
            (void)hipEventDestroy(chunks_[i]->t0);
            (void)hipEventDestroy(chunks_[i]->t1);
            (void)hipEventDestroy(chunks_[i]->tc);
        }
        chunks_[i].reset();
        if (streams_[i]) (void)hipStreamDestroy(streams_[i]);
    }
}

namespace {
using HostClock = std::chrono::steady_clock;
double ms_since(HostClock::time_point t) {
    return std::chrono::duration<double, std::milli>(HostClock::now() - t).count();
}
bool decode_trace() {
    static const bool on = std::getenv("JG_DECODE_TRACE") != nullptr;
    return on;
}
}  // namespace

void EdgestoreDecoder::add(const EdgestoreRows& r) {
    const auto h0 = HostClock::now();
    check_rows(r);
    const bool dev_w = weight_key_set_;  // weights decoded here from the rows (set_weight_key; key -1: all absent)
    if (dev_w && r.weight) fail(JG_ERR_ARG, "entry weights given while the weight key decodes them on the GPU");
    const int wmode = (r.weight || dev_w) ? 1 : 0;
    if (weighted >= 0 && weighted != wmode) fail(JG_ERR_ARG, "entry weights must be given for every chunk or none");
    weighted = wmode;
    DeviceGuard dg(device_);
    const int slot = next_;
    next_ ^= 1;
    EdgestoreChunk& c = *chunks_[slot];
    const auto h1 = HostClock::now();
    if (c.pending) complete(slot);  // its buffers are reused below
    const double t_complete = ms_since(h1);
    hipStream_t s = streams_[slot];
    const int64_t R = r.nrows, E = r.nentries;
    c.R = R;
    c.E = E;
    c.nbytes = r.nbytes;
    // Staging layout (pinned), in the order the copies go out:
    //   narrow (every entry < 256 bytes, the usual case): len [E] u8 | vpos [E] u8 | ...
    //   wide: off [E+1] i64 | vpos [E] i32 | ...
    //   ... | roff [R+1] i64 | keys [R] u64 | weight [E] i32 (optional) | bytes
    // Narrow entries cross PCIe with 2 bytes of offsets and value positions instead of 12; the device
    // rebuilds the offsets with a scan of the lengths.
    // One parallel pass validates every entry (inside the bytes, value position within it) and writes
    // the narrow metadata; a chunk with a long entry is then staged wide instead.
    const size_t narrow_meta = (size_t)E * 2, wide_meta = (size_t)(E + 1) * 8 + (size_t)E * 4;
    const size_t tail = (size_t)(R + 1) * 8 + (size_t)R * 8 + (r.weight ? (size_t)E * 4 : 0) + (size_t)r.nbytes + 1;
    const auto h2 = HostClock::now();
    c.staging.reserve(narrow_meta + tail);
    const double t_reserve = ms_since(h2);
    const auto h3 = HostClock::now();
    int64_t bad[kHostThreads];
    bool wide[kHostThreads];
    for (int t = 0; t < kHostThreads; ++t) {
        bad[t] = -1;
        wide[t] = false;
    }
    {
        uint8_t* len8 = (uint8_t*)c.staging.p;
        uint8_t* vp8 = len8 + E;
        const int64_t* off = r.entry_off;
        const int32_t* vpos = r.vpos;
        const int64_t nbytes = r.nbytes, b0 = r.byte_base;
        parallel_ranges(E, (int64_t)1 << 18, [&](int64_t lo, int64_t hi, int t) {
            bool w = false;
            for (int64_t e = lo; e < hi; ++e) {
                const int64_t o0 = off[e] - b0, o1 = off[e + 1] - b0, len = o1 - o0;
                const int32_t vp = vpos[e];
                if (o0 < 0 || len < 1 || o1 > nbytes || vp < 1 || vp > len) {
                    bad[t] = e;
                    return;
                }
                if (len >= 256) w = true;
                len8[e] = (uint8_t)len;
                vp8[e] = (uint8_t)vp;
            }
            wide[t] = w;
        });
    }
    bool narrow = true;
    for (int t = 0; t < kHostThreads; ++t) {
        if (bad[t] >= 0) fail(JG_ERR_ARG, "entry " + std::to_string(bad[t]) + " out of range");
        narrow = narrow && !wide[t];
    }
    c.narrow = narrow;
    const size_t meta = narrow ? narrow_meta : wide_meta;
    const size_t o_roff = meta, o_keys = o_roff + (size_t)(R + 1) * 8, o_w = o_keys + (size_t)R * 8,
                 o_bytes = o_w + (r.weight ? (size_t)E * 4 : 0);
    c.weighted = r.weight != nullptr || dev_w;
    if (!narrow) c.staging.reserve(meta + tail);  // rare: a chunk holding an entry of 256 bytes or more
    char* st = (char*)c.staging.p;
    if (!narrow) {
        copy_rebased(reinterpret_cast<int64_t*>(st), r.entry_off, E + 1, r.byte_base);
        if (E) copy_parallel(st + (size_t)(E + 1) * 8, r.vpos, (size_t)E * 4);
    }
    if (R) {
        copy_rebased(reinterpret_cast<int64_t*>(st + o_roff), r.row_off, R + 1, r.entry_base);
        copy_parallel(st + o_keys, r.keys, (size_t)R * 8);
    }
    if (E && r.weight) copy_parallel(st + o_w, r.weight, (size_t)E * 4);
    if (r.nbytes) copy_parallel(st + o_bytes, r.bytes, (size_t)r.nbytes);
    const double t_stage = ms_since(h3);
    const auto h4 = HostClock::now();
    auto fit = [](auto& buf, int64_t n) {
        if ((int64_t)buf.size() < std::max<int64_t>(n, 1)) buf.alloc(std::max<int64_t>(n, 1));
    };
    fit(c.d_bytes, r.nbytes + kBytePad);
    fit(c.keep, R);
    fit(c.keep_v, R);
    fit(c.take, E);
    fit(c.d_off, E + 1);
    fit(c.d_roff, R + 1);
    fit(c.row_vid, R);
    fit(c.esrc, E);
    fit(c.edst, E);
    fit(c.block_row, (E + kChunk - 1) / kChunk + 1);
    fit(c.d_keys, R);
    fit(c.d_vpos, E);
    fit(c.err, 1);
    if (c.weighted) fit(c.d_w, E);
    if (narrow) fit(c.d_meta8, 2 * E);
    const bool capped = limit_ > 0;
    if (capped) {
        fit(c.slice, E);
        fit(c.pre, E + 1);  // the scan of E flags writes pre[0..E]; pre[E] = total (read at pre[row_off[R]])
        fit(c.out_flag, E);
        fit(c.in_flag, E);
        fit(c.truncated, 1);
    }
    if (narrow || capped) fit(c.scan_tmp, prim::scan_scratch_size(E + 1));
    auto h2d = [&](void* d, size_t off, size_t bytes) {
        if (bytes) JG_HIP(hipMemcpyAsync(d, st + off, bytes, hipMemcpyHostToDevice, s));
    };
    JG_HIP(hipEventRecord(c.t0, s));
    if (narrow) {
        h2d(c.d_meta8.get(), 0, (size_t)E * 2);
    } else {
        h2d(c.d_off.get(), 0, (size_t)(E + 1) * 8);
        h2d(c.d_vpos.get(), (size_t)(E + 1) * 8, (size_t)E * 4);
    }
    h2d(c.d_roff.get(), o_roff, (size_t)(R + 1) * 8);
    h2d(c.d_keys.get(), o_keys, (size_t)R * 8);
    if (r.weight) h2d(c.d_w.get(), o_w, (size_t)E * 4);
    h2d(c.d_bytes.get(), o_bytes, (size_t)r.nbytes);
    JG_HIP(hipEventRecord(c.tc, s));
    JG_HIP(hipMemsetAsync(c.err.get(), 0, sizeof(int32_t), s));
    if (narrow) {  // off = entry_off[0] + exclusive scan of the lengths; value positions widened
        prim::exclusive_scan_async(c.d_meta8.get(), c.d_off.get(), E, c.scan_tmp.get(), s);
        if (E) {
            widen_entries_kernel<<<grid_for(E + 1), kBlock, 0, s>>>(c.d_meta8.get() + E, E, r.entry_off[0] - r.byte_base,
                                                                  c.d_off.get(), c.d_vpos.get());
            JG_LAUNCH_CHECK();
        }
    }
    const EntryView a{c.d_bytes.get(), c.d_off.get(), c.d_vpos.get(), types_->ids.get(), types_->mult.get(), types_->n};
    if (dev_w && E) {
        WeightSchema w = wschema_;
        w.ids = wkeys_.get();
        w.types = wtypes_.get();
        edgestore_weight_kernel<<<grid_for(E), kBlock, 0, s>>>(a, E, w, c.d_w.get(), c.err.get());
        JG_LAUNCH_CHECK();
    }
    if (R) {
        edgestore_rows_kernel<<<grid_for(R), kBlock, 0, s>>>(a, c.d_keys.get(), c.d_roff.get(), R, pbits_, c.keep.get(),
                                                            c.keep_v.get(), c.row_vid.get(), c.err.get());
        JG_LAUNCH_CHECK();
    }
    if (E) {
        block_rows_kernel<<<grid_for(R), kBlock, 0, s>>>(c.d_roff.get(), R, c.block_row.get());
        JG_LAUNCH_CHECK();
        edgestore_edges_kernel<<<grid_for((E + kEpt - 1) / kEpt, kBlock, 256 * 16), kBlock, 0, s>>>(
            a, c.d_roff.get(), c.block_row.get(), R, E, c.keep.get(), c.row_vid.get(), pbits_, capped, c.take.get(),
            c.esrc.get(), c.edst.get(), c.err.get());
        JG_LAUNCH_CHECK();
    }
    if (capped) {
        JG_HIP(hipMemsetAsync(c.truncated.get(), 0, sizeof(unsigned long long), s));
        if (E) {
            slice_flag_kernel<<<grid_for(E), kBlock, 0, s>>>(c.take.get(), E, c.slice.get());
            JG_LAUNCH_CHECK();
        }
        prim::exclusive_scan_async(c.slice.get(), c.pre.get(), E, c.scan_tmp.get(), s);
        if (R) {
            slice_cap_kernel<<<(unsigned)std::min<int64_t>(R, 4096), kBlock, 0, s>>>(c.d_roff.get(), R, c.pre.get(),
                                                                                     limit_, c.take.get(),
                                                                                     c.truncated.get());
            JG_LAUNCH_CHECK();
        }
    }
    JG_HIP(hipEventRecord(c.t1, s));
    c.pending = true;
    ++chunks_added_;
    rows_ += R;
    entries_ += E;
    bytes_ += r.nbytes;
    h2d_bytes_ += (int64_t)(o_bytes + (size_t)r.nbytes);
    if (decode_trace())
        std::fprintf(stderr, "[jg decode] chunk %lld: R %lld E %lld bytes %lld | host ms: total %.2f complete(prev) %.2f "
                             "pinned reserve %.2f stage %.2f launch %.2f\n",
                     (long long)chunks_added_, (long long)R, (long long)E, (long long)r.nbytes, ms_since(h0),
                     t_complete, t_reserve, t_stage, ms_since(h4));
}

void EdgestoreDecoder::complete(int slot) {
    EdgestoreChunk& c = *chunks_[slot];
    if (!c.pending) return;
    c.pending = false;
    hipStream_t s = streams_[slot];
    int32_t herr = 0;
    JG_HIP(hipMemcpyAsync(&herr, c.err.get(), sizeof(int32_t), hipMemcpyDeviceToHost, s));
    JG_HIP(hipStreamSynchronize(s));
    float ms = 0, cms = 0;
    JG_HIP(hipEventElapsedTime(&ms, c.t0, c.t1));
    JG_HIP(hipEventElapsedTime(&cms, c.t0, c.tc));
    kernel_ms += ms;  // copy + decode of the chunk
    copy_ms += cms;
    if (herr & kErrBadKey) fail(JG_ERR_ARG, "row key with an unrecognized vertex id type");
    if (herr & kErrPartitioned) fail(JG_ERR_ARG, "partitioned vertex row with no partition bits");
    if (herr & kErrMalformed) fail(JG_ERR_ARG, "malformed edgestore entry on a vertex row");
    if (herr & kErrWeightType)
        fail(JG_ERR_UNSUPPORTED, "an edge carries a property of unknown type before the weight key");
    if (herr & kErrWeightValue)
        fail(JG_ERR_UNSUPPORTED, "an edge weight equals Integer.MIN_VALUE (the absent-weight marker)");
    const int64_t cap = std::max<int64_t>(std::max(c.R, c.E), 1);
    if ((int64_t)idx_.size() < cap) idx_.alloc(cap);
    if ((int64_t)tmp_.size() < cap) tmp_.alloc(cap);
    if (c.weighted && (int64_t)tmpw_.size() < cap) tmpw_.alloc(cap);
    const int64_t nk = prim::compact_indices(c.keep_v.get(), c.R, idx_.get(), cpos_, cscan_, s);
    if (nk) {
        gather_kernel<int64_t><<<grid_for(nk), kBlock, 0, s>>>(c.row_vid.get(), idx_.get(), nk, tmp_.get());
        JG_LAUNCH_CHECK();
        grow_append(vid, n, tmp_.get(), nk, s);
    }
    const bool capped = limit_ > 0;
    if (capped && c.E) {
        split_flags_kernel<<<grid_for(c.E), kBlock, 0, s>>>(c.take.get(), c.E, c.out_flag.get(), c.in_flag.get());
        JG_LAUNCH_CHECK();
    }
    if (capped) {
        unsigned long long tr = 0;
        JG_HIP(hipMemcpyAsync(&tr, c.truncated.get(), sizeof tr, hipMemcpyDeviceToHost, s));
        JG_HIP(hipStreamSynchronize(s));
        truncated_rows += (int64_t)tr;
        const int64_t ki = prim::compact_indices(c.in_flag.get(), c.E, idx_.get(), cpos_, cscan_, s);
        if (ki) {
            int64_t m2 = mi;
            gather_kernel<int64_t><<<grid_for(ki), kBlock, 0, s>>>(c.esrc.get(), idx_.get(), ki, tmp_.get());
            JG_LAUNCH_CHECK();
            grow_append(isrc, mi, tmp_.get(), ki, s);
            gather_kernel<int64_t><<<grid_for(ki), kBlock, 0, s>>>(c.edst.get(), idx_.get(), ki, tmp_.get());
            JG_LAUNCH_CHECK();
            grow_append(idst, m2, tmp_.get(), ki, s);
        }
    }
    const int64_t mk = prim::compact_indices(capped ? c.out_flag.get() : c.take.get(), c.E, idx_.get(), cpos_, cscan_, s);
    if (mk) {
        if (capped) {  // the capped OUT list: the same edges, -1 sources beyond the cap
            capped_gather_kernel<<<grid_for(mk), kBlock, 0, s>>>(c.esrc.get(), c.take.get(), idx_.get(), mk, tmp_.get());
            JG_LAUNCH_CHECK();
            grow_append(osrc, mo, tmp_.get(), mk, s);
        }
        int64_t m2 = m;
        gather_kernel<int64_t><<<grid_for(mk), kBlock, 0, s>>>(c.esrc.get(), idx_.get(), mk, tmp_.get());
        JG_LAUNCH_CHECK();
        grow_append(src, m, tmp_.get(), mk, s);
        gather_kernel<int64_t><<<grid_for(mk), kBlock, 0, s>>>(c.edst.get(), idx_.get(), mk, tmp_.get());
        JG_LAUNCH_CHECK();
        grow_append(dst, m2, tmp_.get(), mk, s);
        if (c.weighted) {  // kept entries are edges: their weights follow the same compaction
            gather_kernel<int32_t><<<grid_for(mk), kBlock, 0, s>>>(c.d_w.get(), idx_.get(), mk, tmpw_.get());
            JG_LAUNCH_CHECK();
            grow_append(w, mw, tmpw_.get(), mk, s);
        }
    }
    JG_HIP(hipStreamSynchronize(s));
}

void EdgestoreDecoder::finish() {
    DeviceGuard dg(device_);
    const auto h0 = HostClock::now();
    // chunks complete in the order they were added
    complete(next_);
    complete(next_ ^ 1);
    if (decode_trace()) std::fprintf(stderr, "[jg decode] finish: last chunks completed in %.2f ms\n", ms_since(h0));
}

void add_in_chunks(EdgestoreDecoder& dec, const EdgestoreRows& r) {
    check_rows(r);
    constexpr int64_t kChunkEntries = (int64_t)4 << 20, kChunkBytes = (int64_t)64 << 20;
    // chunk boundaries are cut at entry offsets: the first and last must lie inside the bytes (each
    // chunk then checks its own entries)
    if (r.nentries > 0 && (r.entry_off[0] < 0 || r.entry_off[r.nentries] > r.nbytes))
        fail(JG_ERR_ARG, "entry offsets run outside the byte array");
    const bool has_entries = r.nentries > 0;
    int64_t lo = 0;
    while (lo < r.nrows || (lo == 0 && r.nrows == 0)) {
        int64_t hi = lo + 1;
        const int64_t e0 = r.nrows ? r.row_off[lo] : 0;
        while (hi < r.nrows && r.row_off[hi + 1] - e0 <= kChunkEntries &&
               (!has_entries || r.entry_off[r.row_off[hi + 1]] - r.entry_off[e0] <= kChunkBytes))
            ++hi;
        if (r.nrows == 0) hi = 0;
        EdgestoreRows c = r;
        c.keys = r.keys + lo;
        c.nrows = hi - lo;
        c.row_off = r.row_off + lo;
        c.entry_base = e0;
        const int64_t e1 = r.nrows ? r.row_off[hi] : 0;
        c.nentries = e1 - e0;
        c.entry_off = has_entries ? r.entry_off + e0 : r.entry_off;
        c.vpos = has_entries ? r.vpos + e0 : r.vpos;
        c.byte_base = has_entries ? r.entry_off[e0] : 0;
        c.bytes = has_entries ? r.bytes + c.byte_base : r.bytes;
        c.nbytes = has_entries ? r.entry_off[e1] - c.byte_base : 0;
        if (r.weight) c.weight = r.weight + e0;
        dec.add(c);
        if (r.nrows == 0) break;
        lo = hi;
    }
}

void edgestore_snapshot(const EdgestoreRows& r, int device, DevBuf<int64_t>& vid, int64_t& n, DevBuf<int64_t>& src,
                        DevBuf<int64_t>& dst, int64_t& m, float* kernel_ms) {
    EdgestoreDecoder dec(r.type_ids, r.type_mult, r.ntypes, r.pbits, device);
    add_in_chunks(dec, r);
    dec.finish();
    vid.swap(dec.vid);
    src.swap(dec.src);
    dst.swap(dec.dst);
    n = dec.n;
    m = dec.m;
    if (kernel_ms) *kernel_ms = dec.kernel_ms;
}

}  // namespace jg
