// jg_internal.h — contexts, shards and graphs of libjanusgpu.
//
// HBM layout (per shard = per GPU or logical partition):
//   vertices are relabelled once at build time: sorted by degree (descending; the degree of the
//   adjacency the programs pull over) and dealt round-robin to the P shards, so every shard owns
//   S = ceil(n/P) rows whose degrees are sorted inside the shard.  A vertex's global id is
//   g = shard * S + local; every full-length vertex vector is P*S long, laid out shard-major, so an
//   in-place allgather of the owned slices IS the exchange step (RCCL over xGMI).
//   Csr: row_ptr int64 [rows+1], col int32 [nnz] (global ids), optional weight int32 [nnz].
//   Pull programs stream col once per superstep and gather the source vector at col.
//   Sharded (P > 1, tune halo = 1): the pull adjacencies (IN, BOTH) instead hold COMPACT column ids:
//   each shard's gathered vector holds its own rows, then one segment per peer with just the peer's
//   vertices its rows read (CompactMap), each in degree order, so every segment's hottest entries are
//   its prefix.  The exchange step is a sparse halo exchange (pack, RCCL send/recv per peer straight
//   into the peer's segment) of the values each peer actually reads — ~21% of the dense allgather
//   for RMAT-24 at P = 8.
#pragma once

#include <algorithm>
#include <memory>
#include <atomic>
#include <mutex>
#include <functional>
#include <vector>

#include "jg_common.h"
#include "janusgpu.h"

#include <rccl/rccl.h>

namespace jg {

struct Csr {
    int64_t rows = 0;
    int64_t nnz = 0;
    DevBuf<int64_t> row_ptr;
    DevBuf<int32_t> col;
    DevBuf<int32_t> weight;  // optional (SD weights)
    // rows [empty_from, rows) have no entries (set with the pull plan: 1 + the last non-empty row;
    // -1 when unknown)
    mutable int64_t empty_from = -1;
    // each row's first column (-1: empty row), built on a traversal's first use (bfs_first_col): a
    // bottom-up level probes it with one coalesced load instead of a row_ptr pair and a scattered column
    mutable DevBuf<int32_t> first_col;
    // weight statistics (smallest, sum, count of the non-absent weights), computed on the first weighted
    // shortest distance that needs them (sd_weight_stats)
    mutable long long wstat[4] = {0, 0, 0, 0};  // sd_weight_stats: min, sum, count, max
    mutable bool wstat_ok = false;
    bool present() const { return row_ptr.size() > 0; }
    int64_t bytes() const { return (int64_t)(row_ptr.bytes() + col.bytes() + weight.bytes()); }
};

// Degree-class plan for the pull kernels of one CSR on one shard.  Rows are sorted by degree
// (descending), so each class is a contiguous row range.
constexpr int kNumClasses = 9;  // 0: hub (chunked), 1..7: lanes per row 64,32,16,8,4,2,1, 8: empty rows
constexpr int kZeroClass = kNumClasses - 1;
constexpr int64_t kHubDegree = 8192;
constexpr int kRunMax = 7;  // light rows of degree 1..kRunMax may be addressed by degree run (PullPlan::runs)
constexpr int64_t kHubChunk = 4096;

// One degree band of the sliced split: rows [row_begin, row_end), whose entries are dealt to
// S = 2^bits sub-slices by sub_slice() (sub-slice h belongs to XCD h mod 8).  Each sub-slice is a
// sub-CSR over the band's rows (entries slice-major in `col`, every sub-slice's start aligned to a
// merge task) folded merge-path style in tasks of kMergeTask entries.  Non-empty sub-rows (h, r) are
// numbered sub-slice-major: their partial slot (part_off + number); task carries follow at carry_off.
struct SliceBand {
    int bits = 3;
    int64_t row_begin = 0, row_end = 0;
    int64_t tasks = 0;      // merge tasks over all sub-slices
    int64_t subrows = 0;    // non-empty sub-rows
    int64_t part_off = 0;   // offset of the band's partials in the program's fold buffer
    int64_t carry_off = 0;  // offset of the band's task carries
    DevBuf<int32_t> col;        // entries, sub-slice-major (+ one task of padding); freed once packed
    // The entries as the merge kernel streams them: lane chunk x = entries [8x, 8x + 8) of `col`, each
    // as its sub-slice-local index loc = (c >> (4 + bits)) << 4 | (c & 15) (the sub-slice's hash bits
    // of the line dropped; SliceBand::decode restores them), packed in `width` bits (20, 24 or 32:
    // the fewest that hold the vector's largest loc) as a bit stream over width / 4 dwords, planar:
    // dwords 0..3 in pack_a[x], the rest in pack_b[x * (width / 4 - 4) ...].  RMAT-26 band 0: 20 bits.
    int width = 32;
    DevBuf<uint4> pack_a;
    DevBuf<uint32_t> pack_b;
    DevBuf<int64_t> sub_begin;  // [S] first entry of sub-slice h in col (aligned)
    DevBuf<int64_t> sub_end;    // [S] one past its last entry
    DevBuf<int64_t> sub_base;   // [S+1] first task of sub-slice h
    DevBuf<uint8_t> heads;      // [tasks][64]: byte l = row-start bits of lane l's entries
    DevBuf<int32_t> meta;       // [tasks][2]: sub-row number of the task's first entry; 1 if it is a carry
    // non-empty sub-rows, numbered sub-slice-major: for w = sub_word[h][i>>5], bit i&31 of w.x says
    // whether band row i has entries in sub-slice h; its number is w.y + the set bits of w.x below it
    DevBuf<uint2> sub_word;     // [S][words], words = ceil(rows of the band / 32)
    DevBuf<int32_t> task_rows;  // [tasks][2]: band rows of the task's first and last entry
    int64_t rows() const { return row_end - row_begin; }
};

struct PullPlan {
    int64_t class_row_begin[kNumClasses];
    int64_t class_row_end[kNumClasses];
    int64_t class_block_begin[kNumClasses + 1];  // hub: one block per chunk
    int64_t num_hub_rows = 0;
    int64_t max_hub_row = -1;    // hub rows need not be a prefix (rows follow the relabel's degree)
    int64_t num_chunks = 0;
    DevBuf<int64_t> chunk_row;    // [num_chunks] local row of each hub chunk
    DevBuf<int64_t> chunk_begin;  // [num_chunks] first entry (CSR position)
    DevBuf<int64_t> chunk_end;    // [num_chunks]
    DevBuf<int64_t> hub_chunk_ptr;  // [num_hub_rows+1] chunks of hub row r: [ptr[r], ptr[r+1])
    int64_t total_blocks() const { return class_block_begin[kNumClasses]; }

    // XCD-sliced split of the heavy rows [0, split_rows) of a CSR, in degree bands (rows are
    // degree-sorted, so every band is a row range): see SliceBand and pull_merge_kernel (jg_pull.h).
    // The light rows keep the degree classes above (the light_* table covers [split_rows, rows)).
    int64_t split_rows = 0;
    int64_t col_space = 0;     // length of the gathered vector
    int64_t light_row_begin[kNumClasses] = {};  // the class table of rows [split_rows, rows)
    int64_t light_row_end[kNumClasses] = {};
    int64_t light_block_begin[kNumClasses + 1] = {};
    std::vector<std::unique_ptr<SliceBand>> bands;
    // program-owned fold buffer: per band [subrows] sub-row partials + [tasks] task carries
    int64_t split_partial_len() const {
        int64_t n = 0;
        for (const auto& b : bands) n += b->subrows + b->tasks;
        return std::max<int64_t>(n, 1);
    }
    bool lds_ok = false;  // the gathered vector's hot entries are segment prefixes (see seg_tbits)
    bool temporal = false;  // the vector is large enough for the temporal merge schedule (tune merge_temporal = 1)
    int seg_tbits = 31;   // segmented compact vector (sharded, halo): nseg segments of stride 2^seg_tbits
    int nseg = 1;         // one segment: the hot prefix is [0, hot)
    // Degree runs of the light rows: when rows [run_begin[kRunMax], zero rows) hold degrees
    // kRunMax, ..., 1 in non-increasing order (a degree-sorted shard), rows of degree d are
    // [run_begin[d], run_begin[d-1]) (run_begin[0] = first empty row) and row r of that run starts at
    // run_ptr[d] + (r - run_begin[d]) * d: the 1-lane class needs no row_ptr load.
    bool runs = false;
    int64_t run_begin[kRunMax + 1] = {};
    int64_t run_ptr[kRunMax + 1] = {};
};
constexpr int kXcds = 8;
// Sub-slices of the column space: the 128-byte lines of an fp64 vector (16 elements) are hashed to
// 8 bits (xor of the line index's byte groups); a band of 2^b sub-slices uses the low b bits, and
// sub-slice h belongs to XCD h mod 8.  Inside any aligned group of 2^b lines the hash is a
// permutation (low bits xor a constant of the group), so every sub-slice holds an equal share of
// every hot region and one XCD's L2 only ever caches its own eighth of the gathered vector.  Rows
// of a sliced CSR order their entries by (sub_key, col): sub_key is the bit-reversed hash, so the
// entries of every sub-slice of every band are contiguous in the row.
constexpr int kMergeTask = 512;  // entries per merge task of the sliced split (one wave, 8 per lane)
__host__ __device__ __forceinline__ uint32_t sub_hash(int64_t c) {
    const uint32_t x = (uint32_t)(c >> 4);
    return (x ^ (x >> 8) ^ (x >> 16) ^ (x >> 24)) & 255u;
}
__host__ __device__ __forceinline__ uint32_t brev_bits(uint32_t v, int bits) {
    uint32_t r = 0;
    for (int i = 0; i < bits; ++i) r |= ((v >> i) & 1u) << (bits - 1 - i);
    return r;
}
__host__ __device__ __forceinline__ uint32_t sub_key(int64_t c) { return brev_bits(sub_hash(c), 8); }
__host__ __device__ __forceinline__ int sub_slice(int64_t c, int bits) { return (int)(sub_hash(c) & ((1u << bits) - 1)); }

struct Ctx;

// Compact column ids of one shard's pull adjacency (sharded graphs).  The gathered vector is cut
// into P segments of stride T = 2^tbits: segment 0 holds the shard's own rows [0, rows), segment
// s(q) = q < r ? q + 1 : q the vertices of peer q that this shard reads, in the peer's local (degree)
// order — exactly the run peer q sends, so it is received in place.  Every segment's hottest entries
// are its prefix.
struct CompactMap {
    const uint32_t* bits = nullptr;   // [ceil(P*S/32)] needed remote vertices by global id
    const int64_t* off = nullptr;     // [words + 1] exclusive popcount prefix of bits
    const int64_t* qbase = nullptr;   // [P + 1] popcount prefix at q * S
    int64_t S = 0;
    int r = 0, tbits = 31;
    __host__ __device__ bool on() const { return bits != nullptr; }
    __device__ __forceinline__ int32_t operator()(int64_t g) const {
        const int64_t q = g / S, l = g - q * S;
        if (q == r) return (int32_t)l;
        const uint32_t w = bits[g >> 5];
        const int64_t rank = off[g >> 5] + __popc(w & ((1u << (g & 31)) - 1u)) - qbase[q];
        return (int32_t)(((q < r ? q + 1 : q) << tbits) + rank);
    }
};

// Halo plan of one shard's pull adjacency: which of its own values each peer reads (send lists, by
// peer, ascending local ids) and how many values it reads from each peer (landing at the peer's
// segment).  The lists are static, so a superstep moves values only, no indices.
struct Halo {
    bool on = false;
    int tbits = 31;                      // segment stride 2^tbits
    int64_t C = 0;                       // gathered vector length: P segments
    DevBuf<uint32_t> bits;               // CompactMap storage
    DevBuf<int64_t> off, qbase;
    DevBuf<int32_t> send_src;            // [send_off[P]] own rows packed for the peers, by peer
    std::vector<int64_t> send_off, recv_off;  // [P + 1] element offsets per peer
    DevBuf<uint64_t> send_buf;           // 8-byte scratch elements (4-byte vectors use half)
    int seg_of(int q, int r) const { return q < r ? q + 1 : q; }
    CompactMap map(int64_t S, int r) const {
        CompactMap m;
        if (on) { m.bits = bits.get(); m.off = off.get(); m.qbase = qbase.get(); m.S = S; m.r = r; m.tbits = tbits; }
        return m;
    }
};

// Position of an owned row's value in a gathered vector: base + row (base = shard * S in the
// full-length shard-major layout, 0 in a segmented compact vector).
// Slot of the device vid -> dense hash table (jg_build.hip remap_ids_device): open addressing, linear
// probing, key INT64_MIN = empty.
struct alignas(16) IdSlot {
    unsigned long long key;
    uint32_t val, pad;
};

struct VecPos {
    int64_t base = 0;
    __device__ __forceinline__ int64_t operator()(int64_t row) const { return base + row; }
};

struct Shard {
    int device = 0;
    int index = 0;           // shard id r in [0, P)
    int vtag = -1;           // virtual-device tag (JG_VDEV_CHECK=1 on logical shards: the index; jg_common.h)
    hipStream_t stream = nullptr;
    ncclComm_t comm = nullptr;  // borrowed from the context (may be null)
    int64_t rows = 0;        // owned rows (<= S)
    Csr in, out, both;
    PullPlan plan_in, plan_both;
    PullPlan plan_out;            // built on first use (combiner programs over the OUT adjacency)
    bool plan_out_built = false;
    Halo halo_in, halo_both;      // sharded graphs: compact vectors of the IN / BOTH pull adjacencies
    DevBuf<int32_t> out_degree;   // [rows] out-degree of owned vertices (PageRank edgeCount)
    // host copy of dense_rows (caller's dense index of each owned row), made on first use
    // (jg_api.cpp; the build no longer copies it: 67 MB at RMAT-24 through pageable memory)
    mutable std::vector<int32_t> dense_of_local_host;
    mutable std::mutex lazy_mu;  // guards the lazy host copies (concurrent read-only callers)
    const std::vector<int32_t>& dense_of_local() const;
    DevBuf<int32_t> dense_rows;           // the same on the device (jg_scatter.h)

    // program state (allocated on demand)
    DevBuf<double> pr_contrib[2];  // [P*S] full-length, ping-pong
    DevBuf<double> pr_rank;        // [rows]
    DevBuf<double> pr_hub_partial; // [num_chunks]
    DevBuf<double> pr_split_partial;  // [plan_in.split_partial_len()]
    DevBuf<int32_t> cc_split_partial; // [plan_both.split_partial_len()]
    DevBuf<int32_t> cc_msg[2];     // [P*S] label if sent else INT32_MAX
    DevBuf<int32_t> cc_label;      // [rows]
    DevBuf<int32_t> cc_rank0;      // [rows] String-order rank of each own row's id (cc_prepare_ranks, build time)
    DevBuf<int32_t> cc_depth;      // [rows] one shard's union-find path: the BFS depths
    DevBuf<unsigned long long> cc_linked;  // union-find: entries the second round linked (a stat, read after t1)
    int64_t cc_heavy = -1;                 // union-find: rows of degree >= 64 of the BOTH CSR (-1: not yet found)
    DevBuf<int32_t> cc_hub_partial;
    DevBuf<int32_t> cc_changed;    // [1]
    // single-source DO-BFS scratch, kept across calls (level-parity ping-pong)
    DevBuf<int32_t> bfs_queue[2];            // [rows] frontier vertices
    DevBuf<int64_t> bfs_qoff[2];             // [rows] first push edge of each queue entry
    DevBuf<unsigned long long> bfs_bm[2];    // [ceil(rows/64)] frontier bitmaps (bottom-up)
    DevBuf<uint8_t> bfs_seen;                // [rows] depth-is-set byte map (filters depth probes)
    DevBuf<int32_t> bfs_owner;               // [rows] split top-down levels: claiming edge of each target
    DevBuf<unsigned long long> bfs_ctr;      // [kBfsRing] packed per-level frontier counters
    DevBuf<unsigned char> bfs_state;         // [kBfsRing * sizeof(BfsState)] per-level decisions
    DevBuf<int32_t> bfs_depth;               // [rows] depth of the last traversal
    bool bfs_depth_tail_clean = false;       // BOTH: bfs_depth's empty suffix holds -1 (the init skips it)
    DevBuf<uint8_t> sbfs_stamp;              // sharded DO-BFS: remote-target stamps per compact position
    DevBuf<uint8_t> sbfs_dirty;              //   a flag per 512 stamps: the chunk holds a set stamp
    DevBuf<unsigned long long> sbfs_bq;      // sharded DO-BFS: send lists as row bitmaps [P][rows / 64]
    DevBuf<int32_t> sbfs_bpre;               //   their bit prefixes per word
    bool sbfs_stamp_clean = false;           // ... all zero (set when a traversal completes)
    int bfs_hist[4] = {0, 0, 0, 0};          // level counts of the last single-source traversals (newest first)
    int bfs_hist_n = 0;
    int sd_hist[4] = {0, 0, 0, 0};  // delta-stepping: steps of the last calls (the first batch's size)
    int sd_hist_n = 0;
    DevBuf<int32_t> kept_depth;              // [kept_nsrc][rows] jg_bfs_keep's depth planes (jg_bfs_kept_row)
    // narrow bit-parallel BFS scratch (<= 8 sources, one shard; jg_narrow.hip), kept across calls
    std::vector<DevBuf<uint8_t>> nb_level;   // [levels][rows + pad] each level's frontier byte (= its new bits)
    DevBuf<uint8_t> nb_vis;                  // [rows] visited bits
    DevBuf<unsigned long long> nb_rest;      // [ceil(rows/64)] rows the bottom-up first pass left unfinished
    DevBuf<int32_t> nb_queue[2];             // [rows] top-down queues (level parity)
    DevBuf<int64_t> nb_qoff[2];
    DevBuf<unsigned long long> nb_ctr;       // per-level counters (NbCtr ring)
    DevBuf<unsigned char> nb_state;          // per-level decisions (NbState ring)
    DevBuf<const uint8_t*> nb_table;         // device copy of the level pointers (depth output)

    std::vector<hipEvent_t> prof_events;  // start/stop pairs for the dominant kernel
    std::vector<hipEvent_t> exch_events;  // start/stop pairs around the exchange steps
    std::vector<int> prof_units;          // supersteps each pair spans
};

// Whether shard sh is on physical device dev as far as data placement goes: in the virtual-device check
// mode every logical shard but the first counts as a device of its own (jg_common.h), so the
// multi-device paths (peer copies, per-device tables) run on one GPU.
inline bool same_device(const Shard& sh, int dev) { return sh.device == dev && sh.vtag <= 0; }

struct Graph {
    Ctx* ctx = nullptr;
    int64_t n = 0;         // caller vertices
    int P = 1;             // global shard count
    int64_t S = 0;         // padded rows per shard
    uint32_t flags = 0;
    std::vector<std::unique_ptr<Shard>> shards;  // the shards this process drives
    // caller vid -> dense index: the device hash table the build's id remap made (on shard 0's device;
    // empty for RMAT graphs, whose vid == dense).  Lookups go through dense_of_vids (batched).
    DevBuf<IdSlot> id_table;
    int id_dev = 0;
    std::vector<int64_t> vid;           // host: vid[dense] (empty for RMAT graphs: vid == dense)
    // global padded id of each caller vertex (P*S < 2^31): on the first shard's device (id_dev), the
    // host copy made on first use
    DevBuf<int32_t> padded_dev;
    mutable std::vector<int32_t> padded_host;
    mutable std::mutex lazy_mu;  // guards the lazy host copies (padded_host, cc_vor_host)
    const std::vector<int32_t>& padded_of_dense() const;
    jg_graph_info info{};
    bool has_weights = false;
    // String-order ranks of the ids (graphs with BOTH; jg_cc.hip cc_prepare_ranks, at build): the id of
    // each rank on the first shard's device, its host copy made on first use (sharded CC output)
    int kept_nsrc = 0;  // depth rows kept by jg_bfs_keep
    bool cc_ranks = false;
    DevBuf<int64_t> cc_vor;
    mutable std::vector<int64_t> cc_vor_host;
    const std::vector<int64_t>& vid_of_rank() const;
    // PageRank session
    int pr_cur = 0;
    bool pr_begun = false;
    double pr_damping = 0.85;
    int64_t pr_vertex_count = 1;
    int pr_steps = 0;

    int64_t vid_of(int64_t dense) const { return vid.empty() ? dense : vid[dense]; }
    int64_t padded_len() const { return (int64_t)P * S; }
    // adj: JG_ADJ_IN or JG_ADJ_BOTH — the pull adjacency whose gathered vector this is
    const Halo& halo(const Shard& sh, uint32_t adj) const { return adj == JG_ADJ_BOTH ? sh.halo_both : sh.halo_in; }
    int64_t vec_len(const Shard& sh, uint32_t adj) const {
        const Halo& h = halo(sh, adj);
        return h.on ? std::max<int64_t>(h.C, 1) : padded_len();
    }
    VecPos vec_pos(const Shard& sh, uint32_t adj) const {
        VecPos p;
        p.base = halo(sh, adj).on ? 0 : (int64_t)sh.index * S;
        return p;
    }
};

struct Ctx {
    std::vector<int> devices;   // devices this process drives (one shard each)
    int nranks = 1;             // processes (rank mode) — total shards = nranks * devices.size()
    int rank = 0;
    bool logical = false;       // several shards on one device: exchange by device copies
    bool vdev = false;          // logical shards checked as virtual devices (JG_VDEV_CHECK=1, jg_common.h)
    std::vector<ncclComm_t> comms;
    bool host_transport = false;  // rank mode over jg_transport callbacks (tests) instead of RCCL
    jg_transport transport{};
    std::vector<hipStream_t> streams;
    bool profiling = false;
    jg_stats last{};
    // graphs and builders made from this context and not yet destroyed: they use its streams and
    // communicators, so jg_ctx_destroy refuses while any is alive (JG_ERR_STATE)
    std::atomic<int> live{0};
    int total_shards() const { return nranks * (int)devices.size(); }
};

// ---- build (jg_build.hip) ----
// Dense edge list already on every shard's device as int32 (src, dst) with ids in [0,n) — or -1
// for a ghost endpoint; weights optional.  Builds relabelling, CSRs and pull plans.
struct DenseEdges {
    std::vector<int32_t*> src, dst;    // per local shard device pointers (size m)
    std::vector<int32_t*> weight;      // may hold nullptr
    int64_t m = 0;
    // Fulgora's slice cap (jg_builder_set_query_limit): the OUT adjacency and out-degrees come from
    // (out_src, dst), -1 where the OUT entry lies beyond its row's limit; the IN adjacency from
    // (in_src, in_dst)[m_in] if in_from_in, else from the capped OUT list; BOTH from (src, dst).
    bool capped = false, in_from_in = false;
    std::vector<int32_t*> out_src, in_src, in_dst;
    int64_t m_in = 0;
    int64_t truncated_rows = 0;
};
void build_graph_from_dense(Graph& g, DenseEdges& e);
void generate_rmat_device(int scale, uint64_t seed, int64_t m, int32_t* src, int32_t* dst, hipStream_t s);
// dsrc/ddst = the dense index of each endpoint (-1: not in vid, a ghost).  table: where the vid table is
// built (nullptr: a temporary); a table that already holds this vid list (size != 0) is reused.
void remap_ids_device(const int64_t* d_vid, int64_t n, const int64_t* d_src, const int64_t* d_dst, int64_t m,
                      int32_t* dsrc, int32_t* ddst, hipStream_t s, DevBuf<IdSlot>* table = nullptr);
// out[i] = the dense index of vids[i] (-1 if absent), k host values, one device lookup;
// padded[i] (nullable) = its global padded id (-1 if absent)
void dense_of_vids(const Graph& g, const int64_t* vids, int64_t k, int64_t* out, int64_t* padded = nullptr);
// out[e] = -1 where masked[e] < 0, else dense[e]
void mask_ids_device(const int64_t* masked, const int32_t* dense, int64_t m, int32_t* out, hipStream_t s);
// col_space: length of the gathered vector; vec_entries: entries actually in it, elem_bytes: their
// size (automatic band widths)
void build_pull_plan(Shard& sh, const Csr& csr, PullPlan& plan, int64_t col_space, int64_t vec_entries,
                     int elem_bytes);
int auto_band_bits(int64_t vec_entries, int elem_bytes);

void rccl_check(ncclResult_t r, const char* what);

// ---- exchange (jg_api.cpp, jg_halo.hip) ----
// The exchange step of a gathered vector of the pull adjacency `adj` (JG_ADJ_IN / JG_ADJ_BOTH):
// halo exchange when the shards hold compact vectors, else an in-place allgather of every shard's
// owned slice [r*S, r*S+S) of the full-length vector.
void exchange_vec(Graph& g, uint32_t adj, std::vector<void*>& bufs, size_t elem_bytes, ncclDataType_t type);
void exchange_allgather(Graph& g, std::vector<void*>& bufs, size_t elem_bytes, ncclDataType_t type);
void exchange_halo(Graph& g, uint32_t adj, std::vector<void*>& bufs, size_t elem_bytes, ncclDataType_t type);
// The transpose of the halo exchange: every shard's segment for peer q (values about q's vertices)
// goes back to q, landing in rbufs[q] at q's send-list position for the sender (element j of a
// shard's rbuf is about its own row send_src[j]).
void exchange_halo_reverse(Graph& g, uint32_t adj, std::vector<void*>& vecs, std::vector<void*>& rbufs,
                           size_t elem_bytes, ncclDataType_t type);
// Bit-packed halo exchange (the sharded DO-BFS frontiers): peer q's run of n bits travels as
// ceil(n / 64) words.  A shard's send-list bits sit in `sends[i]` at word woff(h, q) for peer q; the
// receiver's bits about q's vertices sit in its compact bitmap `bitmaps[i]` (one bit per compact-vector
// position) at its segment for q, which starts on a word (stride 2^tbits, tbits >= 13).  Forward: send
// lists -> segments; reverse: segments -> the owners' send-list words.
void exchange_halo_bits(Graph& g, uint32_t adj, std::vector<uint64_t*>& sends, std::vector<uint64_t*>& bitmaps,
                        bool reverse);
// Per-peer runs whose lengths both sides know (the sparse reverse exchange of the sharded bit-parallel
// BFS): local shard i sends scount[i][q] elements from send[i] + soff[i][q] to peer q and receives
// rcount[i][q] elements from q at recv[i] + roff[i][q] (offsets and counts in elements of eb bytes).
void exchange_runs(Graph& g, const std::vector<const char*>& send, const std::vector<std::vector<int64_t>>& soff,
                   const std::vector<std::vector<int64_t>>& scount, const std::vector<char*>& recv,
                   const std::vector<std::vector<int64_t>>& roff, const std::vector<std::vector<int64_t>>& rcount,
                   size_t eb, ncclDataType_t type);
// Both directions of exchange_halo_bits in one grouped step (the sharded DO-BFS, whose level direction is
// decided on the device): forward fsend -> fbitmap segments, and reverse rbitmap segments -> rsend.
void exchange_halo_bits_both(Graph& g, uint32_t adj, std::vector<uint64_t*>& fsend, std::vector<uint64_t*>& fbitmap,
                             std::vector<uint64_t*>& rbitmap, std::vector<uint64_t*>& rsend);
// word offsets of the per-peer send-list runs of exchange_halo_bits ([P + 1])
std::vector<int64_t> halo_word_offsets(const Halo& h, int P);
// Builds shard sh's halo plan for adjacency `which` (0 IN, 2 BOTH) from the full edge list.
void build_halo(Graph& g, Shard& sh, const int32_t* src, const int32_t* dst, const int32_t* padded, int64_t m,
                int which, Halo& h, hipStream_t s);
// The halo plans are a build-time structure only (the lists stay, the maps go).
void release_halo_maps(Halo& h);
// Checks that every shard's send counts equal its peers' receive counts (RCCL: count allgather).
void check_halo_counts(Graph& g, uint32_t adj);

// ---- edgestore decode (jg_decode.hip) ----
void decode_edges(Ctx& c, const uint8_t* bytes, int64_t nbytes, const int64_t* off, const int32_t* vpos, int64_t n,
                  const int64_t* type_ids, const int8_t* type_mult, int32_t ntypes, int64_t* type_out,
                  int8_t* dir_out, int64_t* other_out, int64_t* rel_out);
// The scan's rows as the edgestore holds them (jg_graph_build_edgestore).
struct EdgestoreRows {
    const uint64_t* keys;      // nrows row keys (the 8-byte big-endian key as an unsigned value)
    int64_t nrows;
    const int64_t* row_off;    // nrows + 1: entries of row r are [row_off[r], row_off[r+1])
    const uint8_t* bytes;
    int64_t nbytes;
    const int64_t* entry_off;  // nentries + 1
    const int32_t* vpos;       // nentries
    int64_t nentries;
    const int64_t* type_ids;
    const int8_t* type_mult;
    int32_t ntypes;
    int pbits;                 // cluster.max-partitions = 2^pbits
    const int32_t* weight = nullptr;  // nentries, nullable: the Integer weight property of each entry's edge
    // A chunk cut out of larger arrays: row_off values count from entry_base, entry_off values from
    // byte_base (bytes points at the chunk's first byte).
    int64_t entry_base = 0, byte_base = 0;
};
void edgestore_check(const EdgestoreRows& r);
// Page-locked host memory (async H2D staging).
struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf();
    void reserve(size_t bytes);
};
struct TypeTable;
struct EdgestoreChunk;
// The property keys an edge value may hold before the weight key (jg_builder_set_weight_key)
struct WeightSchema {
    int64_t key = -1;              // inline id of the weight key (-1: none)
    int8_t key_type = 0;           // its JG_PROP_* type (weights are read only for JG_PROP_INT)
    const int64_t* ids = nullptr;  // sorted inline ids of the property keys (device)
    const int8_t* types = nullptr;
    int32_t n = 0;
};
// The snapshot decoder on `device`: add() takes one chunk of rows (a row never spans chunks), stages it
// in pinned memory and enqueues its copy and decode on one of two streams, then returns; the chunk
// before it completes meanwhile (error check, compaction).  After finish(): vid[0, n) = ids of the
// kept rows in the order added, src/dst[0, m) = their OUT edges (vertex ids; ghosts dropped later).
struct EdgestoreDecoder {
    EdgestoreDecoder(const int64_t* type_ids, const int8_t* type_mult, int32_t ntypes, int pbits, int device);
    ~EdgestoreDecoder();
    void add(const EdgestoreRows& r);
    void finish();
    DevBuf<int64_t> vid, src, dst;
    DevBuf<int32_t> w;    // weights of the kept edges (when every chunk carried entry weights)
    int64_t n = 0, m = 0, mw = 0;
    // Slice cap (set_query_limit before the first add): osrc[m] = src, or -1 where the edge's OUT entry
    // is beyond its row's limit; (isrc, idst)[mi] = the edges whose IN entry is within its row's limit.
    void set_query_limit(int64_t limit) { limit_ = limit; }
    // jg_builder_set_weight_key: decode every OUT edge's Integer weight from its value on the GPU
    void set_weight_key(int64_t key, const int64_t* ids, const int8_t* types, int32_t n);
    int64_t query_limit() const { return limit_; }
    DevBuf<int64_t> osrc, isrc, idst;
    int64_t mo = 0, mi = 0, mi2 = 0, truncated_rows = 0;
    int weighted = -1;    // -1 no chunk yet, 0 / 1: the chunks carry no / per-entry weights
    float kernel_ms = 0;  // copy + decode time of every chunk (HIP events)
    float copy_ms = 0;    // its host -> device copies alone
    int64_t chunks_added_ = 0, rows_ = 0, entries_ = 0, bytes_ = 0, h2d_bytes_ = 0;
    int device() const { return device_; }

   private:
    void complete(int slot);
    int pbits_, device_;
    int64_t limit_ = 0;
    int next_ = 0;
    hipStream_t streams_[2] = {nullptr, nullptr};
    std::unique_ptr<EdgestoreChunk> chunks_[2];
    std::unique_ptr<TypeTable> types_;
    DevBuf<int64_t> idx_, tmp_, cpos_, cscan_;
    DevBuf<int32_t> tmpw_;
    WeightSchema wschema_;         // key < 0: no device weight decode
    bool weight_key_set_ = false;  // set_weight_key was called (even if no Integer key exists)
    DevBuf<int64_t> wkeys_;
    DevBuf<int8_t> wtypes_;
};
// Feeds one whole snapshot to the decoder in chunks of whole rows (<= 4 M entries / 64 MB each).
void add_in_chunks(EdgestoreDecoder& dec, const EdgestoreRows& r);
// One-shot: vid = ids of the kept rows (row order), src/dst = their OUT edges, on `device`.
void edgestore_snapshot(const EdgestoreRows& r, int device, DevBuf<int64_t>& vid, int64_t& n, DevBuf<int64_t>& src,
                        DevBuf<int64_t>& dst, int64_t& m, float* kernel_ms);

// ---- programs ----
void pagerank_begin(Graph& g, double damping, int64_t vertex_count);
void pagerank_steps(Graph& g, int nsteps);
void pagerank_end(Graph& g, double* rank_out, double* edge_count_out);
// depth_rows[s] (each nullable, the array too): source s's depths in caller order (n int32)
// keep: the depth rows stay on the device (Shard::kept_depth, Graph::kept_nsrc) for bfs_kept_row
void bfs_run(Graph& g, const int64_t* source_vids, int nsrc, int direction, int max_depth, int32_t* const* depth_rows,
             bool keep = false);
void bfs_kept_row(Graph& g, int s, int32_t* depth_out);  // row s in caller order
void bfs_kept_release(Graph& g);
// Zeroes the occupied positions of a shard's gathered vector of adjacency `adj` (own rows + peer runs).
void zero_gathered(const Graph& g, const Shard& sh, uint32_t adj, void* v, size_t eb);
// jg_graph_neighbors: the adjacency `direction` of caller vertices rows[0, nrows) in caller order
void graph_neighbors(const Graph& g, int direction, const int64_t* rows, int64_t nrows, int64_t* off_out,
                     int64_t* nbr_out);
void shortest_distance_run(Graph& g, int64_t seed_vid, int max_depth, int64_t* dist_out);
void cc_run(Graph& g, int64_t* comp_out, int32_t* iterations_out);
// Build time (graphs with BOTH): the String-order rank of every id (Graph::cc_vor, Shard::cc_rank0).
void cc_prepare_ranks(Graph& g);
// The union-find's result on one shard (jg_cc.hip): parent[v] is v's root for v < ne, minr[root] the
// smallest rank in the root's component; rows [ne, rows) have no edge (Csr::empty_from).
struct CcRoots {
    int32_t* parent;  // overwritten with the labels (each row's component minimum rank)
    const int32_t* rank;
    const int32_t* minr;
    int64_t ne;
};
// One shard, BOTH adjacency: the largest hop distance of a vertex from the minimum-rank vertex of its
// component, by a direction-optimising BFS started at every such vertex that has an edge; -1 if no
// vertex has an edge.  The start also writes the labels into r.parent (jg_traverse.hip).  *edges_out =
// adjacency entries of the rows the traversal reached.
// after_start (nullable): called once the BFS start (which writes the labels) is enqueued, before its levels
// end_ev (nullable): recorded behind the last level batch, before the host reads the final level state
int cc_root_eccentricity(Ctx& ctx, Shard& sh, const CcRoots& r, int32_t* depth, double* edges_out,
                         const std::function<void()>* after_start = nullptr, hipEvent_t end_ev = nullptr);
// Sharded (halo plans, every shard of the process): the same from the rows whose label (r.parent) is
// their rank, r.minr unused, one CcRoots per local shard; -1 if no vertex has an edge (jg_traverse.hip).
int cc_root_eccentricity_sharded(Graph& g, const CcRoots* roots, double* edges_out);
// Allocate the single-shard traversal's scratch (no-op when present; jg_traverse.hip).
void bfs_buffers(Shard& sh);
// Csr::first_col of a traversal's pull adjacency (built on first use, on the shard's stream)
const int32_t* bfs_first_col(Shard& sh, const Csr& c);
// JG_TRACE_MARKS=1: an empty named dispatch before a program's t0 / after its t1 (tools/bench_trace.py)
void region_mark(hipStream_t s, bool begin);
// Narrow bit-parallel direction-optimising BFS (jg_narrow.hip): 2..kNarrowMax sources on one shard,
// one frontier byte per row, each source choosing its own direction every level.  push / pull: the
// traversal's adjacencies (both present); src[s]: source s's local row (-1: not a vertex).  planes
// (device, [ns][rows], nullable): the depths (-1 unreached).  Returns the levels run.
constexpr int kNarrowMax = 8;
struct NarrowRun {
    int levels = 0;
    float ms = 0;            // HIP-event time of the traversal (init to the last level)
    double entries = 0;      // adjacency entries examined (top-down pushes + bottom-up scans)
    double bytes = 0;        // algorithmic bytes of the examined work
    double reached = 0;      // reached (source, row) pairs
};
NarrowRun narrow_bfs(Ctx& ctx, Shard& sh, const Csr& push, const Csr& pull, const int64_t* src, int ns, int max_depth,
                     int32_t* planes);
void combine_run(Graph& g, int direction, int combiner, int wrap32, const int64_t* init, int steps, int64_t* out,
                 uint8_t* received_out);

// Logical OR of a flag over all ranks (identity in single-process contexts).
int allreduce_or(Graph& g, int flag);
// Element-wise sum of vals[0..n) over all ranks, in place (identity in single-process contexts).
void allreduce_sum_i64(Graph& g, int64_t* vals, int n);
// bitwise OR of a 64-bit word over the ranks (rank mode; the caller combines its in-process shards):
// RCCL has no bitwise reduction, so each bit travels as a byte under ncclMax
uint64_t allreduce_or_u64(Graph& g, uint64_t v);

// Diagnostics from the environment: JG_PULL_SPLIT=1 launches each degree class separately,
// JG_DEBUG_PLAN=1 prints every pull plan at build time.
bool pull_split_launches();
bool debug_plan();
bool debug_bfs();  // JG_DEBUG_BFS=1: synchronise and print every DO-BFS level's decision

// Performance knobs (jg_tune_set): algorithm variants and thresholds selectable at run time so that
// they can be A/B-timed in one process (cdna_hip_programming.md §5.4 rule 24).  Variants measured
// slower or equal were deleted with their code (round 5; DESIGN.md §5-6 keep their measurements).
struct Tune {
    int pull_split = 1;   // XCD-sliced split of the heavy rows (pull_merge_kernel): 0 off, 1 on
                          // (read at build time too: the sliced in-CSR and split plan need it)
    // build time: degree bands of the split, highest first: rows of degree >= band_deg[i] (and below
    // band i-1) get 2^band_bits[i] sub-slices; rows below the last used band stay light (0: unused).  Band
    // 0 from 96 entries (round 4, tools/pr_ab.py: PageRank RMAT-22 / 24 -1% against 128, RMAT-26 and the
    // 64-source BFS unchanged; profiles/r04/band0_deg/).  -1: automatic (auto_bands in jg_build.hip: bands
    // 1 and 2 depend on whether the vector fits the Infinity Cache)
    int64_t band_deg[4] = {96, -1, -1, 0};
    int band_bits[4] = {-1, -1, -1, 3};  // log2 sub-slices (0..8); -1: automatic (auto_band_bits, auto_bands)
    int halo = 1;                     // build time, P > 1: compact vectors + halo exchange (0: dense allgather)
    int bfs_alpha = 14;               // DO-BFS: top-down -> bottom-up when frontier edges > unexplored / alpha
                                      // (multi-source starts: CC's eccentricity BFS, MS-BFS and CC push levels)
    int dobfs_alpha = 30;             // the same for single-source traversals (tools/bfs_sweep.py, RMAT-20:
                                      // 0.147 / 0.146 / 0.137 / 0.136 / 0.137 ms at 14 / 20 / 30 / 45 / 70;
                                      // RMAT-26: 2.147 / 2.143 / 2.431 at 14 / 30 / 70)
    int bfs_beta = 24;                //         bottom-up -> top-down when frontier vertices < rows / beta
    int bfs_narrow = 1;               //         2..8 sources on one shard: the narrow byte-word engine (jg_narrow.hip)
    int nb_alpha = 30;                //         its per-source top-down -> bottom-up threshold (RMAT-26, 8 groups of 8
                                      //         sources: slowest group 6.61 / 5.79 / 6.61 / 6.85 ms at 14 / 30 / 60 / 120,
                                      //         profiles/r05/groups/narrow_alpha_sweep_s26.jsonl)
    int nb_first = 16;                //         its bottom-up first pass: entries a lane scans before a wave takes the row
    int cc_push = 1;                  // CC propagation on one shard: push supersteps when the senders have few edges
    int msbfs_sparse = 1;             //         sharded bit-parallel BFS: top-down levels send only the set halo
                                      //         staging slots when they are under half the halo (0: always dense)
    int msbfs_td = 1;                 //         bit-parallel BFS: top-down levels for small frontiers (1: one shard
                                      //         and sharded over the BOTH halo, 2: one shard only, 0: off)
    int cc_first = 1;                 //         one-shard CC union-find: neighbours linked by every vertex in the first round
                                      //         (RMAT-26: 2.82 / 3.05 / 3.31 / 3.53 ms at 1 / 2 / 3 / 4)
    int msbfs_skip = 1;               //         bit-parallel BFS pull levels skip the merge tasks of rows that can gain no bit
    int msbfs_exit = 1;               //         bit-parallel BFS, one shard: rows scanned with early exit instead of merged
                                      //         (0 never, 1 pull levels where few band-0 tasks are live, 2 every pull
                                      //         level).  RMAT-22 / 24 / 26: 1.83 / 4.46 / 17.6 -> 1.67 / 3.83 / 13.4 ms
                                      //         with band 0 alone (profiles/r04/msbfs_exit/); every row since
    int msbfs_td_rowapply = 4;        //         bit-parallel BFS, one shard: a top-down level with >= rows / this frontier
                                      //         edges applies over every row in order, not its touched list (0: never)
    int msbfs_td_noprobe = 2;         //         bit-parallel BFS: top-down levels below this skip the visited probe
                                      //         (RMAT-26 12.49-12.60 -> 12.32 ms, RMAT-24 -1%; profiles/r04/msbfs_td_dense/)
    int msbfs_scan_queue = 50;        //         bit-parallel BFS, one shard: a pull level whose band 0 had fewer live
                                      //         tasks than this permille builds the next top-down queue in its
                                      //         frontier scan (one pass instead of two); 0: never
    int msbfs_exit_first = 16;        //         msbfs_exit: entries a lane scans per row before a wave takes it
                                      //         (RMAT-26 12.29-12.35 / 12.14-12.21 / 12.14-12.18 ms at 8 / 16 / 32,
                                      //         RMAT-24 -1% at 16; profiles/r04/msbfs_exit/first_*.log)
    int msbfs_exit_live = 950;        //         msbfs_exit 1: permille of band 0's merge tasks live below which the rows
                                      //         exit early (the level after the frontier's peak: 45-73%; before it: 100%)
    int cc_uf = 1;                    //         connected components on one shard: union-find + BFS superstep count
    int cc_uf_sharded = 1;            //         sharded (halo plans): local union-find, tree labels over the halo,
                                      //         multi-root sharded BFS for the superstep count (0: propagation)
    int cc_uf_search = 1;             //         ... giant-to-giant links by a bounded search (0: every flagged entry)
    int cc_sparse = 1;                //         ... label rounds after the first move only the labels that fell
                                      //         ((offset, label) pairs) when that is under half the run (0: dense)
    int msbfs_split = 1;              //         bit-parallel BFS pull levels through the sliced split (merge engine)
    int sharded_bfs = 1;              //         single-source BOTH BFS on a sharded graph: DO-BFS over the halo
    int bfs_td_split = 2;             //         DO-BFS top-down levels of >= bfs_td_split_min frontier entries in two
                                      //         launches (targets' owner written, then claimed) instead of one CAS
                                      //         per entry: 0 never, 1 every level, 2 the level(s) in bfs_td_split_levels
    int bfs_td_split_levels = 2;      //         bit mask of the levels mode 2 splits (default: level 1)
    int64_t bfs_td_split_min = 65536; //         frontier entries outside [min, max] claim by CAS anyway (the split
    int64_t bfs_td_split_max = 1 << 20;  //       walks the entries twice: RMAT-26 levels of tens of millions lost
                                      //         1.2 ms; RMAT-20's 329 K-entry level 1 went 64 -> 26 us)
    int bfs_batch0 = 10;              //         DO-BFS: levels in the first batch (then 4, 8, 16, ...)
    int bfs_grid_mult = 4;            //         DO-BFS level grid = sqrt(rows) * bfs_grid_mult / 4 workgroups
    int bfs_grid = 8192;              //         most workgroups of a level launch (sqrt(rows) below; grid-stride)
    int bfs_tail_grid = 64;           //         workgroups of the launches past the deepest of the last 4 traversals
                                      //         (0: every launch at the full grid)
    int sd_dist32 = 1;                // delta-stepping: 32-bit distances when they cannot overflow (0 never,
                                      // 1 from 2^23 rows on, 2 at any size; sd_delta_stepping)
    int sd_delta = -1;                // weighted shortest distance with an unbounded hop count (maxDepth >= rows - 1)
                                      // and no negative weight: near-far delta-stepping with this delta (-1:
                                      // automatic, 0: the frontier Bellman-Ford supersteps)
    int merge_temporal = 1;           // merge blocks sweep their XCD's sub-slices one at a time (L2 locality):
                                      // 0 off, 1 when an XCD's eighth of the vector exceeds 8 MB, 2 always
    int merge_stage[4] = {-1, -1, -1, -1};  // per band: LDS window of a wave's task partials (slots; 0 = direct
                                          // stores, -1 = automatic from the band's heads per task)
    int merge_pack = 1;               // build time: band entries packed in 20/24 bits when the vector allows
                                      // (0: 32 bits, 24: at least 24; tests)
};
Tune& tune();
// rank mode over jg_transport callbacks (jg_api.cpp)
void host_allgather(Ctx& c, const void* in, void* out, size_t bytes);
void host_exchange(Ctx& c, const std::vector<int>& speer, const std::vector<const void*>& sbuf,
                   const std::vector<size_t>& sbytes, const std::vector<int>& rpeer, const std::vector<void*>& rbuf,
                   const std::vector<size_t>& rbytes);
int device_cu_count();  // compute units of the current device

// Profiling of the dominant kernel (HIP events on the shard's stream).
bool prof_enabled(const Ctx& c);
void prof_record_start(Ctx& c, Shard& sh);
void prof_record_stop(Ctx& c, Shard& sh, int units = 1);
void prof_collect(Ctx& c, Graph& g);
// Event pair around an exchange step on the shard's stream (profiling only): exchange_ms.
void exch_record(Ctx& c, Shard& sh);
// Drops the exchange pairs recorded so far (a program's timed region starts: pairs never straddle it).
void prof_discard_exchanges(Graph& g);
// With profiling on, an exchange step is bracketed by events on every local shard's stream
// (jg_stats.exchange_ms: the slowest shard's sum); the leaf exchange functions hold one.
struct ExchTimer {
    Graph& g;
    explicit ExchTimer(Graph& gr);
    ~ExchTimer();
};

}  // namespace jg

struct jg_ctx {
    jg::Ctx impl;
};
struct jg_graph {
    jg::Graph impl;
    explicit jg_graph(jg::Ctx* c) {
        impl.ctx = c;
        c->live.fetch_add(1);
    }
    ~jg_graph() { impl.ctx->live.fetch_sub(1); }
    jg_graph(const jg_graph&) = delete;
    jg_graph& operator=(const jg_graph&) = delete;
};
