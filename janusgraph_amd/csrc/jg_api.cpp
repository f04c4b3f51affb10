// jg_api.cpp — the extern "C" boundary of libjanusgpu (include/janusgpu.h), contexts, the RCCL
// exchange and profiling.  No exception or abort crosses the ABI: every entry point catches and
// returns a status, with the message kept per thread for jg_last_error().
//
// Error style mirrors FulgoraGraphComputer's "Computer is aborting" failures
// (janusgraph-core/.../olap/computer/FulgoraGraphComputer.java:269-286): any failure aborts the
// whole program run; callers wrap a non-zero status in a JanusGraphException.
#include <dlfcn.h>
#include <execinfo.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <mutex>

#include "jg_cache.h"
#include "jg_internal.h"

namespace jg {

namespace {
thread_local std::string g_last_error;
}  // namespace

void rccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) fail(JG_ERR_RCCL, std::string(what) + ": " + ncclGetErrorString(r));
}

void fail(int code, const std::string& msg) { throw Error(code, msg); }

void hip_check(hipError_t e, const char* what, const char* file, int line) {
    if (e != hipSuccess) {
        const char* base = std::strrchr(file, '/');
        fail(e == hipErrorOutOfMemory ? JG_ERR_OOM : JG_ERR_HIP,
             std::string(what) + " failed: " + hipGetErrorString(e) + " (" + (base ? base + 1 : file) + ":" +
                 std::to_string(line) + ")");
    }
}


void transport_check(int rc, const char* what) {
    if (rc != 0) fail(JG_ERR_RCCL, std::string("host transport ") + what + " failed (" + std::to_string(rc) + ")");
}

void host_allgather(Ctx& c, const void* in, void* out, size_t bytes) {
    transport_check(c.transport.allgather(c.transport.user, in, out, bytes), "allgather");
}

void host_exchange(Ctx& c, const std::vector<int>& speer, const std::vector<const void*>& sbuf,
                   const std::vector<size_t>& sbytes, const std::vector<int>& rpeer, const std::vector<void*>& rbuf,
                   const std::vector<size_t>& rbytes) {
    transport_check(c.transport.exchange(c.transport.user, (int)speer.size(), speer.data(), sbuf.data(), sbytes.data(),
                                         (int)rpeer.size(), rpeer.data(), rbuf.data(), rbytes.data()),
                    "exchange");
}

void exchange_allgather(Graph& g, std::vector<void*>& bufs, size_t elem_bytes, ncclDataType_t type) {
    ExchTimer et(g);
    if (g.P == 1) return;
    Ctx& c = *g.ctx;
    const size_t slice = (size_t)g.S * elem_bytes;
    if (c.host_transport) {  // rank mode over host callbacks: one shard per process
        Shard& sh = *g.shards[0];
        DeviceGuard dg(sh);
        std::vector<char> mine(slice), all(slice * (size_t)c.nranks);
        char* base = static_cast<char*>(bufs[0]);
        copy_d2h(mine.data(), base + (size_t)sh.index * slice, slice, sh.stream);
        host_allgather(c, mine.data(), all.data(), slice);
        for (int r = 0; r < c.nranks; ++r)
            if (r != sh.index) copy_h2d(base + (size_t)r * slice, all.data() + (size_t)r * slice, slice, sh.stream);
        return;
    }
    if (c.logical) {  // all shards on one device and stream: device copies of the owned slices
        Shard& s0 = *g.shards[0];
        DeviceGuard dg(s0.device);
        for (size_t dst = 0; dst < g.shards.size(); ++dst)
            for (size_t src = 0; src < g.shards.size(); ++src) {
                if (src == dst) continue;
                const int r = g.shards[src]->index;
                char* d = static_cast<char*>(bufs[dst]) + (size_t)r * slice;
                const char* s = static_cast<const char*>(bufs[src]) + (size_t)r * slice;
                JG_HIP(hipMemcpyAsync(d, s, slice, hipMemcpyDeviceToDevice, s0.stream));
            }
        return;
    }
    rccl_check(ncclGroupStart(), "ncclGroupStart");
    for (size_t i = 0; i < g.shards.size(); ++i) {
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        char* base = static_cast<char*>(bufs[i]);
        rccl_check(ncclAllGather(base + (size_t)sh.index * slice, base, (size_t)g.S,
                                 type, sh.comm, sh.stream),
                   "ncclAllGather");
    }
    rccl_check(ncclGroupEnd(), "ncclGroupEnd");
}

int allreduce_or(Graph& g, int flag) {
    Ctx& c = *g.ctx;
    if (c.nranks == 1) return flag;  // in-process shards already combined by the caller
    Shard& sh = *g.shards[0];
    DeviceGuard dg(sh);
    if (c.host_transport) {
        const int32_t mine = flag ? 1 : 0;
        std::vector<int32_t> all((size_t)c.nranks);
        host_allgather(c, &mine, all.data(), sizeof mine);
        return *std::max_element(all.begin(), all.end());
    }
    DevBuf<int32_t> d(1);
    int32_t v = flag ? 1 : 0;
    JG_HIP(hipMemcpyAsync(d.get(), &v, sizeof v, hipMemcpyHostToDevice, sh.stream));
    rccl_check(ncclAllReduce(d.get(), d.get(), 1, ncclInt32, ncclMax, sh.comm, sh.stream), "ncclAllReduce");
    JG_HIP(hipMemcpyAsync(&v, d.get(), sizeof v, hipMemcpyDeviceToHost, sh.stream));
    JG_HIP(hipStreamSynchronize(sh.stream));
    return v;
}

void allreduce_sum_i64(Graph& g, int64_t* vals, int n) {
    Ctx& c = *g.ctx;
    if (c.nranks == 1) return;  // in-process shards already summed by the caller
    Shard& sh = *g.shards[0];
    DeviceGuard dg(sh);
    if (c.host_transport) {
        std::vector<int64_t> all((size_t)n * c.nranks);
        host_allgather(c, vals, all.data(), (size_t)n * sizeof(int64_t));
        for (int i = 0; i < n; ++i) {
            int64_t t = 0;
            for (int r = 0; r < c.nranks; ++r) t += all[(size_t)r * n + i];
            vals[i] = t;
        }
        return;
    }
    DevBuf<int64_t> d(n);
    JG_HIP(hipMemcpyAsync(d.get(), vals, n * sizeof(int64_t), hipMemcpyHostToDevice, sh.stream));
    rccl_check(ncclAllReduce(d.get(), d.get(), (size_t)n, ncclInt64, ncclSum, sh.comm, sh.stream), "ncclAllReduce");
    JG_HIP(hipMemcpyAsync(vals, d.get(), n * sizeof(int64_t), hipMemcpyDeviceToHost, sh.stream));
    JG_HIP(hipStreamSynchronize(sh.stream));
}

// ---- the caching device allocator behind DevBuf (jg_common.h): jg_cache.h over HIP ----
namespace {
struct HipBackend {
    void* alloc(int dev, size_t bytes) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        if (cur != dev) (void)hipSetDevice(dev);
        void* p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) {
            (void)hipGetLastError();
            p = nullptr;
        }
        if (cur != dev) (void)hipSetDevice(cur);
        return p;
    }
    void release(int dev, void* p) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        if (cur != dev) (void)hipSetDevice(dev);
        (void)hipFree(p);
        if (cur != dev) (void)hipSetDevice(cur);
    }
    void synchronize(const std::vector<int>& devs) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        for (int d : devs) {
            (void)hipSetDevice(d);
            (void)hipDeviceSynchronize();
        }
        (void)hipSetDevice(cur);
    }
};
// never destroyed: a DevBuf released during process exit (after static destructors) still finds it
BlockCache<HipBackend>& cache() {
    static BlockCache<HipBackend>* c = [] {
        auto* b = new BlockCache<HipBackend>();
        b->set_off(std::getenv("JG_NO_DEVCACHE") != nullptr);  // plain hipMalloc / hipFree
        return b;
    }();
    return *c;
}
thread_local bool t_direct_free = false;  // DirectFree scope (jg_graph_destroy)
}  // namespace

namespace {
std::atomic<int> g_vdev_mode{-1};  // JG_VDEV_CHECK, re-read at every context creation (tests toggle it)
int vdev_env() {
    const char* v = std::getenv("JG_VDEV_CHECK");
    return v && *v ? std::atoi(v) : 0;
}
}  // namespace

int vdev_mode() {
    int m = g_vdev_mode.load(std::memory_order_relaxed);
    if (m < 0) {
        m = vdev_env();
        g_vdev_mode.store(m, std::memory_order_relaxed);
    }
    return m;
}
void vdev_refresh() { g_vdev_mode.store(vdev_env(), std::memory_order_relaxed); }

void vdev_violation(int buffer_tag, int current_tag) {
    const std::string msg = "virtual-device check: a buffer of shard " + std::to_string(buffer_tag) + " used under shard " +
                            std::to_string(current_tag) +
                            "'s device guard (on distinct devices this is a cross-device access)";
    if (vdev_mode() == 2 || std::getenv("JG_VDEV_TRACE")) {  // return addresses as library offsets
        void* pcs[16];
        const int k = backtrace(pcs, 16);
        std::string where;
        for (int i = 1; i < k && i < 6; ++i) {
            Dl_info di{};
            if (dladdr(pcs[i], &di) && di.dli_fname && std::strstr(di.dli_fname, "libjanusgpu")) {
                char b[32];
                std::snprintf(b, sizeof b, " +0x%lx", (unsigned long)((const char*)pcs[i] - (const char*)di.dli_fbase));
                where += b;
            }
        }
        static std::mutex mu;
        static std::vector<std::string> seen;
        std::lock_guard<std::mutex> lk(mu);
        if (std::find(seen.begin(), seen.end(), where) == seen.end()) {
            seen.push_back(where);
            std::fprintf(stderr, "[jg vdev] %s at libjanusgpu.so%s\n", msg.c_str(), where.c_str());
        }
        if (vdev_mode() == 2) return;
    }
    fail(JG_ERR_STATE, msg);
}

DirectFree::DirectFree() : prev(t_direct_free) { t_direct_free = true; }
DirectFree::~DirectFree() { t_direct_free = prev; }

void* dev_alloc(size_t bytes) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    return cache().alloc(dev, bytes);
}

void dev_free(void* p, size_t bytes, int dev) { cache().free(dev, p, bytes, t_direct_free); }

void dev_cache_sync() { cache().sync(); }

void dev_cache_release(int dev) { cache().release(dev); }

void dev_cache_drop_ready(int dev) { cache().drop_ready(dev); }

uint64_t allreduce_or_u64(Graph& g, uint64_t v) {
    Ctx& c = *g.ctx;
    if (c.nranks == 1) return v;
    Shard& sh = *g.shards[0];
    DeviceGuard dg(sh);
    if (c.host_transport) {
        std::vector<uint64_t> all((size_t)c.nranks);
        host_allgather(c, &v, all.data(), sizeof v);
        uint64_t r = 0;
        for (uint64_t w : all) r |= w;
        return r;
    }
    uint8_t bytes[64];
    for (int b = 0; b < 64; ++b) bytes[b] = (uint8_t)((v >> b) & 1u);
    DevBuf<uint8_t> d(64);
    JG_HIP(hipMemcpyAsync(d.get(), bytes, sizeof bytes, hipMemcpyHostToDevice, sh.stream));
    rccl_check(ncclAllReduce(d.get(), d.get(), 64, ncclUint8, ncclMax, sh.comm, sh.stream), "ncclAllReduce");
    JG_HIP(hipMemcpyAsync(bytes, d.get(), sizeof bytes, hipMemcpyDeviceToHost, sh.stream));
    JG_HIP(hipStreamSynchronize(sh.stream));
    uint64_t r = 0;
    for (int b = 0; b < 64; ++b) r |= (uint64_t)(bytes[b] != 0) << b;
    return r;
}

bool prof_enabled(const Ctx& c) { return c.profiling; }

static bool env_flag(const char* name) {
    const char* v = std::getenv(name);
    return v && *v && std::strcmp(v, "0") != 0;
}
bool pull_split_launches() {
    static const bool v = env_flag("JG_PULL_SPLIT");
    return v;
}
bool debug_bfs() {
    static const bool v = env_flag("JG_DEBUG_BFS");
    return v;
}
bool debug_plan() {
    static const bool v = env_flag("JG_DEBUG_PLAN");
    return v;
}

Tune& tune() {
    static Tune t;
    return t;
}


int device_cu_count() {
    static int cache[64] = {0};
    int dev = 0;
    JG_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) dev = 0;
    if (!cache[dev]) JG_HIP(hipDeviceGetAttribute(&cache[dev], hipDeviceAttributeMultiprocessorCount, dev));
    return cache[dev];
}

void prof_record_start(Ctx& c, Shard& sh) {
    if (!c.profiling) return;
    hipEvent_t e;
    JG_HIP(hipEventCreate(&e));
    JG_HIP(hipEventRecord(e, sh.stream));
    sh.prof_events.push_back(e);
}

void prof_record_stop(Ctx& c, Shard& sh, int units) {
    if (!c.profiling) return;
    prof_record_start(c, sh);
    sh.prof_units.push_back(units);
}

void exch_record(Ctx& c, Shard& sh) {
    if (!c.profiling) return;
    hipEvent_t e;
    JG_HIP(hipEventCreate(&e));
    JG_HIP(hipEventRecord(e, sh.stream));
    sh.exch_events.push_back(e);
}

ExchTimer::ExchTimer(Graph& gr) : g(gr) {
    if (!g.ctx->profiling) return;
    for (auto& sp : g.shards) {
        DeviceGuard dg(*sp);
        exch_record(*g.ctx, *sp);
    }
}
ExchTimer::~ExchTimer() {
    if (!g.ctx->profiling) return;
    for (auto& sp : g.shards) {
        DeviceGuard dg(*sp);
        try {
            exch_record(*g.ctx, *sp);
        } catch (...) {  // never from a destructor; the pair stays open and prof_collect skips it
        }
    }
}

void prof_discard_exchanges(Graph& g) {
    for (auto& sp : g.shards) {
        Shard& sh = *sp;
        DeviceGuard dg(sh);
        for (auto e : sh.exch_events) (void)hipEventDestroy(e);
        sh.exch_events.clear();
    }
}

void prof_collect(Ctx& c, Graph& g) {
    double total = 0;
    int64_t launches = 0;
    for (auto& sp : g.shards) {
        Shard& sh = *sp;
        DeviceGuard dg(sh);
        double ex = 0;
        for (size_t i = 0; i + 1 < sh.exch_events.size(); i += 2) {
            JG_HIP(hipEventSynchronize(sh.exch_events[i + 1]));
            float ms = 0;
            JG_HIP(hipEventElapsedTime(&ms, sh.exch_events[i], sh.exch_events[i + 1]));
            ex += ms;
        }
        for (auto e : sh.exch_events) (void)hipEventDestroy(e);
        sh.exch_events.clear();
        c.last.exchange_ms = std::max(c.last.exchange_ms, ex);  // the slowest shard of this process
        for (size_t i = 0; i + 1 < sh.prof_events.size(); i += 2) {
            JG_HIP(hipEventSynchronize(sh.prof_events[i + 1]));
            float ms = 0;
            JG_HIP(hipEventElapsedTime(&ms, sh.prof_events[i], sh.prof_events[i + 1]));
            total += ms;
            launches += i / 2 < sh.prof_units.size() ? sh.prof_units[i / 2] : 1;
        }
        for (auto e : sh.prof_events) (void)hipEventDestroy(e);
        sh.prof_events.clear();
        sh.prof_units.clear();
    }
    c.last.kernel_ms_total += total;
    c.last.kernel_launches += launches;
}

const std::vector<int32_t>& Shard::dense_of_local() const {
    std::lock_guard<std::mutex> lk(lazy_mu);
    if ((int64_t)dense_of_local_host.size() != rows) {
        dense_of_local_host.resize((size_t)rows);
        if (rows > 0) {
            DeviceGuard dg(*this);
            copy_d2h(dense_of_local_host.data(), dense_rows.get(), (size_t)rows * sizeof(int32_t), stream);
        }
    }
    return dense_of_local_host;
}

const std::vector<int64_t>& Graph::vid_of_rank() const {
    std::lock_guard<std::mutex> lk(lazy_mu);
    if ((int64_t)cc_vor_host.size() != n) {
        cc_vor_host.resize((size_t)n);
        if (n > 0) {
            const Shard& sh = *shards[0];
            DeviceGuard dg(sh);
            copy_d2h(cc_vor_host.data(), cc_vor.get(), (size_t)n * sizeof(int64_t), sh.stream);
        }
    }
    return cc_vor_host;
}

const std::vector<int32_t>& Graph::padded_of_dense() const {
    std::lock_guard<std::mutex> lk(lazy_mu);
    if ((int64_t)padded_host.size() != n) {
        padded_host.resize((size_t)n);
        if (n > 0) {
            DeviceGuard dg(id_dev);
            copy_d2h(padded_host.data(), padded_dev.get(), (size_t)n * sizeof(int32_t), shards[0]->stream);
        }
    }
    return padded_host;
}

// Host copy of the vertex ids: outputs are indexed like vid[] (vid -> dense lookups and the duplicate
// check go through the device table the id remap builds: dense_of_vids).
static void set_vertex_ids(Graph& g, const int64_t* vid, int64_t n) { g.vid.assign(vid, vid + n); }

static void make_shards(Ctx& c, Graph& g) {
    g.P = c.total_shards();
    for (size_t i = 0; i < c.devices.size(); ++i) {
        auto sh = std::make_unique<Shard>();
        sh->device = c.devices[i];
        sh->index = c.rank * (int)c.devices.size() + (int)i;
        sh->vtag = c.vdev ? sh->index : -1;
        sh->stream = c.streams[i];
        sh->comm = c.comms.empty() ? nullptr : c.comms[i];
        g.shards.push_back(std::move(sh));
    }
}

// Builds g (shards made) from vertex / edge ids already on device `dev0` (written on stream `s0`):
// vid[n] int64, src/dst[m] int64, weight[m] int32 (nullable).  Every shard remaps the whole edge list
// (shards on other devices get a peer copy first), then the CSRs and plans are built.
// The capped edge lists of a snapshot built under Fulgora's slice cap (device pointers on dev0):
// osrc[m] pairs with d_dst (-1 beyond the cap), (isrc, idst)[mi] the IN entries within the cap.
struct CappedIds {
    const int64_t *osrc = nullptr, *isrc = nullptr, *idst = nullptr;
    int64_t mi = 0;
    bool in_from_in = false;
    int64_t truncated_rows = 0;
};

static void build_from_device_ids(Graph& g, int dev0, hipStream_t s0, const int64_t* d_vid, int64_t n,
                                  const int64_t* d_src, const int64_t* d_dst, const int32_t* d_w, int64_t m,
                                  const CappedIds* cap = nullptr) {
    if (n >= (int64_t)INT32_MAX) fail(JG_ERR_ARG, "more than 2^31-1 vertices");
    if (m >= (int64_t)UINT32_MAX) fail(JG_ERR_ARG, "more than 2^32-1 edges");
    {
        DeviceGuard dg(dev0);
        JG_HIP(hipStreamSynchronize(s0));
        std::vector<int64_t> hv((size_t)n);
        if (n) copy_d2h(hv.data(), d_vid, (size_t)n * sizeof(int64_t), s0);
        g.n = n;
        set_vertex_ids(g, hv.data(), n);
    }
    g.has_weights = d_w != nullptr;
    std::vector<DevBuf<int32_t>> ds(g.shards.size()), dd(g.shards.size()), dw(g.shards.size());
    std::vector<DevBuf<int64_t>> pv(g.shards.size()), ps(g.shards.size()), pd(g.shards.size());
    std::vector<DevBuf<int32_t>> dos(g.shards.size()), dis(g.shards.size()), did(g.shards.size());
    DenseEdges e;
    e.m = m;
    if (cap) {
        if (cap->mi >= (int64_t)UINT32_MAX) fail(JG_ERR_ARG, "more than 2^32-1 edges");
        e.capped = true;
        e.in_from_in = cap->in_from_in;
        e.m_in = cap->in_from_in ? cap->mi : 0;
        e.truncated_rows = cap->truncated_rows;
    }
    for (size_t i = 0; i < g.shards.size(); ++i) {
        Shard& sh = *g.shards[i];
        DeviceGuard dg(sh);
        const int64_t *v = d_vid, *a = d_src, *b = d_dst;
        auto peer = [&](void* dst, const void* src, size_t bytes) {
            if (bytes) JG_HIP(hipMemcpyPeerAsync(dst, sh.device, src, dev0, bytes, sh.stream));
        };
        const bool other = !same_device(sh, dev0);  // a virtual device in the check mode counts as another
        if (other) {
            pv[i].alloc(std::max<int64_t>(n, 1));
            ps[i].alloc(std::max<int64_t>(m, 1));
            pd[i].alloc(std::max<int64_t>(m, 1));
            peer(pv[i].get(), d_vid, (size_t)n * sizeof(int64_t));
            peer(ps[i].get(), d_src, (size_t)m * sizeof(int64_t));
            peer(pd[i].get(), d_dst, (size_t)m * sizeof(int64_t));
            v = pv[i].get();
            a = ps[i].get();
            b = pd[i].get();
        }
        ds[i].alloc(std::max<int64_t>(m, 1));
        dd[i].alloc(std::max<int64_t>(m, 1));
        // shard 0's vid table stays with the graph (vid -> dense lookups) and serves every shard on its
        // device; shards on other devices build a temporary one
        if (i == 0) g.id_dev = sh.device;
        DevBuf<IdSlot> tmp_table;
        DevBuf<IdSlot>& table = same_device(sh, g.id_dev) ? g.id_table : tmp_table;
        remap_ids_device(v, n, a, b, m, ds[i].get(), dd[i].get(), sh.stream, &table);
        e.src.push_back(ds[i].peer());
        e.dst.push_back(dd[i].peer());
        if (cap) {
            DevBuf<int64_t> po, pis, pid;
            const int64_t *o = cap->osrc, *is = cap->isrc, *id = cap->idst;
            if (other) {
                po.alloc(std::max<int64_t>(m, 1));
                peer(po.get(), cap->osrc, (size_t)m * sizeof(int64_t));
                o = po.get();
            }
            dos[i].alloc(std::max<int64_t>(m, 1));
            mask_ids_device(o, ds[i].get(), m, dos[i].get(), sh.stream);
            e.out_src.push_back(dos[i].peer());
            if (cap->in_from_in) {
                const int64_t mi = cap->mi;
                if (other) {
                    pis.alloc(std::max<int64_t>(mi, 1));
                    pid.alloc(std::max<int64_t>(mi, 1));
                    peer(pis.get(), cap->isrc, (size_t)mi * sizeof(int64_t));
                    peer(pid.get(), cap->idst, (size_t)mi * sizeof(int64_t));
                    is = pis.get();
                    id = pid.get();
                }
                dis[i].alloc(std::max<int64_t>(mi, 1));
                did[i].alloc(std::max<int64_t>(mi, 1));
                remap_ids_device(v, n, is, id, mi, dis[i].get(), did[i].get(), sh.stream, &table);
                e.in_src.push_back(dis[i].peer());
                e.in_dst.push_back(did[i].peer());
            }
            JG_HIP(hipStreamSynchronize(sh.stream));  // the peer staging buffers are freed here
        }
        if (d_w) {
            dw[i].alloc(std::max<int64_t>(m, 1));
            if (other) peer(dw[i].get(), d_w, (size_t)m * sizeof(int32_t));
            else if (m) JG_HIP(hipMemcpyAsync(dw[i].get(), d_w, (size_t)m * sizeof(int32_t), hipMemcpyDeviceToDevice, sh.stream));
            e.weight.push_back(dw[i].peer());
        } else {
            e.weight.push_back(nullptr);
        }
    }
    build_graph_from_dense(g, e);
}

// HIP-event timer on the first shard's stream.
struct BuildTimer {
    Graph& g;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    explicit BuildTimer(Graph& gr) : g(gr) {
        DeviceGuard dg(g.shards[0]->device);
        JG_HIP(hipEventCreate(&t0));
        JG_HIP(hipEventCreate(&t1));
        JG_HIP(hipEventRecord(t0, g.shards[0]->stream));
    }
    float stop() {
        DeviceGuard dg(g.shards[0]->device);
        JG_HIP(hipEventRecord(t1, g.shards[0]->stream));
        JG_HIP(hipEventSynchronize(t1));
        float ms = 0;
        JG_HIP(hipEventElapsedTime(&ms, t0, t1));
        return ms;
    }
    ~BuildTimer() {
        (void)hipEventDestroy(t0);
        (void)hipEventDestroy(t1);
    }
};

}  // namespace jg

// The chunked snapshot (jg_builder_*): ids accumulate on the first device as they arrive, raw rows are
// decoded there chunk by chunk (EdgestoreDecoder: copy and decode overlap the caller's next chunk).
struct jg_builder {
    jg::Ctx* ctx = nullptr;
    explicit jg_builder(jg::Ctx* c) : ctx(c) { c->live.fetch_add(1); }
    ~jg_builder() { ctx->live.fetch_sub(1); }
    jg_builder(const jg_builder&) = delete;
    jg_builder& operator=(const jg_builder&) = delete;
    int mode = 0;  // 0 empty, 1 ids (vertices / edges), 2 edgestore rows
    int weights = -1;  // ids mode: -1 unknown, 0 no edge weights, 1 every edge weighted
    bool finished = false;
    jg::DevBuf<int64_t> vid, src, dst;
    jg::DevBuf<int32_t> w;
    int64_t n = 0, m = 0, mw = 0;
    std::unique_ptr<jg::EdgestoreDecoder> dec;
    std::vector<int64_t> type_ids;
    std::vector<int8_t> type_mult;
    int pbits = 5;
    bool schema_set = false;
    int64_t query_limit = 0;  // jg_builder_set_query_limit
    int32_t in_entries = JG_DIR_IN;
    bool weight_key = false;  // jg_builder_set_weight_key
    int64_t wkey = -1;
    std::vector<int64_t> wkey_ids;
    std::vector<int8_t> wkey_types;
};

using jg::Error;

#define JG_GUARD_BEGIN try {
#define JG_GUARD_END                                       \
    jg::dev_cache_sync();                                  \
    return JG_OK;                                          \
    }                                                      \
    catch (const Error& e) {                               \
        jg::g_last_error_set(e.what());                    \
        return e.code;                                     \
    }                                                      \
    catch (const std::bad_alloc&) {                        \
        jg::g_last_error_set("host allocation failed");    \
        return JG_ERR_OOM;                                 \
    }                                                      \
    catch (const std::exception& e) {                      \
        jg::g_last_error_set(e.what());                    \
        return JG_ERR_HIP;                                 \
    }

namespace jg {
void g_last_error_set(const char* m) { g_last_error = m ? m : ""; }
}  // namespace jg

#define JG_ARG(cond, msg) \
    if (!(cond)) jg::fail(JG_ERR_ARG, msg)

extern "C" {

int jg_abi_version(void) { return JG_ABI_VERSION; }

int jg_tune_set(const char* key, int64_t value) {
    JG_GUARD_BEGIN
    JG_ARG(key, "null key");
    const std::string k(key);
    jg::Tune& t = jg::tune();
    // int knobs: name, field, allowed range
    struct Knob {
        const char* name;
        int* field;
        int64_t lo, hi;
    };
    const Knob knobs[] = {
        {"pull_split", &t.pull_split, 0, 1},
        {"halo", &t.halo, 0, 1},
        {"bfs_alpha", &t.bfs_alpha, 1, 1000000},
        {"dobfs_alpha", &t.dobfs_alpha, 1, 1000000},
        {"bfs_beta", &t.bfs_beta, 1, 1000000},
        {"bfs_narrow", &t.bfs_narrow, 0, 1},
        {"nb_alpha", &t.nb_alpha, 1, 1000000},
        {"nb_first", &t.nb_first, 4, 4096},
        {"cc_push", &t.cc_push, 0, 1},
        {"msbfs_sparse", &t.msbfs_sparse, 0, 1},
        {"msbfs_td", &t.msbfs_td, 0, 2},
        {"cc_first", &t.cc_first, 1, 64},
        {"msbfs_skip", &t.msbfs_skip, 0, 1},
        {"msbfs_exit", &t.msbfs_exit, 0, 2},
        {"msbfs_td_rowapply", &t.msbfs_td_rowapply, 0, 1024},
        {"msbfs_td_noprobe", &t.msbfs_td_noprobe, 0, 1000},
        {"msbfs_scan_queue", &t.msbfs_scan_queue, 0, 1001},
        {"msbfs_exit_first", &t.msbfs_exit_first, 1, 256},
        {"msbfs_exit_live", &t.msbfs_exit_live, 0, 1000},
        {"cc_uf", &t.cc_uf, 0, 1},
        {"cc_uf_sharded", &t.cc_uf_sharded, 0, 1},
        {"cc_uf_search", &t.cc_uf_search, 0, 1},
        {"cc_sparse", &t.cc_sparse, 0, 1},
        {"msbfs_split", &t.msbfs_split, 0, 1},
        {"sharded_bfs", &t.sharded_bfs, 0, 1},
        {"bfs_td_split", &t.bfs_td_split, 0, 2},
        {"bfs_td_split_levels", &t.bfs_td_split_levels, 0, 0xffff},
        {"bfs_batch0", &t.bfs_batch0, 1, 64},
        {"bfs_grid_mult", &t.bfs_grid_mult, 1, 64},
        {"bfs_grid", &t.bfs_grid, 64, 65536},
        {"bfs_tail_grid", &t.bfs_tail_grid, 0, 65536},
        {"merge_temporal", &t.merge_temporal, 0, 2},
        {"sd_delta", &t.sd_delta, -1, 1 << 30},
        {"sd_dist32", &t.sd_dist32, 0, 2},
    };
    for (const Knob& kn : knobs) {
        if (k != kn.name) continue;
        if (value < kn.lo || value > kn.hi)
            jg::fail(JG_ERR_ARG, k + " must be in [" + std::to_string(kn.lo) + ", " + std::to_string(kn.hi) + "]");
        *kn.field = (int)value;
        return JG_OK;
    }
    if (k.rfind("band", 0) == 0 && k.size() == 9 && k[4] >= '0' && k[4] <= '3' &&
        (k.substr(5) == "_deg" || k.substr(5) == "_bit" || k.substr(5) == "_sub")) {
        // band<i>_deg: minimum degree (0: band unused); band<i>_bit: log2 sub-slices (0: automatic);
        // band<i>_sub: sub-slices, a power of two in [1, 256]
        const int i = k[4] - '0';
        if (k.substr(5) == "_deg") {
            JG_ARG(value >= -1, "band degree must be >= 0 (0: unused) or -1 (automatic)");
            t.band_deg[i] = value;
        } else if (k.substr(5) == "_bit") {
            JG_ARG(value == 0 || (value >= 3 && value <= 8), "band bits must be 0 (automatic) or in [3, 8]");
            t.band_bits[i] = value == 0 ? -1 : (int)value;
        } else {
            JG_ARG(value >= 1 && value <= 256 && (value & (value - 1)) == 0, "band sub-slices must be a power of two in [1, 256]");
            int b = 0;
            while ((1 << b) < value) ++b;
            t.band_bits[i] = b;
        }
    } else if (k.size() == 12 && k.compare(0, 11, "merge_stage") == 0 && k[11] >= '0' && k[11] <= '3') {
        JG_ARG(value == -1 || value == 0 || value == 64 || value == 128 || value == 256 || value == 512,
               "merge_stage<i> must be -1 (automatic), 0, 64, 128, 256 or 512");
        t.merge_stage[k[11] - '0'] = (int)value;
    } else if (k == "bfs_td_split_min" || k == "bfs_td_split_max") {
        JG_ARG(value >= 1 && value <= INT32_MAX, "bfs_td_split_min / _max must be in [1, 2^31)");
        (k == "bfs_td_split_min" ? t.bfs_td_split_min : t.bfs_td_split_max) = value;
    } else if (k == "merge_pack") {
        JG_ARG(value == 0 || value == 1 || value == 24, "merge_pack must be 0 (32 bits), 1 (automatic) or 24 (at least 24)");
        t.merge_pack = (int)value;
    } else if (k == "pull_unroll" || k == "pull_nt" || k == "pull_lds" || k == "light_lds" || k == "slice_lds" ||
               k == "pull_short" || k == "pull_overlap" || k == "bfs_persistent") {
        // retired knobs (their variants were measured and removed, rounds 4-6): accepted, no effect
    } else {
        jg::fail(JG_ERR_ARG, "unknown tuning key: " + k);
    }
    JG_GUARD_END
}

const char* jg_last_error(void) { return jg::g_last_error.c_str(); }

int jg_comm_unique_id(void* out) {
    JG_GUARD_BEGIN
    JG_ARG(out, "null output");
    ncclUniqueId id;
    jg::rccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    static_assert(sizeof(ncclUniqueId) == JG_UNIQUE_ID_BYTES, "unique id size");
    std::memcpy(out, &id, sizeof id);
    JG_GUARD_END
}

int jg_ctx_create(const int* devices, int ndev, jg_ctx** out) {
    JG_GUARD_BEGIN
    JG_ARG(out && devices && ndev > 0, "jg_ctx_create: need devices and an output pointer");
    *out = nullptr;
    int count = 0;
    JG_HIP(hipGetDeviceCount(&count));
    for (int i = 0; i < ndev; ++i)
        JG_ARG(devices[i] >= 0 && devices[i] < count, "jg_ctx_create: device ordinal out of range");
    auto ctx = std::make_unique<jg_ctx>();
    jg::Ctx& c = ctx->impl;
    c.devices.assign(devices, devices + ndev);
    bool all_same = true;
    for (int i = 1; i < ndev; ++i) all_same &= devices[i] == devices[0];
    c.logical = ndev > 1 && all_same;
    jg::vdev_refresh();
    c.vdev = c.logical && jg::vdev_mode() != 0;
    if (ndev > 1 && !all_same) {
        std::vector<int> sorted(c.devices);
        std::sort(sorted.begin(), sorted.end());
        JG_ARG(std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end(),
               "jg_ctx_create: mix of repeated and distinct devices");
    }
    for (int i = 0; i < ndev; ++i) {
        jg::DeviceGuard dg(c.devices[i]);
        hipStream_t s = nullptr;
        if (c.logical && i > 0) s = c.streams[0];  // logical shards share one stream
        else JG_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        c.streams.push_back(s);
    }
    if (ndev > 1 && !c.logical) {
        c.comms.resize(ndev);
        jg::rccl_check(ncclCommInitAll(c.comms.data(), ndev, c.devices.data()), "ncclCommInitAll");
    }
    *out = ctx.release();
    JG_GUARD_END
}

int jg_ctx_create_rank(int device, int nranks, int rank, const void* unique_id, jg_ctx** out) {
    JG_GUARD_BEGIN
    JG_ARG(out && nranks >= 1 && rank >= 0 && rank < nranks, "jg_ctx_create_rank: bad rank arguments");
    JG_ARG(nranks == 1 || unique_id, "jg_ctx_create_rank: unique_id required for nranks > 1");
    *out = nullptr;
    int count = 0;
    JG_HIP(hipGetDeviceCount(&count));
    JG_ARG(device >= 0 && device < count, "jg_ctx_create_rank: device ordinal out of range");
    auto ctx = std::make_unique<jg_ctx>();
    jg::Ctx& c = ctx->impl;
    c.devices = {device};
    c.nranks = nranks;
    c.rank = rank;
    jg::DeviceGuard dg(device);
    hipStream_t s = nullptr;
    JG_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    c.streams.push_back(s);
    if (nranks > 1) {
        ncclUniqueId id;
        std::memcpy(&id, unique_id, sizeof id);
        ncclComm_t comm;
        jg::rccl_check(ncclCommInitRank(&comm, nranks, id, rank), "ncclCommInitRank");
        c.comms.push_back(comm);
    }
    *out = ctx.release();
    JG_GUARD_END
}

int jg_ctx_create_rank_transport(int device, int nranks, int rank, const jg_transport* t, jg_ctx** out) {
    JG_GUARD_BEGIN
    JG_ARG(out && nranks >= 1 && rank >= 0 && rank < nranks, "jg_ctx_create_rank_transport: bad rank arguments");
    JG_ARG(t && t->allgather && t->exchange, "jg_ctx_create_rank_transport: transport callbacks required");
    *out = nullptr;
    int count = 0;
    JG_HIP(hipGetDeviceCount(&count));
    JG_ARG(device >= 0 && device < count, "jg_ctx_create_rank_transport: device ordinal out of range");
    auto ctx = std::make_unique<jg_ctx>();
    jg::Ctx& c = ctx->impl;
    c.devices = {device};
    c.nranks = nranks;
    c.rank = rank;
    c.host_transport = nranks > 1;
    c.transport = *t;
    jg::DeviceGuard dg(device);
    hipStream_t s = nullptr;
    JG_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    c.streams.push_back(s);
    *out = ctx.release();
    JG_GUARD_END
}

int jg_ctx_destroy(jg_ctx* ctx) {
    JG_GUARD_BEGIN
    if (!ctx) return JG_OK;
    jg::Ctx& c = ctx->impl;
    // graphs and builders hold the context's streams and communicators (a graph destroyed after its
    // context synchronised a destroyed stream: gpurun_out/r05f): the caller destroys them first
    const int live = c.live.load();
    if (live > 0)
        jg::fail(JG_ERR_STATE, ("jg_ctx_destroy: " + std::to_string(live) +
                                " graph(s)/builder(s) of this context are still alive; destroy them first").c_str());
    for (auto cm : c.comms) ncclCommDestroy(cm);
    for (size_t i = 0; i < c.streams.size(); ++i) {
        if (c.logical && i > 0) continue;
        jg::DeviceGuard dg(c.devices[i]);
        (void)hipStreamDestroy(c.streams[i]);
    }
    for (size_t i = 0; i < c.devices.size(); ++i)  // the cached device memory goes back with the context
        if (!(c.logical && i > 0)) jg::dev_cache_release(c.devices[i]);
    delete ctx;
    JG_GUARD_END
}

int jg_ctx_last_stats(const jg_ctx* ctx, jg_stats* out) {
    JG_GUARD_BEGIN
    JG_ARG(ctx && out, "null argument");
    *out = ctx->impl.last;
    JG_GUARD_END
}

int jg_ctx_set_profiling(jg_ctx* ctx, int enable) {
    JG_GUARD_BEGIN
    JG_ARG(ctx, "null context");
    ctx->impl.profiling = enable != 0;
    JG_GUARD_END
}

int jg_graph_build(jg_ctx* ctx, const int64_t* vid, int64_t n, const int64_t* src, const int64_t* dst,
                   const int32_t* weight, int64_t m, uint32_t flags, jg_graph** out) {
    JG_GUARD_BEGIN
    JG_ARG(ctx && out, "null argument");
    JG_ARG(n >= 0 && m >= 0, "negative size");
    JG_ARG(n == 0 || vid, "vid is null");
    JG_ARG(m == 0 || (src && dst), "src/dst is null");
    JG_ARG(n < (int64_t)INT32_MAX, "more than 2^31-1 vertices");
    JG_ARG(m < (int64_t)UINT32_MAX, "more than 2^32-1 edges");
    JG_ARG((flags & (JG_ADJ_IN | JG_ADJ_OUT | JG_ADJ_BOTH)) != 0 && (flags & ~7u) == 0, "bad adjacency flags");
    *out = nullptr;
    jg::Ctx& c = ctx->impl;
    auto gh = std::make_unique<jg_graph>(&c);
    jg::Graph& g = gh->impl;
    g.flags = flags;
    jg::make_shards(c, g);
    jg::BuildTimer timer(g);
    jg::Shard& sh0 = *g.shards[0];
    {
        jg::DeviceGuard dg(sh0.device);
        jg::DevBuf<int64_t> dvid(std::max<int64_t>(n, 1)), dsrc(std::max<int64_t>(m, 1)), ddst(std::max<int64_t>(m, 1));
        jg::DevBuf<int32_t> dw;
        if (n) jg::copy_h2d(dvid.get(), vid, n * sizeof(int64_t), sh0.stream);
        if (m) {
            jg::copy_h2d(dsrc.get(), src, m * sizeof(int64_t), sh0.stream);
            jg::copy_h2d(ddst.get(), dst, m * sizeof(int64_t), sh0.stream);
        }
        if (weight) {
            dw.alloc(std::max<int64_t>(m, 1));
            if (m) jg::copy_h2d(dw.get(), weight, m * sizeof(int32_t), sh0.stream);
        }
        jg::build_from_device_ids(g, sh0.device, sh0.stream, dvid.get(), n, dsrc.get(), ddst.get(),
                                  weight ? dw.get() : nullptr, m);
    }
    const float ms = timer.stop();
    c.last = jg_stats{};
    c.last.build_ms = ms;
    *out = gh.release();
    JG_GUARD_END
}

int jg_graph_build_edgestore(jg_ctx* ctx, const uint64_t* row_keys, int64_t nrows, const int64_t* row_entry_off,
                             const uint8_t* bytes, int64_t nbytes, const int64_t* entry_off, const int32_t* value_pos,
                             int64_t nentries, const int64_t* type_ids, const int8_t* type_mult, int32_t ntypes,
                             int32_t partition_bits, uint32_t flags, int64_t* vid_out, int64_t* num_vertices_out,
                             jg_graph** out) {
    JG_GUARD_BEGIN
    JG_ARG(ctx && out, "null argument");
    JG_ARG((flags & (JG_ADJ_IN | JG_ADJ_OUT | JG_ADJ_BOTH)) != 0 && (flags & ~7u) == 0, "bad adjacency flags");
    const jg::EdgestoreRows r{row_keys, nrows,     row_entry_off, bytes,    nbytes,        entry_off,
                              value_pos, nentries, type_ids,      type_mult, ntypes,       partition_bits};
    *out = nullptr;  // the decoder validates the rows and entries as it stages them
    jg::Ctx& c = ctx->impl;
    auto gh = std::make_unique<jg_graph>(&c);
    jg::Graph& g = gh->impl;
    g.flags = flags;
    jg::make_shards(c, g);
    jg::BuildTimer timer(g);
    jg::Shard& sh0 = *g.shards[0];
    jg::EdgestoreDecoder dec(type_ids, type_mult, ntypes, partition_bits, sh0.device);
    // Fed in chunks of whole rows, as the builder is: the pinned staging stays small, and staging a
    // chunk on the host overlaps the copy and decode of the one before.
    jg::add_in_chunks(dec, r);
    dec.finish();
    {
        jg::DeviceGuard dg(sh0.device);
        jg::build_from_device_ids(g, sh0.device, sh0.stream, dec.vid.get(), dec.n, dec.src.get(), dec.dst.get(), nullptr,
                                  dec.m);
    }
    const float ms = timer.stop();
    c.last = jg_stats{};
    c.last.build_ms = ms;
    c.last.kernel_ms_total = dec.kernel_ms;  // copy + decode of the rows
    c.last.exchange_ms = dec.copy_ms;        // the host -> device copies alone
    c.last.kernel_launches = 1;
    // decode kernels: entry bytes + off/vpos/take (13 B) per entry, src/dst (16 B) per kept edge,
    // key/row_off/row_vid/keep (25 B) per row
    c.last.algorithmic_bytes = (double)nbytes + 13.0 * (double)nentries + 16.0 * (double)dec.m + 25.0 * (double)nrows;
    if (vid_out && g.n) std::copy(g.vid.begin(), g.vid.end(), vid_out);
    if (num_vertices_out) *num_vertices_out = g.n;
    *out = gh.release();
    JG_GUARD_END
}

int jg_builder_create(jg_ctx* ctx, jg_builder** out) {
    JG_GUARD_BEGIN
    JG_ARG(ctx && out, "null argument");
    *out = nullptr;
    auto b = std::make_unique<jg_builder>(&ctx->impl);
    *out = b.release();
    JG_GUARD_END
}

int jg_builder_destroy(jg_builder* b) {
    JG_GUARD_BEGIN
    delete b;
    JG_GUARD_END
}

extern "C++" {
namespace {
int builder_device(const jg_builder* b) { return b->ctx->devices.empty() ? 0 : b->ctx->devices[0]; }
hipStream_t builder_stream(const jg_builder* b) { return b->ctx->streams.empty() ? nullptr : b->ctx->streams[0]; }
template <class T>
void builder_append(jg::DevBuf<T>& acc, int64_t& len, const T* host, int64_t k, hipStream_t s) {
    if (k <= 0) return;
    if ((int64_t)acc.size() < len + k) {
        jg::DevBuf<T> bigger(std::max<int64_t>(len + k, 2 * (int64_t)acc.size()));
        if (len) JG_HIP(hipMemcpyAsync(bigger.get(), acc.get(), (size_t)len * sizeof(T), hipMemcpyDeviceToDevice, s));
        JG_HIP(hipStreamSynchronize(s));
        acc.swap(bigger);
    }
    jg::copy_h2d(acc.get() + len, host, (size_t)k * sizeof(T), s);
    len += k;
}
}  // namespace
}  // extern "C++"

int jg_builder_add_vertices(jg_builder* b, const int64_t* vid, int64_t n) {
    JG_GUARD_BEGIN
    JG_ARG(b && n >= 0 && (n == 0 || vid), "bad arguments");
    if (b->finished) jg::fail(JG_ERR_STATE, "builder already finished");
    if (b->mode == 2) jg::fail(JG_ERR_STATE, "builder holds edgestore rows: vertices come from the rows");
    b->mode = 1;
    jg::DeviceGuard dg(builder_device(b));
    builder_append(b->vid, b->n, vid, n, builder_stream(b));
    JG_GUARD_END
}

int jg_builder_add_edges(jg_builder* b, const int64_t* src, const int64_t* dst, const int32_t* weight, int64_t m) {
    JG_GUARD_BEGIN
    JG_ARG(b && m >= 0 && (m == 0 || (src && dst)), "bad arguments");
    if (b->finished) jg::fail(JG_ERR_STATE, "builder already finished");
    if (b->mode == 2) jg::fail(JG_ERR_STATE, "builder holds edgestore rows: edges come from the rows");
    if (m == 0) return JG_OK;
    const int wmode = weight ? 1 : 0;
    if (b->weights >= 0 && b->weights != wmode) jg::fail(JG_ERR_ARG, "edge weights must be given for every chunk or none");
    b->weights = wmode;
    b->mode = 1;
    jg::DeviceGuard dg(builder_device(b));
    hipStream_t s = builder_stream(b);
    int64_t m2 = b->m;
    builder_append(b->src, b->m, src, m, s);
    builder_append(b->dst, m2, dst, m, s);
    if (weight) builder_append(b->w, b->mw, weight, m, s);
    JG_GUARD_END
}

int jg_builder_set_schema(jg_builder* b, const int64_t* type_ids, const int8_t* type_mult, int32_t ntypes,
                          int32_t partition_bits) {
    JG_GUARD_BEGIN
    JG_ARG(b && ntypes >= 0 && (ntypes == 0 || (type_ids && type_mult)), "bad arguments");
    JG_ARG(partition_bits >= 0 && partition_bits <= 16, "partition bits must be in [0, 16]");
    if (b->finished || b->mode != 0) jg::fail(JG_ERR_STATE, "jg_builder_set_schema must precede every chunk");
    b->type_ids.assign(type_ids, type_ids + ntypes);
    b->type_mult.assign(type_mult, type_mult + ntypes);
    b->pbits = partition_bits;
    b->schema_set = true;
    JG_GUARD_END
}

int jg_builder_set_query_limit(jg_builder* b, int64_t limit, int32_t in_entries) {
    JG_GUARD_BEGIN
    JG_ARG(b, "null builder");
    JG_ARG(limit >= 0, "the query limit must be >= 0 (0: no limit)");
    JG_ARG(in_entries == JG_DIR_IN || in_entries == JG_DIR_OUT, "in_entries must be JG_DIR_IN or JG_DIR_OUT");
    if (b->finished || b->mode == 2) jg::fail(JG_ERR_STATE, "jg_builder_set_query_limit must precede every chunk");
    if (b->mode == 1) jg::fail(JG_ERR_STATE, "a query limit applies to edgestore rows, not to vertex / edge ids");
    b->query_limit = limit;
    b->in_entries = in_entries;
    JG_GUARD_END
}

int jg_builder_set_weight_key(jg_builder* b, int64_t weight_key, const int64_t* key_ids, const int8_t* key_types,
                              int32_t nkeys) {
    JG_GUARD_BEGIN
    JG_ARG(b, "null builder");
    JG_ARG(weight_key >= 0 && nkeys >= 0 && (nkeys == 0 || (key_ids && key_types)), "bad weight key arguments");
    for (int32_t i = 0; i < nkeys; ++i)
        JG_ARG(key_types[i] >= 0 && key_types[i] <= JG_PROP_STRING, "property type outside JG_PROP_*");
    if (b->finished || b->mode != 0) jg::fail(JG_ERR_STATE, "jg_builder_set_weight_key must precede every chunk");
    b->weight_key = true;
    b->wkey = weight_key;
    b->wkey_ids.assign(key_ids, key_ids + nkeys);
    b->wkey_types.assign(key_types, key_types + nkeys);
    JG_GUARD_END
}

int jg_builder_add_rows(jg_builder* b, const uint64_t* row_keys, int64_t nrows, const int64_t* row_entry_off,
                        const uint8_t* bytes, int64_t nbytes, const int64_t* entry_off, const int32_t* value_pos,
                        const int32_t* entry_weight, int64_t nentries) {
    JG_GUARD_BEGIN
    JG_ARG(b, "null builder");
    if (b->finished) jg::fail(JG_ERR_STATE, "builder already finished");
    if (b->mode == 1) jg::fail(JG_ERR_STATE, "builder holds vertex / edge ids: rows cannot be mixed in");
    b->mode = 2;
    if (!b->dec) {
        b->dec = std::make_unique<jg::EdgestoreDecoder>(b->type_ids.data(), b->type_mult.data(),
                                                        (int32_t)b->type_ids.size(), b->pbits, builder_device(b));
        b->dec->set_query_limit(b->query_limit);
        if (b->weight_key)
            b->dec->set_weight_key(b->wkey, b->wkey_ids.data(), b->wkey_types.data(), (int32_t)b->wkey_ids.size());
    }
    jg::EdgestoreRows r{row_keys, nrows,      row_entry_off, bytes,
                        nbytes,   entry_off,  value_pos,     nentries,
                        b->type_ids.data(), b->type_mult.data(), (int32_t)b->type_ids.size(), b->pbits};
    r.weight = entry_weight;
    b->dec->add(r);
    JG_GUARD_END
}

int jg_builder_finish(jg_builder* b, uint32_t flags, jg_graph** out) {
    JG_GUARD_BEGIN
    JG_ARG(b && out, "null argument");
    JG_ARG((flags & (JG_ADJ_IN | JG_ADJ_OUT | JG_ADJ_BOTH)) != 0 && (flags & ~7u) == 0, "bad adjacency flags");
    if (b->finished) jg::fail(JG_ERR_STATE, "builder already finished");
    *out = nullptr;
    jg::Ctx& c = *b->ctx;
    auto gh = std::make_unique<jg_graph>(&c);
    jg::Graph& g = gh->impl;
    g.flags = flags;
    jg::make_shards(c, g);
    jg::BuildTimer timer(g);
    const int dev0 = builder_device(b);
    float decode_ms = 0, copy_ms = 0;
    int64_t chunks = 0;
    if (b->mode == 2) {
        b->dec->finish();
        decode_ms = b->dec->kernel_ms;
        copy_ms = b->dec->copy_ms;
        chunks = b->dec->chunks_added_;
        jg::EdgestoreDecoder& d = *b->dec;
        if (d.weighted == 1 && d.w.size() == 0) d.w.alloc(1);
        jg::CappedIds cap;
        if (d.query_limit() > 0 && d.weighted == 1 && b->in_entries == JG_DIR_IN)
            jg::fail(JG_ERR_ARG, "entry weights under a query limit need in_entries = JG_DIR_OUT (ShortestDistance "
                                 "reads its OUT entries)");
        if (d.query_limit() > 0) {
            for (auto* buf : {&d.osrc, &d.isrc, &d.idst})
                if (buf->size() == 0) buf->alloc(1);
            cap.osrc = d.osrc.get();
            cap.isrc = d.isrc.get();
            cap.idst = d.idst.get();
            cap.mi = d.mi;
            cap.in_from_in = b->in_entries == JG_DIR_IN;
            cap.truncated_rows = d.truncated_rows;
        }
        jg::build_from_device_ids(g, dev0, builder_stream(b), d.vid.get(), d.n, d.src.get(), d.dst.get(),
                                  d.weighted == 1 ? d.w.get() : nullptr, d.m, d.query_limit() > 0 ? &cap : nullptr);
    } else {
        jg::DeviceGuard dg(dev0);
        if (b->vid.size() == 0) b->vid.alloc(1);
        if (b->src.size() == 0) { b->src.alloc(1); b->dst.alloc(1); }
        jg::build_from_device_ids(g, dev0, builder_stream(b), b->vid.get(), b->n, b->src.get(), b->dst.get(),
                                  b->weights == 1 ? b->w.get() : nullptr, b->m);
    }
    const float ms = timer.stop();
    b->finished = true;
    b->dec.reset();
    {
        jg::DeviceGuard dg(dev0);
        b->vid.reset();
        b->src.reset();
        b->dst.reset();
        b->w.reset();
    }
    c.last = jg_stats{};
    c.last.build_ms = ms;
    c.last.kernel_ms_total = decode_ms;
    c.last.exchange_ms = copy_ms;
    c.last.kernel_launches = chunks;
    *out = gh.release();
    JG_GUARD_END
}

int jg_graph_vertex_ids(const jg_graph* g, int64_t offset, int64_t count, int64_t* vid_out) {
    JG_GUARD_BEGIN
    JG_ARG(g && (count == 0 || vid_out), "null argument");
    const jg::Graph& gr = g->impl;
    JG_ARG(offset >= 0 && count >= 0 && offset + count <= gr.n, "range outside [0, num_vertices)");
    for (int64_t i = 0; i < count; ++i) vid_out[i] = gr.vid_of(offset + i);
    JG_GUARD_END
}

int jg_graph_build_rmat(jg_ctx* ctx, int scale, int edgefactor, uint64_t seed, uint32_t flags, jg_graph** out) {
    JG_GUARD_BEGIN
    JG_ARG(ctx && out, "null argument");
    JG_ARG(scale >= 1 && scale <= 30 && edgefactor >= 1 && edgefactor <= 64, "bad RMAT scale/edgefactor");
    JG_ARG((flags & (JG_ADJ_IN | JG_ADJ_OUT | JG_ADJ_BOTH)) != 0 && (flags & ~7u) == 0, "bad adjacency flags");
    *out = nullptr;
    const int64_t n = 1ll << scale, m = (int64_t)edgefactor << scale;
    JG_ARG(m < (int64_t)UINT32_MAX, "too many edges");
    jg::Ctx& c = ctx->impl;
    auto gh = std::make_unique<jg_graph>(&c);
    jg::Graph& g = gh->impl;
    g.n = n;
    g.flags = flags;
    jg::make_shards(c, g);
    hipEvent_t t0, t1;
    {
        jg::DeviceGuard dg(g.shards[0]->device);
        JG_HIP(hipEventCreate(&t0));
        JG_HIP(hipEventCreate(&t1));
        JG_HIP(hipEventRecord(t0, g.shards[0]->stream));
    }
    std::vector<jg::DevBuf<int32_t>> ds(g.shards.size()), dd(g.shards.size());
    jg::DenseEdges e;
    e.m = m;
    for (size_t i = 0; i < g.shards.size(); ++i) {
        jg::Shard& sh = *g.shards[i];
        jg::DeviceGuard dg(sh);
        ds[i].alloc(m);
        dd[i].alloc(m);
        jg::generate_rmat_device(scale, seed, m, ds[i].get(), dd[i].get(), sh.stream);
        e.src.push_back(ds[i].peer());
        e.dst.push_back(dd[i].peer());
        e.weight.push_back(nullptr);
    }
    jg::build_graph_from_dense(g, e);
    {
        jg::DeviceGuard dg(g.shards[0]->device);
        JG_HIP(hipEventRecord(t1, g.shards[0]->stream));
        JG_HIP(hipEventSynchronize(t1));
        float ms = 0;
        JG_HIP(hipEventElapsedTime(&ms, t0, t1));
        c.last = jg_stats{};
        c.last.build_ms = ms;
        (void)hipEventDestroy(t0);
        (void)hipEventDestroy(t1);
    }
    *out = gh.release();
    JG_GUARD_END
}

int jg_graph_info_get(const jg_graph* g, jg_graph_info* out) {
    JG_GUARD_BEGIN
    JG_ARG(g && out, "null argument");
    *out = g->impl.info;
    const jg::Graph& gr = g->impl;
    out->exchange_values = 0;
    if (gr.P > 1) {
        const uint32_t adj = (gr.flags & JG_ADJ_IN) ? JG_ADJ_IN : JG_ADJ_BOTH;
        for (const auto& sp : gr.shards) {
            const jg::Halo& h = gr.halo(*sp, adj);
            if (!h.on) {
                out->exchange_values += (int64_t)(gr.P - 1) * gr.S;
                continue;
            }
            for (int q = 0; q < gr.P; ++q)
                if (q != sp->index) out->exchange_values += h.recv_off[q + 1] - h.recv_off[q];
        }
    }
    JG_GUARD_END
}

int jg_graph_destroy(jg_graph* g) {
    JG_GUARD_BEGIN
    if (!g) return JG_OK;
    std::vector<int> devs;
    for (auto& sp : g->impl.shards) {
        jg::DeviceGuard dg(*sp);
        (void)hipStreamSynchronize(sp->stream);
        if (std::find(devs.begin(), devs.end(), sp->device) == devs.end()) devs.push_back(sp->device);
    }
    // The snapshot's device memory goes back to the device, not to the library's block cache (ADVICE r03:
    // a dropped snapshot must not keep memory from other users of the device for the context's lifetime).
    // Its streams are synchronised above, so its blocks are freed directly, and the cache's ready blocks
    // go back without a device-wide synchronisation (that blocked on other contexts' work);
    // blocks other callers freed and not yet synchronised stay pending.
    {
        jg::DirectFree direct;
        delete g;
    }
    for (int d : devs) jg::dev_cache_drop_ready(d);
    JG_GUARD_END
}

int jg_ctx_trim(jg_ctx* ctx) {
    JG_GUARD_BEGIN
    JG_ARG(ctx, "null context");
    jg::Ctx& c = ctx->impl;
    for (size_t i = 0; i < c.devices.size(); ++i)
        if (!(c.logical && i > 0)) jg::dev_cache_release(c.devices[i]);
    JG_GUARD_END
}

int jg_graph_sync(jg_graph* g) {
    JG_GUARD_BEGIN
    JG_ARG(g, "null graph");
    for (auto& sp : g->impl.shards) {
        jg::DeviceGuard dg(*sp);
        JG_HIP(hipStreamSynchronize(sp->stream));
    }
    JG_GUARD_END
}

int jg_pagerank_begin(jg_graph* g, double damping, int64_t vertex_count) {
    JG_GUARD_BEGIN
    JG_ARG(g, "null graph");
    g->impl.ctx->last = jg_stats{};
    jg::pagerank_begin(g->impl, damping, vertex_count);
    JG_GUARD_END
}

int jg_pagerank_step(jg_graph* g, int32_t nsteps) {
    JG_GUARD_BEGIN
    JG_ARG(g && nsteps >= 0, "bad arguments");
    jg::pagerank_steps(g->impl, nsteps);
    JG_GUARD_END
}

int jg_pagerank_end(jg_graph* g, double* rank_out, double* edge_count_out) {
    JG_GUARD_BEGIN
    JG_ARG(g, "null graph");
    jg::pagerank_end(g->impl, rank_out, edge_count_out);
    jg::Graph& gr = g->impl;
    jg::Ctx& c = *gr.ctx;
    c.last.supersteps = gr.pr_steps + 1;
    double nnz = 0;
    for (auto& sp : gr.shards) nnz += (double)sp->in.nnz;
    c.last.edges_traversed = nnz * gr.pr_steps;
    c.last.algorithmic_bytes = (12.0 * nnz + 32.0 * (double)gr.n) * gr.pr_steps;
    JG_GUARD_END
}

int jg_pagerank(jg_graph* g, double damping, int64_t vertex_count, int32_t iterations, double* rank_out,
                double* edge_count_out) {
    JG_GUARD_BEGIN
    JG_ARG(g, "null graph");
    JG_ARG(iterations >= 0, "negative iterations");
    jg::Graph& gr = g->impl;
    if (iterations == 0) {  // only superstep 0 runs: no property is written
        if (rank_out) std::fill(rank_out, rank_out + gr.n, std::numeric_limits<double>::quiet_NaN());
        if (edge_count_out) std::fill(edge_count_out, edge_count_out + gr.n, std::numeric_limits<double>::quiet_NaN());
        gr.ctx->last = jg_stats{};
        return JG_OK;
    }
    gr.ctx->last = jg_stats{};
    jg::Shard& sh0 = *gr.shards[0];
    jg::DeviceGuard dg(sh0.device);
    hipEvent_t t0, t1;
    JG_HIP(hipEventCreate(&t0));
    JG_HIP(hipEventCreate(&t1));
    JG_HIP(hipEventRecord(t0, sh0.stream));
    jg::pagerank_begin(gr, damping, vertex_count);
    jg::pagerank_steps(gr, iterations - 1);
    JG_HIP(hipEventRecord(t1, sh0.stream));
    jg::pagerank_end(gr, rank_out, edge_count_out);
    float ms = 0;
    JG_HIP(hipEventSynchronize(t1));
    JG_HIP(hipEventElapsedTime(&ms, t0, t1));
    (void)hipEventDestroy(t0);
    (void)hipEventDestroy(t1);
    jg::Ctx& c = *gr.ctx;
    c.last.compute_ms = ms;
    c.last.supersteps = iterations;
    double nnz = 0;
    for (auto& sp : gr.shards) nnz += (double)sp->in.nnz;
    c.last.edges_traversed = nnz * (iterations - 1);
    c.last.algorithmic_bytes = (12.0 * nnz + 32.0 * (double)gr.n) * (iterations - 1);
    JG_GUARD_END
}

int jg_shortest_distance(jg_graph* g, int64_t seed_vid, int32_t max_depth, int64_t* dist_out) {
    JG_GUARD_BEGIN
    JG_ARG(g && dist_out, "null argument");
    JG_ARG(max_depth >= 0, "negative maxDepth");
    jg::shortest_distance_run(g->impl, seed_vid, max_depth, dist_out);
    JG_GUARD_END
}

int jg_bfs(jg_graph* g, const int64_t* source_vids, int32_t nsrc, int32_t direction, int32_t max_depth,
           int32_t* depth_out) {
    JG_GUARD_BEGIN
    JG_ARG(g && source_vids, "null argument");
    JG_ARG(nsrc > 0, "nsrc must be positive");
    std::vector<int32_t*> rows;
    if (depth_out)
        for (int32_t s = 0; s < nsrc; ++s) rows.push_back(depth_out + (int64_t)s * g->impl.n);
    jg::bfs_run(g->impl, source_vids, nsrc, direction, max_depth, depth_out ? rows.data() : nullptr);
    JG_GUARD_END
}

int jg_bfs_rows(jg_graph* g, const int64_t* source_vids, int32_t nsrc, int32_t direction, int32_t max_depth,
                int32_t* const* depth_rows) {
    JG_GUARD_BEGIN
    JG_ARG(g && source_vids, "null argument");
    jg::bfs_run(g->impl, source_vids, nsrc, direction, max_depth, depth_rows);
    JG_GUARD_END
}

int jg_bfs_keep(jg_graph* g, const int64_t* source_vids, int32_t nsrc, int32_t direction, int32_t max_depth) {
    JG_GUARD_BEGIN
    JG_ARG(g && source_vids, "null argument");
    jg::bfs_run(g->impl, source_vids, nsrc, direction, max_depth, nullptr, true);
    JG_GUARD_END
}

int jg_bfs_kept_row(jg_graph* g, int32_t s, int32_t* depth_out) {
    JG_GUARD_BEGIN
    JG_ARG(g && depth_out, "null argument");
    jg::bfs_kept_row(g->impl, s, depth_out);
    JG_GUARD_END
}

int jg_bfs_kept_release(jg_graph* g) {
    JG_GUARD_BEGIN
    JG_ARG(g, "null graph");
    jg::bfs_kept_release(g->impl);
    JG_GUARD_END
}

int jg_graph_neighbors(const jg_graph* g, int32_t direction, const int64_t* rows, int64_t nrows, int64_t* off_out,
                       int64_t* nbr_out) {
    JG_GUARD_BEGIN
    JG_ARG(g, "null graph");
    jg::graph_neighbors(g->impl, direction, rows, nrows, off_out, nbr_out);
    JG_GUARD_END
}

int jg_decode_edges(jg_ctx* ctx, const uint8_t* bytes, int64_t nbytes, const int64_t* entry_off,
                    const int32_t* value_pos, int64_t n, const int64_t* type_ids, const int8_t* type_mult,
                    int32_t ntypes, int64_t* type_out, int8_t* dir_out, int64_t* other_out, int64_t* relation_out) {
    JG_GUARD_BEGIN
    JG_ARG(ctx, "null context");
    jg::decode_edges(ctx->impl, bytes, nbytes, entry_off, value_pos, n, type_ids, type_mult, ntypes, type_out, dir_out,
                     other_out, relation_out);
    JG_GUARD_END
}

int jg_combine_steps(jg_graph* g, int32_t direction, int32_t combiner, int32_t int32_wrap, const int64_t* init,
                     int32_t steps, int64_t* out, uint8_t* received_out) {
    JG_GUARD_BEGIN
    JG_ARG(g, "null graph");
    JG_ARG(out || g->impl.n == 0, "null output");
    jg::combine_run(g->impl, direction, combiner, int32_wrap, init, steps, out, received_out);
    JG_GUARD_END
}

int jg_connected_components(jg_graph* g, int64_t* component_vid_out, int32_t* iterations_out) {
    JG_GUARD_BEGIN
    JG_ARG(g, "null graph");
    jg::cc_run(g->impl, component_vid_out, iterations_out);
    JG_GUARD_END
}

}  // extern "C"
