// jg_common.h — shared internals of libjanusgpu (gfx950 only; wave64).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace jg {

constexpr int kWave = 64;    // CDNA wavefront width
constexpr int kBlock = 256;  // threads per workgroup for every kernel in the library

// Internal failures travel as exceptions and are turned into status codes at the C-ABI
// (jg_api.cpp); nothing crosses the ABI as an exception.
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

[[noreturn]] void fail(int code, const std::string& msg);
void hip_check(hipError_t e, const char* what, const char* file, int line);

#define JG_HIP(call) ::jg::hip_check((call), #call, __FILE__, __LINE__)
#define JG_LAUNCH_CHECK() ::jg::hip_check(hipGetLastError(), "kernel launch", __FILE__, __LINE__)

// Device memory behind DevBuf (jg_api.cpp over jg_cache.h).  hipFree synchronises the whole device,
// and a snapshot build frees ~240 temporaries (RMAT-20: 9.6 ms of a 49 ms build went to hipFree), so
// freed blocks of up to 1 GiB are kept per device and size class instead.  A freed block is "pending"
// until the device has been synchronised once after its free (dev_cache_sync: at the end of every entry
// point that left blocks pending); only synchronised blocks are handed out again, so a block is never
// reused while work queued before its free may still touch it (what hipFree guaranteed per call).
// JG_NO_DEVCACHE=1 in the environment restores plain hipMalloc / hipFree.
void* dev_alloc(size_t bytes);                 // current device; nullptr when the device is out of memory
void dev_free(void* p, size_t bytes, int dev);
void dev_cache_sync();                          // pending blocks of every device become reusable
void dev_cache_release(int dev);                // synchronise and return every cached block of dev
void dev_cache_drop_ready(int dev);             // return dev's synchronised blocks (no synchronisation)
// While one is alive on a thread, DevBuf frees on that thread bypass the cache (the caller has
// synchronised every stream that used the blocks).
struct DirectFree {
    bool prev;
    DirectFree();
    ~DirectFree();
};

// Virtual-device check (JG_VDEV_CHECK=1, logical shards).  A context that drives
// several devices in one process (computer.gpu.devices=0,1,...) must keep every shard's buffers on that
// shard's device.  Logical shards share one device, so there a misplaced buffer works and no test sees
// it.  In the check mode every logical shard is a "virtual device": DeviceGuard(shard) makes the shard's
// tag current on the thread, each DevBuf records the tag current at its allocation, and DevBuf::get()
// under another shard's guard fails the call (vdev_violation: JG_ERR_STATE) instead of handing a kernel
// or copy on that shard's stream a pointer of another device.  A plain DeviceGuard(int) is graph-level
// work on the first device: tag 0 (the first shard's) in the check mode, so a per-shard buffer
// allocated there is caught too.  Tag -1 (outside the check mode) checks nothing.  peer() is the
// unchecked accessor for deliberate accesses across devices (the exchange's peer copies) and for
// collecting pointers that another shard's guard will use.  JG_VDEV_CHECK=2 reports every violation
// (return addresses as library offsets) and continues.
inline thread_local int t_vtag = -1;
int vdev_mode();     // JG_VDEV_CHECK: 0 off, 1 fail, 2 report and continue
void vdev_refresh();  // re-read JG_VDEV_CHECK (jg_ctx_create)
void vdev_violation(int buffer_tag, int current_tag);

// Owning device allocation (dev_alloc on the current device).
template <typename T>
class DevBuf {
   public:
    DevBuf() = default;
    explicit DevBuf(size_t n) { alloc(n); }
    ~DevBuf() { reset(); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p_(o.p_), n_(o.n_), dev_(o.dev_), tag_(o.tag_) { o.p_ = nullptr; o.n_ = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) { reset(); p_ = o.p_; n_ = o.n_; dev_ = o.dev_; tag_ = o.tag_; o.p_ = nullptr; o.n_ = 0; }
        return *this;
    }
    void alloc(size_t n) {
        reset();
        n_ = n;
        tag_ = t_vtag;
        JG_HIP(hipGetDevice(&dev_));
        if (n) {
            p_ = static_cast<T*>(dev_alloc(n * sizeof(T)));
            if (!p_) {
                n_ = 0;
                fail(-2, "device allocation of " + std::to_string(n * sizeof(T)) + " bytes failed");
            }
        }
    }
    void reset() {
        if (p_) dev_free(p_, n_ * sizeof(T), dev_);
        p_ = nullptr;
        n_ = 0;
    }
    T* get() const {
        if (tag_ >= 0 && t_vtag >= 0 && tag_ != t_vtag) vdev_violation(tag_, t_vtag);
        return p_;
    }
    T* peer() const { return p_; }  // a deliberate access from another shard's device (peer copies)
    size_t size() const { return n_; }
    size_t bytes() const { return n_ * sizeof(T); }
    int tag() const { return tag_; }
    void swap(DevBuf& o) {
        std::swap(p_, o.p_);
        std::swap(n_, o.n_);
        std::swap(dev_, o.dev_);
        std::swap(tag_, o.tag_);
    }

   private:
    T* p_ = nullptr;
    size_t n_ = 0;
    int dev_ = 0;
    int tag_ = -1;  // the virtual device current at allocation (-1: none)
};

inline unsigned grid_for(int64_t work, int per_block = kBlock, int64_t cap = 256 * 16) {
    int64_t b = (work + per_block - 1) / per_block;
    if (b < 1) b = 1;
    if (cap > 0 && b > cap) b = cap;
    return static_cast<unsigned>(b);
}

inline int bits_for(uint64_t x) {  // number of bits to represent values in [0, x]
    int b = 0;
    while (b < 64 && (x >> b) != 0) ++b;
    return b;
}

// Host<->device copies ordered on the library's (non-blocking) stream `s`, then synchronised.
// Plain hipMemcpy runs on the legacy stream, which does NOT wait for non-blocking streams.
// Small read-backs (level counters and states, read once per level or batch) wait by polling the stream
// instead of a blocking synchronise: the host sees the end sooner (round 6, tools/workload.py medians of
// ten calls, blocking / polling: 64-source BFS RMAT-26 9.751 / 9.711 ms, CC RMAT-26 2.107 / 2.095 ms,
// delta-stepping RMAT-20 0.907 / 0.896 ms; profiles/r06/spin/).  JG_SPIN_SYNC=0 turns it off.
inline bool spin_sync_on() {
    static const int v = [] {
        const char* e = std::getenv("JG_SPIN_SYNC");
        return e ? std::atoi(e) : 1;
    }();
    return v != 0;
}
inline void copy_d2h(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (!bytes) return;
    JG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
    if (bytes <= 256 && spin_sync_on()) {
        hipError_t e;
        while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
        }
        JG_HIP(e);
        return;
    }
    JG_HIP(hipStreamSynchronize(s));
}
inline void copy_h2d(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (!bytes) return;
    JG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    JG_HIP(hipStreamSynchronize(s));
}

// RAII device switch.  DeviceGuard(shard) also makes the shard's virtual-device tag current (the
// check mode above); DeviceGuard(int) clears it (graph-level work, unchecked).
struct DeviceGuard {
    int prev = 0, prev_tag = -1;
    explicit DeviceGuard(int dev) : prev_tag(t_vtag) {
        JG_HIP(hipGetDevice(&prev));
        if (prev != dev) JG_HIP(hipSetDevice(dev));
        t_vtag = vdev_mode() ? 0 : -1;
    }
    template <class S, class = decltype(std::declval<const S&>().vtag)>
    explicit DeviceGuard(const S& sh) : DeviceGuard(sh.device) {
        t_vtag = sh.vtag;
    }
    ~DeviceGuard() {
        (void)hipSetDevice(prev);
        t_vtag = prev_tag;
    }
};

}  // namespace jg
