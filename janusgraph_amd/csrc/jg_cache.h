// jg_cache.h — the block cache behind DevBuf (jg_common.h), backend-agnostic.
//
// hipFree synchronises the whole device and a snapshot build frees ~240 temporaries, so freed blocks of
// up to kBlockMax bytes are kept per device and size class.  A freed block is "pending" until every device
// holding cached memory has been synchronised after its free (sync(): at the end of every entry point that
// left blocks pending); only synchronised ("ready") blocks are handed out again, so a block is never reused
// while work queued before its free may still touch it.
//
// The Backend supplies the device side: void* alloc(int dev, size_t), void release(int dev, void*) (the
// real free) and void synchronize(const std::vector<int>& devs).  jg_api.cpp instantiates it over HIP;
// tests/san/cache_stress.cpp over malloc, to run the locking under ASan and TSan on the host (SURVEY.md
// §5 race detection; the reference's VertexState mutators are `synchronized`, VertexState.java:77,85,135).
#pragma once

#include <cstddef>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

namespace jg {

template <class Backend>
class BlockCache {
   public:
    static constexpr size_t kBlockMax = 1ull << 30;  // larger blocks go straight to the backend
    static constexpr size_t kBytesMax = 16ull << 30; // per device: beyond it, synchronise and free half

    explicit BlockCache(Backend b = Backend{}) : be_(std::move(b)) {}

    // size class: at most 1/8 above the request (granularity = a power of two >= 4 KiB, 1/8 of the
    // request's leading power of two)
    static size_t round(size_t b) {
        size_t top = 1;
        while (top * 2 <= b) top *= 2;
        const size_t g = top / 8 > 4096 ? top / 8 : 4096;
        return (b + g - 1) / g * g;
    }

    // nullptr when the device is out of memory even after the cached blocks went back
    void* alloc(int dev, size_t bytes) {
        const bool cached = !off_ && bytes <= kBlockMax;
        const size_t rb = cached ? round(bytes) : bytes;
        if (cached) {
            std::lock_guard<std::mutex> lk(mu_);
            Dev& c = devs_[dev];
            auto it = c.ready.find(rb);
            if (it != c.ready.end()) {
                void* p = it->second;
                c.ready.erase(it);
                c.bytes -= rb;
                return p;
            }
        }
        void* p = be_.alloc(dev, rb);
        if (!p) {
            release(dev);  // hand the cached blocks back, then try once more
            p = be_.alloc(dev, rb);
        }
        return p;
    }

    // direct: the caller has synchronised every stream that used the block (jg_graph_destroy), so it
    // goes back to the backend at once instead of into the cache
    void free(int dev, void* p, size_t bytes, bool direct = false) {
        if (!p) return;
        if (off_ || direct || bytes > kBlockMax) {
            be_.release(dev, p);
            return;
        }
        bool over = false;
        {
            std::lock_guard<std::mutex> lk(mu_);
            Dev& c = devs_[dev];
            const size_t rb = round(bytes);
            c.pending.emplace_back(rb, p);
            c.bytes += rb;
            over = c.bytes > kBytesMax;
        }
        if (over) sync_dev(dev, true);
    }

    // pending blocks of every device become reusable
    void sync() {
        std::vector<int> devs;
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (auto& kv : devs_)
                if (!kv.second.pending.empty()) devs.push_back(kv.first);
        }
        for (int d : devs) sync_dev(d, false);
    }

    // synchronise, then return every cached block of dev to the backend
    void release(int dev) {
        sync_dev(dev, false);
        drop_ready(dev);
    }

    // return dev's ready blocks to the backend without synchronising anything (they were synchronised
    // when they became ready); pending blocks stay
    void drop_ready(int dev) {
        std::vector<void*> drop;
        {
            std::lock_guard<std::mutex> lk(mu_);
            Dev& c = devs_[dev];
            for (auto& kv : c.ready) drop.push_back(kv.second);
            c.ready.clear();
            c.bytes = 0;
            for (auto& b : c.pending) c.bytes += b.first;
        }
        for (void* p : drop) be_.release(dev, p);
    }

    void set_off(bool off) { off_ = off; }
    size_t cached_bytes(int dev) {
        std::lock_guard<std::mutex> lk(mu_);
        return devs_[dev].bytes;
    }

   private:
    struct Dev {
        std::multimap<size_t, void*> ready;            // synchronised since their free: reusable
        std::vector<std::pair<size_t, void*>> pending;  // freed since the device's last synchronisation
        size_t bytes = 0;                               // ready + pending
    };
    // synchronise every device that holds cached memory (a block of one device may be read by another's
    // peer copy) and move dev's pending blocks taken before the synchronisation to ready; with `trim`,
    // free ready blocks until the cache holds at most half its cap
    void sync_dev(int dev, bool trim) {
        std::vector<std::pair<size_t, void*>> snap;
        std::vector<int> devs;
        {
            std::lock_guard<std::mutex> lk(mu_);
            snap.swap(devs_[dev].pending);
            for (auto& kv : devs_) devs.push_back(kv.first);
        }
        if (snap.empty() && !trim) return;
        be_.synchronize(devs);
        std::vector<void*> drop;
        {
            std::lock_guard<std::mutex> lk(mu_);
            Dev& c = devs_[dev];
            for (auto& b : snap) c.ready.emplace(b.first, b.second);
            while (trim && c.bytes > kBytesMax / 2 && !c.ready.empty()) {
                auto it = std::prev(c.ready.end());  // the largest first
                c.bytes -= it->first;
                drop.push_back(it->second);
                c.ready.erase(it);
            }
        }
        for (void* p : drop) be_.release(dev, p);
    }

    Backend be_;
    std::mutex mu_;
    std::map<int, Dev> devs_;
    bool off_ = false;
};

}  // namespace jg
