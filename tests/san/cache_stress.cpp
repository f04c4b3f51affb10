// Host stress test of the device block cache (janusgraph_amd/csrc/jg_cache.h) under ASan/UBSan and TSan
// (tests/test_sanitizers.py): the cache over a malloc backend, hammered by threads that allocate, stamp,
// check and free blocks of random size classes on two "devices" while others synchronise, release and
// drop ready blocks.  A block handed to two owners at once fails the stamp check; a block the cache gave
// back to the backend while still owned is a heap-use-after-free under ASan; unsynchronised access to the
// cache's maps is a data race under TSan.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "jg_cache.h"

namespace {
std::atomic<long> g_live{0}, g_syncs{0};
struct MallocBackend {
    void* alloc(int, size_t bytes) {
        g_live.fetch_add(1, std::memory_order_relaxed);
        return std::malloc(bytes);
    }
    void release(int, void* p) {
        g_live.fetch_sub(1, std::memory_order_relaxed);
        std::free(p);
    }
    void synchronize(const std::vector<int>&) { g_syncs.fetch_add(1, std::memory_order_relaxed); }
};
}  // namespace

int main(int argc, char** argv) {
    const int threads = argc > 1 ? std::atoi(argv[1]) : 8;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 20000;
    jg::BlockCache<MallocBackend> cache;
    std::atomic<int> bad{0};
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
        pool.emplace_back([&, t] {
            std::mt19937_64 rng(1234 + t);
            struct Held {
                void* p;
                size_t bytes;
                int dev;
                unsigned long long stamp;
            };
            std::vector<Held> held;
            for (int i = 0; i < iters; ++i) {
                const unsigned op = (unsigned)(rng() % 100);
                if (op < 55 || held.empty()) {
                    const size_t bytes = 64 + (size_t)(rng() % 6) * 4096 + (rng() % 3 ? 0 : (size_t)(rng() % 200000));
                    const int dev = (int)(rng() % 2);
                    void* p = cache.alloc(dev, bytes);
                    if (!p) {
                        bad.fetch_add(1);
                        continue;
                    }
                    const unsigned long long stamp = ((unsigned long long)t << 40) | (unsigned long long)i;
                    std::memcpy(p, &stamp, sizeof stamp);
                    std::memset(static_cast<char*>(p) + sizeof stamp, t & 0xFF, bytes - sizeof stamp);
                    held.push_back({p, bytes, dev, stamp});
                } else if (op < 95) {
                    const size_t k = (size_t)(rng() % held.size());
                    Held h = held[k];
                    held[k] = held.back();
                    held.pop_back();
                    unsigned long long now = 0;
                    std::memcpy(&now, h.p, sizeof now);
                    const unsigned char last = static_cast<unsigned char*>(h.p)[h.bytes - 1];
                    if (now != h.stamp || last != (unsigned char)(t & 0xFF)) bad.fetch_add(1);  // another owner wrote it
                    cache.free(h.dev, h.p, h.bytes, rng() % 16 == 0);
                } else if (op < 98) {
                    cache.sync();
                } else if (op < 99) {
                    cache.drop_ready((int)(rng() % 2));
                } else {
                    cache.release((int)(rng() % 2));
                }
            }
            for (const Held& h : held) cache.free(h.dev, h.p, h.bytes);
        });
    for (auto& th : pool) th.join();
    cache.release(0);
    cache.release(1);
    std::printf("cache_stress: %d threads x %d ops, %ld blocks still with the backend, %ld synchronisations, %d bad\n",
                threads, iters, g_live.load(), g_syncs.load(), bad.load());
    return bad.load() == 0 && g_live.load() == 0 ? 0 : 1;
}
