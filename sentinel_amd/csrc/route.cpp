// Host-side event routing for the multi-GPU token server: rules shard by
// splitmix64(flowId) mod G, and a global batch is split into G per-shard batches by a stable
// counting sort, so every shard sees its requests in arrival order (per-rule order is all the
// decisions depend on).  T threads: each counts a contiguous slice, the per-(shard, thread)
// offsets are one exclusive scan in shard-major / thread-minor order, then each thread places its
// slice -- stable because slices are in arrival order.
#include "../../include/sentinel_amd.h"
#include "common.hpp"

#include <algorithm>
#include <cerrno>
#include <thread>
#include <vector>

extern "C" int sga_route_shards(const int64_t *flow_id, size_t n, uint32_t n_shards, uint32_t n_threads,
                                uint32_t *order, uint64_t *shard_off) {
    if ((n && (!flow_id || !order)) || !shard_off || n_shards == 0 || n_shards > 4096) return -EINVAL;
    if (n_threads == 0) n_threads = 1;
    n_threads = (uint32_t)std::min<size_t>(n_threads, std::max<size_t>(1, n / 65536 + 1));
    if (n > 0xFFFFFFFFull) return -ERANGE;
    const size_t T = n_threads, G = n_shards;
    std::vector<uint64_t> cnt(T * G, 0);  // [thread][shard]
    auto slice = [&](size_t t, size_t &lo, size_t &hi) {
        lo = n * t / T;
        hi = n * (t + 1) / T;
    };
    auto count = [&](size_t t) {
        size_t lo, hi;
        slice(t, lo, hi);
        uint64_t *c = cnt.data() + t * G;
        for (size_t i = lo; i < hi; ++i) ++c[sga::splitmix64((uint64_t)flow_id[i]) % G];
    };
    auto place = [&](size_t t, std::vector<uint64_t> &pos) {
        size_t lo, hi;
        slice(t, lo, hi);
        uint64_t *p = pos.data() + t * G;
        for (size_t i = lo; i < hi; ++i) order[p[sga::splitmix64((uint64_t)flow_id[i]) % G]++] = (uint32_t)i;
    };
    std::vector<std::thread> th;
    for (size_t t = 1; t < T; ++t) th.emplace_back(count, t);
    count(0);
    for (auto &x : th) x.join();
    th.clear();
    std::vector<uint64_t> pos(T * G);
    uint64_t run = 0;
    for (size_t g = 0; g < G; ++g) {
        shard_off[g] = run;
        for (size_t t = 0; t < T; ++t) {
            pos[t * G + g] = run;
            run += cnt[t * G + g];
        }
    }
    shard_off[G] = run;
    for (size_t t = 1; t < T; ++t) th.emplace_back(place, t, std::ref(pos));
    place(0, pos);
    for (auto &x : th) x.join();
    return 0;
}
