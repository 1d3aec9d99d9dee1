// Cluster concurrency tokens on the device (see concurrent.hpp for the reference map).
//
// conc_ops, per batch of n operations in arrival order:
//   k_conc_classify  validation (DefaultTokenService.requestConcurrentToken :67-78), rule lookup,
//                    token lookup for releases; packs (slot << 40 | index) for the sort
//   radix_sort_u64   stable by slot: each rule's operations stay in arrival order
//   k_conc_runs      one lane per rule present in the batch walks its operations in order:
//                    acquire = the double-checked nowCalls test + getAndAdd + a TokenCacheNode put,
//                    release = remove (CAS on the entry) + getAndAdd(-acquire)
// Different rules touch disjoint nowCalls counters; token inserts of different lanes meet only in
// the table, where a slot is claimed by CAS.
#include "concurrent.hpp"

namespace sga {

namespace {

constexpr int kThreads = 256;
constexpr int kIdxBits = 26;
constexpr int kSlotShift = 40;
constexpr uint32_t kNone = 0xFFFFFFFFu;

enum : int32_t { ST_BAD_REQUEST = -4, ST_OK = 0, ST_BLOCKED = 1, ST_NO_RULE_EXISTS = 3, ST_RELEASE_OK = 6,
                 ST_ALREADY_RELEASE = 7 };

struct alignas(16) ConcOut {
    int64_t token;
    int32_t status;
    int32_t pad;
};

__device__ __forceinline__ uint32_t tok_hash(int64_t token, uint32_t mask) {
    return (uint32_t)splitmix64((uint64_t)token ^ 0xC0DEC0DEULL) & mask;
}

// ClusterFlowRuleManager.getFlowRuleById: slot of an active rule, kNone when absent.
__device__ __forceinline__ uint32_t rule_slot(const ClusterState &cs, int64_t fid) {
    if (fid <= 0) return kNone;
    if (cs.dense_n) {
        if (fid > (int64_t)cs.dense_n) return kNone;
        const uint32_t u = (uint32_t)cs.dense[fid - 1];
        return u == ~0u ? kNone : (u & 0xFFFFFFu);
    }
    uint32_t h = (uint32_t)hash_flow_id(fid) & cs.hmask;
    for (uint32_t probe = 0; probe <= cs.hmask; ++probe) {
        const HashEntry e = cs.htab[h];
        if (e.key == fid) return e.slot;
        if (e.key == 0) return kNone;
        h = (h + 1) & cs.hmask;
    }
    return kNone;
}

// TokenCacheNodeManager.getTokenCacheNode: index of the live entry of `token`, kNone when absent.
__device__ __forceinline__ uint32_t tok_find(const ConcState &st, int64_t token) {
    uint32_t h = tok_hash(token, st.tmask);
    for (uint32_t probe = 0; probe <= st.tmask; ++probe) {
        const uint32_t s = __atomic_load_n(&st.tok[h].state, __ATOMIC_RELAXED);
        if (s == kTokEmpty) return kNone;
        if (s == kTokLive && st.tok[h].token == token) return h;
        h = (h + 1) & st.tmask;
    }
    return kNone;
}

// TokenCacheNodeManager.putTokenCacheNode.  The host keeps the table at most half full, so a free
// entry (empty, or a tombstone of an earlier epoch) is always reached.
__device__ __forceinline__ void tok_insert(TokenEntry *tab, uint32_t mask, uint32_t epoch, const TokenEntry &e) {
    uint32_t h = tok_hash(e.token, mask);
    const uint32_t cur_tomb = tok_tomb(epoch);
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        uint32_t s = __atomic_load_n(&tab[h].state, __ATOMIC_RELAXED);
        while (s == kTokEmpty || ((s & 3u) == 2u && s != cur_tomb)) {
            const uint32_t seen = atomicCAS(&tab[h].state, s, kTokBusy);
            if (seen == s) {
                TokenEntry &d = tab[h];
                d.token = e.token;
                d.flow_id = e.flow_id;
                d.client_deadline = e.client_deadline;
                d.resource_deadline = e.resource_deadline;
                d.acquire = e.acquire;
                d.client = e.client;
                __threadfence();
                atomicExch(&tab[h].state, kTokLive);
                return;
            }
            s = seen;
        }
        h = (h + 1) & mask;
    }
}

__global__ void __launch_bounds__(kThreads) k_conc_classify(ConcState st, const uint8_t *op, const uint32_t *client,
                                                            const int64_t *id, const int32_t *acquire, uint32_t n,
                                                            uint32_t invalid_key, uint64_t *el, uint32_t *aux,
                                                            ConcOut *out) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    uint32_t key = invalid_key;
    int32_t status = ST_OK;
    const int64_t x = id[i];
    if (op[i] == 0) {
        // notValidRequest(address, id, count), DefaultTokenService.java:92-94
        if (client[i] == kNone || x <= 0 || acquire[i] <= 0) {
            status = ST_BAD_REQUEST;
        } else {
            const uint32_t s = rule_slot(st.cs, x);
            if (s == kNone) status = ST_NO_RULE_EXISTS;  // :73-75
            else key = s;
        }
    } else {
        // ConcurrentClusterFlowChecker.releaseConcurrentToken :81-95
        const uint32_t e = tok_find(st, x);
        if (e == kNone) {
            status = ST_ALREADY_RELEASE;
        } else {
            const uint32_t s = rule_slot(st.cs, st.tok[e].flow_id);
            if (s == kNone) {
                status = ST_NO_RULE_EXISTS;  // the token stays cached
            } else {
                key = s;
                aux[i] = e;
            }
        }
    }
    el[i] = ((uint64_t)key << kSlotShift) | i;
    if (key == invalid_key) out[i] = ConcOut{0, status, 0};
}

__global__ void __launch_bounds__(kThreads) k_conc_runs(ConcState st, const uint64_t *el, uint32_t n,
                                                        uint32_t invalid_key, const uint8_t *op, const uint32_t *client,
                                                        const int64_t *id, const int32_t *acquire, const int64_t *ts,
                                                        const uint32_t *aux, uint64_t token_base, ConcOut *out) {
    const uint32_t p = blockIdx.x * kThreads + threadIdx.x;
    if (p >= n) return;
    const uint32_t key = (uint32_t)(el[p] >> kSlotShift);
    if (key == invalid_key) return;
    if (p > 0 && (uint32_t)(el[p - 1] >> kSlotShift) == key) return;  // not the first operation of its rule
    const uint32_t slot = key;
    const ConcParam prm = st.cparam[slot];
    int32_t now_calls = st.now_calls[slot];
    int32_t live = 0, tombs = 0;
    for (uint32_t q = p; q < n; ++q) {
        const uint64_t e = el[q];
        if ((uint32_t)(e >> kSlotShift) != key) break;
        const uint32_t i = (uint32_t)(e & ((1u << kIdxBits) - 1));
        if (op[i] == 0) {
            const int32_t a = acquire[i];
            // nowCalls.get() + acquireCount > calcGlobalThreshold(rule): int addition, then double
            const int32_t sum = (int32_t)((uint32_t)now_calls + (uint32_t)a);
            if ((double)sum > prm.thr) {
                out[i] = ConcOut{0, ST_BLOCKED, 0};
                continue;
            }
            now_calls = sum;  // getAndAdd(acquireCount)
            TokenEntry t{};
            t.token = (int64_t)splitmix64(token_base + i);
            t.flow_id = id[i];
            t.client_deadline = prm.client_offline + ts[i];
            t.resource_deadline = prm.resource_timeout + ts[i];
            t.acquire = a;
            t.client = client[i];
            tok_insert(st.tok, st.tmask, st.epoch, t);
            ++live;
            out[i] = ConcOut{t.token, ST_OK, 0};
        } else {
            const uint32_t ix = aux[i];
            if (atomicCAS(&st.tok[ix].state, kTokLive, tok_tomb(st.epoch)) == kTokLive) {
                now_calls = (int32_t)((uint32_t)now_calls - (uint32_t)st.tok[ix].acquire);
                --live;
                ++tombs;
                out[i] = ConcOut{0, ST_RELEASE_OK, 0};
            } else {
                out[i] = ConcOut{0, ST_ALREADY_RELEASE, 0};  // removed earlier in this batch
            }
        }
    }
    st.now_calls[slot] = now_calls;
    if (live) atomicAdd(&st.ctr[0], (uint32_t)live);
    if (tombs) atomicAdd(&st.ctr[1], (uint32_t)tombs);
}

// RegularExpireStrategy.clearToken (:78-121) for every live token.  A token whose rule is gone and
// whose client is online is kept (the reference's pass would stop at it on a null rule).
__global__ void __launch_bounds__(kThreads) k_conc_expire(ConcState st, int64_t now, const uint32_t *online_bits,
                                                          uint32_t nclients) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j > st.tmask) return;
    TokenEntry &t = st.tok[j];
    if (__atomic_load_n(&t.state, __ATOMIC_RELAXED) != kTokLive) return;
    const uint32_t slot = rule_slot(st.cs, t.flow_id);
    const uint32_t c = t.client;
    const bool online = c < nclients && ((online_bits[c >> 5] >> (c & 31)) & 1u);
    bool remove = false;
    if (!online && t.client_deadline - now < 0) remove = true;  // client offline for clientOfflineTime
    else if (slot != kNone && now - t.resource_deadline > st.cparam[slot].resource_timeout) remove = true;
    if (!remove) return;
    if (atomicCAS(&t.state, kTokLive, tok_tomb(st.epoch)) != kTokLive) return;
    if (slot != kNone) atomicSub(&st.now_calls[slot], t.acquire);  // nowCalls == null: no decrement
    atomicSub(&st.ctr[0], 1u);
    atomicAdd(&st.ctr[1], 1u);
    atomicAdd(&st.ctr[2], 1u);
}

__global__ void __launch_bounds__(kThreads) k_conc_rehash(const TokenEntry *old, uint32_t old_n, TokenEntry *nt,
                                                          uint32_t nmask) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= old_n || old[j].state != kTokLive) return;
    tok_insert(nt, nmask, 0, old[j]);
}

__global__ void k_conc_reset(int32_t *now_calls, const uint32_t *slots, uint32_t n) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j < n) now_calls[slots[j]] = 0;
}

__global__ void k_conc_find(ConcState st, int64_t token, TokenEntry *out) {
    if (threadIdx.x != 0) return;
    const uint32_t e = tok_find(st, token);
    if (e == kNone) {
        TokenEntry z{};
        *out = z;
    } else {
        *out = st.tok[e];
    }
}

size_t align_up(size_t b) { return (b + 255) & ~(size_t)255; }

size_t conc_hist_entries(size_t cap) {
    size_t m = 0;
    for (int b = 1; b <= 25; ++b) m = std::max(m, ((size_t)1 << radix64_digit_bits(b)) * radix64_tiles(cap));
    return m;
}

}  // namespace

size_t conc_scratch_bytes(size_t cap) {
    const size_t hist = conc_hist_entries(cap);
    return 2 * align_up(cap * 8) + align_up(cap * 4) + 2 * align_up(hist * 4) +
           align_up(scan_partials_needed(hist) * 4 + 64) + align_up(kRadixGhistWords * 4) + align_up(64);
}

void conc_scratch_carve(ConcScratch &sc, void *base, size_t cap) {
    const size_t hist = conc_hist_entries(cap);
    char *p = (char *)base;
    auto take = [&](size_t bytes) {
        void *r = p;
        p += align_up(bytes);
        return r;
    };
    sc.el[0] = (uint64_t *)take(cap * 8);
    sc.el[1] = (uint64_t *)take(cap * 8);
    sc.aux = (uint32_t *)take(cap * 4);
    sc.radix.hist = (uint32_t *)take(hist * 4);
    sc.radix.hist_scan = (uint32_t *)take(hist * 4);
    sc.radix.partial = (uint32_t *)take(scan_partials_needed(hist) * 4 + 64);
    sc.radix.ghist = (uint32_t *)take(kRadixGhistWords * 4);
    sc.radix.err = (uint32_t *)take(64);
    sc.cap = cap;
}

void conc_ops(const ConcState &st, ConcScratch &sc, const uint8_t *op, const uint32_t *client, const int64_t *id,
              const int32_t *acquire, const int64_t *ts, uint32_t n, uint64_t token_base, void *out_v, hipStream_t s) {
    if (n == 0) return;
    ConcOut *out = (ConcOut *)out_v;
    int bits = 1;
    while (((uint64_t)1 << bits) < (uint64_t)st.cs.nslots + 1) ++bits;
    const uint32_t invalid_key = st.cs.nslots;
    const uint32_t blocks = (n + kThreads - 1) / kThreads;
    hipLaunchKernelGGL(k_conc_classify, dim3(blocks), dim3(kThreads), 0, s, st, op, client, id, acquire, n,
                       invalid_key, sc.el[0], sc.aux, out);
    if (radix64_lookback()) SGA_HIP_CHECK(hipMemsetAsync(sc.radix.err, 0, sizeof(uint32_t), s));
    const int np = radix_sort_u64(sc.el[0], sc.el[1], n, kSlotShift, bits, sc.radix, s, false);
    const uint64_t *sorted = (np & 1) ? sc.el[1] : sc.el[0];
    hipLaunchKernelGGL(k_conc_runs, dim3(blocks), dim3(kThreads), 0, s, st, sorted, n, invalid_key, op, client, id,
                       acquire, ts, sc.aux, token_base, out);
}

void conc_expire(const ConcState &st, int64_t now, const uint32_t *online_bits, uint32_t nclients, hipStream_t s) {
    const uint32_t n = st.tmask + 1;
    SGA_HIP_CHECK(hipMemsetAsync(st.ctr + 2, 0, sizeof(uint32_t), s));
    hipLaunchKernelGGL(k_conc_expire, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, s, st, now, online_bits,
                       nclients);
}

void conc_rehash(const TokenEntry *old, uint32_t old_n, TokenEntry *nt, uint32_t nmask, hipStream_t s) {
    SGA_HIP_CHECK(hipMemsetAsync(nt, 0, ((size_t)nmask + 1) * sizeof(TokenEntry), s));
    if (old_n)
        hipLaunchKernelGGL(k_conc_rehash, dim3((old_n + kThreads - 1) / kThreads), dim3(kThreads), 0, s, old, old_n,
                           nt, nmask);
}

void conc_reset_calls(int32_t *now_calls, const uint32_t *slots, uint32_t n, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_conc_reset, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, s, now_calls, slots, n);
}

void conc_find(const ConcState &st, int64_t token, TokenEntry *d_out, hipStream_t s) {
    hipLaunchKernelGGL(k_conc_find, dim3(1), dim3(64), 0, s, st, token, d_out);
}

}  // namespace sga
