// Cluster concurrency tokens: ConcurrentClusterFlowChecker + TokenCacheNodeManager +
// CurrentConcurrencyManager + RegularExpireStrategy on the device
// (CS = sentinel-cluster/sentinel-cluster-server-default/src/main/java/com/alibaba/csp/sentinel/cluster):
//   CS/flow/ConcurrentClusterFlowChecker.java:37-104
//   CS/flow/statistic/concurrent/TokenCacheNode.java, TokenCacheNodeManager.java,
//   CurrentConcurrencyManager.java, expire/RegularExpireStrategy.java:64-134
//
// State in HBM: per rule slot the nowCalls counter and (threshold, resourceTimeout,
// clientOfflineTime); one open-addressing token table (48 B entries) keyed by tokenId.
// A batch of acquire / release operations in arrival order is grouped by rule slot with the u64
// radix sort; one lane walks each rule's operations in order (the reference's
// synchronized (nowCalls) section), so every decision equals the sequential one.
#pragma once
#include "cluster.hpp"

namespace sga {

struct ConcParam {
    double thr;                // ConcurrentClusterFlowChecker.calcGlobalThreshold(rule), :37-46
    int64_t resource_timeout;  // ClusterFlowConfig.resourceTimeout
    int64_t client_offline;    // ClusterFlowConfig.clientOfflineTime
};

// TokenCacheNode (TokenCacheNode.java:25-60): deadlines are the absolute times the setters store.
struct alignas(16) TokenEntry {
    int64_t token;
    int64_t flow_id;
    int64_t client_deadline;    // clientOfflineTime + creation time
    int64_t resource_deadline;  // resourceTimeout + creation time
    int32_t acquire;
    uint32_t client;            // client address id (host table)
    uint32_t state;             // kTokEmpty, kTokLive, kTokBusy or a tombstone (epoch << 2 | 2)
    uint32_t pad;
};
constexpr uint32_t kTokEmpty = 0, kTokLive = 1, kTokBusy = 3;
SGA_HD uint32_t tok_tomb(uint32_t epoch) { return (epoch << 2) | 2u; }

struct ConcState {
    ClusterState cs;          // flowId -> rule slot lookup (active rules)
    const ConcParam *cparam;  // per slot
    int32_t *now_calls;       // per slot: CurrentConcurrencyManager NOW_CALLS_MAP value
    TokenEntry *tok;
    uint32_t tmask;
    uint32_t epoch;           // tombstones of this epoch are not reused inside the batch
    uint32_t *ctr;            // [0] live tokens, [1] tombstones, [2] removed by the last expire pass
};

struct ConcScratch {
    uint64_t *el[2] = {nullptr, nullptr};
    uint32_t *aux = nullptr;  // release: token table index found by classify
    RadixScratch radix;
    size_t cap = 0;
};

size_t conc_scratch_bytes(size_t cap);
void conc_scratch_carve(ConcScratch &sc, void *base, size_t cap);

// One batch of operations (op 0 = acquire: id = flowId; op 1 = release: id = tokenId) in arrival
// order; out = sga_concurrent_result per operation.  Tokens are splitmix64(token_base + i).
void conc_ops(const ConcState &st, ConcScratch &sc, const uint8_t *op, const uint32_t *client, const int64_t *id,
              const int32_t *acquire, const int64_t *ts, uint32_t n, uint64_t token_base, void *out, hipStream_t s);
// RegularExpireStrategy.clearToken over every live token at `now`; online_bits[c >> 5] bit c & 31 =
// ConnectionManager.isClientOnline(client c).
void conc_expire(const ConcState &st, int64_t now, const uint32_t *online_bits, uint32_t nclients, hipStream_t s);
// Moves the live tokens of `old` into the empty table `nt` (nmask + 1 entries).
void conc_rehash(const TokenEntry *old, uint32_t old_n, TokenEntry *nt, uint32_t nmask, hipStream_t s);
// CurrentConcurrencyManager.put(flowId, 0) for the listed slots.
void conc_reset_calls(int32_t *now_calls, const uint32_t *slots, uint32_t n, hipStream_t s);
// TokenCacheNodeManager.getTokenCacheNode: the live entry of `token` (state 0 when absent).
void conc_find(const ConcState &st, int64_t token, TokenEntry *d_out, hipStream_t s);

}  // namespace sga
