/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- CPU restatement of the cluster concurrency-token path
 * (the parity checker for sga_concurrent_ops / sga_concurrent_expire; never linked into the
 * product library).  CS = sentinel-cluster/sentinel-cluster-server-default/src/main/java/com/
 * alibaba/csp/sentinel/cluster:
 *
 *   DefaultTokenService.requestConcurrentToken / releaseConcurrentToken   CS/flow/DefaultTokenService.java:67-95
 *   ConcurrentClusterFlowChecker.calcGlobalThreshold / acquire / release  CS/flow/ConcurrentClusterFlowChecker.java:37-104
 *   TokenCacheNode.generateTokenCacheNode (timeouts = config + now)       CS/flow/statistic/concurrent/TokenCacheNode.java:40-75
 *   TokenCacheNodeManager (get / put / remove / size)                     CS/flow/statistic/concurrent/TokenCacheNodeManager.java:52-75
 *   RegularExpireStrategy.clearToken / removeToken                        CS/flow/statistic/concurrent/expire/RegularExpireStrategy.java:78-134
 *   CurrentConcurrencyManager (put when absent, remove with the rule)     CS/flow/statistic/concurrent/CurrentConcurrencyManager.java,
 *                                                                         CS/flow/rule/ClusterFlowRuleManager.java:277-297,356-358
 *
 * Token ids are inputs here: the reference draws UUID.randomUUID().getMostSignificantBits(), the
 * engine a splitmix64 counter, and the test hands the engine's ids to the oracle.
 * One deliberate difference from the reference's timer task, restated identically by the engine:
 * a pass examines every cached token (the reference stops after 1000 keys / 800 ms of wall time and
 * at the first token whose rule is gone, a NullPointerException caught by the task).  A token
 * whose rule is gone and whose client is online is kept.
 */
#include "oracle_internal.h"
#include "sentinel_oracle.h"

#include <stdlib.h>
#include <string.h>

enum { C_BAD_REQUEST = -4, C_OK = 0, C_BLOCKED = 1, C_NO_RULE_EXISTS = 3, C_RELEASE_OK = 6, C_ALREADY_RELEASE = 7 };

typedef struct otok {
    int64_t token, flow_id, client_deadline, resource_deadline;
    int32_t acquire;
    uint32_t client;
    int used; /* 0 empty, 1 live, 2 deleted */
} otok;

struct orc_conc {
    otok *tab;
    size_t cap, live, deleted;
};

struct orc_conc **orc_cluster_conc_slot(orc_cluster *c);
const orc_cluster_rule *orc_cluster_active_rule(orc_cluster *c, int64_t flow_id, int *ns, int32_t **now_calls);
int32_t orc_cluster_connected(orc_cluster *c, int ns);

static uint64_t tmix(uint64_t z) {
    z ^= 0xA5A5A5A55A5A5A5AULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static struct orc_conc *conc_of(orc_cluster *c) {
    struct orc_conc **pp = orc_cluster_conc_slot(c);
    if (!*pp) *pp = (struct orc_conc *)calloc(1, sizeof(struct orc_conc));
    return *pp;
}

void orc_conc_free_all(orc_cluster *c) {
    struct orc_conc **pp = orc_cluster_conc_slot(c);
    if (*pp) {
        free((*pp)->tab);
        free(*pp);
        *pp = NULL;
    }
}

static otok *tok_get(struct orc_conc *q, int64_t token) {
    if (!q->cap) return NULL;
    size_t h = tmix((uint64_t)token) & (q->cap - 1);
    while (q->tab[h].used) {
        if (q->tab[h].used == 1 && q->tab[h].token == token) return &q->tab[h];
        h = (h + 1) & (q->cap - 1);
    }
    return NULL;
}

static void tok_put(struct orc_conc *q, const otok *t) {
    if ((q->live + q->deleted + 1) * 2 > q->cap) {
        size_t ncap = 64;
        while (ncap < 4 * (q->live + 1)) ncap <<= 1;
        otok *nt = (otok *)calloc(ncap, sizeof(otok));
        for (size_t i = 0; i < q->cap; i++) {
            if (q->tab[i].used != 1) continue;
            size_t h = tmix((uint64_t)q->tab[i].token) & (ncap - 1);
            while (nt[h].used) h = (h + 1) & (ncap - 1);
            nt[h] = q->tab[i];
        }
        free(q->tab);
        q->tab = nt;
        q->cap = ncap;
        q->deleted = 0;
    }
    otok *old = tok_get(q, t->token); /* ConcurrentMap.put replaces an equal key */
    if (old) {
        *old = *t;
        old->used = 1;
        return;
    }
    size_t h = tmix((uint64_t)t->token) & (q->cap - 1);
    while (q->tab[h].used == 1) h = (h + 1) & (q->cap - 1);
    if (q->tab[h].used == 2) q->deleted--;
    q->tab[h] = *t;
    q->tab[h].used = 1;
    q->live++;
}

static void tok_del(struct orc_conc *q, otok *t) {
    t->used = 2;
    q->live--;
    q->deleted++;
}

/* ConcurrentClusterFlowChecker.calcGlobalThreshold, :37-46 */
static double calc_global_threshold(orc_cluster *c, const orc_cluster_rule *r, int ns) {
    if (r->threshold_type == 1) return r->count;
    return r->count * (double)orc_cluster_connected(c, ns);
}

/* DefaultTokenService.requestConcurrentToken -> ConcurrentClusterFlowChecker.acquireConcurrentToken.
 * client = ORC_CLIENT_NONE for a null or empty address. */
orc_conc_result orc_cluster_concurrent_acquire(orc_cluster *c, uint32_t client, int64_t flow_id, int32_t acquire,
                                               int64_t now, int64_t token_id) {
    orc_conc_result res = {C_OK, 0, 0};
    if (client == ORC_CLIENT_NONE || flow_id <= 0 || acquire <= 0) { /* notValidRequest, :92-94 */
        res.status = C_BAD_REQUEST;
        return res;
    }
    int ns = -1;
    int32_t *now_calls = NULL;
    const orc_cluster_rule *r = orc_cluster_active_rule(c, flow_id, &ns, &now_calls);
    if (!r) {
        res.status = C_NO_RULE_EXISTS;
        return res;
    }
    if (!now_calls) { /* CurrentConcurrencyManager.get == null: FAIL (unreachable while the rule exists) */
        res.status = -1;
        return res;
    }
    /* nowCalls.get() + acquireCount > calcGlobalThreshold(rule): int addition, widened to double */
    const int32_t sum = (int32_t)((uint32_t)*now_calls + (uint32_t)acquire);
    if ((double)sum > calc_global_threshold(c, r, ns)) {
        res.status = C_BLOCKED;
        return res;
    }
    *now_calls = sum;
    otok t;
    memset(&t, 0, sizeof(t));
    t.token = token_id;
    t.flow_id = flow_id;
    t.client_deadline = r->client_offline_time_ms + now; /* setClientTimeout(clientOfflineTime) */
    t.resource_deadline = r->resource_timeout_ms + now;  /* setResourceTimeout(resourceTimeout) */
    t.acquire = acquire;
    t.client = client;
    tok_put(conc_of(c), &t);
    res.token_id = token_id;
    return res;
}

/* ConcurrentClusterFlowChecker.releaseConcurrentToken, :81-104 */
int32_t orc_cluster_concurrent_release(orc_cluster *c, int64_t token_id) {
    struct orc_conc *q = conc_of(c);
    otok *t = tok_get(q, token_id);
    if (!t) return C_ALREADY_RELEASE;
    int32_t *now_calls = NULL;
    if (!orc_cluster_active_rule(c, t->flow_id, NULL, &now_calls)) return C_NO_RULE_EXISTS;
    const int32_t a = t->acquire;
    tok_del(q, t);
    if (now_calls) *now_calls = (int32_t)((uint32_t)*now_calls - (uint32_t)a);
    return C_RELEASE_OK;
}

/* RegularExpireStrategy.clearToken over every cached token; returns the tokens removed */
uint64_t orc_cluster_concurrent_expire(orc_cluster *c, int64_t now, const uint32_t *online_bits, uint32_t nclients) {
    struct orc_conc *q = conc_of(c);
    uint64_t removed = 0;
    for (size_t i = 0; i < q->cap; i++) {
        otok *t = &q->tab[i];
        if (t->used != 1) continue;
        const uint32_t cl = t->client;
        const int online = cl < nclients && ((online_bits[cl >> 5] >> (cl & 31)) & 1u);
        int32_t *now_calls = NULL;
        const orc_cluster_rule *r = orc_cluster_active_rule(c, t->flow_id, NULL, &now_calls);
        int remove = 0;
        if (!online && t->client_deadline - now < 0) remove = 1;
        else if (r && now - t->resource_deadline > r->resource_timeout_ms) remove = 1;
        if (!remove) continue;
        if (now_calls) *now_calls = (int32_t)((uint32_t)*now_calls - (uint32_t)t->acquire); /* removeToken */
        tok_del(q, t);
        removed++;
    }
    return removed;
}

int orc_cluster_concurrent_now_calls(orc_cluster *c, int64_t flow_id, int32_t *out) {
    int32_t *now_calls = NULL;
    orc_cluster_active_rule(c, flow_id, NULL, &now_calls);
    if (!now_calls) return 0;
    *out = *now_calls;
    return 1;
}

size_t orc_cluster_concurrent_tokens(orc_cluster *c) { return conc_of(c)->live; }

/* TokenCacheNodeManager.getTokenCacheNode: 1 and the node fields when cached */
int orc_cluster_concurrent_get(orc_cluster *c, int64_t token_id, int64_t *flow_id, int64_t *client_deadline,
                               int64_t *resource_deadline, int32_t *acquire) {
    otok *t = tok_get(conc_of(c), token_id);
    if (!t) return 0;
    *flow_id = t->flow_id;
    *client_deadline = t->client_deadline;
    *resource_deadline = t->resource_deadline;
    *acquire = t->acquire;
    return 1;
}
