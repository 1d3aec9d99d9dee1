/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- CPU restatement of the cluster parameter-flow token path
 * (the parity checker for sga_request_param_tokens; never linked into the product library).
 *
 *   DefaultTokenService.requestParamToken        CS/flow/DefaultTokenService.java:52-64,87-89
 *   ClusterParamFlowChecker.acquireClusterToken  CS/flow/ClusterParamFlowChecker.java:37-120
 *   ClusterParamMetric (getSum/getAvg/addValue)  CS/flow/statistic/metric/ClusterParamMetric.java:41-88
 *   ClusterParameterLeapArray (new bucket = empty map, reset = clear)
 *                                                CS/flow/statistic/metric/ClusterParameterLeapArray.java:33-49
 *   LeapArray.currentWindow / values             CORE/slots/statistic/base/LeapArray.java:121-222,265-296
 *   ClusterParamFlowRuleManager.applyClusterParamRules / clearAndResetRules*
 *                                                CS/flow/rule/ClusterParamFlowRuleManager.java:195-223,318-368
 *   ParamFlowRuleUtil.isValidRule / checkCluster PF/slots/block/flow/param/ParamFlowRuleUtil.java:46-70
 *
 * Each bucket's value map is the reference's per-bucket CacheMap: a ConcurrentLinkedHashMapWrapper of
 * capacity ClusterParamMetric.DEFAULT_CLUSTER_MAX_CAPACITY = 4000 (ClusterParamMetric.java:37,42,49;
 * ClusterParameterLeapArray.java:40-41, a new map per new bucket, cleared on reset :45-47), restated as a
 * strict LRU of that capacity (concurrentlinkedhashmap-lru 1.4.2 is not vendored; for one thread its
 * published policy is LRU: reads -- getSum's bucket.get(value) on every valid bucket, :57-62 -- and
 * putIfAbsent of a present key move the key to the most recent end, an insert into a full map evicts the
 * least recent one, :79-88).  getTopValues' keySet(true) + get(o) walk each map from its least recent key,
 * moving every key to the most recent end in that same order, so it leaves the order as it was
 * (:90-133).  orc_cluster_set_param_capacity changes the capacity of metrics created afterwards (tests);
 * parity against CLHM itself is unpinned (Oracle).
 */
#include "oracle_internal.h"
#include "java_semantics.h"
#include "sentinel_oracle.h"

#include <stdlib.h>
#include <string.h>

enum { P_BAD_REQUEST = -4, P_TOO_MANY_REQUEST = -2, P_FAIL = -1, P_OK = 0, P_BLOCKED = 1, P_NO_RULE_EXISTS = 3 };
static const int64_t P_ABSENT = INT64_MIN;

/* value -> LongAdder sum, open addressing (one per bucket); rec = the key's last access (LRU order) */
typedef struct vmap {
    int64_t *key, *val;
    uint64_t *rec;
    uint8_t *used;
    size_t cap, n;
} vmap;

static uint64_t vmix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static void vmap_grow(vmap *m) {
    size_t ncap = m->cap ? m->cap * 2 : 16;
    vmap nm = {calloc(ncap, 8), calloc(ncap, 8), calloc(ncap, 8), calloc(ncap, 1), ncap, 0};
    for (size_t i = 0; i < m->cap; i++) {
        if (!m->used[i]) continue;
        size_t h = vmix((uint64_t)m->key[i]) & (ncap - 1);
        while (nm.used[h]) h = (h + 1) & (ncap - 1);
        nm.used[h] = 1;
        nm.key[h] = m->key[i];
        nm.val[h] = m->val[i];
        nm.rec[h] = m->rec[i];
        nm.n++;
    }
    free(m->key);
    free(m->val);
    free(m->rec);
    free(m->used);
    *m = nm;
}

/* the key's table index, or -1 */
static long vmap_find(const vmap *m, int64_t k) {
    if (m->cap == 0) return -1;
    size_t h = vmix((uint64_t)k) & (m->cap - 1);
    while (m->used[h]) {
        if (m->key[h] == k) return (long)h;
        h = (h + 1) & (m->cap - 1);
    }
    return -1;
}

static int64_t *vmap_slot(vmap *m, int64_t k, int create) {
    long f = vmap_find(m, k);
    if (f >= 0) return &m->val[f];
    if (!create) return NULL;
    if (m->cap == 0 || (m->n + 1) * 2 > m->cap) vmap_grow(m);
    size_t h = vmix((uint64_t)k) & (m->cap - 1);
    while (m->used[h]) h = (h + 1) & (m->cap - 1);
    m->used[h] = 1;
    m->key[h] = k;
    m->val[h] = 0;
    m->rec[h] = 0;
    m->n++;
    return &m->val[h];
}

/* linear-probing removal (backward shift: later keys of the probe run move up) */
static void vmap_erase(vmap *m, size_t i) {
    m->used[i] = 0;
    m->n--;
    size_t j = i;
    for (;;) {
        j = (j + 1) & (m->cap - 1);
        if (!m->used[j]) return;
        size_t h = vmix((uint64_t)m->key[j]) & (m->cap - 1);
        /* move j to the hole i when its home h is not within (i, j] cyclically */
        if ((j > i && (h <= i || h > j)) || (j < i && (h <= i && h > j))) {
            m->used[i] = 1;
            m->key[i] = m->key[j];
            m->val[i] = m->val[j];
            m->rec[i] = m->rec[j];
            m->used[j] = 0;
            i = j;
        }
    }
}

static void vmap_clear(vmap *m) {
    if (m->cap) memset(m->used, 0, m->cap);
    m->n = 0;
}

static void vmap_free(vmap *m) {
    free(m->key);
    free(m->val);
    free(m->rec);
    free(m->used);
    memset(m, 0, sizeof(*m));
}

/* ClusterParamMetric over ClusterParameterLeapArray(sampleCount, intervalInMs) */
typedef struct pmetric {
    int S, interval, W;
    double interval_sec;
    int64_t *start; /* P_ABSENT = array slot null */
    vmap *map;
    size_t capacity; /* each bucket map's maxCapacity */
    uint64_t clock;  /* access order (LRU) */
} pmetric;

static size_t g_param_capacity = 4000; /* ClusterParamMetric.DEFAULT_CLUSTER_MAX_CAPACITY */
void orc_cluster_set_param_capacity(size_t cap) { g_param_capacity = cap ? cap : 4000; }

static pmetric *pm_new(int S, int interval) {
    pmetric *m = calloc(1, sizeof(pmetric));
    m->capacity = g_param_capacity;
    m->S = S;
    m->interval = interval;
    m->W = interval / S;
    m->interval_sec = interval / 1000.0;
    m->start = malloc(sizeof(int64_t) * S);
    m->map = calloc(S, sizeof(vmap));
    for (int j = 0; j < S; j++) m->start[j] = P_ABSENT;
    return m;
}

static void pm_free(pmetric *m) {
    if (!m) return;
    for (int j = 0; j < m->S; j++) vmap_free(&m->map[j]);
    free(m->map);
    free(m->start);
    free(m);
}

/* LeapArray.currentWindow(t): bucket index, or -1 for the detached bucket handed out when the
 * clock went backwards (LeapArray.java:216-220; its adds are lost). */
static int pm_current_window(pmetric *m, int64_t t) {
    int idx = (int)((t / m->W) % m->S);
    int64_t ws = t - t % m->W;
    if (m->start[idx] == P_ABSENT) {        /* newEmptyBucket: empty map */
        m->start[idx] = ws;
        vmap_clear(&m->map[idx]);
        return idx;
    }
    if (ws == m->start[idx]) return idx;
    if (ws > m->start[idx]) {               /* resetWindowTo: map cleared */
        m->start[idx] = ws;
        vmap_clear(&m->map[idx]);
        return idx;
    }
    return -1;
}

/* ClusterParamMetric.getSum(value): currentWindow() then sum over values(); every bucket.get(value) that
 * finds the value is an access (LRU order) */
static int64_t pm_sum(pmetric *m, int64_t value, int64_t t) {
    pm_current_window(m, t);
    int64_t s = 0;
    for (int j = 0; j < m->S; j++) {
        if (m->start[j] == P_ABSENT || t - m->start[j] > m->interval) continue;  /* isWindowDeprecated */
        const long f = vmap_find(&m->map[j], value);
        if (f >= 0) {
            s += m->map[j].val[f];
            m->map[j].rec[f] = ++m->clock;
        }
    }
    return s;
}

/* addValue: putIfAbsent into the current bucket's map (a present key is an access; a new key into a full
 * map evicts the least recently accessed one, ClusterParamMetric.java:79-88) */
static void pm_add(pmetric *m, int64_t value, int count, int64_t t) {
    int idx = pm_current_window(m, t);
    if (idx < 0) return;
    vmap *b = &m->map[idx];
    long f = vmap_find(b, value);
    if (f < 0) {
        if (b->n >= m->capacity) { /* evict the least recent key */
            size_t lru = 0;
            uint64_t best = UINT64_MAX;
            for (size_t i = 0; i < b->cap; i++)
                if (b->used[i] && b->rec[i] < best) {
                    best = b->rec[i];
                    lru = i;
                }
            vmap_erase(b, lru);
        }
        vmap_slot(b, value, 1);
        f = vmap_find(b, value);
    }
    b->val[f] += count;
    b->rec[f] = ++m->clock;
}

typedef struct prule {
    int64_t flow_id;
    orc_cparam_rule r;
    int64_t *hot_v;
    int32_t *hot_c;
    int ns;
    int active;
    pmetric *metric; /* ClusterParamMetricStatistics entry (may outlive the rule) */
} prule;

struct orc_cparam {
    prule *tab;
    size_t cap, used;
};

int orc_cluster_ns_index(orc_cluster *c, const char *ns, int create);
/* accessors of orc_cluster internals (sentinel_oracle.c) */
struct orc_cparam **orc_cluster_param_slot(orc_cluster *c);
int32_t orc_cluster_connected(orc_cluster *c, int ns);
int orc_cluster_limiter_try_pass(orc_cluster *c, int ns, int64_t now);

static prule *ptab_find(struct orc_cparam *p, int64_t id, int create) {
    if (p->cap == 0 || (create && (p->used + 1) * 2 > p->cap)) {
        size_t ncap = p->cap ? p->cap * 2 : 256;
        prule *nt = calloc(ncap, sizeof(prule));
        for (size_t i = 0; i < p->cap; i++) {
            if (p->tab[i].flow_id == 0) continue;
            size_t h = vmix((uint64_t)p->tab[i].flow_id) & (ncap - 1);
            while (nt[h].flow_id != 0) h = (h + 1) & (ncap - 1);
            nt[h] = p->tab[i];
        }
        free(p->tab);
        p->tab = nt;
        p->cap = ncap;
    }
    size_t h = vmix((uint64_t)id) & (p->cap - 1);
    while (p->tab[h].flow_id != 0) {
        if (p->tab[h].flow_id == id) return &p->tab[h];
        h = (h + 1) & (p->cap - 1);
    }
    if (!create) return NULL;
    memset(&p->tab[h], 0, sizeof(prule));
    p->tab[h].flow_id = id;
    p->tab[h].ns = -1;
    p->used++;
    return &p->tab[h];
}

static struct orc_cparam *param_of(orc_cluster *c) {
    struct orc_cparam **pp = orc_cluster_param_slot(c);
    if (!*pp) *pp = calloc(1, sizeof(struct orc_cparam));
    return *pp;
}

void orc_cparam_free_all(orc_cluster *c) {
    struct orc_cparam **pp = orc_cluster_param_slot(c);
    struct orc_cparam *p = *pp;
    if (!p) return;
    for (size_t i = 0; i < p->cap; i++) {
        pm_free(p->tab[i].metric);
        free(p->tab[i].hot_v);
        free(p->tab[i].hot_c);
    }
    free(p->tab);
    free(p);
    *pp = NULL;
}

/* ParamFlowRuleUtil.isValidRule (PF/.../ParamFlowRuleUtil.java:46-70) for a cluster-mode rule */
static int cparam_valid(const orc_cparam_rule *r) {
    if (!(r->count >= 0 && r->grade >= 0 && r->param_idx_set && r->burst_count >= 0 && r->control_behavior >= 0 &&
          r->duration_in_sec > 0 && r->max_queueing_time_ms >= 0))
        return 0;
    if (!(r->sample_count > 0 && r->window_interval_ms > 0 && r->window_interval_ms % r->sample_count == 0)) return 0;
    return r->flow_id > 0; /* validClusterRuleId */
}

/* ClusterParamFlowRuleManager.applyClusterParamRules, ClusterParamFlowRuleManager.java:318-368 */
int orc_cluster_load_param_rules(orc_cluster *c, const char *ns, const orc_cparam_rule *rules, size_t n) {
    struct orc_cparam *p = param_of(c);
    int nsi = orc_cluster_ns_index(c, ns, 1);
    if (nsi < 0) return -1;
    if (n == 0) { /* clearAndResetRulesFor (:195-207): rules and namespace mapping dropped, metrics kept */
        for (size_t i = 0; i < p->cap; i++)
            if (p->tab[i].flow_id != 0 && p->tab[i].ns == nsi && p->tab[i].active) p->tab[i].active = 0;
        return 0;
    }
    for (size_t i = 0; i < p->cap; i++)
        if (p->tab[i].flow_id != 0 && p->tab[i].ns == nsi && p->tab[i].active) p->tab[i].active = 2;
    int applied = 0;
    for (size_t j = 0; j < n; j++) {
        const orc_cparam_rule *r = &rules[j];
        if (!cparam_valid(r)) continue;
        prule *e = ptab_find(p, r->flow_id, 1);
        e->r = *r;
        free(e->hot_v);
        free(e->hot_c);
        e->hot_v = NULL;
        e->hot_c = NULL;
        if (r->n_hot > 0) { /* parsed hotItems: HashMap put, later items win */
            e->hot_v = malloc(sizeof(int64_t) * r->n_hot);
            e->hot_c = malloc(sizeof(int32_t) * r->n_hot);
            memcpy(e->hot_v, r->hot_values, sizeof(int64_t) * r->n_hot);
            memcpy(e->hot_c, r->hot_counts, sizeof(int32_t) * r->n_hot);
        }
        e->r.hot_values = NULL;
        e->r.hot_counts = NULL;
        e->ns = nsi;
        e->active = 1;
        if (!e->metric) e->metric = pm_new(r->sample_count, r->window_interval_ms); /* putMetricIfAbsent */
        applied++;
    }
    /* clearAndResetRulesConditional: ids of this namespace not in the new map lose rule AND metric */
    for (size_t i = 0; i < p->cap; i++) {
        if (p->tab[i].flow_id != 0 && p->tab[i].ns == nsi && p->tab[i].active == 2) {
            p->tab[i].active = 0;
            pm_free(p->tab[i].metric);
            p->tab[i].metric = NULL;
        }
    }
    return applied;
}

/* ParamFlowRule.retrieveExclusiveItemCount + ClusterParamFlowChecker.calcGlobalThreshold (:101-120) */
static double cparam_threshold(orc_cluster *c, const prule *e, int64_t value) {
    double count = e->r.count;
    for (int i = e->r.n_hot - 1; i >= 0; i--) {
        if (e->hot_v[i] == value) {
            count = (double)e->hot_c[i];
            break;
        }
    }
    if (e->r.threshold_type == 1) return count;  /* FLOW_THRESHOLD_GLOBAL */
    return count * (double)orc_cluster_connected(c, e->ns);
}

static orc_token_result ptr_(int32_t s, int32_t rem) {
    orc_token_result t;
    t.status = s;
    t.remaining = rem;
    t.wait_in_ms = 0;
    return t;
}

orc_token_result orc_cluster_request_param_token(orc_cluster *c, int64_t flow_id, int32_t acquire,
                                                 const int64_t *values, size_t nvalues, int64_t now) {
    /* DefaultTokenService.requestParamToken: notValidRequest || params empty -> BAD_REQUEST (:54-56) */
    if (flow_id <= 0 || acquire <= 0 || nvalues == 0) return ptr_(P_BAD_REQUEST, 0);
    struct orc_cparam *p = param_of(c);
    prule *e = ptab_find(p, flow_id, 0);
    if (!e || e->active != 1) return ptr_(P_NO_RULE_EXISTS, 0);
    /* allowProceed -> GlobalRequestLimiter.tryPass(namespace), ClusterParamFlowChecker.java:37-47 */
    if (!orc_cluster_limiter_try_pass(c, e->ns, now)) return ptr_(P_TOO_MANY_REQUEST, 0);
    pmetric *m = e->metric;
    if (!m) return ptr_(P_FAIL, 0);
    double remaining = -1;
    int passed = 1;
    for (size_t i = 0; i < nvalues; i++) { /* :61-71 */
        double latest_qps = (double)pm_sum(m, values[i], now) / m->interval_sec;
        double threshold = cparam_threshold(c, e, values[i]);
        double next_remaining = threshold - latest_qps - (double)acquire;
        remaining = next_remaining;
        if (next_remaining < 0) {
            passed = 0;
            break;
        }
    }
    if (passed)
        for (size_t i = 0; i < nvalues; i++) pm_add(m, values[i], acquire, now);  /* :73-76 */
    if (nvalues > 1) remaining = -1;                                             /* :81-84 */
    return passed ? ptr_(P_OK, j_d2i(remaining)) : ptr_(P_BLOCKED, 0);
}

void orc_cluster_param_replay(orc_cluster *c, size_t n, const int64_t *flow_id, const int32_t *acquire,
                              const uint32_t *value_offsets, const int64_t *values, const int64_t *ts,
                              orc_token_result *out) {
    for (size_t i = 0; i < n; i++)
        out[i] = orc_cluster_request_param_token(c, flow_id[i], acquire[i], values + value_offsets[i],
                                                 value_offsets[i + 1] - value_offsets[i], ts[i]);
}

int64_t orc_cluster_param_sum(orc_cluster *c, int64_t flow_id, int64_t value, int64_t now) {
    prule *e = ptab_find(param_of(c), flow_id, 0);
    if (!e || !e->metric) return -1;
    return pm_sum(e->metric, value, now);
}

/* ClusterParamMetric.getTopValues(number), ClusterParamMetric.java:90-133: currentWindow(), merge
 * every valid bucket's map, largest sums first.  Equal sums: smaller value key first (the
 * reference sorts its HashMap's entries stably, so its order among equal sums is the HashMap's
 * iteration order of the Java objects -- not restated: parity unpinned for ties).  Returns the
 * number of values written (0 when the flow has no metric). */
static int top_before(int64_t c1, int64_t v1, int64_t c2, int64_t v2) { return c1 > c2 || (c1 == c2 && v1 < v2); }

size_t orc_cluster_param_top_values(orc_cluster *c, int64_t flow_id, int64_t now, size_t number, int64_t *vals,
                                    double *qps) {
    prule *e = ptab_find(param_of(c), flow_id, 0);
    if (!e || !e->metric || number == 0) return 0;
    pmetric *m = e->metric;
    pm_current_window(m, now);
    vmap acc = {0};
    for (int j = 0; j < m->S; j++) {
        if (m->start[j] == P_ABSENT || now - m->start[j] > m->interval) continue; /* values(): valid buckets */
        const vmap *b = &m->map[j];
        for (size_t i = 0; i < b->cap; i++)
            if (b->used[i]) *vmap_slot(&acc, b->key[i], 1) += b->val[i];
    }
    size_t got = 0;
    int64_t lc = INT64_MAX, lv = INT64_MIN;
    while (got < number) {
        int64_t bc = -1, bv = 0;
        for (size_t i = 0; i < acc.cap; i++) {
            if (!acc.used[i]) continue;
            const int64_t cc = acc.val[i], v = acc.key[i];
            if (top_before(lc, lv, cc, v) && top_before(cc, v, bc, bv)) {
                bc = cc;
                bv = v;
            }
        }
        if (bc <= 0) break; /* x.getValue() == 0: stop */
        vals[got] = bv;
        qps[got] = (double)bc / m->interval_sec;
        lc = bc;
        lv = bv;
        got++;
    }
    vmap_free(&acc);
    return got;
}

/* standalone ClusterParamMetric for the transcribed ClusterParamMetricTest (values are the caller's
 * 64-bit stand-ins for the Java Objects) */
typedef struct orc_pmetric orc_pmetric;
orc_pmetric *orc_pmetric_new(int sample_count, int interval_ms) {
    return (orc_pmetric *)pm_new(sample_count, interval_ms);
}
void orc_pmetric_free(orc_pmetric *m) { pm_free((pmetric *)m); }
void orc_pmetric_add(orc_pmetric *m, int64_t now, int64_t value, int32_t count) { pm_add((pmetric *)m, value, count, now); }
int64_t orc_pmetric_sum(orc_pmetric *m, int64_t now, int64_t value) { return pm_sum((pmetric *)m, value, now); }
double orc_pmetric_avg(orc_pmetric *m, int64_t now, int64_t value) {
    return (double)pm_sum((pmetric *)m, value, now) / ((pmetric *)m)->interval_sec;
}
