/*
 * ORACLE / TEST INFRASTRUCTURE ONLY (see sentinel_oracle.h, oracle_ext.h).
 * ParamFlowChecker / ParameterMetric and DegradeSlot circuit breakers, and the
 * full local slot chain entry/exit of the engine's local path.
 *   PF = sentinel-extension/sentinel-parameter-flow-control/src/main/java/com/alibaba/csp/sentinel
 *   CB = CORE/slots/block/degrade/circuitbreaker
 */
#include "oracle_internal.h"
#include "java_semantics.h"

#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- u64 -> i64 map */
struct orc_pmap {
    uint64_t *k;
    int64_t *v;
    uint8_t *used;
    size_t cap, n;
};

static uint64_t pm_hash(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static orc_pmap *pm_new(void) {
    orc_pmap *m = (orc_pmap *)calloc(1, sizeof(orc_pmap));
    m->cap = 64;
    m->k = (uint64_t *)calloc(m->cap, 8);
    m->v = (int64_t *)calloc(m->cap, 8);
    m->used = (uint8_t *)calloc(m->cap, 1);
    return m;
}

static void pm_free(orc_pmap *m) {
    if (!m) return;
    free(m->k);
    free(m->v);
    free(m->used);
    free(m);
}

static int64_t *pm_find(orc_pmap *m, uint64_t key) {
    size_t h = pm_hash(key) & (m->cap - 1);
    while (m->used[h]) {
        if (m->k[h] == key) return &m->v[h];
        h = (h + 1) & (m->cap - 1);
    }
    return NULL;
}

static void pm_put(orc_pmap *m, uint64_t key, int64_t val) {
    int64_t *p = pm_find(m, key);
    if (p) {
        *p = val;
        return;
    }
    if ((m->n + 1) * 2 > m->cap) {
        orc_pmap big = {0};
        big.cap = m->cap * 2;
        big.k = (uint64_t *)calloc(big.cap, 8);
        big.v = (int64_t *)calloc(big.cap, 8);
        big.used = (uint8_t *)calloc(big.cap, 1);
        for (size_t i = 0; i < m->cap; i++)
            if (m->used[i]) pm_put(&big, m->k[i], m->v[i]);
        free(m->k);
        free(m->v);
        free(m->used);
        m->k = big.k;
        m->v = big.v;
        m->used = big.used;
        m->cap = big.cap;
        m->n = big.n;
    }
    size_t h = pm_hash(key) & (m->cap - 1);
    while (m->used[h]) h = (h + 1) & (m->cap - 1);
    m->used[h] = 1;
    m->k[h] = key;
    m->v[h] = val;
    m->n++;
}

static void pm_remove(orc_pmap *m, uint64_t key) {
    size_t h = pm_hash(key) & (m->cap - 1);
    while (m->used[h]) {
        if (m->k[h] == key) break;
        h = (h + 1) & (m->cap - 1);
    }
    if (!m->used[h]) return;
    m->used[h] = 0;
    m->n--;
    /* re-insert the rest of the cluster (linear probing deletion) */
    size_t j = (h + 1) & (m->cap - 1);
    while (m->used[j]) {
        uint64_t k = m->k[j];
        int64_t v = m->v[j];
        m->used[j] = 0;
        m->n--;
        pm_put(m, k, v);
        j = (j + 1) & (m->cap - 1);
    }
}

/* ---------------------------------------------------------------- capacity-bounded LRU map
 * CacheMap / ConcurrentLinkedHashMapWrapper (PF/slots/statistic/cache/ConcurrentLinkedHashMapWrapper.java:
 * 35-44) over com.googlecode.concurrentlinkedhashmap:concurrentlinkedhashmap-lru:1.4.2, which is not
 * vendored in the reference.  Restated from CLHM's published algorithm for ONE thread: an
 * access-ordered deque; get / putIfAbsent on a present key record a read (the key moves to the MRU
 * end), put / an insert record a write (MRU end), and after an insert that takes the size above the
 * capacity the LRU end is evicted (singleton weigher: every entry weighs 1).  CLHM buffers reads and
 * drains them before a write is applied, so single-threaded its order is exactly this strict LRU.
 * Parity vs CLHM itself: unpinned (no reference test evicts); exact vs this restatement. */
typedef struct {
    uint64_t key;
    int64_t val;
    int32_t prev, next; /* towards LRU / towards MRU; -1 at the ends */
} lru_node;

struct orc_lru {
    orc_pmap *idx; /* key -> node index */
    lru_node *nodes;
    int32_t *free_list;
    int32_t nfree, head, tail; /* head = least recently used */
    size_t cap, n, alloc, hw;
    uint64_t evictions;
};

static orc_lru *lru_new(size_t cap) {
    orc_lru *m = (orc_lru *)calloc(1, sizeof(orc_lru));
    m->idx = pm_new();
    m->cap = cap;
    m->head = m->tail = -1;
    return m;
}

static void lru_free(orc_lru *m) {
    if (!m) return;
    pm_free(m->idx);
    free(m->nodes);
    free(m->free_list);
    free(m);
}

static void lru_unlink(orc_lru *m, int32_t i) {
    lru_node *x = &m->nodes[i];
    if (x->prev >= 0) m->nodes[x->prev].next = x->next;
    else m->head = x->next;
    if (x->next >= 0) m->nodes[x->next].prev = x->prev;
    else m->tail = x->prev;
    x->prev = x->next = -1;
}

static void lru_append(orc_lru *m, int32_t i) { /* at the MRU end */
    lru_node *x = &m->nodes[i];
    x->prev = m->tail;
    x->next = -1;
    if (m->tail >= 0) m->nodes[m->tail].next = i;
    else m->head = i;
    m->tail = i;
}

static void lru_touch(orc_lru *m, int32_t i) {
    if (m->tail == i) return;
    lru_unlink(m, i);
    lru_append(m, i);
}

static void lru_drop(orc_lru *m, int32_t i) {
    lru_unlink(m, i);
    pm_remove(m->idx, m->nodes[i].key);
    m->free_list[m->nfree++] = i;
    m->n--;
}

/* the node of `key` without recording an access, or NULL */
static int64_t *lru_peek(orc_lru *m, uint64_t key) {
    int64_t *p = pm_find(m->idx, key);
    return p ? &m->nodes[*p].val : NULL;
}

/* CacheMap.get: a read of a present key */
static int64_t *lru_get(orc_lru *m, uint64_t key) {
    int64_t *p = pm_find(m->idx, key);
    if (!p) return NULL;
    const int32_t i = (int32_t)*p;
    lru_touch(m, i);
    return &m->nodes[i].val;
}

static int32_t lru_insert(orc_lru *m, uint64_t key, int64_t val) {
    int32_t i;
    if (m->nfree) {
        i = m->free_list[--m->nfree];
    } else {
        if (m->hw == m->alloc) {
            const size_t na = m->alloc ? m->alloc * 2 : 64;
            m->nodes = (lru_node *)realloc(m->nodes, na * sizeof(lru_node));
            m->free_list = (int32_t *)realloc(m->free_list, na * sizeof(int32_t));
            m->alloc = na;
        }
        i = (int32_t)m->hw++;
    }
    m->nodes[i].key = key;
    m->nodes[i].val = val;
    pm_put(m->idx, key, i);
    m->n++;
    lru_append(m, i);
    while (m->n > m->cap && m->head >= 0) { /* evict from the LRU end */
        m->evictions++;
        lru_drop(m, m->head);
    }
    return i;
}

/* CacheMap.putIfAbsent: NULL after inserting `val` (the key was absent), else the present value
 * (a read: the key moves to the MRU end, the value is kept) */
static int64_t *lru_put_if_absent(orc_lru *m, uint64_t key, int64_t val) {
    int64_t *p = pm_find(m->idx, key);
    if (p) {
        const int32_t i = (int32_t)*p;
        lru_touch(m, i);
        return &m->nodes[i].val;
    }
    lru_insert(m, key, val);
    return NULL;
}

/* CacheMap.put: insert or replace (a write: MRU end) */
static void lru_put(orc_lru *m, uint64_t key, int64_t val) {
    int64_t *p = pm_find(m->idx, key);
    if (p) {
        const int32_t i = (int32_t)*p;
        m->nodes[i].val = val;
        lru_touch(m, i);
        return;
    }
    lru_insert(m, key, val);
}

/* CacheMap.remove */
static void lru_remove(orc_lru *m, uint64_t key) {
    int64_t *p = pm_find(m->idx, key);
    if (p) lru_drop(m, (int32_t)*p);
}

size_t orc_lru_size(const orc_lru *m) { return m ? m->n : 0; }
uint64_t orc_lru_evictions(const orc_lru *m) { return m ? m->evictions : 0; }
/* the keys from least to most recently used (test introspection) */
size_t orc_lru_keys(const orc_lru *m, uint64_t *out, int64_t *vals, size_t cap) {
    size_t k = 0;
    for (int32_t i = m ? m->head : -1; i >= 0 && k < cap; i = m->nodes[i].next, k++) {
        out[k] = m->nodes[i].key;
        if (vals) vals[k] = m->nodes[i].val;
    }
    return k;
}

/* ---------------------------------------------------------------- param rules */
/* ParameterMetric capacities, PF/slots/block/flow/param/ParameterMetric.java:37-39 */
#define PM_THREAD_COUNT_MAX_CAPACITY 4000
#define PM_BASE_PARAM_MAX_CAPACITY 4000
#define PM_TOTAL_MAX_CAPACITY 200000

struct orc_prule {
    orc_param_rule r;
    int32_t idx;      /* paramIdx after ParamFlowSlot.applyRealParamIdx (ParamFlowSlot.java:56-66) */
    int resolved;     /* the rule was checked once: idx is final (the reference mutates the rule) */
    uint64_t *hot_v;
    int32_t *hot_t;
    orc_lru *time;   /* ParameterMetric.ruleTimeCounters[rule], capacity min(4000 * duration, 200000) */
    orc_lru *token;  /* ParameterMetric.ruleTokenCounter[rule], same capacity (ParameterMetric.java:95-112) */
};

static size_t param_capacity(const orc_param_rule *r) { /* Math.min(BASE * durationInSec, TOTAL) */
    const int64_t c = (int64_t)PM_BASE_PARAM_MAX_CAPACITY * (int64_t)r->duration_in_sec;
    return (size_t)(c < PM_TOTAL_MAX_CAPACITY ? c : PM_TOTAL_MAX_CAPACITY);
}

orc_prule *orc_prule_new(const orc_param_rule *r) {
    orc_prule *p = (orc_prule *)calloc(1, sizeof(orc_prule));
    p->r = *r;
    if (r->n_hot) {
        p->hot_v = (uint64_t *)malloc(8 * r->n_hot);
        p->hot_t = (int32_t *)malloc(4 * r->n_hot);
        memcpy(p->hot_v, r->hot_values, 8 * r->n_hot);
        memcpy(p->hot_t, r->hot_thresholds, 4 * r->n_hot);
    }
    p->r.hot_values = p->hot_v;
    p->r.hot_thresholds = p->hot_t;
    p->time = lru_new(param_capacity(r));
    p->token = lru_new(param_capacity(r));
    return p;
}

void orc_prule_free(orc_prule *p) {
    if (!p) return;
    free(p->hot_v);
    free(p->hot_t);
    lru_free(p->time);
    lru_free(p->token);
    free(p);
}

static int hot_lookup(const orc_prule *p, uint64_t value, int64_t *thr) {
    for (uint32_t i = 0; i < p->r.n_hot; i++)
        if (p->hot_v[i] == value) {
            *thr = p->hot_t[i];
            return 1;
        }
    return 0;
}

static int64_t lwrap_mul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
static int64_t lwrap_add(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }

/* ParamFlowChecker.passDefaultLocalCheck, PF/slots/block/flow/param/ParamFlowChecker.java:132-222.
 * Every map call below is an access of the LRU maps (CacheMap.putIfAbsent / get).  The time and the
 * token map have the same capacity and see the same key sequence (each check that reaches the maps
 * accesses the time map, then the token map, with the same value), so single-threaded they always
 * hold the same keys: the reference's spin (:205-219, time kept and token evicted: Thread.yield until
 * passTime > duration) cannot arise here.  Should it, it is resolved as the spin ends in the
 * reference: the refill branch at the current time (token = maxCount - acquireCount, time = now). */
static int pass_default(orc_prule *p, uint64_t value, int acquire, int64_t now) {
    int64_t token_count = j_d2l(p->r.count);
    int64_t hot;
    if (hot_lookup(p, value, &hot)) token_count = hot;
    if (token_count == 0) return 0;
    const int64_t max_count = lwrap_add(token_count, p->r.burst_count);
    if ((int64_t)acquire > max_count) return 0;
    int64_t *last = lru_put_if_absent(p->time, value, now);
    if (!last) { /* token never added */
        lru_put_if_absent(p->token, value, max_count - acquire);
        return 1;
    }
    const int64_t pass_time = now - *last;
    const int64_t dur_ms = lwrap_mul(p->r.duration_in_sec, 1000);
    if (pass_time > dur_ms) {
        int64_t *old = lru_put_if_absent(p->token, value, max_count - acquire);
        if (!old) {
            *lru_peek(p->time, value) = now; /* lastAddTokenTime.set(currentTime) */
            return 1;
        }
        const int64_t rest = *old;
        const int64_t to_add = lwrap_mul(pass_time, token_count) / dur_ms;
        const int64_t new_qps =
            lwrap_add(to_add, rest) > max_count ? max_count - acquire : lwrap_add(rest, to_add) - acquire;
        if (new_qps < 0) return 0;
        *old = new_qps;
        *lru_peek(p->time, value) = now;
        return 1;
    }
    int64_t *old = lru_get(p->token, value);
    if (old) {
        if (*old - acquire >= 0) {
            *old -= acquire;
            return 1;
        }
        return 0;
    }
    /* the spin case (unreachable under one thread, see above): the refill branch at `now` */
    lru_put_if_absent(p->token, value, max_count - acquire);
    *lru_peek(p->time, value) = now;
    return 1;
}

/* ParamFlowChecker.passThrottleLocalCheck, ParamFlowChecker.java:224-281 (time map only) */
static int pass_throttle(orc_prule *p, uint64_t value, int acquire, int64_t now, int64_t *wait_ms) {
    int64_t token_count = j_d2l(p->r.count);
    int64_t hot;
    if (hot_lookup(p, value, &hot)) token_count = hot;
    if (token_count == 0) return 0;
    const int64_t cost =
        j_round(1.0 * 1000 * (double)acquire * (double)p->r.duration_in_sec / (double)token_count);
    int64_t *rec = lru_put_if_absent(p->time, value, now);
    if (!rec) return 1;
    const int64_t last = *rec;
    const int64_t expected = last + cost;
    if (expected <= now || expected - now < p->r.max_queueing_time_ms) {
        rec = lru_get(p->time, value); /* timeRecorderMap.get(value): already the MRU key */
        *rec = now;
        const int64_t wait = expected - now;
        if (wait > 0) {
            *rec = expected;
            *wait_ms = wait;
        }
        return 1;
    }
    return 0;
}

/* ParamFlowChecker.passSingleValueCheck, ParamFlowChecker.java:103-130 */
int orc_prule_pass_single(orc_prule *p, uint64_t value, int acquire, int64_t now, int64_t thread_count,
                          int64_t *wait_ms) {
    int64_t dummy;
    if (!wait_ms) wait_ms = &dummy;
    *wait_ms = 0;
    if (p->r.grade == ORC_GRADE_QPS) {
        if (p->r.control_behavior == ORC_CTRL_RATE_LIMITER) return pass_throttle(p, value, acquire, now, wait_ms);
        return pass_default(p, value, acquire, now);
    }
    if (p->r.grade == ORC_GRADE_THREAD) {
        int64_t hot;
        if (hot_lookup(p, value, &hot)) return ++thread_count <= hot;
        return ++thread_count <= j_d2l(p->r.count);
    }
    return 1;
}

/* ---------------------------------------------------------------- circuit breakers */
enum { CB_CLOSED = 0, CB_OPEN = 1, CB_HALF_OPEN = 2 };

struct orc_cb {
    orc_degrade_rule r;
    int state;
    int64_t next_retry;
    int64_t recovery_ms;      /* timeWindow * 1000, AbstractCircuitBreaker.java:54 */
    int64_t max_allowed_rt;   /* Math.round(count), ResponseTimeCircuitBreaker.java:52 */
    int64_t probe_t;          /* time of the entry that moved it OPEN -> HALF_OPEN (its whenTerminate hook) */
    orc_leap *stat;           /* LeapArray(1, statIntervalMs) of {err|slow, total} */
};

static orc_cb *cb_new(const orc_degrade_rule *r) {
    orc_cb *c = (orc_cb *)calloc(1, sizeof(orc_cb));
    c->r = *r;
    c->state = CB_CLOSED;
    c->recovery_ms = (int64_t)r->time_window * 1000;
    c->max_allowed_rt = j_round(r->count);
    c->stat = orc_leap_new(ORC_LEAP_UNARY, 1, r->stat_interval_ms);
    return c;
}

static void cb_free(orc_cb *c) {
    if (!c) return;
    orc_leap_free(c->stat);
    free(c);
}

/* AbstractCircuitBreaker.tryPass, AbstractCircuitBreaker.java:73-87 (+fromOpenToHalfOpen :117-139) */
static int cb_try_pass(orc_cb *c, int64_t now, int *to_half_open) {
    *to_half_open = 0;
    if (c->state == CB_CLOSED) return 1;
    if (c->state == CB_OPEN) {
        if (now >= c->next_retry) {
            c->state = CB_HALF_OPEN;
            c->probe_t = now;
            *to_half_open = 1;
            return 1;
        }
        return 0;
    }
    return 0;
}

static void cb_to_open(orc_cb *c, int64_t now) { /* transformToOpen / fromHalfOpenToOpen */
    if (c->state == CB_CLOSED || c->state == CB_HALF_OPEN) {
        c->state = CB_OPEN;
        c->next_retry = now + c->recovery_ms; /* updateNextRetryTimestamp */
    }
}

/* onRequestComplete: ExceptionCircuitBreaker.java:69-128 / ResponseTimeCircuitBreaker.java:64-128.
 * Bucket counter 0 = error or slow count, counter 1 = total count. */
static void cb_on_complete(orc_cb *c, int64_t now, int64_t rt, int error) {
    const int is_rt = c->r.grade == 0;
    const int bad = is_rt ? (rt > c->max_allowed_rt) : error;
    if (bad) orc_leap_add(c->stat, now, 0, 1);
    orc_leap_add(c->stat, now, 1, 1);
    if (c->state == CB_OPEN) return;
    if (c->state == CB_HALF_OPEN) {
        if (bad) {
            cb_to_open(c, now);
        } else {
            c->state = CB_CLOSED; /* fromHalfOpenToClose -> resetStat: currentWindow().value().reset() */
            orc_leap_current_window(c->stat, now);
            int64_t e = orc_leap_current_get(c->stat, now, 0), t = orc_leap_current_get(c->stat, now, 1);
            orc_leap_add(c->stat, now, 0, -e);
            orc_leap_add(c->stat, now, 1, -t);
        }
        return;
    }
    const int64_t bad_count = orc_leap_values_sum(c->stat, now, 0, NULL);
    const int64_t total = orc_leap_values_sum(c->stat, now, 1, NULL);
    if (total < c->r.min_request_amount) return;
    if (is_rt) {
        const double ratio = (double)bad_count * 1.0 / (double)total;
        if (ratio > c->r.slow_ratio_threshold) cb_to_open(c, now);
        /* Double.compare(ratio, max) == 0 && Double.compare(max, 1.0) == 0 */
        if (ratio == c->r.slow_ratio_threshold && c->r.slow_ratio_threshold == 1.0) cb_to_open(c, now);
    } else {
        double cur = (double)bad_count;
        if (c->r.grade == 1) cur = (double)bad_count * 1.0 / (double)total;
        if (cur > c->r.count) cb_to_open(c, now);
    }
}

int orc_flow_cb_state(orc_flow *f, uint32_t resource, int k) {
    if (resource >= f->n || k >= f->res[resource].ncb) return -1;
    return f->res[resource].cb[k]->state;
}

/* ---------------------------------------------------------------- rule loading */
static int param_rule_valid(const orc_param_rule *r) { /* ParamFlowRuleUtil.isValidRule + checkCluster, :46-69 */
    if (!(r->count >= 0 && r->grade >= 0 && r->duration_in_sec > 0 && r->burst_count >= 0 &&
          r->control_behavior >= 0 && r->max_queueing_time_ms >= 0))
        return 0;
    if (!r->cluster_mode) return 1;
    if (!(r->cluster_sample_count > 0 && r->cluster_window_ms > 0 && r->cluster_window_ms % r->cluster_sample_count == 0))
        return 0; /* FlowRuleUtil.isWindowConfigValid */
    return r->cluster_flow_id > 0; /* validClusterRuleId */
}

/* ParamFlowRule.equals (ParamFlowRule.java:192-210) of a loaded rule `old` -- whose paramIdx the slot
 * may have rewritten (applyRealParamIdx mutates the rule object) -- and a new rule b */
static int param_rule_equal(const orc_prule *old, const orc_param_rule *b) {
    const orc_param_rule *a = &old->r;
    const int32_t aidx = old->resolved ? old->idx : a->param_idx;
    if (a->grade != b->grade || a->count != b->count || a->control_behavior != b->control_behavior ||
        a->max_queueing_time_ms != b->max_queueing_time_ms || a->burst_count != b->burst_count ||
        aidx != b->param_idx || a->duration_in_sec != b->duration_in_sec || a->n_hot != b->n_hot ||
        a->cluster_mode != b->cluster_mode)
        return 0;
    if (a->cluster_mode && (a->cluster_fallback != b->cluster_fallback || a->cluster_flow_id != b->cluster_flow_id ||
                            a->cluster_sample_count != b->cluster_sample_count ||
                            a->cluster_window_ms != b->cluster_window_ms))
        return 0;
    for (uint32_t i = 0; i < a->n_hot; i++)
        if (a->hot_values[i] != b->hot_values[i] || a->hot_thresholds[i] != b->hot_thresholds[i]) return 0;
    return 1;
}

static void thread_map_remove(flow_res *fr, int32_t idx) { /* threadCountMap.remove(idx) */
    for (int k = 0; k < fr->npt; k++)
        if (fr->pt_idx[k] == idx) {
            lru_free(fr->pt_map[k]);
            fr->pt_idx[k] = fr->pt_idx[fr->npt - 1];
            fr->pt_map[k] = fr->pt_map[fr->npt - 1];
            fr->npt--;
            return;
        }
}

static void thread_maps_clear(flow_res *fr) { /* ParameterMetricStorage.clearParamMetricForResource */
    for (int k = 0; k < fr->npt; k++) lru_free(fr->pt_map[k]);
    fr->npt = 0;
}

/* ParamFlowRuleManager.loadRules (ParamFlowRuleManager.java:101-150): rules grouped by resource in list
 * order; the ParameterMetric maps are keyed by the rule (equal rules keep their maps).
 * aggregateAndPrepareParamRules: no rules at all clears every metric; a resource left without rules
 * loses its metric; each removed rule clears its maps and the thread-count map of its paramIdx
 * (ParameterMetric.clearForRule, ParameterMetric.java:86-92). */
int orc_flow_load_param_rules(orc_flow *f, const orc_param_rule *rules, size_t n) {
    int valid = 0;
    for (size_t j = 0; j < n; j++)
        if (rules[j].resource < f->n && param_rule_valid(&rules[j])) valid++;
    if (valid == 0)
        for (uint32_t i = 0; i < f->n; i++) thread_maps_clear(&f->res[i]);
    valid = 0;
    for (uint32_t i = 0; i < f->n; i++) {
        flow_res *fr = &f->res[i];
        orc_prule **old = fr->prule;
        int nold = fr->nprule;
        fr->prule = NULL;
        fr->nprule = 0;
        for (size_t j = 0; j < n; j++) {
            if (rules[j].resource != i || !param_rule_valid(&rules[j])) continue;
            orc_prule *keep = NULL;
            for (int k = 0; k < nold; k++)
                if (old[k] && param_rule_equal(old[k], &rules[j])) {
                    keep = old[k];
                    old[k] = NULL;
                    break;
                }
            if (!keep) keep = orc_prule_new(&rules[j]);
            fr->prule = (orc_prule **)realloc(fr->prule, sizeof(orc_prule *) * (size_t)(fr->nprule + 1));
            fr->prule[fr->nprule++] = keep;
            valid++;
        }
        if (nold && !fr->nprule) thread_maps_clear(fr);
        for (int k = 0; k < nold; k++) {
            if (old[k] && fr->nprule) thread_map_remove(fr, old[k]->resolved ? old[k]->idx : old[k]->r.param_idx);
            orc_prule_free(old[k]);
        }
        free(old);
    }
    return valid;
}

static int degrade_rule_valid(const orc_degrade_rule *r) { /* DegradeRuleManager.isValidRule, :171-203 */
    if (!(r->count >= 0 && r->time_window > 0)) return 0;
    if (r->min_request_amount <= 0 || r->stat_interval_ms <= 0) return 0;
    switch (r->grade) {
    case 0: return r->slow_ratio_threshold >= 0 && r->slow_ratio_threshold <= 1;
    case 1: return r->count <= 1;
    case 2: return 1;
    default: return 0;
    }
}

static int degrade_rule_equal(const orc_degrade_rule *a, const orc_degrade_rule *b) {
    return a->grade == b->grade && a->count == b->count && a->time_window == b->time_window &&
           a->min_request_amount == b->min_request_amount && a->slow_ratio_threshold == b->slow_ratio_threshold &&
           a->stat_interval_ms == b->stat_interval_ms;
}

/* DegradeRuleManager.loadRules -> buildCircuitBreakers: an unchanged rule keeps its breaker
 * (getExistingSameCbOrNew, DegradeRuleManager.java:150-163). */
int orc_flow_load_degrade_rules(orc_flow *f, const orc_degrade_rule *rules, size_t n) {
    int valid = 0;
    for (uint32_t i = 0; i < f->n; i++) {
        flow_res *fr = &f->res[i];
        orc_cb **old = fr->cb;
        int nold = fr->ncb;
        fr->cb = NULL;
        fr->ncb = 0;
        for (size_t j = 0; j < n; j++) {
            if (rules[j].resource != i || !degrade_rule_valid(&rules[j])) continue;
            orc_cb *keep = NULL;
            for (int k = 0; k < nold; k++)
                if (old[k] && degrade_rule_equal(&old[k]->r, &rules[j])) {
                    keep = old[k];
                    old[k] = NULL;
                    break;
                }
            if (!keep) keep = cb_new(&rules[j]);
            fr->cb = (orc_cb **)realloc(fr->cb, sizeof(orc_cb *) * (size_t)(fr->ncb + 1));
            fr->cb[fr->ncb++] = keep;
            valid++;
        }
        for (int k = 0; k < nold; k++) cb_free(old[k]);
        free(old);
    }
    return valid;
}

void orc_flow_res_free_ext(flow_res *fr) {
    for (int k = 0; k < fr->nprule; k++) orc_prule_free(fr->prule[k]);
    free(fr->prule);
    for (int k = 0; k < fr->npt; k++) lru_free(fr->pt_map[k]);
    free(fr->pt_map);
    free(fr->pt_idx);
    for (int k = 0; k < fr->ncb; k++) cb_free(fr->cb[k]);
    free(fr->cb);
}

/* ---------------------------------------------------------------- slot chain */
/* ---- the event's arguments ------------------------------------------------------------------
 * args[k] of the current event: the argument vector (SGA_EV_ARGS), else the round-2 forms (args = [param]
 * with has_param, a Collection / array args[0] with plist, or args = []). */
enum { ARG_SCALAR = 0, ARG_NULL = 1, ARG_LIST = 2 };

static uint32_t ev_nargs(const orc_flow *f, int has_param) { return f->args ? f->nargs : (has_param ? 1u : 0u); }

static int ev_arg(const orc_flow *f, uint32_t k, uint64_t param, const uint64_t **vals, uint32_t *n) {
    if (f->args) {
        const uint64_t h = f->args[2 * k], w = f->args[2 * k + 1];
        const int kind = (int)(h >> 62);
        if (kind == ARG_LIST) {
            *vals = f->args_pvals + w;
            *n = (uint32_t)(h & 0xffffffffu);
        } else {
            *vals = &f->args[2 * k + 1];
            *n = 1;
        }
        return kind;
    }
    if (k == 0 && f->plist) {
        *vals = f->plist;
        *n = f->plist_n;
        return ARG_LIST;
    }
    static uint64_t scratch; /* single-threaded oracle */
    scratch = param;
    *vals = &scratch;
    *n = 1;
    return ARG_SCALAR;
}

/* ParameterMetric.threadCountMap.get(index), or NULL (ParameterMetric.java:53, 115-120) */
static orc_lru *thread_map(const flow_res *fr, int32_t idx) {
    for (int k = 0; k < fr->npt; k++)
        if (fr->pt_idx[k] == idx) return fr->pt_map[k];
    return NULL;
}

/* ParameterMetricStorage.initParamMetricsFor -> ParameterMetric.initialize(rule): the thread map of the
 * rule's paramIdx is created once (:113-121) */
static void thread_map_init(flow_res *fr, int32_t idx) {
    if (thread_map(fr, idx)) return;
    fr->pt_idx = (int32_t *)realloc(fr->pt_idx, sizeof(int32_t) * (size_t)(fr->npt + 1));
    fr->pt_map = (orc_lru **)realloc(fr->pt_map, sizeof(orc_lru *) * (size_t)(fr->npt + 1));
    fr->pt_idx[fr->npt] = idx;
    fr->pt_map[fr->npt] = lru_new(PM_THREAD_COUNT_MAX_CAPACITY);
    fr->npt++;
}

/* ParameterMetric.addThreadCount / decreaseThreadCount (ParameterMetric.java:125-230): for every argument
 * index that has a thread map, every element of a Collection / array argument, else the value; null
 * arguments are skipped.  Each map is a CacheMap of capacity 4000, LRU as above. */
static void param_threads(const orc_flow *f, flow_res *fr, int has_param, uint64_t param, int delta) {
    if (!fr->npt) return;
    const uint32_t na = ev_nargs(f, has_param);
    for (uint32_t k = 0; k < na; k++) {
        orc_lru *m = thread_map(fr, (int32_t)k);
        if (!m) continue;
        const uint64_t *v;
        uint32_t nv;
        if (ev_arg(f, k, param, &v, &nv) == ARG_NULL) continue;
        for (uint32_t i = 0; i < nv; i++) {
            int64_t *c = lru_put_if_absent(m, v[i], 0); /* putIfAbsent(value, new AtomicInteger()) */
            if (delta > 0) {
                if (c) (*c)++;                 /* oldValue.incrementAndGet() */
                else lru_put(m, v[i], 1);      /* put(value, new AtomicInteger(1)) */
            } else if (c && --(*c) <= 0) {     /* absent: stays as a 0 entry */
                lru_remove(m, v[i]);
            }
        }
    }
}
static void param_thread_add(const orc_flow *f, flow_res *fr, int has_param, uint64_t param) {
    param_threads(f, fr, has_param, param, 1);
}
static void param_thread_dec(const orc_flow *f, flow_res *fr, int has_param, uint64_t param) {
    param_threads(f, fr, has_param, param, -1);
}

/* ParamFlowChecker.passLocalCheck (ParamFlowChecker.java:79-106): every element of a Collection / array
 * must pass, in order (the elements before a failing one keep their token updates) */
static int param_local_check(flow_res *fr, orc_prule *p, const uint64_t *vals, uint32_t nv, int acquire,
                             int64_t now, int64_t *total_wait) {
    for (uint32_t q = 0; q < nv; q++) {
        int64_t tc = 0;
        if (p->r.grade == ORC_GRADE_THREAD) { /* getThreadCount(rule.getParamIdx(), value): CacheMap.get */
            orc_lru *m = thread_map(fr, p->idx);
            int64_t *c = m ? lru_get(m, vals[q]) : NULL;
            tc = c ? *c : 0;
        }
        int64_t w = 0;
        if (!orc_prule_pass_single(p, vals[q], acquire, now, tc, &w)) return 0;
        *total_wait += w;
    }
    return 1;
}

int32_t orc_flow_param_idx(const orc_flow *f, uint32_t r, int k) {
    if (r >= f->n || k >= f->res[r].nprule) return INT32_MIN;
    const orc_prule *p = f->res[r].prule[k];
    return p->resolved ? p->idx : INT32_MIN;
}

/* CtSph.entryWithPriority -> StatisticSlot.entry (StatisticSlot.java:64-145) around
 * ParamFlowSlot.checkFlow (ParamFlowSlot.java:65-92), FlowSlot (FlowSlot.java:161-172)
 * and DegradeSlot.performChecking (DegradeSlot.java:49-66). */
int orc_flow_entry_p(orc_flow *f, uint32_t resource, int64_t now, int acquire, int prioritized, int has_param,
                     uint64_t param, int64_t *wait_ms) {
    int64_t dummy;
    if (!wait_ms) wait_ms = &dummy;
    *wait_ms = 0;
    if (resource >= f->n) return ORC_PASS;
    flow_res *fr = &f->res[resource];
    int64_t total_wait = 0;
    /* ParamFlowSlot.checkFlow: args is never null here (SphU.entry passes an empty array) */
    const uint32_t nargs = ev_nargs(f, has_param);
    for (int k = 0; k < fr->nprule; k++) {
        orc_prule *p = fr->prule[k];
        if (!p->resolved) { /* applyRealParamIdx: a negative index is rewritten on the rule, once */
            int idx = p->r.param_idx;
            if (idx < 0) idx = (-idx <= (int)nargs) ? (int)nargs + idx : -idx;
            p->idx = idx;
            p->resolved = 1;
        }
        thread_map_init(fr, p->idx); /* ParameterMetricStorage.initParamMetricsFor */
        /* ParamFlowChecker.passCheck (:48-77): args.length <= paramIdx or a null value pass */
        if ((int64_t)nargs <= (int64_t)p->idx) continue;
        const uint64_t *vals;
        uint32_t nv;
        if (ev_arg(f, (uint32_t)p->idx, param, &vals, &nv) == ARG_NULL) continue;
        int ok;
        if (p->r.cluster_mode && p->r.grade == ORC_GRADE_QPS) {
            /* passClusterCheck (:305-333): requestParamToken(flowId, count, toCollection(value)) to the
             * embedded server; OK passes, BLOCKED blocks, anything else (or no service) falls back:
             * fallbackToLocalOrPass (:335-343) checks the collection locally or passes */
            int st = -1; /* TokenResultStatus.FAIL: no token service */
            if (f->server && f->cluster_mode == 1) {
                const orc_token_result r = orc_cluster_request_param_token(f->server, p->r.cluster_flow_id, acquire,
                                                                           (const int64_t *)vals, nv, now);
                st = r.status;
            }
            if (st == 0) ok = 1;
            else if (st == 1) ok = 0;
            else ok = p->r.cluster_fallback ? param_local_check(fr, p, vals, nv, acquire, now, &total_wait) : 1;
        } else {
            ok = param_local_check(fr, p, vals, nv, acquire, now, &total_wait);
        }
        if (!ok) {
            orc_node_increase_block_qps(fr->node, now, acquire);
            *wait_ms = k; /* block detail: the ParamFlowRule's index in the resource's list */
            return ORC_BLOCK_PARAM;
        }
    }
    /* FlowSlot */
    int64_t w = 0;
    int d = orc_flow_rule_check(f, resource, now, acquire, prioritized, &w);
    if (d == ORC_BLOCK_FLOW) {
        orc_node_increase_block_qps(fr->node, now, acquire);
        *wait_ms = w; /* block detail: the blocking FlowRule's index */
        return ORC_BLOCK_FLOW;
    }
    if (d == ORC_PASS_WAIT) { /* PriorityWaitException: thread++ and entry callbacks only */
        orc_node_increase_thread_num(fr->node);
        param_thread_add(f, fr, has_param, param);
        *wait_ms = w;
        return ORC_PASS_WAIT;
    }
    total_wait += w;
    /* DegradeSlot */
    uint8_t half_open_here[64];
    for (int k = 0; k < fr->ncb; k++) {
        int half = 0;
        const int ok = cb_try_pass(fr->cb[k], now, &half);
        if (k < 64) half_open_here[k] = (uint8_t)half;
        if (!ok) {
            /* DegradeException: CtSph exits the entry; the whenTerminate handlers of the
             * breakers that turned half-open for THIS entry see the block error and move
             * HALF_OPEN -> OPEN without touching nextRetryTimestamp (AbstractCircuitBreaker.java:123-134) */
            for (int q = 0; q < k && q < 64; q++)
                if (half_open_here[q] && fr->cb[q]->state == CB_HALF_OPEN) fr->cb[q]->state = CB_OPEN;
            orc_node_increase_block_qps(fr->node, now, acquire);
            *wait_ms = k; /* block detail: the breaker's index */
            return ORC_BLOCK_DEGRADE;
        }
    }
    orc_node_increase_thread_num(fr->node);
    orc_node_add_pass_request(fr->node, now, acquire);
    param_thread_add(f, fr, has_param, param);
    *wait_ms = total_wait;
    return ORC_PASS;
}

/* Entry.exit of a passed entry: StatisticSlot.exit (:147-175), ParamFlowStatisticExitCallback,
 * DegradeSlot.exit (DegradeSlot.java:68-89). */
void orc_flow_exit_p(orc_flow *f, uint32_t resource, int64_t now, int64_t rt, int count, int error, int has_param,
                     uint64_t param) {
    if (resource >= f->n) return;
    flow_res *fr = &f->res[resource];
    orc_node *n = fr->node;
    orc_node_add_rt_and_success(n, now, rt, count);
    orc_node_decrease_thread_num(n);
    if (error) orc_node_increase_exception_qps(n, now, count);
    param_thread_dec(f, fr, has_param, param);
    for (int k = 0; k < fr->ncb; k++) cb_on_complete(fr->cb[k], now, rt, error);
}

/* ---- SystemSlot (CORE/slots/system) --------------------------------------- */
#include <float.h>

/* SystemPropertyListener.restoreSetting, SystemRuleManager.java:225-240 */
void orc_flow_system_restore(orc_flow *f) {
    f->sys.check = 0;
    f->sys.load = DBL_MAX;
    f->sys.cpu = DBL_MAX;
    f->sys.qps = DBL_MAX;
    f->sys.max_rt = INT64_MAX;
    f->sys.max_thread = INT64_MAX;
    f->sys.load_set = 0;
    f->sys.cpu_set = 0;
}

/* SystemPropertyListener.configUpdate + loadSystemConf, SystemRuleManager.java:191-300: every field
 * >= 0 lowers its threshold; checkSystemStatus ends as the LAST rule's "some field set" (the
 * reference sets it per rule); an empty list switches the check off.  Returns the rules applied. */
int orc_flow_load_system_rules(orc_flow *f, const orc_system_rule *rules, size_t n) {
    orc_flow_system_restore(f);
    int applied = 0;
    for (size_t i = 0; i < n; i++) {
        const orc_system_rule *r = &rules[i];
        int st = 0;
        if (r->highest_system_load >= 0) {
            if (r->highest_system_load < f->sys.load) f->sys.load = r->highest_system_load;
            f->sys.load_set = 1;
            st = 1;
        }
        if (r->highest_cpu_usage >= 0 && r->highest_cpu_usage <= 1) { /* > 1: ignored as invalid */
            if (r->highest_cpu_usage < f->sys.cpu) f->sys.cpu = r->highest_cpu_usage;
            f->sys.cpu_set = 1;
            st = 1;
        }
        if (r->avg_rt >= 0) {
            if (r->avg_rt < f->sys.max_rt) f->sys.max_rt = r->avg_rt;
            st = 1;
        }
        if (r->max_thread >= 0) {
            if (r->max_thread < f->sys.max_thread) f->sys.max_thread = r->max_thread;
            st = 1;
        }
        if (r->qps >= 0) {
            if (r->qps < f->sys.qps) f->sys.qps = r->qps;
            st = 1;
        }
        f->sys.check = st;
        applied += st;
    }
    return applied;
}

/* SystemStatusListener readings (OperatingSystemMXBean load average / CPU usage, sampled each second) */
void orc_flow_set_system_status(orc_flow *f, double avg_load, double cpu_usage) {
    f->sys.cur_load = avg_load;
    f->sys.cur_cpu = cpu_usage;
}

/* SystemRuleManager.checkSystem + checkBbr for an inbound entry, SystemRuleManager.java:298-353: the check
 * that throws (SystemBlockException limitType 0 "qps", 1 "thread", 2 "rt", 3 "load", 4 "cpu") or -1 */
static int system_block_type(orc_flow *f, int64_t now, int count) {
    if (!f->sys.check) return -1;
    orc_node *e = f->entry;
    if (orc_node_pass_qps(e, now) + count > f->sys.qps) return 0;
    const int32_t thr = orc_node_cur_thread_num(e);
    if ((int64_t)thr > f->sys.max_thread) return 1;
    if (orc_node_avg_rt(e, now) > (double)f->sys.max_rt) return 2;
    if (f->sys.load_set && f->sys.cur_load > f->sys.load) {
        if (thr > 1 && thr > orc_node_max_success_qps(e, now) * orc_node_min_rt(e, now) / 1000) return 3;
    }
    if (f->sys.cpu_set && f->sys.cur_cpu > f->sys.cpu) return 4;
    return -1;
}

/* The slot chain for one entry with its EntryType: SystemSlot before ParamFlowSlot / FlowSlot /
 * DegradeSlot, and StatisticSlot's ENTRY_NODE updates for inbound traffic (StatisticSlot.java:54-137). */
int orc_flow_entry_x(orc_flow *f, uint32_t resource, int64_t now, int acquire, int prioritized, int has_param,
                     uint64_t param, int inbound, int64_t *wait_ms) {
    int64_t dummy;
    if (!wait_ms) wait_ms = &dummy;
    *wait_ms = 0;
    if (resource >= f->n) return ORC_PASS;
    int d;
    const int sb = inbound ? system_block_type(f, now, acquire) : -1;
    if (sb >= 0) {
        orc_node_increase_block_qps(f->res[resource].node, now, acquire);
        d = ORC_BLOCK_SYSTEM;
        *wait_ms = sb; /* block detail: the SystemRule check */
    } else {
        d = orc_flow_entry_p(f, resource, now, acquire, prioritized, has_param, param, wait_ms);
    }
    if (inbound) {
        if (d == ORC_PASS) {
            orc_node_increase_thread_num(f->entry);
            orc_node_add_pass_request(f->entry, now, acquire);
        } else if (d == ORC_PASS_WAIT) {
            orc_node_increase_thread_num(f->entry);
        } else {
            orc_node_increase_block_qps(f->entry, now, acquire);
        }
    }
    return d;
}

void orc_flow_exit_x(orc_flow *f, uint32_t resource, int64_t now, int64_t rt, int count, int error, int has_param,
                     uint64_t param, int inbound) {
    if (resource >= f->n) return;
    orc_flow_exit_p(f, resource, now, rt, count, error, has_param, param);
    if (inbound) { /* recordCompleteFor(Constants.ENTRY_NODE, ...) */
        orc_node_add_rt_and_success(f->entry, now, rt, count);
        orc_node_decrease_thread_num(f->entry);
        if (error) orc_node_increase_exception_qps(f->entry, now, count);
    }
}

orc_node *orc_flow_entry_node(orc_flow *f) { return f->entry; }

/* As orc_flow_replay_p, with flags bit 4 (SGA_EV_PARAM_LIST): args[0] is a Collection / array whose
 * values are pvals[param >> 32 .. (param >> 32) + (param & 0xffffffff)). */
void orc_flow_replay_pl(orc_flow *f, size_t n, const uint8_t *kind, const uint32_t *resource, const int64_t *ts,
                        const int32_t *acquire, const uint8_t *flags, const int64_t *rt, const uint64_t *param,
                        const uint64_t *pvals, int8_t *decision, int32_t *wait_ms) {
    for (size_t i = 0; i < n; i++) {
        const uint8_t fl = flags ? flags[i] : 0;
        if ((fl & 16) && (fl & 4)) {
            f->plist = pvals + (param[i] >> 32);
            f->plist_n = (uint32_t)(param[i] & 0xffffffffu);
        }
        orc_flow_replay_p(f, 1, kind ? kind + i : NULL, resource + i, ts + i, acquire + i, flags ? flags + i : NULL,
                          rt ? rt + i : NULL, param ? param + i : NULL, decision ? decision + i : NULL,
                          wait_ms ? wait_ms + i : NULL);
        f->plist = NULL;
        f->plist_n = 0;
    }
}

void orc_flow_replay_args(orc_flow *f, size_t n, const uint8_t *kind, const uint32_t *resource, const int64_t *ts,
                          const int32_t *acquire, const uint8_t *flags, const int64_t *rt, const uint64_t *param,
                          const uint64_t *pvals, int8_t *decision, int32_t *wait_ms) {
    for (size_t i = 0; i < n; i++) {
        const uint8_t fl = flags ? flags[i] : 0;
        if (fl & 32) {
            f->args = pvals + (param[i] >> 32);
            f->args_pvals = pvals;
            f->nargs = (uint32_t)(param[i] & 0xffffffffu);
        } else if ((fl & 16) && (fl & 4)) {
            f->plist = pvals + (param[i] >> 32);
            f->plist_n = (uint32_t)(param[i] & 0xffffffffu);
        }
        orc_flow_replay_p(f, 1, kind ? kind + i : NULL, resource + i, ts + i, acquire + i, flags ? flags + i : NULL,
                          rt ? rt + i : NULL, param ? param + i : NULL, decision ? decision + i : NULL,
                          wait_ms ? wait_ms + i : NULL);
        f->args = NULL;
        f->args_pvals = NULL;
        f->nargs = 0;
        f->plist = NULL;
        f->plist_n = 0;
    }
}

/* flags: bit 0 prioritized, bit 1 error, bit 2 has_param, bit 3 inbound (EntryType.IN), bit 5 args */
void orc_flow_replay_p(orc_flow *f, size_t n, const uint8_t *kind, const uint32_t *resource, const int64_t *ts,
                       const int32_t *acquire, const uint8_t *flags, const int64_t *rt, const uint64_t *param,
                       int8_t *decision, int32_t *wait_ms) {
    for (size_t i = 0; i < n; i++) {
        const uint8_t fl = flags ? flags[i] : 0;
        const int hp = (fl & 4) != 0 || (fl & 32) != 0;
        const int in = (fl & 8) != 0;
        const uint64_t pv = param ? param[i] : 0;
        if (kind && kind[i] == 2) { /* StatisticSlot: a BlockException thrown by a slot outside the engine */
            if (resource[i] < f->n) {
                orc_node_increase_block_qps(f->res[resource[i]].node, ts[i], acquire[i]);
                if (in) orc_node_increase_block_qps(f->entry, ts[i], acquire[i]);
            }
            if (decision) decision[i] = ORC_PASS;
            if (wait_ms) wait_ms[i] = 0;
            continue;
        }
        if (kind && kind[i] == 3) { /* SGA_KIND_REVOKE: a later slot blocked a passed entry (StatisticSlot.java:71-84,
                                     * 121-135: the pass accounting never ran, the block is counted) */
            if (resource[i] < f->n) {
                flow_res *fr = &f->res[resource[i]];
                orc_node_decrease_thread_num(fr->node);
                orc_node_add_pass_request(fr->node, ts[i], -acquire[i]);
                orc_node_increase_block_qps(fr->node, ts[i], acquire[i]);
                param_thread_dec(f, fr, hp, pv);
                /* the probe's whenTerminate hook (AbstractCircuitBreaker.java:117-139): blockError set, so a
                 * breaker this entry moved to HALF_OPEN falls back to OPEN; the revoke carries the entry's time */
                for (int k = 0; k < fr->ncb; k++)
                    if (fr->cb[k]->state == CB_HALF_OPEN && fr->cb[k]->probe_t == ts[i]) fr->cb[k]->state = CB_OPEN;
                if (in) {
                    orc_node_decrease_thread_num(f->entry);
                    orc_node_add_pass_request(f->entry, ts[i], -acquire[i]);
                    orc_node_increase_block_qps(f->entry, ts[i], acquire[i]);
                }
            }
            if (decision) decision[i] = ORC_PASS;
            if (wait_ms) wait_ms[i] = 0;
            continue;
        }
        if (kind && kind[i] == 1) {
            orc_flow_exit_x(f, resource[i], ts[i], rt ? rt[i] : 0, acquire[i], (fl & 2) != 0, hp, pv, in);
            if (decision) decision[i] = ORC_PASS;
            if (wait_ms) wait_ms[i] = 0;
            continue;
        }
        int64_t w = 0;
        int d = orc_flow_entry_x(f, resource[i], ts[i], acquire[i], fl & 1, hp, pv, in, &w);
        if (decision) decision[i] = (int8_t)d;
        if (wait_ms) wait_ms[i] = (int32_t)w;
    }
}

/* Test introspection of the LRU maps: which = 0 time map, 1 token map of a rule */
size_t orc_prule_map_size(const orc_prule *p, int which) { return orc_lru_size(which ? p->token : p->time); }
uint64_t orc_prule_map_evictions(const orc_prule *p, int which) {
    return orc_lru_evictions(which ? p->token : p->time);
}
size_t orc_prule_map_keys(const orc_prule *p, int which, uint64_t *keys, int64_t *vals, size_t cap) {
    return orc_lru_keys(which ? p->token : p->time, keys, vals, cap);
}
/* resource `r`'s k-th parameter rule's maps (which 0/1) or its thread map (which 2) */
size_t orc_flow_param_map_size(const orc_flow *f, uint32_t r, int k, int which) {
    if (r >= f->n) return 0;
    const flow_res *fr = &f->res[r];
    if (which == 2) return orc_lru_size(fr->npt ? fr->pt_map[0] : NULL);
    if (k >= fr->nprule) return 0;
    return orc_prule_map_size(fr->prule[k], which);
}
