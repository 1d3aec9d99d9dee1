/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- the CPU baseline's contended form (bench.py / bench_local.py
 * `cpu_baseline`): the reference's multi-threaded path restated with its concurrency
 * design, for timing only (the decisions race exactly as the reference's do, so they are not a parity
 * check; the single-threaded replay in sentinel_oracle.c is the checker):
 *
 *   LongAdder (striped cells, base CAS first, a cell per thread probe, rehash on CAS failure)
 *                                      java.util.concurrent.atomic.LongAdder / Striped64 (JDK), as used by
 *                                      MetricBucket.java:20-45 and ClusterMetricBucket.java
 *   LeapArray.currentWindow            CORE/slots/statistic/base/LeapArray.java:121-170 (CAS of a new bucket into
 *                                      the AtomicReferenceArray, updateLock.tryLock() around resetWindowTo,
 *                                      Thread.yield() otherwise, a detached bucket when time goes back)
 *   ClusterMetricLeapArray.resetWindowTo + occupy transfer
 *                                      CS/flow/statistic/metric/ClusterMetricLeapArray.java:43-92
 *   ClusterMetric.getSum / getAvg / tryOccupyNext
 *                                      CS/flow/statistic/metric/ClusterMetric.java:39-98
 *   ClusterFlowChecker.acquireClusterToken
 *                                      CS/flow/ClusterFlowChecker.java:55-112
 *   StatisticNode (second 2 x 500 ms, minute 60 x 1 s, curThreadNum) + DefaultController.canPass +
 *   StatisticSlot entry/exit           CORE/node/StatisticNode.java:94-260, CORE/slots/block/flow/controller/
 *                                      DefaultController.java:48-84, CORE/slots/statistic/StatisticSlot.java:54-175
 *
 * T threads share one rule table and its windows; request i is handled by thread i mod T, each thread in
 * its requests' order, all threads at once (the clients of one token server / one JVM).
 */
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define NCELL 16 /* Striped64: cells grow to the next power of two >= NCPU; the 16 threads of the box */

typedef struct {
    _Alignas(64) atomic_llong v; /* @Contended cell */
} cell_t;

typedef struct {
    atomic_llong base;
    _Atomic(cell_t *) cells;
} ladder;

static _Thread_local uint32_t t_probe; /* ThreadLocalRandom probe */

static uint32_t probe_next(uint32_t p) { /* advanceProbe: xorshift */
    p ^= p << 13;
    p ^= p >> 17;
    p ^= p << 5;
    return p;
}

static void la_add(ladder *a, long long x) {
    cell_t *cs = atomic_load_explicit(&a->cells, memory_order_acquire);
    if (!cs) {
        long long b = atomic_load_explicit(&a->base, memory_order_relaxed);
        if (atomic_compare_exchange_strong(&a->base, &b, b + x)) return;
        cell_t *n = (cell_t *)aligned_alloc(64, sizeof(cell_t) * NCELL);
        for (int i = 0; i < NCELL; i++) atomic_init(&n[i].v, 0);
        cell_t *exp = NULL;
        if (!atomic_compare_exchange_strong(&a->cells, &exp, n)) {
            free(n);
            cs = exp;
        } else {
            cs = n;
        }
    }
    uint32_t p = t_probe;
    for (;;) {
        cell_t *c = &cs[p & (NCELL - 1)];
        long long v = atomic_load_explicit(&c->v, memory_order_relaxed);
        if (atomic_compare_exchange_weak(&c->v, &v, v + x)) break;
        p = probe_next(p); /* contended: move to another cell */
    }
    t_probe = p;
}

static long long la_sum(ladder *a) {
    long long s = atomic_load_explicit(&a->base, memory_order_relaxed);
    cell_t *cs = atomic_load_explicit(&a->cells, memory_order_acquire);
    if (cs)
        for (int i = 0; i < NCELL; i++) s += atomic_load_explicit(&cs[i].v, memory_order_relaxed);
    return s;
}

static void la_reset(ladder *a) {
    atomic_store_explicit(&a->base, 0, memory_order_relaxed);
    cell_t *cs = atomic_load_explicit(&a->cells, memory_order_acquire);
    if (cs)
        for (int i = 0; i < NCELL; i++) atomic_store_explicit(&cs[i].v, 0, memory_order_relaxed);
}

static long long la_sum_then_reset(ladder *a) {
    long long s = atomic_exchange(&a->base, 0);
    cell_t *cs = atomic_load_explicit(&a->cells, memory_order_acquire);
    if (cs)
        for (int i = 0; i < NCELL; i++) s += atomic_exchange(&cs[i].v, 0);
    return s;
}

static void la_free(ladder *a) { free(atomic_load(&a->cells)); }

/* ---- LeapArray<bucket> with the reference's currentWindow -------------------------------------------- */
enum { EV_PASS, EV_BLOCK, EV_PASS_REQUEST, EV_BLOCK_REQUEST, EV_OCCUPIED_PASS, EV_OCCUPIED_BLOCK, EV_WAITING,
       EV_N_CLUSTER };
enum { MB_PASS, MB_BLOCK, MB_EXCEPTION, MB_SUCCESS, MB_RT, MB_OCCUPIED_PASS, MB_N };

typedef struct wwrap {
    _Atomic long long start; /* WindowWrap.windowStart (written under the update lock) */
    ladder c[EV_N_CLUSTER];  /* the bucket's counters (ClusterMetricBucket: 7 events; MetricBucket: 6) */
    _Atomic long long min_rt;
} wwrap;

typedef struct {
    int S, W, interval;
    double isec;
    _Atomic(wwrap *) *arr;   /* AtomicReferenceArray<WindowWrap> */
    pthread_mutex_t lock;    /* updateLock (ReentrantLock) */
    /* ClusterMetricLeapArray only */
    ladder occ[EV_N_CLUSTER];
    atomic_int has_occ;
} leap;

static void leap_init(leap *l, int S, int interval) {
    l->S = S;
    l->interval = interval;
    l->W = interval / S;
    l->isec = interval / 1000.0;
    l->arr = calloc((size_t)S, sizeof(*l->arr));
    pthread_mutex_init(&l->lock, NULL);
    memset(l->occ, 0, sizeof(l->occ));
    atomic_init(&l->has_occ, 0);
}

static wwrap *wrap_new(long long start, long long max_rt) {
    wwrap *w = (wwrap *)calloc(1, sizeof(wwrap));
    atomic_init(&w->start, start);
    atomic_init(&w->min_rt, max_rt);
    return w;
}

static void leap_free(leap *l) {
    for (int j = 0; j < l->S; j++) {
        wwrap *w = atomic_load(&l->arr[j]);
        if (w) {
            for (int k = 0; k < EV_N_CLUSTER; k++) la_free(&w->c[k]);
            free(w);
        }
    }
    for (int k = 0; k < EV_N_CLUSTER; k++) la_free(&l->occ[k]);
    free(l->arr);
    pthread_mutex_destroy(&l->lock);
}

/* the bucket for time t; *detached = 1 for the throwaway bucket handed out when time went backwards
 * (the caller frees it) */
static wwrap *current_window(leap *l, long long t, int cluster, long long max_rt, int *detached) {
    const int idx = (int)((t / l->W) % l->S);
    const long long ws = t - t % l->W;
    *detached = 0;
    for (;;) {
        wwrap *old = atomic_load_explicit(&l->arr[idx], memory_order_acquire);
        if (!old) {
            wwrap *w = wrap_new(ws, max_rt);
            wwrap *exp = NULL;
            if (atomic_compare_exchange_strong(&l->arr[idx], &exp, w)) return w;
            free(w);
            sched_yield();
        } else if (ws == atomic_load_explicit(&old->start, memory_order_acquire)) {
            return old;
        } else if (ws > atomic_load_explicit(&old->start, memory_order_acquire)) {
            if (pthread_mutex_trylock(&l->lock) == 0) {
                if (ws > atomic_load(&old->start)) { /* resetWindowTo (another thread may have reset it) */
                    atomic_store(&old->start, ws);
                    for (int k = 0; k < EV_N_CLUSTER; k++) la_reset(&old->c[k]);
                    atomic_store(&old->min_rt, max_rt);
                    if (cluster && atomic_load(&l->has_occ)) { /* transferOccupyToBucket */
                        la_add(&old->c[EV_OCCUPIED_PASS], la_sum(&l->occ[EV_PASS]));
                        la_add(&old->c[EV_PASS], la_sum_then_reset(&l->occ[EV_PASS]));
                        la_add(&old->c[EV_PASS_REQUEST], la_sum_then_reset(&l->occ[EV_PASS_REQUEST]));
                        atomic_store(&l->has_occ, 0);
                    }
                }
                pthread_mutex_unlock(&l->lock);
                return old;
            }
            sched_yield();
        } else {
            *detached = 1;
            return wrap_new(ws, max_rt);
        }
    }
}

static void leap_add(leap *l, long long t, int ev, long long x, int cluster, long long max_rt) {
    int det;
    wwrap *w = current_window(l, t, cluster, max_rt, &det);
    la_add(&w->c[ev], x);
    if (det) {
        for (int k = 0; k < EV_N_CLUSTER; k++) la_free(&w->c[k]);
        free(w);
    }
}

/* getSum: currentWindow() then the valid buckets (LeapArray.values / isWindowDeprecated) */
static long long leap_sum(leap *l, long long t, int ev, int cluster, long long max_rt) {
    int det;
    wwrap *cw = current_window(l, t, cluster, max_rt, &det);
    if (det) {
        for (int k = 0; k < EV_N_CLUSTER; k++) la_free(&cw->c[k]);
        free(cw);
    }
    long long s = 0;
    for (int j = 0; j < l->S; j++) {
        wwrap *w = atomic_load_explicit(&l->arr[j], memory_order_acquire);
        if (!w || t - atomic_load_explicit(&w->start, memory_order_relaxed) > l->interval) continue;
        s += la_sum(&w->c[ev]);
    }
    return s;
}

/* ---- ClusterFlowChecker over ClusterMetric --------------------------------------------------------- */
typedef struct {
    int64_t fid;
    double thr;
    leap m;
} crule;

typedef struct {
    crule *rules;
    size_t nrules;
    uint32_t *htab; /* flowId -> rule index + 1 (read-only during the run: ClusterFlowRuleManager's map) */
    size_t hmask;
    double max_occupy_ratio;
    /* the trace */
    size_t n;
    const int64_t *fid;
    const int32_t *acq;
    const uint8_t *prio;
    const int64_t *ts;
    int32_t *status;
    int nthreads;
} cctx;

static uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static crule *crule_find(cctx *c, int64_t fid) {
    size_t h = mix64((uint64_t)fid) & c->hmask;
    while (c->htab[h]) {
        crule *r = &c->rules[c->htab[h] - 1];
        if (r->fid == fid) return r;
        h = (h + 1) & c->hmask;
    }
    return NULL;
}

static int32_t cluster_token(cctx *c, int64_t fid, int32_t a, int p, long long t) {
    if (fid <= 0 || a <= 0) return -4; /* BAD_REQUEST */
    crule *r = crule_find(c, fid);
    if (!r) return 3; /* NO_RULE_EXISTS */
    leap *m = &r->m;
    const double latest = (double)leap_sum(m, t, EV_PASS, 1, 0) / m->isec;
    const double next = r->thr - latest - (double)a;
    if (next >= 0) {
        leap_add(m, t, EV_PASS, a, 1, 0);
        leap_add(m, t, EV_PASS_REQUEST, 1, 1, 0);
        if (p) leap_add(m, t, EV_OCCUPIED_PASS, a, 1, 0);
        return 0;
    }
    if (p) {
        const double occ_avg = (double)leap_sum(m, t, EV_WAITING, 1, 0) / m->isec;
        if (occ_avg <= c->max_occupy_ratio * r->thr) { /* tryOccupyNext */
            const double latest2 = (double)leap_sum(m, t, EV_PASS, 1, 0) / m->isec;
            /* getValidHead: the bucket after the current one, if still valid */
            const int hidx = (int)(((t + m->W) / m->W) % m->S);
            wwrap *hw = atomic_load(&m->arr[hidx]);
            long long head = 0;
            if (hw && !(t - atomic_load(&hw->start) > m->interval)) head = la_sum(&hw->c[EV_PASS]);
            if (latest2 + (double)(a + la_sum(&m->occ[EV_PASS])) - (double)head <= r->thr) {
                la_add(&m->occ[EV_PASS], a);
                la_add(&m->occ[EV_PASS_REQUEST], 1);
                atomic_store(&m->has_occ, 1);
                leap_add(m, t, EV_WAITING, a, 1, 0);
                if (1000 / m->S > 0) return 2; /* SHOULD_WAIT */
            }
        }
    }
    leap_add(m, t, EV_BLOCK, a, 1, 0);
    leap_add(m, t, EV_BLOCK_REQUEST, 1, 1, 0);
    if (p) leap_add(m, t, EV_OCCUPIED_BLOCK, a, 1, 0);
    return 1; /* BLOCKED */
}

typedef struct {
    void *ctx;
    int k;
    pthread_barrier_t *bar;
} targ;

static void *cluster_worker(void *v) {
    targ *ta = (targ *)v;
    cctx *c = (cctx *)ta->ctx;
    t_probe = (uint32_t)mix64((uint64_t)ta->k + 1) | 1u;
    pthread_barrier_wait(ta->bar);
    for (size_t i = (size_t)ta->k; i < c->n; i += (size_t)c->nthreads) {
        const int32_t s = cluster_token(c, c->fid[i], c->acq[i], c->prio ? c->prio[i] : 0, c->ts[i]);
        if (c->status) c->status[i] = s;
    }
    return NULL;
}

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + t.tv_nsec * 1e-9;
}

static double run_threads(void *ctx, int nthreads, void *(*fn)(void *)) {
    pthread_t th[256];
    targ ta[256];
    pthread_barrier_t bar;
    if (nthreads > 256) nthreads = 256;
    pthread_barrier_init(&bar, NULL, (unsigned)nthreads + 1);
    for (int k = 0; k < nthreads; k++) {
        ta[k].ctx = ctx;
        ta[k].k = k;
        ta[k].bar = &bar;
        pthread_create(&th[k], NULL, fn, &ta[k]);
    }
    pthread_barrier_wait(&bar);
    const double t0 = now_s();
    for (int k = 0; k < nthreads; k++) pthread_join(th[k], NULL);
    const double dt = now_s() - t0;
    pthread_barrier_destroy(&bar);
    return dt;
}

/* C3: `nthreads` threads over the cluster trace (request i on thread i mod nthreads) against `nrules` GLOBAL
 * cluster FlowRules (flowId, count) of sampleCount S over interval_ms.  Returns the wall seconds of the
 * threads' run (rules and windows set up before the clock starts); status_out (may be NULL) gets each
 * request's TokenResultStatus. */
double orc_contended_cluster(int nthreads, size_t nrules, const int64_t *rule_fid, const double *rule_count, int S,
                             int interval_ms, size_t n, const int64_t *fid, const int32_t *acq, const uint8_t *prio,
                             const int64_t *ts, int32_t *status_out) {
    cctx c;
    memset(&c, 0, sizeof(c));
    c.rules = (crule *)calloc(nrules ? nrules : 1, sizeof(crule));
    c.nrules = nrules;
    size_t hc = 16;
    while (hc < 2 * nrules) hc <<= 1;
    c.htab = (uint32_t *)calloc(hc, sizeof(uint32_t));
    c.hmask = hc - 1;
    c.max_occupy_ratio = 1.0;
    for (size_t i = 0; i < nrules; i++) {
        c.rules[i].fid = rule_fid[i];
        c.rules[i].thr = rule_count[i] * 1.0; /* GLOBAL threshold x exceedCount 1.0 */
        leap_init(&c.rules[i].m, S, interval_ms);
        size_t h = mix64((uint64_t)rule_fid[i]) & c.hmask;
        while (c.htab[h]) h = (h + 1) & c.hmask;
        c.htab[h] = (uint32_t)(i + 1);
    }
    c.n = n;
    c.fid = fid;
    c.acq = acq;
    c.prio = prio;
    c.ts = ts;
    c.status = status_out;
    c.nthreads = nthreads < 1 ? 1 : nthreads;
    const double dt = run_threads(&c, c.nthreads, cluster_worker);
    for (size_t i = 0; i < nrules; i++) leap_free(&c.rules[i].m);
    free(c.rules);
    free(c.htab);
    return dt;
}

/* ---- StatisticNode + DefaultController (C1 HelloWorld) -------------------------------------------- */
#define MAX_RT 5000 /* SentinelConfig.statisticMaxRt default */
typedef struct {
    leap second, minute;
    ladder threads;
    double count;
    size_t n;
    const uint8_t *kind;
    const int64_t *ts, *rt;
    int8_t *dec;
    int nthreads;
} hctx;

static void node_add(hctx *h, long long t, int ev, long long x) {
    leap_add(&h->second, t, ev, x, 0, MAX_RT);
    leap_add(&h->minute, t, ev, x, 0, MAX_RT);
}

static void node_rt(hctx *h, long long t, long long rt) { /* addRtAndSuccess: RT, SUCCESS, minRt (volatile) */
    leap *ls[2] = {&h->second, &h->minute};
    for (int k = 0; k < 2; k++) {
        int det;
        wwrap *w = current_window(ls[k], t, 0, MAX_RT, &det);
        la_add(&w->c[MB_RT], rt);
        la_add(&w->c[MB_SUCCESS], 1);
        if (rt < atomic_load_explicit(&w->min_rt, memory_order_relaxed)) atomic_store(&w->min_rt, rt);
        if (det) {
            for (int e = 0; e < EV_N_CLUSTER; e++) la_free(&w->c[e]);
            free(w);
        }
    }
}

static void *hello_worker(void *v) {
    targ *ta = (targ *)v;
    hctx *h = (hctx *)ta->ctx;
    t_probe = (uint32_t)mix64((uint64_t)ta->k + 7) | 1u;
    pthread_barrier_wait(ta->bar);
    for (size_t i = (size_t)ta->k; i < h->n; i += (size_t)h->nthreads) {
        const long long t = h->ts[i];
        if (h->kind[i] == 0) { /* entry: FlowSlot (DefaultController.canPass, QPS) then StatisticSlot */
            const double cur = (double)leap_sum(&h->second, t, MB_PASS, 0, MAX_RT) / h->second.isec;
            const int pass = !(cur + 1 > h->count);
            if (pass) {
                la_add(&h->threads, 1);
                node_add(h, t, MB_PASS, 1);
            } else {
                node_add(h, t, MB_BLOCK, 1);
            }
            if (h->dec) h->dec[i] = pass ? 0 : 1;
        } else { /* exit: StatisticSlot.exit */
            node_rt(h, t, h->rt[i]);
            la_add(&h->threads, -1);
        }
    }
    return NULL;
}

/* C1: one resource with a QPS FlowRule of `count` (DefaultController), entries (kind 0) and exits (kind 1)
 * of the trace over `nthreads` threads (event i on thread i mod nthreads). */
double orc_contended_hello(int nthreads, double count, size_t n, const uint8_t *kind, const int64_t *ts,
                           const int64_t *rt, int8_t *dec_out) {
    hctx h;
    memset(&h, 0, sizeof(h));
    leap_init(&h.second, 2, 1000);
    leap_init(&h.minute, 60, 60000);
    h.count = count;
    h.n = n;
    h.kind = kind;
    h.ts = ts;
    h.rt = rt;
    h.dec = dec_out;
    h.nthreads = nthreads < 1 ? 1 : nthreads;
    const double dt = run_threads(&h, h.nthreads, hello_worker);
    leap_free(&h.second);
    leap_free(&h.minute);
    la_free(&h.threads);
    return dt;
}
