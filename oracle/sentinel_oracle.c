/*
 * ORACLE / TEST INFRASTRUCTURE ONLY (see sentinel_oracle.h).  Single-threaded
 * C restatement of the reference hot path under a mocked clock.  Each function
 * cites the reference file:line it restates.  Multi-threaded LongAdder/CAS
 * behaviour collapses to plain integer arithmetic in a single-threaded replay
 * (LongAdder sums are order-independent; every CAS in the path succeeds).
 */
#include "oracle_internal.h"
#include "java_semantics.h"

#include <stdlib.h>
#include <string.h>


/* ========================================================================== */
/* LeapArray family                                                            */
/* ========================================================================== */



orc_leap *orc_leap_new(int kind, int sample_count, int interval_ms) {
    /* LeapArray.java:61-72 */
    if (sample_count <= 0 || interval_ms <= 0 || interval_ms % sample_count != 0) return NULL;
    orc_leap *l = (orc_leap *)calloc(1, sizeof(orc_leap));
    l->kind = kind;
    l->sample_count = sample_count;
    l->interval_ms = interval_ms;
    l->window_ms = interval_ms / sample_count;
    l->interval_sec = interval_ms / 1000.0;
    l->b = (obucket *)calloc((size_t)sample_count, sizeof(obucket));
    l->present = (uint8_t *)calloc((size_t)sample_count, 1);
    if (kind == ORC_LEAP_OCCUPIABLE) /* OccupiableBucketLeapArray.java:33-37 */
        l->borrow = orc_leap_new(ORC_LEAP_FUTURE, sample_count, interval_ms);
    return l;
}

void orc_leap_free(orc_leap *l) {
    if (!l) return;
    orc_leap_free(l->borrow);
    free(l->b);
    free(l->present);
    free(l);
}

static void bucket_zero(obucket *w) {
    memset(w->c, 0, sizeof(w->c));
    w->min_rt = ORC_STATISTIC_MAX_RT; /* MetricBucket.initMinRt, MetricBucket.java:56-58 */
}

static int leap_idx(const orc_leap *l, int64_t t) { /* LeapArray.java:105-109 */
    return (int)((t / l->window_ms) % l->sample_count);
}

static int leap_deprecated(const orc_leap *l, int64_t time, const obucket *w) {
    if (l->kind == ORC_LEAP_FUTURE) return time >= w->start; /* FutureBucketLeapArray.java:49-52 */
    return time - w->start > l->interval_ms;                 /* LeapArray.java:294-296 */
}

/* LeapArray.getWindowValue, LeapArray.java:265-278 */
static obucket *leap_window_value(orc_leap *l, int64_t t) {
    if (t < 0) return NULL;
    int idx = leap_idx(l, t);
    if (!l->present[idx]) return NULL;
    obucket *w = &l->b[idx];
    if (!(w->start <= t && t < w->start + l->window_ms)) return NULL; /* WindowWrap.isTimeInWindow */
    return w;
}

static void leap_new_empty(orc_leap *l, obucket *w, int64_t t) {
    bucket_zero(w);
    if (l->kind == ORC_LEAP_OCCUPIABLE) { /* OccupiableBucketLeapArray.newEmptyBucket, :40-48 */
        obucket *bb = leap_window_value(l->borrow, t);
        if (bb) { /* MetricBucket.reset(bucket), MetricBucket.java:47-54 */
            memcpy(w->c, bb->c, sizeof(w->c));
            w->min_rt = ORC_STATISTIC_MAX_RT;
        }
    }
}

static void leap_reset_to(orc_leap *l, obucket *w, int64_t start) {
    w->start = start;
    switch (l->kind) {
    case ORC_LEAP_OCCUPIABLE: { /* OccupiableBucketLeapArray.resetWindowTo, :50-64 */
        obucket *bb = leap_window_value(l->borrow, start);
        bucket_zero(w);
        if (bb) w->c[ORC_EV_PASS] += (int64_t)(int32_t)bb->c[ORC_EV_PASS]; /* addPass((int)borrow.pass()) */
        break;
    }
    case ORC_LEAP_CLUSTER: /* ClusterMetricLeapArray.resetWindowTo + transferOccupyToBucket, :48-71 */
        bucket_zero(w);
        if (l->has_occ) {
            w->c[ORC_CEV_OCCUPIED_PASS] += l->occ[ORC_CEV_PASS];
            w->c[ORC_CEV_PASS] += l->occ[ORC_CEV_PASS];
            l->occ[ORC_CEV_PASS] = 0;
            w->c[ORC_CEV_PASS_REQUEST] += l->occ[ORC_CEV_PASS_REQUEST];
            l->occ[ORC_CEV_PASS_REQUEST] = 0;
            l->has_occ = 0;
        }
        break;
    default: /* BucketLeapArray.java:40-46, FutureBucketLeapArray.java:40-46, UnaryLeapArray */
        bucket_zero(w);
        break;
    }
}

/* LeapArray.currentWindow(long), LeapArray.java:121-222 */
static obucket *leap_current(orc_leap *l, int64_t t) {
    if (t < 0) return NULL;
    int idx = leap_idx(l, t);
    int64_t ws = t - t % l->window_ms;
    if (!l->present[idx]) {
        leap_new_empty(l, &l->b[idx], t);
        l->b[idx].start = ws;
        l->present[idx] = 1;
        return &l->b[idx];
    }
    obucket *old = &l->b[idx];
    if (ws == old->start) return old;
    if (ws > old->start) {
        leap_reset_to(l, old, ws);
        return old;
    }
    /* clock went backwards: a detached bucket, adds are lost (:216-220) */
    leap_new_empty(l, &l->detached, t);
    l->detached.start = ws;
    return &l->detached;
}

int64_t orc_leap_current_window(orc_leap *l, int64_t t) {
    obucket *w = leap_current(l, t);
    return w ? w->start : INT64_MIN;
}

void orc_leap_add(orc_leap *l, int64_t t, int ev, int64_t n) {
    obucket *w = leap_current(l, t);
    if (w) w->c[ev] += n;
}

static void bucket_add_rt(obucket *w, int64_t rt) { /* MetricBucket.addRT, MetricBucket.java:130-137 */
    w->c[ORC_EV_RT] += rt;
    if (rt < w->min_rt) w->min_rt = rt;
}

void orc_leap_add_rt(orc_leap *l, int64_t t, int64_t rt) {
    obucket *w = leap_current(l, t);
    if (w) bucket_add_rt(w, rt);
}

int64_t orc_leap_current_get(orc_leap *l, int64_t t, int ev) {
    obucket *w = leap_current(l, t);
    return w ? w->c[ev] : 0;
}

/* LeapArray.values(long), LeapArray.java:358-373 */
int64_t orc_leap_values_sum(orc_leap *l, int64_t t, int ev, int *count) {
    int64_t s = 0;
    int n = 0;
    if (t >= 0) {
        for (int i = 0; i < l->sample_count; i++) {
            if (!l->present[i] || leap_deprecated(l, t, &l->b[i])) continue;
            s += l->b[i].c[ev];
            n++;
        }
    }
    if (count) *count = n;
    return s;
}

/* LeapArray.getPreviousWindow(long), LeapArray.java:230-248 (deprecation vs TimeUtil.now) */
static obucket *leap_previous(orc_leap *l, int64_t t, int64_t now) {
    if (t < 0) return NULL;
    int idx = leap_idx(l, t - l->window_ms);
    t = t - l->window_ms;
    if (!l->present[idx]) return NULL;
    obucket *w = &l->b[idx];
    if (leap_deprecated(l, now, w)) return NULL;
    if (w->start + l->window_ms < t) return NULL;
    return w;
}

int orc_leap_previous_window(orc_leap *l, int64_t t, int64_t now, int64_t *start, int64_t *pass) {
    obucket *w = leap_previous(l, t, now);
    if (!w) return 0;
    if (start) *start = w->start;
    if (pass) *pass = w->c[ORC_EV_PASS];
    return 1;
}

/* LeapArray.getValidHead, LeapArray.java:382-401 */
static obucket *leap_valid_head(orc_leap *l, int64_t now) {
    int idx = leap_idx(l, now + l->window_ms);
    if (!l->present[idx]) return NULL;
    obucket *w = &l->b[idx];
    if (leap_deprecated(l, now, w)) return NULL;
    return w;
}

int orc_leap_valid_head(orc_leap *l, int64_t now, int64_t *start, int64_t *pass) {
    obucket *w = leap_valid_head(l, now);
    if (!w) return 0;
    if (start) *start = w->start;
    if (pass) *pass = w->c[0];
    return 1;
}

/* OccupiableBucketLeapArray.addWaiting, :76-80 */
void orc_leap_add_waiting(orc_leap *l, int64_t t, int n) {
    obucket *w = leap_current(l->borrow, t);
    if (w) w->c[ORC_EV_PASS] += n;
}

/* OccupiableBucketLeapArray.currentWaiting, :66-74 */
int64_t orc_leap_current_waiting(orc_leap *l, int64_t now) {
    if (l->kind != ORC_LEAP_OCCUPIABLE) return 0; /* LeapArray.currentWaiting default */
    leap_current(l->borrow, now);
    return orc_leap_values_sum(l->borrow, now, ORC_EV_PASS, NULL);
}

int64_t orc_leap_window_value_pass(orc_leap *l, int64_t t) {
    obucket *w = leap_window_value(l, t);
    return w ? w->c[ORC_EV_PASS] : -1;
}

/* ========================================================================== */
/* ArrayMetric / StatisticNode                                                  */
/* ========================================================================== */


orc_node *orc_node_new(void) {
    orc_node *n = (orc_node *)calloc(1, sizeof(orc_node));
    n->second = orc_leap_new(ORC_LEAP_OCCUPIABLE, ORC_SAMPLE_COUNT, ORC_INTERVAL);
    n->minute = orc_leap_new(ORC_LEAP_BUCKET, 60, 60 * 1000);
    n->last_fetch = -1;
    return n;
}

/* StatisticNode.metrics() (StatisticNode.java:120-157) over ArrayMetric.details() (ArrayMetric.java:166-218)
 * and LeapArray.list(now) (LeapArray.java:304-326). */
size_t orc_node_metrics(orc_node *n, int64_t now, uint32_t resource, orc_metric_node *out, size_t cap) {
    const int64_t current = now - now % 1000;
    orc_leap *m = n->minute;
    orc_leap_current_window(m, now); /* data.currentWindow() */
    int64_t newlast = n->last_fetch;
    size_t k = 0;
    for (int j = 0; j < m->sample_count; j++) {
        if (!m->present[j]) continue;
        const obucket *b = &m->b[j];
        if (now - b->start > m->interval_ms) continue; /* isWindowDeprecated */
        orc_metric_node x;
        memset(&x, 0, sizeof(x));
        x.timestamp = b->start;
        x.pass_qps = b->c[ORC_EV_PASS];
        x.block_qps = b->c[ORC_EV_BLOCK];
        x.success_qps = b->c[ORC_EV_SUCCESS];
        x.exception_qps = b->c[ORC_EV_EXCEPTION];
        x.rt = x.success_qps != 0 ? b->c[ORC_EV_RT] / x.success_qps : b->c[ORC_EV_RT];
        x.occupied_pass_qps = b->c[ORC_EV_OCCUPIED_PASS];
        x.resource = resource;
        const int in_time = x.timestamp > n->last_fetch && x.timestamp < current;
        const int valid = x.pass_qps > 0 || x.block_qps > 0 || x.success_qps > 0 || x.exception_qps > 0 ||
                          x.rt > 0 || x.occupied_pass_qps > 0;
        if (in_time && valid) {
            if (k < cap) out[k] = x;
            k++;
            if (x.timestamp > newlast) newlast = x.timestamp;
        }
    }
    n->last_fetch = newlast;
    return k;
}

/* MetricTimerListener.run over every resource's ClusterNode (MetricTimerListener.java:44-65) */
size_t orc_flow_metrics(orc_flow *f, int64_t now, orc_metric_node *out, size_t cap) {
    size_t k = 0;
    for (uint32_t r = 0; r < f->n; r++) {
        if (!f->res[r].node) continue;
        k += orc_node_metrics(f->res[r].node, now, r, out ? out + (k < cap ? k : cap) : NULL, k < cap ? cap - k : 0);
    }
    /* MetricTimerListener.run aggregates Constants.ENTRY_NODE after the cluster nodes (:56) */
    k += orc_node_metrics(f->entry, now, ORC_ENTRY_NODE, out ? out + (k < cap ? k : cap) : NULL, k < cap ? cap - k : 0);
    return k;
}

orc_node *orc_node_new_mock(double pass_qps, double previous_pass_qps, int32_t threads) {
    orc_node *n = orc_node_new();
    orc_node_set_mock(n, pass_qps, previous_pass_qps, threads);
    return n;
}

void orc_node_set_mock(orc_node *n, double pass_qps, double previous_pass_qps, int32_t threads) {
    n->mock = 1;
    n->mock_pass_qps = pass_qps;
    n->mock_prev_pass_qps = previous_pass_qps;
    n->mock_threads = threads;
}

void orc_node_free(orc_node *n) {
    if (!n) return;
    orc_leap_free(n->second);
    orc_leap_free(n->minute);
    free(n);
}

/* ArrayMetric.<counter>(): data.currentWindow() then sum values(), ArrayMetric.java:62-70 etc */
static int64_t am_sum(orc_leap *l, int64_t now, int ev) {
    leap_current(l, now);
    return orc_leap_values_sum(l, now, ev, NULL);
}

double orc_node_pass_qps(orc_node *n, int64_t now) { /* StatisticNode.java:210-212 */
    if (n->mock) return n->mock_pass_qps;
    return (double)am_sum(n->second, now, ORC_EV_PASS) / n->second->interval_sec;
}
double orc_node_block_qps(orc_node *n, int64_t now) {
    return (double)am_sum(n->second, now, ORC_EV_BLOCK) / n->second->interval_sec;
}
double orc_node_success_qps(orc_node *n, int64_t now) {
    return (double)am_sum(n->second, now, ORC_EV_SUCCESS) / n->second->interval_sec;
}
double orc_node_exception_qps(orc_node *n, int64_t now) {
    return (double)am_sum(n->second, now, ORC_EV_EXCEPTION) / n->second->interval_sec;
}
double orc_node_occupied_pass_qps(orc_node *n, int64_t now) {
    return (double)am_sum(n->second, now, ORC_EV_OCCUPIED_PASS) / n->second->interval_sec;
}
/* StatisticNode.previousPassQps -> ArrayMetric.previousWindowPass, ArrayMetric.java:283-290 */
double orc_node_previous_pass_qps(orc_node *n, int64_t now) {
    if (n->mock) return n->mock_prev_pass_qps;
    leap_current(n->minute, now);
    obucket *w = leap_previous(n->minute, now, now);
    return w ? (double)w->c[ORC_EV_PASS] : 0.0;
}
/* StatisticNode.previousBlockQps -> ArrayMetric.previousWindowBlock, StatisticNode.java:180-182,
 * ArrayMetric.java:273-280 */
double orc_node_previous_block_qps(orc_node *n, int64_t now) {
    leap_current(n->minute, now);
    obucket *w = leap_previous(n->minute, now, now);
    return w ? (double)w->c[ORC_EV_BLOCK] : 0.0;
}
/* StatisticNode.avgRt, StatisticNode.java:238-245 */
double orc_node_avg_rt(orc_node *n, int64_t now) {
    int64_t success = am_sum(n->second, now, ORC_EV_SUCCESS);
    if (success == 0) return 0;
    return (double)am_sum(n->second, now, ORC_EV_RT) * 1.0 / (double)success;
}
/* ArrayMetric.minRt, ArrayMetric.java:152-163 */
double orc_node_min_rt(orc_node *n, int64_t now) {
    orc_leap *l = n->second;
    leap_current(l, now);
    int64_t rt = ORC_STATISTIC_MAX_RT;
    for (int i = 0; i < l->sample_count; i++) {
        if (!l->present[i] || leap_deprecated(l, now, &l->b[i])) continue;
        if (l->b[i].min_rt < rt) rt = l->b[i].min_rt;
    }
    return (double)(rt < 1 ? 1 : rt);
}
/* StatisticNode.maxSuccessQps = ArrayMetric.maxSuccess() * sampleCount / intervalInSec,
 * StatisticNode.java:225-230, ArrayMetric.java:82-93 */
double orc_node_max_success_qps(orc_node *n, int64_t now) {
    orc_leap *l = n->second;
    leap_current(l, now);
    int64_t s = 0;
    for (int i = 0; i < l->sample_count; i++) {
        if (!l->present[i] || leap_deprecated(l, now, &l->b[i])) continue;
        if (l->b[i].c[ORC_EV_SUCCESS] > s) s = l->b[i].c[ORC_EV_SUCCESS];
    }
    if (s < 1) s = 1;
    return (double)s * (double)l->sample_count / l->interval_sec;
}
int64_t orc_node_total_pass(orc_node *n, int64_t now) { return am_sum(n->minute, now, ORC_EV_PASS); }
int64_t orc_node_total_block(orc_node *n, int64_t now) { return am_sum(n->minute, now, ORC_EV_BLOCK); }
int64_t orc_node_total_success(orc_node *n, int64_t now) { return am_sum(n->minute, now, ORC_EV_SUCCESS); }
int64_t orc_node_total_exception(orc_node *n, int64_t now) { return am_sum(n->minute, now, ORC_EV_EXCEPTION); }
int32_t orc_node_cur_thread_num(orc_node *n) {
    if (n->mock) return n->mock_threads;
    return (int32_t)n->threads; /* (int)curThreadNum.sum(), StatisticNode.java:248-250 */
}
int64_t orc_node_waiting(orc_node *n, int64_t now) { return orc_leap_current_waiting(n->second, now); }

/* StatisticNode.addPassRequest, :260-263 */
void orc_node_add_pass_request(orc_node *n, int64_t now, int count) {
    orc_leap_add(n->second, now, ORC_EV_PASS, count);
    orc_leap_add(n->minute, now, ORC_EV_PASS, count);
}
/* StatisticNode.addRtAndSuccess, :266-272 */
void orc_node_add_rt_and_success(orc_node *n, int64_t now, int64_t rt, int count) {
    orc_leap_add(n->second, now, ORC_EV_SUCCESS, count);
    orc_leap_add_rt(n->second, now, rt);
    orc_leap_add(n->minute, now, ORC_EV_SUCCESS, count);
    orc_leap_add_rt(n->minute, now, rt);
}
void orc_node_increase_block_qps(orc_node *n, int64_t now, int count) { /* :275-278 */
    orc_leap_add(n->second, now, ORC_EV_BLOCK, count);
    orc_leap_add(n->minute, now, ORC_EV_BLOCK, count);
}
void orc_node_increase_exception_qps(orc_node *n, int64_t now, int count) { /* :281-284 */
    orc_leap_add(n->second, now, ORC_EV_EXCEPTION, count);
    orc_leap_add(n->minute, now, ORC_EV_EXCEPTION, count);
}
void orc_node_increase_thread_num(orc_node *n) { n->threads++; }
void orc_node_decrease_thread_num(orc_node *n) { n->threads--; }

/* StatisticNode.tryOccupyNext, StatisticNode.java:302-334 */
int64_t orc_node_try_occupy_next(orc_node *n, int64_t now, int acquire, double threshold) {
    double max_count = threshold * ORC_INTERVAL / 1000;
    int64_t current_borrow = orc_leap_current_waiting(n->second, now);
    if ((double)current_borrow >= max_count) return ORC_OCCUPY_TIMEOUT;
    int window_length = ORC_INTERVAL / ORC_SAMPLE_COUNT;
    int64_t earliest = now - now % window_length + window_length - ORC_INTERVAL;
    int idx = 0;
    int64_t current_pass = am_sum(n->second, now, ORC_EV_PASS);
    while (earliest < now) {
        int64_t wait = (int64_t)idx * window_length + window_length - now % window_length;
        if (wait >= ORC_OCCUPY_TIMEOUT) break;
        obucket *w = leap_window_value(n->second, earliest); /* ArrayMetric.getWindowPass */
        int64_t window_pass = w ? w->c[ORC_EV_PASS] : 0;
        if ((double)(current_pass + current_borrow + acquire - window_pass) <= max_count) return wait;
        earliest += window_length;
        current_pass -= window_pass;
        idx++;
    }
    return ORC_OCCUPY_TIMEOUT;
}

/* StatisticNode.addWaitingRequest, :342-345 */
void orc_node_add_waiting_request(orc_node *n, int64_t future_time, int acquire) {
    orc_leap_add_waiting(n->second, future_time, acquire);
}
/* StatisticNode.addOccupiedPass, :347-350 */
void orc_node_add_occupied_pass(orc_node *n, int64_t now, int acquire) {
    orc_leap_add(n->minute, now, ORC_EV_OCCUPIED_PASS, acquire);
    orc_leap_add(n->minute, now, ORC_EV_PASS, acquire);
}

/* ========================================================================== */
/* Traffic shaping controllers                                                  */
/* ========================================================================== */


/* WarmUpController.construct, WarmUpController.java:83-106 */
static void warmup_construct(orc_ctrl *c, double count, int period, int cold_factor) {
    c->count = count;
    c->cold_factor = cold_factor;
    c->warning_token = j_d2i((double)period * count) / (cold_factor - 1);
    c->max_token = c->warning_token + j_d2i(2 * period * count / (1.0 + cold_factor));
    c->slope = (cold_factor - 1.0) / count / (double)(c->max_token - c->warning_token);
    c->stored_tokens = 0;
    c->last_filled_time = 0;
}

orc_ctrl *orc_ctrl_new(int behavior, int grade, double count, int warm_up_period_sec, int max_queueing_time_ms,
                       int cold_factor) {
    orc_ctrl *c = (orc_ctrl *)calloc(1, sizeof(orc_ctrl));
    /* FlowRuleUtil.generateRater, FlowRuleUtil.java:141-162: non-QPS grades get DefaultController */
    c->behavior = grade == ORC_GRADE_QPS ? behavior : ORC_CTRL_DEFAULT;
    if (c->behavior < 0 || c->behavior > 3) c->behavior = ORC_CTRL_DEFAULT;
    c->grade = grade;
    c->count = count;
    c->max_queueing_time_ms = max_queueing_time_ms;
    c->latest_passed_time = -1;
    if (c->behavior == ORC_CTRL_WARM_UP || c->behavior == ORC_CTRL_WARM_UP_RATE_LIMITER)
        warmup_construct(c, count, warm_up_period_sec, cold_factor);
    return c;
}

void orc_ctrl_free(orc_ctrl *c) { free(c); }

/* WarmUpController.coolDownTokens, WarmUpController.java:161-175 */
static int64_t warmup_cool_down(orc_ctrl *c, int64_t current_time, int64_t pass_qps) {
    int64_t old_value = c->stored_tokens;
    int64_t new_value = old_value;
    if (old_value < c->warning_token) {
        new_value = j_d2l((double)old_value + (double)(current_time - c->last_filled_time) * c->count / 1000);
    } else if (old_value > c->warning_token) {
        if (pass_qps < (int64_t)(j_d2i(c->count) / c->cold_factor)) {
            new_value = j_d2l((double)old_value + (double)(current_time - c->last_filled_time) * c->count / 1000);
        }
    }
    return new_value < (int64_t)c->max_token ? new_value : (int64_t)c->max_token;
}

/* WarmUpController.syncToken, WarmUpController.java:140-159 */
static void warmup_sync(orc_ctrl *c, int64_t now, int64_t pass_qps) {
    int64_t current_time = now - now % 1000;
    if (current_time <= c->last_filled_time) return;
    int64_t new_value = warmup_cool_down(c, current_time, pass_qps);
    c->stored_tokens = new_value;
    c->stored_tokens -= pass_qps;
    if (c->stored_tokens < 0) c->stored_tokens = 0;
    c->last_filled_time = current_time;
}

/* queueing tail shared by RateLimiterController.java:62-90 and
 * WarmUpRateLimiterController.java:61-86 (single-threaded: the re-check after
 * addAndGet never fails). */
static int pace_tail(orc_ctrl *c, int64_t now, int64_t cost, int64_t *wait_ms) {
    int64_t expected = cost + c->latest_passed_time;
    if (expected <= now) {
        c->latest_passed_time = now;
        *wait_ms = 0;
        return ORC_PASS;
    }
    int64_t wait = cost + c->latest_passed_time - now;
    if (wait > c->max_queueing_time_ms) return ORC_BLOCK_FLOW;
    c->latest_passed_time += cost;
    wait = c->latest_passed_time - now;
    if (wait > c->max_queueing_time_ms) { /* unreachable single-threaded, kept for fidelity */
        c->latest_passed_time -= cost;
        return ORC_BLOCK_FLOW;
    }
    *wait_ms = wait > 0 ? wait : 0;
    return ORC_PASS;
}

int orc_ctrl_can_pass(orc_ctrl *c, orc_node *node, int64_t now, int acquire, int prioritized, int64_t *wait_ms) {
    int64_t dummy;
    if (!wait_ms) wait_ms = &dummy;
    *wait_ms = 0;
    switch (c->behavior) {
    case ORC_CTRL_RATE_LIMITER: { /* RateLimiterController.canPass, :46-91 */
        if (acquire <= 0) return ORC_PASS;
        if (c->count <= 0) return ORC_BLOCK_FLOW;
        int64_t cost = j_round(1.0 * acquire / c->count * 1000);
        return pace_tail(c, now, cost, wait_ms);
    }
    case ORC_CTRL_WARM_UP: { /* WarmUpController.canPass, :113-138 */
        int64_t pass_qps = j_d2l(orc_node_pass_qps(node, now));
        int64_t previous_qps = j_d2l(orc_node_previous_pass_qps(node, now));
        warmup_sync(c, now, previous_qps);
        int64_t rest = c->stored_tokens;
        if (rest >= c->warning_token) {
            int64_t above = rest - c->warning_token;
            double warning_qps = j_next_up(1.0 / ((double)above * c->slope + 1.0 / c->count));
            if ((double)(pass_qps + acquire) <= warning_qps) return ORC_PASS;
        } else {
            if ((double)(pass_qps + acquire) <= c->count) return ORC_PASS;
        }
        return ORC_BLOCK_FLOW;
    }
    case ORC_CTRL_WARM_UP_RATE_LIMITER: { /* WarmUpRateLimiterController.canPass, :43-87 */
        int64_t previous_qps = j_d2l(orc_node_previous_pass_qps(node, now));
        warmup_sync(c, now, previous_qps);
        int64_t rest = c->stored_tokens;
        int64_t cost;
        if (rest >= c->warning_token) {
            int64_t above = rest - c->warning_token;
            double warming_qps = j_next_up(1.0 / ((double)above * c->slope + 1.0 / c->count));
            cost = j_round(1.0 * acquire / warming_qps * 1000);
        } else {
            cost = j_round(1.0 * acquire / c->count * 1000);
        }
        return pace_tail(c, now, cost, wait_ms);
    }
    default: { /* DefaultController.canPass, DefaultController.java:49-78 */
        int32_t cur;
        if (!node) cur = 0;
        else if (c->grade == ORC_GRADE_THREAD) cur = orc_node_cur_thread_num(node);
        else cur = j_d2i(orc_node_pass_qps(node, now));
        int32_t sum = (int32_t)((uint32_t)cur + (uint32_t)acquire); /* int + int wraps */
        if ((double)sum > c->count) {
            if (prioritized && c->grade == ORC_GRADE_QPS && node && !node->mock) {
                int64_t wait = orc_node_try_occupy_next(node, now, acquire, c->count);
                if (wait < ORC_OCCUPY_TIMEOUT) {
                    orc_node_add_waiting_request(node, now + wait, acquire);
                    orc_node_add_occupied_pass(node, now, acquire);
                    *wait_ms = wait;
                    return ORC_PASS_WAIT; /* PriorityWaitException */
                }
            }
            return ORC_BLOCK_FLOW;
        }
        return ORC_PASS;
    }
    }
}

int64_t orc_ctrl_latest_passed_time(const orc_ctrl *c) { return c->latest_passed_time; }
int64_t orc_ctrl_stored_tokens(const orc_ctrl *c) { return c->stored_tokens; }
int64_t orc_ctrl_last_filled_time(const orc_ctrl *c) { return c->last_filled_time; }
int32_t orc_ctrl_warning_token(const orc_ctrl *c) { return c->warning_token; }
int32_t orc_ctrl_max_token(const orc_ctrl *c) { return c->max_token; }
double orc_ctrl_slope(const orc_ctrl *c) { return c->slope; }

/* ========================================================================== */
/* Local flow engine: StatisticSlot + FlowSlot (single default context)         */
/* ========================================================================== */



orc_flow *orc_flow_new(uint32_t n_resources, int cold_factor) {
    orc_flow *f = (orc_flow *)calloc(1, sizeof(orc_flow));
    f->n = n_resources;
    f->cold_factor = cold_factor > 1 ? cold_factor : 3; /* SentinelConfig.coldFactor, :224-238 */
    f->res = (flow_res *)calloc(n_resources, sizeof(flow_res));
    for (uint32_t i = 0; i < n_resources; i++) f->res[i].node = orc_node_new();
    f->entry = orc_node_new();
    orc_flow_system_restore(f);
    f->sys.cur_load = -1;
    f->sys.cur_cpu = -1;
    return f;
}

void orc_flow_free(orc_flow *f) {
    if (!f) return;
    for (uint32_t i = 0; i < f->n; i++) {
        for (int k = 0; k < f->res[i].nctrl; k++) orc_ctrl_free(f->res[i].ctrl[k]);
        free(f->res[i].ctrl);
        free(f->res[i].cmode);
        free(f->res[i].cfallback);
        free(f->res[i].cflow);
        orc_node_free(f->res[i].node);
        orc_flow_res_free_ext(&f->res[i]);
    }
    free(f->res);
    orc_node_free(f->entry);
    free(f);
}

/* FlowRuleUtil.isValidRule (local, non-cluster), FlowRuleUtil.java:176-235 */
static int flow_rule_valid(const orc_flow_rule *r) {
    if (!(r->count >= 0 && r->grade >= 0 && r->strategy >= 0 && r->control_behavior >= 0)) return 0;
    if (r->cluster_mode) { /* FlowRuleUtil.checkClusterField / checkClusterConcurrentField, :197-240 */
        if (r->cluster_flow_id <= 0) return 0;                                   /* validClusterRuleId */
        if (!(r->cluster_sample_count > 0 && r->cluster_window_ms > 0 &&
              r->cluster_window_ms % r->cluster_sample_count == 0)) return 0;      /* isWindowConfigValid */
        if (r->grade == ORC_GRADE_QPS && r->cluster_strategy != 0) return 0;      /* NORMAL only */
    }
    if (r->grade == ORC_GRADE_QPS) {
        if (r->strategy != 0) return 0; /* engine supports DIRECT only (RELATE/CHAIN need refResource) */
        switch (r->control_behavior) {
        case ORC_CTRL_WARM_UP: return r->warm_up_period_sec > 0;
        case ORC_CTRL_RATE_LIMITER: return r->max_queueing_time_ms > 0;
        case ORC_CTRL_WARM_UP_RATE_LIMITER: return r->warm_up_period_sec > 0 && r->max_queueing_time_ms > 0;
        default: return 1;
        }
    }
    if (r->grade == ORC_GRADE_THREAD) return r->strategy == 0;
    return 0;
}

/* FlowRuleManager.loadRules -> FlowRuleUtil.buildFlowRuleMap, FlowRuleUtil.java:84-135.
 * Rules keep their input order per resource (all local, limitApp default: the
 * FlowRuleComparator sees them as equal and Collections.sort is stable). */
int orc_flow_load_rules(orc_flow *f, const orc_flow_rule *rules, size_t n) {
    for (uint32_t i = 0; i < f->n; i++) {
        for (int k = 0; k < f->res[i].nctrl; k++) orc_ctrl_free(f->res[i].ctrl[k]);
        free(f->res[i].ctrl);
        free(f->res[i].cmode);
        free(f->res[i].cfallback);
        free(f->res[i].cflow);
        f->res[i].ctrl = NULL;
        f->res[i].cmode = f->res[i].cfallback = NULL;
        f->res[i].cflow = NULL;
        f->res[i].nctrl = 0;
    }
    int valid = 0;
    for (size_t j = 0; j < n; j++) {
        const orc_flow_rule *r = &rules[j];
        if (r->resource >= f->n || !flow_rule_valid(r)) continue;
        flow_res *fr = &f->res[r->resource];
        fr->ctrl = (orc_ctrl **)realloc(fr->ctrl, sizeof(orc_ctrl *) * (size_t)(fr->nctrl + 1));
        fr->cmode = (int32_t *)realloc(fr->cmode, sizeof(int32_t) * (size_t)(fr->nctrl + 1));
        fr->cfallback = (int32_t *)realloc(fr->cfallback, sizeof(int32_t) * (size_t)(fr->nctrl + 1));
        fr->cflow = (int64_t *)realloc(fr->cflow, sizeof(int64_t) * (size_t)(fr->nctrl + 1));
        fr->cmode[fr->nctrl] = r->cluster_mode ? 1 : 0;
        fr->cfallback[fr->nctrl] = r->cluster_fallback ? 1 : 0;
        fr->cflow[fr->nctrl] = r->cluster_flow_id;
        fr->ctrl[fr->nctrl++] = orc_ctrl_new(r->control_behavior, r->grade, r->count, r->warm_up_period_sec,
                                             r->max_queueing_time_ms, f->cold_factor);
        valid++;
    }
    return valid;
}

orc_node *orc_flow_node(orc_flow *f, uint32_t resource) { return resource < f->n ? f->res[resource].node : NULL; }

void orc_flow_set_cluster(orc_flow *f, orc_cluster *server, int mode) {
    f->server = server;
    f->cluster_mode = mode;
}

/* FlowSlot.checkFlow (FlowSlot.java:161-172, FlowRuleChecker.java:44-60; DIRECT +
 * default limitApp selects the ClusterNode, FlowRuleChecker.java:118-166):
 * the resource's raters in order; ORC_PASS (with accumulated sleeps),
 * ORC_BLOCK_FLOW or ORC_PASS_WAIT (PriorityWaitException). No statistics. */
int orc_flow_rule_check(orc_flow *f, uint32_t resource, int64_t now, int acquire, int prioritized, int64_t *wait_ms) {
    flow_res *fr = &f->res[resource];
    int64_t total_wait = 0;
    *wait_ms = 0;
    for (int k = 0; k < fr->nctrl; k++) {
        int64_t w = 0;
        if (fr->cmode && fr->cmode[k]) {
            /* FlowRuleChecker.passClusterCheck (:168-188): pickClusterService -> requestToken ->
             * applyTokenResult (:203-230); no service -> fallbackToLocalOrPass (:190-198) */
            int status = -1; /* TokenResultStatus.FAIL stands for "no service" (both fall back) */
            int32_t tw = 0;
            if (f->server && f->cluster_mode == 1) {
                const orc_token_result r = orc_cluster_request_token(f->server, fr->cflow[k], acquire, prioritized, now);
                status = r.status;
                tw = r.wait_in_ms;
            }
            if (status == 0) continue;                      /* OK */
            if (status == 2) { total_wait += tw; continue; } /* SHOULD_WAIT: sleep, then pass */
            if (status == 1) { *wait_ms = k; return ORC_BLOCK_FLOW; } /* BLOCKED (block detail: rule index) */
            if (status != 3 && status != -4 && status != -1 && status != -2) { *wait_ms = k; return ORC_BLOCK_FLOW; }
            if (!fr->cfallback[k]) continue;                /* fallbackToLocalOrPass: pass */
        }
        int d = orc_ctrl_can_pass(fr->ctrl[k], fr->node, now, acquire, prioritized, &w);
        if (d == ORC_BLOCK_FLOW) {
            *wait_ms = k; /* block detail: the rule's index in FlowRuleComparator order */
            return ORC_BLOCK_FLOW;
        }
        if (d == ORC_PASS_WAIT) {
            *wait_ms = w;
            return ORC_PASS_WAIT;
        }
        total_wait += w;
    }
    *wait_ms = total_wait;
    return ORC_PASS;
}

int orc_flow_entry(orc_flow *f, uint32_t resource, int64_t now, int acquire, int prioritized, int64_t *wait_ms) {
    return orc_flow_entry_p(f, resource, now, acquire, prioritized, 0, 0, wait_ms);
}

void orc_flow_exit(orc_flow *f, uint32_t resource, int64_t now, int64_t rt, int count, int error) {
    orc_flow_exit_p(f, resource, now, rt, count, error, 0, 0);
}

void orc_flow_replay(orc_flow *f, size_t n, const uint8_t *kind, const uint32_t *resource, const int64_t *ts,
                     const int32_t *acquire, const uint8_t *flags, const int64_t *rt, int8_t *decision,
                     int32_t *wait_ms) {
    for (size_t i = 0; i < n; i++) {
        if (kind && kind[i] == 1) {
            orc_flow_exit(f, resource[i], ts[i], rt ? rt[i] : 0, acquire[i], flags ? (flags[i] & 2) != 0 : 0);
            if (decision) decision[i] = ORC_PASS;
            if (wait_ms) wait_ms[i] = 0;
            continue;
        }
        int64_t w = 0;
        int d = orc_flow_entry(f, resource[i], ts[i], acquire[i], flags ? (flags[i] & 1) : 0, &w);
        if (decision) decision[i] = (int8_t)d;
        if (wait_ms) wait_ms[i] = (int32_t)w;
    }
}

/* ========================================================================== */
/* Cluster token server                                                         */
/* ========================================================================== */

/* TokenResultStatus, CORE/cluster/TokenResultStatus.java:27-60 */
enum { TRS_BAD_REQUEST = -4, TRS_TOO_MANY_REQUEST = -2, TRS_FAIL = -1, TRS_OK = 0, TRS_BLOCKED = 1,
       TRS_SHOULD_WAIT = 2, TRS_NO_RULE_EXISTS = 3 };

struct orc_cmetric {
    orc_leap *l; /* ClusterMetric.metric (ClusterMetricLeapArray) */
};

orc_cmetric *orc_cmetric_new(int sample_count, int interval_ms) { /* ClusterMetric.java:32-37 */
    orc_leap *l = orc_leap_new(ORC_LEAP_CLUSTER, sample_count, interval_ms);
    if (!l) return NULL;
    orc_cmetric *m = (orc_cmetric *)calloc(1, sizeof(orc_cmetric));
    m->l = l;
    return m;
}
void orc_cmetric_free(orc_cmetric *m) {
    if (!m) return;
    orc_leap_free(m->l);
    free(m);
}
void orc_cmetric_add(orc_cmetric *m, int64_t now, int ev, int64_t n) { orc_leap_add(m->l, now, ev, n); } /* :39-41 */
int64_t orc_cmetric_sum(orc_cmetric *m, int64_t now, int ev) { return am_sum(m->l, now, ev); }         /* :53-62 */
double orc_cmetric_avg(orc_cmetric *m, int64_t now, int ev) {                                         /* :70-72 */
    return (double)orc_cmetric_sum(m, now, ev) / m->l->interval_sec;
}
/* ClusterMetric.tryOccupyNext + canOccupy, ClusterMetric.java:79-98;
 * ClusterMetricLeapArray.addOccupyPass/getOccupiedCount/getFirstCountOfWindow, :73-92 */
int32_t orc_cmetric_try_occupy_next(orc_cmetric *m, int64_t now, int ev, int32_t acquire, double threshold) {
    double latest = orc_cmetric_avg(m, now, ORC_CEV_PASS);
    obucket *head = leap_valid_head(m->l, now);
    int64_t head_pass = head ? head->c[ev] : 0;
    int64_t occupied = m->l->occ[ev];
    if (!(latest + (double)((int64_t)acquire + occupied) - (double)head_pass <= threshold)) return 0;
    m->l->occ[ORC_CEV_PASS] += acquire;
    m->l->occ[ORC_CEV_PASS_REQUEST] += 1;
    m->l->has_occ = 1;
    orc_cmetric_add(m, now, ORC_CEV_WAITING, acquire);
    return 1000 / m->l->sample_count;
}

struct orc_limiter { /* RequestLimiter.java:29-87 over UnaryLeapArray(10, 1000) */
    double qps_allowed;
    orc_leap *l;
};
orc_limiter *orc_limiter_new(double qps_allowed) {
    orc_limiter *r = (orc_limiter *)calloc(1, sizeof(orc_limiter));
    r->qps_allowed = qps_allowed;
    r->l = orc_leap_new(ORC_LEAP_UNARY, 10, 1000);
    return r;
}
void orc_limiter_free(orc_limiter *r) {
    if (!r) return;
    orc_leap_free(r->l);
    free(r);
}
void orc_limiter_add(orc_limiter *r, int64_t now, int x) { orc_leap_add(r->l, now, 0, x); }
int64_t orc_limiter_sum(orc_limiter *r, int64_t now) { return am_sum(r->l, now, 0); }
double orc_limiter_qps(orc_limiter *r, int64_t now) { return (double)orc_limiter_sum(r, now) / r->l->interval_sec; }
int orc_limiter_can_pass(orc_limiter *r, int64_t now) { return orc_limiter_qps(r, now) + 1 <= r->qps_allowed; }
int orc_limiter_try_pass(orc_limiter *r, int64_t now) {
    if (orc_limiter_can_pass(r, now)) {
        orc_limiter_add(r, now, 1);
        return 1;
    }
    return 0;
}

/* --- flowId -> rule map (ClusterFlowRuleManager FLOW_RULES / metrics) ------- */
typedef struct crule {
    int64_t flow_id;
    orc_cluster_rule r;
    int ns;               /* namespace index */
    int active;           /* in FLOW_RULES */
    orc_cmetric *metric;  /* ClusterMetricStatistics entry (may outlive the rule) */
    int conc_live;        /* CurrentConcurrencyManager NOW_CALLS_MAP holds flow_id */
    int32_t now_calls;    /* its AtomicInteger */
} crule;

#define ORC_MAX_NS 64
struct orc_cluster {
    double exceed_count, max_occupy_ratio;
    crule *tab;
    size_t cap, used;
    struct orc_cparam *param;  /* ClusterParamFlowRuleManager state (oracle_cparam.c) */
    struct orc_conc *conc;     /* TokenCacheNodeManager state (oracle_conc.c) */
    char *ns_name[ORC_MAX_NS];
    int32_t ns_connected[ORC_MAX_NS];
    orc_limiter *ns_limiter[ORC_MAX_NS];
    int nns;
};

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static crule *ctab_find(orc_cluster *c, int64_t id, int create) {
    if (c->cap == 0 || (create && (c->used + 1) * 2 > c->cap)) {
        size_t ncap = c->cap ? c->cap * 2 : 1024;
        crule *nt = (crule *)calloc(ncap, sizeof(crule));
        for (size_t i = 0; i < c->cap; i++) {
            if (c->tab[i].flow_id == 0) continue;
            size_t h = mix64((uint64_t)c->tab[i].flow_id) & (ncap - 1);
            while (nt[h].flow_id != 0) h = (h + 1) & (ncap - 1);
            nt[h] = c->tab[i];
        }
        free(c->tab);
        c->tab = nt;
        c->cap = ncap;
    }
    size_t h = mix64((uint64_t)id) & (c->cap - 1);
    while (c->tab[h].flow_id != 0) {
        if (c->tab[h].flow_id == id) return &c->tab[h];
        h = (h + 1) & (c->cap - 1);
    }
    if (!create) return NULL;
    memset(&c->tab[h], 0, sizeof(crule));
    c->tab[h].flow_id = id;
    c->tab[h].ns = -1;
    c->used++;
    return &c->tab[h];
}

orc_cluster *orc_cluster_new(double exceed_count, double max_occupy_ratio) {
    orc_cluster *c = (orc_cluster *)calloc(1, sizeof(orc_cluster));
    c->exceed_count = exceed_count;   /* ServerFlowConfig.DEFAULT_EXCEED_COUNT = 1.0 */
    c->max_occupy_ratio = max_occupy_ratio; /* ServerFlowConfig.DEFAULT_MAX_OCCUPY_RATIO = 1.0 */
    return c;
}

void orc_cparam_free_all(orc_cluster *c);
void orc_conc_free_all(orc_cluster *c);
void orc_cluster_free(orc_cluster *c) {
    if (!c) return;
    orc_cparam_free_all(c);
    orc_conc_free_all(c);
    for (size_t i = 0; i < c->cap; i++) orc_cmetric_free(c->tab[i].metric);
    free(c->tab);
    for (int i = 0; i < c->nns; i++) {
        free(c->ns_name[i]);
        orc_limiter_free(c->ns_limiter[i]);
    }
    free(c);
}

int orc_cluster_ns_index(orc_cluster *c, const char *ns, int create);
static int ns_index(orc_cluster *c, const char *ns, int create) { return orc_cluster_ns_index(c, ns, create); }
int orc_cluster_ns_index(orc_cluster *c, const char *ns, int create) {
    for (int i = 0; i < c->nns; i++)
        if (strcmp(c->ns_name[i], ns) == 0) return i;
    if (!create || c->nns >= ORC_MAX_NS) return -1;
    c->ns_name[c->nns] = strdup(ns);
    c->ns_connected[c->nns] = 0;
    return c->nns++;
}

/* ClusterFlowRuleManager.applyClusterFlowRule, ClusterFlowRuleManager.java:310-364 */
int orc_cluster_load_rules(orc_cluster *c, const char *ns, const orc_cluster_rule *rules, size_t n) {
    int nsi = ns_index(c, ns, 1);
    if (nsi < 0) return -1;
    if (n == 0) { /* clearAndResetRulesFor (:281-296): rules dropped, metrics kept */
        for (size_t i = 0; i < c->cap; i++)
            if (c->tab[i].flow_id != 0 && c->tab[i].ns == nsi) {
                c->tab[i].active = 0;
                c->tab[i].conc_live = 0; /* CurrentConcurrencyManager.remove(flowId) */
            }
        return 0;
    }
    /* mark every flowId of this namespace as "old" */
    for (size_t i = 0; i < c->cap; i++)
        if (c->tab[i].flow_id != 0 && c->tab[i].ns == nsi && c->tab[i].active) c->tab[i].active = 2;
    int applied = 0;
    for (size_t j = 0; j < n; j++) {
        const orc_cluster_rule *r = &rules[j];
        /* FlowRuleUtil.isValidRule + checkClusterField, FlowRuleUtil.java:176-231 */
        if (!(r->count >= 0 && r->grade >= 0 && r->strategy >= 0)) continue;
        if (r->flow_id <= 0) continue;
        if (!(r->sample_count > 0 && r->window_interval_ms > 0 && r->window_interval_ms % r->sample_count == 0))
            continue;
        if (r->strategy != 0) continue;
        crule *e = ctab_find(c, r->flow_id, 1);
        e->r = *r;
        e->ns = nsi;
        e->active = 1;
        if (!e->conc_live) { /* CurrentConcurrencyManager.put(flowId, 0) when absent (:356-358) */
            e->conc_live = 1;
            e->now_calls = 0;
        }
        if (!e->metric) e->metric = orc_cmetric_new(r->sample_count, r->window_interval_ms); /* putMetricIfAbsent */
        applied++;
    }
    /* clearAndResetRulesConditional: drop rules (and their metrics) no longer present */
    for (size_t i = 0; i < c->cap; i++) {
        if (c->tab[i].flow_id != 0 && c->tab[i].ns == nsi && c->tab[i].active == 2) {
            c->tab[i].active = 0;
            c->tab[i].conc_live = 0;
            orc_cmetric_free(c->tab[i].metric);
            c->tab[i].metric = NULL;
        }
    }
    return applied;
}

struct orc_cparam **orc_cluster_param_slot(orc_cluster *c) { return &c->param; }
struct orc_conc **orc_cluster_conc_slot(orc_cluster *c) { return &c->conc; }
/* ClusterFlowRuleManager.getFlowRuleById + CurrentConcurrencyManager.get: the active rule (NULL when
 * absent), its namespace and its nowCalls counter (*now_calls = NULL when absent). */
const orc_cluster_rule *orc_cluster_active_rule(orc_cluster *c, int64_t flow_id, int *ns, int32_t **now_calls) {
    crule *e = flow_id > 0 ? ctab_find(c, flow_id, 0) : NULL;
    if (now_calls) *now_calls = (e && e->conc_live) ? &e->now_calls : NULL;
    if (!e || !e->active) return NULL;
    if (ns) *ns = e->ns;
    return &e->r;
}
int32_t orc_cluster_connected(orc_cluster *c, int ns) { return ns >= 0 ? c->ns_connected[ns] : 0; }
/* GlobalRequestLimiter.tryPass(namespace): no limiter for the namespace -> pass */
int orc_cluster_limiter_try_pass(orc_cluster *c, int ns, int64_t now) {
    if (ns < 0) return 0;
    return c->ns_limiter[ns] ? orc_limiter_try_pass(c->ns_limiter[ns], now) : 1;
}

void orc_cluster_set_namespace_limit(orc_cluster *c, const char *ns, double max_allowed_qps) {
    int i = ns_index(c, ns, 1);
    if (i < 0) return;
    if (!c->ns_limiter[i]) c->ns_limiter[i] = orc_limiter_new(max_allowed_qps); /* GlobalRequestLimiter.initIfAbsent */
    else c->ns_limiter[i]->qps_allowed = max_allowed_qps;                     /* applyMaxQpsChange */
}

void orc_cluster_set_connected_count(orc_cluster *c, const char *ns, int32_t n) {
    int i = ns_index(c, ns, 1);
    if (i >= 0) c->ns_connected[i] = n;
}

static orc_token_result tr(int32_t s, int32_t rem, int32_t wait) {
    orc_token_result t;
    t.status = s;
    t.remaining = rem;
    t.wait_in_ms = wait;
    return t;
}

/* DefaultTokenService.requestToken (CS/flow/DefaultTokenService.java:39-50) ->
 * ClusterFlowChecker.acquireClusterToken (CS/flow/ClusterFlowChecker.java:55-112) */
orc_token_result orc_cluster_request_token(orc_cluster *c, int64_t flow_id, int32_t acquire, int prioritized,
                                           int64_t now) {
    if (flow_id <= 0 || acquire <= 0) return tr(TRS_BAD_REQUEST, 0, 0);
    crule *e = ctab_find(c, flow_id, 0);
    if (!e || e->active != 1) return tr(TRS_NO_RULE_EXISTS, 0, 0);
    /* allowProceed -> GlobalRequestLimiter.tryPass(namespace), :50-53 */
    if (e->ns < 0) return tr(TRS_TOO_MANY_REQUEST, 0, 0);
    if (c->ns_limiter[e->ns] && !orc_limiter_try_pass(c->ns_limiter[e->ns], now)) return tr(TRS_TOO_MANY_REQUEST, 0, 0);
    orc_cmetric *m = e->metric;
    if (!m) return tr(TRS_FAIL, 0, 0);
    double latest_qps = orc_cmetric_avg(m, now, ORC_CEV_PASS);
    double base = e->r.threshold_type == 1 ? e->r.count : e->r.count * (double)c->ns_connected[e->ns]; /* :38-48 */
    double global_threshold = base * c->exceed_count;
    double next_remaining = global_threshold - latest_qps - (double)acquire;
    if (next_remaining >= 0) {
        orc_cmetric_add(m, now, ORC_CEV_PASS, acquire);
        orc_cmetric_add(m, now, ORC_CEV_PASS_REQUEST, 1);
        if (prioritized) orc_cmetric_add(m, now, ORC_CEV_OCCUPIED_PASS, acquire);
        return tr(TRS_OK, j_d2i(next_remaining), 0);
    }
    if (prioritized) {
        double occupy_avg = orc_cmetric_avg(m, now, ORC_CEV_WAITING);
        if (occupy_avg <= c->max_occupy_ratio * global_threshold) {
            int32_t wait = orc_cmetric_try_occupy_next(m, now, ORC_CEV_PASS, acquire, global_threshold);
            if (wait > 0) return tr(TRS_SHOULD_WAIT, 0, wait);
        }
    }
    orc_cmetric_add(m, now, ORC_CEV_BLOCK, acquire);
    orc_cmetric_add(m, now, ORC_CEV_BLOCK_REQUEST, 1);
    if (prioritized) orc_cmetric_add(m, now, ORC_CEV_OCCUPIED_BLOCK, acquire);
    return tr(TRS_BLOCKED, 0, 0);
}

/* SimpleClusterFlowChecker.acquireClusterToken, RLS/flow/SimpleClusterFlowChecker.java:33-65 */
orc_token_result orc_cluster_request_token_simple(orc_cluster *c, int64_t flow_id, int32_t acquire, int64_t now) {
    crule *e = ctab_find(c, flow_id, 0);
    if (!e || e->active != 1) return tr(TRS_NO_RULE_EXISTS, 0, 0);
    orc_cmetric *m = e->metric;
    if (!m) return tr(TRS_FAIL, 0, 0);
    double latest_qps = orc_cmetric_avg(m, now, ORC_CEV_PASS);
    double global_threshold = e->r.count * c->exceed_count;
    double next_remaining = global_threshold - latest_qps - (double)acquire;
    if (next_remaining >= 0) {
        orc_cmetric_add(m, now, ORC_CEV_PASS, acquire);
        orc_cmetric_add(m, now, ORC_CEV_PASS_REQUEST, 1);
        return tr(TRS_OK, j_d2i(next_remaining), 0);
    }
    orc_cmetric_add(m, now, ORC_CEV_BLOCK, acquire);
    orc_cmetric_add(m, now, ORC_CEV_BLOCK_REQUEST, 1);
    return tr(TRS_BLOCKED, 0, 0);
}

void orc_cluster_replay(orc_cluster *c, size_t n, const int64_t *flow_id, const int32_t *acquire,
                        const uint8_t *prio, const int64_t *ts, orc_token_result *out) {
    for (size_t i = 0; i < n; i++)
        out[i] = orc_cluster_request_token(c, flow_id[i], acquire[i], prio ? prio[i] : 0, ts[i]);
}

/* Envoy RLS replay: SimpleClusterFlowChecker per descriptor (sentinel-cluster-server-envoy-rls
 * .../flow/SimpleClusterFlowChecker.java:35-60), descriptors in order. */
void orc_cluster_replay_simple(orc_cluster *c, size_t n, const int64_t *flow_id, const int32_t *acquire,
                               const int64_t *ts, orc_token_result *out) {
    for (size_t i = 0; i < n; i++) out[i] = orc_cluster_request_token_simple(c, flow_id[i], acquire[i], ts[i]);
}

int64_t orc_cluster_metric_sum(orc_cluster *c, int64_t flow_id, int ev, int64_t now) {
    crule *e = ctab_find(c, flow_id, 0);
    if (!e || !e->metric) return -1;
    return orc_cmetric_sum(e->metric, now, ev);
}

/* ========================================================================== */
int64_t orc_java_round(double d) { return j_round(d); }
double orc_java_next_up(double d) { return j_next_up(d); }
int32_t orc_java_d2i(double d) { return j_d2i(d); }
int64_t orc_java_d2l(double d) { return j_d2l(d); }
int32_t orc_java_string_hash(const char *s) { return j_string_hash_utf8(s, strlen(s)); }
