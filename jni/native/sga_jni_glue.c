/* Plain-C half of the JNI shim (see sga_jni_glue.h). */
#include "sga_jni_glue.h"

#include <stdlib.h>
#include <string.h>

static void token_out(const sga_token_result *r, int32_t out3[3]) {
    out3[0] = r->status;
    out3[1] = r->remaining;
    out3[2] = r->wait_in_ms;
}

int sgaj_create(int32_t device, uint32_t max_batch, uint32_t max_rules, sga_engine **out) {
    sga_config cfg;
    sga_config_default(&cfg);
    cfg.device = device;
    if (max_batch) cfg.max_batch = max_batch;
    if (max_rules) cfg.max_rules = max_rules;
    return sga_create(&cfg, out);
}

int sgaj_load_cluster_flow_rules(sga_engine *e, const char *ns, const int64_t *flow_id, const double *count,
                                 const int32_t *threshold_type, const int32_t *sample_count,
                                 const int32_t *window_interval_ms, size_t n) {
    /* the engine's load replaces the namespace's rule set, so the whole list goes in one call */
    sga_cluster_flow_rule buf[64];
    sga_cluster_flow_rule *r = n <= 64 ? buf : (sga_cluster_flow_rule *)malloc(n * sizeof(*r));
    if (!r) return SGA_ENOMEM;
    for (size_t i = 0; i < n; i++) {
        memset(&r[i], 0, sizeof(r[i]));
        r[i].flow_id = flow_id[i];
        r[i].count = count[i];
        r[i].threshold_type = threshold_type ? threshold_type[i] : 0;       /* AVG_LOCAL */
        r[i].sample_count = sample_count ? sample_count[i] : 10;            /* DEFAULT_CLUSTER_SAMPLE_COUNT */
        r[i].window_interval_ms = window_interval_ms ? window_interval_ms[i] : 1000;
        r[i].grade = 1;                                                     /* FLOW_GRADE_QPS */
        r[i].resource_timeout_ms = 2000;
        r[i].client_offline_time_ms = 2000;
    }
    const int rc = sga_load_cluster_flow_rules(e, ns, r, n);
    if (r != buf) free(r);
    return rc;
}

int sgaj_request_token(sga_engine *e, int64_t flow_id, int32_t acquire, int32_t prioritized, int64_t now_ms,
                       int32_t out3[3]) {
    sga_token_result r;
    const int rc = sga_request_token_one(e, flow_id, acquire, prioritized ? 1 : 0, now_ms, &r);
    if (rc == SGA_OK) token_out(&r, out3);
    return rc;
}

int sgaj_submit(sga_engine *e, int64_t flow_id, int32_t acquire, int32_t prioritized, int64_t now_ms,
                uint64_t *ticket) {
    return sga_token_submit(e, flow_id, acquire, prioritized ? 1 : 0, now_ms, ticket);
}

int sgaj_poll(sga_engine *e, uint64_t ticket, int32_t out3[3]) {
    sga_token_result r;
    const int rc = sga_poll(e, ticket, &r);
    if (rc == SGA_OK) token_out(&r, out3);
    return rc;
}

int sgaj_request_param_token(sga_engine *e, int64_t flow_id, int32_t acquire, const int64_t *values,
                             uint32_t n_values, int64_t now_ms, int32_t out3[3]) {
    const uint32_t off[2] = {0, n_values};
    sga_token_result r;
    const int rc = sga_request_param_tokens(e, &flow_id, &acquire, off, values, &now_ms, 1, &r);
    if (rc == SGA_OK) token_out(&r, out3);
    return rc;
}

int sgaj_concurrent(sga_engine *e, int32_t op, uint32_t client, int64_t id, int32_t acquire, int64_t now_ms,
                    int64_t out2[2]) {
    const uint8_t o = (uint8_t)op;
    sga_concurrent_result r;
    const int rc = sga_concurrent_ops(e, &o, &client, &id, &acquire, &now_ms, 1, &r);
    if (rc == SGA_OK) {
        out2[0] = r.status;
        out2[1] = r.token_id;
    }
    return rc;
}

int sgaj_entry(sga_engine *e, uint32_t resource, int64_t now_ms, int32_t count, uint32_t flags, uint64_t param,
               int32_t dec_wait[2]) {
    const uint8_t kind = 0, fl = (uint8_t)flags;
    const int64_t rt = 0;
    int8_t dec = 0;
    int32_t wait = 0;
    /* through the coalescing queue: concurrent SphU.entry callers share one engine batch */
    const int rc = sga_event_one(e, kind, resource, now_ms, count, fl, rt, param, NULL, 0, &dec, &wait);
    if (rc == SGA_OK) {
        dec_wait[0] = dec;
        dec_wait[1] = wait;
    }
    return rc;
}

int sgaj_exit(sga_engine *e, uint32_t resource, int64_t now_ms, int32_t count, uint32_t flags, int64_t rt_ms,
              uint64_t param) {
    const uint8_t kind = 1, fl = (uint8_t)flags;
    /* Entry.exit returns nothing: queued without waiting (decided in ticket order before anything this thread
       queues or calls later) */
    return sga_event_post(e, kind, resource, now_ms, count, fl, rt_ms, param, NULL, 0, NULL);
}

int sgaj_entry_args(sga_engine *e, uint32_t resource, int64_t now_ms, int32_t count, uint32_t flags,
                    const uint64_t *words, uint32_t nargs, uint32_t nwords, int32_t dec_wait[2]) {
    const uint8_t kind = SGA_KIND_ENTRY, fl = (uint8_t)(flags | SGA_EV_ARGS);
    const int64_t rt = 0;
    const uint64_t param = (uint64_t)nargs; /* the pairs start at offset 0 */
    int8_t dec = 0;
    int32_t wait = 0;
    const int rc = sga_event_one(e, kind, resource, now_ms, count, fl, rt, param, words, nwords, &dec, &wait);
    if (rc == SGA_OK) {
        dec_wait[0] = dec;
        dec_wait[1] = wait;
    }
    return rc;
}

int sgaj_exit_args(sga_engine *e, uint32_t resource, int64_t now_ms, int32_t count, uint32_t flags, int64_t rt_ms,
                   const uint64_t *words, uint32_t nargs, uint32_t nwords) {
    const uint8_t kind = SGA_KIND_EXIT, fl = (uint8_t)(flags | SGA_EV_ARGS);
    const uint64_t param = (uint64_t)nargs;
    return sga_event_post(e, kind, resource, now_ms, count, fl, rt_ms, param, words, nwords, NULL);
}

int sgaj_revoke_args(sga_engine *e, uint32_t resource, int64_t now_ms, int32_t count, uint32_t flags,
                     const uint64_t *words, uint32_t nargs, uint32_t nwords) {
    const uint8_t kind = SGA_KIND_REVOKE, fl = (uint8_t)(flags | SGA_EV_ARGS);
    const int64_t rt = 0;
    const uint64_t param = (uint64_t)nargs;
    return sga_event_post(e, kind, resource, now_ms, count, fl, rt, param, words, nwords, NULL);
}

int sgaj_blocked(sga_engine *e, uint32_t resource, int64_t now_ms, int32_t count, uint32_t flags) {
    const uint8_t kind = SGA_KIND_BLOCKED, fl = (uint8_t)flags;
    const int64_t rt = 0;
    const uint64_t param = 0;
    return sga_event_post(e, kind, resource, now_ms, count, fl, rt, param, NULL, 0, NULL);
}

int sgaj_load_param_rules(sga_engine *e, size_t n, const uint32_t *resource, const int32_t *grade,
                          const double *count, const int32_t *behavior, const int32_t *max_queue,
                          const int32_t *burst, const int32_t *param_idx, const int64_t *duration_sec,
                          const uint32_t *hot_off, const int64_t *hot_values, const int32_t *hot_counts,
                          const int32_t *cluster_mode, const int32_t *cluster_fallback,
                          const int64_t *cluster_flow_id, const int32_t *cluster_sample_count,
                          const int32_t *cluster_window_ms) {
    sga_param_rule *r = (sga_param_rule *)calloc(n ? n : 1, sizeof(*r));
    if (!r) return SGA_ENOMEM;
    for (size_t i = 0; i < n; i++) {
        r[i].resource = resource[i];
        r[i].grade = grade[i];
        r[i].count = count[i];
        r[i].control_behavior = behavior[i];
        r[i].max_queueing_time_ms = max_queue[i];
        r[i].burst_count = burst[i];
        r[i].param_idx = param_idx[i];
        r[i].duration_in_sec = duration_sec[i];
        if (hot_off) {
            r[i].n_hot = hot_off[i + 1] - hot_off[i];
            r[i].hot_values = (const uint64_t *)hot_values + hot_off[i];
            r[i].hot_thresholds = hot_counts + hot_off[i];
        }
        if (cluster_mode && cluster_mode[i]) {
            r[i].cluster_mode = 1;
            r[i].cluster_fallback = cluster_fallback ? cluster_fallback[i] : 0;
            r[i].cluster_flow_id = cluster_flow_id ? cluster_flow_id[i] : 0;
            r[i].cluster_sample_count = cluster_sample_count ? cluster_sample_count[i] : 10;
            r[i].cluster_window_ms = cluster_window_ms ? cluster_window_ms[i] : 1000;
        }
    }
    const int rc = sga_load_param_rules(e, r, n);
    free(r);
    return rc;
}

int sgaj_load_degrade_rules(sga_engine *e, size_t n, const uint32_t *resource, const int32_t *grade,
                            const double *count, const int32_t *time_window, const int32_t *min_request,
                            const double *slow_ratio, const int32_t *stat_interval_ms) {
    sga_degrade_rule *r = (sga_degrade_rule *)calloc(n ? n : 1, sizeof(*r));
    if (!r) return SGA_ENOMEM;
    for (size_t i = 0; i < n; i++) {
        r[i].resource = resource[i];
        r[i].grade = grade[i];
        r[i].count = count[i];
        r[i].time_window = time_window[i];
        r[i].min_request_amount = min_request[i];
        r[i].slow_ratio_threshold = slow_ratio[i];
        r[i].stat_interval_ms = stat_interval_ms[i];
    }
    const int rc = sga_load_degrade_rules(e, r, n);
    free(r);
    return rc;
}

int sgaj_load_system_rules(sga_engine *e, size_t n, const double *load, const double *cpu, const double *qps,
                           const int64_t *avg_rt, const int64_t *max_thread) {
    sga_system_rule *r = (sga_system_rule *)calloc(n ? n : 1, sizeof(*r));
    if (!r) return SGA_ENOMEM;
    for (size_t i = 0; i < n; i++) {
        r[i].highest_system_load = load[i];
        r[i].highest_cpu_usage = cpu[i];
        r[i].qps = qps[i];
        r[i].avg_rt = avg_rt[i];
        r[i].max_thread = max_thread[i];
    }
    const int rc = sga_load_system_rules(e, r, n);
    free(r);
    return rc;
}

int sgaj_set_system_status(sga_engine *e, double avg_load, double cpu_usage) {
    return sga_set_system_status(e, avg_load, cpu_usage);
}

int sgaj_load_cluster_param_rules(sga_engine *e, const char *ns, size_t n, const int64_t *flow_id,
                                  const double *count, const int32_t *threshold_type, const int32_t *sample_count,
                                  const int32_t *window_ms, const uint32_t *hot_off, const int64_t *hot_values,
                                  const int32_t *hot_counts) {
    sga_cluster_param_rule *r = (sga_cluster_param_rule *)calloc(n ? n : 1, sizeof(*r));
    if (!r) return SGA_ENOMEM;
    for (size_t i = 0; i < n; i++) {
        r[i].flow_id = flow_id[i];
        r[i].count = count[i];
        r[i].threshold_type = threshold_type ? threshold_type[i] : 0; /* AVG_LOCAL */
        r[i].sample_count = sample_count ? sample_count[i] : 10;
        r[i].window_interval_ms = window_ms ? window_ms[i] : 1000;
        r[i].grade = 1;
        r[i].param_idx_set = 1;
        r[i].duration_in_sec = 1;
        if (hot_off) {
            r[i].n_hot = (int32_t)(hot_off[i + 1] - hot_off[i]);
            r[i].hot_values = hot_values + hot_off[i];
            r[i].hot_counts = hot_counts + hot_off[i];
        }
    }
    const int rc = sga_load_cluster_param_rules(e, ns, r, n);
    free(r);
    return rc;
}

int sgaj_set_connected_count(sga_engine *e, const char *ns, int32_t connected) {
    return sga_set_connected_count(e, ns, connected);
}

int sgaj_set_namespace_limit(sga_engine *e, const char *ns, double max_qps) {
    return sga_set_namespace_limit(e, ns, max_qps);
}

int sgaj_set_cluster_server(sga_engine *e, int32_t mode) { return sga_set_cluster_server(e, mode); }

int sgaj_query_node(sga_engine *e, uint32_t resource, int64_t now_ms, double d8[10], int64_t l6[6]) {
    sga_node_view v;
    const int rc = sga_query_node(e, resource, now_ms, &v);
    if (rc != SGA_OK) return rc;
    d8[0] = v.pass_qps;
    d8[1] = v.block_qps;
    d8[2] = v.success_qps;
    d8[3] = v.exception_qps;
    d8[4] = v.occupied_pass_qps;
    d8[5] = v.avg_rt;
    d8[6] = v.min_rt;
    d8[7] = v.previous_pass_qps;
    d8[8] = v.max_success_qps;
    d8[9] = v.previous_block_qps;
    l6[0] = v.total_pass;
    l6[1] = v.total_block;
    l6[2] = v.total_success;
    l6[3] = v.total_exception;
    l6[4] = v.cur_thread_num;
    l6[5] = v.waiting;
    return SGA_OK;
}

int sgaj_metrics_snapshot(sga_engine *e, int64_t now_ms, int64_t *rows8, size_t cap, size_t *n) {
    sga_metric_node *m = (sga_metric_node *)calloc(cap ? cap : 1, sizeof(*m));
    if (!m) return SGA_ENOMEM;
    size_t k = 0;
    const int rc = sga_metrics_snapshot(e, now_ms, m, cap, &k);
    for (size_t i = 0; i < k && i < cap; i++) {
        int64_t *r = rows8 + 8 * i;
        r[0] = m[i].timestamp;
        r[1] = m[i].resource;
        r[2] = m[i].pass_qps;
        r[3] = m[i].block_qps;
        r[4] = m[i].success_qps;
        r[5] = m[i].exception_qps;
        r[6] = m[i].rt;
        r[7] = m[i].occupied_pass_qps;
    }
    *n = k;
    free(m);
    return rc;
}
