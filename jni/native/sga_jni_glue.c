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
    const int rc = sga_submit_events(e, &kind, &resource, &now_ms, &count, &fl, &rt, &param, 1, &dec, &wait);
    if (rc == SGA_OK) {
        dec_wait[0] = dec;
        dec_wait[1] = wait;
    }
    return rc;
}

int sgaj_exit(sga_engine *e, uint32_t resource, int64_t now_ms, int32_t count, uint32_t flags, int64_t rt_ms,
              uint64_t param) {
    const uint8_t kind = 1, fl = (uint8_t)flags;
    int8_t dec = 0;
    int32_t wait = 0;
    return sga_submit_events(e, &kind, &resource, &now_ms, &count, &fl, &rt_ms, &param, 1, &dec, &wait);
}
