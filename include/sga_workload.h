/*
 * sga_workload.h -- synthetic C3 workload generator on the GPU (bench / test
 * support only; libsga_workload.so, not part of the decision path).
 * Same counter-based generator as sentinel_amd/workload.py:
 *   u64(stream, i) = splitmix64(seed + stream*0xD1B54A32D192ED03 + i*0x9E3779B97F4A7C15)
 *   rank ~ Zipf(s) by rejection-inversion, flowId = perm[rank-1] + 1,
 *   prioritized = u64(PRIO, i) % 100 < prio_pct, acquire = 1,
 *   ts = T0 + i*1000/lambda.
 */
#ifndef SGA_WORKLOAD_H
#define SGA_WORKLOAD_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct sgaw_cluster_params {
    uint64_t seed;
    int64_t t0;
    int64_t lambda;     /* events per virtual second */
    int64_t n_rules;    /* Zipf support 1..n_rules */
    double zipf_s;
    int32_t prio_pct;
    int32_t n_shards;   /* keep only events with splitmix64(flowId) % n_shards == shard */
    int32_t shard;
    int32_t reserved;
} sgaw_cluster_params;

/* Generates global events [start, start+m) and appends the ones of `shard`
 * (arrival order kept) to the output arrays; ts_off is relative to ts_base.
 * *d_count (device u32) receives the number kept.  d_tmp must hold 4*m+64
 * u32 words.  Asynchronous on hip_stream. */
int sgaw_gen_cluster(const sgaw_cluster_params *p, uint64_t start, uint32_t m, const int64_t *d_perm, int64_t ts_base,
                     int64_t *d_fid, int32_t *d_acq, uint8_t *d_prio, uint32_t *d_ts_off, uint32_t *d_count,
                     uint32_t *d_tmp, void *hip_stream);

/* histogram of flowIds (1..n) of a device array into d_hist (u32[n+1]); for bytes_alg touched-key counts */
int sgaw_flow_histogram(const int64_t *d_fid, uint32_t m, uint32_t *d_hist, int64_t n, void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif
