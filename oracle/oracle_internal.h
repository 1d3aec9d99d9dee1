/* ORACLE / TEST INFRASTRUCTURE ONLY: internal structures shared by the oracle's
 * translation units (not an interface). */
#ifndef SENTINEL_ORACLE_INTERNAL_H
#define SENTINEL_ORACLE_INTERNAL_H
#include "sentinel_oracle.h"
#include "oracle_ext.h"

#define ORC_STATISTIC_MAX_RT 5000 /* CORE/config/SentinelConfig.java:69 DEFAULT_STATISTIC_MAX_RT */
#define ORC_SAMPLE_COUNT 2        /* CORE/node/SampleCountProperty.java:39 */
#define ORC_INTERVAL 1000         /* CORE/node/IntervalProperty.java:41 */
#define ORC_OCCUPY_TIMEOUT 500    /* CORE/node/OccupyTimeoutProperty.java:40 */
#define ORC_NCOUNTERS 7

typedef struct obucket {
    int64_t start;
    int64_t c[ORC_NCOUNTERS];
    int64_t min_rt;
} obucket;

struct orc_leap {
    int kind;
    int sample_count, interval_ms, window_ms;
    double interval_sec;
    obucket *b;
    uint8_t *present;
    obucket detached;
    orc_leap *borrow;           /* OccupiableBucketLeapArray.borrowArray */
    int64_t occ[ORC_NCOUNTERS]; /* ClusterMetricLeapArray.occupyCounter */
    int has_occ;                /* ClusterMetricLeapArray.hasOccupied */
};

struct orc_node {
    orc_leap *second; /* ArrayMetric(SAMPLE_COUNT, INTERVAL): occupiable, StatisticNode.java:99-100 */
    orc_leap *minute; /* ArrayMetric(60, 60*1000, false), StatisticNode.java:106 */
    int64_t threads;  /* curThreadNum LongAdder */
    int64_t last_fetch; /* StatisticNode.lastFetchTime, StatisticNode.java:118 */
    int mock;
    double mock_pass_qps, mock_prev_pass_qps;
    int32_t mock_threads;
};

struct orc_ctrl {
    int behavior, grade;
    double count;
    int max_queueing_time_ms;
    int64_t latest_passed_time; /* RateLimiterController.java:33 / WarmUpRateLimiterController.java:30 */
    /* WarmUpController.java:66-73 */
    int cold_factor;
    int32_t warning_token, max_token;
    double slope;
    int64_t stored_tokens, last_filled_time;
};

typedef struct orc_cb orc_cb;        /* circuit breaker (oracle_ext.c) */
typedef struct orc_pmap orc_pmap;    /* u64 -> i64 map (oracle_ext.c) */
typedef struct orc_lru orc_lru;      /* capacity-bounded LRU CacheMap (oracle_ext.c) */

typedef struct flow_res {
    orc_node *node;  /* ClusterNode of the resource (ClusterBuilderSlot.java:82-110) */
    orc_ctrl **ctrl; /* rules' raters in FlowRuleComparator order */
    int nctrl;
    int32_t *cmode, *cfallback; /* per rule: clusterMode, fallbackToLocalWhenFail */
    int64_t *cflow;             /* per rule: ClusterFlowConfig.flowId */
    orc_prule **prule;  /* ParamFlowRuleManager rules of the resource, list order */
    int nprule;
    /* ParameterMetric.threadCountMap: paramIdx -> CacheMap (LRU, capacity 4000), created by
     * ParameterMetric.initialize(rule) for the rule's (resolved) paramIdx */
    int32_t *pt_idx;
    orc_lru **pt_map;
    int npt;
    orc_cb **cb;        /* DegradeRuleManager circuit breakers, list order */
    int ncb;
} flow_res;

/* SystemRuleManager thresholds (SystemRuleManager.java:62-74) and SystemStatusListener readings */
typedef struct orc_sys {
    int check;  /* checkSystemStatus */
    int load_set, cpu_set;
    double load, cpu, qps;
    int64_t max_rt, max_thread;
    double cur_load, cur_cpu;  /* SystemStatusListener: -1 until measured */
} orc_sys;

struct orc_flow {
    uint32_t n;
    int cold_factor;
    flow_res *res;
    orc_node *entry; /* Constants.ENTRY_NODE: inbound traffic of every resource */
    orc_sys sys;
    struct orc_cluster *server; /* embedded token server (cluster-mode rules), or NULL */
    int cluster_mode;           /* 1: the server decides; 0: no token service */
    /* args[0] of the current event when it is a Collection / array (ParamFlowChecker.passLocalCheck
     * checks every element): its values, or NULL for a single value */
    const uint64_t *plist;
    uint32_t plist_n;
    /* the current event's argument vector (SGA_EV_ARGS), or NULL: word pairs, see oracle_ext.h */
    const uint64_t *args;
    const uint64_t *args_pvals;
    uint32_t nargs;
};

/* helpers implemented in sentinel_oracle.c / oracle_ext.c */
void orc_flow_system_restore(orc_flow *f);
int orc_flow_rule_check(orc_flow *f, uint32_t resource, int64_t now, int acquire, int prioritized, int64_t *wait_ms);
void orc_flow_res_free_ext(flow_res *fr);

#endif
