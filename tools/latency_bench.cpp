// Single-call latency through the C ABI (what every drop-in call pays):
//   requestToken  : sga_request_token_one (coalescing queue) from 1 thread and from T threads at once
//                   (the Netty worker pattern of FlowRequestProcessor.java:43), 100k cluster rules;
//   batch of one  : sga_request_tokens with n = 1 (no queue) for comparison;
//   SphU.entry    : sga_submit_events with one entry event (the local slot chain per call), 10k rules;
//                   and through the coalescing event queue (sga_event_one) from 1 and T threads, each passed
//                   entry followed by its exit (calls_per_s counts entries).
// Prints one JSON line per case: p50 / p99 / max in microseconds and calls per second.
// Build: g++ -O2 -std=c++17 tools/latency_bench.cpp -Iinclude -Lsentinel_amd -lsentinel_amd -lpthread
// Run (GPU box): LD_LIBRARY_PATH=sentinel_amd ./tools/latency_bench [threads] [calls]
#include "sentinel_amd.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

using clk = std::chrono::steady_clock;

static double us_since(clk::time_point t) {
    return std::chrono::duration<double, std::micro>(clk::now() - t).count();
}

static void report(const char *name, std::vector<double> &lat, double wall_s, int threads) {
    std::sort(lat.begin(), lat.end());
    const size_t n = lat.size();
    std::printf("{\"case\": \"%s\", \"threads\": %d, \"calls\": %zu, \"p50_us\": %.1f, \"p99_us\": %.1f, "
                "\"max_us\": %.1f, \"calls_per_s\": %.0f}\n",
                name, threads, n, lat[n / 2], lat[(size_t)(n * 0.99)], lat[n - 1], n / wall_s);
    std::fflush(stdout);
}

int main(int argc, char **argv) {
    const int threads = argc > 1 ? std::atoi(argv[1]) : 16;
    const int calls = argc > 2 ? std::atoi(argv[2]) : 2000;
    sga_config cfg;
    sga_config_default(&cfg);
    cfg.max_batch = 1 << 16;
    cfg.max_rules = 1 << 17;
    sga_engine *e = nullptr;
    if (sga_create(&cfg, &e) != SGA_OK) {
        std::fprintf(stderr, "sga_create failed\n");
        return 1;
    }
    const int n_rules = 100000;
    std::vector<sga_cluster_flow_rule> rules(n_rules);
    for (int i = 0; i < n_rules; ++i) {
        sga_cluster_flow_rule &r = rules[i];
        r = sga_cluster_flow_rule{};
        r.flow_id = i + 1;
        r.count = 10 + (i % 1000);
        r.threshold_type = 1;
        r.sample_count = 10;
        r.window_interval_ms = 1000;
        r.grade = 1;
        r.resource_timeout_ms = 2000;
        r.client_offline_time_ms = 2000;
    }
    if (sga_load_cluster_flow_rules(e, "default", rules.data(), rules.size()) < 0) {
        std::fprintf(stderr, "load rules: %s\n", sga_last_error(e));
        return 1;
    }
    const int64_t t0 = 1700000000000LL;
    std::atomic<int64_t> clock_ms{t0};
    // warm up both paths
    for (int i = 0; i < 200; ++i) {
        sga_token_result r;
        sga_request_token_one(e, 1 + (i % n_rules), 1, 0, clock_ms.load(), &r);
    }
    {  // requestToken, one thread
        std::vector<double> lat;
        const auto w0 = clk::now();
        for (int i = 0; i < calls; ++i) {
            sga_token_result r;
            const auto t = clk::now();
            sga_request_token_one(e, 1 + ((i * 7919) % n_rules), 1, 0, t0 + i / 10, &r);
            lat.push_back(us_since(t));
        }
        report("requestToken (sga_request_token_one)", lat, us_since(w0) / 1e6, 1);
    }
    {  // requestToken, T threads at once
        std::vector<std::vector<double>> lat(threads);
        std::vector<std::thread> th;
        const auto w0 = clk::now();
        for (int k = 0; k < threads; ++k)
            th.emplace_back([&, k] {
                for (int i = 0; i < calls; ++i) {
                    sga_token_result r;
                    const auto t = clk::now();
                    sga_request_token_one(e, 1 + ((i * 7919 + k * 104729) % n_rules), 1, 0, t0 + 1000 + i / 10, &r);
                    lat[k].push_back(us_since(t));
                }
            });
        for (auto &t : th) t.join();
        const double wall = us_since(w0) / 1e6;
        std::vector<double> all;
        for (auto &v : lat) all.insert(all.end(), v.begin(), v.end());
        report("requestToken (sga_request_token_one, concurrent)", all, wall, threads);
    }
    {  // batch of one, no queue
        std::vector<double> lat;
        const auto w0 = clk::now();
        for (int i = 0; i < calls; ++i) {
            sga_token_result r;
            const int64_t f = 1 + ((i * 7919) % n_rules), ts = t0 + 5000 + i / 10;
            const int32_t a = 1;
            const uint8_t p = 0;
            const auto t = clk::now();
            sga_request_tokens(e, &f, &a, &p, &ts, 1, &r);
            lat.push_back(us_since(t));
        }
        report("requestToken (sga_request_tokens, n = 1)", lat, us_since(w0) / 1e6, 1);
    }
    {  // SphU.entry: one entry event through the local slot chain
        const uint32_t n_res = 10000;
        sga_flow_set_resources(e, n_res);
        std::vector<sga_flow_rule> fr(n_res);
        for (uint32_t i = 0; i < n_res; ++i) {
            fr[i] = sga_flow_rule{};
            fr[i].resource = i;
            fr[i].grade = 1;
            fr[i].count = 100;
            fr[i].warm_up_period_sec = 10;
            fr[i].max_queueing_time_ms = 500;
        }
        sga_load_flow_rules(e, fr.data(), fr.size());
        std::vector<double> lat;
        const auto w0 = clk::now();
        for (int i = 0; i < calls; ++i) {
            const uint8_t kind = 0, flags = 0;
            const uint32_t res = (uint32_t)((i * 7919) % n_res);
            const int64_t ts = t0 + 10000 + i / 10, rt = 0;
            const int32_t acq = 1;
            const uint64_t param = 0;
            int8_t dec;
            int32_t wait;
            const auto t = clk::now();
            sga_submit_events(e, &kind, &res, &ts, &acq, &flags, &rt, &param, 1, &dec, &wait);
            lat.push_back(us_since(t));
        }
        report("SphU.entry (sga_submit_events, one entry)", lat, us_since(w0) / 1e6, 1);
        // SphU.entry + Entry.exit through the coalescing event queue (sga_event_one), 1 thread and T threads:
        // what GpuStatisticSlot calls per entry (jni/native/sga_jni_glue.c sgaj_entry / sgaj_exit)
        for (int post = 0; post < 2; ++post)  // exits waited for (sga_event_one) or posted (sga_event_post)
        for (int nt : {1, threads}) {
            std::vector<std::vector<double>> l2(nt);
            std::vector<std::thread> th;
            std::atomic<int> passed{0};
            const auto w1 = clk::now();
            for (int k = 0; k < nt; ++k)
                th.emplace_back([&, k] {
                    for (int i = 0; i < calls; ++i) {
                        const uint32_t res = (uint32_t)((i * 7919 + k * 104729) % n_res);
                        const int64_t ts = t0 + 20000 + (nt > 1 ? 50000 : 0) + post * 100000 + i / 10;
                        int8_t dec;
                        int32_t wait;
                        const auto t = clk::now();
                        sga_event_one(e, 0, res, ts, 1, 0, 0, 0, nullptr, 0, &dec, &wait);
                        l2[k].push_back(us_since(t));
                        if (dec == 0) {
                            passed.fetch_add(1);
                            if (post) sga_event_post(e, 1, res, ts + 5, 1, 0, 5, 0, nullptr, 0, nullptr);
                            else sga_event_one(e, 1, res, ts + 5, 1, 0, 5, 0, nullptr, 0, &dec, &wait);
                        }
                    }
                });
            for (auto &t : th) t.join();
            const double wall = us_since(w1) / 1e6;
            std::vector<double> all;
            for (auto &v : l2) all.insert(all.end(), v.begin(), v.end());
            report(post ? (nt == 1 ? "SphU.entry (sga_event_one; each passed entry's exit posted, sga_event_post)"
                                   : "SphU.entry (sga_event_one, concurrent; each passed entry's exit posted)")
                        : (nt == 1 ? "SphU.entry (sga_event_one; each passed entry also exits)"
                                   : "SphU.entry (sga_event_one, concurrent; each passed entry also exits)"),
                   all, wall, nt);
        }
    }
    sga_destroy(e);
    return 0;
}
