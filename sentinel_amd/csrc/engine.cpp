// Host side of the admission engine: rule management (the ClusterFlowRuleManager
// mirror), device state ownership and the extern "C" ABI of include/sentinel_amd.h.
#include "../../include/sentinel_amd.h"
#include "cluster.hpp"
#include "cluster_exact.hpp"  // the window record layout (rec_units)
#include "concurrent.hpp"
#include "flow.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <thread>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

namespace sga {

struct SlotHost {
    int64_t flow_id = 0;
    bool allocated = false;  // ClusterMetricStatistics holds a metric for flow_id
    bool active = false;     // FLOW_RULES holds the rule
    int ns = -1;
    double count = 0;
    int threshold_type = 0;
    int S = 0, interval = 0;  // metric geometry, fixed at metric creation (putMetricIfAbsent)
    uint32_t boff = 0, bcap = 0;
    int64_t resource_timeout = 2000, client_offline = 2000;  // ClusterFlowConfig defaults
    bool conc_live = false;  // CurrentConcurrencyManager holds flow_id
};

// Cluster parameter rule slot (ClusterParamFlowRuleManager PARAM_RULES + ClusterParamMetricStatistics).
// Slots are never reused: keys (rule slot, value) of a dropped metric can never match a new one.
// A few persistent host threads for the page-locked staging copies of large host-buffer batches
// (run_host_batch): run(f) calls f(t) for t in [0, size()) on them and returns when all are done.
class HostPool {
  public:
    ~HostPool() {
        {
            std::lock_guard<std::mutex> l(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int size() {
        if (th_.empty()) start();
        return (int)th_.size();
    }
    void run(const std::function<void(int)> &f) {
        if (th_.empty()) start();
        std::unique_lock<std::mutex> l(mu_);
        job_ = &f;
        pending_ = (int)th_.size();
        ++gen_;
        cv_.notify_all();
        done_.wait(l, [&] { return pending_ == 0; });
        job_ = nullptr;
    }

  private:
    void start() {
        int n = (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
        if (const char *e = getenv("SGA_HOST_THREADS")) n = std::max(1, std::min(64, atoi(e)));
        for (int t = 0; t < n; ++t)
            th_.emplace_back([this, t] {
                uint64_t seen = 0;
                for (;;) {
                    const std::function<void(int)> *f;
                    {
                        std::unique_lock<std::mutex> l(mu_);
                        cv_.wait(l, [&] { return stop_ || gen_ != seen; });
                        if (stop_) return;
                        seen = gen_;
                        f = job_;
                    }
                    (*f)(t);
                    std::lock_guard<std::mutex> l(mu_);
                    if (--pending_ == 0) done_.notify_one();
                }
            });
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)> *job_ = nullptr;
    uint64_t gen_ = 0;
    int pending_ = 0;
    bool stop_ = false;
};

struct PSlotHost {
    int64_t flow_id = 0;
    bool allocated = false;  // metric exists
    bool active = false;     // PARAM_RULES holds the rule
    int ns = -1;
    double count = 0;
    int threshold_type = 0;
    int S = 0, interval = 0;  // metric geometry, fixed at creation
    uint32_t boff = 0;
    uint32_t cap = 4000;     // each bucket map's maxCapacity, fixed at creation
    std::vector<std::pair<int64_t, int32_t>> hot;  // ascending value
    uint64_t lru_off = 0, lru_words = 0;  // LRU mode: the metric's queue areas in the pool (lru_words = 0: none)
};

struct NamespaceHost {
    std::string name;
    int32_t connected = 0;
    bool has_limit = false;
    double max_qps = 0;
};

// Coalescing queue of single token requests (TokenService.requestToken is called once per request,
// from many Netty threads: FlowRequestProcessor.java:43).  Producers take a ticket with one atomic
// add and fill the ring slot the ticket names (a bounded multi-producer ring with per-slot sequence
// numbers: slot seq == t free for ticket t, t + 1 filled, t + 2 decided; the poller frees it for
// t + kCap).  Whoever polls while no batch is running becomes the combiner: it takes every filled
// slot from the head in ticket order and decides them as ONE engine batch, so concurrent callers
// share a launch, and decisions equal one batch per call in ticket order.
struct TokenQueue {
    static constexpr uint64_t kCap = 1u << 16;
    struct Slot {
        std::atomic<uint64_t> seq{0};
        int64_t flow_id = 0, ts = 0;
        int32_t acquire = 0;
        uint8_t prio = 0;
        uint64_t result = 0;
    };
    std::unique_ptr<Slot[]> ring{new Slot[kCap]};
    std::atomic<uint64_t> tail{0};
    uint64_t head = 0;  // combiner only
    std::atomic<bool> combining{false};
    std::vector<int64_t> fid, ts;
    std::vector<int32_t> acq;
    std::vector<uint8_t> prio;
    std::vector<uint64_t> out;
    TokenQueue() {
        for (uint64_t i = 0; i < kCap; ++i) ring[i].seq.store(i, std::memory_order_relaxed);
    }
};

// The same coalescing queue for the local path's events (SphU.entry / Entry.exit through GpuStatisticSlot, one
// synchronous call per entry from every application thread: CtSph.entryWithPriority, CtSph.java:117-168).  A
// slot holds one event and a copy of its argument words (SGA_EV_ARGS pairs and list values, at most kWords);
// the combiner concatenates the slots' words, rebases their offsets and decides every filled slot from the head
// as ONE sga_submit_events_ex batch, in ticket order.
struct EventQueue {
    static constexpr uint64_t kCap = 1u << 14;
    static constexpr uint32_t kWords = 64;
    struct Slot {
        std::atomic<uint64_t> seq{0};
        int64_t ts = 0, rt = 0;
        uint64_t param = 0;
        uint32_t resource = 0;
        int32_t acquire = 0;
        uint8_t kind = 0, flags = 0;
        uint32_t nwords = 0;
        bool posted = false;  // sga_event_post: nobody polls it, the combiner frees the slot
        uint64_t words[kWords];
        int8_t decision = 0;
        int32_t wait = 0;
    };
    std::unique_ptr<Slot[]> ring{new Slot[kCap]};
    std::atomic<uint64_t> tail{0};
    uint64_t head = 0;                // combiner only
    std::atomic<uint64_t> done{0};    // head as published after each round (event_flush)
    std::atomic<bool> combining{false};
    std::atomic<bool> post_err{false};  // a round holding posted events failed: the next sga_event_post says so
    std::vector<uint8_t> kind, flags;
    std::vector<uint32_t> res;
    std::vector<int64_t> ts, rt;
    std::vector<int32_t> acq, wait;
    std::vector<uint64_t> param, vals;
    std::vector<int8_t> dec;
    EventQueue() {
        for (uint64_t i = 0; i < kCap; ++i) ring[i].seq.store(i, std::memory_order_relaxed);
    }
};

struct Engine {
    sga_config cfg{};
    hipStream_t stream = nullptr;
    std::string err;
    std::mutex mu;
    TokenQueue tq;
    EventQueue eq;
    // cluster-mode FlowRules of the local path: ClusterStateManager mode (sga_set_cluster_server) and
    // a generation of the cluster rule set their slots were resolved against
    int32_t cluster_server = 0;
    uint64_t cluster_gen = 1;

    // ---- cluster rules (host mirror)
    std::vector<SlotHost> slots;
    std::vector<uint32_t> free_slots;
    std::unordered_map<int64_t, uint32_t> slot_of;  // flowId -> slot (metric exists)
    std::vector<NamespaceHost> nss;
    uint32_t bucket_used = 0;

    // ---- device state
    DevBuf<SlotParam> d_param;
    DevBuf<int64_t> d_rec;  // 8 int64 per bucket
    DevBuf<HashEntry> d_htab;
    DevBuf<int64_t> d_slot_fid;  // flowId per slot (metric snapshots)
    DevBuf<uint32_t> d_ncount;
    DevBuf<uint8_t> d_nodes;
    DevBuf<uint32_t> d_dense;  // dense flowId table (see sync_device): slot | wcode << 24 per flowId
    DevBuf<uint32_t> d_dkey;   // the hot path's key table (ClusterState::dkey) of the first scratch set
    DevBuf<uint32_t> d_wtab;
    uint32_t dense_n = 0;
    DevBuf<uint32_t> d_fresh;
    uint32_t hmask = 0;
    DevBuf<uint8_t> d_scratch;
    BatchScratch scratch;
    uint32_t scratch_slots_cap = 0;
    // ---- pipelined device batches (sga_request_tokens_device_pipelined): batch k + 1's stage 1 (key pass,
    // count scans, sorts) runs on cls_stream while batch k's stage 2 (decisions) runs on the engine stream.
    // Batches alternate between two scratch sets, each with its own hot set and its own key table (whose
    // entries the hot set writes); a set is reused once its previous batch's
    // stage 2 is done (ev_dec).  Every other engine call joins the pipeline first (join_pipeline).
    DevBuf<uint8_t> d_scratch2;
    BatchScratch scratch2;
    DevBuf<uint32_t> d_dkey2;
    hipStream_t cls_stream = nullptr;
    hipEvent_t ev_cls[2] = {nullptr, nullptr}, ev_dec[2] = {nullptr, nullptr}, ev_in = nullptr, ev_other = nullptr;
    bool dec_recorded[2] = {false, false};
    bool pipe_live = false;   // stage-1 work may be in flight on cls_stream
    bool pipe_dirty = true;   // other engine work queued since the last pipelined batch
    int parity = 0;
    const BatchScratch *last_sc = &scratch;  // the scratch of the last batch (sga_cluster_batch_info)
    // host API staging
    DevBuf<int64_t> d_in_fid;
    DevBuf<int32_t> d_in_acq;
    DevBuf<uint8_t> d_in_prio;
    DevBuf<uint32_t> d_in_ts;
    DevBuf<uint64_t> d_out;
    // small batches (<= kSmallStage requests): inputs packed [flowId | acquire | ts offset | prio] in
    // page-locked memory, one copy each way
    static constexpr size_t kSmallStage = 4096;
    PinnedBuf h_stage, h_res;
    // large host batches: kPipeSlots page-locked chunks of kPipeChunk requests each way, the batch's
    // int64 times on the device (offsets computed there), the copy threads
    static constexpr size_t kPipeChunk = 1u << 20, kPipeSlots = 3;
    PinnedBuf h_pin_in, h_pin_out;
    DevBuf<int32_t> d_tsd;  // times as int32 deltas from the batch's first time
    DevBuf<int64_t> d_ts64, d_tminmax;  // registered host buffers: the int64 times, their min / max
    std::vector<std::pair<uintptr_t, uintptr_t>> host_regs;  // sga_host_register ranges [lo, hi)
    bool registered(const void *p, size_t bytes) const {
        const uintptr_t a = (uintptr_t)p, b = a + bytes;
        for (auto &r : host_regs)
            if (a >= r.first && b <= r.second) return true;
        return false;
    }
    hipEvent_t ev_pin_in[kPipeSlots] = {}, ev_pin_out[kPipeSlots] = {};
    HostPool host_pool;
    static constexpr size_t kPipeIn = 8 + 4 + 4 + 1;  // flowId, time delta, acquire, prio
    // page-locked slots (each DMA'd once at allocation: the first transfers from fresh page-locked pages
    // run at half rate), events, the device delta buffer
    void ensure_pipe_staging() {
        if (!h_pin_in.p) {
            h_pin_in.alloc(kPipeSlots * kPipeChunk * kPipeIn);
            h_pin_out.alloc(kPipeSlots * kPipeChunk * 8);
            std::memset(h_pin_in.p, 0, h_pin_in.n);
            std::memset(h_pin_out.p, 0, h_pin_out.n);
            for (size_t s = 0; s < kPipeSlots; ++s) {
                SGA_HIP_CHECK(hipEventCreateWithFlags(&ev_pin_in[s], hipEventDisableTiming));
                SGA_HIP_CHECK(hipEventCreateWithFlags(&ev_pin_out[s], hipEventDisableTiming));
            }
        }
        if (d_tsd.n < cfg.max_batch) {
            d_tsd.alloc(cfg.max_batch);
            const size_t w = std::min(h_pin_in.n, d_tsd.bytes());
            SGA_HIP_CHECK(hipMemcpyAsync(d_tsd.p, h_pin_in.p, w, hipMemcpyHostToDevice, stream));
            SGA_HIP_CHECK(hipMemcpyAsync(h_pin_out.p, d_tsd.p, std::min(h_pin_out.n, d_tsd.bytes()),
                                         hipMemcpyDeviceToHost, stream));
            SGA_HIP_CHECK(hipStreamSynchronize(stream));
        }
    }
    ~Engine() {
        for (size_t s = 0; s < kPipeSlots; ++s) {
            if (ev_pin_in[s]) (void)hipEventDestroy(ev_pin_in[s]);
            if (ev_pin_out[s]) (void)hipEventDestroy(ev_pin_out[s]);
        }
    }
    DevBuf<uint8_t> d_stage;
    DevBuf<int64_t> d_tmp7;
    DevBuf<NsLimiterDev> d_lim;  // one per namespace index (used when the namespace has a limiter)

    // ---- cluster parameter flow
    std::vector<PSlotHost> pslots;
    std::unordered_map<int64_t, uint32_t> pslot_of;  // flowId -> slot (metric exists)
    uint32_t pbucket_used = 0;
    DevBuf<PRuleParam> d_pparam;
    DevBuf<int64_t> d_prstart, d_ptmax;
    DevBuf<uint8_t> d_pcoupled;
    DevBuf<HashEntry> d_phtab;
    uint32_t phmask = 0;
    DevBuf<int64_t> d_hot_v;
    DevBuf<int32_t> d_hot_c;
    DevBuf<int32_t> d_ns_conn;
    DevBuf<int64_t> d_vtab;
    DevBuf<uint64_t> d_ktab;
    DevBuf<uint32_t> d_koff, d_kslot;
    DevBuf<int64_t> d_kval, d_krec;
    DevBuf<uint32_t> d_pctl;
    uint32_t vmask = 0, kmask = 0;
    DevBuf<uint8_t> d_pscratch;
    CParamScratch pscratch{};
    DevBuf<uint32_t> d_in_voff;
    DevBuf<int64_t> d_in_vals;
    DevBuf<int64_t> d_top_list, d_top_val;
    DevBuf<double> d_top_qps;
    DevBuf<uint32_t> d_top_n;
    // CacheMap capacity (cparam_exact.hpp): per slot key counts, per bucket LRU queue areas and sizes
    uint32_t pcap_default = 4000;  // ClusterParamMetric.DEFAULT_CLUSTER_MAX_CAPACITY
    DevBuf<uint32_t> d_pnkeys, d_ppsize, d_psw;
    DevBuf<uint64_t> d_ppq, d_pqoff;
    DevBuf<PLruRec> d_plpool;
    uint64_t plpool_used = 0;
    std::unordered_map<uint64_t, std::vector<uint64_t>> plpool_free;  // area size -> offsets of dropped metrics' areas

    // ---- cluster concurrency tokens
    DevBuf<ConcParam> d_cparam;   // per slot
    DevBuf<int32_t> d_now_calls;  // per slot
    DevBuf<TokenEntry> d_tok;
    DevBuf<uint32_t> d_tctr;      // [0] live [1] tombstones [2] expired by the last pass
    uint32_t tmask = 0, tepoch = 1;
    uint64_t tlive = 0, ttomb = 0;
    uint64_t token_base = 0;
    DevBuf<uint8_t> d_cscratch;
    ConcScratch cscratch;
    DevBuf<uint8_t> d_cin_op;
    DevBuf<uint32_t> d_cin_client, d_online, d_creset;
    DevBuf<int64_t> d_cin_id, d_cin_ts;
    DevBuf<int32_t> d_cin_acq;
    DevBuf<sga_concurrent_result> d_cout;
    DevBuf<TokenEntry> d_tfind;

    ConcState cstate() const {
        ConcState c{};
        c.cs = state();
        c.cparam = d_cparam.p;
        c.now_calls = d_now_calls.p;
        c.tok = d_tok.p;
        c.tmask = tmask;
        c.epoch = tepoch;
        c.ctr = d_tctr.p;
        return c;
    }

    // token table + operation scratch, created with the first concurrency call
    void ensure_conc() {
        if (d_cscratch.p) return;
        const size_t cap = cfg.max_batch;
        d_cscratch.alloc(conc_scratch_bytes(cap));
        conc_scratch_carve(cscratch, d_cscratch.p, cap);
        d_cin_op.alloc(cap);
        d_cin_client.alloc(cap);
        d_cin_id.alloc(cap);
        d_cin_ts.alloc(cap);
        d_cin_acq.alloc(cap);
        d_cout.alloc(cap);
        d_tctr.alloc(4);
        d_tfind.alloc(1);
        SGA_HIP_CHECK(hipMemsetAsync(d_tctr.p, 0, d_tctr.bytes(), stream));
        d_tok.alloc(1024);
        SGA_HIP_CHECK(hipMemsetAsync(d_tok.p, 0, d_tok.bytes(), stream));
        tmask = 1023;
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
    }

    // keeps live + tombstones + `incoming` at most half the table (rehash drops the tombstones)
    bool reserve_tokens(uint64_t incoming) {
        const uint64_t cap = (uint64_t)tmask + 1;
        if (2 * (tlive + ttomb + incoming) <= cap) return true;
        uint64_t ncap = 1024;
        while (ncap < 4 * (tlive + incoming)) ncap <<= 1;
        if (ncap > (1ull << 31)) return false;
        DevBuf<TokenEntry> nt;
        nt.alloc(ncap);
        conc_rehash(d_tok.p, (uint32_t)cap, nt.p, (uint32_t)(ncap - 1), stream);
        const uint32_t z = 0;
        SGA_HIP_CHECK(hipMemcpyAsync(d_tctr.p + 1, &z, 4, hipMemcpyHostToDevice, stream));
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
        std::swap(d_tok.p, nt.p);
        std::swap(d_tok.n, nt.n);
        tmask = (uint32_t)(ncap - 1);
        ttomb = 0;
        return true;
    }

    void read_token_counters() {
        uint32_t c[3];
        SGA_HIP_CHECK(hipMemcpy(c, d_tctr.p, 12, hipMemcpyDeviceToHost));
        tlive = c[0];
        ttomb = c[1];
    }

    CParamState pstate() {
        CParamState st{};
        st.param = d_pparam.p;
        st.rstart = d_prstart.p;
        st.tmax = d_ptmax.p;
        st.coupled = d_pcoupled.p;
        st.htab = d_phtab.p;
        st.hmask = phmask;
        st.nslots = (uint32_t)pslots.size();
        st.hot_v = d_hot_v.p;
        st.hot_c = d_hot_c.p;
        st.ns_connected = d_ns_conn.p;
        st.vtab = d_vtab.p;
        st.vmask = vmask;
        st.ktab = d_ktab.p;
        st.kmask = kmask;
        st.koff = d_koff.p;
        st.kslot = d_kslot.p;
        st.kval = d_kval.p;
        st.krec = d_krec.p;
        st.krec_cap = d_krec.n;
        st.ctl = d_pctl.p;
        st.nkeys = d_pnkeys.p;
        st.pq = d_ppq.p;
        st.psize = d_ppsize.p;
        st.lpool = d_plpool.p;
        st.sw_list = d_psw.p;
        st.seq = flow.seq;  // one access order with the local path's embedded-server calls
        return st;
    }

    // Rules the last stage-1 / count pass listed (ctl[4] of them, nsw > 0) switch to LRU mode: each gets
    // S queue areas of 2 cap + 3 records from the pool, filled from the keys' access stamps.
    void cparam_lru_switch_host(uint32_t nsw, hipStream_t s) {
        std::vector<uint32_t> lst(nsw);
        SGA_HIP_CHECK(hipMemcpyAsync(lst.data(), d_psw.p, nsw * 4, hipMemcpyDeviceToHost, s));
        SGA_HIP_CHECK(hipStreamSynchronize(s));
        std::vector<uint64_t> qoff(nsw);
        uint64_t need = 0;
        uint32_t max_s = 1;
        for (uint32_t w = 0; w < nsw; ++w) {
            PSlotHost &h = pslots[lst[w]];
            max_s = std::max<uint32_t>(max_s, (uint32_t)h.S);
            const uint64_t words = (uint64_t)h.S * (2ull * h.cap + 3);
            auto fl = plpool_free.find(words);  // the areas of dropped metrics are reused first
            if (fl != plpool_free.end() && !fl->second.empty()) {
                qoff[w] = fl->second.back();
                fl->second.pop_back();
            } else {
                qoff[w] = plpool_used + need;
                need += words;
            }
            h.lru_off = qoff[w];
            h.lru_words = words;
        }
        if (d_plpool.n < plpool_used + need) d_plpool.grow(std::max<uint64_t>(plpool_used + need, 2 * d_plpool.n), s);
        plpool_used += need;
        if (d_pqoff.n < nsw) d_pqoff.alloc(std::max<size_t>(nsw, 2 * d_pqoff.n));
        SGA_HIP_CHECK(hipMemcpyAsync(d_pqoff.p, qoff.data(), nsw * 8, hipMemcpyHostToDevice, s));
        cparam_lru_switch(pstate(), d_pqoff.p, nsw, max_s, s);
        SGA_HIP_CHECK(hipMemsetAsync(d_pctl.p + 4, 0, 4, s));
        SGA_HIP_CHECK(hipStreamSynchronize(s));
    }

    // key store + batch scratch of the param path, created with the first param rules
    void ensure_param_store() {
        if (d_pctl.p) return;
        const uint32_t keys = cfg.max_param_keys ? cfg.max_param_keys : (1u << 20);
        uint32_t cap = 1024;
        while (cap < 2ull * keys) cap <<= 1;
        d_vtab.alloc((size_t)cap + 1);
        d_ktab.alloc(cap);
        d_koff.alloc(cap);
        d_kslot.alloc(cap);
        d_kval.alloc(cap);
        d_krec.alloc((size_t)keys * 30);  // 3 x 10 buckets per key on average
        d_pctl.alloc(8);
        SGA_HIP_CHECK(hipMemsetAsync(d_vtab.p, 0x00, d_vtab.bytes(), stream));
        std::vector<int64_t> empty(d_vtab.n, INT64_MIN);  // kAbsent = empty value slot
        SGA_HIP_CHECK(hipMemcpyAsync(d_vtab.p, empty.data(), d_vtab.bytes(), hipMemcpyHostToDevice, stream));
        SGA_HIP_CHECK(hipMemsetAsync(d_ktab.p, 0, d_ktab.bytes(), stream));
        SGA_HIP_CHECK(hipMemsetAsync(d_pctl.p, 0, d_pctl.bytes(), stream));
        vmask = cap - 1;
        kmask = cap - 1;
        d_pscratch.alloc(cparam_scratch_bytes(cfg.max_batch));
        cparam_scratch_carve(pscratch, d_pscratch.p, cfg.max_batch);
        d_in_voff.alloc((size_t)cfg.max_batch + 1);
        d_in_vals.alloc(cfg.max_batch);
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
    }

    // Upload the param rule table, its flowId hash, hot items and connected counts.
    void sync_param_device(const std::vector<uint32_t> &fresh) {
        const size_t ns = pslots.size();
        if (d_pparam.n < std::max<size_t>(ns, 1)) {
            const size_t c = std::max<size_t>(std::max<size_t>(ns, 1), d_pparam.n * 2);
            d_pparam.grow(c, stream);
            d_ptmax.grow(c, stream);
            d_pcoupled.grow(c, stream);
        }
        if (d_pnkeys.n < d_pparam.n) {  // new slots: no keys, free mode
            const size_t o = d_pnkeys.n;
            d_pnkeys.grow(d_pparam.n, stream);
            SGA_HIP_CHECK(hipMemsetAsync(d_pnkeys.p + o, 0, (d_pnkeys.n - o) * 4, stream));
            d_psw.alloc(d_pparam.n);
        }
        if (d_prstart.n < std::max<uint32_t>(pbucket_used, 1))
            d_prstart.grow(std::max<size_t>(pbucket_used, d_prstart.n * 2), stream);
        if (d_ppq.n < d_prstart.n) {
            const size_t o = d_ppq.n;
            d_ppq.grow(d_prstart.n, stream);
            d_ppsize.grow(d_prstart.n, stream);
            SGA_HIP_CHECK(hipMemsetAsync(d_ppq.p + o, 0xFF, (d_ppq.n - o) * 8, stream));  // kPNoQueue
            SGA_HIP_CHECK(hipMemsetAsync(d_ppsize.p + o, 0, (d_ppsize.n - o) * 4, stream));
        }
        std::vector<PRuleParam> hp(ns);
        std::vector<int64_t> hv;
        std::vector<int32_t> hc;
        for (size_t i = 0; i < ns; ++i) {
            const PSlotHost &h = pslots[i];
            PRuleParam &q = hp[i];
            std::memset(&q, 0, sizeof(q));
            q.count = h.count;
            q.isec = h.interval / 1000.0;
            q.boff = h.boff;
            q.S = h.S ? h.S : 1;
            q.W = h.S ? h.interval / h.S : 1;
            q.interval = h.interval;
            q.active = h.active ? 1 : 0;
            q.ns = h.ns;
            q.threshold_type = h.threshold_type;
            q.cap = h.cap;
            q.hot_off = (uint32_t)hv.size();
            q.n_hot = (uint32_t)h.hot.size();
            for (auto &kv : h.hot) {
                hv.push_back(kv.first);
                hc.push_back(kv.second);
            }
        }
        if (ns) SGA_HIP_CHECK(hipMemcpyAsync(d_pparam.p, hp.data(), ns * sizeof(PRuleParam), hipMemcpyHostToDevice, stream));
        if (d_hot_v.n < std::max<size_t>(hv.size(), 1)) {
            SGA_HIP_CHECK(hipStreamSynchronize(stream));
            d_hot_v.alloc(std::max<size_t>(hv.size(), 1));
            d_hot_c.alloc(std::max<size_t>(hv.size(), 1));
        }
        if (!hv.empty()) {
            SGA_HIP_CHECK(hipMemcpyAsync(d_hot_v.p, hv.data(), hv.size() * 8, hipMemcpyHostToDevice, stream));
            SGA_HIP_CHECK(hipMemcpyAsync(d_hot_c.p, hc.data(), hc.size() * 4, hipMemcpyHostToDevice, stream));
        }
        size_t nact = 0;
        for (auto &h : pslots) nact += h.active ? 1 : 0;
        size_t hcap = 1024;
        while (hcap < 2 * nact + 1) hcap <<= 1;
        std::vector<HashEntry> ht(hcap);
        std::memset(ht.data(), 0, hcap * sizeof(HashEntry));
        for (size_t i = 0; i < ns; ++i) {
            if (!pslots[i].active) continue;
            uint32_t h = (uint32_t)hash_flow_id(pslots[i].flow_id) & (uint32_t)(hcap - 1);
            while (ht[h].key != 0) h = (h + 1) & (uint32_t)(hcap - 1);
            ht[h].key = pslots[i].flow_id;
            ht[h].slot = (uint32_t)i;
            ht[h].W = (uint32_t)(pslots[i].interval / pslots[i].S);
        }
        if (d_phtab.n != hcap) {
            SGA_HIP_CHECK(hipStreamSynchronize(stream));
            d_phtab.alloc(hcap);
        }
        SGA_HIP_CHECK(hipMemcpyAsync(d_phtab.p, ht.data(), hcap * sizeof(HashEntry), hipMemcpyHostToDevice, stream));
        phmask = (uint32_t)(hcap - 1);
        upload_connected();
        for (uint32_t sl : fresh) cparam_init_rule(pstate(), sl, stream);
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
    }

    void upload_connected() {
        std::vector<int32_t> c(std::max<size_t>(nss.size(), 1), 0);
        for (size_t i = 0; i < nss.size(); ++i) c[i] = nss[i].connected;
        if (d_ns_conn.n < c.size()) {
            SGA_HIP_CHECK(hipStreamSynchronize(stream));
            d_ns_conn.alloc(c.size() + 16);
        }
        SGA_HIP_CHECK(hipMemcpyAsync(d_ns_conn.p, c.data(), c.size() * 4, hipMemcpyHostToDevice, stream));
    }

    // ---- local flow engine
    FlowEngine flow;

    int32_t uni_S = 0, uni_W = 0, uni_iv = 0;  // ClusterState::uni_S (sync_device)
    // pset 1: the second pipelined scratch set's dense table
    ClusterState state(int pset = 0) const {
        ClusterState st{};
        st.param = d_param.p;
        st.rec = d_rec.p;
        st.htab = d_htab.p;
        st.dense = d_dense.p;
        st.dkey = dense_n ? ((pset && d_dkey2.p) ? d_dkey2.p : d_dkey.p) : nullptr;
        st.slot_fid = d_slot_fid.p;
        st.wtab = d_wtab.p;
        st.dense_n = dense_n;
        st.hmask = hmask;
        st.nslots = (uint32_t)slots.size();
        st.max_occupy_ratio = cfg.max_occupy_ratio;
        st.uni_S = uni_S;
        st.uni_W = uni_W;
        st.uni_iv = uni_iv;
        return st;
    }

    int ns_index(const char *ns, bool create) {
        for (size_t i = 0; i < nss.size(); ++i)
            if (nss[i].name == ns) return (int)i;
        if (!create) return -1;
        NamespaceHost h;
        h.name = ns;
        nss.push_back(h);
        return (int)nss.size() - 1;
    }

    void ensure_scratch() {
        const uint32_t need_slots = std::max<uint32_t>((uint32_t)slots.size(), 1024u);
        if (d_scratch.p && need_slots <= scratch_slots_cap) return;
        uint32_t cap_slots = std::max<uint32_t>(need_slots, cfg.max_rules);
        // round to the next power of two so the radix digit layout fits
        uint32_t p2 = 1024;
        while (p2 < cap_slots) p2 <<= 1;
        const size_t bytes = batch_scratch_bytes(cfg.max_batch, p2);
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
        d_scratch.alloc(bytes);
        batch_scratch_carve(scratch, d_scratch.p, cfg.max_batch, p2);
        scratch.hot_lane_order = lds_lane_order_ok(stream) ? 1 : 0;
        scratch_slots_cap = p2;
        hot_reset(state(), scratch, p2, stream);
        if (d_scratch2.p) {  // the pipelined set follows
            d_scratch2.release();
            ensure_pipeline();
        }
    }

    // the second scratch set, the dense table copy, the classify stream and its events (first pipelined batch)
    void ensure_pipeline() {
        if (d_scratch2.p) return;
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
        d_scratch2.alloc(batch_scratch_bytes(cfg.max_batch, scratch_slots_cap));
        batch_scratch_carve(scratch2, d_scratch2.p, cfg.max_batch, scratch_slots_cap);
        scratch2.tmax_all = scratch.tmax_all;  // one latest time for both sets
        scratch2.hot_lane_order = scratch.hot_lane_order;
        scratch2.hot_enabled = scratch.hot_enabled;
        scratch2.hot_min = scratch.hot_min;
        scratch2.small_max = scratch.small_max;
        sync_dkey2();
        hot_reset(state(1), scratch2, scratch_slots_cap, stream);
        if (!cls_stream) {
            SGA_HIP_CHECK(hipStreamCreateWithFlags(&cls_stream, hipStreamNonBlocking));
            for (int k = 0; k < 2; ++k) {
                SGA_HIP_CHECK(hipEventCreateWithFlags(&ev_cls[k], hipEventDisableTiming));
                SGA_HIP_CHECK(hipEventCreateWithFlags(&ev_dec[k], hipEventDisableTiming));
            }
            SGA_HIP_CHECK(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
            SGA_HIP_CHECK(hipEventCreateWithFlags(&ev_other, hipEventDisableTiming));
        }
        dec_recorded[0] = dec_recorded[1] = false;
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
    }

    // the second scratch set's key table (hot_reset then fills it from the dense table)
    void sync_dkey2() {
        if (!d_scratch2.p) return;
        if (!dense_n) return;
        if (d_dkey2.n < d_dense.n) d_dkey2.alloc(d_dense.n);
    }

    // every engine call but a pipelined batch: order it after the pipeline's in-flight stage-1 work (stage 2
    // runs on the engine stream already), and the next pipelined stage 1 after it
    void join_pipeline() {
        pipe_dirty = true;
        if (!pipe_live) return;
        SGA_HIP_CHECK(hipEventRecord(ev_other, cls_stream));
        SGA_HIP_CHECK(hipStreamWaitEvent(stream, ev_other, 0));
        pipe_live = false;
    }

    // ---- caller streams (device entries).  Every device batch is ordered after all earlier
    // engine work and all later engine work is ordered after it, whichever stream it ran on: the
    // caller's stream first waits for the engine stream, then the engine stream waits for the
    // caller's stream.  Rule loads, the shared batch scratch and host-side calls therefore never
    // overlap a batch still in flight on another stream.
    hipEvent_t ev_eng = nullptr, ev_call = nullptr;

    hipStream_t enter_stream(void *hs) {
        if (!hs || (hipStream_t)hs == stream) return stream;
        if (!ev_eng) {
            SGA_HIP_CHECK(hipEventCreateWithFlags(&ev_eng, hipEventDisableTiming));
            SGA_HIP_CHECK(hipEventCreateWithFlags(&ev_call, hipEventDisableTiming));
        }
        SGA_HIP_CHECK(hipEventRecord(ev_eng, stream));
        SGA_HIP_CHECK(hipStreamWaitEvent((hipStream_t)hs, ev_eng, 0));
        return (hipStream_t)hs;
    }

    void leave_stream(hipStream_t cs) {
        if (cs == stream) return;
        SGA_HIP_CHECK(hipEventRecord(ev_call, cs));
        SGA_HIP_CHECK(hipStreamWaitEvent(stream, ev_call, 0));
    }

    void release_events() {
        if (ev_eng) (void)hipEventDestroy(ev_eng);
        if (ev_call) (void)hipEventDestroy(ev_call);
        ev_eng = ev_call = nullptr;
    }

    uint32_t alloc_slot() {
        if (!free_slots.empty()) {
            uint32_t s = free_slots.back();
            free_slots.pop_back();
            return s;
        }
        slots.emplace_back();
        return (uint32_t)slots.size() - 1;
    }

    // Upload param table + hash table; init buckets of new metrics.
    void sync_device(const std::vector<uint32_t> &fresh) {
        const size_t ns = slots.size();
        // capacity growth
        const size_t slot_cap = std::max<size_t>(ns, 1);
        if (d_param.n < slot_cap) {
            size_t c = std::max<size_t>(slot_cap, d_param.n * 2);
            d_param.grow(c, stream);
        }
        if (d_rec.n < 8 * (size_t)std::max<uint32_t>(bucket_used, 1)) {
            size_t c = std::max<size_t>(8 * (size_t)bucket_used, d_rec.n * 2);
            d_rec.grow(c, stream);
        }
        // param table
        std::vector<SlotParam> hp(ns);
        for (size_t i = 0; i < ns; ++i) {
            const SlotHost &h = slots[i];
            SlotParam &p = hp[i];
            std::memset(&p, 0, sizeof(p));
            if (!h.allocated) continue;
            const int conn = h.ns >= 0 ? nss[h.ns].connected : 0;
            // ClusterFlowChecker.calcGlobalThreshold(rule) * exceedCount, :38-48,68
            const double base = h.threshold_type == 1 ? h.count : h.count * (double)conn;
            p.thr = base * cfg.exceed_count;
            p.thr_simple = h.count * cfg.exceed_count;  // SimpleClusterFlowChecker.java:43
            p.isec = h.interval / 1000.0;
            p.boff = h.boff;
            p.S = h.S;
            p.W = h.interval / h.S;
            p.interval = h.interval;
            p.active = h.active ? 1 : 0;
            p.ns = h.ns;
        }
        if (ns) SGA_HIP_CHECK(hipMemcpyAsync(d_param.p, hp.data(), ns * sizeof(SlotParam), hipMemcpyHostToDevice, stream));
        // uniform geometry (ClusterState::uni_S): every allocated slot's record at slot * rec_units(S) units
        uni_S = 0;
        {
            int32_t S0 = 0, W0 = 0, I0 = 0;
            bool uni = true;
            for (size_t i = 0; i < ns && uni; ++i) {
                const SlotParam &p = hp[i];
                if (!slots[i].allocated) continue;
                if (!S0) {
                    S0 = p.S;
                    W0 = p.W;
                    I0 = p.interval;
                }
                uni = p.S == S0 && p.W == W0 && p.interval == I0 && (uint64_t)p.boff == (uint64_t)i * (uint64_t)sga::rec_units(S0);
            }
            static const bool no_uni = getenv("SGA_NO_UNI") && atoi(getenv("SGA_NO_UNI"));  // A/B knob
            if (uni && !no_uni && S0 > 0 && S0 <= 64) {
                uni_S = S0;
                uni_W = W0;
                uni_iv = I0;
            }
        }
        {  // concurrency: ConcurrentClusterFlowChecker.calcGlobalThreshold (no exceedCount), timeouts
            if (d_cparam.n < slot_cap) {
                const size_t c = std::max<size_t>(slot_cap, d_cparam.n * 2);
                d_cparam.grow(c, stream);
                d_now_calls.grow(c, stream);
            }
            std::vector<ConcParam> cp(ns);
            for (size_t i = 0; i < ns; ++i) {
                const SlotHost &h = slots[i];
                const int conn = h.ns >= 0 ? nss[h.ns].connected : 0;
                cp[i].thr = h.threshold_type == 1 ? h.count : h.count * (double)conn;
                cp[i].resource_timeout = h.resource_timeout;
                cp[i].client_offline = h.client_offline;
            }
            if (ns) SGA_HIP_CHECK(hipMemcpyAsync(d_cparam.p, cp.data(), ns * sizeof(ConcParam), hipMemcpyHostToDevice,
                                                 stream));
        }
        {
            std::vector<int64_t> fids(std::max<size_t>(ns, 1), 0);
            for (size_t i = 0; i < ns; ++i) fids[i] = slots[i].flow_id;
            if (d_slot_fid.n < fids.size()) {
                SGA_HIP_CHECK(hipStreamSynchronize(stream));
                d_slot_fid.alloc(std::max<size_t>(fids.size(), 2 * d_slot_fid.n));
            }
            SGA_HIP_CHECK(hipMemcpyAsync(d_slot_fid.p, fids.data(), fids.size() * 8, hipMemcpyHostToDevice, stream));
        }
        // hash table over active rules
        size_t nact = 0;
        for (auto &h : slots) nact += h.active ? 1 : 0;
        size_t hcap = 1024;
        while (hcap < 2 * nact + 1) hcap <<= 1;
        std::vector<HashEntry> ht(hcap);
        std::memset(ht.data(), 0, hcap * sizeof(HashEntry));
        for (size_t i = 0; i < ns; ++i) {
            if (!slots[i].active) continue;
            uint32_t h = (uint32_t)hash_flow_id(slots[i].flow_id) & (uint32_t)(hcap - 1);
            while (ht[h].key != 0) h = (h + 1) & (uint32_t)(hcap - 1);
            ht[h].key = slots[i].flow_id;
            ht[h].slot = (uint32_t)i;
            ht[h].W = (uint32_t)(slots[i].interval / slots[i].S);
        }
        if (d_htab.n != hcap) {
            SGA_HIP_CHECK(hipStreamSynchronize(stream));
            d_htab.alloc(hcap);
        }
        SGA_HIP_CHECK(hipMemcpyAsync(d_htab.p, ht.data(), hcap * sizeof(HashEntry), hipMemcpyHostToDevice, stream));
        hmask = (uint32_t)(hcap - 1);
        // Dense flowIds (the usual 1..N assignment): a direct table of 4-byte entries replaces the
        // probe sequence when it costs at most 16 B per active rule and the rules use <= 126
        // distinct window lengths (the key table's entries keep bit 31 for the hot set).  Same lookup
        // result as FLOW_RULES.get(flowId).
        {
            int64_t maxid = 0;
            std::vector<uint32_t> wvals;
            bool ok = nact > 0;
            for (size_t i = 0; i < ns && ok; ++i) {
                if (!slots[i].active) continue;
                maxid = std::max(maxid, slots[i].flow_id);
                const uint32_t W = (uint32_t)(slots[i].interval / slots[i].S);
                if (std::find(wvals.begin(), wvals.end(), W) == wvals.end()) wvals.push_back(W);
                if (wvals.size() > 126) ok = false;
            }
            if (ok && maxid <= (int64_t)(4 * nact + 4096) && maxid < (int64_t)0xFFFFFFFF) {
                // entry: slot | wcode << 24 (the key tables are filled from it by hot_reset below)
                std::vector<uint32_t> dt((size_t)maxid, 0xFFFFFFFFu);
                for (size_t i = 0; i < ns; ++i) {
                    if (!slots[i].active) continue;
                    const uint32_t W = (uint32_t)(slots[i].interval / slots[i].S);
                    const uint32_t code = (uint32_t)(std::find(wvals.begin(), wvals.end(), W) - wvals.begin());
                    dt[(size_t)slots[i].flow_id - 1] = (uint32_t)i | (code << 24);
                }
                wvals.resize(256, 1);
                if (d_dense.n < dt.size()) {
                    SGA_HIP_CHECK(hipStreamSynchronize(stream));
                    d_dense.alloc(dt.size());
                    d_dkey.alloc(dt.size());
                    if (d_dkey2.p) d_dkey2.alloc(dt.size());
                }
                if (d_wtab.n < 256) d_wtab.alloc(256);
                SGA_HIP_CHECK(hipMemcpyAsync(d_dense.p, dt.data(), dt.size() * 4, hipMemcpyHostToDevice, stream));
                SGA_HIP_CHECK(hipMemcpyAsync(d_wtab.p, wvals.data(), 256 * 4, hipMemcpyHostToDevice, stream));
                SGA_HIP_CHECK(hipStreamSynchronize(stream));
                dense_n = (uint32_t)maxid;
            } else {
                dense_n = 0;
            }
        }
        // fresh metrics: empty windows, no occupy (one kernel for all of them)
        if (!fresh.empty()) {
            if (d_fresh.n < fresh.size()) {
                SGA_HIP_CHECK(hipStreamSynchronize(stream));
                d_fresh.alloc(fresh.size());
            }
            SGA_HIP_CHECK(hipMemcpyAsync(d_fresh.p, fresh.data(), fresh.size() * 4, hipMemcpyHostToDevice, stream));
            cluster_init_slots(state(), d_fresh.p, (uint32_t)fresh.size(), stream);
        }
        // every record's copy of its threshold (the closed forms read it from the record's header)
        if (ns) cluster_sync_rec_thr(state(), (uint32_t)ns, stream);
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
        ensure_scratch();
        // slots may have been freed or reused: forget the hot-rule set (the next batch re-chooses it)
        hot_reset(state(), scratch, scratch_slots_cap, stream);
        if (d_scratch2.p) {
            sync_dkey2();
            hot_reset(state(1), scratch2, scratch_slots_cap, stream);
        }
        SGA_HIP_CHECK(hipStreamSynchronize(stream));
    }
};

}  // namespace sga

struct sga_engine {
    sga::Engine impl;
};

using sga::Engine;
using sga::SlotHost;
using sga::CEV_N;

// No exception crosses the C ABI: HIP errors map to -EIO, host allocation failures to -ENOMEM and
// anything else (a standard-library container throwing, say) to -EIO with its message.
static void event_flush(sga_engine *e);
template <typename F>
static int guarded(sga_engine *e, F &&f, bool join = true) {
    if (!e) return SGA_EINVAL;
    event_flush(e);  // events queued before this call (posted exits included) take effect first
    std::lock_guard<std::mutex> lk(e->impl.mu);
    try {
        if (join) e->impl.join_pipeline();
        return f(e->impl);
    } catch (const sga::HipError &h) {
        e->impl.err = h.what;
        return SGA_EIO;
    } catch (const std::bad_alloc &) {
        e->impl.err = "out of host memory";
        return SGA_ENOMEM;
    } catch (const std::exception &x) {
        e->impl.err = std::string("internal error: ") + x.what();
        return SGA_EIO;
    } catch (...) {
        e->impl.err = "internal error";
        return SGA_EIO;
    }
}

extern "C" {

int sga_abi_version(void) { return SGA_ABI_VERSION; }

void sga_config_default(sga_config *c) {
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    c->device = 0;
    c->max_batch = 1u << 20;
    c->max_rules = 1u << 16;
    c->cold_factor = 3;          // SentinelConfig.DEFAULT_COLD_FACTOR
    c->statistic_max_rt = 5000;  // SentinelConfig.DEFAULT_STATISTIC_MAX_RT
    c->exceed_count = 1.0;       // ServerFlowConfig.DEFAULT_EXCEED_COUNT
    c->max_occupy_ratio = 1.0;   // ServerFlowConfig.DEFAULT_MAX_OCCUPY_RATIO
}

int sga_create(const sga_config *cfg, sga_engine **out) {
    if (!out) return SGA_EINVAL;
    *out = nullptr;
    sga_config c;
    if (cfg) c = *cfg;
    else sga_config_default(&c);
    if (c.max_batch == 0 || c.max_batch > sga::kMaxBatch) return SGA_EINVAL;
    if (c.cold_factor <= 1) c.cold_factor = 3;  // SentinelConfig.coldFactor() fallback, :224-238
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= c.device || c.device < 0) return SGA_ENODEV;
    sga_engine *e = new (std::nothrow) sga_engine();
    if (!e) return SGA_ENOMEM;
    e->impl.cfg = c;
    int rc = guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(c.device));
        hipDeviceProp_t prop;
        SGA_HIP_CHECK(hipGetDeviceProperties(&prop, c.device));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            g.err = std::string("device is ") + prop.gcnArchName + ", engine is built for gfx950";
            return SGA_ENODEV;
        }
        SGA_HIP_CHECK(hipStreamCreateWithFlags(&g.stream, hipStreamNonBlocking));
        g.d_tmp7.alloc(8);
        g.flow.init(c, g.stream);
        g.ensure_scratch();
        if (c.max_batch >= 4 * Engine::kPipeChunk) {  // host-buffer batches this large: staging ready up front
            g.ensure_pipe_staging();
            (void)g.host_pool.size();
        }
        std::random_device rd;  // token ids: a random start, then splitmix64 of a counter (bijective)
        g.token_base = ((uint64_t)rd() << 32) ^ (uint64_t)rd();
        return SGA_OK;
    });
    if (rc != SGA_OK) {
        delete e;
        return rc;
    }
    *out = e;
    return SGA_OK;
}

int sga_destroy(sga_engine *e) {
    if (!e) return SGA_EINVAL;
    {
        std::lock_guard<std::mutex> lk(e->impl.mu);
        if (e->impl.stream) {
            (void)hipStreamSynchronize(e->impl.stream);
            e->impl.release_events();
            batch_scratch_release(e->impl.scratch);
            batch_scratch_release(e->impl.scratch2);
            if (e->impl.cls_stream) {
                (void)hipStreamSynchronize(e->impl.cls_stream);
                for (int k = 0; k < 2; ++k) {
                    (void)hipEventDestroy(e->impl.ev_cls[k]);
                    (void)hipEventDestroy(e->impl.ev_dec[k]);
                }
                (void)hipEventDestroy(e->impl.ev_in);
                (void)hipEventDestroy(e->impl.ev_other);
                (void)hipStreamDestroy(e->impl.cls_stream);
            }
            e->impl.flow.release();
            e->impl.h_stage.release();
            e->impl.h_res.release();
            (void)hipStreamDestroy(e->impl.stream);
        }
    }
    delete e;
    return SGA_OK;
}

const char *sga_last_error(const sga_engine *e) { return e ? e->impl.err.c_str() : "null engine"; }

void *sga_engine_stream(sga_engine *e) { return e ? (void *)e->impl.stream : nullptr; }

// ClusterFlowRuleManager.applyClusterFlowRule, CS/flow/rule/ClusterFlowRuleManager.java:325-374
int sga_load_cluster_flow_rules(sga_engine *e, const char *ns, const sga_cluster_flow_rule *rules, size_t n) {
    if (!ns || !*ns || (n && !rules)) return SGA_EINVAL;  // AssertUtil.notEmpty(namespace)
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        ++g.cluster_gen;  // cluster-mode local rules re-resolve their slots
        const int nsi = g.ns_index(ns, true);
        std::vector<uint32_t> fresh;
        if (n == 0) {  // clearAndResetRulesFor: rules dropped, metrics kept (:281-296)
            for (auto &h : g.slots)
                if (h.allocated && h.ns == nsi) {
                    h.active = false;
                    h.conc_live = false;  // CurrentConcurrencyManager.remove(flowId)
                }
            g.sync_device(fresh);
            return 0;
        }
        std::unordered_map<int64_t, const sga_cluster_flow_rule *> rule_map;
        std::vector<int64_t> order;
        std::vector<uint32_t> reset;
        for (size_t i = 0; i < n; ++i) {
            const sga_cluster_flow_rule &r = rules[i];
            // FlowRuleUtil.isValidRule + checkClusterField (FlowRuleUtil.java:176-231)
            if (!(r.count >= 0 && r.grade >= 0 && r.strategy >= 0)) continue;
            if (r.flow_id <= 0) continue;
            if (!(r.sample_count > 0 && r.window_interval_ms > 0 && r.window_interval_ms % r.sample_count == 0))
                continue;
            if (r.strategy != 0) continue;
            if (!rule_map.count(r.flow_id)) order.push_back(r.flow_id);
            rule_map[r.flow_id] = &r;  // ruleMap.put: last one wins
        }
        {  // rule slots are 24-bit inside the packed sort element (cluster.hpp kMaxSlots)
            size_t fresh_ids = 0;
            for (int64_t fid : order) fresh_ids += g.slot_of.count(fid) ? 0 : 1;
            if (g.slots.size() - g.free_slots.size() + fresh_ids > sga::kMaxSlots) {
                g.err = "more than 16M cluster rules on one engine";
                return SGA_ERANGE;
            }
        }
        // clearAndResetRulesConditional: flowIds of this namespace not in the new map lose rule AND metric
        for (uint32_t s = 0; s < g.slots.size(); ++s) {
            SlotHost &h = g.slots[s];
            if (!h.allocated || h.ns != nsi || !h.active) continue;
            if (rule_map.count(h.flow_id)) continue;
            h.active = false;
            h.allocated = false;
            h.conc_live = false;
            g.slot_of.erase(h.flow_id);
            g.free_slots.push_back(s);
        }
        for (int64_t fid : order) {
            const sga_cluster_flow_rule &r = *rule_map[fid];
            auto it = g.slot_of.find(fid);
            uint32_t s;
            if (it == g.slot_of.end()) {  // putMetricIfAbsent -> new ClusterMetric(sampleCount, windowIntervalMs)
                s = g.alloc_slot();
                SlotHost &h = g.slots[s];
                const uint32_t need = sga::rec_units(r.sample_count);  // the window record (64-byte units, cluster_exact.hpp)
                if (h.bcap < need) {
                    h.boff = g.bucket_used;
                    h.bcap = need;
                    g.bucket_used += need;
                }
                h.flow_id = fid;
                h.allocated = true;
                h.S = r.sample_count;
                h.interval = r.window_interval_ms;
                g.slot_of[fid] = s;
                fresh.push_back(s);
            } else {
                s = it->second;  // existing metric keeps its geometry and counters
            }
            SlotHost &h = g.slots[s];
            h.active = true;
            h.ns = nsi;
            h.count = r.count;
            h.threshold_type = r.threshold_type;
            h.resource_timeout = r.resource_timeout_ms;
            h.client_offline = r.client_offline_time_ms;
            if (!h.conc_live) {  // CurrentConcurrencyManager.put(flowId, 0) when absent (:356-358)
                h.conc_live = true;
                reset.push_back(s);
            }
        }
        g.sync_device(fresh);
        if (!reset.empty()) {
            if (g.d_creset.n < reset.size()) g.d_creset.alloc(reset.size());
            SGA_HIP_CHECK(hipMemcpyAsync(g.d_creset.p, reset.data(), reset.size() * 4, hipMemcpyHostToDevice, g.stream));
            sga::conc_reset_calls(g.d_now_calls.p, g.d_creset.p, (uint32_t)reset.size(), g.stream);
            SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
        }
        return (int)order.size();
    });
}

// GlobalRequestLimiter.initIfAbsent(namespace) (first call: new RequestLimiter(maxAllowedQps))
// and applyMaxQpsChange (later calls: setQpsAllowed), GlobalRequestLimiter.java:32-80.
int sga_set_hot_rules(sga_engine *e, int32_t enabled, uint32_t min_requests) {
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        for (sga::BatchScratch *sc : {&g.scratch, &g.scratch2}) {
            sc->hot_enabled = enabled ? 1 : 0;
            sc->hot_min = min_requests ? min_requests : 1;
        }
        if (g.d_scratch.p) sga::hot_reset(g.state(), g.scratch, g.scratch_slots_cap, g.stream);
        if (g.d_scratch2.p) sga::hot_reset(g.state(1), g.scratch2, g.scratch_slots_cap, g.stream);
        SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
        return SGA_OK;
    });
}

// Engine tuning (no reference counterpart): token batches of at most max_requests requests (at
// most 4096; 0 turns it off) are classified and sorted by one workgroup (k_small_sort) instead of
// the multi-launch pipeline -- the path a single requestToken takes.  Decisions do not depend on it.
int sga_set_small_batch(sga_engine *e, uint32_t max_requests) {
    return guarded(e, [&](Engine &g) {
        g.scratch.small_max = g.scratch2.small_max = std::min<uint32_t>(max_requests, 4096u);
        // the local path's one-workgroup replay of small host chunks (k_lsmall), at most kSmallEvents events
        g.flow.small_max = std::min<uint32_t>(max_requests, sga::FlowEngine::kSmallEvents);
        return SGA_OK;
    });
}

int sga_set_namespace_limit(sga_engine *e, const char *ns, double max_allowed_qps) {
    if (!ns || !*ns || !(max_allowed_qps >= 0)) return SGA_EINVAL;  // AssertUtil.isTrue(qpsAllowed >= 0)
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        ++g.cluster_gen;  // cluster-mode local rules re-resolve their slots
        const int i = g.ns_index(ns, true);
        if (g.d_lim.n < g.nss.size()) g.d_lim.grow(std::max<size_t>(g.nss.size(), 2 * g.d_lim.n), g.stream);
        if (!g.nss[i].has_limit) {
            sga::cluster_init_limiter(g.d_lim.p + i, g.stream);
            g.nss[i].has_limit = true;
        }
        g.nss[i].max_qps = max_allowed_qps;
        SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
        return SGA_OK;
    });
}

int sga_set_connected_count(sga_engine *e, const char *ns, int32_t connected) {
    if (!ns || !*ns || connected < 0) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        const int i = g.ns_index(ns, true);
        g.nss[i].connected = connected;
        std::vector<uint32_t> none;
        g.sync_device(none);
        g.upload_connected();
        SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
        return SGA_OK;
    });
}

static std::vector<sga::LimiterPass> limiter_passes(Engine &g) {
    std::vector<sga::LimiterPass> v;
    for (size_t i = 0; i < g.nss.size(); ++i)
        if (g.nss[i].has_limit) v.push_back(sga::LimiterPass{(int32_t)i, g.nss[i].max_qps, g.d_lim.p + i});
    return v;
}

int sga_request_tokens_device(sga_engine *e, const int64_t *d_flow_id, const int32_t *d_acquire,
                              const uint8_t *d_prio, int64_t ts_base, const uint32_t *d_ts_off, size_t n,
                              sga_token_result *d_out, void *hip_stream) {
    if (n && (!d_flow_id || !d_acquire || !d_ts_off || !d_out)) return SGA_EINVAL;
    if (ts_base < 0) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        if (n > g.cfg.max_batch) return SGA_ERANGE;
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        hipStream_t s = g.enter_stream(hip_stream);
        const auto lims = limiter_passes(g);
        sga::cluster_decide_batch(g.state(), g.scratch, d_flow_id, d_acquire, d_prio, ts_base, d_ts_off, (uint32_t)n,
                                  0, d_out, s, lims.data(), (int)lims.size());
        g.last_sc = &g.scratch;
        SGA_HIP_CHECK(hipGetLastError());
        g.leave_stream(s);
        return SGA_OK;
    });
}

int sga_request_tokens_packed_device(sga_engine *e, const sga_token_request *d_req, int64_t ts_base, size_t n,
                                     sga_token_result *d_out, void *hip_stream) {
    static_assert(sizeof(sga_token_request) == 12, "packed request = three words");
    if (n && (!d_req || !d_out)) return SGA_EINVAL;
    if (ts_base < 0 || ((uintptr_t)d_req & 3u)) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        if (n > g.cfg.max_batch) return SGA_ERANGE;
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        hipStream_t s = g.enter_stream(hip_stream);
        const auto lims = limiter_passes(g);
        sga::cluster_decide_batch_packed(g.state(), g.scratch, reinterpret_cast<const uint32_t *>(d_req), ts_base,
                                         (uint32_t)n, d_out, s, lims.data(), (int)lims.size());
        g.last_sc = &g.scratch;
        SGA_HIP_CHECK(hipGetLastError());
        g.leave_stream(s);
        return SGA_OK;
    });
}

// Pipelined device batches: stage 1 of this batch (sga::cluster_classify_hot) starts as soon as the inputs are
// ready on hip_stream and its scratch set is free, beside the previous batch's decisions; stage 2 runs on the
// engine stream after every earlier batch.  The outputs are on hip_stream after sga_stream_wait (or sga_sync).
// Batches the hot path does not take (small, limited) join the pipeline and run as sga_request_tokens_device.
int sga_request_tokens_device_pipelined(sga_engine *e, const int64_t *d_flow_id, const int32_t *d_acquire,
                                        const uint8_t *d_prio, int64_t ts_base, const uint32_t *d_ts_off, size_t n,
                                        sga_token_result *d_out, void *hip_stream) {
    if (n && (!d_flow_id || !d_acquire || !d_ts_off || !d_out)) return SGA_EINVAL;
    if (ts_base < 0) return SGA_EINVAL;
    return guarded(
        e,
        [&](Engine &g) {
            if (n > g.cfg.max_batch) return SGA_ERANGE;
            SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
            const auto lims = limiter_passes(g);
            if (!g.d_scratch.p || !sga::cluster_hot_eligible(g.state(), g.scratch, (uint32_t)n, 0, (int)lims.size())) {
                g.join_pipeline();
                hipStream_t s = g.enter_stream(hip_stream);
                sga::cluster_decide_batch(g.state(), g.scratch, d_flow_id, d_acquire, d_prio, ts_base, d_ts_off,
                                          (uint32_t)n, 0, d_out, s, lims.data(), (int)lims.size());
                g.last_sc = &g.scratch;
                SGA_HIP_CHECK(hipGetLastError());
                g.leave_stream(s);
                return SGA_OK;
            }
            g.ensure_pipeline();
            const int p = g.parity;
            sga::BatchScratch &sc = p ? g.scratch2 : g.scratch;
            hipStream_t cs = g.cls_stream;
            // stage 1 after: the inputs, other engine work queued since the last pipelined batch, and the
            // previous batch on this scratch set (its stage 2 leaves the hot set this batch reads)
            if (hip_stream && (hipStream_t)hip_stream != g.stream) {
                SGA_HIP_CHECK(hipEventRecord(g.ev_in, (hipStream_t)hip_stream));
                SGA_HIP_CHECK(hipStreamWaitEvent(cs, g.ev_in, 0));
            } else {
                g.pipe_dirty = true;  // inputs made on the engine stream
            }
            if (g.pipe_dirty) {
                SGA_HIP_CHECK(hipEventRecord(g.ev_other, g.stream));
                SGA_HIP_CHECK(hipStreamWaitEvent(cs, g.ev_other, 0));
                g.pipe_dirty = false;
            }
            if (g.dec_recorded[p]) SGA_HIP_CHECK(hipStreamWaitEvent(cs, g.ev_dec[p], 0));
            const sga::ClusterState st = g.state(p);
            sga::cluster_classify_hot(st, sc, d_flow_id, d_acquire, d_prio, ts_base, d_ts_off, (uint32_t)n, d_out, cs);
            SGA_HIP_CHECK(hipEventRecord(g.ev_cls[p], cs));
            SGA_HIP_CHECK(hipStreamWaitEvent(g.stream, g.ev_cls[p], 0));
            sga::cluster_decide_hot(st, sc, d_acquire, d_prio, ts_base, d_ts_off, (uint32_t)n, d_out, g.stream);
            SGA_HIP_CHECK(hipEventRecord(g.ev_dec[p], g.stream));
            g.dec_recorded[p] = true;
            g.pipe_live = true;
            g.parity ^= 1;
            g.last_sc = &sc;
            SGA_HIP_CHECK(hipGetLastError());
            return SGA_OK;
        },
        false);
}

// Kept for callers of the round-1 ABI: the device entry already returns once the batch is queued,
// so the "async" form is the same call (batches run in submission order on the engine stream).
int sga_request_tokens_device_async(sga_engine *e, const int64_t *d_flow_id, const int32_t *d_acquire,
                                    const uint8_t *d_prio, int64_t ts_base, const uint32_t *d_ts_off, size_t n,
                                    sga_token_result *d_out, void *hip_stream) {
    return sga_request_tokens_device(e, d_flow_id, d_acquire, d_prio, ts_base, d_ts_off, n, d_out, hip_stream);
}

int sga_stream_wait(sga_engine *e, void *hip_stream) {
    return guarded(e, [&](Engine &g) {
        if (!hip_stream || (hipStream_t)hip_stream == g.stream) return SGA_OK;
        (void)g.enter_stream(hip_stream);  // the caller's stream waits for every queued engine batch
        return SGA_OK;
    });
}

int sga_sync(sga_engine *e) {
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
        return SGA_OK;
    });
}

// One engine batch from host buffers at PCIe rate: the host threads copy chunk c of the inputs into a
// page-locked slot -- the times as int32 deltas from the batch's first time, with their min / max -- while
// the DMA engine moves chunk c - 1 to the device (17 B per request); the device turns the deltas into u32
// offsets from the minimum; after the pipeline the results come back the same way, chunk by chunk through
// page-locked slots the threads copy out of.  Returns 1 (nothing decided) when a time lies more than
// 2^31 - 1 ms from the first one.
static int run_host_batch_pipelined(Engine &g, const int64_t *flow_id, const int32_t *acquire, const uint8_t *prio,
                                    const int64_t *ts, size_t n, uint64_t *out, int simple,
                                    const std::vector<sga::LimiterPass> &lims) {
    constexpr size_t C = Engine::kPipeChunk, K = Engine::kPipeSlots;
    constexpr size_t kIn = Engine::kPipeIn;
    g.ensure_pipe_staging();
    sga::HostPool &pool = g.host_pool;
    const int T = pool.size();
    std::vector<int64_t> tmin(T), tmax(T);
    std::vector<uint8_t> tbad(T);
    const int64_t t0 = ts[0];
    int64_t lo = INT64_MAX, hi = INT64_MIN;  // deltas
    bool bad = false;
    const size_t nch = (n + C - 1) / C;
    static const bool dbg = getenv("SGA_PIPE_DEBUG") != nullptr;  // diagnostics only: phase times on stderr
    using clk = std::chrono::steady_clock;
    double t_fill = 0, t_win = 0, t_wout = 0, t_copy = 0;
    const auto t_start = clk::now();
    auto since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    for (size_t c = 0; c < nch; ++c) {
        const size_t s = c % K, c0 = c * C, m = std::min(C, n - c0);
        auto ta = clk::now();
        if (c >= K) SGA_HIP_CHECK(hipEventSynchronize(g.ev_pin_in[s]));  // the slot's last copy is done
        t_win += since(ta);
        ta = clk::now();
        uint8_t *slot = g.h_pin_in.p + s * C * kIn;
        int64_t *pf = reinterpret_cast<int64_t *>(slot);
        int32_t *pt = reinterpret_cast<int32_t *>(slot + 8 * C), *pa = reinterpret_cast<int32_t *>(slot + 12 * C);
        uint8_t *pp = slot + 16 * C;
        pool.run([&](int t) {
            const size_t a = m * t / T, b = m * (t + 1) / T;
            int64_t mn = INT64_MAX, mx = INT64_MIN;
            for (size_t i = a; i < b; ++i) {
                const int64_t x = ts[c0 + i] - t0;
                pt[i] = (int32_t)x;
                mn = std::min(mn, x);
                mx = std::max(mx, x);
            }
            tmin[t] = mn;
            tmax[t] = mx;
            tbad[t] = mn < INT32_MIN || mx > INT32_MAX || mn + t0 < 0;
            std::memcpy(pf + a, flow_id + c0 + a, (b - a) * 8);
            std::memcpy(pa + a, acquire + c0 + a, (b - a) * 4);
            if (prio) std::memcpy(pp + a, prio + c0 + a, b - a);
        });
        t_fill += since(ta);
        for (int t = 0; t < T; ++t) {
            lo = std::min(lo, tmin[t]);
            hi = std::max(hi, tmax[t]);
            bad |= tbad[t] != 0;
        }
        SGA_HIP_CHECK(hipMemcpyAsync(g.d_in_fid.p + c0, pf, m * 8, hipMemcpyHostToDevice, g.stream));
        SGA_HIP_CHECK(hipMemcpyAsync(g.d_tsd.p + c0, pt, m * 4, hipMemcpyHostToDevice, g.stream));
        SGA_HIP_CHECK(hipMemcpyAsync(g.d_in_acq.p + c0, pa, m * 4, hipMemcpyHostToDevice, g.stream));
        if (prio) SGA_HIP_CHECK(hipMemcpyAsync(g.d_in_prio.p + c0, pp, m, hipMemcpyHostToDevice, g.stream));
        SGA_HIP_CHECK(hipEventRecord(g.ev_pin_in[s], g.stream));
    }
    if (bad) {  // a negative time (LeapArray.currentWindow(t < 0) returns null: -EINVAL from the chunked path)
        SGA_HIP_CHECK(hipStreamSynchronize(g.stream));  // or a delta past int32: the chunked path
        return 1;
    }
    if (!prio) SGA_HIP_CHECK(hipMemsetAsync(g.d_in_prio.p, 0, n, g.stream));
    sga::cluster_ts_offsets(g.d_tsd.p, lo, g.d_in_ts.p, (uint32_t)n, g.stream);
    sga::cluster_decide_batch(g.state(), g.scratch, g.d_in_fid.p, g.d_in_acq.p, g.d_in_prio.p, t0 + lo, g.d_in_ts.p,
                              (uint32_t)n, simple, g.d_out.p, g.stream, lims.data(), (int)lims.size());
    SGA_HIP_CHECK(hipGetLastError());
    auto d2h = [&](size_t c) {
        const size_t s = c % K, c0 = c * C, m = std::min(C, n - c0);
        SGA_HIP_CHECK(hipMemcpyAsync(g.h_pin_out.p + s * C * 8, g.d_out.p + c0, m * 8, hipMemcpyDeviceToHost,
                                     g.stream));
        SGA_HIP_CHECK(hipEventRecord(g.ev_pin_out[s], g.stream));
    };
    const double t_queued = since(t_start);
    for (size_t c = 0; c < std::min(K, nch); ++c) d2h(c);
    for (size_t c = 0; c < nch; ++c) {
        const size_t s = c % K, c0 = c * C, m = std::min(C, n - c0);
        auto ta = clk::now();
        SGA_HIP_CHECK(hipEventSynchronize(g.ev_pin_out[s]));
        t_wout += since(ta);
        ta = clk::now();
        const uint64_t *src = reinterpret_cast<const uint64_t *>(g.h_pin_out.p + s * C * 8);
        pool.run([&](int t) {
            const size_t a = m * t / T, b = m * (t + 1) / T;
            std::memcpy(out + c0 + a, src + a, (b - a) * 8);
        });
        t_copy += since(ta);
        if (c + K < nch) d2h(c + K);
    }
    if (dbg)
        fprintf(stderr, "pipe n=%zu threads=%d: fill %.2f wait-in %.2f queued-at %.2f wait-out %.2f copy-out %.2f total %.2f ms\n",
                n, T, t_fill, t_win, t_queued, t_wout, t_copy, since(t_start));
    if (sga::radix64_lookback()) {
        uint32_t err = 0;
        SGA_HIP_CHECK(hipMemcpy(&err, g.scratch.radix.err, 4, hipMemcpyDeviceToHost));
        if (err) {
            g.err = "radix look-back timed out";
            return SGA_EIO;
        }
    }
    return SGA_OK;
}

// One engine batch whose arrays all lie in sga_host_register'ed buffers: DMA straight from and to them
// (21 B in, 8 B out per request); the times' min / max come from a device reduction (one 16-byte read
// back), the offsets from the minimum are computed on the device.  Returns 1 (nothing decided) when the
// times span more than u32 offsets or one is negative.
static int run_host_batch_registered(Engine &g, const int64_t *flow_id, const int32_t *acquire, const uint8_t *prio,
                                     const int64_t *ts, size_t n, uint64_t *out, int simple,
                                     const std::vector<sga::LimiterPass> &lims) {
    if (g.d_ts64.n < g.cfg.max_batch) g.d_ts64.alloc(g.cfg.max_batch);
    if (!g.d_tminmax.p) g.d_tminmax.alloc(2);
    SGA_HIP_CHECK(hipMemcpyAsync(g.d_ts64.p, ts, n * 8, hipMemcpyHostToDevice, g.stream));
    sga::cluster_ts_minmax(g.d_ts64.p, (uint32_t)n, g.d_tminmax.p, g.stream);
    int64_t mm[2];
    SGA_HIP_CHECK(hipMemcpyAsync(mm, g.d_tminmax.p, 16, hipMemcpyDeviceToHost, g.stream));
    SGA_HIP_CHECK(hipMemcpyAsync(g.d_in_fid.p, flow_id, n * 8, hipMemcpyHostToDevice, g.stream));
    SGA_HIP_CHECK(hipMemcpyAsync(g.d_in_acq.p, acquire, n * 4, hipMemcpyHostToDevice, g.stream));
    if (prio) SGA_HIP_CHECK(hipMemcpyAsync(g.d_in_prio.p, prio, n, hipMemcpyHostToDevice, g.stream));
    else SGA_HIP_CHECK(hipMemsetAsync(g.d_in_prio.p, 0, n, g.stream));
    SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
    if (mm[0] < 0 || mm[1] - mm[0] > (int64_t)0xFFFFFFFFLL) return 1;
    sga::cluster_ts_offsets64(g.d_ts64.p, mm[0], g.d_in_ts.p, (uint32_t)n, g.stream);
    sga::cluster_decide_batch(g.state(), g.scratch, g.d_in_fid.p, g.d_in_acq.p, g.d_in_prio.p, mm[0], g.d_in_ts.p,
                              (uint32_t)n, simple, g.d_out.p, g.stream, lims.data(), (int)lims.size());
    SGA_HIP_CHECK(hipGetLastError());
    SGA_HIP_CHECK(hipMemcpyAsync(out, g.d_out.p, n * 8, hipMemcpyDeviceToHost, g.stream));
    SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
    if (sga::radix64_lookback()) {
        uint32_t err = 0;
        SGA_HIP_CHECK(hipMemcpy(&err, g.scratch.radix.err, 4, hipMemcpyDeviceToHost));
        if (err) {
            g.err = "radix look-back timed out";
            return SGA_EIO;
        }
    }
    return SGA_OK;
}

static int run_host_batch(Engine &g, const int64_t *flow_id, const int32_t *acquire, const uint8_t *prio,
                          const int64_t *ts, size_t n, uint64_t *out, int simple) {
    SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
    const size_t cap = g.cfg.max_batch;
    if (g.d_in_fid.n < cap) {
        g.d_in_fid.alloc(cap);
        g.d_in_acq.alloc(cap);
        g.d_in_prio.alloc(cap);
        g.d_in_ts.alloc(cap);
        g.d_out.alloc(cap);
    }
    std::vector<uint32_t> off;
    const auto lims = limiter_passes(g);
    if (n <= std::min(Engine::kSmallStage, cap) && n > 0) {  // one staged copy each way
        int64_t lo = ts[0], hi = ts[0];
        for (size_t i = 0; i < n; ++i) {
            if (ts[i] < 0) return SGA_EINVAL;  // LeapArray.currentWindow(t < 0) returns null
            lo = std::min(lo, ts[i]);
            hi = std::max(hi, ts[i]);
        }
        if (hi - lo <= (int64_t)0xFFFFFFFFLL) {
            const size_t cap_b = Engine::kSmallStage * 17;
            if (!g.h_stage.p) {
                g.h_stage.alloc(cap_b);
                g.h_res.alloc(Engine::kSmallStage * 8);
                g.d_stage.alloc(cap_b);
            }
            uint8_t *h = g.h_stage.p;
            std::memcpy(h, flow_id, n * 8);
            std::memcpy(h + 8 * n, acquire, n * 4);
            uint32_t *to = reinterpret_cast<uint32_t *>(h + 12 * n);
            for (size_t i = 0; i < n; ++i) to[i] = (uint32_t)(ts[i] - lo);
            if (prio) std::memcpy(h + 16 * n, prio, n);
            else std::memset(h + 16 * n, 0, n);
            SGA_HIP_CHECK(hipMemcpyAsync(g.d_stage.p, h, 17 * n, hipMemcpyHostToDevice, g.stream));
            uint8_t *d = g.d_stage.p;
            sga::cluster_decide_batch(g.state(), g.scratch, reinterpret_cast<const int64_t *>(d),
                                      reinterpret_cast<const int32_t *>(d + 8 * n), d + 16 * n, lo,
                                      reinterpret_cast<const uint32_t *>(d + 12 * n), (uint32_t)n, simple, g.d_out.p,
                                      g.stream, lims.data(), (int)lims.size());
            SGA_HIP_CHECK(hipGetLastError());
            SGA_HIP_CHECK(hipMemcpyAsync(g.h_res.p, g.d_out.p, n * 8, hipMemcpyDeviceToHost, g.stream));
            SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
            std::memcpy(out, g.h_res.p, n * 8);
            if (sga::radix64_lookback()) {
                uint32_t err = 0;
                SGA_HIP_CHECK(hipMemcpy(&err, g.scratch.radix.err, 4, hipMemcpyDeviceToHost));
                if (err) {
                    g.err = "radix look-back timed out";
                    return SGA_EIO;
                }
            }
            return SGA_OK;
        }
    }
    if (n >= Engine::kPipeChunk && n <= cap) {
        const bool reg = !g.host_regs.empty() && g.registered(flow_id, n * 8) && g.registered(acquire, n * 4) &&
                         g.registered(ts, n * 8) && g.registered(out, n * 8) && (!prio || g.registered(prio, n));
        const int rc = reg ? run_host_batch_registered(g, flow_id, acquire, prio, ts, n, out, simple, lims)
                           : run_host_batch_pipelined(g, flow_id, acquire, prio, ts, n, out, simple, lims);
        if (rc != 1) return rc;  // 1: the batch's times span more than u32 offsets: the chunked path below
    }
    for (size_t b = 0; b < n;) {
        // chunk: at most cap events and a timestamp span that fits u32 offsets
        size_t m = std::min(cap, n - b);
        int64_t lo = ts[b], hi = ts[b];
        for (size_t i = 0; i < m; ++i) {
            const int64_t t = ts[b + i];
            if (t < 0) return SGA_EINVAL;  // LeapArray.currentWindow(t < 0) returns null
            const int64_t nlo = std::min(lo, t), nhi = std::max(hi, t);
            if (nhi - nlo > (int64_t)0xFFFFFFFFLL) {
                m = i;
                break;
            }
            lo = nlo;
            hi = nhi;
        }
        off.resize(m);
        for (size_t i = 0; i < m; ++i) off[i] = (uint32_t)(ts[b + i] - lo);
        SGA_HIP_CHECK(hipMemcpyAsync(g.d_in_fid.p, flow_id + b, m * 8, hipMemcpyHostToDevice, g.stream));
        SGA_HIP_CHECK(hipMemcpyAsync(g.d_in_acq.p, acquire + b, m * 4, hipMemcpyHostToDevice, g.stream));
        if (prio) SGA_HIP_CHECK(hipMemcpyAsync(g.d_in_prio.p, prio + b, m, hipMemcpyHostToDevice, g.stream));
        else SGA_HIP_CHECK(hipMemsetAsync(g.d_in_prio.p, 0, m, g.stream));
        SGA_HIP_CHECK(hipMemcpyAsync(g.d_in_ts.p, off.data(), m * 4, hipMemcpyHostToDevice, g.stream));
        sga::cluster_decide_batch(g.state(), g.scratch, g.d_in_fid.p, g.d_in_acq.p, g.d_in_prio.p, lo, g.d_in_ts.p,
                                  (uint32_t)m, simple, g.d_out.p, g.stream, lims.data(), (int)lims.size());
        SGA_HIP_CHECK(hipGetLastError());
        SGA_HIP_CHECK(hipMemcpyAsync(out + b, g.d_out.p, m * 8, hipMemcpyDeviceToHost, g.stream));
        SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
        if (sga::radix64_lookback()) {  // a look-back that gave up would have sorted wrongly
            uint32_t err = 0;
            SGA_HIP_CHECK(hipMemcpy(&err, g.scratch.radix.err, 4, hipMemcpyDeviceToHost));
            if (err) {
                g.err = "radix look-back timed out";
                return SGA_EIO;
            }
        }
        b += m;
    }
    return SGA_OK;
}

int sga_host_register(sga_engine *e, void *ptr, size_t bytes) {
    if (!ptr || bytes == 0) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        if (hipHostRegister(ptr, bytes, hipHostRegisterDefault) != hipSuccess) {
            (void)hipGetLastError();
            g.err = "hipHostRegister failed";
            return SGA_ENOMEM;
        }
        g.host_regs.emplace_back((uintptr_t)ptr, (uintptr_t)ptr + bytes);
        return SGA_OK;
    });
}

int sga_host_unregister(sga_engine *e, void *ptr) {
    if (!ptr) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        for (size_t i = 0; i < g.host_regs.size(); ++i)
            if (g.host_regs[i].first == (uintptr_t)ptr) {
                SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
                (void)hipHostUnregister(ptr);
                g.host_regs.erase(g.host_regs.begin() + (long)i);
                return SGA_OK;
            }
        return SGA_EINVAL;
    });
}

int sga_request_tokens(sga_engine *e, const int64_t *flow_id, const int32_t *acquire, const uint8_t *prio,
                       const int64_t *ts, size_t n, sga_token_result *out) {
    if (n && (!flow_id || !acquire || !ts || !out)) return SGA_EINVAL;
    static_assert(sizeof(sga_token_result) == 8, "token result is 8 bytes");
    return guarded(e, [&](Engine &g) {
        return run_host_batch(g, flow_id, acquire, prio, ts, n, (uint64_t *)out, 0);
    });
}

// ---- coalescing queue (TokenQueue above)
static int combine_round(sga_engine *e);

int sga_token_submit(sga_engine *e, int64_t flow_id, int32_t acquire, uint8_t prioritized, int64_t ts,
                     uint64_t *ticket) {
    if (!e || !ticket) return SGA_EINVAL;
    // what would fail the whole coalesced batch is refused here, for this caller only (the engine
    // answers an invalid flowId / acquireCount with BAD_REQUEST inside the batch)
    if (ts < 0) return SGA_EINVAL;
    sga::TokenQueue &q = e->impl.tq;
    const uint64_t t = q.tail.fetch_add(1, std::memory_order_relaxed);
    sga::TokenQueue::Slot &sl = q.ring[t & (sga::TokenQueue::kCap - 1)];
    // The slot still holds ticket t - kCap.  Decided but never polled (its caller gave up): reclaim it --
    // a later sga_poll of that ticket answers SGA_EINVAL.  Filled but not decided: decide it (this caller
    // becomes the combiner if none is running).  Free but not yet filled by its producer: wait for it.
    const uint64_t prev = t - sga::TokenQueue::kCap;
    for (int spin = 0;; ++spin) {
        uint64_t s = sl.seq.load(std::memory_order_acquire);
        if (s == t) break;
        if (t >= sga::TokenQueue::kCap && s == prev + 2 &&
            sl.seq.compare_exchange_strong(s, t, std::memory_order_acq_rel))
            break;
        if (t >= sga::TokenQueue::kCap && s == prev + 1) (void)combine_round(e);
        else if (spin > 64) std::this_thread::yield();
    }
    sl.flow_id = flow_id;
    sl.acquire = acquire;
    sl.prio = prioritized ? 1 : 0;
    sl.ts = ts;
    sl.seq.store(t + 1, std::memory_order_release);
    *ticket = t;
    return SGA_OK;
}

// One combining round: decide every filled slot from the head as one batch (at most max_batch).
// Returns the engine status of the batch (results of a failed batch carry TokenResultStatus.FAIL).
static int combine_round(sga_engine *e) {
    sga::TokenQueue &q = e->impl.tq;
    bool expect = false;
    if (!q.combining.compare_exchange_strong(expect, true, std::memory_order_acquire)) return SGA_OK;
    const uint64_t h = q.head;
    const uint64_t cap = std::min<uint64_t>(e->impl.cfg.max_batch, sga::TokenQueue::kCap);
    uint64_t k = 0;
    q.fid.clear();
    q.acq.clear();
    q.prio.clear();
    q.ts.clear();
    while (k < cap) {
        sga::TokenQueue::Slot &sl = q.ring[(h + k) & (sga::TokenQueue::kCap - 1)];
        if (sl.seq.load(std::memory_order_acquire) != h + k + 1) break;  // not filled yet: next round
        q.fid.push_back(sl.flow_id);
        q.acq.push_back(sl.acquire);
        q.prio.push_back(sl.prio);
        q.ts.push_back(sl.ts);
        ++k;
    }
    int rc = SGA_OK;
    if (k) {
        q.out.assign(k, 0);
        rc = sga_request_tokens(e, q.fid.data(), q.acq.data(), q.prio.data(), q.ts.data(), k,
                                reinterpret_cast<sga_token_result *>(q.out.data()));
        for (uint64_t j = 0; j < k; ++j) {
            sga::TokenQueue::Slot &sl = q.ring[(h + j) & (sga::TokenQueue::kCap - 1)];
            if (rc == SGA_OK) {
                sl.result = q.out[j];
            } else {  // TokenResultStatus.FAIL (-1) in the status byte
                sga_token_result r{};
                r.status = -1;
                std::memcpy(&sl.result, &r, sizeof(r));
            }
            sl.seq.store(h + j + 2, std::memory_order_release);
        }
        q.head = h + k;
    }
    q.combining.store(false, std::memory_order_release);
    return rc;
}

int sga_poll(sga_engine *e, uint64_t ticket, sga_token_result *out) {
    if (!e || !out) return SGA_EINVAL;
    sga::TokenQueue &q = e->impl.tq;
    sga::TokenQueue::Slot &sl = q.ring[ticket & (sga::TokenQueue::kCap - 1)];
    for (int pass = 0; pass < 2; ++pass) {
        uint64_t s = sl.seq.load(std::memory_order_acquire);
        if (s == ticket + 2) {
            sga_token_result r;
            std::memcpy(&r, &sl.result, sizeof(r));
            // a producer kCap tickets later may reclaim the slot at the same time (sga_token_submit)
            if (!sl.seq.compare_exchange_strong(s, ticket + sga::TokenQueue::kCap, std::memory_order_acq_rel))
                return SGA_EINVAL;
            *out = r;
            return SGA_OK;
        }
        if (s != ticket + 1) return SGA_EINVAL;  // not a live ticket
        if (pass == 0) (void)combine_round(e);
    }
    return SGA_EAGAIN;
}

int sga_request_token_one(sga_engine *e, int64_t flow_id, int32_t acquire, uint8_t prioritized, int64_t ts,
                          sga_token_result *out) {
    if (!e || !out) return SGA_EINVAL;
    uint64_t t = 0;
    int rc = sga_token_submit(e, flow_id, acquire, prioritized, ts, &t);
    if (rc != SGA_OK) return rc;
    for (int spin = 0;; ++spin) {
        rc = sga_poll(e, t, out);
        if (rc != SGA_EAGAIN) return rc;
        if (spin > 16) std::this_thread::yield();
    }
}

// ---- coalescing queue of local events (EventQueue above)
static int event_combine_round(sga_engine *e);
static thread_local bool tl_in_combiner = false;

static int event_enqueue(sga_engine *e, uint8_t kind, uint32_t resource, int64_t ts, int32_t acquire, uint8_t flags,
                         int64_t rt, uint64_t param, const uint64_t *param_values, size_t n_values, uint64_t *ticket,
                         bool posted) {
    if (!e || !ticket) return SGA_EINVAL;
    // refused here, for this caller only, what would fail the whole coalesced batch
    if (ts < 0 || acquire < 0 || kind > SGA_KIND_REVOKE) return SGA_EINVAL;
    const bool args = (flags & SGA_EV_ARGS) != 0;
    const bool list = !args && (flags & (SGA_EV_PARAM_LIST | SGA_EV_HAS_PARAM)) == (SGA_EV_PARAM_LIST | SGA_EV_HAS_PARAM);
    if (args || list) {
        if (n_values > sga::EventQueue::kWords) return SGA_ERANGE;  // the caller submits it directly
        if (n_values && !param_values) return SGA_EINVAL;
        const uint64_t off = param >> 32, na = param & 0xFFFFFFFFu;
        if (list && off + na > n_values) return SGA_EINVAL;
        if (args) {
            if (off + 2 * na > n_values) return SGA_EINVAL;
            for (uint64_t k = 0; k < na; ++k) {
                const uint64_t h = param_values[off + 2 * k], w = param_values[off + 2 * k + 1];
                if ((h >> 62) > 2 || ((h >> 62) == SGA_ARG_LIST && w + (h & 0xFFFFFFFFu) > n_values)) return SGA_EINVAL;
            }
        }
    }
    sga::EventQueue &q = e->impl.eq;
    const uint64_t t = q.tail.fetch_add(1, std::memory_order_relaxed);
    sga::EventQueue::Slot &sl = q.ring[t & (sga::EventQueue::kCap - 1)];
    const uint64_t prev = t - sga::EventQueue::kCap;  // as sga_token_submit: reclaim, decide or wait
    for (int spin = 0;; ++spin) {
        uint64_t s = sl.seq.load(std::memory_order_acquire);
        if (s == t) break;
        if (t >= sga::EventQueue::kCap && s == prev + 2 &&
            sl.seq.compare_exchange_strong(s, t, std::memory_order_acq_rel))
            break;
        if (t >= sga::EventQueue::kCap && s == prev + 1) (void)event_combine_round(e);
        else if (spin > 64) std::this_thread::yield();
    }
    sl.kind = kind;
    sl.resource = resource;
    sl.ts = ts;
    sl.acquire = acquire;
    sl.flags = flags;
    sl.rt = rt;
    sl.param = param;
    sl.nwords = (args || list) ? (uint32_t)n_values : 0u;
    if (sl.nwords) std::memcpy(sl.words, param_values, sl.nwords * 8);
    sl.posted = posted;
    sl.seq.store(t + 1, std::memory_order_release);
    *ticket = t;
    return SGA_OK;
}

int sga_event_submit(sga_engine *e, uint8_t kind, uint32_t resource, int64_t ts, int32_t acquire, uint8_t flags,
                     int64_t rt, uint64_t param, const uint64_t *param_values, size_t n_values, uint64_t *ticket) {
    return event_enqueue(e, kind, resource, ts, acquire, flags, rt, param, param_values, n_values, ticket, false);
}

int sga_event_post(sga_engine *e, uint8_t kind, uint32_t resource, int64_t ts, int32_t acquire, uint8_t flags,
                   int64_t rt, uint64_t param, const uint64_t *param_values, size_t n_values, uint64_t *ticket) {
    if (!e || kind == SGA_KIND_ENTRY) return SGA_EINVAL;  // an entry's caller needs its decision
    uint64_t t = 0;
    const int rc = event_enqueue(e, kind, resource, ts, acquire, flags, rt, param, param_values, n_values, &t, true);
    if (rc == SGA_ERANGE) {  // more argument words than a queue slot holds: its own batch, after the queued ones
        int8_t d = 0;
        int32_t w = 0;
        if (ticket) *ticket = ~0ull;
        return sga_submit_events_ex(e, &kind, &resource, &ts, &acquire, &flags, &rt, &param, 1, param_values,
                                    n_values, &d, &w);
    }
    if (rc != SGA_OK) return rc;
    if (ticket) *ticket = t;
    return e->impl.eq.post_err.exchange(false) ? SGA_EIO : SGA_OK;
}

// One combining round: every filled slot from the head as one sga_submit_events_ex batch (at most max_batch);
// each slot's argument words appended to one value array, their offsets rebased.
static int event_combine_round(sga_engine *e) {
    sga::EventQueue &q = e->impl.eq;
    bool expect = false;
    if (!q.combining.compare_exchange_strong(expect, true, std::memory_order_acquire)) return SGA_OK;
    const uint64_t h = q.head;
    const uint64_t cap = std::min<uint64_t>(e->impl.cfg.max_batch, sga::EventQueue::kCap);
    uint64_t k = 0;
    q.kind.clear();
    q.flags.clear();
    q.res.clear();
    q.ts.clear();
    q.rt.clear();
    q.acq.clear();
    q.param.clear();
    q.vals.clear();
    while (k < cap) {
        sga::EventQueue::Slot &sl = q.ring[(h + k) & (sga::EventQueue::kCap - 1)];
        if (sl.seq.load(std::memory_order_acquire) != h + k + 1) break;  // not filled yet: next round
        uint64_t pv = sl.param;
        if (sl.nwords) {
            const uint64_t base = q.vals.size();
            q.vals.insert(q.vals.end(), sl.words, sl.words + sl.nwords);
            if (sl.flags & SGA_EV_ARGS) {
                const uint64_t off = pv >> 32, na = pv & 0xFFFFFFFFu;
                for (uint64_t j = 0; j < na; ++j)
                    if ((q.vals[base + off + 2 * j] >> 62) == SGA_ARG_LIST) q.vals[base + off + 2 * j + 1] += base;
            }
            pv = (((pv >> 32) + base) << 32) | (pv & 0xFFFFFFFFu);
        }
        q.kind.push_back(sl.kind);
        q.flags.push_back(sl.flags);
        q.res.push_back(sl.resource);
        q.ts.push_back(sl.ts);
        q.rt.push_back(sl.rt);
        q.acq.push_back(sl.acquire);
        q.param.push_back(pv);
        ++k;
    }
    int rc = SGA_OK;
    if (k) {
        q.dec.assign(k, 0);
        q.wait.assign(k, 0);
        tl_in_combiner = true;  // the batch's own call must not wait for the queue it is draining
        rc = sga_submit_events_ex(e, q.kind.data(), q.res.data(), q.ts.data(), q.acq.data(), q.flags.data(),
                                  q.rt.data(), q.param.data(), k, q.vals.empty() ? nullptr : q.vals.data(),
                                  q.vals.size(), q.dec.data(), q.wait.data());
        tl_in_combiner = false;
        bool posted_failed = false;
        for (uint64_t j = 0; j < k; ++j) {
            sga::EventQueue::Slot &sl = q.ring[(h + j) & (sga::EventQueue::kCap - 1)];
            if (sl.posted) {  // nobody polls it: free the slot for the ticket kCap later
                posted_failed |= rc != SGA_OK;
                sl.seq.store(h + j + sga::EventQueue::kCap, std::memory_order_release);
                continue;
            }
            sl.decision = rc == SGA_OK ? q.dec[j] : (int8_t)-1;  // a failed batch: -1 for every event
            sl.wait = rc == SGA_OK ? q.wait[j] : 0;
            sl.seq.store(h + j + 2, std::memory_order_release);
        }
        if (posted_failed) q.post_err.store(true, std::memory_order_release);
        q.head = h + k;
        q.done.store(h + k, std::memory_order_release);
    }
    q.combining.store(false, std::memory_order_release);
    return rc;
}

// Every event queued before this call decided (rounds run by this thread or another).  Not inside a round's own
// batch call (tl_in_combiner).
static void event_flush(sga_engine *e) {
    if (tl_in_combiner) return;
    sga::EventQueue &q = e->impl.eq;
    const uint64_t t = q.tail.load(std::memory_order_acquire);
    for (int spin = 0; q.done.load(std::memory_order_acquire) < t; ++spin) {
        (void)event_combine_round(e);
        if (spin > 16) std::this_thread::yield();
    }
}

int sga_event_poll(sga_engine *e, uint64_t ticket, int8_t *decision, int32_t *wait_ms) {
    if (!e || !decision) return SGA_EINVAL;
    sga::EventQueue &q = e->impl.eq;
    sga::EventQueue::Slot &sl = q.ring[ticket & (sga::EventQueue::kCap - 1)];
    for (int pass = 0; pass < 2; ++pass) {
        uint64_t s = sl.seq.load(std::memory_order_acquire);
        if (s == ticket + 2) {
            const int8_t d = sl.decision;
            const int32_t w = sl.wait;
            if (!sl.seq.compare_exchange_strong(s, ticket + sga::EventQueue::kCap, std::memory_order_acq_rel))
                return SGA_EINVAL;
            *decision = d;
            if (wait_ms) *wait_ms = w;
            return d < 0 ? SGA_EIO : SGA_OK;
        }
        if (s != ticket + 1) return SGA_EINVAL;  // not a live ticket
        if (pass == 0) (void)event_combine_round(e);
    }
    return SGA_EAGAIN;
}

int sga_event_one(sga_engine *e, uint8_t kind, uint32_t resource, int64_t ts, int32_t acquire, uint8_t flags,
                  int64_t rt, uint64_t param, const uint64_t *param_values, size_t n_values, int8_t *decision,
                  int32_t *wait_ms) {
    if (!e || !decision) return SGA_EINVAL;
    uint64_t t = 0;
    int rc = sga_event_submit(e, kind, resource, ts, acquire, flags, rt, param, param_values, n_values, &t);
    if (rc == SGA_ERANGE)  // more argument words than a queue slot holds: its own batch
        return sga_submit_events_ex(e, &kind, &resource, &ts, &acquire, &flags, &rt, &param, 1, param_values,
                                    n_values, decision, wait_ms);
    if (rc != SGA_OK) return rc;
    for (int spin = 0;; ++spin) {
        rc = sga_event_poll(e, t, decision, wait_ms);
        if (rc != SGA_EAGAIN) return rc;
        if (spin > 16) std::this_thread::yield();
    }
}

int sga_cluster_metric_sums(sga_engine *e, int64_t flow_id, int64_t now, int64_t *out7) {
    if (!out7 || now < 0) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        auto it = g.slot_of.find(flow_id);
        if (it == g.slot_of.end()) return SGA_EINVAL;
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        sga::cluster_metric_sums(g.state(), it->second, now, g.d_tmp7.p, g.stream);
        SGA_HIP_CHECK(hipMemcpyAsync(out7, g.d_tmp7.p, 7 * 8, hipMemcpyDeviceToHost, g.stream));
        SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
        return SGA_OK;
    });
}

// ClusterParamFlowRuleManager.applyClusterParamRules, CS/flow/rule/ClusterParamFlowRuleManager.java:318-368
int sga_load_cluster_param_rules(sga_engine *e, const char *ns, const sga_cluster_param_rule *rules, size_t n) {
    if (!ns || !*ns || (n && !rules)) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        g.ensure_param_store();
        const int nsi = g.ns_index(ns, true);
        std::vector<uint32_t> fresh;
        if (n == 0) {  // clearAndResetRulesFor (:195-207): rules dropped, metrics kept
            for (auto &h : g.pslots)
                if (h.allocated && h.ns == nsi) h.active = false;
            g.sync_param_device(fresh);
            return 0;
        }
        std::unordered_map<int64_t, const sga_cluster_param_rule *> rule_map;
        std::vector<int64_t> order;
        std::unordered_map<int64_t, const sga_cluster_param_rule *> first;  // putMetricIfAbsent geometry
        for (size_t i = 0; i < n; ++i) {
            const sga_cluster_param_rule &r = rules[i];
            // ParamFlowRuleUtil.isValidRule + checkCluster (PF/.../ParamFlowRuleUtil.java:46-70)
            if (!(r.count >= 0 && r.grade >= 0 && r.param_idx_set && r.burst_count >= 0 && r.control_behavior >= 0 &&
                  r.duration_in_sec > 0 && r.max_queueing_time_ms >= 0))
                continue;
            if (!(r.sample_count > 0 && r.window_interval_ms > 0 && r.window_interval_ms % r.sample_count == 0))
                continue;
            if (r.flow_id <= 0) continue;
            if (r.n_hot < 0 || (r.n_hot > 0 && (!r.hot_values || !r.hot_counts))) return SGA_EINVAL;
            if (!rule_map.count(r.flow_id)) {
                order.push_back(r.flow_id);
                first[r.flow_id] = &r;
            }
            rule_map[r.flow_id] = &r;  // ruleMap.put: last one wins
        }
        // clearAndResetRulesConditional: ids of this namespace not in the new map lose rule AND metric
        for (auto &h : g.pslots) {
            if (!h.allocated || h.ns != nsi || !h.active) continue;
            if (rule_map.count(h.flow_id)) continue;
            h.active = false;
            h.allocated = false;
            g.pslot_of.erase(h.flow_id);
            if (h.lru_words) {  // the metric's LRU queue areas go back to the pool
                g.plpool_free[h.lru_words].push_back(h.lru_off);
                h.lru_words = 0;
            }
            // the dead slot's device state (queue pointers, starts, key count) is reset before its area can
            // be handed to another rule: k_plru_collect must never see the dead rule's keys as queued
            fresh.push_back((uint32_t)(&h - g.pslots.data()));
        }
        for (int64_t fid : order) {
            const sga_cluster_param_rule &r = *rule_map[fid];
            auto it = g.pslot_of.find(fid);
            uint32_t sl;
            if (it == g.pslot_of.end()) {  // putMetricIfAbsent -> new ClusterParamMetric(sampleCount, windowIntervalMs)
                if (g.pslots.size() >= sga::kMaxSlots) {
                    g.err = "too many cluster parameter rules";
                    return SGA_ERANGE;
                }
                sl = (uint32_t)g.pslots.size();
                g.pslots.emplace_back();
                sga::PSlotHost &h = g.pslots.back();
                const sga_cluster_param_rule &geo = *first[fid];
                h.flow_id = fid;
                h.allocated = true;
                h.S = geo.sample_count;
                h.interval = geo.window_interval_ms;
                h.boff = g.pbucket_used;
                h.cap = g.pcap_default;
                g.pbucket_used += (uint32_t)h.S;
                g.pslot_of[fid] = sl;
                fresh.push_back(sl);
            } else {
                sl = it->second;
            }
            sga::PSlotHost &h = g.pslots[sl];
            h.active = true;
            h.ns = nsi;
            h.count = r.count;
            h.threshold_type = r.threshold_type;
            std::unordered_map<int64_t, int32_t> hot;  // parsed hotItems (HashMap: later wins)
            for (int32_t k = 0; k < r.n_hot; ++k) hot[r.hot_values[k]] = r.hot_counts[k];
            h.hot.assign(hot.begin(), hot.end());
            std::sort(h.hot.begin(), h.hot.end());
        }
        g.sync_param_device(fresh);
        return (int)order.size();
    });
}

int sga_request_param_tokens(sga_engine *e, const int64_t *flow_id, const int32_t *acquire,
                             const uint32_t *value_offsets, const int64_t *values, const int64_t *ts, size_t n,
                             sga_token_result *out) {
    if (n && (!flow_id || !acquire || !value_offsets || !ts || !out)) return SGA_EINVAL;
    if (n && value_offsets[n] > value_offsets[0] && !values) return SGA_EINVAL;
    for (size_t i = 0; i < n; ++i)
        if (value_offsets[i + 1] < value_offsets[i] || ts[i] < 0) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        g.ensure_param_store();
        const size_t cap = g.cfg.max_batch;
        if (g.d_in_fid.n < cap) {
            g.d_in_fid.alloc(cap);
            g.d_in_acq.alloc(cap);
            g.d_in_prio.alloc(cap);
            g.d_in_ts.alloc(cap);
            g.d_out.alloc(cap);
        }
        const auto lims = limiter_passes(g);
        std::vector<uint32_t> off, voff;
        for (size_t b = 0; b < n;) {
            // chunk: <= cap requests, <= cap values, timestamp span within u32 offsets
            size_t m = 0;
            int64_t lo = ts[b], hi = ts[b];
            while (b + m < n && m < cap) {
                const size_t i = b + m;
                if ((size_t)(value_offsets[i + 1] - value_offsets[b]) > cap) break;
                const int64_t nlo = std::min(lo, ts[i]), nhi = std::max(hi, ts[i]);
                if (nhi - nlo > (int64_t)0xFFFFFFFFLL) break;
                lo = nlo;
                hi = nhi;
                ++m;
            }
            if (m == 0) {
                g.err = "a request carries more parameter values than max_batch";
                return SGA_ERANGE;
            }
            off.resize(m);
            voff.resize(m + 1);
            for (size_t i = 0; i < m; ++i) off[i] = (uint32_t)(ts[b + i] - lo);
            for (size_t i = 0; i <= m; ++i) voff[i] = value_offsets[b + i] - value_offsets[b];
            const uint32_t nv = voff[m];
            SGA_HIP_CHECK(hipMemcpyAsync(g.d_in_fid.p, flow_id + b, m * 8, hipMemcpyHostToDevice, g.stream));
            SGA_HIP_CHECK(hipMemcpyAsync(g.d_in_acq.p, acquire + b, m * 4, hipMemcpyHostToDevice, g.stream));
            SGA_HIP_CHECK(hipMemcpyAsync(g.d_in_ts.p, off.data(), m * 4, hipMemcpyHostToDevice, g.stream));
            SGA_HIP_CHECK(hipMemcpyAsync(g.d_in_voff.p, voff.data(), (m + 1) * 4, hipMemcpyHostToDevice, g.stream));
            if (nv)
                SGA_HIP_CHECK(hipMemcpyAsync(g.d_in_vals.p, values + value_offsets[b], (size_t)nv * 8,
                                             hipMemcpyHostToDevice, g.stream));
            sga::CParamState st = g.pstate();
            sga::cparam_stage1(st, g.scratch, g.pscratch, g.d_in_fid.p, g.d_in_acq.p, g.d_in_voff.p, g.d_in_vals.p, lo,
                               g.d_in_ts.p, (uint32_t)m, g.d_out.p, g.stream, lims.data(), (int)lims.size());
            uint32_t ctl[5];
            SGA_HIP_CHECK(hipMemcpyAsync(ctl, g.d_pctl.p, sizeof(ctl), hipMemcpyDeviceToHost, g.stream));
            SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
            if (ctl[1]) {
                g.err = (ctl[1] & 1) ? "cluster parameter key table full (raise sga_config.max_param_keys)"
                                     : "cluster parameter record pool full (raise sga_config.max_param_keys)";
                return SGA_ENOMEM;
            }
            if (ctl[4]) {
                g.cparam_lru_switch_host(ctl[4], g.stream);
                st = g.pstate();  // the queue pool may have moved
            }
            sga::cparam_stage2(st, g.scratch, g.pscratch, g.d_in_acq.p, g.d_in_voff.p, g.d_in_vals.p, lo, g.d_in_ts.p,
                               (uint32_t)m, ctl[2], g.d_out.p, g.stream);
            SGA_HIP_CHECK(hipGetLastError());
            SGA_HIP_CHECK(hipMemcpyAsync(out + b, g.d_out.p, m * 8, hipMemcpyDeviceToHost, g.stream));
            uint32_t err = 0;
            SGA_HIP_CHECK(hipMemcpyAsync(&err, g.d_pctl.p + 1, 4, hipMemcpyDeviceToHost, g.stream));
            SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
            g.flow.seq += m;  // access stamps of the next call come after these
            if (err & 4) {
                g.err = "cluster parameter LRU queue check failed";
                return SGA_ENOMEM;
            }
            b += m;
        }
        return SGA_OK;
    });
}

int sga_cluster_set_param_capacity(sga_engine *e, uint32_t capacity) {
    if (capacity > (1u << 24)) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        g.pcap_default = capacity ? capacity : 4000;
        return SGA_OK;
    });
}

int sga_cluster_param_sum(sga_engine *e, int64_t flow_id, int64_t value, int64_t now, int64_t *out) {
    if (!out || now < 0) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        auto it = g.pslot_of.find(flow_id);
        if (it == g.pslot_of.end() || !g.d_pctl.p) return SGA_EINVAL;
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        sga::cparam_sum(g.pstate(), it->second, value, now, g.d_tmp7.p, g.stream);
        SGA_HIP_CHECK(hipMemcpyAsync(out, g.d_tmp7.p, 8, hipMemcpyDeviceToHost, g.stream));
        SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
        g.flow.seq += 1;  // getSum's gets are accesses
        return SGA_OK;
    });
}

// ClusterParamMetric.getTopValues, CS/flow/statistic/metric/ClusterParamMetric.java:90-133
int sga_cluster_param_top_values(sga_engine *e, int64_t flow_id, int64_t now, uint32_t number, int64_t *values,
                                 double *qps, uint32_t *n_out) {
    if (!values || !qps || !n_out || number == 0 || number > 1024 || now < 0) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        *n_out = 0;
        auto it = g.pslot_of.find(flow_id);
        if (it == g.pslot_of.end() || !g.d_pctl.p) return SGA_OK;  // no metric: empty map
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        const size_t nk = (size_t)g.kmask + 1;
        if (g.d_top_list.n < 2 * nk) g.d_top_list.alloc(2 * nk);
        if (g.d_top_val.n < number) {
            g.d_top_val.alloc(number);
            g.d_top_qps.alloc(number);
        }
        if (!g.d_top_n.p) g.d_top_n.alloc(2);
        sga::cparam_top_values(g.pstate(), it->second, now, number, g.d_top_list.p, g.d_top_n.p + 1, g.d_top_val.p,
                               g.d_top_qps.p, g.d_top_n.p, g.stream);
        SGA_HIP_CHECK(hipGetLastError());
        uint32_t n = 0;
        SGA_HIP_CHECK(hipMemcpyAsync(&n, g.d_top_n.p, 4, hipMemcpyDeviceToHost, g.stream));
        SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
        if (n) {
            SGA_HIP_CHECK(hipMemcpy(values, g.d_top_val.p, n * 8, hipMemcpyDeviceToHost));
            SGA_HIP_CHECK(hipMemcpy(qps, g.d_top_qps.p, n * 8, hipMemcpyDeviceToHost));
        }
        *n_out = n;
        return SGA_OK;
    });
}

int sga_cluster_stats(sga_engine *e, uint64_t *n_active, uint64_t *state_bytes) {
    return guarded(e, [&](Engine &g) {
        uint64_t a = 0;
        for (auto &h : g.slots) a += h.active ? 1 : 0;
        if (n_active) *n_active = a;
        if (state_bytes)
            *state_bytes = (uint64_t)g.bucket_used * 64 + g.slots.size() * sizeof(sga::SlotParam);
        return SGA_OK;
    });
}

// Path taken by the last token batch (engine diagnostics, no reference counterpart).
int sga_cluster_batch_info(sga_engine *e, uint32_t *out, size_t n) {
    if (!out || n == 0) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        uint32_t c[sga::CTL_WORDS];
        uint32_t hc[8];
        // a hot-path batch leaves its words in counters_last (k_hot_fin clears the live ones)
        const sga::BatchScratch &ls = *g.last_sc;
        const uint32_t *src = ls.counters_clean ? ls.counters_last : ls.counters;
        SGA_HIP_CHECK(hipMemcpyAsync(c, src, sizeof(c), hipMemcpyDeviceToHost, g.stream));
        SGA_HIP_CHECK(hipMemcpyAsync(hc, ls.hot_ctl, sizeof(hc), hipMemcpyDeviceToHost, g.stream));
        SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
        const uint32_t v[11] = {c[sga::CTL_MODE],  c[sga::CTL_FLAGS], c[sga::CTL_NSORT], c[sga::CTL_NCOLD],
                                c[sga::CTL_NPRIO], hc[0],             c[sga::CTL_BDLO],  c[sga::CTL_BDHI],
                                c[sga::CTL_HOTERR], c[sga::CTL_NPRE], (uint32_t)g.scratch.hot_lane_order};
        for (size_t i = 0; i < n && i < 11; ++i) out[i] = v[i];
        return SGA_OK;
    });
}

// ---------------------------------------------------------------- concurrency tokens
// DefaultTokenService.requestConcurrentToken / releaseConcurrentToken (CS/flow/DefaultTokenService.java:67-86)
int sga_concurrent_ops(sga_engine *e, const uint8_t *op, const uint32_t *client, const int64_t *id,
                       const int32_t *acquire, const int64_t *ts, size_t n, sga_concurrent_result *out) {
    if (n && (!op || !client || !id || !acquire || !ts || !out)) return SGA_EINVAL;
    static_assert(sizeof(sga_concurrent_result) == 16, "concurrent result is 16 bytes");
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        g.ensure_conc();
        g.ensure_scratch();
        const size_t cap = g.cfg.max_batch;
        for (size_t b = 0; b < n;) {
            const size_t m = std::min(cap, n - b);
            size_t nacq = 0;
            for (size_t i = 0; i < m; ++i) {
                if (op[b + i] > 1) return SGA_EINVAL;
                nacq += op[b + i] == 0;
            }
            if (!g.reserve_tokens(nacq)) {
                g.err = "token cache above 2^29 tokens";
                return SGA_ENOMEM;
            }
            SGA_HIP_CHECK(hipMemcpyAsync(g.d_cin_op.p, op + b, m, hipMemcpyHostToDevice, g.stream));
            SGA_HIP_CHECK(hipMemcpyAsync(g.d_cin_client.p, client + b, m * 4, hipMemcpyHostToDevice, g.stream));
            SGA_HIP_CHECK(hipMemcpyAsync(g.d_cin_id.p, id + b, m * 8, hipMemcpyHostToDevice, g.stream));
            SGA_HIP_CHECK(hipMemcpyAsync(g.d_cin_acq.p, acquire + b, m * 4, hipMemcpyHostToDevice, g.stream));
            SGA_HIP_CHECK(hipMemcpyAsync(g.d_cin_ts.p, ts + b, m * 8, hipMemcpyHostToDevice, g.stream));
            ++g.tepoch;
            sga::conc_ops(g.cstate(), g.cscratch, g.d_cin_op.p, g.d_cin_client.p, g.d_cin_id.p, g.d_cin_acq.p,
                          g.d_cin_ts.p, (uint32_t)m, g.token_base, g.d_cout.p, g.stream);
            SGA_HIP_CHECK(hipGetLastError());
            g.token_base += m;
            SGA_HIP_CHECK(hipMemcpyAsync(out + b, g.d_cout.p, m * sizeof(sga_concurrent_result), hipMemcpyDeviceToHost,
                                         g.stream));
            SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
            g.read_token_counters();
            if (sga::radix64_lookback()) {
                uint32_t err = 0;
                SGA_HIP_CHECK(hipMemcpy(&err, g.cscratch.radix.err, 4, hipMemcpyDeviceToHost));
                if (err) {
                    g.err = "radix look-back timed out";
                    return SGA_EIO;
                }
            }
            b += m;
        }
        return SGA_OK;
    });
}

// RegularExpireStrategy.clearToken, CS/flow/statistic/concurrent/expire/RegularExpireStrategy.java:78-134
int sga_concurrent_expire(sga_engine *e, int64_t now, const uint32_t *online_bits, uint32_t n_clients,
                          uint64_t *n_removed) {
    if (n_clients && !online_bits) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        g.ensure_conc();
        const size_t words = std::max<size_t>(((size_t)n_clients + 31) / 32, 1);
        if (g.d_online.n < words) g.d_online.alloc(std::max<size_t>(words, 2 * g.d_online.n));
        if (n_clients)
            SGA_HIP_CHECK(hipMemcpyAsync(g.d_online.p, online_bits, ((size_t)n_clients + 31) / 32 * 4,
                                         hipMemcpyHostToDevice, g.stream));
        ++g.tepoch;
        sga::conc_expire(g.cstate(), now, g.d_online.p, n_clients, g.stream);
        SGA_HIP_CHECK(hipGetLastError());
        SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
        uint32_t c[3];
        SGA_HIP_CHECK(hipMemcpy(c, g.d_tctr.p, 12, hipMemcpyDeviceToHost));
        g.tlive = c[0];
        g.ttomb = c[1];
        if (n_removed) *n_removed = c[2];
        return SGA_OK;
    });
}

int sga_concurrent_now_calls(sga_engine *e, int64_t flow_id, int32_t *now_calls) {
    if (!now_calls) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        auto it = g.slot_of.find(flow_id);
        if (it == g.slot_of.end() || !g.slots[it->second].conc_live) return 0;
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
        SGA_HIP_CHECK(hipMemcpy(now_calls, g.d_now_calls.p + it->second, 4, hipMemcpyDeviceToHost));
        return 1;
    });
}

int sga_concurrent_token_count(sga_engine *e, uint64_t *n) {
    if (!n) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        *n = g.tlive;
        return SGA_OK;
    });
}

int sga_concurrent_get_token(sga_engine *e, int64_t token_id, sga_token_cache_node *out) {
    if (!out) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        g.ensure_conc();
        sga::conc_find(g.cstate(), token_id, g.d_tfind.p, g.stream);
        SGA_HIP_CHECK(hipGetLastError());
        sga::TokenEntry t;
        SGA_HIP_CHECK(hipMemcpyAsync(&t, g.d_tfind.p, sizeof(t), hipMemcpyDeviceToHost, g.stream));
        SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
        if (t.state != sga::kTokLive) return 0;
        out->token_id = t.token;
        out->flow_id = t.flow_id;
        out->client_timeout = t.client_deadline;
        out->resource_timeout = t.resource_deadline;
        out->acquire_count = t.acquire;
        out->client = t.client;
        return 1;
    });
}

// SentinelEnvoyRlsServiceImpl.shouldRateLimit, RLS/SentinelEnvoyRlsServiceImpl.java:51-101
int sga_rls_should_rate_limit(sga_engine *e, const uint32_t *desc_offsets, size_t n_requests,
                              const int64_t *desc_flow_id, const int32_t *hits_addend, const int64_t *ts,
                              int8_t *desc_status, int32_t *desc_remaining, int32_t *code) {
    if (n_requests && (!desc_offsets || !hits_addend || !ts || !code)) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        const size_t nd = desc_offsets[n_requests];
        std::vector<int64_t> fid;
        std::vector<int32_t> acq;
        std::vector<int64_t> t;
        std::vector<size_t> where;
        fid.reserve(nd);
        for (size_t r = 0; r < n_requests; ++r) {
            int32_t a = hits_addend[r];
            if (a < 0) continue;  // onError(IllegalArgumentException): no descriptor is checked
            if (a == 0) a = 1;    // "Not present, use the default 1"
            for (uint32_t d = desc_offsets[r]; d < desc_offsets[r + 1]; ++d) {
                fid.push_back(desc_flow_id[d]);
                acq.push_back(a);
                t.push_back(ts[r]);
                where.push_back(d);
            }
        }
        std::vector<uint64_t> res(fid.size());
        int rc = fid.empty() ? SGA_OK
                             : run_host_batch(g, fid.data(), acq.data(), nullptr, t.data(), fid.size(), res.data(), 1);
        if (rc != SGA_OK) return rc;
        // a request with hitsAddend < 0 checks nothing: its descriptors report NO_RULE_EXISTS, 0
        std::vector<int8_t> st(nd, SGA_TOKEN_NO_RULE_EXISTS);
        std::vector<int32_t> rem(nd, 0);
        for (size_t k = 0; k < res.size(); ++k) {
            st[where[k]] = (int8_t)(res[k] >> 48);
            rem[where[k]] = (int32_t)(uint32_t)res[k];
        }
        for (size_t r = 0; r < n_requests; ++r) {
            if (hits_addend[r] < 0) {
                code[r] = -1;
                continue;
            }
            bool blocked = false;
            // an absent rule passes (NO_RULE_EXISTS -> OK, :65-68)
            for (uint32_t d = desc_offsets[r]; d < desc_offsets[r + 1]; ++d)
                blocked |= st[d] != SGA_TOKEN_OK && st[d] != SGA_TOKEN_NO_RULE_EXISTS;
            code[r] = blocked ? 2 : 1;  // Code.OVER_LIMIT : Code.OK
        }
        if (desc_status) std::copy(st.begin(), st.end(), desc_status);
        if (desc_remaining) std::copy(rem.begin(), rem.end(), desc_remaining);
        return SGA_OK;
    });
}

int sga_rls_should_rate_limit_device(sga_engine *e, const uint32_t *d_desc_offsets, size_t n_requests,
                                     size_t n_descriptors, const int64_t *d_desc_flow_id,
                                     const int32_t *d_hits_addend, int64_t ts_base, const uint32_t *d_ts_off,
                                     int8_t *d_desc_status, int32_t *d_desc_remaining, int32_t *d_code,
                                     void *hip_stream) {
    if (n_requests && (!d_desc_offsets || !d_hits_addend || !d_ts_off || !d_code)) return SGA_EINVAL;
    if (n_descriptors && !d_desc_flow_id) return SGA_EINVAL;
    if (ts_base < 0) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        if (n_descriptors > g.cfg.max_batch || n_requests > g.cfg.max_batch) return SGA_ERANGE;
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        const size_t cap = g.cfg.max_batch;
        if (g.d_in_fid.n < cap) {  // grown on the engine stream before a caller stream is ordered after it
            g.d_in_fid.alloc(cap);
            g.d_in_acq.alloc(cap);
            g.d_in_prio.alloc(cap);
            g.d_in_ts.alloc(cap);
            g.d_out.alloc(cap);
        }
        hipStream_t s = g.enter_stream(hip_stream);
        const auto lims = limiter_passes(g);
        sga::rls_expand(d_desc_offsets, (uint32_t)n_requests, d_desc_flow_id, d_hits_addend, d_ts_off, g.d_in_fid.p,
                        g.d_in_acq.p, g.d_in_ts.p, s);
        if (n_descriptors)
            sga::cluster_decide_batch(g.state(), g.scratch, g.d_in_fid.p, g.d_in_acq.p, nullptr, ts_base, g.d_in_ts.p,
                                      (uint32_t)n_descriptors, 1, g.d_out.p, s, lims.data(), (int)lims.size());
        sga::rls_finish(d_desc_offsets, (uint32_t)n_requests, d_hits_addend, g.d_out.p, d_desc_status,
                        d_desc_remaining, d_code, s);
        SGA_HIP_CHECK(hipGetLastError());
        g.leave_stream(s);
        return SGA_OK;
    });
}

// ---------------------------------------------------------------- local path
int sga_flow_set_resources(sga_engine *e, uint32_t n_resources) {
    if (n_resources == 0 || n_resources >= (1u << 30)) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        return g.flow.set_resources(n_resources);
    });
}

int sga_set_cluster_server(sga_engine *e, int32_t mode) {
    if (mode != 0 && mode != 1) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        g.cluster_server = mode;
        ++g.cluster_gen;
        return SGA_OK;
    });
}

int sga_load_flow_rules(sga_engine *e, const sga_flow_rule *rules, size_t n) {
    if (n && !rules) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        return g.flow.load_flow_rules(rules, n);
    });
}

int sga_load_param_rules(sga_engine *e, const sga_param_rule *rules, size_t n) {
    if (n && !rules) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        return g.flow.load_param_rules(rules, n);
    });
}

int sga_load_degrade_rules(sga_engine *e, const sga_degrade_rule *rules, size_t n) {
    if (n && !rules) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        return g.flow.load_degrade_rules(rules, n);
    });
}

// Cluster-mode parameter rules of the local path (ParamFlowChecker.passClusterCheck): the embedded server's
// parameter path state, refused (-ENOSYS) when a rule's flowId lives in a namespace with a request limiter
// (the local path does not apply GlobalRequestLimiter)
static int cluster_param_plumb(Engine &g) {
    g.flow.cparam_st = sga::CParamState{};
    g.flow.cparam_hook = nullptr;
    if (!g.flow.has_cluster_prules || g.cluster_server != 1) return SGA_OK;
    if (g.d_pctl.p) {
        g.flow.cparam_st = g.pstate();
        g.flow.cparam_hook = [&g](hipStream_t s) {  // after the local count pass created this batch's keys
            sga::cparam_lru_decide(g.pstate(), s);
            uint32_t ctl[5];
            SGA_HIP_CHECK(hipMemcpyAsync(ctl, g.d_pctl.p, sizeof(ctl), hipMemcpyDeviceToHost, s));
            SGA_HIP_CHECK(hipStreamSynchronize(s));
            if (ctl[4]) g.cparam_lru_switch_host(ctl[4], s);
            g.flow.cparam_st = g.pstate();  // the pool may have moved
        };
    }
    for (const sga_param_rule &r : g.flow.h_prule_src) {
        if (!r.cluster_mode) continue;
        auto it = g.pslot_of.find(r.cluster_flow_id);
        if (it == g.pslot_of.end()) continue;
        const sga::PSlotHost &h = g.pslots[it->second];
        if (h.active && h.ns >= 0 && g.nss[h.ns].has_limit) {
            g.err = "cluster-mode parameter rule: its namespace has a request limiter";
            return SGA_ENOSYS;
        }
    }
    return SGA_OK;
}

int sga_submit_events(sga_engine *e, const uint8_t *kind, const uint32_t *resource, const int64_t *ts,
                      const int32_t *acquire, const uint8_t *flags, const int64_t *rt, const uint64_t *param,
                      size_t n, int8_t *decision, int32_t *wait_ms) {
    return sga_submit_events_ex(e, kind, resource, ts, acquire, flags, rt, param, n, nullptr, 0, decision, wait_ms);
}

int sga_submit_events_ex(sga_engine *e, const uint8_t *kind, const uint32_t *resource, const int64_t *ts,
                         const int32_t *acquire, const uint8_t *flags, const int64_t *rt, const uint64_t *param,
                         size_t n, const uint64_t *param_values, size_t n_values, int8_t *decision,
                         int32_t *wait_ms) {
    if (n && (!kind || !resource || !ts || !acquire || !decision)) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        g.flow.cluster_on = g.cluster_server == 1 ? 1 : 0;
        if (const int rc = cluster_param_plumb(g); rc != SGA_OK) return rc;
        if (g.flow.has_cluster_rules) {
            g.flow.cluster_st = g.state();
            const int rc = g.flow.resolve_cluster(
                [&](int64_t fid) -> int32_t {
                    auto it = g.slot_of.find(fid);
                    if (it == g.slot_of.end()) return -1;
                    const SlotHost &h = g.slots[it->second];
                    if (!h.active) return -1;
                    if (h.ns >= 0 && g.nss[h.ns].has_limit) return -2;
                    return (int32_t)it->second;
                },
                g.cluster_gen);
            if (rc != SGA_OK) {
                g.err = "cluster-mode flow rule: flowId shared by two resources or namespace with a request limiter";
                return rc;
            }
        }
        return g.flow.submit(kind, resource, ts, acquire, flags, rt, param, n, decision, wait_ms, param_values,
                             n_values);
    });
}

int sga_submit_events_device(sga_engine *e, const uint8_t *d_kind, const uint32_t *d_resource, int64_t ts_base,
                             const uint32_t *d_ts_off, const int32_t *d_acquire, const uint8_t *d_flags,
                             const int64_t *d_rt, const uint64_t *d_param, size_t n, const uint64_t *d_param_values,
                             size_t n_values, int8_t *d_decision, int32_t *d_wait_ms, void *hip_stream) {
    if (n && (!d_kind || !d_resource || !d_ts_off || !d_acquire || !d_decision)) return SGA_EINVAL;
    if (ts_base < 0) return SGA_EINVAL;  // LeapArray.currentWindow(t < 0) returns null
    return guarded(e, [&](Engine &g) {
        if (n > g.cfg.max_batch) return SGA_ERANGE;
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        g.flow.cluster_on = g.cluster_server == 1 ? 1 : 0;
        if (const int rc = cluster_param_plumb(g); rc != SGA_OK) return rc;
        if (g.flow.has_cluster_rules) {
            g.flow.cluster_st = g.state();
            const int rc = g.flow.resolve_cluster(
                [&](int64_t fid) -> int32_t {
                    auto it = g.slot_of.find(fid);
                    if (it == g.slot_of.end()) return -1;
                    const SlotHost &h = g.slots[it->second];
                    if (!h.active) return -1;
                    if (h.ns >= 0 && g.nss[h.ns].has_limit) return -2;
                    return (int32_t)it->second;
                },
                g.cluster_gen);
            if (rc != SGA_OK) {
                g.err = "cluster-mode flow rule: flowId shared by two resources or namespace with a request limiter";
                return rc;
            }
        }
        // buffers grow on the engine stream before a caller stream is ordered after it
        if (const int rc = g.flow.ensure_scratch()) return rc;
        if (const int rc = g.flow.ensure_maps(n + n_values)) return rc;
        hipStream_t s = g.enter_stream(hip_stream);
        const int rc = g.flow.submit_device(d_kind, d_resource, ts_base, d_ts_off, d_acquire, d_flags, d_rt, d_param, n,
                                            d_param_values, n_values, d_decision, d_wait_ms, s);
        g.leave_stream(s);
        return rc;
    });
}

int sga_events_device_status(sga_engine *e) {
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        return g.flow.device_status();
    });
}

int sga_query_node(sga_engine *e, uint32_t resource, int64_t now, sga_node_view *out) {
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        return g.flow.query(resource, now, out);
    });
}

int sga_load_system_rules(sga_engine *e, const sga_system_rule *rules, size_t n) {
    if (n && !rules) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) { return g.flow.load_system_rules(rules, n); });
}

int sga_set_system_status(sga_engine *e, double avg_load, double cpu_usage) {
    return guarded(e, [&](Engine &g) {
        g.flow.sys.cur_load = avg_load;
        g.flow.sys.cur_cpu = cpu_usage;
        return SGA_OK;
    });
}

int sga_metrics_snapshot(sga_engine *e, int64_t now, sga_metric_node *out, size_t cap, size_t *n) {
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        return g.flow.metrics(now, out, cap, n);
    });
}

static int cluster_nodes_impl(Engine &g, int64_t now, void *d_out, size_t cap, uint32_t *d_n, hipStream_t s) {
    if (cap > 0xFFFFFFFFu) cap = 0xFFFFFFFFu;
    if (!g.d_slot_fid.p) {
        SGA_HIP_CHECK(hipMemsetAsync(d_n, 0, 4, s));
        return SGA_OK;
    }
    sga::cluster_metric_nodes(g.state(), g.d_slot_fid.p, now, d_out, (uint32_t)cap, d_n, s);
    SGA_HIP_CHECK(hipGetLastError());
    return SGA_OK;
}

int sga_cluster_metric_nodes(sga_engine *e, int64_t now, sga_cluster_metric_node *out, size_t cap, size_t *n) {
    if (now < 0 || !n || (cap && !out)) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        const size_t dcap = std::max<size_t>(cap, 1);
        if (g.d_nodes.n < dcap * sizeof(sga_cluster_metric_node)) g.d_nodes.alloc(dcap * sizeof(sga_cluster_metric_node));
        if (!g.d_ncount.p) g.d_ncount.alloc(1);
        cluster_nodes_impl(g, now, g.d_nodes.p, cap, g.d_ncount.p, g.stream);
        uint32_t cnt = 0;
        SGA_HIP_CHECK(hipMemcpyAsync(&cnt, g.d_ncount.p, 4, hipMemcpyDeviceToHost, g.stream));
        SGA_HIP_CHECK(hipStreamSynchronize(g.stream));
        const size_t w = std::min<size_t>(cnt, cap);
        if (w) SGA_HIP_CHECK(hipMemcpy(out, g.d_nodes.p, w * sizeof(sga_cluster_metric_node), hipMemcpyDeviceToHost));
        *n = w;
        return cnt > cap ? SGA_ERANGE : SGA_OK;
    });
}

int sga_cluster_metric_nodes_device(sga_engine *e, int64_t now, sga_cluster_metric_node *d_out, size_t cap,
                                    uint32_t *d_n, void *hip_stream) {
    if (now < 0 || !d_n || (cap && !d_out)) return SGA_EINVAL;
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        hipStream_t s = g.enter_stream(hip_stream);  // the window rotations write rule state
        const int rc = cluster_nodes_impl(g, now, d_out, cap, d_n, s);
        g.leave_stream(s);
        return rc;
    });
}

int sga_circuit_breaker_state(sga_engine *e, uint32_t resource, uint32_t k) {
    return guarded(e, [&](Engine &g) {
        SGA_HIP_CHECK(hipSetDevice(g.cfg.device));
        return g.flow.cb_state(resource, k);
    });
}

}  // extern "C"
