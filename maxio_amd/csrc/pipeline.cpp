// pipeline.cpp — end-to-end host-memory batch encode (the PUT path as MaxIO
// sees it: request bodies in host memory, parity chunks and digests back in
// host memory), spread over every device of the context.
//
// Per device (one host thread each; objects dealt round-robin over devices
// when the batch is uniform, by bytes when it is mixed, deal.hpp):
//   * an HBM object pool holds a whole wave of objects (k+m shard slots and
//     k+m digests each, up to kPoolCap bytes), so the latency-bound SHA-256
//     launches of many groups run concurrently instead of waiting on a small
//     staging window (288 GB of HBM makes this the cheap resource);
//   * uploads go on a dedicated H2D stream, straight from the caller's buffer
//     when it is pinned (hipHostMalloc / hipHostRegister), else through a ring
//     of pinned staging buffers filled by memcpy;
//   * each group of objects gets its RS launch(es) on the RS stream right
//     behind its upload; one SHA-256 launch then covers every chunk of the
//     wave (a message's hash latency does not depend on the batch size, so
//     one launch finishes as early as any split of it); descriptor tables
//     come from a per-wave arena so nothing throttles the launches in flight;
//   * parity returns group by group on a D2H stream as RS finishes, digests
//     after the SHA launch, direct to pinned destinations or via a pinned ring.
// Results are bit-identical to mxec_encode (same kernels, same planner).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <system_error>
#include <thread>
#include <tuple>
#include <vector>

#include <sys/syscall.h>
#include <unistd.h>

#include "../../include/maxio_ec.h"
#ifdef MXEC_LAB
#include <cstdio>
#include <string>
#endif
#include "deal.hpp"
#include "kernels.hpp"
#include "piece_grid.hpp"
#include "ops.hpp"

namespace mxec {
namespace {

constexpr uint64_t kAlign = 256;
constexpr uint64_t kPoolCap = uint64_t(96) << 30;     // pool HBM per device, over the calls in flight
constexpr uint64_t kGroupBytes = uint64_t(256) << 20;  // input bytes per group
constexpr uint64_t kRingBuf = uint64_t(64) << 20;      // pinned ring buffer size
constexpr int kRing = 4;
constexpr int kComputeStreams = 2;  // RS stream + SHA stream (4 HW queues per process)

uint64_t rup(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

bool is_pinned(const void* p, uint64_t len) { return pinned_range(p, len); }

struct HostObj {
    int k, m;
    uint64_t S;
    const uint8_t* const* data;
    const uint64_t* dlen;
    uint8_t* const* parity;
    uint8_t (*dig)[32];
    uint64_t pool_off = 0;  // device image: k+m shard slots of rup(S) bytes
    uint64_t slot() const { return rup(S, kAlign); }
    uint64_t bytes() const { return uint64_t(k + m) * slot(); }
};

// One object of a host reconstruct batch (mxec_reconstruct_batch_host).
struct RecObj {
    int k, m;
    uint64_t S;
    uint8_t* const* shards;          // k + m host buffers (present: read; missing: rebuilt into)
    const uint64_t* len;             // k + m, clamped to S
    uint8_t* present;                // k + m, in/out
    const uint8_t (*expected)[32];   // k + m digests, or null (no verification)
    int32_t* status;                 // out: MXEC_OK or MXEC_E_TOO_FEW_SHARDS_PRESENT
    uint64_t pool_off = 0;
    uint64_t slot() const { return rup(S, kAlign); }
    uint64_t bytes() const { return uint64_t(k + m) * slot(); }
};

class PinRing {
public:
    int init(int node = -1) {
        for (int i = 0; i < kRing; ++i) {
            buf_[i].node = node;
            MXEC_TRY(buf_[i].ensure(kRingBuf));
            unsigned flags = hipEventDisableTiming;
#ifdef MXEC_LAB
            if (const char* e = getenv("MXEC_RING_TIMED_EVENTS"); e && *e == '1') flags = hipEventDefault;  // lab: exit probe
#endif
            MXEC_HIP(hipEventCreateWithFlags(&ev_[i], flags));
        }
        return MXEC_OK;
    }
    ~PinRing() {
        for (auto e : ev_)
            if (e) (void)hipEventDestroy(e);
    }
    int next() const { return next_; }
    void* ptr(int i) { return buf_[i].p; }
    hipEvent_t event(int i) { return ev_[i]; }
    // Claim the next buffer, waiting for the DMA that last used it.
    int take(int* i) {
        *i = next_;
        next_ = (next_ + 1) % kRing;
        if (busy_[*i]) MXEC_HIP(hipEventSynchronize(ev_[*i]));
        busy_[*i] = false;
        return MXEC_OK;
    }
    int mark(int i, hipStream_t s) {
        MXEC_HIP(hipEventRecord(ev_[i], s));
        busy_[i] = true;
        return MXEC_OK;
    }
    void release_all() {
        for (auto& b : busy_) b = false;
    }

private:
    PinnedBuf buf_[kRing];
    hipEvent_t ev_[kRing] = {};
    bool busy_[kRing] = {};
    int next_ = 0;
};

// Per-call resources of the pipeline (a lane): one host-batch call holds a
// lane from admission to return, so concurrent calls on one device never
// share a pool, staging ring, descriptor arena or verdict buffer.  Lanes
// are kept for later calls (their pools stay allocated: a re-size frees,
// and hipFree waits for the whole device).
struct PipeLane {
    PinRing in, out;
    DescArena arena;
    DevBuf pool, digests;
    DevBuf chain_state;  // SHA-256 chain states between pieces (host reconstruct)
    PinnedBuf flags;  // verification verdicts read back (host reconstruct)
    Slot desc_slot;  // unused ring owner for DescWriter (tables come from the arena)
    uint64_t admitted = 0;  // pool bytes this call was admitted with
    bool ready = false;
    // On a context over several NUMA nodes the staging rings and the
    // verdict buffer live on the device's node.
    int init(const Device& dev) {
        if (ready) return MXEC_OK;
        desc_slot.owner = &dev;
        arena.owner = &dev;
        const int node = dev.ctx_multi_node ? dev.numa_node : -1;
        flags.node = node;
        MXEC_TRY(in.init(node));
        MXEC_TRY(out.init(node));
        ready = true;
        return MXEC_OK;
    }
};

// NUMA node of the page at p (get_mempolicy MPOL_F_NODE | MPOL_F_ADDR), or -1.
int page_node(const void* p) {
    if (!p) return -1;
    int node = -1;
    return syscall(SYS_get_mempolicy, &node, nullptr, 0, const_cast<void*>(p), 3 /* MPOL_F_NODE | MPOL_F_ADDR */) == 0
               ? node
               : -1;
}

// Device of each object of a host batch: o mod D / by bytes (deal_objects);
// on a context over several NUMA nodes, by the node of each object's first
// host page (`first[o]`), balanced (deal_objects_numa).
std::vector<uint32_t> deal_batch(const Ctx& c, const std::vector<uint64_t>& bytes, const std::vector<const void*>& first) {
    const uint32_t D = uint32_t(c.devs.size());
    if (D <= 1 || !c.devs[0]->ctx_multi_node) return deal_objects(bytes, D);
    std::vector<int> dev_node(D), node(bytes.size(), -1);
    for (uint32_t d = 0; d < D; ++d) dev_node[d] = c.devs[d]->numa_node;
    for (size_t o = 0; o < bytes.size(); ++o) node[o] = page_node(first[o]);
    return deal_objects_numa(bytes, node, dev_node);
}

// The device's pipeline: four streams shared by every call -- H2D, D2H and
// two compute streams (the process gets 4 hardware queues; more streams
// would share them and serialise behind each other) -- and the lanes.
//
// Concurrent calls (MaxIO serves PUTs and GETs at once
// on its tokio runtime, main.rs:81): up to MXEC_PIPE_LANES calls hold lanes
// at once, admitted while the pool bytes of the calls in flight stay within
// kPoolCap (a lone call is always admitted).  Their waves interleave on the
// same streams:
//   * each call takes the compute stream fewer calls in flight use (use())
//     and queues all its kernels there, so a PUT's chains and a GET's run
//     side by side instead of one queueing behind the other, and no call's
//     RS piece waits behind another call's chain piece;
//   * a call that finds another in flight paces its enqueue (pace()): it
//     queues a piece (or group) only after its own piece kPaceDepth back
//     is up, so the streams, which run in submission order, carry the calls'
//     work in the order it can run instead of all of one call's uploads and
//     then the other's;
//   * the SDMA watch is off while calls share the copy streams (a bracket
//     would time the other call's copies too).
struct PipeHub {
    hipStream_t h2d = nullptr, d2h = nullptr;
    hipStream_t cs[kComputeStreams] = {};
    std::mutex mu;
    std::condition_variable cv;  // a lane came back
    std::vector<std::unique_ptr<PipeLane>> lanes;
    std::vector<PipeLane*> idle;
    int in_flight = 0;            // calls holding a lane
    uint64_t admitted_bytes = 0;  // their pool bytes
    int users[kComputeStreams] = {0, 0};  // calls in flight per compute stream (use())
    std::atomic<int> calls{0};    // in_flight, readable without the lock
    bool ready = false;
    int init(const Device& dev) {
        if (ready) return MXEC_OK;
        MXEC_TRY(create_streams(dev));
        affinity_tag(h2d, &dev);
        affinity_tag(d2h, &dev);
        for (auto s : cs) affinity_tag(s, &dev);
        ready = true;
        return MXEC_OK;
    }
    // A lane for a call whose waves need up to `bytes` of pool (capped at
    // kPoolCap): waits while MXEC_PIPE_LANES calls are in flight, or while
    // the calls in flight hold pool bytes that would push the total past
    // kPoolCap.  Returns the lane and the bytes the call may use per wave.
    int acquire(const Device& dev, uint64_t bytes, PipeLane** out, bool* shared) {
        const int max_lanes = dev.kn ? dev.kn->pipe_lanes : 4;
        bytes = std::min(bytes, kPoolCap);
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] {
            return in_flight == 0 || (in_flight < max_lanes && admitted_bytes + bytes <= kPoolCap);
        });
        if (in_flight == 0)  // nothing of ours runs: buffers retired by re-sizes can go now
            for (auto& ln : lanes) ln->pool.free_retired();
        PipeLane* l = nullptr;
        if (!idle.empty()) {
            // the idle lane with the largest pool (fewest re-sizes)
            size_t best = 0;
            for (size_t i = 1; i < idle.size(); ++i)
                if (idle[i]->pool.cap > idle[best]->pool.cap) best = i;
            l = idle[best];
            idle.erase(idle.begin() + long(best));
        } else {
            lanes.emplace_back(new PipeLane());
            l = lanes.back().get();
        }
        *shared = in_flight > 0;
        ++in_flight;
        calls.store(in_flight);
        admitted_bytes += bytes;
        l->admitted = bytes;
        lk.unlock();
        const int rc = l->init(dev);
        if (rc != MXEC_OK) release(l);
        *out = rc == MXEC_OK ? l : nullptr;
        return rc;
    }
    void release(PipeLane* l) {
        {
            std::lock_guard<std::mutex> g(mu);
            --in_flight;
            calls.store(in_flight);
            admitted_bytes -= l->admitted;
            l->admitted = 0;
            idle.push_back(l);
        }
        cv.notify_all();
    }
    // The compute stream fewer calls in flight use (ties: `prefer`), counted
    // until unuse().  A call puts all its kernels there (its SHA-256 chains
    // and its RS launches; a verified GET's speculative decodes go on the
    // D2H stream): a kernel queued on a stream another call's chains use
    // waits for that call's chain pieces (a PUT's RS pieces behind a GET's
    // 4 MiB chain pieces held the PUT's chain to the GET's pace: the pair
    // ran 0.45-0.48 s, no faster than the two calls one after the other).
    int use(int prefer) {
        std::lock_guard<std::mutex> g(mu);
        const int c = users[1 - prefer] < users[prefer] ? 1 - prefer : prefer;
        ++users[c];
        return c;
    }
    void unuse(int c) {
        std::lock_guard<std::mutex> g(mu);
        --users[c];
    }
    // Plain non-blocking streams.  Lab builds can put the copy streams on a
    // few masked CUs and the compute streams on the rest
    // (MXEC_PIPE_COPY_CUS = n; measured no different from unmasked at the
    // wave copies' 16 workgroups, profiles/r4/get_stall/) or at different
    // priorities (MXEC_PIPE_COPY_PRIO 1 = copies highest, 2 = compute, 3 =
    // all four: the high-priority queue pool, apart from the process's
    // GPU_MAX_HW_QUEUES normal ones).
    int create_streams(const Device& dev) {
#ifdef MXEC_LAB
        const bool waves = dev.kn && dev.kn->pipe_copy != 0;
        const char* ce = getenv("MXEC_PIPE_COPY_CUS");
        const char* pe = getenv("MXEC_PIPE_COPY_PRIO");
        const int prio_mode = pe ? atoi(pe) : 0;
        (void)waves;
        if (prio_mode >= 1 && prio_mode <= 3) {
            int least = 0, greatest = 0;
            MXEC_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
            const int pc = prio_mode != 2 ? greatest : least, pk = prio_mode >= 2 ? greatest : least;
            MXEC_HIP(hipStreamCreateWithPriority(&h2d, hipStreamNonBlocking, pc));
            MXEC_HIP(hipStreamCreateWithPriority(&d2h, hipStreamNonBlocking, pc));
            for (auto& s : cs) MXEC_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, pk));
            return MXEC_OK;
        }
        const int n = dev.n_cus > 0 ? dev.n_cus : 256;
        const int copy_cus = waves && ce ? std::min(atoi(ce), n / 2) : 0;
        if (copy_cus > 0) {
            const int every = n / copy_cus;
            std::vector<uint32_t> cm(size_t((n + 31) / 32), 0u), rm(cm.size(), 0u);
            for (int i = 0; i < n; ++i)
                ((i % every == every - 1 && i / every < copy_cus) ? cm : rm)[size_t(i / 32)] |= 1u << (i % 32);
            MXEC_HIP(hipExtStreamCreateWithCUMask(&h2d, uint32_t(cm.size()), cm.data()));
            MXEC_HIP(hipExtStreamCreateWithCUMask(&d2h, uint32_t(cm.size()), cm.data()));
            for (auto& s : cs) MXEC_HIP(hipExtStreamCreateWithCUMask(&s, uint32_t(rm.size()), rm.data()));
            return MXEC_OK;
        }
        if (const char* e = getenv("MXEC_PIPE_SPLIT_CUS"); e && *e == '1') {  // lab A/B
            // The two compute streams on complementary halves of the CUs (even
            // / odd): two calls' SHA-256 chains, each a few workgroups, never
            // share a CU (side by side on one CU each runs at half speed).
            std::vector<uint32_t> ev(size_t((n + 31) / 32), 0u), od(ev.size(), 0u);
            for (int i = 0; i < n; ++i) (i % 2 ? od : ev)[size_t(i / 32)] |= 1u << (i % 32);
            MXEC_HIP(hipStreamCreateWithFlags(&h2d, hipStreamNonBlocking));
            MXEC_HIP(hipStreamCreateWithFlags(&d2h, hipStreamNonBlocking));
            MXEC_HIP(hipExtStreamCreateWithCUMask(&cs[0], uint32_t(ev.size()), ev.data()));
            MXEC_HIP(hipExtStreamCreateWithCUMask(&cs[1], uint32_t(od.size()), od.data()));
            return MXEC_OK;
        }
        if (const char* e = getenv("MXEC_PIPE_OWN_QUEUES"); e && *e == '1') {  // lab A/B
            // Every CU in the mask: the stream gets a hardware queue of its own
            // (a CU mask is a queue property), not one of the process's
            // GPU_MAX_HW_QUEUES shared ones.
            std::vector<uint32_t> all(size_t((n + 31) / 32), 0xFFFFFFFFu);
            MXEC_HIP(hipExtStreamCreateWithCUMask(&h2d, uint32_t(all.size()), all.data()));
            MXEC_HIP(hipExtStreamCreateWithCUMask(&d2h, uint32_t(all.size()), all.data()));
            for (auto& s : cs) MXEC_HIP(hipExtStreamCreateWithCUMask(&s, uint32_t(all.size()), all.data()));
            return MXEC_OK;
        }
        if (const char* e = getenv("MXEC_PIPE_NORMAL_PRIO"); e && *e == '1') {  // lab A/B: round 5's streams
            MXEC_HIP(hipStreamCreateWithFlags(&h2d, hipStreamNonBlocking));
            MXEC_HIP(hipStreamCreateWithFlags(&d2h, hipStreamNonBlocking));
            for (auto& s : cs) MXEC_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            return MXEC_OK;
        }
#else
        (void)dev;
#endif
        // The highest stream priority, created when the context opens
        // (pipe_open): HIP serves a process's streams from GPU_MAX_HW_QUEUES
        // (4) hardware queues per priority, and normal-priority streams --
        // the context's slots, the table stream, torch's -- already share
        // them.  Two of the pipeline's streams on one queue serialise
        // across it: with a GET's chain stream and the D2H stream on one
        // queue every hash piece waited for the previous piece's speculative
        // decode and download (26 ms per 1 MiB piece against 19;
        // profiles/r6/).  The high-priority pool is empty at mxec_open, so
        // the four streams get four queues; the compute streams are created
        // first, so the SHA-256 combiner's high-priority streams (created
        // on its first use) share the compute streams' queues, never a copy
        // stream's.
        int least = 0, greatest = 0;
        MXEC_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        for (auto& s : cs) MXEC_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest));
        MXEC_HIP(hipStreamCreateWithPriority(&h2d, hipStreamNonBlocking, greatest));
        MXEC_HIP(hipStreamCreateWithPriority(&d2h, hipStreamNonBlocking, greatest));
        return MXEC_OK;
    }
    // Context close (mxec_close, after the device is idle): the lanes'
    // rings, pools and events, then the streams.
    ~PipeHub() {
        lanes.clear();
        for (auto s : cs)
            if (s) {
                affinity_untag(s);
                (void)hipStreamDestroy(s);
            }
        affinity_untag(h2d);
        affinity_untag(d2h);
        if (h2d) (void)hipStreamDestroy(h2d);
        if (d2h) (void)hipStreamDestroy(d2h);
    }
};

// A lane of the device's pipeline for the duration of one call.
class LaneScope {
public:
    LaneScope() = default;
    LaneScope(const LaneScope&) = delete;
    LaneScope& operator=(const LaneScope&) = delete;
    ~LaneScope() {
        if (lane_) hub_->release(lane_);
    }
    int open(Device& dev, uint64_t bytes) {
        {
            std::lock_guard<std::mutex> g(dev.pipe_mu);
            if (!dev.pipe) dev.pipe = std::make_shared<PipeHub>();
            keep_ = dev.pipe;
        }
        hub_ = static_cast<PipeHub*>(keep_.get());
        {
            std::lock_guard<std::mutex> g(dev.pipe_mu);  // stream creation, once
            MXEC_TRY(hub_->init(dev));
        }
        bool shared = false;
        MXEC_TRY(hub_->acquire(dev, bytes, &lane_, &shared));
        ++dev.pipe_calls;
        if (shared) ++dev.pipe_calls_shared;
        return MXEC_OK;
    }
    PipeHub& hub() { return *hub_; }
    PipeLane& lane() { return *lane_; }

private:
    std::shared_ptr<void> keep_;
    PipeHub* hub_ = nullptr;
    PipeLane* lane_ = nullptr;
};

#ifdef MXEC_LAB
// MXEC_PIPE_TRACE=1 (lab builds): where a host reconstruct wave's time goes
// -- timing events on the copy and compute streams and host clocks around
// every wait, one stderr JSON line per wave (tools: the GET-stall study).
// The marks of every traced wave are reported against one process-wide
// reference event (recorded and completed by the first traced wave) and the
// host clock against one reference instant, so concurrent calls' traces line
// up.
struct PipeTrace {
    bool on = false;
    std::chrono::steady_clock::time_point h0;
    hipEvent_t e0 = nullptr;
    std::vector<std::pair<std::string, hipEvent_t>> ev;
    std::vector<std::pair<std::string, double>> host;
    static hipEvent_t& ref() {
        static hipEvent_t r = nullptr;
        return r;
    }
    static std::chrono::steady_clock::time_point& href() {
        static std::chrono::steady_clock::time_point t{};
        return t;
    }
    void start(hipStream_t s) {
        const char* e = getenv("MXEC_PIPE_TRACE");
        on = e && *e == '1';
        if (!on) return;
        static std::mutex mu;
        {
            std::lock_guard<std::mutex> g(mu);
            if (!ref()) {
                hipStream_t rs = nullptr;
                (void)hipStreamCreateWithFlags(&rs, hipStreamNonBlocking);
                (void)hipEventCreate(&ref());
                (void)hipEventRecord(ref(), rs);
                (void)hipEventSynchronize(ref());
                href() = std::chrono::steady_clock::now();
            }
        }
        h0 = href();
        e0 = ref();
        mark("start", s);
        now("start");
    }
    void mark(const char* what, hipStream_t s) {
        if (!on) return;
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        (void)hipEventRecord(e, s);
        ev.emplace_back(what, e);
    }
    void now(const char* what) {
        if (!on) return;
        host.emplace_back(what, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count());
    }
    void report(const char* tag) {
        if (!on) return;
        now("end");
        std::string out = std::string("{\"pipe_trace\": \"") + tag + "\", \"gpu_ms\": [";
        for (size_t i = 0; i < ev.size(); ++i) {
            float ms = -1;
            (void)hipEventSynchronize(ev[i].second);
            (void)hipEventElapsedTime(&ms, e0, ev[i].second);
            char b[96];
            snprintf(b, sizeof b, "%s[\"%s\", %.3f]", i ? ", " : "", ev[i].first.c_str(), ms);
            out += b;
            (void)hipEventDestroy(ev[i].second);
        }
        out += "], \"host_ms\": [";
        for (size_t i = 0; i < host.size(); ++i) {
            char b[96];
            snprintf(b, sizeof b, "%s[\"%s\", %.3f]", i ? ", " : "", host[i].first.c_str(), host[i].second);
            out += b;
        }
        out += "]}";
        fprintf(stderr, "%s\n", out.c_str());
        ev.clear();
        host.clear();
    }
};
#define PTRACE(x) tr_.x
#else
#define PTRACE(x) ((void)0)
#endif

class DevicePipeline {
public:
    DevicePipeline(Device& d, PipeHub& h, PipeLane& l)
        : d_(d), h2d_(h.h2d), d2h_(h.d2h), cs_(h.cs), in_(l.in), out_(l.out), arena_(l.arena),
          pool_(l.pool), scratch_(l.digests), state_(l.chain_state), flags_(l.flags), slot_(l.desc_slot),
          hub_(h), cap_(std::max<uint64_t>(l.admitted, 1)) {}
    ~DevicePipeline() {
        if (cs_idx_ >= 0) hub_.unuse(cs_idx_);
        for (auto e : events_) (void)hipEventDestroy(e);
    }

    // MXEC_PIPE_COPY (knobs.hpp): sdma; waves (every host batch); auto (the
    // default) -- SDMA while it runs at its normal rate, CU-wave copies while
    // it does not (watch_open / watch_judge below).  Measured (profiles/r4/get_stall/,
    // e2e_get_modes/): in a healthy process SDMA is the faster engine
    // (RS-only GET 0.101 s against 0.119 by waves at 128 objects; the PUT
    // with digests 0.218 against 0.264, copy waves beside the SHA-256 chains
    // slowing the chains), but after heavy HBM churn SDMA copies collapsed
    // for seconds to ~7 GB/s ([0.33, 0.92, 0.33, 0.92, 0.27] s verified GETs
    // against 0.263 by waves).
    int run(std::vector<HostObj>& objs) {
        start_copy_mode();
        cs_idx_ = hub_.use(1);
        size_t o = 0;
        while (o < objs.size()) {  // waves that fit the pool
            uint64_t need = 0, desc = 1 << 20;
            size_t e = o;
            while (e < objs.size() && (e == o || need + objs[e].bytes() <= cap_)) {
                objs[e].pool_off = need;
                need += objs[e].bytes();
                desc += uint64_t(objs[e].k + objs[e].m) * 48 + 256;
                ++e;
            }
            MXEC_TRY(pool_.replace(need));  // no free while other calls run (retired until idle)
            MXEC_TRY(arena_.reserve(desc * 2));
            MXEC_TRY(wave(objs, o, e));
            o = e;
        }
        return watch_drain();
    }

    // Host reconstruct batch: waves that fit the pool, as run().
    int run_rec(std::vector<RecObj>& objs, bool data_only) {
        start_copy_mode();
        cs_idx_ = hub_.use(0);
        size_t o = 0;
        while (o < objs.size()) {
            uint64_t need = 0, desc = 1 << 20;
            size_t e = o;
            while (e < objs.size() && (e == o || need + objs[e].bytes() <= cap_)) {
                objs[e].pool_off = need;
                need += objs[e].bytes();
                // pointer / length / digest-index tables, the SHA tables and one
                // 16-byte record per tile of the grouped launch (tiles >= 8 KiB)
                desc += uint64_t(objs[e].k + objs[e].m) * 96 + 512 + (objs[e].S / 8192 + 2) * 32;
                ++e;
            }
            MXEC_TRY(pool_.replace(need));  // no free while other calls run (retired until idle)
            MXEC_TRY(arena_.reserve(desc * 2));
            MXEC_TRY(rec_wave(objs, o, e, data_only));
            o = e;
        }
        return watch_drain();
    }

private:
    // Copy engine under MXEC_PIPE_COPY=auto: SDMA, watched.  The uploads of
    // each piece (or group) of a wave are bracketed by timing events on the
    // upload stream (watch_open / watch_close).  The host never waits for a
    // bracket (pacing the enqueue loop two brackets deep held back the group
    // form's downloads: RS-only PUT at 128 objects 0.188 s against 0.112):
    // brackets are judged when the host finds them complete, at the latest
    // when the call has synchronised (watch_drain).  A bracket of at least
    // kWatchMinBytes (16 MiB) of direct DMAs (no staging ring) that ran
    // below MXEC_PIPE_SDMA_FLOOR GB/s (default 20; healthy 1-4 MiB copies run
    // 33-43, the collapse seen after heavy HBM churn ran ~7) switches the
    // rest of the call's uploads of mxec_host_alloc memory (if any are still
    // to be issued) and the device's for the next kWavesHoldMs to the wave
    // kernels; a download bracket (RS-only GET, below) does the same for
    // downloads.  A slow-down lasts ~3.5 s after 60 GB of HBM is freed
    // (profiles/r5/copy_engine/slow_duration_after_60GB_free_r5m.jsonl).
    static constexpr uint64_t kWatchMinBytes = uint64_t(16) << 20;
    // Downloads hold for 1 s: their slow spells follow HBM frees and last
    // about freed bytes / 17 GB/s, so a 2 s hold after a pool-sized free
    // kept an RS-only GET on waves (0.111 s) after SDMA had recovered
    // (0.101; profiles/r5/copy_engine/vg_churn0_r5s.jsonl).
    static constexpr int kWavesHoldMs = 2000, kDownWavesHoldMs = 1000;
    static constexpr int kDownSlowRun = 2;  // slow download brackets in a row for a verdict
    struct Bracket {
        hipEvent_t a, b;
        uint64_t bytes, copies;
        bool staged;
        bool down;
    };
    // Only brackets whose DMAs average at least this much are judged: many
    // small copies run near the floor on a healthy SDMA (a 10 MiB chunk's
    // 256 KiB tail piece, 512 copies, read 9 GB/s in a fresh process).
    static constexpr uint64_t kWatchMinCopy = uint64_t(1) << 20;
    std::vector<Bracket> watch_;
    hipEvent_t watch_a_ = nullptr, dwatch_a_ = nullptr;
    bool watch_staged_ = false, dwatch_staged_ = false;
    uint64_t watch_bytes_ = 0, dwatch_bytes_ = 0;    // SDMA bytes issued in the open brackets
    uint64_t watch_copies_ = 0, dwatch_copies_ = 0;  // and the DMAs (2D: rows) that moved them
    static int64_t now_ns() {
        return std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    void start_copy_mode() {
        const int mode = d_.kn ? d_.kn->pipe_copy : 0;
        const int64_t now = now_ns();
        waves_now_ = mode == 1 || (mode == 2 && now < d_.waves_up_until_ns.load());
        down_waves_ = mode == 1 || (mode == 2 && now < d_.waves_down_until_ns.load());
#ifdef MXEC_LAB
        const char* dw = getenv("MXEC_PIPE_DOWN_WAVES");
        down_waves_ = down_waves_ || (dw && *dw == '1');
#endif
    }
    // Not while another call shares the copy streams: its copies would land
    // inside this call's brackets.
    bool watching(bool down = false) const {
        return d_.kn && d_.kn->pipe_copy == 2 && d_.kn->pipe_sdma_floor > 0 && !(down ? down_waves_ : waves_now_) &&
               !shared_now();
    }
    bool shared_now() const { return hub_.calls.load() > 1; }
    int new_timed_event(hipEvent_t* e) {
        MXEC_HIP(hipEventCreate(e));
        events_.push_back(*e);
        return MXEC_OK;
    }
    // A bracket opens (watch_open) before its copies are queued, but its
    // start event is recorded only after its first SDMA copy (watch_count),
    // which it does not time: an event recorded on an idle copy stream
    // completes at once, and the bracket would then time the host queueing
    // the first copy too.
    bool watch_on_ = false, dwatch_on_ = false;
    int watch_open() {
        if (!watching() || watch_on_) return MXEC_OK;
        watch_on_ = true;
        watch_a_ = nullptr;
        watch_staged_ = false;
        watch_bytes_ = 0;
        watch_copies_ = 0;
        return MXEC_OK;
    }
    // After an SDMA copy of `bytes` in `copies` DMAs (2D: rows) was queued.
    int watch_count(bool down, uint64_t bytes, uint64_t copies) {
        if (!(down ? dwatch_on_ : watch_on_)) return MXEC_OK;
        hipEvent_t& a = down ? dwatch_a_ : watch_a_;
        if (!a) {
            MXEC_TRY(new_timed_event(&a));
            MXEC_HIP(hipEventRecord(a, down ? d2h_ : h2d_));
            return MXEC_OK;
        }
        (down ? dwatch_bytes_ : watch_bytes_) += bytes;
        (down ? dwatch_copies_ : watch_copies_) += copies;
        return MXEC_OK;
    }
    // After the bracket's copies are issued (issue_up done).
    int watch_close() {
        if (!watch_on_) return MXEC_OK;
        watch_on_ = false;
        if (!watch_a_) return MXEC_OK;  // no SDMA copy to time
        hipEvent_t b = nullptr;
        MXEC_TRY(new_timed_event(&b));
        MXEC_HIP(hipEventRecord(b, h2d_));
        watch_.push_back(Bracket{watch_a_, b, watch_bytes_, watch_copies_, watch_staged_, false});
        watch_bytes_ = 0;
        watch_copies_ = 0;
        watch_a_ = nullptr;
        return watch_poll();
    }
    // Downloads (an RS-only GET's rebuilt shards, rebuild_list): the bracket
    // opens after the d2h stream's wait for the rebuild, so it times the
    // copies alone.  The PUT's parity downloads are not bracketed: in the
    // seconds after a large HBM free, timing events among the
    // PUT-with-digests pieces' downloads slowed that call by 63 % (0.336 s
    // against 0.206 at 128 objects,
    // profiles/r5/copy_engine/auto_dwatch_churn60_r5l2.jsonl), and its SDMA
    // downloads otherwise beat waves (0.204 s against 0.238 fresh).
    bool dwatch_off_ = false;
    int dwatch_open() {
        if (!watching(true) || dwatch_off_ || dwatch_on_) return MXEC_OK;
        dwatch_on_ = true;
        dwatch_a_ = nullptr;
        dwatch_staged_ = false;
        dwatch_bytes_ = 0;
        dwatch_copies_ = 0;
        return MXEC_OK;
    }
    int dwatch_close() {
        if (!dwatch_on_) return MXEC_OK;
        dwatch_on_ = false;
        if (!dwatch_a_) return MXEC_OK;
        hipEvent_t b = nullptr;
        MXEC_TRY(new_timed_event(&b));
        MXEC_HIP(hipEventRecord(b, d2h_));
        watch_.push_back(Bracket{dwatch_a_, b, dwatch_bytes_, dwatch_copies_, dwatch_staged_, true});
        dwatch_bytes_ = 0;
        dwatch_copies_ = 0;
        dwatch_a_ = nullptr;
        return watch_poll();
    }
    int watch_poll() {
        while (!watch_.empty()) {  // the finished ones, oldest first, without waiting
            if (hipEventQuery(watch_.front().b) != hipSuccess) {
                (void)hipGetLastError();
                break;
            }
            MXEC_TRY(watch_judge());
        }
        return MXEC_OK;
    }
    int watch_judge() {
        const Bracket k = watch_.front();
        watch_.erase(watch_.begin());
        MXEC_HIP(hipEventSynchronize(k.b));
        float ms = 0;
        MXEC_HIP(hipEventElapsedTime(&ms, k.a, k.b));
        if (k.staged || k.bytes < kWatchMinBytes || k.bytes < k.copies * kWatchMinCopy || ms <= 0) return MXEC_OK;
        const double gbps = double(k.bytes) / (double(ms) * 1e6);
        // A GET's download brackets run at 54-55 GB/s on a healthy box and
        // ~24 in the seconds after a large HBM free (uploads: 33-55 healthy,
        // unaffected by the free), so they are judged against twice the floor.
        const double floor = double(d_.kn ? d_.kn->pipe_sdma_floor : 20) * (k.down ? 2.0 : 1.0);
        const bool slow = gbps < floor;
        const int64_t hold = now_ns() + int64_t(k.down ? kDownWavesHoldMs : kWavesHoldMs) * 1000000;
        if (k.down) {
            // Two slow download brackets in a row make a verdict: an RS-only
            // GET's downloads share the link with its uploads, and a lone
            // bracket under the bar sent healthy calls to waves for a second
            // (0.128 s against 0.101 by SDMA; profiles/r6/final_r6aq/), where
            // a real slow state repeats bracket after bracket (~24 GB/s).
            ++d_.sdma_down_probes;
            d_.sdma_down_last_mbps = uint64_t(gbps * 1e3);
            if (!slow) {
                d_.down_slow_run = 0;
            } else if (!down_waves_ && d_.down_slow_run.fetch_add(1) + 1 >= kDownSlowRun) {
                d_.down_slow_run = 0;
                ++d_.sdma_down_slow_verdicts;
                down_waves_ = true;  // the rest of this call's downloads
                d_.waves_down_until_ns = hold;
            }
        } else {
            ++d_.sdma_probes;
            d_.sdma_last_mbps = uint64_t(gbps * 1e3);
            if (!waves_now_ && slow) {
                ++d_.sdma_slow_verdicts;
                waves_now_ = true;  // the rest of this call's uploads
                d_.waves_up_until_ns = hold;
            }
        }
        return MXEC_OK;
    }
    // End of a call: judge what is left (its copies are done), for the
    // device's next calls.
    int watch_drain() {
        watch_a_ = nullptr;
        dwatch_a_ = nullptr;
        watch_on_ = dwatch_on_ = false;
        while (!watch_.empty()) MXEC_TRY(watch_judge());
        return MXEC_OK;
    }

    // One wave of a host reconstruct batch (try_reconstruct_data_chunk,
    // chunk_reader.rs:157-226, per object).
    //
    // Verified waves (expected digests given) run piece-major when their
    // messages fit the lag quad form: piece p of every present shard goes up
    // and is hashed with the chains carried in device state slots, so every
    // chain starts after the first piece (verify_enqueue), and -- with
    // MXEC_GET_SPECULATE (default) -- piece p of every missing shard is
    // decoded from the first k present shards as soon as piece p is up, on
    // the assumption that they verify, and goes down at once (spec_piece).
    // The verdict then only confirms: an object whose shards all verified is
    // done; one with a mismatch is decoded again with the corrected mask and
    // its shards overwritten (a mismatch is an erasure, :176-196); one left
    // short of k shards fails with MXEC_E_TOO_FEW_SHARDS_PRESENT -- its
    // present shards untouched, its missing shards' buffers undefined (the
    // reference returns Err and no data, :203-206).  Without speculation the
    // rebuild waits for the verdict (nothing is written to a failing
    // object's buffers), and a large wave runs as a few verification groups
    // (verify_cuts) so that group j's rebuild and download overlap group
    // j + 1's upload and chains; with it the downloads already overlap
    // everything and the wave is one group.
    //
    // Other waves: the present shards go up group by group (coalesced,
    // direct from pinned memory), are verified by one SHA-256 launch once
    // all are up when digests are given, each group is rebuilt (one grouped
    // launch, run_rs_mixed) as soon as it is up (and verified), and its
    // rebuilt shards go down while later groups still upload.
    int rec_wave(std::vector<RecObj>& objs, size_t o0, size_t o1, bool data_only) {
        PTRACE(start(h2d_));
        uint64_t msgs = 0;
        bool verify = false;
        for (size_t o = o0; o < o1; ++o) {
            msgs += uint64_t(objs[o].k + objs[o].m);
            verify = verify || objs[o].expected;
        }
        // Expected digests of the wave (message order) after room for the
        // verdict flags, on the device.
        const uint64_t fo = rup(msgs, 256);
        uint8_t* ok = nullptr;
        uint8_t* exp = nullptr;
        if (verify) {
            MXEC_TRY(scratch_.grow(fo + msgs * 32));
            ok = static_cast<uint8_t*>(scratch_.p);
            exp = ok + fo;
        }
        const bool down_before = down_waves_;
        const bool auto_copy = d_.kn && d_.kn->pipe_copy == 2;
        dwatch_off_ = verify;  // a verified wave's downloads are not bracketed
        uint64_t vmsgs = 0;  // present shards to verify
        for (size_t o = o0; o < o1; ++o)
            if (objs[o].expected)
                for (int i = 0; i < objs[o].k + objs[o].m; ++i) vmsgs += objs[o].present[i] ? 1 : 0;
        uint64_t up_bytes = 0, longest_msg = 0;
        for (size_t o = o0; o < o1; ++o)
            for (int i = 0; i < objs[o].k + objs[o].m; ++i)
                if (objs[o].present[i]) {
                    up_bytes += objs[o].len[i];
                    if (objs[o].expected) longest_msg = std::max(longest_msg, objs[o].len[i]);
                }
        const uint64_t P = piece_bytes(up_bytes, longest_msg);
        if (verify && P && vmsgs && vmsgs <= uint64_t(kShaLagMsgs) * uint64_t(d_.n_cus ? d_.n_cus : 256)) {
            const bool shared = shared_now();
            const bool spec = !d_.kn || d_.kn->get_speculate;
            uint64_t down_bytes = 0;
            for (size_t o = o0; o < o1; ++o)
                for (int i = 0; i < objs[o].k + objs[o].m; ++i) down_bytes += objs[o].present[i] ? 0 : objs[o].len[i];
            // One group when speculating (the downloads overlap the chains
            // already) or when another call shares the device (one compute
            // stream each: a second group's chains would queue behind the
            // first's on it).
            const std::vector<size_t> cut = verify_cuts(objs, o0, o1, up_bytes, longest_msg, down_bytes, spec || shared);
            MXEC_TRY(state_.grow(msgs * 32));
            MXEC_TRY(flags_.grow(msgs));
            std::vector<uint64_t> mbase(cut.size(), 0);
            for (size_t j = 1; j < cut.size(); ++j) {
                mbase[j] = mbase[j - 1];
                for (size_t o = cut[j - 1]; o < cut[j]; ++o) mbase[j] += uint64_t(objs[o].k + objs[o].m);
            }
            const size_t G = cut.size() - 1;
            // auto: a chain-bound wave verified as one group uploads by waves
            // (one copy launch per piece instead of a DMA per piece of every
            // shard: 128 x 4+2 x 10 MiB 0.240 s against 0.256 by SDMA, 256
            // objects 0.363 against 0.371); an upload-bound wave keeps SDMA
            // uploads (512: 0.590 against 0.679 by waves, whose copies beside
            // the downloads and chains slow both;
            // profiles/r5/copy_engine/verified_uploads_r5z.jsonl), and so does
            // a call that shares the device.
            const bool up_before = waves_now_;
            bool up_override = auto_copy && G == 1 && piece_ramp_ && !shared;
#ifdef MXEC_LAB
            if (const char* e = getenv("MXEC_GET_WAVE_UPLOADS"); e && *e == '0') up_override = false;  // lab A/B
#endif
            if (up_override) waves_now_ = true;
            // A lone speculating wave's downloads run beside its chains and
            // uploads: by SDMA, unless an earlier call found them slow there
            // (spec_judge) less than kSpecWavesHoldMs ago.
            const bool spec_sdma = spec && auto_copy && !shared && !down_waves_;
            if (spec && auto_copy && !shared &&
                (spec_down_waves() || now_ns() < d_.spec_waves_until_ns.load()))
                down_waves_ = true;  // restored at the end
            const bool judge = spec_sdma && !down_waves_;
            int64_t t_verdict = 0;
            bool redo = false;
            // Without speculation the last group's rebuilt shards (on the
            // critical path, alone on the link) go down by waves, earlier
            // groups' by SDMA beside the later groups' uploads and chains
            // (wave copies there slow the chains: 0.64 s against 0.59 at 512
            // objects, G = 2).  Speculative downloads run beside the chains,
            // so they keep SDMA.
            std::vector<hipEvent_t> verdict(G, nullptr);
            auto enqueue = [&](size_t j) {
                return verify_enqueue(objs, cut[j], cut[j + 1], ok, exp, mbase[j], P, cs_[(cs_idx_ + int(j)) & 1],
                                      &verdict[j], spec, data_only);
            };
            MXEC_TRY(enqueue(0));
            for (size_t j = 0; j < G; ++j) {
                if (j + 1 < G) MXEC_TRY(enqueue(j + 1));
                std::vector<size_t> changed;
                MXEC_TRY(verify_collect(objs, cut[j], cut[j + 1], mbase[j], verdict[j], &changed));
                PTRACE(now("verified"));
                t_verdict = now_ns();
                redo = redo || !changed.empty();
                if (spec) {
                    MXEC_TRY(confirm(objs, cut[j], cut[j + 1], changed, data_only));
                    // The objects with a mismatch, decoded again with their
                    // verified masks on the D2H stream: behind the
                    // speculative downloads, which read the slots this
                    // decode rewrites.
                    if (!changed.empty()) {
                        d_.spec_redos += changed.size();
                        MXEC_TRY(rebuild_list(objs, changed, d2h_, nullptr, data_only));
                    }
                } else {
                    if (auto_copy && !shared) down_waves_ = down_before || j + 1 == G;
                    for (const auto& q : object_groups(objs, cut[j], cut[j + 1]))
                        MXEC_TRY(rebuild_range(objs, q.first, q.second, cs_[(cs_idx_ + int(j)) & 1], nullptr, data_only));
                }
            }
            d_.verify_groups += G;
            d_.verify_waves += 1;
            if (up_override) waves_now_ = up_before;  // only the override is undone
            judge_ = judge && !redo;
            t_verdict_ = t_verdict;
        } else {
            const auto groups = object_groups(objs, o0, o1);
            hipStream_t cs = cs_[cs_idx_];
            std::vector<hipEvent_t> up;  // per group: its upload is done
            MXEC_TRY(upload_and_verify(objs, o0, o1, groups, ok, exp, verify, cs, &up));
            // Per group, rebuild once it is up (without verification, as soon
            // as it is up), then its shards down.
            for (size_t q = 0; q < groups.size(); ++q)
                MXEC_TRY(rebuild_range(objs, groups[q].first, groups[q].second, cs, verify ? nullptr : up[q], data_only));
        }
        MXEC_TRY(issue_down());
        PTRACE(mark("d2h", d2h_));
        PTRACE(now("down_queued"));
        const int frc = flush();
        PTRACE(report("rec_wave"));
        if (frc == MXEC_OK && judge_) spec_judge();
        judge_ = false;
        down_waves_ = down_before;
        dwatch_off_ = false;
        return frc;
    }

    // Objects [o0, o1) of a speculatively rebuilt group whose present masks
    // the verdict left as they were (all but `changed`): their rebuilt
    // shards are already on their way down; status and present flags.
    // Workgroups of a speculative piece decode: four per CU.  It runs beside
    // the wave's SHA-256 chains; at the RS kernel's default grid (512-1024
    // per CU, 0.13-0.26 M workgroups for a 1 MiB piece of 128 x 4+2) it
    // either slowed the chains (19 -> 35 ms a piece) or was starved by them
    // (a piece's decode + download 42 ms instead of 9), which of the two
    // changing from call to call: 0.19-0.46 s for the same 128-object GET
    // (pipe traces, profiles/r6/spec_grid/).  A piece's decode moves ~0.8 GB
    // in the ~9 ms the link takes to bring the next piece up; at one
    // workgroup per CU the GET ended ~6 ms later than at four
    // (profiles/r6/spec_grid/spec_grid_ab_r6q.jsonl).
    uint32_t spec_blocks() const {
        uint32_t b = 4u * (d_.n_cus ? uint32_t(d_.n_cus) : 256u);
#ifdef MXEC_LAB
        if (const char* e = getenv("MXEC_SPEC_BLOCKS")) b = uint32_t(atol(e));  // lab A/B (0: default grid)
#endif
        return b;
    }
    // A lone speculating wave's speculative downloads go by SDMA: healthy,
    // they keep pace with the chains and the wave ends ~1 ms after its last
    // verdict (128 x 4+2 x 10 MiB: 0.193 s).  But in some processes, and in
    // the seconds after a large HBM free, those SDMA downloads crawl at
    // ~6 GB/s while the chains run and the same GET takes 0.42-0.47 s; by CU
    // waves it takes 0.24 s in either state (and without speculation 0.242;
    // profiles/r6/spec_grid/get_churn_ab_*.jsonl).  Nothing measured ahead of
    // the wave tells the states apart: a 32 MiB D2H copy on the idle link ran
    // at 54-55 GB/s in both, the same copy beside the first piece's upload
    // at 13.4 GB/s in both (get_churn_ab_r6u/r6v), and the pieces' own
    // download brackets during the upload phase run at ~6 GB/s in both.  So
    // the wave is judged after the fact: downloads still running more than
    // kSpecTailMs after the last verdict (healthy ~1 ms, slow ~140) send the
    // device's next lone speculating waves' downloads to waves for
    // kSpecWavesHoldMs, doubled for each slow verdict in a row up to 16 s;
    // the first wave after the hold tries SDMA again (a healthy one ends the
    // run of slow verdicts).
    static constexpr int64_t kSpecTailMs = 25, kSpecWavesHoldMs = 2000;
    bool judge_ = false;
    int64_t t_verdict_ = 0;
    void spec_judge() {
        if (!t_verdict_) return;
        const int64_t tail_ms = (now_ns() - t_verdict_) / 1000000;
        ++d_.sdma_down_probes;
        if (tail_ms <= kSpecTailMs) {
            d_.spec_slow_run = 0;
            return;
        }
        ++d_.sdma_down_slow_verdicts;
        const int run = std::min(d_.spec_slow_run.fetch_add(1), 3);
        d_.spec_waves_until_ns = now_ns() + (kSpecWavesHoldMs << run) * 1000000;
    }
    // Speculative downloads by CU waves instead of SDMA (lab A/B).
    static bool spec_down_waves() {
#ifdef MXEC_LAB
        const char* e = getenv("MXEC_SPEC_DOWN_WAVES");
        return e && *e == '1';
#else
        return false;
#endif
    }
    // The stream of a speculative piece decode (cs: the wave's chain stream).
    hipStream_t spec_stream(hipStream_t cs) const {
#ifdef MXEC_LAB
        if (const char* e = getenv("MXEC_SPEC_STREAM")) {
            if (!strcmp(e, "chain")) return cs;
            if (!strcmp(e, "other")) return shared_now() ? cs : cs_[(cs_idx_ + 1) & 1];
        }
#endif
        return d2h_;
    }

    int confirm(std::vector<RecObj>& objs, size_t o0, size_t o1, const std::vector<size_t>& changed, bool data_only) {
        size_t c = 0;
        for (size_t o = o0; o < o1; ++o) {
            if (c < changed.size() && changed[c] == o) {
                ++c;
                continue;
            }
            // decode_plan's rule (gf256.cpp): k present shards make a plan,
            // and its missing shards are every absent one (data_only: every
            // absent data shard)
            RecObj& h = objs[o];
            int np = 0;
            for (int i = 0; i < h.k + h.m; ++i) np += h.present[i] ? 1 : 0;
            *h.status = np >= h.k ? MXEC_OK : MXEC_E_TOO_FEW_SHARDS_PRESENT;
            if (np >= h.k)
                for (int i = 0; i < h.k + (data_only ? 0 : h.m); ++i) h.present[i] = 1;
        }
        return MXEC_OK;
    }

    // Consecutive objects up to kGroupBytes of present input.
    static std::vector<std::pair<size_t, size_t>> object_groups(const std::vector<RecObj>& objs, size_t o0,
                                                                size_t o1) {
        std::vector<std::pair<size_t, size_t>> groups;
        for (size_t g0 = o0; g0 < o1;) {
            size_t g1 = g0;
            uint64_t in_bytes = 0;
            while (g1 < o1) {
                uint64_t b = 0;
                for (int i = 0; i < objs[g1].k + objs[g1].m; ++i) b += objs[g1].present[i] ? objs[g1].len[i] : 0;
                if (g1 > g0 && in_bytes + b > kGroupBytes) break;
                in_bytes += b;
                ++g1;
            }
            groups.emplace_back(g0, g1);
            g0 = g1;
        }
        return groups;
    }

    // Verification groups of a piece-major reconstruct wave: cut points
    // (first o0, last o1) by upload bytes; MXEC_GET_VGROUPS of them, or (0,
    // the default) the count the model below picks per wave.  Group j + 1's
    // pieces go up and hash while group j's verdicts come back and its
    // rebuilt shards go down, so only the last group's download follows the
    // last verdict.  Measured at 512 x 4+2 x 10 MiB with SDMA downloads
    // (profiles/r5/get_groups/vgroups_*_r5q.jsonl): one group 0.634 s, two
    // 0.588, three 0.584, four 0.618; with every group's download by waves
    // no count gained (0.637-0.690: wave copies beside the later groups'
    // SHA-256 chains slow the chains).  Round 5's first measurement (one
    // 0.655, two 0.818) predates the one-copy expected-digest upload.
    // `one`: one group unless MXEC_GET_VGROUPS forces a count (rec_wave).
    std::vector<size_t> verify_cuts(const std::vector<RecObj>& objs, size_t o0, size_t o1, uint64_t up_bytes,
                                    uint64_t longest, uint64_t down_bytes, bool one) const {
        int G = d_.kn ? int(d_.kn->get_vgroups) : 1;
        if (G == 0 && one) G = 1;
        if (G == 0) {
            // Per wave: the G that minimises max(T, (G-1)/G T + C) + D/G --
            // the upload T (~50 GB/s), the chain C of the longest message,
            // the rebuilt shards' download D (~55 GB/s), of which only the
            // last group's is on the critical path.  512 x 4+2 x 10 MiB: 2
            // (0.588 s against 0.634 for one group, with SDMA downloads);
            // 128: 1 (the chain outlasts the upload).
            const double T = double(up_bytes) / 50e9, D = double(down_bytes) / 55e9;
            const double C = double(longest / 64) * kShaLagUsPerBlock * 1e-6;
            double best = 0;
            for (int g = 1; g <= 4; ++g) {
                const double t = std::max(T, (g - 1) * T / g + C) + D / g + 0.005 * (g - 1);
                if (g == 1 || t < best) {
                    best = t;
                    G = g;
                }
            }
        }
        std::vector<size_t> cut{o0};
        const size_t n = o1 - o0;
        if (G > 1 && n >= size_t(G)) {
            uint64_t acc = 0;
            int next = 1;
            for (size_t o = o0; o < o1 && next < G; ++o) {
                for (int i = 0; i < objs[o].k + objs[o].m; ++i) acc += objs[o].present[i] ? objs[o].len[i] : 0;
                if (double(acc) >= double(up_bytes) * next / G && o + 1 < o1) {
                    cut.push_back(o + 1);
                    ++next;
                }
            }
        }
        cut.push_back(o1);
        return cut;
    }

    // The expected digests of objects [o0, o1) (message order from message
    // mb) up in one copy: one per object went through the four-buffer
    // staging ring, so every fourth object waited for the upload stream to
    // reach the copy three objects back (the host enqueue crawled beside the
    // GPU, and so did the watch's bracket around it).
    int upload_expected(const std::vector<RecObj>& objs, size_t o0, size_t o1, uint8_t* exp, uint64_t mb) {
        uint64_t gm = 0;
        bool any = false;
        for (size_t o = o0; o < o1; ++o) {
            gm += uint64_t(objs[o].k + objs[o].m);
            any = any || objs[o].expected;
        }
        if (!any || !gm) return MXEC_OK;
        exp_host_.assign(gm * 32, 0);
        uint64_t g = 0;
        for (size_t o = o0; o < o1; ++o) {
            const RecObj& h = objs[o];
            if (h.expected) std::memcpy(&exp_host_[g * 32], &h.expected[0][0], uint64_t(h.k + h.m) * 32);
            g += uint64_t(h.k + h.m);
        }
        MXEC_TRY(flush_up());
        return upload(exp + mb * 32, exp_host_.data(), gm * 32);
    }
    std::vector<uint8_t> exp_host_;  // staging source of upload_expected (consumed by upload's ring copy)

    // Objects `which` of a wave, their present shards up (or verified):
    // rebuild each object's missing shards from its decode plan (one grouped
    // launch, run_rs_mixed, on cs after `up` if given), then send them down
    // to the caller's buffers and mark them present.  An object short of k
    // shards gets MXEC_E_TOO_FEW_SHARDS_PRESENT and none of its buffers is
    // written here.
    int rebuild_range(std::vector<RecObj>& objs, size_t q0, size_t q1, hipStream_t cs, hipEvent_t up, bool data_only) {
        std::vector<size_t> which(q1 - q0);
        for (size_t o = q0; o < q1; ++o) which[o - q0] = o;
        return rebuild_list(objs, which, cs, up, data_only);
    }
    int rebuild_list(std::vector<RecObj>& objs, const std::vector<size_t>& which, hipStream_t cs, hipEvent_t up,
                     bool data_only) {
        uint8_t* base = static_cast<uint8_t*>(pool_.p);
        if (cs == d2h_) MXEC_TRY(issue_down());  // wave copy blocks queued for d2h go before this launch
        if (up) MXEC_HIP(hipStreamWaitEvent(cs, up, 0));
        {
            const size_t n = which.size();
            std::vector<std::shared_ptr<const DecodePlan>> plans(n);
            std::vector<uint32_t> offs(n);
            std::vector<const uint8_t*> in;
            std::vector<uint8_t*> out;
            std::vector<uint64_t> il, ol;
            std::map<int, std::vector<RsMixedObject>> rs_groups;
            auto collect = [&]() -> int {
                for (size_t t = 0; t < n; ++t) {
                    const RecObj& h = objs[which[t]];
                    MXEC_TRY(decode_plan(d_, h.k, h.m, h.present, data_only, &plans[t], &offs[t]));
                }
                return MXEC_OK;
            };
            auto launch = [&]() -> int {
                size_t n_in = 0, n_out = 0;
                for (size_t t = 0; t < n; ++t)
                    if (plans[t] && !plans[t]->missing.empty()) {
                        n_in += size_t(objs[which[t]].k);
                        n_out += plans[t]->missing.size();
                    }
                in.assign(n_in, nullptr);
                out.assign(n_out, nullptr);
                il.assign(n_in, 0);
                ol.assign(n_out, 0);
                rs_groups.clear();
                size_t pi = 0, po = 0;
                for (size_t t = 0; t < n; ++t) {
                    if (!plans[t] || plans[t]->missing.empty()) continue;
                    const RecObj& h = objs[which[t]];
                    const DecodePlan& p = *plans[t];
                    const int r = int(p.missing.size());
                    uint8_t* ob = base + h.pool_off;
                    for (int v = 0; v < h.k; ++v) {
                        in[pi + v] = ob + uint64_t(p.valid[size_t(v)]) * h.slot();
                        il[pi + v] = h.len[p.valid[size_t(v)]];
                    }
                    for (int e = 0; e < r; ++e) {
                        out[po + e] = ob + uint64_t(p.missing[size_t(e)]) * h.slot();
                        ol[po + e] = h.len[p.missing[size_t(e)]];
                    }
                    rs_groups[r].push_back(
                        RsMixedObject{h.k, h.S, RsObject{&in[pi], &il[pi], &out[po], &ol[po], offs[t]}});
                    pi += size_t(h.k);
                    po += size_t(r);
                }
                return run_rs_mixed(d_, slot_, cs, rs_groups, &arena_);
            };
            MXEC_TRY(with_stable_coef(d_, cs, collect, launch));
            PTRACE(mark("rs", cs));
            PTRACE(now("rs_queued"));
            MXEC_TRY(issue_down());
            if (cs != d2h_) {
                hipEvent_t rs_done;
                MXEC_TRY(new_event(&rs_done));
                MXEC_HIP(hipEventRecord(rs_done, cs));
                MXEC_HIP(hipStreamWaitEvent(d2h_, rs_done, 0));
            }
            MXEC_TRY(dwatch_open());
            for (size_t t = 0; t < n; ++t) {
                RecObj& h = objs[which[t]];
                const auto& p = plans[t];
                *h.status = p ? MXEC_OK : MXEC_E_TOO_FEW_SHARDS_PRESENT;
                if (!p) continue;
                for (int e : p->missing) {
                    MXEC_TRY(queue_down(h.shards[e], base + h.pool_off + uint64_t(e) * h.slot(), h.len[e]));
                    if (h.len[e] != h.slot()) MXEC_TRY(flush_down());
                    h.present[e] = 1;
                }
            }
            MXEC_TRY(flush_down());
            MXEC_TRY(dwatch_close());
        }
        return MXEC_OK;
    }

    // Speculative rebuild of piece [off, off + pw) of objects [o0, o1)
    // (MXEC_GET_SPECULATE): once the piece of every present shard is up
    // (`up`), the same piece of each object's missing shards is decoded from
    // its first k present shards -- RS is bytewise, so a piece of the output
    // comes from the same piece of the inputs, as in the PUT's piece-major
    // encode -- and goes down to the caller's buffers.  Launch and downloads
    // both on the D2H stream, so the downloads follow the decode in order.
    // An object short of k present shards is skipped (it fails anyway).
    // ds: the stream the decode runs on (spec_stream) -- the D2H stream
    // itself, or another, the downloads then waiting for it.
    int spec_piece(std::vector<RecObj>& objs, size_t o0, size_t o1, uint64_t off, uint64_t pw, hipEvent_t up,
                   bool data_only, hipStream_t ds) {
        uint8_t* base = static_cast<uint8_t*>(pool_.p);
        const size_t n = o1 - o0;
        std::vector<std::shared_ptr<const DecodePlan>> plans(n);
        std::vector<uint32_t> offs(n);
        std::vector<const uint8_t*> in;
        std::vector<uint8_t*> out;
        std::vector<uint64_t> il, ol;
        std::map<int, std::vector<RsMixedObject>> rs_groups;
        auto collect = [&]() -> int {
            for (size_t t = 0; t < n; ++t) {
                const RecObj& h = objs[o0 + t];
                plans[t].reset();
                if (h.S > off) MXEC_TRY(decode_plan(d_, h.k, h.m, h.present, data_only, &plans[t], &offs[t]));
            }
            return MXEC_OK;
        };
        auto launch = [&]() -> int {
            size_t n_in = 0, n_out = 0;
            for (size_t t = 0; t < n; ++t)
                if (plans[t] && !plans[t]->missing.empty()) {
                    n_in += size_t(objs[o0 + t].k);
                    n_out += plans[t]->missing.size();
                }
            in.assign(n_in, nullptr);
            out.assign(n_out, nullptr);
            il.assign(n_in, 0);
            ol.assign(n_out, 0);
            rs_groups.clear();
            size_t pi = 0, po = 0;
            for (size_t t = 0; t < n; ++t) {
                if (!plans[t] || plans[t]->missing.empty()) continue;
                const RecObj& h = objs[o0 + t];
                const DecodePlan& p = *plans[t];
                const int r = int(p.missing.size());
                uint8_t* ob = base + h.pool_off + off;
                for (int v = 0; v < h.k; ++v) {
                    const uint64_t L = h.len[p.valid[size_t(v)]];
                    in[pi + v] = ob + uint64_t(p.valid[size_t(v)]) * h.slot();
                    il[pi + v] = L > off ? std::min(pw, L - off) : 0;
                }
                for (int e = 0; e < r; ++e) {
                    const uint64_t L = h.len[p.missing[size_t(e)]];
                    out[po + e] = ob + uint64_t(p.missing[size_t(e)]) * h.slot();
                    ol[po + e] = L > off ? std::min(pw, L - off) : 0;
                }
                rs_groups[r].push_back(RsMixedObject{h.k, std::min(pw, h.S - off),
                                                     RsObject{&in[pi], &il[pi], &out[po], &ol[po], offs[t]}});
                pi += size_t(h.k);
                po += size_t(r);
            }
            return rs_groups.empty() ? MXEC_OK : run_rs_mixed(d_, slot_, ds, rs_groups, &arena_, spec_blocks());
        };
        MXEC_TRY(flush_down());
        MXEC_TRY(issue_down());  // wave copy blocks queued earlier go before the wait
        if (ds == d2h_) {
            MXEC_HIP(hipStreamWaitEvent(d2h_, up, 0));
            MXEC_TRY(with_stable_coef(d_, d2h_, collect, launch));
        } else {
            MXEC_HIP(hipStreamWaitEvent(ds, up, 0));
            MXEC_TRY(with_stable_coef(d_, ds, collect, launch));
            hipEvent_t done;
            MXEC_TRY(new_event(&done));
            MXEC_HIP(hipEventRecord(done, ds));
            MXEC_HIP(hipStreamWaitEvent(d2h_, done, 0));
        }
        bool any = false;
        for (size_t t = 0; t < n; ++t) {
            if (!plans[t]) continue;
            const RecObj& h = objs[o0 + t];
            for (int e : plans[t]->missing) {
                const uint64_t L = h.len[e];
                if (off >= L) continue;
                MXEC_TRY(queue_down(h.shards[e] + off, base + h.pool_off + uint64_t(e) * h.slot() + off,
                                    std::min(pw, L - off)));
                any = true;
            }
        }
        MXEC_TRY(flush_down());
        PTRACE(mark("sdown", d2h_));
        if (any) ++d_.spec_pieces;
        return MXEC_OK;
    }

    // Piece-major upload of every present shard of objects [o0, o1) (and the
    // expected digests), each piece of the shards to verify hashed on cs as
    // soon as it is up with the chains carried in device state slots
    // (run_sha_pieces, slot = message index in the wave starting at mb,
    // verdict ok[slot]); after the last piece the verdicts are copied back
    // and *verdict recorded.  Returns without waiting.
    // P: the wave's piece size (piece_bytes over the whole wave: a group's
    // copies are as large as the wave's, whatever its share of the upload).
    // Above 1 MiB the same piece of an object's adjacent present shards goes
    // up as one 2D copy, as in the PUT's upload-bound waves.
    // spec: each piece's missing shards are also decoded and sent down as
    // soon as the piece is up (spec_piece).
    int verify_enqueue(std::vector<RecObj>& objs, size_t o0, size_t o1, uint8_t* ok, uint8_t* exp, uint64_t mb,
                       uint64_t P, hipStream_t cs, hipEvent_t* verdict, bool spec, bool data_only) {
        uint8_t* base = static_cast<uint8_t*>(pool_.p);
        uint32_t* state = static_cast<uint32_t*>(state_.p);
        uint64_t longest = 0, gm = 0;
        for (size_t o = o0; o < o1; ++o) {
            gm += uint64_t(objs[o].k + objs[o].m);
            for (int i = 0; i < objs[o].k + objs[o].m; ++i)
                if (objs[o].present[i]) longest = std::max(longest, objs[o].len[i]);
        }
        PieceGrid grid(P, piece_ramp_);
        MXEC_TRY(upload_expected(objs, o0, o1, exp, mb));
        struct TwoD {
            bool& f;
            TwoD(bool& flag, bool on) : f(flag) { f = on; }
            ~TwoD() { f = false; }
        } twod(pieces2d_, !waves_now_ && P > (uint64_t(1) << 20));
        for (uint64_t pc = 0; pc < grid.count(longest); ++pc) {
            widen_if_shared(grid, pc);
            // the ramp's small pieces are not timed: their many small copies
            // run near the floor on a healthy SDMA (a false verdict sent the
            // default line's PUT with digests to waves, 0.316 s)
            if (grid.width(pc) == grid.P) MXEC_TRY(watch_open());
            const uint64_t off = grid.start(pc), pw = grid.width(pc);
            uint64_t g = mb;
            std::vector<const uint8_t*> sp;
            std::vector<uint64_t> sl, st;
            std::vector<uint32_t> ss;
            for (size_t o = o0; o < o1; ++o) {
                const RecObj& h = objs[o];
                for (int i = 0; i < h.k + h.m; ++i, ++g) {
                    if (!h.present[i]) continue;
                    const uint64_t L = h.len[i];
                    uint8_t* dev = base + h.pool_off + uint64_t(i) * h.slot();
                    if (off < L) MXEC_TRY(queue_up(dev + off, h.shards[i] + off, std::min(pw, L - off)));
                    if (!h.expected || (off >= L && !(pc == 0 && L == 0))) continue;
                    const uint64_t len = L > off ? std::min(pw, L - off) : 0;
                    sp.push_back(dev + off);
                    sl.push_back(len);
                    st.push_back(off + len == L ? L : kShaNotFinal);
                    ss.push_back(uint32_t(g));
                }
            }
            MXEC_TRY(flush_up());
            hipEvent_t up;
            MXEC_TRY(new_event(&up));
            MXEC_TRY(issue_up());
            MXEC_HIP(hipEventRecord(up, h2d_));
            MXEC_TRY(watch_close());
            PTRACE(mark("up", h2d_));
            MXEC_HIP(hipStreamWaitEvent(cs, up, 0));
            if (!sp.empty())
                MXEC_TRY(run_sha_pieces(d_, slot_, cs, sp, sl, ss, st, state, pc > 0, nullptr, &arena_, exp, ok));
            PTRACE(mark("sha", cs));
            if (spec) MXEC_TRY(spec_piece(objs, o0, o1, off, pw, up, data_only, spec_stream(cs)));
            MXEC_TRY(pace(up));
        }
        paced_.clear();
        PTRACE(now("pieces_queued"));
        MXEC_HIP(hipMemcpyAsync(static_cast<uint8_t*>(flags_.p) + mb, ok + mb, gm, hipMemcpyDeviceToHost, cs));
        MXEC_TRY(new_event(verdict));
        MXEC_HIP(hipEventRecord(*verdict, cs));
        return MXEC_OK;
    }

    // Waits for objects [o0, o1)'s verdicts (verify_enqueue): a mismatch
    // becomes an erasure (chunk_reader.rs:176-196).
    // The objects whose masks changed go to *changed (ascending).
    int verify_collect(std::vector<RecObj>& objs, size_t o0, size_t o1, uint64_t mb, hipEvent_t verdict,
                       std::vector<size_t>* changed) {
        MXEC_HIP(hipEventSynchronize(verdict));
        const auto* okh = static_cast<const uint8_t*>(flags_.p);
        uint64_t g = mb;
        for (size_t o = o0; o < o1; ++o) {
            RecObj& h = objs[o];
            bool c = false;
            for (int i = 0; i < h.k + h.m; ++i, ++g)
                if (h.expected && h.present[i] && !okh[g]) {
                    h.present[i] = 0;
                    c = true;
                }
            if (c) changed->push_back(o);
        }
        return MXEC_OK;
    }

    // Phase 1: every upload, one event per group; phase 2 (verification
    // only): one launch over every present shard of the objects that carry
    // digests once all are up, verdicts read back.
    int upload_and_verify(std::vector<RecObj>& objs, size_t o0, size_t o1,
                          const std::vector<std::pair<size_t, size_t>>& groups, uint8_t* ok, uint8_t* exp, bool verify,
                          hipStream_t cs, std::vector<hipEvent_t>* up_out) {
        uint8_t* base = static_cast<uint8_t*>(pool_.p);
        std::vector<hipEvent_t>& up = *up_out;
        up.assign(groups.size(), nullptr);
        if (verify) MXEC_TRY(upload_expected(objs, o0, o1, exp, 0));
        uint64_t g = 0;
        for (size_t q = 0; q < groups.size(); ++q) {
            MXEC_TRY(watch_open());
            for (size_t o = groups[q].first; o < groups[q].second; ++o) {
                const RecObj& h = objs[o];
                for (int i = 0; i < h.k + h.m; ++i) {
                    if (!h.present[i]) continue;
                    MXEC_TRY(queue_up(base + h.pool_off + uint64_t(i) * h.slot(), h.shards[i], h.len[i]));
                    if (h.len[i] != h.slot()) MXEC_TRY(flush_up());
                }
                MXEC_TRY(flush_up());
                g += uint64_t(h.k + h.m);
            }
            MXEC_TRY(flush_up());
            MXEC_TRY(new_event(&up[q]));
            MXEC_TRY(issue_up());
            MXEC_HIP(hipEventRecord(up[q], h2d_));
            MXEC_TRY(watch_close());
            MXEC_TRY(pace(up[q]));
        }
        paced_.clear();
        if (verify) {
            std::vector<const uint8_t*> sp;
            std::vector<uint64_t> sl, idx;
            std::vector<std::pair<size_t, int>> who;  // message -> (object, shard)
            g = 0;
            for (size_t o = o0; o < o1; ++o) {
                const RecObj& h = objs[o];
                for (int i = 0; i < h.k + h.m; ++i, ++g) {
                    if (!h.expected || !h.present[i]) continue;
                    sp.push_back(base + h.pool_off + uint64_t(i) * h.slot());
                    sl.push_back(h.len[i]);
                    idx.push_back(g);
                    who.emplace_back(o, i);
                }
            }
            MXEC_HIP(hipStreamWaitEvent(cs, up.back(), 0));
            if (!sp.empty()) {
                MXEC_TRY(run_sha(d_, slot_, cs, sp, sl, nullptr, exp, ok, &idx, &arena_));
                MXEC_TRY(flags_.grow(sp.size()));
                MXEC_HIP(hipMemcpyAsync(flags_.p, ok, sp.size(), hipMemcpyDeviceToHost, cs));
                MXEC_TRY(sync_point(cs));  // not the stream: another call's work may follow on it
                const auto* okh = static_cast<const uint8_t*>(flags_.p);
                for (size_t t = 0; t < who.size(); ++t)
                    if (!okh[t]) objs[who[t].first].present[who[t].second] = 0;
            }
        }
        return MXEC_OK;
    }

    struct Pending {  // ring DMA to copy out into pageable memory
        int ring;
        uint8_t* dst;
        uint64_t len;
    };

    Device& d_;
    hipStream_t h2d_, d2h_;
    hipStream_t* cs_;
    PinRing& in_;
    PinRing& out_;
    DescArena& arena_;
    DevBuf& pool_;
    DevBuf& scratch_;  // the wave's digests, message order
#ifdef MXEC_LAB
    PipeTrace tr_;
#endif
    DevBuf& state_;    // chain states of a piece-major verification
    PinnedBuf& flags_;
    Slot& slot_;
    PipeHub& hub_;
    const uint64_t cap_;  // pool bytes per wave (the lane's admission)
    int cs_idx_ = -1;     // the compute stream this call's kernels run on (PipeHub::use)
    std::vector<Pending> pend_;
    std::vector<hipEvent_t> events_;

    int new_event(hipEvent_t* e) {
        MXEC_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
        events_.push_back(*e);
        return MXEC_OK;
    }
    // Wait for this call's work queued on `s` so far (an event, not the
    // stream: calls share the streams, and a stream sync would wait for the
    // other calls' later work too).
    int sync_point(hipStream_t s) {
        hipEvent_t e;
        MXEC_TRY(new_event(&e));
        MXEC_HIP(hipEventRecord(e, s));
        MXEC_HIP(hipEventSynchronize(e));
        return MXEC_OK;
    }
    // While another call shares the device, a call keeps at most
    // kPaceBytes of its own uploads queued ahead of the piece (or group) it
    // has just queued: the shared streams run in submission order, and a
    // call that queued all its pieces at once would put the other call's
    // uploads (and what waits on them) behind all of its own.  Bytes, not
    // pieces: with two pieces each, a GET's 1 GB pieces took twice the
    // link a PUT's 512 MiB pieces got, and the starved PUT chain set the
    // pair's end.  A lone call never waits here.
    static constexpr uint64_t kPaceBytes = uint64_t(1) << 30;
    std::deque<std::pair<hipEvent_t, uint64_t>> paced_;
    uint64_t up_since_pace_ = 0;  // bytes queue_up took since the last pace()
    int pace(hipEvent_t up) {
        paced_.emplace_back(up, up_since_pace_);
        up_since_pace_ = 0;
        auto ahead = [&] {  // queued before the newest entry
            uint64_t b = 0;
            for (size_t i = 0; i + 1 < paced_.size(); ++i) b += paced_[i].second;
            return b;
        };
        while (paced_.size() > 1) {
            hipEvent_t e = paced_.front().first;
            const hipError_t q = hipEventQuery(e);
            if (q == hipSuccess) {
                paced_.pop_front();
                continue;
            }
            (void)hipGetLastError();
            if (!shared_now() || ahead() <= kPaceBytes) break;
            ++d_.pace_waits;
            PTRACE(now("pace"));
            MXEC_HIP(hipEventSynchronize(e));
            PTRACE(now("paced"));
            paced_.pop_front();
        }
        return MXEC_OK;
    }

    // Wave copies (MXEC_PIPE_COPY, run / run_rec): copies from / to
    // mxec_host_alloc memory go as CU-wave copy launches (copy_kernel.hip)
    // instead of SDMA DMAs; they are collected here and issued as one launch
    // at the next point the stream is waited on or marked (issue_up /
    // issue_down).
    bool wave_copy(const void* host, const void* dev, uint64_t len, bool down = false) const {
        return (down ? down_waves_ : waves_now_) && copy_phase_ok(host, dev) && pinned_mapped(host, len);
    }
    bool waves_now_ = false;  // this call's copies of mxec_host_alloc memory go by waves
    bool down_waves_ = false;  // its downloads (lab: MXEC_PIPE_DOWN_WAVES=1 forces them)
    static void add_blocks(std::vector<CopyBlk>& v, uint8_t* dst, const uint8_t* src, uint64_t len) {
        for (uint64_t o = 0; o < len; o += kCopyBlock)
            v.push_back(CopyBlk{reinterpret_cast<uint64_t>(dst + o), reinterpret_cast<uint64_t>(src + o),
                                std::min(kCopyBlock, len - o), 0});
    }
    // The block table goes into the arena's page-locked host half, which the
    // kernel reads in place (no table upload through the copy engines).
    int issue_blocks(std::vector<CopyBlk>& v, bool to_host, hipStream_t s) {
        if (v.empty()) return MXEC_OK;
        const size_t bytes = (v.size() * sizeof(CopyBlk) + 255) & ~size_t(255);
        char* h = nullptr;
        char* d = nullptr;
        MXEC_TRY(arena_.take(bytes, &h, &d));
        std::memcpy(h, v.data(), v.size() * sizeof(CopyBlk));
        uint32_t grid = kCopyGrid;
#ifdef MXEC_LAB
        if (const char* e = getenv("MXEC_PIPE_COPY_GRID")) grid = uint32_t(atoi(e));  // lab
#endif
        MXEC_HIP(launch_copy_blocks(reinterpret_cast<const CopyBlk*>(h), v.size(), to_host, grid, s));
        d_.copy_wave_blocks += v.size();
        v.clear();
        return MXEC_OK;
    }
    int issue_up() { return issue_blocks(up_blks_, false, h2d_); }
    int issue_down() {
        if (down_blks_.empty()) return MXEC_OK;
        MXEC_TRY(issue_blocks(down_blks_, true, d2h_));
        return mark_d2h();
    }
    // This call's newest work on the D2H stream, re-recorded after each of
    // its enqueues there: the call's end waits for it, not for a fresh event
    // behind the other calls' downloads queued since (a verified GET beside a
    // PUT ended with the PUT's parity downloads, ~100 ms after its own).
    hipEvent_t d2h_mark_ = nullptr;
    int mark_d2h() {
        if (!d2h_mark_) MXEC_TRY(new_event(&d2h_mark_));
        MXEC_HIP(hipEventRecord(d2h_mark_, d2h_));
        return MXEC_OK;
    }
    std::vector<CopyBlk> up_blks_, down_blks_;
    // Workgroups per copy launch: few, so the copy's host loads in flight do
    // not queue ahead of the SHA-256 chains' HBM loads (128 slowed the chains
    // 5x; 16 moves 57 GB/s alone and left the verified GET's chains alone).
    static constexpr uint32_t kCopyGrid = 16;

    int upload(uint8_t* dst, const uint8_t* src, uint64_t len) {
        if (!len) return MXEC_OK;
        if (affinity_on(d_)) {
            const void* p = dst;
            MXEC_TRY(affinity_check(d_, &slot_, h2d_, "pipeline upload", &arena_, &p, 1));
        }
        if (wave_copy(src, dst, len)) {
            add_blocks(up_blks_, dst, src, len);
            return MXEC_OK;
        }
        if (is_pinned(src, len)) {
            MXEC_HIP(hipMemcpyAsync(dst, src, len, hipMemcpyHostToDevice, h2d_));
            ++d_.copies_1d;
            return watch_count(false, len, 1);
        }
        watch_staged_ = true;  // host memcpy through the ring: not an SDMA rate
        for (uint64_t off = 0; off < len; off += kRingBuf) {
            const uint64_t n = std::min(kRingBuf, len - off);
            int r;
            MXEC_TRY(in_.take(&r));
            std::memcpy(in_.ptr(r), src + off, n);
            MXEC_HIP(hipMemcpyAsync(dst + off, in_.ptr(r), n, hipMemcpyHostToDevice, h2d_));
            ++d_.copies_1d;
            MXEC_TRY(in_.mark(r, h2d_));
        }
        return MXEC_OK;
    }

    // Adjacent copies -- the next one starts where the last one ended, on the
    // host and on the device -- go as one DMA: an object's k data chunks are
    // usually contiguous in the request body and always in its device image
    // (and its m parity chunks likewise), so 4+2 objects take 2 copies
    // instead of 6.  In the PUT's piece-major waves (SDMA copies), copies of
    // one width at one pitch on each side -- the same piece of an object's k
    // data chunks, of its m parity chunks -- go as one 2D copy when the host
    // side is page-locked -- when the wave is upload-bound (pieces above
    // 1 MiB): PUT with digests 0.516 -> 0.457 s at 512 objects, 0.301 ->
    // 0.283 at 256 (profiles/r4/e2e_pieces/copy2d/).  At 1 MiB pieces (a
    // chain-bound wave, 128 objects) 2D copies won 2 % in the e2e tool but
    // the default bench line's leg ran 0.300 s against 0.219 with 1D copies
    // (`copy2d/bench_2d_at_1MiB_*.json`), as in round 3, so they stay 1D
    // there.  Nowhere else: in round 3 the GET group form's 2D runs of
    // whole 10 MiB shards fell from 0.113 to 0.150-0.266 s
    // (profiles/r3/pieces/).  MXEC_PIPE_COPY2D=0/1 (lab builds) forces it
    // off / on everywhere.  queue_up / queue_down collect; flush_up /
    // flush_down issue (before an event is recorded on the copy stream).
    struct Run {
        uint8_t* dst = nullptr;
        const uint8_t* src = nullptr;
        uint64_t len = 0;   // row width (0: empty)
        uint64_t rows = 0;
        uint64_t dpitch = 0, spitch = 0;
    };
    bool copy2d_on() const {
#ifdef MXEC_LAB
        if (const char* e = getenv("MXEC_PIPE_COPY2D")) return atoi(e) != 0;  // lab override
#endif
        return pieces2d_;
    }
    bool pieces2d_ = false;  // set while a PUT piece-major wave queues its copies
    bool extend(Run& r, uint8_t* dst, const uint8_t* src, uint64_t len) const {
        if (!r.len) return false;
        if (r.rows == 1 && r.dst + r.len == dst && r.src + r.len == src) {
            r.len += len;
            return true;
        }
        if (len != r.len || !copy2d_on()) return false;
        if (r.rows == 1) {
            if (dst < r.dst + len || src < r.src + len) return false;
            r.dpitch = uint64_t(dst - r.dst);
            r.spitch = uint64_t(src - r.src);
            r.rows = 2;
            return true;
        }
        if (dst != r.dst + r.rows * r.dpitch || src != r.src + r.rows * r.spitch) return false;
        ++r.rows;
        return true;
    }
    Run up_run_, down_run_;
    int queue_up(uint8_t* dst, const uint8_t* src, uint64_t len) {
        if (!len) return MXEC_OK;
        up_since_pace_ += len;
        if (extend(up_run_, dst, src, len)) return MXEC_OK;
        MXEC_TRY(flush_up());
        up_run_ = Run{dst, src, len, 1, 0, 0};
        return MXEC_OK;
    }
    int flush_up() {
        const Run r = up_run_;
        up_run_ = Run{};
        if (!r.len) return MXEC_OK;
        if (r.rows == 1) return upload(r.dst, r.src, r.len);
        if (!waves_now_ && is_pinned(r.src, (r.rows - 1) * r.spitch + r.len)) {
            if (affinity_on(d_)) {
                const void* p = r.dst;
                MXEC_TRY(affinity_check(d_, &slot_, h2d_, "pipeline upload 2d", &arena_, &p, 1));
            }
            MXEC_HIP(hipMemcpy2DAsync(r.dst, r.dpitch, r.src, r.spitch, r.len, r.rows, hipMemcpyHostToDevice, h2d_));
            ++d_.copies_2d;
            d_.copies_2d_rows += r.rows;
            return watch_count(false, r.len * r.rows, r.rows);
        }
        for (uint64_t i = 0; i < r.rows; ++i) MXEC_TRY(upload(r.dst + i * r.dpitch, r.src + i * r.spitch, r.len));
        return MXEC_OK;
    }
    int queue_down(uint8_t* dst, const uint8_t* src, uint64_t len) {
        if (!len) return MXEC_OK;
        if (extend(down_run_, dst, src, len)) return MXEC_OK;
        MXEC_TRY(flush_down());
        down_run_ = Run{dst, src, len, 1, 0, 0};
        return MXEC_OK;
    }
    int flush_down() {
        if (!down_run_.len) return MXEC_OK;
        MXEC_TRY(flush_down_run());
        return mark_d2h();
    }
    int flush_down_run() {
        const Run r = down_run_;
        down_run_ = Run{};
        if (!r.len) return MXEC_OK;
        if (r.rows == 1) return download(r.dst, r.src, r.len);
        if (!down_waves_ && is_pinned(r.dst, (r.rows - 1) * r.dpitch + r.len)) {
            if (affinity_on(d_)) {
                const void* p = r.src;
                MXEC_TRY(affinity_check(d_, &slot_, d2h_, "pipeline download 2d", &arena_, &p, 1));
            }
            MXEC_HIP(hipMemcpy2DAsync(r.dst, r.dpitch, r.src, r.spitch, r.len, r.rows, hipMemcpyDeviceToHost, d2h_));
            ++d_.copies_2d;
            d_.copies_2d_rows += r.rows;
            return watch_count(true, r.len * r.rows, r.rows);
        }
        for (uint64_t i = 0; i < r.rows; ++i) MXEC_TRY(download(r.dst + i * r.dpitch, r.src + i * r.spitch, r.len));
        return MXEC_OK;
    }

    // Copy out the pending ring buffer the next take() will reuse.
    int drain_next() {
        const int r = out_.next();
        for (size_t i = 0; i < pend_.size(); ++i) {
            if (pend_[i].ring != r) continue;
            MXEC_HIP(hipEventSynchronize(out_.event(r)));
            std::memcpy(pend_[i].dst, out_.ptr(r), pend_[i].len);
            pend_.erase(pend_.begin() + long(i));
            break;
        }
        return MXEC_OK;
    }

    int download(uint8_t* dst, const uint8_t* src, uint64_t len) {
        if (!len) return MXEC_OK;
        if (affinity_on(d_)) {
            const void* p = src;
            MXEC_TRY(affinity_check(d_, &slot_, d2h_, "pipeline download", &arena_, &p, 1));
        }
        if (wave_copy(dst, src, len, true)) {
            add_blocks(down_blks_, dst, src, len);
            return MXEC_OK;
        }
        if (is_pinned(dst, len)) {
            MXEC_HIP(hipMemcpyAsync(dst, src, len, hipMemcpyDeviceToHost, d2h_));
            ++d_.copies_1d;
            return watch_count(true, len, 1);
        }
        dwatch_staged_ = true;
        for (uint64_t off = 0; off < len; off += kRingBuf) {
            const uint64_t n = std::min(kRingBuf, len - off);
            MXEC_TRY(drain_next());
            int r;
            MXEC_TRY(out_.take(&r));
            MXEC_HIP(hipMemcpyAsync(out_.ptr(r), src + off, n, hipMemcpyDeviceToHost, d2h_));
            ++d_.copies_1d;
            MXEC_TRY(out_.mark(r, d2h_));
            pend_.push_back(Pending{r, dst + off, n});
        }
        return MXEC_OK;
    }

    int flush() {
        MXEC_TRY(issue_down());  // marks what it issues
        if (d2h_mark_) MXEC_HIP(hipEventSynchronize(d2h_mark_));
        for (auto& p : pend_) std::memcpy(p.dst, out_.ptr(p.ring), p.len);
        pend_.clear();
        out_.release_all();
        return MXEC_OK;
    }

    // Piece-major form of a wave with digests (MXEC_PIPE_PIECE_MB, default 1;
    // 0 = the group form below).  The group form uploads object after object
    // and hashes once all parity exists, so the last-uploaded chunk's chain
    // (163 840 blocks for 10 MiB) starts after the whole upload: 94 + 203 ms
    // for 128 x 4+2 x 10 MiB.  Here piece p (bytes [pP, (p+1)P) of every
    // chunk) goes up, is encoded, hashed -- the chains carried from piece to
    // piece in device state slots (run_sha_pieces) -- and its parity goes
    // down, piece after piece, so every chain starts after the first piece
    // (~9 ms) and the wave ends near one chain's length.  Taken when the
    // wave's messages fit the lag quad form (64 per CU).
    //
    // Piece size (MXEC_PIPE_PIECE_MB; unset = per wave): small pieces start
    // the chains early, but each piece of each chunk is its own copy, and
    // 1 MiB copies move ~33 GB/s where 4 MiB ones move ~43 (PUT with digests,
    // 512 x 4+2 x 10 MiB: 0.645 s at 1 MiB, 0.557 at 2, 0.503 at 4; 128
    // objects: 0.218 / 0.227 / 0.246 s, profiles/r4/e2e_pieces/).  So a wave
    // takes the smallest piece whose upload, at that piece's copy rate, still
    // fits inside the longest chain (the wave's floor either way), else 4 MiB.
    //
    // A chain-bound verified GET wave (its upload fits inside its longest
    // chain) also ramps its first pieces up from 256 KiB (piece_ramp_,
    // PieceGrid): it ends about one chain after its first piece is up, so a
    // smaller first piece ends it sooner -- 128 x 4+2 x 10 MiB 0.2406 s
    // against 0.2475 with its uploads by waves (rec_wave).  The PUT with
    // digests lost to the same ramp (0.214-0.223 against 0.2033 by SDMA;
    // profiles/r5/get_groups/ramp_ab_final_r5ab.jsonl), and an upload-bound
    // wave loses to the extra copies (512 objects: 0.606 against 0.588,
    // ramp_*_r5u.jsonl), so wave() clears it and only chain-bound waves set it.
    //
    // While other calls share the device, they share its upload link too: the
    // wave's upload is weighed as if it were the calls-in-flight times larger
    // (a PUT with digests beside a verified GET, 128 x 4+2 x 10 MiB each:
    // 10.7 GB over the link against a 191 ms chain, upload-bound, so 4 MiB
    // pieces and 2D copies instead of 1 MiB ones at ~33 GB/s).
    uint64_t piece_bytes(uint64_t upload_bytes, uint64_t longest) {
        piece_ramp_ = 0;
        if (!d_.kn) return uint64_t(1) << 20;
        if (!d_.kn->pipe_piece_auto) return d_.kn->pipe_piece;
        bool share = true;
#ifdef MXEC_LAB
        if (const char* e = getenv("MXEC_PIPE_SHARE_PIECES")) share = *e != '0';  // lab A/B
#endif
        const int calls = std::max(1, hub_.calls.load());
        if (share) upload_bytes *= uint64_t(calls);
        const double chain_s = double(longest / 64) * kShaLagUsPerBlock * 1e-6;
        static constexpr struct {
            uint64_t bytes;
            double gbps;  // sustained H2D rate of copies this size, measured (above)
        } kSteps[] = {{uint64_t(1) << 20, 33.0}, {uint64_t(2) << 20, 38.0}};
        for (const auto& s : kSteps)
            if (double(upload_bytes) / (s.gbps * 1e9) <= chain_s) {
                piece_ramp_ = uint64_t(256) << 10;
                return s.bytes;
            }
        // Upload-bound.  A wave that shares the link still ramps: its first
        // pieces go up between the other call's, so both calls' chains start
        // early (without, a GET's first 4 MiB piece -- 2 GB for 128 x 4+2 --
        // held a PUT's first piece back 45 ms, and the PUT's chain set the
        // pair's end).
        if (share && calls > 1) {
            piece_ramp_ = uint64_t(256) << 10;
            return uint64_t(2) << 20;  // pieces the other call's can interleave with (2D copies above 1 MiB)
        }
        return uint64_t(4) << 20;
    }
    uint64_t piece_ramp_ = 0;  // first piece of the current wave's ramp (0: none)

    // A wave sized while it had the device to itself (1 MiB pieces: its
    // upload fit inside its chains) goes on in 2 MiB pieces, 2D copies, once
    // another call shares the link -- piece_bytes' choice had it known (a
    // PUT with digests admitted just before a verified GET otherwise kept
    // its ~33 GB/s 1 MiB copies through the pair and ended ~90 ms after the
    // GET).
    void widen_if_shared(PieceGrid& grid, uint64_t pc) {
        static constexpr uint64_t kShared = uint64_t(2) << 20;
        if (!d_.kn || !d_.kn->pipe_piece_auto || pc < grid.starts.size() || grid.P >= kShared || !shared_now())
            return;
#ifdef MXEC_LAB
        if (const char* e = getenv("MXEC_PIPE_WIDEN"))
            if (*e == '0') return;  // lab A/B
#endif
        grid.widen(pc, kShared);
        pieces2d_ = !waves_now_;
    }

    int wave_pieces(std::vector<HostObj>& objs, size_t o0, size_t o1, uint64_t P) {
        Slot& slot = slot_;
        uint8_t* base = static_cast<uint8_t*>(pool_.p);
        // Chains: every chunk of every object that wants digests, message order.
        struct Chain {
            uint8_t* dev;
            uint64_t len;
        };
        std::vector<Chain> ch;
        uint64_t longest = 0;
        for (size_t o = o0; o < o1; ++o) {
            const HostObj& h = objs[o];
            longest = std::max(longest, h.S);
            if (!h.dig) continue;
            for (int j = 0; j < h.k + h.m; ++j)
                ch.push_back(Chain{base + h.pool_off + uint64_t(j) * h.slot(),
                                   j < h.k ? std::min<uint64_t>(h.dlen[j], h.S) : h.S});
        }
        const uint64_t nm = ch.size();
        MXEC_TRY(scratch_.grow(nm * 64));  // digests [nm][32], then chain states [nm][8] words
        uint8_t* digests = static_cast<uint8_t*>(scratch_.p);
        uint32_t* state = reinterpret_cast<uint32_t*>(digests + nm * 32);
        PieceGrid grid(P, piece_ramp_);
        // RS and the chains on the call's compute stream (PipeHub::use): each
        // piece's RS ahead of its hash, so no piece of this call waits behind
        // another call's chains.
        hipStream_t sha_s = cs_[cs_idx_], rs_s = sha_s;
        hipEvent_t sha_done = nullptr;
        struct TwoD {  // 2D piece copies for this wave's SDMA copies (queue_up)
            bool& f;
            TwoD(bool& flag, bool on) : f(flag) { f = on; }
            ~TwoD() { f = false; }
        } twod(pieces2d_, !waves_now_ && P > (uint64_t(1) << 20));
        PTRACE(start(h2d_));
        for (uint64_t pc = 0; pc < grid.count(longest); ++pc) {
            widen_if_shared(grid, pc);
            // No SDMA watch here: in the seconds after a large HBM free the
            // bracket events among the pieces cost the PUT with digests 63 %
            // (0.335 s against 0.206 unwatched at 128 objects,
            // profiles/r5/copy_engine/final_churn60_r5ag.jsonl) while its
            // uploads ran at full rate; its downloads, the direction that
            // slows, stay on SDMA either way (waves cost it 14-18 %).
            const uint64_t off = grid.start(pc), pw = grid.width(pc);
            for (size_t o = o0; o < o1; ++o) {
                const HostObj& h = objs[o];
                for (int j = 0; j < h.k; ++j) {
                    const uint64_t L = std::min<uint64_t>(h.dlen[j], h.S);
                    if (off < L)
                        MXEC_TRY(queue_up(base + h.pool_off + uint64_t(j) * h.slot() + off, h.data[j] + off,
                                          std::min(pw, L - off)));
                }
            }
            MXEC_TRY(flush_up());
            hipEvent_t up, rs_done;
            MXEC_TRY(new_event(&up));
            MXEC_TRY(new_event(&rs_done));
            MXEC_TRY(issue_up());
            MXEC_HIP(hipEventRecord(up, h2d_));
            MXEC_TRY(watch_close());
            PTRACE(mark("up", h2d_));
            PTRACE(now("up_queued"));
            MXEC_HIP(hipStreamWaitEvent(rs_s, up, 0));
            // Parity of this piece: RS is bytewise, so bytes [off, off + P) of
            // the parity come from the same bytes of the data (short data
            // chunks read as zeros past their end, as in the whole-chunk form).
            std::map<std::tuple<int, int, uint64_t>, std::vector<size_t>> classes;
            for (size_t o = o0; o < o1; ++o)
                if (objs[o].S > off) classes[{objs[o].k, objs[o].m, objs[o].S}].push_back(o);
            for (auto& c : classes) {
                const int k = std::get<0>(c.first), m = std::get<1>(c.first);
                const uint64_t S = std::get<2>(c.first), W = std::min(pw, S - off);
                uint32_t coff = 0;
                const size_t n = c.second.size();
                std::vector<const uint8_t*> ins(n * size_t(k));
                std::vector<uint8_t*> outs(n * size_t(m));
                std::vector<uint64_t> lens(n * size_t(k + m), W);
                std::vector<RsObject> ro(n);
                for (size_t t = 0; t < n; ++t) {
                    const HostObj& h = objs[c.second[t]];
                    uint8_t* ob = base + h.pool_off + off;
                    for (int j = 0; j < k; ++j) {
                        ins[t * k + j] = ob + uint64_t(j) * h.slot();
                        const uint64_t L = std::min<uint64_t>(h.dlen[j], S);
                        lens[t * (k + m) + j] = L > off ? std::min(W, L - off) : 0;
                    }
                    for (int i = 0; i < m; ++i) outs[t * m + i] = ob + uint64_t(k + i) * h.slot();
                    ro[t] = RsObject{&ins[t * k], &lens[t * (k + m)], &outs[t * m], &lens[t * (k + m) + k], 0};
                }
                MXEC_TRY(with_stable_coef(
                    d_, rs_s, [&] { return encode_coef(d_, k, m, &coff); },
                    [&] {
                        for (auto& r : ro) r.coef_off = coff;
                        return run_rs(d_, slot, rs_s, W, k, m, ro, &arena_);
                    }));
            }
            MXEC_HIP(hipEventRecord(rs_done, rs_s));
            // This piece of every chain (the hash stream runs the pieces in
            // order, each continuing the chains the previous one left).
            std::vector<const uint8_t*> sp;
            std::vector<uint64_t> sl, st;
            std::vector<uint32_t> ss;
            for (uint64_t q = 0; q < nm; ++q) {
                const Chain& c = ch[q];
                if (off >= c.len && !(pc == 0 && c.len == 0)) continue;  // ended in an earlier piece
                const uint64_t len = c.len > off ? std::min(pw, c.len - off) : 0;
                sp.push_back(c.dev + off);
                sl.push_back(len);
                st.push_back(off + len == c.len ? c.len : kShaNotFinal);
                ss.push_back(uint32_t(q));
            }
            if (!sp.empty()) {
                MXEC_HIP(hipStreamWaitEvent(sha_s, rs_done, 0));
                MXEC_TRY(run_sha_pieces(d_, slot, sha_s, sp, sl, ss, st, state, pc > 0, digests, &arena_));
                PTRACE(mark("sha", sha_s));
            }
            PTRACE(mark("rs", rs_s));
            // This piece of every parity chunk goes down.
            MXEC_TRY(issue_down());
            MXEC_HIP(hipStreamWaitEvent(d2h_, rs_done, 0));
            for (size_t o = o0; o < o1; ++o) {
                const HostObj& h = objs[o];
                if (h.S <= off) continue;
                uint8_t* ob = base + h.pool_off + off;
                for (int i = 0; i < h.m; ++i)
                    MXEC_TRY(queue_down(h.parity[i] + off, ob + uint64_t(h.k + i) * h.slot(), std::min(pw, h.S - off)));
            }
            MXEC_TRY(flush_down());
            PTRACE(mark("down", d2h_));
            PTRACE(now("piece_queued"));
            MXEC_TRY(pace(up));
        }
        paced_.clear();
        if (nm) {
            MXEC_TRY(new_event(&sha_done));
            MXEC_HIP(hipEventRecord(sha_done, sha_s));
            MXEC_TRY(issue_down());
            MXEC_HIP(hipStreamWaitEvent(d2h_, sha_done, 0));
            uint64_t msg0 = 0;
            for (size_t o = o0; o < o1; ++o) {
                const HostObj& h = objs[o];
                if (!h.dig) continue;
                MXEC_TRY(queue_down(reinterpret_cast<uint8_t*>(h.dig), digests + msg0 * 32, uint64_t(h.k + h.m) * 32));
                msg0 += uint64_t(h.k + h.m);
            }
            MXEC_TRY(flush_down());
        }
        const int frc = flush();
        PTRACE(report("wave_pieces"));
        return frc;
    }

    int wave(std::vector<HostObj>& objs, size_t o0, size_t o1) {
        {
            uint64_t msgs = 0, up_bytes = 0, longest_msg = 0;
            for (size_t o = o0; o < o1; ++o) {
                for (int j = 0; j < objs[o].k; ++j) up_bytes += std::min<uint64_t>(objs[o].dlen[j], objs[o].S);
                if (!objs[o].dig) continue;
                msgs += uint64_t(objs[o].k + objs[o].m);
                longest_msg = std::max(longest_msg, objs[o].S);
            }
            const uint64_t P = piece_bytes(up_bytes, longest_msg);
            if (!shared_now()) piece_ramp_ = 0;  // a lone PUT keeps uniform pieces (the ramp cost it 5-9 %, below)
            if (P && msgs && msgs <= uint64_t(kShaLagMsgs) * uint64_t(d_.n_cus ? d_.n_cus : 256))
                return wave_pieces(objs, o0, o1, P);
        }
        Slot& slot = slot_;
        uint8_t* base = static_cast<uint8_t*>(pool_.p);
        uint64_t msgs = 0;
        for (size_t o = o0; o < o1; ++o) msgs += uint64_t(objs[o].k + objs[o].m);
        MXEC_TRY(scratch_.grow(msgs * 32));
        uint8_t* digests = static_cast<uint8_t*>(scratch_.p);
        // Groups: consecutive objects up to kGroupBytes of input.
        std::vector<std::pair<size_t, size_t>> groups;
        for (size_t g0 = o0; g0 < o1;) {
            size_t g1 = g0;
            uint64_t in_bytes = 0;
            while (g1 < o1 && (g1 == g0 || in_bytes + uint64_t(objs[g1].k) * objs[g1].S <= kGroupBytes)) {
                in_bytes += uint64_t(objs[g1].k) * objs[g1].S;
                ++g1;
            }
            groups.emplace_back(g0, g1);
            g0 = g1;
        }
        // Phase 1: each group's upload and RS launch(es), in order.  The
        // host only waits on the input ring (an H2D copy), so uploads stream
        // at PCIe rate while RS runs behind them.
        std::vector<hipEvent_t> done(groups.size());
        bool any_dig = false;
        for (size_t o = o0; o < o1; ++o) any_dig = any_dig || objs[o].dig;
        hipStream_t rs_s = cs_[cs_idx_], sha_s = rs_s;
        // Each group's parity down: group by group after phase 1 (a lone
        // call queues all of phase 1 at once); while another call shares the
        // device, right behind the group's RS, since the paced phase 1 would
        // hold phase 3 back until the last uploads were queued.
        const bool down_early = shared_now();
        size_t downed = 0;
        auto down_group = [&](size_t g) -> int {
            MXEC_TRY(issue_down());
            MXEC_HIP(hipStreamWaitEvent(d2h_, done[g], 0));
            for (size_t o = groups[g].first; o < groups[g].second; ++o) {
                const HostObj& h = objs[o];
                uint8_t* ob = base + h.pool_off;
                for (int i = 0; i < h.m; ++i) {
                    MXEC_TRY(queue_down(h.parity[i], ob + uint64_t(h.k + i) * h.slot(), h.S));
                    if (h.S != h.slot()) MXEC_TRY(flush_down());
                }
            }
            MXEC_TRY(flush_down());  // before the next group's wait
            downed = g + 1;
            return MXEC_OK;
        };
        for (size_t g = 0; g < groups.size(); ++g) {
            MXEC_TRY(watch_open());
            const size_t g0 = groups[g].first, g1 = groups[g].second;
            for (size_t o = g0; o < g1; ++o) {
                const HostObj& h = objs[o];
                for (int j = 0; j < h.k; ++j) {
                    // a short chunk ends a run: the next chunk's slot does not follow its bytes
                    MXEC_TRY(queue_up(base + h.pool_off + uint64_t(j) * h.slot(), h.data[j], h.dlen[j]));
                    if (h.dlen[j] != h.slot()) MXEC_TRY(flush_up());
                }
            }
            MXEC_TRY(flush_up());
            hipEvent_t up;
            MXEC_TRY(new_event(&up));
            MXEC_TRY(new_event(&done[g]));
            MXEC_TRY(issue_up());
            MXEC_HIP(hipEventRecord(up, h2d_));
            MXEC_TRY(watch_close());
            MXEC_HIP(hipStreamWaitEvent(rs_s, up, 0));
            std::map<std::tuple<int, int, uint64_t>, std::vector<size_t>> classes;
            for (size_t o = g0; o < g1; ++o) classes[{objs[o].k, objs[o].m, objs[o].S}].push_back(o);
            for (auto& c : classes) {
                const int k = std::get<0>(c.first), m = std::get<1>(c.first);
                const uint64_t S = std::get<2>(c.first);
                uint32_t coff = 0;
                const size_t n = c.second.size();
                std::vector<const uint8_t*> ins(n * size_t(k));
                std::vector<uint8_t*> outs(n * size_t(m));
                std::vector<uint64_t> lens(n * size_t(k + m), S);
                std::vector<RsObject> ro(n);
                for (size_t t = 0; t < n; ++t) {
                    const HostObj& h = objs[c.second[t]];
                    uint8_t* ob = base + h.pool_off;
                    for (int j = 0; j < k; ++j) {
                        ins[t * k + j] = ob + uint64_t(j) * h.slot();
                        lens[t * (k + m) + j] = std::min<uint64_t>(h.dlen[j], S);
                    }
                    for (int i = 0; i < m; ++i) outs[t * m + i] = ob + uint64_t(k + i) * h.slot();
                    ro[t] = RsObject{&ins[t * k], &lens[t * (k + m)], &outs[t * m], &lens[t * (k + m) + k], 0};
                }
                MXEC_TRY(with_stable_coef(
                    d_, rs_s, [&] { return encode_coef(d_, k, m, &coff); },
                    [&] {
                        for (auto& r : ro) r.coef_off = coff;
                        return run_rs(d_, slot, rs_s, S, k, m, ro, &arena_);
                    }));
            }
            MXEC_HIP(hipEventRecord(done[g], rs_s));
            if (down_early) MXEC_TRY(down_group(g));
            MXEC_TRY(pace(up));
        }
        paced_.clear();
        // Phase 2: ONE SHA-256 launch over every chunk of the wave once all
        // parity exists.  A message's hash time does not depend on how many
        // messages share the launch (up to the split-form limit), so one
        // launch ends as early as any split of it would, and it needs no
        // more than one hardware queue.
        std::vector<const uint8_t*> sp;
        std::vector<uint64_t> sl;
        for (size_t o = o0; o < o1; ++o) {
            const HostObj& h = objs[o];
            if (!h.dig) continue;  // caller asked for no digests
            for (int j = 0; j < h.k + h.m; ++j) {
                sp.push_back(base + h.pool_off + uint64_t(j) * h.slot());
                sl.push_back(j < h.k ? std::min<uint64_t>(h.dlen[j], h.S) : h.S);
            }
        }
        hipEvent_t sha_done = nullptr;
        if (!sp.empty()) {
            MXEC_TRY(new_event(&sha_done));
            MXEC_HIP(hipStreamWaitEvent(sha_s, done.back(), 0));
            MXEC_TRY(run_sha(d_, slot, sha_s, sp, sl, digests, nullptr, nullptr, nullptr, &arena_));
            MXEC_HIP(hipEventRecord(sha_done, sha_s));
        }
        // Phase 3: parity back group by group as RS finishes, digests last.
        for (size_t g = downed; g < groups.size(); ++g) MXEC_TRY(down_group(g));
        if (sha_done) {
            MXEC_TRY(issue_down());
            MXEC_HIP(hipStreamWaitEvent(d2h_, sha_done, 0));
            uint64_t msg0 = 0;
            for (size_t o = o0; o < o1; ++o) {
                const HostObj& h = objs[o];
                if (!h.dig) continue;
                MXEC_TRY(queue_down(reinterpret_cast<uint8_t*>(h.dig), digests + msg0 * 32, uint64_t(h.k + h.m) * 32));
                msg0 += uint64_t(h.k + h.m);
            }
            MXEC_TRY(flush_down());
        }
        return flush();
    }

};

}  // namespace
}  // namespace mxec

using namespace mxec;

namespace mxec {
// The device's pipeline hub and its four streams, at context open (their
// hardware queues depend on what the process created before them).
int pipe_open(Device& dev) {
    std::lock_guard<std::mutex> g(dev.pipe_mu);
    if (!dev.pipe) dev.pipe = std::make_shared<PipeHub>();
    return static_cast<PipeHub*>(dev.pipe.get())->init(dev);
}
}  // namespace mxec

extern "C" int mxec_encode_batch_host(mxec_ctx* ctx, const mxec_object* objs, uint64_t n_obj,
                                      const uint8_t* const* data, const uint64_t* data_len,
                                      uint8_t* const* parity, uint8_t (*digests)[32],
                                      int32_t* status_out) {
    try {
        if (n_obj == 0) return MXEC_OK;
        if (!ctx || !objs || !data || !parity) return set_error(MXEC_E_INVALID_ARG, "null argument");
        const size_t D = ctx->c.devs.size();
        if (!D) return set_error(MXEC_E_NO_DEVICE, "context has no device");
        uint64_t dsum = 0;
        for (uint64_t o = 0; o < n_obj; ++o) dsum += uint64_t(std::max(objs[o].k, 0));
        std::vector<uint64_t> dlen(size_t(dsum), 0);
        std::vector<std::vector<HostObj>> per(D);
        // Device of each object: o mod D for a uniform batch, balanced by
        // bytes for a mixed one (deal.hpp).
        std::vector<uint64_t> obj_bytes(size_t(n_obj), 0);
        for (uint64_t o = 0; o < n_obj; ++o)
            obj_bytes[o] = uint64_t(std::max(objs[o].k, 0) + std::max(objs[o].m, 0)) * rup(objs[o].shard_size, kAlign);
        std::vector<const void*> first(size_t(n_obj), nullptr);
        for (uint64_t o = 0, j = 0; o < n_obj; j += uint64_t(std::max(objs[o].k, 0)), ++o)
            if (objs[o].k > 0) first[o] = data[j];
        const std::vector<uint32_t> owner = deal_batch(ctx->c, obj_bytes, first);
        uint64_t doff = 0, poff = 0, goff = 0;
        int first_err = MXEC_OK;
        std::string first_msg;
        for (uint64_t o = 0; o < n_obj; ++o) {
            const int k = objs[o].k, m = objs[o].m;
            const uint64_t S = objs[o].shard_size;
            int st = check_km(k, m);
            if (st == MXEC_OK && S == 0) st = set_error(MXEC_E_EMPTY_SHARD, mxec_strerror(MXEC_E_EMPTY_SHARD));
            for (int j = 0; st == MXEC_OK && j < k; ++j) {
                const uint64_t l = data_len ? data_len[doff + uint64_t(j)] : S;
                if (l > S) st = set_error(MXEC_E_INCORRECT_SHARD_SIZE, "data chunk longer than shard_size");
                dlen[size_t(doff) + size_t(j)] = l;
            }
            if (status_out) status_out[o] = st;
            if (st != MXEC_OK) {
                if (first_err == MXEC_OK) {
                    first_err = st;
                    first_msg = last_error();
                }
            } else {
                HostObj h{k, m, S, data + doff, &dlen[size_t(doff)], parity + poff, digests ? digests + goff : nullptr};
                per[owner[o]].push_back(h);
            }
            doff += uint64_t(std::max(k, 0));
            poff += uint64_t(std::max(m, 0));
            goff += uint64_t(std::max(k, 0) + std::max(m, 0));
        }
        std::vector<int> rcs(D, MXEC_OK);
        std::vector<std::string> errs(D);
        // One worker per device.  Every thread is joined on every path (a
        // joinable std::thread destroyed during unwinding would terminate the
        // process), and no exception leaves a worker.
        struct Joiner {
            std::vector<std::thread> th;
            ~Joiner() {
                for (auto& t : th)
                    if (t.joinable()) t.join();
            }
        } j;
        auto work = [&](size_t d) {
            try {
                Device& dev = *ctx->c.devs[d];
                rcs[d] = [&]() -> int {
                    MXEC_HIP(hipSetDevice(dev.id));
                    uint64_t bytes = 0;
                    for (const auto& h : per[d]) bytes += h.bytes();
                    LaneScope lane;
                    MXEC_TRY(lane.open(dev, bytes));
                    DevicePipeline p(dev, lane.hub(), lane.lane());
                    return p.run(per[d]);
                }();
                if (rcs[d] != MXEC_OK) errs[d] = last_error();
            } catch (const std::bad_alloc&) {
                rcs[d] = MXEC_E_OOM;
                errs[d] = "host allocation failed";
            } catch (const std::exception& e) {
                rcs[d] = MXEC_E_INVALID_ARG;
                errs[d] = e.what();
            }
        };
        for (size_t d = 0; d < D; ++d) {
            if (per[d].empty()) continue;
            try {
                j.th.emplace_back(work, d);
            } catch (const std::system_error&) {
                work(d);  // no thread to be had: run this device's share here
            }
        }
        for (auto& t : j.th) t.join();
        for (size_t d = 0; d < D; ++d)
            if (rcs[d] != MXEC_OK) return set_error(rcs[d], errs[d]);
        if (first_err != MXEC_OK) return set_error(first_err, first_msg);
        return MXEC_OK;
    } catch (const std::bad_alloc&) {
        return set_error(MXEC_E_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return set_error(MXEC_E_INVALID_ARG, e.what());
    }
}

extern "C" int mxec_reconstruct_batch_host(mxec_ctx* ctx, const mxec_object* objs, uint64_t n_obj,
                                           uint8_t* const* shards, const uint64_t* shard_len, uint8_t* present,
                                           const uint8_t (*expected_sha256)[32], uint32_t flags,
                                           int32_t* status_out) {
    try {
        if (n_obj == 0) return MXEC_OK;
        if (!ctx || !objs || !shards || !present) return set_error(MXEC_E_INVALID_ARG, "null argument");
        const size_t D = ctx->c.devs.size();
        if (!D) return set_error(MXEC_E_NO_DEVICE, "context has no device");
        uint64_t sum = 0;
        for (uint64_t o = 0; o < n_obj; ++o) {
            if (int rc = rs_check(objs[o].k, objs[o].m))
                return set_error(rc, std::string("RS init error: ") + mxec_strerror(rc));
            if (objs[o].shard_size == 0) return set_error(MXEC_E_EMPTY_SHARD, mxec_strerror(MXEC_E_EMPTY_SHARD));
            sum += uint64_t(objs[o].k + objs[o].m);
        }
        // Every shard pointer is needed: present ones are read, missing ones
        // are where the rebuilt bytes go.
        for (uint64_t g = 0; g < sum; ++g)
            if (!shards[g]) return set_error(MXEC_E_INVALID_ARG, "null shard pointer " + std::to_string(g));
        std::vector<uint64_t> len(size_t(sum), 0);
        std::vector<int32_t> st(size_t(n_obj), MXEC_OK);
        std::vector<uint64_t> obj_bytes(size_t(n_obj), 0);
        std::vector<RecObj> all;
        all.reserve(size_t(n_obj));
        uint64_t g0 = 0;
        for (uint64_t o = 0; o < n_obj; ++o) {
            const int k = objs[o].k, m = objs[o].m;
            const uint64_t S = objs[o].shard_size;
            for (int i = 0; i < k + m; ++i) len[g0 + uint64_t(i)] = shard_len ? std::min<uint64_t>(shard_len[g0 + i], S) : S;
            all.push_back(RecObj{k, m, S, shards + g0, &len[g0], present + g0,
                                 expected_sha256 ? expected_sha256 + g0 : nullptr, &st[o]});
            obj_bytes[o] = all.back().bytes();
            g0 += uint64_t(k + m);
        }
        std::vector<const void*> first(size_t(n_obj), nullptr);
        for (uint64_t o = 0; o < n_obj; ++o)
            for (int i = 0; i < all[o].k + all[o].m && !first[o]; ++i)
                if (all[o].present[i]) first[o] = all[o].shards[i];
        const std::vector<uint32_t> owner = deal_batch(ctx->c, obj_bytes, first);
        std::vector<std::vector<RecObj>> per(D);
        for (uint64_t o = 0; o < n_obj; ++o) per[owner[o]].push_back(all[o]);
        const bool data_only = (flags & MXEC_F_DATA_ONLY) != 0;
        std::vector<int> rcs(D, MXEC_OK);
        std::vector<std::string> errs(D);
        struct Joiner {
            std::vector<std::thread> th;
            ~Joiner() {
                for (auto& t : th)
                    if (t.joinable()) t.join();
            }
        } j;
        auto work = [&](size_t d) {
            try {
                Device& dev = *ctx->c.devs[d];
                rcs[d] = [&]() -> int {
                    MXEC_HIP(hipSetDevice(dev.id));
                    uint64_t bytes = 0;
                    for (const auto& h : per[d]) bytes += h.bytes();
                    LaneScope lane;
                    MXEC_TRY(lane.open(dev, bytes));
                    DevicePipeline p(dev, lane.hub(), lane.lane());
                    return p.run_rec(per[d], data_only);
                }();
                if (rcs[d] != MXEC_OK) errs[d] = last_error();
            } catch (const std::bad_alloc&) {
                rcs[d] = MXEC_E_OOM;
                errs[d] = "host allocation failed";
            } catch (const std::exception& e) {
                rcs[d] = MXEC_E_INVALID_ARG;
                errs[d] = e.what();
            }
        };
        for (size_t d = 0; d < D; ++d) {
            if (per[d].empty()) continue;
            try {
                j.th.emplace_back(work, d);
            } catch (const std::system_error&) {
                work(d);
            }
        }
        for (auto& t : j.th) t.join();
        for (size_t d = 0; d < D; ++d)
            if (rcs[d] != MXEC_OK) return set_error(rcs[d], errs[d]);
        int first_err = MXEC_OK;
        g0 = 0;
        for (uint64_t o = 0; o < n_obj; ++o) {
            const int total = objs[o].k + objs[o].m;
            if (status_out) status_out[o] = st[o];
            if (st[o] != MXEC_OK && first_err == MXEC_OK) {
                int np = 0;
                for (int i = 0; i < total; ++i) np += present[g0 + uint64_t(i)] != 0;
                first_err = st[o];
                set_error(first_err, too_few_msg(np, objs[o].k, total));
            }
            g0 += uint64_t(total);
        }
        return first_err;
    } catch (const std::bad_alloc&) {
        return set_error(MXEC_E_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return set_error(MXEC_E_INVALID_ARG, e.what());
    }
}
