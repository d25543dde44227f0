// combiner.cpp — cross-request coalescing of SHA-256 verification.
//
// SHA-256 of one message is a serial chain (1.17 us per 64-byte block in the
// lag pair form, ~1.8 in the split form: kernels.hpp kShaLagUsPerBlock /
// kShaSplitUsPerBlock, sha256_kernel.hip), so a launch over 8 chunks of one GET takes as
// long as a launch over thousands: per-request launches leave the GPU nearly
// idle and, past GPU_MAX_HW_QUEUES streams, even queue behind each other.
// Concurrent callers on one device (MaxIO's tokio workers serving GETs, chunk
// verification in chunk_reader.rs:87-152 / :176-196) therefore hand their
// device-resident messages to one combiner: a caller that finds a launch
// lane free and nobody gathering becomes the leader, takes every pending
// request, and runs ONE launch over all their messages on that lane's private
// stream; callers that arrive meanwhile form the next batch, which starts on
// the next free lane without waiting for the first to finish (flat
// combining, no service thread).  A batch of N requests costs about one
// request's latency.
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <functional>

#include "kernels.hpp"
#include "ops.hpp"

namespace mxec {


struct ShaCombiner {
    struct Req {
        const std::vector<const uint8_t*>* ptrs = nullptr;
        const std::vector<uint64_t>* lens = nullptr;
        uint8_t* out = nullptr;  // host, n * 32
        hipEvent_t ready = nullptr;  // on the caller's stream: its messages are complete
        // Run by the leader right after the hash launch is queued, before it
        // waits for the digests (the caller is blocked meanwhile, so its slot
        // and stream are free to use): work that should run beside the hash.
        const std::function<int()>* after_launch = nullptr;
        uint64_t longest = 0;  // bytes of the longest message (set before queueing)
        int after_rc = MXEC_OK;
        std::string after_msg;
        int rc = MXEC_OK;
        std::string msg;
        bool done = false;
    };
    std::mutex mu;
    // Two wait queues, so that an arrival wakes only the gathering leader and
    // a finished launch wakes the waiters once (one shared queue woke every
    // waiting thread on every arrival: ~60 futex wake-ups per request at 64
    // request threads).
    std::condition_variable cv_gather;  // the gathering leader
    std::condition_variable cv_done;    // everyone else
    std::vector<Req*> pending;
    bool gathering = false;  // a leader is collecting its batch
    size_t last_batch = 1;   // requests in the previous launch
    // A caller that only ever arrives alone (one thread verifying one GET
    // after another) stops paying the lone leader's gather window: after
    // kLoneStreak launches in a row that carried one request each, with no
    // arrival while another request was pending or in flight, a leader
    // launches at once.  The first overlapping arrival ends the streak.
    static constexpr int kLoneStreak = 8;
    int lone_launches = 0;
    bool overlap = false;    // an arrival found company since the last launch
    size_t pending_msgs = 0;   // messages of `pending`
    size_t inflight_msgs = 0;  // messages of the launches running now
    size_t lane_limit = 0;     // a second lane opens only below this (see below)
    // Launch lanes: up to slots.size() batches in flight at once (default
    // two), each on its own stream and buffers, so that a request arriving
    // while a small launch runs starts its own instead of queueing behind it
    // (lane_limit keeps chip-filling batches one at a time).
    std::vector<std::unique_ptr<Slot>> slots;
    std::vector<Slot*> free_slots;
    uint64_t batches = 0, messages = 0;  // guarded by mu

    ~ShaCombiner() {
        for (auto& sl : slots) {
            if (sl->stream) (void)hipStreamSynchronize(sl->stream);
            slot_destroy(*sl);
        }
    }

    // One launch over every message of `batch` on `slot`; digests land in
    // each request's host buffer.  Called by a leader without the lock held.
    static int run(Device& d, Slot& slot, const std::vector<Req*>& batch) {
        std::vector<const uint8_t*> ptrs;
        std::vector<uint64_t> lens;
        for (const Req* r : batch) {
            ptrs.insert(ptrs.end(), r->ptrs->begin(), r->ptrs->end());
            lens.insert(lens.end(), r->lens->begin(), r->lens->end());
        }
        const size_t n = ptrs.size();
        if (n == 0) return MXEC_OK;
        hipStream_t s = slot.stream;
        // Each caller's shards are complete once its stream reaches its
        // event; the launch waits on the device, not on the host, so
        // callers whose preceding work finishes at different times still
        // arrive together (config 3c: the decodes of the previous step).
        for (const Req* r : batch)
            if (r->ready) MXEC_HIP(hipStreamWaitEvent(s, r->ready, 0));
        MXEC_TRY(slot.digests.grow(n * 32));
        // The kernel's own choice by message count: the lag quad form up
        // to 64 messages per CU, the split form up to 3/4 of a 64-message
        // group per SIMD, beyond that the stream form (segments of every
        // chain dealt to persistent waves keep every SIMD busy to the end:
        // 81 920 x 1 MiB 55.8 ms vs 96.1 split), whose timeout word comes
        // back with the digests.  (Until late round 3 this call pinned the
        // split form below the stream size, so combined verifications -- a
        // lone GET's included -- never got the quad forms: configs[0]'s
        // 10 MiB GET took 280 ms against a 203 ms chain.)
        const uint32_t* tmo = nullptr;
        MXEC_TRY(run_sha(d, slot, s, ptrs, lens, static_cast<uint8_t*>(slot.digests.p), nullptr, nullptr, nullptr,
                         nullptr, 0, &tmo));
        // The callers' work to run beside the hash is queued before this
        // launch's digest copy: copies of different streams can share a copy
        // engine queue in submission order, and work queued behind the
        // digest copy (which waits for the hash) would wait for the hash too
        // -- the speculative decodes' descriptor uploads did, measured.
        const auto ta = std::chrono::steady_clock::now();
        for (Req* r : batch) {
            if (!r->after_launch) continue;
            try {
                r->after_rc = (*r->after_launch)();
            } catch (...) {
                r->after_rc = set_error(MXEC_E_OOM, "host allocation failed");
            }
            if (r->after_rc) r->after_msg = last_error();
        }
        if (d.kn && d.kn->combine_log)
            std::fprintf(stderr, "[mxec combine] after-launch work %lld us\n",
                         (long long)std::chrono::duration_cast<std::chrono::microseconds>(
                             std::chrono::steady_clock::now() - ta).count());
        MXEC_TRY(slot.hdig.grow(n * 32 + 16));
        auto* hflag = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(slot.hdig.p) + n * 32);
        *hflag = 0;
        MXEC_HIP(hipMemcpyAsync(slot.hdig.p, slot.digests.p, n * 32, hipMemcpyDeviceToHost, s));
        if (tmo) MXEC_HIP(hipMemcpyAsync(hflag, tmo, 4, hipMemcpyDeviceToHost, s));
        MXEC_TRY(slot_wait(slot, s));
        if (*hflag != 0)
            return set_error(MXEC_E_DEVICE, "SHA-256 stream kernel: a wave timed out waiting for its predecessor segment");
        const auto* h = static_cast<const uint8_t*>(slot.hdig.p);
        size_t o = 0;
        for (Req* r : batch) {
            const size_t k = r->ptrs->size();
            std::memcpy(r->out, h + o * 32, k * 32);
            o += k;
        }
        return MXEC_OK;
    }
};

// Every request is combined by default, chip-filling ones too: eight
// concurrent 10 240-message batches (config 3c) ran 1.34x faster as one
// split-form launch than as eight launches on eight streams
// (profiles/r1_bench_cfg3c_w8_combine_below_*.json).  MXEC_COMBINE_BELOW=n
// (Knobs::combine_below) sends requests of n or more messages to their own
// launch on the caller's stream instead.
bool sha_combines(const Device& d, size_t n) {
    const size_t below = d.kn ? d.kn->combine_below : 0;
    return below == 0 || n < below;
}

namespace {

// The combiner's windows (knobs.hpp): MXEC_GATHER_US, how long a lone leader
// waits for company (default 100 us); MXEC_GATHER_MAX_US, the bound when
// waiting for the previous batch size (default 2 ms); MXEC_GATHER_IDLE_US,
// once a batch is forming, how long a gap between arrivals still counts as
// "more are coming" (default 300 us).  MXEC_COMBINE_LOG=1: one stderr line
// per combined launch (requests, messages, gathering and launch times).
const Knobs& knobs_of(const Device& d) {
    static const Knobs dflt;
    return d.kn ? *d.kn : dflt;
}

// MXEC_COMBINE_STREAMS: launches in flight per device (default 2).  A second
// launch starts beside a running one only while both together stay under
// one quad-form workgroup per CU of messages (lane_limit): light request traffic then
// no longer waits out the batch in flight (16-thread GET 2.5 -> 3.5 GiB/s,
// profiles/r1_combine_lanes2.txt), while chip-filling batches still go one
// at a time -- unconditional lanes split them and issue-bound launches side
// by side share the SIMDs (config 3c 509 -> 344 GiB/s with two lanes,
// profiles/r1_combine_lanes.txt).
//
// MXEC_COMBINE_PRIORITY (default 1): the combiner's streams get the highest
// stream priority, i.e. a hardware queue of their own.  Streams share
// GPU_MAX_HW_QUEUES = 4 queues, so a 30 ms hash launch on a normal-priority
// stream held up the uploads of a quarter of the request streams behind it
// (64-thread GET: host upload + wait 6.4 -> 2.7 ms per request, 7.3 -> 8.0 GiB/s).

ShaCombiner* combiner_of(Device& d) {
    std::lock_guard<std::mutex> g(d.comb_mu);
    if (!d.comb) {
        auto c = std::make_shared<ShaCombiner>();
        for (int i = 0; i < knobs_of(d).combine_streams; ++i) {
            auto sl = std::make_unique<Slot>();
            sl->owner = &d;
            int least = 0, greatest = 0;
            const bool prio = knobs_of(d).combine_priority &&
                              hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess &&
                              hipStreamCreateWithPriority(&sl->stream, hipStreamNonBlocking, greatest) == hipSuccess;
            if (!prio && hipStreamCreateWithFlags(&sl->stream, hipStreamNonBlocking) != hipSuccess) return nullptr;
            affinity_tag(sl->stream, &d);
            c->free_slots.push_back(sl.get());
            c->slots.push_back(std::move(sl));
        }
        // Both lanes' launches together within one lag-form workgroup
        // (64 messages, one wave per SIMD) per CU.
        c->lane_limit = size_t(d.n_cus) * kShaLagMsgs;
        d.comb = c;
    }
    return static_cast<ShaCombiner*>(d.comb.get());
}

}  // namespace

int sha256_combined(Device& d, Slot& slot, hipStream_t s, const std::vector<const uint8_t*>& ptrs,
                    const std::vector<uint64_t>& lens, uint8_t* out, hipEvent_t ready,
                    const std::function<int()>* after_launch) {
    if (ptrs.empty()) return MXEC_OK;
    if (!sha_combines(d, ptrs.size())) {
        // Opted out by MXEC_COMBINE_BELOW: its own launch on the caller's
        // stream (the kernel picks its form by message count).
        const size_t n = ptrs.size();
        MXEC_TRY(slot.digests.grow(n * 32));
        MXEC_TRY(run_sha(d, slot, s, ptrs, lens, static_cast<uint8_t*>(slot.digests.p), nullptr, nullptr));
        MXEC_TRY(slot.hdig.grow(n * 32));
        MXEC_HIP(hipMemcpyAsync(slot.hdig.p, slot.digests.p, n * 32, hipMemcpyDeviceToHost, s));
        if (after_launch) MXEC_TRY((*after_launch)());  // same stream: after the hash, not beside it
        MXEC_TRY(slot_wait(slot, s));
        std::memcpy(out, slot.hdig.p, n * 32);
        return MXEC_OK;
    }
    ShaCombiner* c = combiner_of(d);
    if (!c) return set_error(MXEC_E_DEVICE, "combiner stream creation failed");
    ShaCombiner::Req me;
    me.ptrs = &ptrs;
    me.lens = &lens;
    me.out = out;
    if (!ready) {
        if (!slot.ready_ev) MXEC_HIP(hipEventCreateWithFlags(&slot.ready_ev, hipEventDisableTiming));
        MXEC_HIP(hipEventRecord(slot.ready_ev, s));
        ready = slot.ready_ev;
    }
    me.ready = ready;
    me.after_launch = after_launch;
    for (uint64_t l : lens) me.longest = std::max(me.longest, l);  // outside the lock
    std::unique_lock<std::mutex> lk(c->mu);
    if (!c->pending.empty() || c->inflight_msgs > 0 || c->gathering) c->overlap = true;
    c->pending.push_back(&me);
    c->pending_msgs += ptrs.size();
    if (c->gathering) c->cv_gather.notify_one();  // the gathering leader may be waiting for us
    while (!me.done) {
        // Lead when a launch lane is free and nobody else is gathering (a
        // gathering leader takes this request too); else wait.
        if (c->gathering || c->free_slots.empty() ||
            (c->inflight_msgs > 0 && c->inflight_msgs + c->pending_msgs > c->lane_limit)) {
            c->cv_done.wait(lk);
            continue;
        }
        c->gathering = true;
        // Adaptive gathering: a leader waits (bounded) until as many requests
        // are pending as the previous launch carried, so a steady stream of
        // concurrent callers keeps landing in few launches instead of a lone
        // first request and the rest; a lone leader waits a short window.  A
        // launch lasts >= kShaLagUsPerBlock (1.17 us) per 64-byte block of its
        // longest message (~21 ms per 1 MiB chunk), so the wait costs a few percent at most, and
        // the previous size is forgotten as soon as fewer come.
        const size_t want = c->last_batch;
        const Knobs& kn = knobs_of(d);
        const long wait_us = want > 1 ? kn.gather_max_us
                             : c->lone_launches >= ShaCombiner::kLoneStreak ? 0 : kn.gather_us;
        const auto t0 = std::chrono::steady_clock::now();
        if (c->pending.size() < std::max<size_t>(want, 2) && wait_us > 0)
            c->cv_gather.wait_for(lk, std::chrono::microseconds(wait_us),
                           [&] { return c->pending.size() >= std::max<size_t>(want, 2); });
        // Then, while requests keep arriving (each within gather_idle_us of
        // the last), keep gathering up to gather_max_us in all: the previous
        // batch size is a floor, not a cap.  Without this, eight concurrent
        // 10 240-chunk verifications (config 3c) settled into two launches of
        // four (split form, 640 groups each) instead of one of 81 920
        // messages, which takes the stream form.  Only when the launch will
        // be long next to the idle window: a chain takes kShaLagUsPerBlock or
        // kShaSplitUsPerBlock per 64-byte block of the longest pending message
        // (launch_us below), and the extension is taken
        // only while one idle window costs at most 2 % of that, so small
        // latency-bound verifications (64 KiB chunks: a ~1.3 ms launch) do
        // not pay it, while 1 MiB chunks (~21-28 ms) still gather.
        // (Stopping at the stream form's size instead split config 3c's
        // eight batches into launches of five and three: 585 vs 970 GiB/s.)
        // For such long launches the idle window grows to 2 % of the launch
        // (590 us for 1 MiB chunks) and the whole gather may run to 15 % of
        // it (4.4 ms) while arrivals keep coming: a 2 ms cap (and then 8 %)
        // sometimes split a config-3c step's eight arrivals into two
        // launches, doubling that step (831 / 942 vs 1 040 GiB/s).  A lone request never waits for this
        // part: it only continues while requests keep arriving.
        auto launch_us = [&] {
            uint64_t longest = 0;
            for (const ShaCombiner::Req* r : c->pending) longest = std::max(longest, r->longest);
            // The form the kernel will pick for this many messages sets the
            // chain's pace (kernels.hpp kShaLagUsPerBlock / kShaSplitUsPerBlock).
            const bool lag = c->pending_msgs <= size_t(kShaLagMsgs) * size_t(d.n_cus);
            return double(longest / 64) * (lag ? kShaLagUsPerBlock : kShaSplitUsPerBlock);
        };
        const double est_us = c->pending.size() >= 2 ? launch_us() : 0.0;
        if (c->pending.size() >= 2 && est_us * 0.02 >= double(kn.gather_idle_us)) {
            const auto hard = t0 + std::chrono::microseconds(std::max<long>(kn.gather_max_us, long(est_us * 0.15)));
            const long idle = std::max<long>(kn.gather_idle_us, long(est_us * 0.02));
            for (size_t seen = c->pending.size(); std::chrono::steady_clock::now() < hard;) {
                c->cv_gather.wait_for(lk, std::chrono::microseconds(idle),
                                      [&] { return c->pending.size() > seen; });
                if (c->pending.size() == seen) break;
                seen = c->pending.size();
            }
        }
        std::vector<ShaCombiner::Req*> batch;
        batch.swap(c->pending);
        size_t batch_msgs = c->pending_msgs;
        c->pending_msgs = 0;
        c->inflight_msgs += batch_msgs;
        c->last_batch = batch.size();
        c->lone_launches = batch.size() == 1 && !c->overlap ? c->lone_launches + 1 : 0;
        c->overlap = false;
        c->gathering = false;
        Slot* slot_run = c->free_slots.back();
        c->free_slots.pop_back();
        // Requests that arrived while this leader gathered are in its batch,
        // so nobody waits for the gathering to end unless another lane is
        // free for them.
        if (!c->free_slots.empty() && c->inflight_msgs + c->pending_msgs <= c->lane_limit) c->cv_done.notify_all();
        lk.unlock();
        int rc = MXEC_OK;
        const auto t1 = std::chrono::steady_clock::now();
        try {
            rc = ShaCombiner::run(d, *slot_run, batch);
        } catch (...) {
            rc = set_error(MXEC_E_OOM, "host allocation failed");
        }
        if (kn.combine_log) {
            const auto t2 = std::chrono::steady_clock::now();
            using us = std::chrono::microseconds;
            std::fprintf(stderr, "[mxec combine] requests %zu messages %zu gather_us %lld run_us %lld rc %d\n",
                         batch.size(), batch_msgs, (long long)std::chrono::duration_cast<us>(t1 - t0).count(),
                         (long long)std::chrono::duration_cast<us>(t2 - t1).count(), rc);
        }
        const std::string msg = rc ? std::string(last_error()) : std::string();
        lk.lock();
        if (rc == MXEC_OK) {
            ++c->batches;
            for (const auto* r : batch) c->messages += r->ptrs->size();
        }
        for (auto* r : batch) {
            r->rc = rc;
            r->msg = msg;
            r->done = true;
        }
        c->free_slots.push_back(slot_run);
        c->inflight_msgs -= batch_msgs;
        c->cv_done.notify_all();
    }
    if (me.rc) return set_error(me.rc, me.msg);
    if (me.after_rc) return set_error(me.after_rc, me.after_msg);
    return MXEC_OK;
}

void combiner_stats(Device& d, uint64_t* batches, uint64_t* messages) {
    std::shared_ptr<void> keep;
    {
        std::lock_guard<std::mutex> g(d.comb_mu);
        keep = d.comb;
    }
    auto* c = static_cast<ShaCombiner*>(keep.get());
    *batches = *messages = 0;
    if (!c) return;
    std::lock_guard<std::mutex> g(c->mu);
    *batches = c->batches;
    *messages = c->messages;
}

}  // namespace mxec
