// ops.hpp — device-pointer level operations shared by every C entry point.
#pragma once

#include <cstdint>
#include <exception>
#include <mutex>
#include <new>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "gf256.hpp"
#include "runtime.hpp"

namespace mxec {


// One object of an RS launch: k inputs -> r outputs, device pointers.
struct RsObject {
    const uint8_t* const* in;  // k
    const uint64_t* in_len;    // k
    uint8_t* const* out;       // r
    const uint64_t* out_len;   // r
    uint32_t coef_off;         // dword offset of this object's [j][i][8] table
};

// Applies each object's matrix; all objects share (k, r, shard_size).
// arena: take the descriptor tables from it instead of the slot's ring (many
// launches in flight, see pipeline.cpp).
// tune = false: the default grid, and the grid tuner neither picks nor
// records (the batch allocator's placement probes, placement.cpp).
int run_rs(Device& dev, Slot& slot, hipStream_t s, uint64_t shard_size, int k, int r,
           const std::vector<RsObject>& objs, DescArena* arena = nullptr, bool tune = true,
           uint32_t max_blocks = 0);

// Grid tuner of large uniform RS launches (runtime.hpp GridTuner):
// rs_grid_pick sets *bpc (0 = the default grid) and, while a shape is still
// being tuned, hands back a trial whose events the caller records around
// the launch and passes to rs_grid_record.  rs_grid_in_use: the workgroups
// per CU a shape runs at now (0 while undecided).  MXEC_RS_TUNE=0 disables,
// MXEC_RS_BPC fixes the grid.
int rs_grid_pick(Device& dev, int k, int r, uint64_t shard_size, double gb, uint32_t* bpc,
                 GridTuner::Trial* trial);
void rs_grid_record(Device& dev, int k, int r, uint64_t shard_size, const GridTuner::Trial& trial);
int rs_grid_in_use(Device& dev, int k, int r, uint64_t shard_size);
void rs_grid_release(Device& dev);

// An object of a mixed batch: its own k and shard size.
struct RsMixedObject {
    int k;
    uint64_t shard_size;
    RsObject o;
};
// Applies each object's matrix, objects grouped by r (map key).  Per r, the
// objects whose pointers are all 16-byte aligned (r <= 8) share one grouped
// launch (rs_apply_fast<GRP>), every grouped launch's tables in one upload;
// when two or more such groups all have r <= 4 they run as ONE multi-r
// launch instead (rs_apply_multi; MXEC_RS_MULTI=0 disables).  The others run
// one run_rs per (k, shard_size).  A lone uniform group runs the uniform
// kernel.
// max_blocks (here and in run_rs): a cap on each launch's workgroups, the
// grid tuner left alone (0: the default grid, or mxec_open_test's cap).
int run_rs_mixed(Device& dev, Slot& slot, hipStream_t s, const std::map<int, std::vector<RsMixedObject>>& groups,
                 DescArena* arena = nullptr, uint32_t max_blocks = 0);

// SHA-256 of n device buffers.  digests_dev / expected_dev / ok_dev may be
// null (see ShaArgs).
// tmo_dev: a caller that reads back a 4-byte device word after the launch
// (and fails the call if it is not 0) passes this; only then may a batch of
// more 64-message groups than SIMDs take the stream form (sha256_kernel.hip),
// whose word it is.  Set to null when another form ran.
int run_sha(Device& dev, Slot& slot, hipStream_t s, const std::vector<const uint8_t*>& ptrs,
            const std::vector<uint64_t>& lens, uint8_t* digests_dev, const uint8_t* expected_dev,
            uint8_t* ok_dev, const std::vector<uint64_t>* exp_idx = nullptr,
            DescArena* arena = nullptr, int form = 0, const uint32_t** tmo_dev = nullptr);
// One piece of every listed chain (ShaPiece, kernels.hpp), lag quad form
// with two messages per quad:
// message i is the next lens[i] bytes of the chain in state slot slots[i]
// (state_dev: [slots][8] words, carried between launches on one stream);
// totals[i] = the message's length if this piece ends it (digest into
// digests_dev[slots[i]]; with expected_dev, ok_dev[slots[i]] = digest ==
// expected_dev[slots[i]]), kShaNotFinal otherwise (lens[i] a multiple of 64).
// At most kShaLagMsgs messages per CU.
int run_sha_pieces(Device& dev, Slot& slot, hipStream_t s, const std::vector<const uint8_t*>& ptrs,
                   const std::vector<uint64_t>& lens, const std::vector<uint32_t>& slots,
                   const std::vector<uint64_t>& totals, uint32_t* state_dev, bool resume, uint8_t* digests_dev,
                   DescArena* arena, const uint8_t* expected_dev = nullptr, uint8_t* ok_dev = nullptr);

// SHA-256 digests (host out, n * 32 bytes) of n device-resident messages on
// `dev`, blocking; the caller's work on `s` must have produced them (the
// caller synchronises `s` first).  Concurrent small requests on one device
// share one launch on the combiner's stream (combiner.cpp); large ones run on
// the caller's slot and stream.
// The stream form pays once a batch has more 64-message groups than 3/4 of
// the SIMDs (sha256_kernel.hip kSplitMaxMessages).
inline bool sha_stream_size(uint64_t groups, uint64_t simds) { return groups * 4 > simds * 3; }

// `ready` (optional): an event the caller recorded on `s` when its messages
// were complete; without one the call records it now.  `after_launch`
// (optional) runs once the hash launch is queued, before the wait for its
// digests -- work to queue on `s` beside the hash; its status is the call's
// if the hash itself succeeded.
int sha256_combined(Device& dev, Slot& slot, hipStream_t s, const std::vector<const uint8_t*>& ptrs,
                    const std::vector<uint64_t>& lens, uint8_t* out, hipEvent_t ready = nullptr,
                    const std::function<int()>* after_launch = nullptr);
void combiner_stats(Device& dev, uint64_t* batches, uint64_t* messages);
// Whether a request of n messages goes through the combiner.
bool sha_combines(const Device& d, size_t n);

// Coefficient table of the (k, m) encoding matrix's parity rows.
int encode_coef(Device& dev, int k, int m, uint32_t* off);
// Coefficient table of a decode plan.
int decode_coef(Device& dev, const DecodePlan& plan, bool data_only, uint32_t* off);

// Decode plan + table offset for one erasure pattern (present: k+m flags),
// memoised per device so a batch that repeats patterns pays one hash lookup
// per object.  *plan is null when fewer than k shards are present.
int decode_plan(Device& dev, int k, int m, const uint8_t* present, bool data_only,
                std::shared_ptr<const DecodePlan>* plan, uint32_t* off);

// Host-API staging: shard slots are this many bytes apart on the device.
constexpr uint64_t kSlotAlign = 256;
inline uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

// Runs an entry point body; no C++ exception crosses the C ABI.
template <class F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return set_error(MXEC_E_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return set_error(MXEC_E_INVALID_ARG, e.what());
    } catch (...) {
        return set_error(MXEC_E_INVALID_ARG, "unknown exception");
    }
}

// A device of the context (dev_index < 0: round robin) with one of its slots
// locked for the duration of a call.
// On the way out (any path, the lock still held) it waits for DMAs still
// reading the caller's page-locked buffers (Slot::borrowed).
struct DevScope {
    Device* d = nullptr;
    std::unique_lock<std::mutex> lk;
    Slot* slot = nullptr;
    DevScope() = default;
    DevScope(const DevScope&) = delete;
    DevScope& operator=(const DevScope&) = delete;
    ~DevScope() {
        if (slot && slot->borrowed) {
            const std::string keep = last_error();  // an early return's message stays
            (void)slot_wait(*slot, slot->borrowed);
            if (slot->borrowed) {  // the wait itself failed: drain the device
                (void)hipStreamSynchronize(slot->borrowed);
                slot->borrowed = nullptr;
            }
            set_error(0, keep);
        }
    }
    int open(mxec_ctx* ctx, int dev_index) {
        if (!ctx) return set_error(MXEC_E_INVALID_ARG, "null context");
        d = pick_device(&ctx->c, dev_index);
        if (!d) return set_error(MXEC_E_INVALID_ARG, "no such device in context");
        MXEC_HIP(hipSetDevice(d->id));
        slot = &lock_slot(*d, lk);
        return MXEC_OK;
    }
};


// PUT body digests of device-resident bodies into mxec_body_sums records
// (sums.cpp); enqueued on s.
int run_body_sums(Device& d, Slot& slot, hipStream_t s, const std::vector<const uint8_t*>& ptrs,
                  const std::vector<uint64_t>& lens, uint32_t which, uint8_t* out_dev, uint64_t stride);

// Creates the device's host-pipeline hub and its streams (pipeline.cpp),
// called by mxec_open for every device.
int pipe_open(Device& dev);

// filesystem.rs:1095 guard, then the crate's ReedSolomon::new checks.
int check_km(int k, int m);

// chunk_reader.rs:203-206's error text for an object short of k shards.
inline std::string too_few_msg(int present, int k, int total) {
    return "too many missing/corrupt shards: only " + std::to_string(present) + " of " +
           std::to_string(k) + " required shards available (" + std::to_string(total - present) +
           " missing)";
}

// Coefficient-table offsets are valid while their generation's half of the
// device's table arena is not reused (runtime.hpp Device::coef_*): `collect`
// takes a batch's offsets (noting each table's generation and upload),
// `s` waits on the GPU for any of those tables still being uploaded,
// `launch` enqueues the kernels that read them on `s`; then, under the arena's lock,
// either every generation used is still live and an event on `s` fences the
// batch (a later recycle of those halves waits for it), or one was recycled
// between `collect` and here, and the pair runs again.  A launch queued with
// a recycled half's offsets may have read foreign tables; its re-run is
// queued behind it on the same stream over the same outputs (the RS kernels
// read only inputs and write only outputs), so the last pass wins and the
// result is exact.
template <class C, class L>
int with_stable_coef(Device& d, hipStream_t s, C&& collect, L&& launch) {
    for (int attempt = 0; attempt < 8; ++attempt) {
        CoefUse use;
        CoefUse* outer = coef_use_swap(&use);
        int rc = collect();
        if (rc == MXEC_OK) rc = coef_wait_uploads(d, use, s);  // tables still on their way up
        if (rc == MXEC_OK) rc = launch();
        coef_use_swap(outer);
        MXEC_TRY(rc);
        bool live = true;
        MXEC_TRY(coef_fence(d, use, s, &live));
        if (live) return MXEC_OK;
    }
    return set_error(MXEC_E_INVALID_ARG,
                     "the coefficient tables of one batch exceed the device's table arena (recycled under it 8 times)");
}

}  // namespace mxec
