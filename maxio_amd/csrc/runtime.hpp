// runtime.hpp — per-device state of the C ABI: streams, staging buffers,
// descriptor rings and the coefficient-table arena.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/maxio_ec.h"
#include "knobs.hpp"

namespace mxec {

int set_error(int code, const std::string& msg);
const char* last_error();

#define MXEC_HIP(expr)                                                                  \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess)                                                           \
            return ::mxec::set_error(_e == hipErrorOutOfMemory ? MXEC_E_OOM : MXEC_E_DEVICE, \
                                     std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

#define MXEC_TRY(expr)              \
    do {                            \
        int _rc = (expr);           \
        if (_rc != MXEC_OK) return _rc; \
    } while (0)

// ensure(n): at least n bytes (a re-size frees the old buffer, and hipFree
// waits for the whole device).  grow(n): for buffers re-sized call after
// call while earlier launches may still read them (descriptor rings,
// per-launch scratch, digest landing zones): at least 1 MiB and at least
// twice the old capacity, and the old buffer is retired, not freed, until
// release() -- a free there stalled the host until the device drained,
// leaving the GPU idle ~0.5-1 ms before the next launch.  Geometric growth
// keeps the retired bytes below the live ones.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    std::vector<void*> retired;
    int ensure(size_t n);
    int grow(size_t n);
    // At least n bytes, exactly n when it re-sizes; the old buffer is retired
    // (no free, so no device-wide wait while other work runs) until
    // free_retired() or release().
    int replace(size_t n);
    void free_retired();
    void release();
    ~DevBuf() { release(); }
    static constexpr size_t kGrowFloor = size_t(1) << 20;
};

// Page-locked host memory (hipHostMalloc) on NUMA node `node` (-1: where
// the calling thread's policy puts it): the thread prefers that node around
// the call (hipHostMallocNumaUser) and gets its policy back after; if the
// node does not exist or the policy calls are refused, the plain allocation.
hipError_t host_malloc_on_node(void** p, size_t n, int node, unsigned flags);

struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    int node = -1;  // NUMA node its pages go on (host_malloc_on_node; -1: anywhere)
    std::vector<void*> retired;
    int ensure(size_t n);
    int grow(size_t n);
    void release();
    ~PinnedBuf() { release(); }
};

// One descriptor staging pair (pinned host + device) guarded by an event
// recorded after the last launch that reads it.
struct DescBuf {
    PinnedBuf host;
    DevBuf dev;
    DevBuf scratch;  // per-launch device scratch (DescWriter::scratch), same lifetime
    hipEvent_t done = nullptr;
    hipEvent_t uploaded = nullptr;  // the tables' copy on Slot::upload finished
    bool pending = false;
};

struct Device;

struct Slot {
    std::mutex mu;
    const Device* owner = nullptr;  // the (logical) device whose queues these are
    hipStream_t stream = nullptr;
    DevBuf shards;    // host-API staging: shard images on the device
    DevBuf digests;   // host-API digests / ok flags
    PinnedBuf hdig;   // pinned landing zone for digests / flags
    static constexpr int kRing = 4;
    DescBuf ring[kRing];
    int ring_next = 0;
    // Descriptor tables of 256 KiB and more are copied on this stream of
    // their own and the launch stream waits for the copy's event: the copy
    // then runs while earlier kernels still execute, where an in-stream copy
    // left the GPU idle for ~60-70 us between two kernels (19-21 us with the
    // event wait; MXEC_DESC_UPLOAD=inline / stream force one way).
    hipStream_t upload = nullptr;
    // Host-API uploads go through this pinned pair (pieces of kStagePiece,
    // double-buffered): one DMA per piece instead of HIP's pageable staging.
    PinnedBuf stage[2];
    hipEvent_t stage_done[2] = {nullptr, nullptr};
    // Blocking-sync event for the host-API waits (slot_wait).
    hipEvent_t sync_ev = nullptr;
    // Recorded on the caller's stream when it hands messages to the SHA-256
    // combiner: the combined launch waits for it on the device, so a caller
    // need not wait on the host for the work that produces its shards.
    hipEvent_t ready_ev = nullptr;
    // Set by upload_segments when it queued DMAs straight from the caller's
    // page-locked memory (no staging copy): the call must not return before
    // they finish, on any path.  slot_wait clears it; DevScope waits on it.
    hipStream_t borrowed = nullptr;
};

// Wait for everything enqueued on `s` so far.  An event created with
// hipEventBlockingSync sleeps in the driver instead of spinning a core: with
// dozens of request threads waiting on ~30 ms hash launches, spin-waiting
// took more host cores than the data copies (MXEC_SPIN_WAIT=1 restores
// hipStreamSynchronize).
int slot_wait(Slot& slot, hipStream_t s);
// Destroy a slot's events and stream (context close).
void slot_destroy(Slot& slot);

// One host -> device upload segment: len bytes from src to dst_off.
struct UploadSeg {
    uint64_t dst_off;
    const void* src;
    uint64_t len;
};
constexpr uint64_t kStagePiece = uint64_t(8) << 20;
// Copy host segments to dev_base + dst_off, enqueued on `s`: pageable ones
// through the slot's pinned pair, page-locked ones by direct DMA from the
// caller's memory.  In the direct case the slot is marked `borrowed` and the
// call must wait on `s` before it returns to its caller (slot_wait, or the
// DevScope destructor on an early error return).  Segments must be sorted by
// dst_off and not overlap.
// waves: segments wholly inside mxec_host_alloc memory may move by a CU-wave
// copy kernel (copy_kernel.hip) instead of SDMA (the host reconstruct and
// hash paths, MXEC_PIPE_COPY auto / waves; pipeline.cpp has the measurements).
int upload_segments(Slot& slot, hipStream_t s, uint8_t* dev_base, const std::vector<UploadSeg>& segs,
                    bool waves = false);
// One device -> host download segment: len bytes from src_off to dst.
struct DownloadSeg {
    uint64_t src_off;
    void* dst;
    uint64_t len;
};
// The reverse of upload_segments, through the same pinned pair; returns when
// every byte has landed (waits for everything enqueued on `s` before it,
// too).  Segments sorted by src_off, not overlapping.
int download_segments(Slot& slot, hipStream_t s, const uint8_t* dev_base, const std::vector<DownloadSeg>& segs,
                      bool waves = false);

// Page-locked host ranges.  mxec_host_alloc registers its allocations so the
// copy paths recognise them without a hipPointerGetAttributes call per
// segment; other page-locked memory (hipHostRegister) is asked of HIP, at both
// ends of the range.
void pinned_register(const void* p, size_t n);
void pinned_unregister(const void* p);
// True when every byte of [p, p + len) is page-locked host memory.
bool pinned_range(const void* p, uint64_t len);
// True when [p, p + len) lies in one mxec_host_alloc allocation: page-locked
// and mapped into every GPU's address space at its host address, so kernels
// may load and store it directly (copy_kernel.hip).
bool pinned_mapped(const void* p, uint64_t len);

// Online choice among three grid sizes (the default, half and a quarter of
// it) for the large uniform RS launches of one shape (ops.cpp
// rs_grid_pick): which runs fastest depends on the box and on where the
// batch sits in HBM (profiles/r3/grid_ab/: 512 workgroups per CU 3.6 % ahead
// of 1024 on one box, 0.8 % behind on another; profiles/r4/placement_full/:
// on configs[1] batches that 1024 runs at 6.06-6.07 TB/s, 256 runs at 6.24,
// and where 1024 is fast 256 trails it by ~1 %), so the first launches of a
// shape cycle through the three, timed with events on the caller's stream,
// and the fastest is kept for the context's life.
struct GridTuner {
    static constexpr int kCands = 3;
    struct Trial {
        hipEvent_t a = nullptr, b = nullptr;
        int cand = 0;
        double gb = 0;  // bytes of the launch, in GB
    };
    struct State {
        int cands[kCands] = {0, 0, 0};
        int launches = 0;
        int samples[kCands] = {0, 0, 0};
        double best_ms_per_gb[kCands] = {1e30, 1e30, 1e30};
        int decided = -1;
        std::vector<Trial> pending;
    };
    std::mutex mu;
    std::map<std::tuple<int, int, uint64_t>, State> states;  // (k, r, shard_size)
};

struct Device {
    int id = 0;
    int n_cus = 256;
    // NUMA node of the GPU (sysfs; -1 unknown; mxec_open_test logical copies
    // alternate between pretend nodes 0 and 1), and whether the context's
    // devices sit on more than one node: only then does the host pipeline
    // deal objects by where their pages are and keep its page-locked rings
    // on the device's node (pipeline.cpp).
    int numa_node = -1;
    bool ctx_multi_node = false;
    const Knobs* kn = nullptr;  // the context's settings (read at mxec_open)
    GridTuner tuner;
    std::vector<std::unique_ptr<Slot>> slots;
    std::atomic<unsigned> next_slot{0};
    // Coefficient tables (gf256.hpp coef_tables) for every matrix in use,
    // keyed by matrix identity; uploaded once, read by every launch.  The
    // arena is two halves (kCoefArenaDwords each, or mxec_open_test coef_arena_bytes):
    // generation g fills half g & 1; when it is full, generation g + 1 takes
    // the other half, after waiting for the events that fence the launches
    // which read that half's tables (generation g - 1) -- no device-wide
    // wait, other streams keep running.  A launch whose tables came from a
    // generation recycled before its fence was registered is queued again
    // (with_stable_coef, ops.hpp).
    //
    // New tables go up asynchronously: the host writes them into a page-locked
    // mirror of the arena (1 MiB chunks, allocated on first touch) and
    // hipMemcpyAsync moves them on the device's own table stream, whose
    // event every launch that reads a not-yet-landed table waits on
    // (coef_wait_uploads; a GPU-side wait, not a host one).  A half's mirror
    // is rewritten only after a recycle, which waits for the last upload of
    // the generation it replaces (its event sits among that half's fences).
    // A recycle that must wait for fences releases coef_mu while it waits
    // (coef_recycling holds other allocations back; lookups of live tables
    // go on): no thread holds the lock across a device wait.
    std::mutex coef_mu;
    std::condition_variable coef_cv;  // a recycle's fence wait finished
    bool coef_recycling = false;
    DevBuf coef;
    size_t coef_half = 0;     // dwords per half (set on first use)
    size_t coef_used = 0;     // dwords used in the current half
    uint64_t coef_gen = 0;    // current generation
    struct CoefEntry {
        uint32_t off;  // dword offset
        uint64_t gen;  // generation
        uint64_t seq;  // upload sequence number (coef_seq when it was queued)
    };
    std::map<std::vector<uint8_t>, CoefEntry> coef_index;
    std::vector<hipEvent_t> coef_fences[2];  // after launches that read half h (and its last upload)
    std::vector<hipEvent_t> coef_free;       // spare fence events
    std::vector<PinnedBuf> coef_mirror;      // page-locked image of the arena, in chunks
    size_t coef_mirror_chunk = 0;            // dwords per mirror chunk
    hipStream_t coef_stream = nullptr;       // the table uploads, in order
    hipEvent_t coef_uploaded = nullptr;      // recorded after the newest upload
    uint64_t coef_seq = 0, coef_done = 0;    // uploads queued / known landed
    uint64_t coef_recycles = 0, coef_relaunches = 0, coef_fence_waits = 0, coef_uploads = 0;
    // CRC32 / CRC32C constant tables (sums.cpp), uploaded on first use.
    std::mutex sums_mu;
    DevBuf crc_tables;
    DevBuf aes_te;  // AES T-tables (gcm.cpp)
    // Erasure pattern -> (decode plan, table offset, generation), resolved
    // once per device and dropped with its generation's half (ops.cpp
    // decode_plan).  Key: presence bitmask over k+m <= 256 shards, plus
    // (k, m, data_only).
    struct PatternKey {
        std::array<uint64_t, 4> mask{};
        uint32_t kmf = 0;
        bool operator==(const PatternKey& o) const { return kmf == o.kmf && mask == o.mask; }
    };
    struct PatternHash {
        size_t operator()(const PatternKey& a) const {
            return size_t(a.mask[0] * 0x9E3779B97F4A7C15ull ^ a.mask[1] * 0xC2B2AE3D27D4EB4Full ^
                          a.mask[2] * 0x165667B19E3779F9ull ^ a.mask[3] ^ uint64_t(a.kmf) << 40);
        }
    };
    struct PatternVal {
        std::shared_ptr<const void> plan;
        uint32_t off;
        uint64_t gen;
        uint64_t seq;  // the table's upload (Device::CoefEntry)
    };
    std::unordered_map<PatternKey, PatternVal, PatternHash> patterns;
    // Host-batch pipeline state (pipeline.cpp PipeHub): the four shared
    // streams and the per-call lanes (pinned rings, pools, descriptor
    // arenas); created on first use and kept.  Up to MXEC_PIPE_LANES calls
    // run at once per device, their waves interleaving on the same streams.
    std::mutex pipe_mu;  // guards creation of `pipe`
    std::shared_ptr<void> pipe;
    // Copies the host pipeline issued (mxec_ctx_copy_stats): 1D SDMA DMAs,
    // 2D SDMA DMAs and their rows, CU-wave copy blocks (copy_kernel.hip; the
    // single-request calls' wave copies count too).
    std::atomic<uint64_t> copies_1d{0}, copies_2d{0}, copies_2d_rows{0};
    mutable std::atomic<uint64_t> copy_wave_blocks{0};
    // SDMA watch of the host pipeline (MXEC_PIPE_COPY=auto): upload brackets
    // judged, how many ran below the floor, the last one's rate (MB/s).
    std::atomic<uint64_t> sdma_probes{0}, sdma_slow_verdicts{0}, sdma_last_mbps{0};
    std::atomic<uint64_t> sdma_down_probes{0}, sdma_down_slow_verdicts{0}, sdma_down_last_mbps{0};
    // Piece-major verified reconstruct waves and the verification groups
    // they ran as (pipeline.cpp verify_cuts).
    std::atomic<uint64_t> verify_waves{0}, verify_groups{0};
    // The watch's verdicts as holds (steady_clock ns): calls that start
    // before these instants copy mxec_host_alloc memory by waves, uploads /
    // downloads.  Only a measured slow bracket sets one, and it lapses on its
    // own: the single-request calls read the same instants
    // (capi.cpp copy_waves_get).
    std::atomic<int64_t> waves_up_until_ns{0}, waves_down_until_ns{0};
    // Until this instant a lone speculating verified GET wave downloads by
    // waves (pipeline.cpp spec_judge).
    std::atomic<int64_t> spec_waves_until_ns{0};
    std::atomic<int> spec_slow_run{0};  // slow verdicts in a row
    std::atomic<int> down_slow_run{0};  // slow SDMA download brackets in a row (pipeline watch_judge)
    // Host-batch calls (per device share), those admitted while another ran
    // on the device, speculative piece rebuilds of verified GETs and the
    // objects re-decoded after a verdict, and host waits that paced a shared
    // call's enqueue (pipeline.cpp).
    std::atomic<uint64_t> pipe_calls{0}, pipe_calls_shared{0}, spec_pieces{0}, spec_redos{0}, pace_waits{0};
    // SHA-256 combiner (combiner.cpp): one launch for the verification work
    // of every concurrent caller on this device.
    std::mutex comb_mu;
    std::shared_ptr<void> comb;
};

struct Ctx {
    Knobs knobs;  // read once by mxec_open; every device points at it
    std::vector<std::unique_ptr<Device>> devs;
    std::atomic<unsigned> rr{0};
    // Worker threads of the *_async entry points (async.cpp), created on
    // first use; async_shutdown drains and joins them (mxec_close).
    std::mutex pool_mu;
    std::shared_ptr<void> pool;
};
void async_shutdown(Ctx& c);

// Descriptor tables of many launches in flight at once (host pipeline):
// pinned + device blocks, bump-allocated, never reused until reserve().  The
// first block is sized by the caller's estimate; a wave that needs more (a
// piece-major wave's tables grow with pieces x classes) chains further
// blocks instead of failing, and keeps them for later waves.  Growing costs
// a hipMalloc / hipHostMalloc (no device-wide wait); only re-sizing the
// first block frees memory.
struct DescArena {
    const Device* owner = nullptr;
    struct Block {
        PinnedBuf host;
        DevBuf dev;
    };
    std::vector<std::unique_ptr<Block>> blocks;
    size_t cur = 0;   // block being filled
    size_t used = 0;  // bytes used in it
    uint64_t grown = 0;  // blocks chained beyond the first, over the arena's life (stats)
    // Start a wave: the first block holds at least `bytes`; everything is
    // free.  A first block too small is not re-sized (a free waits for the
    // whole device, and concurrent host-batch calls share it): a new one of
    // `bytes` goes in front, the old ones stay chained behind it.
    int reserve(size_t bytes) {
        if (blocks.empty() || blocks[0]->host.cap < bytes || blocks[0]->dev.cap < bytes) {
            std::unique_ptr<Block> b(new Block());
            MXEC_TRY(b->host.ensure(bytes));
            MXEC_TRY(b->dev.ensure(bytes));
            blocks.insert(blocks.begin(), std::move(b));
        }
        cur = 0;
        used = 0;
        return 0;
    }
    // n bytes (a multiple of 256) of host staging and their device twin.
    int take(size_t n, char** h, char** d) {
        if (blocks.empty()) MXEC_TRY(reserve(size_t(1) << 20));
        while (used + n > blocks[cur]->host.cap || used + n > blocks[cur]->dev.cap) {
            ++cur;
            used = 0;
            if (cur == blocks.size()) {
                const size_t cap = std::max(n, blocks[0]->host.cap);
                blocks.emplace_back(new Block());
                MXEC_TRY(blocks[cur]->host.ensure(cap));
                MXEC_TRY(blocks[cur]->dev.ensure(cap));
                ++grown;
            }
        }
        *h = static_cast<char*>(blocks[cur]->host.p) + used;
        *d = static_cast<char*>(blocks[cur]->dev.p) + used;
        used += n;
        return 0;
    }
};

// Builds one launch's descriptor tables in a pinned ring buffer, uploads
// them on `stream`, and hands back device pointers.
class DescWriter {
public:
    explicit DescWriter(Slot& slot, DescArena* arena = nullptr) : slot_(slot), arena_(arena) {}
    // Reserve `bytes` (16-byte aligned); returns its offset.  Host pointers
    // into the tables are data() + offset, valid once every add() is done.
    size_t add(size_t bytes);
    char* data() { return tmp_.data(); }
    // Upload; dev_base receives the device base to add offsets to.
    int commit(hipStream_t stream, char** dev_base);
    // No upload: the tables stay in the ring entry's page-locked host buffer
    // (mapped into the GPU's address space), which kernels read in place;
    // host_base receives that buffer.  Slot ring only.
    int commit_host(char** host_base);
    // Device scratch of `bytes` that lives as long as this launch's tables
    // (the ring entry is not reused before finish()'s event): after commit,
    // slot ring only (not with an arena).
    int scratch(size_t bytes, void** dev);
    // Record completion after the launches that read the tables.
    int finish(hipStream_t stream);

private:
    Slot& slot_;
    DescArena* arena_;
    DescBuf* buf_ = nullptr;
    std::vector<char> tmp_;
};

// Dwords per half of the coefficient arena (64 MiB of tables).
constexpr size_t kCoefArenaDwords = size_t(16) << 20;

// Device offset (in dwords) of a coefficient table, uploading it on first
// use; records the table's generation with coef_note_use.
int coef_offset(Device& dev, const std::vector<uint8_t>& key, const std::vector<uint32_t>& table,
                uint32_t* off);

// The generations of the tables one batch collected (with_stable_coef):
// coef_offset and the memoised lookups note every table's generation in the
// calling thread's current CoefUse, if one is set.
struct CoefUse {
    uint64_t lo = UINT64_MAX, hi = 0;
    uint64_t seq = 0;  // newest table upload the batch reads (0: none)
    bool any() const { return lo != UINT64_MAX; }
};
void coef_note_use(uint64_t gen, uint64_t seq);
// Before a batch's launches on `s`: if a table it reads may not have landed
// yet, `s` waits (on the GPU) for the table stream's newest upload.
int coef_wait_uploads(Device& dev, const CoefUse& use, hipStream_t s);
CoefUse* coef_use_swap(CoefUse* u);  // sets the thread's current CoefUse, returns the previous
// After a batch's launches are queued on `s`: if every table it used is
// still live, fence them with an event on `s` (a later recycle of their half
// waits for it) and return true; false if one of their halves was recycled
// in the meantime (the batch must be queued again).
int coef_fence(Device& dev, const CoefUse& use, hipStream_t s, bool* live);
// Release the arena's events (context close).
void coef_release(Device& dev);

Device* pick_device(Ctx* ctx, int dev_index);

// MXEC_DEBUG_AFFINITY=1 (tests; read at mxec_open, per context): every launch and copy checks
// that the HIP current device, the stream, the slot, the descriptor arena and
// the data pointers all belong to the device doing the work.  Internal
// streams are tagged with their (logical) device when created, so on
// mxec_open_test logical-device runs -- one card presented as several devices,
// where physical ids cannot tell them apart -- a stream, slot or arena of
// another logical device is still caught.  A violation fails the call with
// MXEC_E_DEVICE; mxec_close prints the running totals to stderr.
bool affinity_on(const Device& d);
void affinity_tag(hipStream_t s, const Device* d);
void affinity_untag(hipStream_t s);  // before the stream is destroyed
int affinity_check(const Device& d, const Slot* slot, hipStream_t s, const char* where,
                   const DescArena* arena = nullptr, const void* const* ptrs = nullptr, size_t n_ptrs = 0);
void affinity_report();  // the process's totals (mxec_close of a context with the checks on)

}  // namespace mxec

// The opaque handle of include/maxio_ec.h.
struct mxec_ctx {
    mxec::Ctx c;
};

namespace mxec {
Slot& lock_slot(Device& dev, std::unique_lock<std::mutex>& lk);

}  // namespace mxec
