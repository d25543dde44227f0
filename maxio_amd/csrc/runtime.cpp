// runtime.cpp — device buffers, descriptor rings, coefficient arena.
#include "runtime.hpp"

#include "kernels.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>

#include <sys/syscall.h>
#include <unistd.h>

namespace mxec {

namespace {
thread_local std::string t_last_error;
}

int set_error(int code, const std::string& msg) {
    t_last_error = msg;
    return code;
}

const char* last_error() { return t_last_error.c_str(); }

int DevBuf::ensure(size_t n) {
    if (n <= cap && p) return MXEC_OK;
    release();
    size_t want = n < 4096 ? 4096 : n;
    MXEC_HIP(hipMalloc(&p, want));
    cap = want;
    return MXEC_OK;
}

int DevBuf::grow(size_t n) {
    if (n <= cap && p) return MXEC_OK;
    const size_t want = std::max(std::max(n, cap * 2), kGrowFloor);
    void* q = nullptr;
    MXEC_HIP(hipMalloc(&q, want));
    if (p) retired.push_back(p);
    p = q;
    cap = want;
    return MXEC_OK;
}

int DevBuf::replace(size_t n) {
    if (n <= cap && p) return MXEC_OK;
    void* q = nullptr;
    MXEC_HIP(hipMalloc(&q, n < 4096 ? 4096 : n));
    if (p) retired.push_back(p);
    p = q;
    cap = n < 4096 ? 4096 : n;
    return MXEC_OK;
}

void DevBuf::free_retired() {
    for (void* q : retired) (void)hipFree(q);
    retired.clear();
}

void DevBuf::release() {
    if (p) (void)hipFree(p);
    for (void* q : retired) (void)hipFree(q);
    retired.clear();
    p = nullptr;
    cap = 0;
}

hipError_t host_malloc_on_node(void** p, size_t n, int node, unsigned flags) {
    constexpr unsigned long kMaxNode = 1024;
    int old_mode = 0;
    unsigned long old_mask[kMaxNode / 64] = {}, mask[kMaxNode / 64] = {};
    bool bound = false;
    if (node >= 0 && unsigned(node) < kMaxNode &&
        syscall(SYS_get_mempolicy, &old_mode, old_mask, kMaxNode + 1, nullptr, 0) == 0) {
        mask[node / 64] = 1ul << (node % 64);
        bound = syscall(SYS_set_mempolicy, 1 /* MPOL_PREFERRED */, mask, kMaxNode + 1) == 0;
    }
    const hipError_t e = hipHostMalloc(p, n, flags | (bound ? hipHostMallocNumaUser : 0));
    if (bound) (void)syscall(SYS_set_mempolicy, old_mode, old_mode ? old_mask : nullptr, old_mode ? kMaxNode + 1 : 0);
    return e;
}

int PinnedBuf::ensure(size_t n) {
    if (n <= cap && p) return MXEC_OK;
    release();
    size_t want = n < 4096 ? 4096 : n;
    MXEC_HIP(host_malloc_on_node(&p, want, node, hipHostMallocDefault));
    cap = want;
    return MXEC_OK;
}

int slot_wait(Slot& slot, hipStream_t s) {
    if (slot.owner && slot.owner->kn && slot.owner->kn->spin_wait) {
        MXEC_HIP(hipStreamSynchronize(s));
        if (slot.borrowed == s) slot.borrowed = nullptr;
        return MXEC_OK;
    }
    if (!slot.sync_ev)
        MXEC_HIP(hipEventCreateWithFlags(&slot.sync_ev, hipEventBlockingSync | hipEventDisableTiming));
    MXEC_HIP(hipEventRecord(slot.sync_ev, s));
    MXEC_HIP(hipEventSynchronize(slot.sync_ev));
    if (slot.borrowed == s) slot.borrowed = nullptr;
    return MXEC_OK;
}

void slot_destroy(Slot& slot) {
    for (auto& rb : slot.ring) {
        if (rb.done) (void)hipEventDestroy(rb.done);
        if (rb.uploaded) (void)hipEventDestroy(rb.uploaded);
    }
    affinity_untag(slot.upload);
    affinity_untag(slot.stream);
    if (slot.upload) (void)hipStreamDestroy(slot.upload);
    slot.upload = nullptr;
    for (auto& e : slot.stage_done)
        if (e) (void)hipEventDestroy(e);
    if (slot.sync_ev) (void)hipEventDestroy(slot.sync_ev);
    if (slot.ready_ev) (void)hipEventDestroy(slot.ready_ev);
    if (slot.stream) (void)hipStreamDestroy(slot.stream);
    slot.stream = nullptr;
}

namespace {
bool hip_says_pinned(const void* p) {
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory is reported as an error
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

// base -> bytes (mxec_host_alloc).  Never destroyed: a caller may free its
// page-locked buffers from its own exit handlers, after this library's
// static destructors would have run.
struct PinnedSet {
    std::mutex mu;
    std::map<uintptr_t, size_t> map;
};
PinnedSet& pinned_set() {
    static PinnedSet* p = new PinnedSet();
    return *p;
}
}  // namespace

void pinned_register(const void* p, size_t n) {
    PinnedSet& ps = pinned_set();
    std::lock_guard<std::mutex> g(ps.mu);
    ps.map[reinterpret_cast<uintptr_t>(p)] = n;
}

void pinned_unregister(const void* p) {
    PinnedSet& ps = pinned_set();
    std::lock_guard<std::mutex> g(ps.mu);
    ps.map.erase(reinterpret_cast<uintptr_t>(p));
}

bool pinned_range(const void* p, uint64_t len) {
    if (!p || !len) return false;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    {
        PinnedSet& ps = pinned_set();
        std::lock_guard<std::mutex> g(ps.mu);
        auto it = ps.map.upper_bound(a);
        if (it != ps.map.begin()) {
            --it;
            if (a - it->first < it->second) return len <= it->second - (a - it->first);
        }
    }
    return hip_says_pinned(p) && hip_says_pinned(static_cast<const uint8_t*>(p) + len - 1);
}

bool pinned_mapped(const void* p, uint64_t len) {
    if (!p || !len) return false;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    PinnedSet& ps = pinned_set();
    std::lock_guard<std::mutex> g(ps.mu);
    auto it = ps.map.upper_bound(a);
    if (it == ps.map.begin()) return false;
    --it;
    return a - it->first < it->second && len <= it->second - (a - it->first);
}

namespace {
// The segments as CU-wave copy blocks, the table read in place from the
// slot's descriptor ring (copy_kernel.hip; 16 workgroups, as pipeline.cpp).
int wave_copy_segments(Slot& slot, hipStream_t s, const std::vector<CopyBlk>& blks, bool to_host) {
    if (blks.empty()) return MXEC_OK;
    DescWriter w(slot);
    const size_t o = w.add(sizeof(CopyBlk) * blks.size());
    std::memcpy(w.data() + o, blks.data(), sizeof(CopyBlk) * blks.size());
    char* hb = nullptr;
    MXEC_TRY(w.commit_host(&hb));
    MXEC_HIP(launch_copy_blocks(reinterpret_cast<const CopyBlk*>(hb + o), blks.size(), to_host, 16, s));
    if (slot.owner) slot.owner->copy_wave_blocks += blks.size();
    return w.finish(s);
}
void add_blocks(std::vector<CopyBlk>& v, uint64_t dst, uint64_t src, uint64_t len) {
    for (uint64_t o = 0; o < len; o += kCopyBlock) v.push_back(CopyBlk{dst + o, src + o, std::min(kCopyBlock, len - o), 0});
}
}  // namespace

int upload_segments(Slot& slot, hipStream_t s, uint8_t* dev_base, const std::vector<UploadSeg>& segs, bool waves) {
    if (slot.owner) {
        const void* b = dev_base;
        MXEC_TRY(affinity_check(*slot.owner, &slot, s, "upload_segments", nullptr, &b, 1));
    }
    if (segs.empty()) return MXEC_OK;
    if (waves) {
        bool mapped = true;
        for (const auto& g : segs)
            mapped = mapped && (g.len == 0 || (pinned_mapped(g.src, g.len) && copy_phase_ok(g.src, dev_base + g.dst_off)));
        if (mapped) {
            std::vector<CopyBlk> blks;
            for (const auto& g : segs)
                if (g.len)
                    add_blocks(blks, reinterpret_cast<uint64_t>(dev_base + g.dst_off), reinterpret_cast<uint64_t>(g.src),
                               g.len);
            slot.borrowed = s;  // the kernel reads the caller's buffers: wait before returning
            return wave_copy_segments(slot, s, blks, false);
        }
    }
    bool all_pinned = true;
    for (const auto& g : segs) all_pinned = all_pinned && (g.len == 0 || pinned_range(g.src, g.len));
    if (all_pinned) {  // DMA straight from the caller's page-locked buffers
        slot.borrowed = s;  // from here on every exit of the call waits on s
        // Segments contiguous on both sides (a GET range's chunks land back
        // to back in the caller's buffer and in 256-byte-aligned slots) go
        // up as one DMA: per-copy submission cost, not bytes, is what the
        // direct path pays over staging.
        for (size_t i = 0; i < segs.size();) {
            if (!segs[i].len) {
                ++i;
                continue;
            }
            const auto* src = static_cast<const uint8_t*>(segs[i].src);
            const uint64_t dst = segs[i].dst_off;
            uint64_t len = segs[i].len;
            size_t j = i + 1;
            while (j < segs.size() && segs[j].len && segs[j].src == src + len && segs[j].dst_off == dst + len)
                len += segs[j++].len;
            MXEC_HIP(hipMemcpyAsync(dev_base + dst, src, len, hipMemcpyHostToDevice, s));
            i = j;
        }
        return MXEC_OK;
    }
    for (auto& e : slot.stage_done)
        if (!e) MXEC_HIP(hipEventCreateWithFlags(&e, hipEventBlockingSync | hipEventDisableTiming));
    // Walk the destination range [lo, hi) in pieces; each piece gathers the
    // bytes of the segments it overlaps (gaps between segments are padding
    // nobody reads) and goes up in one DMA.
    const uint64_t lo = segs.front().dst_off;
    const uint64_t hi = segs.back().dst_off + segs.back().len;
    const uint64_t piece = std::min<uint64_t>(kStagePiece, hi - lo);
    for (auto& b : slot.stage) MXEC_TRY(b.ensure(piece));
    size_t si = 0;
    int buf = 0;
    for (uint64_t a = lo; a < hi; a += piece, buf ^= 1) {
        const uint64_t b = std::min(hi, a + piece);
        // The DMA that last read this buffer must be done before refilling it.
        MXEC_HIP(hipEventSynchronize(slot.stage_done[buf]));
        auto* h = static_cast<uint8_t*>(slot.stage[buf].p);
        while (si < segs.size() && segs[si].dst_off + segs[si].len <= a) ++si;
        for (size_t j = si; j < segs.size() && segs[j].dst_off < b; ++j) {
            const uint64_t x = std::max(a, segs[j].dst_off), y = std::min(b, segs[j].dst_off + segs[j].len);
            if (y > x) std::memcpy(h + (x - a), static_cast<const uint8_t*>(segs[j].src) + (x - segs[j].dst_off), y - x);
        }
        MXEC_HIP(hipMemcpyAsync(dev_base + a, h, b - a, hipMemcpyHostToDevice, s));
        MXEC_HIP(hipEventRecord(slot.stage_done[buf], s));
    }
    return MXEC_OK;
}

int download_segments(Slot& slot, hipStream_t s, const uint8_t* dev_base, const std::vector<DownloadSeg>& segs,
                      bool waves) {
    if (slot.owner) {
        const void* b = dev_base;
        MXEC_TRY(affinity_check(*slot.owner, &slot, s, "download_segments", nullptr, &b, 1));
    }
    if (segs.empty()) return slot_wait(slot, s);
    if (waves) {
        bool mapped = true;
        for (const auto& g : segs)
            mapped = mapped && (g.len == 0 || (pinned_mapped(g.dst, g.len) && copy_phase_ok(g.dst, dev_base + g.src_off)));
        if (mapped) {
            std::vector<CopyBlk> blks;
            for (const auto& g : segs)
                if (g.len)
                    add_blocks(blks, reinterpret_cast<uint64_t>(g.dst), reinterpret_cast<uint64_t>(dev_base + g.src_off),
                               g.len);
            MXEC_TRY(wave_copy_segments(slot, s, blks, true));
            return slot_wait(slot, s);
        }
    }
    bool all_pinned = true;
    for (const auto& g : segs) all_pinned = all_pinned && (g.len == 0 || pinned_range(g.dst, g.len));
    if (all_pinned) {  // DMA straight into the caller's page-locked buffers
        for (size_t i = 0; i < segs.size();) {  // contiguous runs as one DMA (as uploads)
            if (!segs[i].len) {
                ++i;
                continue;
            }
            auto* dst = static_cast<uint8_t*>(segs[i].dst);
            const uint64_t src = segs[i].src_off;
            uint64_t len = segs[i].len;
            size_t j = i + 1;
            while (j < segs.size() && segs[j].len && segs[j].dst == dst + len && segs[j].src_off == src + len)
                len += segs[j++].len;
            MXEC_HIP(hipMemcpyAsync(dst, dev_base + src, len, hipMemcpyDeviceToHost, s));
            i = j;
        }
        return slot_wait(slot, s);
    }
    for (auto& e : slot.stage_done)
        if (!e) MXEC_HIP(hipEventCreateWithFlags(&e, hipEventBlockingSync | hipEventDisableTiming));
    const uint64_t lo = segs.front().src_off;
    const uint64_t hi = segs.back().src_off + segs.back().len;
    const uint64_t piece = std::min<uint64_t>(kStagePiece, hi - lo);
    for (auto& b : slot.stage) MXEC_TRY(b.ensure(piece));
    // Piece i+1's DMA is in flight while piece i is copied out.
    size_t si = 0;
    auto drain = [&](uint64_t a, int buf) -> int {
        const uint64_t b = std::min(hi, a + piece);
        MXEC_HIP(hipEventSynchronize(slot.stage_done[buf]));
        const auto* h = static_cast<const uint8_t*>(slot.stage[buf].p);
        while (si < segs.size() && segs[si].src_off + segs[si].len <= a) ++si;
        for (size_t j = si; j < segs.size() && segs[j].src_off < b; ++j) {
            const uint64_t x = std::max(a, segs[j].src_off), y = std::min(b, segs[j].src_off + segs[j].len);
            if (y > x)
                std::memcpy(static_cast<uint8_t*>(segs[j].dst) + (x - segs[j].src_off),
                            h + (x - a), y - x);
        }
        return MXEC_OK;
    };
    int buf = 0;
    uint64_t prev = UINT64_MAX;
    for (uint64_t a = lo; a < hi; a += piece, buf ^= 1) {
        const uint64_t b = std::min(hi, a + piece);
        // This buffer's previous piece was drained before the one before
        // this iteration's (strict alternation), so it is free.
        MXEC_HIP(hipMemcpyAsync(slot.stage[buf].p, dev_base + a, b - a, hipMemcpyDeviceToHost, s));
        MXEC_HIP(hipEventRecord(slot.stage_done[buf], s));
        if (prev != UINT64_MAX) MXEC_TRY(drain(prev, buf ^ 1));
        prev = a;
    }
    return drain(prev, buf ^ 1);
}

int PinnedBuf::grow(size_t n) {
    if (n <= cap && p) return MXEC_OK;
    const size_t want = std::max(std::max(n, cap * 2), DevBuf::kGrowFloor);
    void* q = nullptr;
    MXEC_HIP(host_malloc_on_node(&q, want, node, hipHostMallocDefault));
    if (p) retired.push_back(p);
    p = q;
    cap = want;
    return MXEC_OK;
}

void PinnedBuf::release() {
    if (p) (void)hipHostFree(p);
    for (void* q : retired) (void)hipHostFree(q);
    retired.clear();
    p = nullptr;
    cap = 0;
}

size_t DescWriter::add(size_t bytes) {
    size_t off = (tmp_.size() + 15) & ~size_t(15);
    tmp_.resize(off + ((bytes + 15) & ~size_t(15)), 0);
    return off;
}

int DescWriter::commit(hipStream_t stream, char** dev_base) {
    if (slot_.owner) MXEC_TRY(affinity_check(*slot_.owner, &slot_, stream, "descriptor upload", arena_));
    if (arena_) {
        const size_t n = std::max<size_t>((tmp_.size() + 255) & ~size_t(255), 256);
        char* h = nullptr;
        char* d = nullptr;
        MXEC_TRY(arena_->take(n, &h, &d));
        std::memcpy(h, tmp_.data(), tmp_.size());
        MXEC_HIP(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, stream));
        *dev_base = d;
        return MXEC_OK;
    }
    buf_ = &slot_.ring[slot_.ring_next];
    slot_.ring_next = (slot_.ring_next + 1) % Slot::kRing;
    if (!buf_->done) MXEC_HIP(hipEventCreateWithFlags(&buf_->done, hipEventDisableTiming));
    if (buf_->pending) {
        MXEC_HIP(hipEventSynchronize(buf_->done));
        buf_->pending = false;
    }
    const size_t n = tmp_.empty() ? 16 : tmp_.size();
    MXEC_TRY(buf_->host.grow(n));
    MXEC_TRY(buf_->dev.grow(n));
    std::memcpy(buf_->host.p, tmp_.data(), tmp_.size());
    // Large tables (a mixed batch's: MiBs) go on the side stream; small ones
    // stay in the launch stream, where the extra cross-stream wait measured
    // no better (config 3c's per-call decodes, profiles/r2_desc_upload_ab.txt).
    const int mode = slot_.owner && slot_.owner->kn ? slot_.owner->kn->desc_upload : 1;
    if (mode == 0 || (mode == 1 && n < (size_t(256) << 10))) {
        MXEC_HIP(hipMemcpyAsync(buf_->dev.p, buf_->host.p, n, hipMemcpyHostToDevice, stream));
    } else {
        // The entry's previous launches are done (waited above), so the copy
        // needs no ordering against `stream`; only the launches that follow
        // wait for it.
        if (!slot_.upload) {
            MXEC_HIP(hipStreamCreateWithFlags(&slot_.upload, hipStreamNonBlocking));
            affinity_tag(slot_.upload, slot_.owner);
        }
        if (!buf_->uploaded) MXEC_HIP(hipEventCreateWithFlags(&buf_->uploaded, hipEventDisableTiming));
        MXEC_HIP(hipMemcpyAsync(buf_->dev.p, buf_->host.p, n, hipMemcpyHostToDevice, slot_.upload));
        MXEC_HIP(hipEventRecord(buf_->uploaded, slot_.upload));
        MXEC_HIP(hipStreamWaitEvent(stream, buf_->uploaded, 0));
    }
    *dev_base = static_cast<char*>(buf_->dev.p);
    return MXEC_OK;
}

int DescWriter::commit_host(char** host_base) {
    if (arena_) return set_error(MXEC_E_INVALID_ARG, "commit_host: slot ring only");
    buf_ = &slot_.ring[slot_.ring_next];
    slot_.ring_next = (slot_.ring_next + 1) % Slot::kRing;
    if (!buf_->done) MXEC_HIP(hipEventCreateWithFlags(&buf_->done, hipEventDisableTiming));
    if (buf_->pending) {
        MXEC_HIP(hipEventSynchronize(buf_->done));
        buf_->pending = false;
    }
    MXEC_TRY(buf_->host.grow(tmp_.empty() ? 16 : tmp_.size()));
    std::memcpy(buf_->host.p, tmp_.data(), tmp_.size());
    *host_base = static_cast<char*>(buf_->host.p);
    return MXEC_OK;
}

int DescWriter::scratch(size_t bytes, void** dev) {
    if (arena_ || !buf_) return set_error(MXEC_E_INVALID_ARG, "descriptor scratch needs a committed ring entry");
    MXEC_TRY(buf_->scratch.grow(bytes));
    *dev = buf_->scratch.p;
    return MXEC_OK;
}

int DescWriter::finish(hipStream_t stream) {
    if (arena_ || !buf_) return MXEC_OK;
    MXEC_HIP(hipEventRecord(buf_->done, stream));
    buf_->pending = true;
    return MXEC_OK;
}

namespace {
thread_local CoefUse* t_coef_use = nullptr;

// Drop fences whose launches finished (keeps the lists short).
void coef_prune(Device& dev, int h) {
    auto& v = dev.coef_fences[h];
    size_t w = 0;
    for (size_t i = 0; i < v.size(); ++i) {
        if (hipEventQuery(v[i]) == hipSuccess) dev.coef_free.push_back(v[i]);
        else v[w++] = v[i];
    }
    (void)hipGetLastError();  // hipErrorNotReady from the queries
    v.resize(w);
}
}  // namespace

void coef_note_use(uint64_t gen, uint64_t seq) {
    if (!t_coef_use) return;
    t_coef_use->lo = std::min(t_coef_use->lo, gen);
    t_coef_use->hi = std::max(t_coef_use->hi, gen);
    t_coef_use->seq = std::max(t_coef_use->seq, seq);
}

CoefUse* coef_use_swap(CoefUse* u) {
    CoefUse* p = t_coef_use;
    t_coef_use = u;
    return p;
}

namespace {
// An event from the spare list (or a new one).  Under coef_mu.
int coef_take_event(Device& dev, hipEvent_t* e) {
    if (!dev.coef_free.empty()) {
        *e = dev.coef_free.back();
        dev.coef_free.pop_back();
        return MXEC_OK;
    }
    MXEC_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
    return MXEC_OK;
}

// First use of the device's arena: the device halves, the table stream and
// its event.  Under coef_mu.
int coef_init(Device& dev) {
    const uint64_t test = dev.kn ? dev.kn->test_coef_arena : 0;
    dev.coef_half = test ? size_t(test / 4) : kCoefArenaDwords;
    MXEC_TRY(dev.coef.ensure(dev.coef_half * 2 * 4));
    dev.coef_used = 0;
    dev.coef_mirror_chunk = std::min(dev.coef_half * 2, size_t(1) << 18);  // <= 1 MiB
    dev.coef_mirror.resize((dev.coef_half * 2 + dev.coef_mirror_chunk - 1) / dev.coef_mirror_chunk);
    if (!dev.coef_stream) {
        MXEC_HIP(hipStreamCreateWithFlags(&dev.coef_stream, hipStreamNonBlocking));
        affinity_tag(dev.coef_stream, &dev);
    }
    if (!dev.coef_uploaded) MXEC_HIP(hipEventCreateWithFlags(&dev.coef_uploaded, hipEventDisableTiming));
    return MXEC_OK;
}

// Queue dwords [o, o + n) of the arena's mirror up to the device.  Under
// coef_mu; nothing here waits for the device.
int coef_upload(Device& dev, uint32_t o, const std::vector<uint32_t>& table) {
    const size_t C = dev.coef_mirror_chunk;
    for (size_t done = 0; done < table.size();) {
        const size_t at = size_t(o) + done, c = at / C, in = at % C;
        const size_t n = std::min(table.size() - done, C - in);
        PinnedBuf& chunk = dev.coef_mirror[c];
        if (!chunk.p) MXEC_TRY(chunk.ensure(C * 4));
        uint32_t* h = static_cast<uint32_t*>(chunk.p) + in;
        std::memcpy(h, table.data() + done, n * 4);
        MXEC_HIP(hipMemcpyAsync(static_cast<uint32_t*>(dev.coef.p) + at, h, n * 4, hipMemcpyHostToDevice,
                                dev.coef_stream));
        done += n;
    }
    MXEC_HIP(hipEventRecord(dev.coef_uploaded, dev.coef_stream));
    ++dev.coef_seq;
    ++dev.coef_uploads;
    return MXEC_OK;
}
}  // namespace

int coef_offset(Device& dev, const std::vector<uint8_t>& key, const std::vector<uint32_t>& table,
                uint32_t* off) {
    std::unique_lock<std::mutex> lk(dev.coef_mu);
    for (;;) {
        auto it = dev.coef_index.find(key);
        if (it != dev.coef_index.end()) {
            *off = it->second.off;
            coef_note_use(it->second.gen, it->second.seq);
            return MXEC_OK;
        }
        if (!dev.coef.p) MXEC_TRY(coef_init(dev));
        if (table.size() > dev.coef_half)
            return set_error(MXEC_E_INVALID_ARG, "coefficient table larger than the arena");
        if (dev.coef_recycling) {  // another thread is waiting out a recycle's fences
            dev.coef_cv.wait(lk);
            continue;
        }
        if (dev.coef_used + table.size() <= dev.coef_half) break;
        // This half is full: the next generation takes the other half, whose
        // tables (two generations old) may still be read by fenced launches
        // or, for the newest of them, still be on their way up.  Wait for
        // those outside the lock, then look again.
        const uint64_t next = dev.coef_gen + 1;
        const int h = int(next & 1);
        std::vector<hipEvent_t> busy;
        for (hipEvent_t e : dev.coef_fences[h])
            if (hipEventQuery(e) != hipSuccess) busy.push_back(e);
        (void)hipGetLastError();
        if (!busy.empty()) {
            ++dev.coef_fence_waits;
            dev.coef_recycling = true;
            lk.unlock();
            int rc = MXEC_OK;
            for (hipEvent_t e : busy)
                if (hipEventSynchronize(e) != hipSuccess) rc = set_error(MXEC_E_DEVICE, "coefficient fence wait failed");
            lk.lock();
            dev.coef_recycling = false;
            dev.coef_cv.notify_all();
            MXEC_TRY(rc);
            continue;  // fences added meanwhile are waited for too
        }
        for (hipEvent_t e : dev.coef_fences[h]) dev.coef_free.push_back(e);
        dev.coef_fences[h].clear();
        // The generation being closed: its last upload fences its half, so
        // that half's mirror is not rewritten before the copies read it.
        hipEvent_t last = nullptr;
        MXEC_TRY(coef_take_event(dev, &last));
        if (hipEventRecord(last, dev.coef_stream) != hipSuccess) {
            dev.coef_free.push_back(last);
            return set_error(MXEC_E_DEVICE, "coefficient upload fence: hipEventRecord failed");
        }
        dev.coef_fences[dev.coef_gen & 1].push_back(last);
        for (auto i = dev.coef_index.begin(); i != dev.coef_index.end();)
            i = i->second.gen + 1 < next ? dev.coef_index.erase(i) : std::next(i);
        for (auto i = dev.patterns.begin(); i != dev.patterns.end();)
            i = i->second.gen + 1 < next ? dev.patterns.erase(i) : std::next(i);
        dev.coef_gen = next;
        dev.coef_used = 0;
        ++dev.coef_recycles;
        break;
    }
    const uint32_t o = uint32_t(size_t(dev.coef_gen & 1) * dev.coef_half + dev.coef_used);
    MXEC_TRY(coef_upload(dev, o, table));
    dev.coef_used += (table.size() + 3) & ~size_t(3);
    dev.coef_index.emplace(key, Device::CoefEntry{o, dev.coef_gen, dev.coef_seq});
    coef_note_use(dev.coef_gen, dev.coef_seq);
    *off = o;
    return MXEC_OK;
}

int coef_wait_uploads(Device& dev, const CoefUse& use, hipStream_t s) {
    if (use.seq == 0) return MXEC_OK;
    std::lock_guard<std::mutex> g(dev.coef_mu);
    if (use.seq <= dev.coef_done) return MXEC_OK;
    if (hipEventQuery(dev.coef_uploaded) == hipSuccess) {
        dev.coef_done = dev.coef_seq;  // the newest upload landed, and every one before it
        return MXEC_OK;
    }
    (void)hipGetLastError();
    // The wait is captured at this call: later re-records of the event do not
    // move it (it may wait for a few newer uploads too, which is harmless).
    MXEC_HIP(hipStreamWaitEvent(s, dev.coef_uploaded, 0));
    return MXEC_OK;
}

int coef_fence(Device& dev, const CoefUse& use, hipStream_t s, bool* live) {
    *live = true;
    if (!use.any()) return MXEC_OK;
    std::lock_guard<std::mutex> g(dev.coef_mu);
    // Generation lo's half is reused by generation lo + 2.
    if (dev.coef_gen > use.lo + 1) {
        *live = false;
        ++dev.coef_relaunches;
        return MXEC_OK;
    }
    for (uint64_t gen = use.lo; gen <= use.hi; ++gen) {
        const int h = int(gen & 1);
        if (dev.coef_fences[h].size() >= 64) coef_prune(dev, h);
        hipEvent_t e = nullptr;
        if (!dev.coef_free.empty()) {
            e = dev.coef_free.back();
            dev.coef_free.pop_back();
        } else {
            MXEC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        if (hipEventRecord(e, s) != hipSuccess) {
            dev.coef_free.push_back(e);
            return set_error(MXEC_E_DEVICE, "coefficient fence: hipEventRecord failed");
        }
        dev.coef_fences[h].push_back(e);
    }
    return MXEC_OK;
}

void coef_release(Device& dev) {
    std::lock_guard<std::mutex> g(dev.coef_mu);
    if (dev.coef_stream) (void)hipStreamSynchronize(dev.coef_stream);
    for (auto& v : dev.coef_fences) {
        for (hipEvent_t e : v) (void)hipEventDestroy(e);
        v.clear();
    }
    for (hipEvent_t e : dev.coef_free) (void)hipEventDestroy(e);
    dev.coef_free.clear();
    if (dev.coef_uploaded) (void)hipEventDestroy(dev.coef_uploaded);
    dev.coef_uploaded = nullptr;
    if (dev.coef_stream) {
        affinity_untag(dev.coef_stream);
        (void)hipStreamDestroy(dev.coef_stream);
    }
    dev.coef_stream = nullptr;
    dev.coef_mirror.clear();
}

namespace {
std::atomic<uint64_t> g_aff_checks{0}, g_aff_bad{0};
std::mutex g_aff_mu;
std::unordered_map<hipStream_t, const Device*>& aff_streams() {
    static auto* m = new std::unordered_map<hipStream_t, const Device*>();
    return *m;
}
}  // namespace

bool affinity_on(const Device& d) { return d.kn && d.kn->debug_affinity; }

void affinity_tag(hipStream_t s, const Device* d) {
    if (!s || !d || !affinity_on(*d)) return;
    std::lock_guard<std::mutex> g(g_aff_mu);
    aff_streams()[s] = d;
}

void affinity_untag(hipStream_t s) {
    // Always (the tag may have been set while the check was on): a destroyed
    // stream's handle can come back as another device's stream.
    if (!s) return;
    std::lock_guard<std::mutex> g(g_aff_mu);
    aff_streams().erase(s);
}

int affinity_check(const Device& d, const Slot* slot, hipStream_t s, const char* where, const DescArena* arena,
                   const void* const* ptrs, size_t n_ptrs) {
    if (!affinity_on(d)) return MXEC_OK;
    g_aff_checks.fetch_add(1);
    std::string bad;
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != d.id)
        bad = "current HIP device " + std::to_string(cur) + ", work for device " + std::to_string(d.id);
    if (bad.empty() && slot && slot->owner && slot->owner != &d) bad = "slot of another (logical) device";
    if (bad.empty() && arena && arena->owner && arena->owner != &d) bad = "descriptor arena of another (logical) device";
    if (bad.empty() && s) {
        {
            std::lock_guard<std::mutex> g(g_aff_mu);
            auto it = aff_streams().find(s);
            if (it != aff_streams().end() && it->second != &d) bad = "stream of another (logical) device";
        }
        int sd = -1;
        if (bad.empty() && hipStreamGetDevice(s, &sd) == hipSuccess && sd != d.id)
            bad = "stream on HIP device " + std::to_string(sd);
        (void)hipGetLastError();
    }
    for (size_t i = 0; bad.empty() && i < n_ptrs; ++i) {
        hipPointerAttribute_t at{};
        if (ptrs[i] && hipPointerGetAttributes(&at, ptrs[i]) == hipSuccess && at.type == hipMemoryTypeDevice &&
            at.device != d.id)
            bad = "device pointer of HIP device " + std::to_string(at.device);
        (void)hipGetLastError();
    }
    if (bad.empty()) return MXEC_OK;
    g_aff_bad.fetch_add(1);
    fprintf(stderr, "maxio_ec affinity violation in %s: %s\n", where, bad.c_str());
    return set_error(MXEC_E_DEVICE, std::string("affinity violation in ") + where + ": " + bad);
}

void affinity_report() {
    fprintf(stderr, "maxio_ec affinity: %llu checks, %llu violations\n",
            static_cast<unsigned long long>(g_aff_checks.load()), static_cast<unsigned long long>(g_aff_bad.load()));
}

Device* pick_device(Ctx* ctx, int dev_index) {
    if (!ctx || ctx->devs.empty()) return nullptr;
    if (dev_index < 0) dev_index = int(ctx->rr.fetch_add(1) % ctx->devs.size());
    if (dev_index >= int(ctx->devs.size())) return nullptr;
    return ctx->devs[size_t(dev_index)].get();
}

Slot& lock_slot(Device& dev, std::unique_lock<std::mutex>& lk) {
    const size_t n = dev.slots.size();
    const unsigned start = dev.next_slot.fetch_add(1);
    for (size_t t = 0; t < n; ++t) {
        Slot& s = *dev.slots[(start + t) % n];
        std::unique_lock<std::mutex> l(s.mu, std::try_to_lock);
        if (l.owns_lock()) {
            lk = std::move(l);
            return s;
        }
    }
    Slot& s = *dev.slots[start % n];
    lk = std::unique_lock<std::mutex>(s.mu);
    return s;
}

}  // namespace mxec
