// capi.cpp — extern "C" entry points of include/maxio_ec.h (context, host
// pointer drop-ins, device-resident batches).  No exception crosses the ABI.
#include <algorithm>
#include <array>
#include <cctype>
#include <chrono>
#include <fstream>
#include <cstdio>
#include <cstdlib>
#include <unordered_map>
#include <cstring>
#include <map>
#include <string>
#include <tuple>

#include <sys/syscall.h>
#include <unistd.h>

#include "../../include/maxio_ec.h"
#include "ops.hpp"

using namespace mxec;

namespace {

// MXEC_PIPE_COPY (knobs.hpp): whether a host-pointer call's copies of
// mxec_host_alloc memory may go by CU-wave copy kernels -- the reconstruct /
// hash (GET) paths under auto and waves, the encode (PUT) path under waves
// only (pipeline.cpp has the measurements behind the split).
bool copy_waves_get(const Device& d) {
    if (!d.kn) return false;
    if (d.kn->pipe_copy == 1) return true;
    if (d.kn->pipe_copy != 2) return false;
    const int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                            std::chrono::steady_clock::now().time_since_epoch()).count();
    return now < d.waves_up_until_ns.load() || now < d.waves_down_until_ns.load();
}
bool copy_waves_put(const Device& d) { return d.kn && d.kn->pipe_copy == 1; }

// One object of a device-resident reconstruct batch (device shard pointers).
struct BatchObj {
    int k, m;
    uint64_t shard_size;
    uint8_t* const* shards;  // k + m
    const uint64_t* len;     // k + m, clamped to shard_size
    uint8_t* present;        // k + m, host
};

// Rebuilds objects `which` of a batch from their present masks as they stand
// (chunk_reader.rs:190-211 per object): one decode plan per object, one launch
// per number of shards to rebuild, shared by objects of every (k, m) and
// shard size (run_rs_mixed).  Rebuilt shards become present; an object short
// of k shards gets MXEC_E_TOO_FEW_SHARDS_PRESENT in st.
int rebuild_batch(Device& d, Slot& slot, hipStream_t s, bool data_only, const std::vector<BatchObj>& all,
                  const std::vector<uint64_t>& which, std::vector<int32_t>& st) {
    std::vector<std::shared_ptr<const DecodePlan>> plans(which.size());
    std::vector<uint32_t> offs(which.size());
    std::vector<const uint8_t*> in;
    std::vector<uint8_t*> out;
    std::vector<uint64_t> il, ol;
    std::map<int, std::vector<RsMixedObject>> groups;
    auto collect = [&]() -> int {
        for (size_t t = 0; t < which.size(); ++t) {
            const BatchObj& b = all[which[t]];
            MXEC_TRY(decode_plan(d, b.k, b.m, b.present, data_only, &plans[t], &offs[t]));
        }
        return MXEC_OK;
    };
    auto launch = [&]() -> int {
        // Pointer and length tables of every rebuilt object, sized up front
        // (the RsObjects point into them).
        size_t n_in = 0, n_out = 0;
        for (size_t t = 0; t < which.size(); ++t) {
            st[which[t]] = plans[t] ? MXEC_OK : MXEC_E_TOO_FEW_SHARDS_PRESENT;
            if (plans[t] && !plans[t]->missing.empty()) {
                n_in += size_t(all[which[t]].k);
                n_out += plans[t]->missing.size();
            }
        }
        in.assign(n_in, nullptr);
        out.assign(n_out, nullptr);
        il.assign(n_in, 0);
        ol.assign(n_out, 0);
        groups.clear();
        size_t pi = 0, po = 0;
        for (size_t t = 0; t < which.size(); ++t) {
            if (!plans[t] || plans[t]->missing.empty()) continue;
            const BatchObj& b = all[which[t]];
            const DecodePlan& p = *plans[t];
            const int r = int(p.missing.size());
            for (int v = 0; v < b.k; ++v) {
                in[pi + v] = b.shards[p.valid[size_t(v)]];
                il[pi + v] = b.len[p.valid[size_t(v)]];
            }
            for (int e = 0; e < r; ++e) {
                out[po + e] = b.shards[p.missing[size_t(e)]];
                ol[po + e] = b.len[p.missing[size_t(e)]];
            }
            groups[r].push_back(RsMixedObject{b.k, b.shard_size, RsObject{&in[pi], &il[pi], &out[po], &ol[po], offs[t]}});
            pi += size_t(b.k);
            po += size_t(r);
        }
        return run_rs_mixed(d, slot, s, groups);
    };
    MXEC_TRY(with_stable_coef(d, s, collect, launch));
    for (size_t t = 0; t < which.size(); ++t)
        if (plans[t])
            for (int e : plans[t]->missing) all[which[t]].present[e] = 1;
    return MXEC_OK;
}

}  // namespace

extern "C" {

const char* mxec_version(void) {
#ifdef MXEC_LAB
    return "maxio_ec 0.1.0 (gfx950, lab build)";
#else
    return "maxio_ec 0.1.0 (gfx950)";
#endif
}

const char* mxec_strerror(int code) {
    switch (code) {
        case MXEC_OK: return "ok";
        case MXEC_E_TOO_FEW_SHARDS: return "The number of provided shards is smaller than the one in codec";
        case MXEC_E_TOO_MANY_SHARDS: return "The number of provided shards is greater than the one in codec";
        case MXEC_E_TOO_FEW_DATA_SHARDS: return "The number of provided data shards is smaller than the one in codec";
        case MXEC_E_TOO_MANY_DATA_SHARDS: return "The number of provided data shards is greater than the one in codec";
        case MXEC_E_TOO_FEW_PARITY_SHARDS: return "The number of provided parity shards is smaller than the one in codec";
        case MXEC_E_TOO_MANY_PARITY_SHARDS: return "The number of provided parity shards is greater than the one in codec";
        case MXEC_E_TOO_FEW_BUFFER_SHARDS: return "The number of provided buffer shards is smaller than the number of parity shards in codec";
        case MXEC_E_TOO_MANY_BUFFER_SHARDS: return "The number of provided buffer shards is greater than the number of parity shards in codec";
        case MXEC_E_INCORRECT_SHARD_SIZE: return "At least one of the provided shards is not of the correct size";
        case MXEC_E_TOO_FEW_SHARDS_PRESENT: return "The number of shards present is smaller than number of parity shards, cannot reconstruct missing shards";
        case MXEC_E_EMPTY_SHARD: return "The first shard provided is of zero length";
        case MXEC_E_INVALID_SHARD_FLAGS: return "The number of flags does not match the total number of shards";
        case MXEC_E_INVALID_INDEX: return "The data shard index provided is greater or equal to the number of data shards in codec";
        case MXEC_E_SINGULAR_MATRIX: return "singular matrix";
        case MXEC_E_TOO_MANY_SHARDS_255: return "too many shards (> 255, GF(2^8) limit)";
        case MXEC_E_INVALID_ARG: return "invalid argument";
        case MXEC_E_DEVICE: return "HIP device error";
        case MXEC_E_OOM: return "out of memory";
        case MXEC_E_NO_DEVICE: return "no HIP device";
        case MXEC_E_IO: return "IO error";
        case MXEC_E_INTEGRITY: return "integrity error";
        case MXEC_E_JSON: return "JSON error";
        default: return "unknown error";
    }
}

const char* mxec_last_error(void) { return last_error(); }

int mxec_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

namespace {

// NUMA node of HIP device `dev` (sysfs, through its PCI bus id), or -1.
int device_numa_node(int dev) {
    char bus[64] = {};
    if (hipDeviceGetPCIBusId(bus, int(sizeof bus), dev) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    for (char& c : bus) c = char(std::tolower(static_cast<unsigned char>(c)));
    std::ifstream f(std::string("/sys/bus/pci/devices/") + bus + "/numa_node");
    int node = -1;
    return f >> node ? node : -1;
}

// The node all of the context's devices sit on, or -1 (unknown or several).
int ctx_numa_node(const mxec_ctx* ctx) {
    int node = -1;
    for (const auto& d : ctx->c.devs) {
        const int n = d->numa_node;
        if (n < 0 || (node >= 0 && n != node)) return -1;
        node = n;
    }
    return node;
}

}  // namespace

namespace {
// The one open path.  `logical` > 1 (mxec_open_test only) opens every
// selected device that many times, each copy with its own slots, streams,
// arenas, combiner and pipeline, so the multi-device paths (per-device
// workers, round robin, error aggregation) run on a one-GPU box.
mxec_ctx* open_ctx(uint32_t device_mask, int streams_per_device, const Knobs& kn) {
    try {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
            set_error(MXEC_E_NO_DEVICE, "no HIP device visible");
            return nullptr;
        }
        if (streams_per_device < 1) streams_per_device = 1;
        const int logical = kn.test_logical_devices;
        auto* ctx = new mxec_ctx();
        ctx->c.knobs = kn;
        for (int dl = 0; dl < n * logical && dl < 32 * logical; ++dl) {
            const int d = dl / logical;
            if (device_mask && !(device_mask & (1u << d))) continue;
            auto dev = std::make_unique<Device>();
            dev->id = d;
            dev->kn = &ctx->c.knobs;
            if (hipSetDevice(d) != hipSuccess) continue;
            int cus = 0;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && cus > 0)
                dev->n_cus = cus;
            // test-only logical copies pretend to sit on two nodes, so the
            // host pipeline's NUMA dealing runs on a one-card box
            dev->numa_node = logical > 1 ? (dl % logical) % 2 : device_numa_node(d);
            bool ok = true;
            for (int s = 0; s < streams_per_device; ++s) {
                auto slot = std::make_unique<Slot>();
                slot->owner = dev.get();
                if (hipStreamCreateWithFlags(&slot->stream, hipStreamNonBlocking) != hipSuccess) {
                    ok = false;
                    break;
                }
                affinity_tag(slot->stream, dev.get());
                // Descriptor ring entries at their 1 MiB floor now, so the
                // first calls on each slot do not allocate (and a later
                // re-size, which frees and so waits for the device, is rare).
                for (auto& rb : slot->ring)
                    if (rb.host.grow(1) || rb.dev.grow(1)) {
                        ok = false;
                        break;
                    }
                if (!ok) {
                    slot_destroy(*slot);
                    break;
                }
                dev->slots.push_back(std::move(slot));
            }
            if (ok && pipe_open(*dev) != MXEC_OK) {
                for (auto& sl : dev->slots) slot_destroy(*sl);
                ok = false;
            }
            if (ok) ctx->c.devs.push_back(std::move(dev));
        }
        if (ctx->c.devs.empty()) {
            delete ctx;
            set_error(MXEC_E_NO_DEVICE, "no selected HIP device could be opened");
            return nullptr;
        }
        bool multi = false;
        for (const auto& d : ctx->c.devs)
            multi = multi || (d->numa_node >= 0 && d->numa_node != ctx->c.devs[0]->numa_node);
        for (auto& d : ctx->c.devs) d->ctx_multi_node = multi && d->numa_node >= 0;
        return ctx;
    } catch (...) {
        set_error(MXEC_E_OOM, "context allocation failed");
        return nullptr;
    }
}
}  // namespace

// Every documented setting is read once, here (knobs.hpp).
mxec_ctx* mxec_open(uint32_t device_mask, int streams_per_device) {
    return open_ctx(device_mask, streams_per_device, read_knobs());
}

// Test-only settings come as arguments, never from the environment, so no
// variable a production host may carry can make one card pose as several
// devices, cap the RS grid or shrink the coefficient arena.
mxec_ctx* mxec_open_test(uint32_t device_mask, int streams_per_device, int logical_devices, uint32_t rs_grid_cap,
                         uint64_t coef_arena_bytes) {
    Knobs kn = read_knobs();
    if (logical_devices < 1 || logical_devices > 8 || coef_arena_bytes > (uint64_t(64) << 20) ||
        rs_grid_cap > (1u << 30)) {
        set_error(MXEC_E_INVALID_ARG, "mxec_open_test: logical_devices 1..8, rs_grid_cap <= 2^30, "
                                      "coef_arena_bytes <= 64 MiB");
        return nullptr;
    }
    kn.test_logical_devices = logical_devices;
    kn.test_rs_grid = rs_grid_cap;
    kn.test_coef_arena = coef_arena_bytes & ~uint64_t(3);
    return open_ctx(device_mask, streams_per_device, kn);
}

void mxec_close(mxec_ctx* ctx) {
    if (!ctx) return;
    async_shutdown(ctx->c);  // every queued *_async call finishes first
    if (ctx->c.knobs.debug_affinity) affinity_report();
    for (auto& d : ctx->c.devs) {
        (void)hipSetDevice(d->id);
        (void)hipDeviceSynchronize();
        // The host pipeline's lanes (pinned rings, pools, descriptor arenas,
        // events) and its four streams, and the combiner's streams, go first
        // and explicitly, while the device is idle.
        {
            std::lock_guard<std::mutex> g(d->pipe_mu);
            d->pipe.reset();
        }
        {
            std::lock_guard<std::mutex> g(d->comb_mu);
            d->comb.reset();
        }
        rs_grid_release(*d);
        coef_release(*d);
        for (auto& s : d->slots) slot_destroy(*s);
    }
    delete ctx;
}

int mxec_ctx_device_count(const mxec_ctx* ctx) { return ctx ? int(ctx->c.devs.size()) : 0; }

int mxec_ctx_device_id(const mxec_ctx* ctx, int i) {
    if (!ctx || i < 0 || i >= int(ctx->c.devs.size())) return -1;
    return ctx->c.devs[size_t(i)]->id;
}

int mxec_ctx_pipe_stats(mxec_ctx* ctx, int dev, uint64_t* out, int n) {
    if (!ctx || dev < 0 || dev >= int(ctx->c.devs.size()) || !out || n < 0)
        return set_error(MXEC_E_INVALID_ARG, "mxec_ctx_pipe_stats: no such device or no output");
    const Device& d = *ctx->c.devs[size_t(dev)];
    const uint64_t v[MXEC_PIPE_STAT_COUNT] = {d.copies_1d.load(),        d.copies_2d.load(),
                                              d.copies_2d_rows.load(),   d.copy_wave_blocks.load(),
                                              d.sdma_probes.load(),      d.sdma_slow_verdicts.load(),
                                              d.verify_waves.load(),     d.verify_groups.load(),
                                              d.sdma_last_mbps.load(),   d.sdma_down_probes.load(),
                                              d.sdma_down_slow_verdicts.load(), d.sdma_down_last_mbps.load(),
                                              d.pipe_calls.load(),       d.pipe_calls_shared.load(),
                                              d.spec_pieces.load(),      d.spec_redos.load(),
                                              d.pace_waits.load()};
    const int k = std::min(n, int(MXEC_PIPE_STAT_COUNT));
    for (int i = 0; i < k; ++i) out[i] = v[i];
    return k;
}

int mxec_ctx_combiner_stats(mxec_ctx* ctx, int i, uint64_t* launches, uint64_t* messages) {
    if (!ctx || i < 0 || i >= int(ctx->c.devs.size()) || !launches || !messages)
        return set_error(MXEC_E_INVALID_ARG, "invalid argument");
    combiner_stats(*ctx->c.devs[size_t(i)], launches, messages);
    return MXEC_OK;
}

int mxec_ctx_coef_stats(mxec_ctx* ctx, int dev, uint64_t* recycles, uint64_t* relaunches, uint64_t* fence_waits) {
    if (!ctx || dev < 0 || dev >= int(ctx->c.devs.size()) || !recycles || !relaunches)
        return set_error(MXEC_E_INVALID_ARG, "invalid argument");
    Device& d = *ctx->c.devs[size_t(dev)];
    std::lock_guard<std::mutex> g(d.coef_mu);
    *recycles = d.coef_recycles;
    *relaunches = d.coef_relaunches;
    if (fence_waits) *fence_waits = d.coef_fence_waits;
    return MXEC_OK;
}

int mxec_ctx_rs_grid(mxec_ctx* ctx, int dev, int k, int m, uint64_t shard_size) {
    if (!ctx || dev < 0 || dev >= int(ctx->c.devs.size()) || k < 1 || m < 1)
        return set_error(MXEC_E_INVALID_ARG, "invalid argument");
    return guarded([&] { return rs_grid_in_use(*ctx->c.devs[size_t(dev)], k, m, shard_size); });
}


// Page-locked memory on the NUMA node of the context's GPUs with
// MXEC_HOST_NUMA=1 (default: wherever the calling thread's policy puts it).  The pages are placed when
// hipHostMalloc pins them, so the thread's policy is set to that node around
// the call (hipHostMallocNumaUser) and restored after; if the node is unknown
// or the policy calls are refused, the allocation is the plain one.  A
// process may run on every core of a two-socket host, and a DMA from the far
// socket's memory crosses the socket link.
namespace {
void* host_alloc_on(size_t bytes, int node) {
    void* p = nullptr;
    if (host_malloc_on_node(&p, bytes, node, hipHostMallocPortable) != hipSuccess) {
        (void)hipGetLastError();
        set_error(MXEC_E_OOM, "pinned host allocation failed");
        return nullptr;
    }
    pinned_register(p, bytes);
    return p;
}
}  // namespace

void* mxec_host_alloc(mxec_ctx* ctx, size_t bytes) {
    if (!ctx || bytes == 0) return nullptr;
    return host_alloc_on(bytes, ctx->c.knobs.host_numa ? ctx_numa_node(ctx) : -1);  // opt-in until measured
}

// On a two-socket host a context spans both nodes and mxec_host_alloc has no
// one node to pick (ctx_numa_node gives up): a request body meant for device
// `dev` goes on that device's node, whatever MXEC_HOST_NUMA says, and the
// host batch calls then deal the object to a device on that node
// (deal.hpp deal_objects_numa).
void* mxec_host_alloc_device(mxec_ctx* ctx, int dev, size_t bytes) {
    if (!ctx || bytes == 0 || dev < 0 || dev >= int(ctx->c.devs.size())) {
        set_error(MXEC_E_INVALID_ARG, "mxec_host_alloc_device: no such device or zero bytes");
        return nullptr;
    }
    return host_alloc_on(bytes, ctx->c.devs[size_t(dev)]->numa_node);
}

void mxec_host_free(mxec_ctx* ctx, void* p) {
    (void)ctx;
    if (!p) return;
    pinned_unregister(p);
    (void)hipHostFree(p);
}

int mxec_rs_check(int k, int m) { return rs_check(k, m); }

int mxec_rs_parity_matrix(int k, int m, uint8_t* out) {
    return guarded([&] {
        int rc = rs_check(k, m);
        if (rc) return rc;
        if (!out) return set_error(MXEC_E_INVALID_ARG, "null output");
        auto mat = rs_matrix(k, m);
        if (!mat) return set_error(MXEC_E_SINGULAR_MATRIX, "matrix construction failed");
        for (int i = 0; i < m; ++i)
            for (int j = 0; j < k; ++j) out[size_t(i) * k + j] = mat->at(k + i, j);
        return MXEC_OK;
    });
}

int mxec_sha256_batch(mxec_ctx* ctx, const uint8_t* const* bufs, const size_t* lens, size_t n,
                      uint8_t (*out)[32]) {
    return guarded([&] {
        if (n == 0) return MXEC_OK;
        if (!bufs || !lens || !out) return set_error(MXEC_E_INVALID_ARG, "null argument");
        DevScope ds;
        MXEC_TRY(ds.open(ctx, -1));
        Slot& slot = *ds.slot;
        hipStream_t s = slot.stream;
        uint64_t total = 0;
        std::vector<uint64_t> off(n);
        for (size_t i = 0; i < n; ++i) {
            off[i] = total;
            total += round_up(lens[i] ? lens[i] : 1, kSlotAlign);
        }
        MXEC_TRY(slot.shards.ensure(total));
        MXEC_TRY(slot.digests.grow(n * 32));
        auto* base = static_cast<uint8_t*>(slot.shards.p);
        std::vector<const uint8_t*> ptrs(n);
        std::vector<uint64_t> l(n);
        std::vector<UploadSeg> segs;
        segs.reserve(n);
        for (size_t i = 0; i < n; ++i) {
            if (lens[i]) segs.push_back({off[i], bufs[i], lens[i]});
            ptrs[i] = base + off[i];
            l[i] = lens[i];
        }
        MXEC_TRY(upload_segments(slot, s, base, segs, copy_waves_get(*ds.d)));
        MXEC_TRY(slot_wait(slot, s));  // uploads done: the combiner hashes on its own stream
        return sha256_combined(*ds.d, slot, s, ptrs, l, &out[0][0]);
    });
}

int mxec_encode(mxec_ctx* ctx, int k, int m, size_t shard_size, const uint8_t* const* data,
                const size_t* data_len, uint8_t* const* parity, uint8_t (*sha256_out)[32]) {
    return guarded([&] {
        MXEC_TRY(check_km(k, m));
        if (shard_size == 0) return set_error(MXEC_E_EMPTY_SHARD, mxec_strerror(MXEC_E_EMPTY_SHARD));
        if (!data || !parity) return set_error(MXEC_E_INVALID_ARG, "null shard array");
        std::vector<uint64_t> len(static_cast<size_t>(k + m), shard_size);
        for (int j = 0; j < k; ++j) {
            len[size_t(j)] = data_len ? data_len[j] : shard_size;
            if (len[size_t(j)] > shard_size)
                return set_error(MXEC_E_INCORRECT_SHARD_SIZE, "data chunk longer than shard_size");
            if (len[size_t(j)] && !data[j]) return set_error(MXEC_E_INVALID_ARG, "null data chunk");
        }
        DevScope ds;
        MXEC_TRY(ds.open(ctx, -1));
        Slot& slot = *ds.slot;
        hipStream_t s = slot.stream;
        const uint64_t sa = round_up(shard_size, kSlotAlign);
        MXEC_TRY(slot.shards.ensure(sa * uint64_t(k + m)));
        auto* base = static_cast<uint8_t*>(slot.shards.p);
        std::vector<const uint8_t*> in(static_cast<size_t>(k));
        std::vector<uint8_t*> out(static_cast<size_t>(m));
        std::vector<UploadSeg> up;
        for (int j = 0; j < k; ++j) {
            in[size_t(j)] = base + sa * uint64_t(j);
            if (len[size_t(j)]) up.push_back({sa * uint64_t(j), data[j], len[size_t(j)]});
        }
        MXEC_TRY(upload_segments(slot, s, base, up, copy_waves_put(*ds.d)));
        for (int i = 0; i < m; ++i) out[size_t(i)] = base + sa * uint64_t(k + i);
        uint32_t off = 0;
        MXEC_TRY(with_stable_coef(
            *ds.d, s, [&] { return encode_coef(*ds.d, k, m, &off); },
            [&] {
                RsObject ob{in.data(), len.data(), out.data(), len.data() + k, off};
                return run_rs(*ds.d, slot, s, shard_size, k, m, {ob});
            }));
        std::vector<DownloadSeg> down;
        for (int i = 0; i < m; ++i) down.push_back({sa * uint64_t(k + i), parity[i], shard_size});
        MXEC_TRY(download_segments(slot, s, base, down, copy_waves_put(*ds.d)));
        if (sha256_out) {
            // write_chunk / compute_and_write_parity digests (filesystem.rs:1070,
            // :1131), combined with every concurrent caller's verification work.
            std::vector<const uint8_t*> ptrs(in.begin(), in.end());
            for (auto* p : out) ptrs.push_back(p);
            return sha256_combined(*ds.d, slot, s, ptrs, len, &sha256_out[0][0]);
        }
        return MXEC_OK;
    });
}

int mxec_reconstruct(mxec_ctx* ctx, int k, int m, size_t shard_size, uint8_t* const* shards,
                     const size_t* shard_len, const uint8_t (*expected_sha256)[32],
                     uint8_t* present_inout, uint32_t flags, int* n_present) {
    return guarded([&] {
        int rc = rs_check(k, m);
        if (rc) return set_error(rc, std::string("RS init error: ") + mxec_strerror(rc));
        if (shard_size == 0) return set_error(MXEC_E_EMPTY_SHARD, mxec_strerror(MXEC_E_EMPTY_SHARD));
        if (!shards || !present_inout) return set_error(MXEC_E_INVALID_ARG, "null argument");
        const int total = k + m;
        std::vector<uint64_t> len(static_cast<size_t>(total));
        for (int i = 0; i < total; ++i) {
            len[size_t(i)] = shard_len ? std::min<uint64_t>(shard_len[i], shard_size) : shard_size;
            if (!shards[i]) return set_error(MXEC_E_INVALID_ARG, "null shard buffer");
        }
        DevScope ds;
        MXEC_TRY(ds.open(ctx, -1));
        Slot& slot = *ds.slot;
        hipStream_t s = slot.stream;
        const uint64_t sa = round_up(shard_size, kSlotAlign);
        MXEC_TRY(slot.shards.ensure(sa * uint64_t(total) + uint64_t(total) * 64));
        auto* base = static_cast<uint8_t*>(slot.shards.p);
        std::vector<uint8_t> present(present_inout, present_inout + total);
        std::vector<const uint8_t*> sp;
        std::vector<uint64_t> sl;
        std::vector<int> si;
        std::vector<UploadSeg> up;
        for (int i = 0; i < total; ++i) {
            if (!present[size_t(i)]) continue;
            if (len[size_t(i)]) up.push_back({sa * uint64_t(i), shards[i], len[size_t(i)]});
            sp.push_back(base + sa * uint64_t(i));
            sl.push_back(len[size_t(i)]);
            si.push_back(i);
        }
        MXEC_TRY(upload_segments(slot, s, base, up, copy_waves_get(*ds.d)));
        if (expected_sha256 && !sp.empty()) {
            // chunk_reader.rs:176-196: hash every present shard; mismatch -> erasure.
            MXEC_TRY(slot_wait(slot, s));
            std::vector<uint8_t> dig(sp.size() * 32);
            MXEC_TRY(sha256_combined(*ds.d, slot, s, sp, sl, dig.data()));
            for (size_t t = 0; t < si.size(); ++t)
                if (std::memcmp(&dig[t * 32], expected_sha256[si[t]], 32) != 0) present[size_t(si[t])] = 0;
        }
        int np = 0;
        for (int i = 0; i < total; ++i) np += present[size_t(i)] ? 1 : 0;
        if (n_present) *n_present = np;
        if (np < k) return set_error(MXEC_E_TOO_FEW_SHARDS_PRESENT, too_few_msg(np, k, total));
        const bool data_only = (flags & MXEC_F_DATA_ONLY) != 0;
        std::shared_ptr<const DecodePlan> plan;
        uint32_t off = 0;
        std::vector<const uint8_t*> in;
        std::vector<uint64_t> in_len, out_len;
        std::vector<uint8_t*> out;
        auto collect = [&]() -> int {
            MXEC_TRY(decode_plan(*ds.d, k, m, present.data(), data_only, &plan, &off));
            if (!plan) return set_error(MXEC_E_SINGULAR_MATRIX, "decode matrix inversion failed");
            return MXEC_OK;
        };
        auto launch = [&]() -> int {
            if (plan->missing.empty()) return MXEC_OK;
            in.clear();
            in_len.clear();
            out.clear();
            out_len.clear();
            for (int v : plan->valid) {
                in.push_back(base + sa * uint64_t(v));
                in_len.push_back(len[size_t(v)]);
            }
            for (int e : plan->missing) {
                out.push_back(base + sa * uint64_t(e));
                out_len.push_back(len[size_t(e)]);
            }
            RsObject ob{in.data(), in_len.data(), out.data(), out_len.data(), off};
            return run_rs(*ds.d, slot, s, shard_size, k, int(out.size()), {ob});
        };
        MXEC_TRY(with_stable_coef(*ds.d, s, collect, launch));
        if (!plan->missing.empty()) {
            std::vector<DownloadSeg> down;
            for (size_t t = 0; t < out.size(); ++t)
                if (out_len[t]) down.push_back({sa * uint64_t(plan->missing[t]), shards[plan->missing[t]], out_len[t]});
            // plan->missing is ascending, so are the offsets.
            MXEC_TRY(download_segments(slot, s, base, down, copy_waves_get(*ds.d)));
            for (int e : plan->missing) present[size_t(e)] = 1;
        } else {
            // Nothing to rebuild: the uploads may still be reading the
            // caller's buffers (direct DMA from page-locked memory).
            MXEC_TRY(slot_wait(slot, s));
        }
        std::memcpy(present_inout, present.data(), size_t(total));
        return MXEC_OK;
    });
}

int mxec_encode_strided_device(mxec_ctx* ctx, int dev, void* stream, int k, int m,
                               uint64_t shard_size, uint64_t n_obj, const uint8_t* data,
                               uint64_t data_obj_stride, uint64_t data_shard_stride,
                               const uint64_t* data_len, uint8_t* parity,
                               uint64_t parity_obj_stride, uint64_t parity_shard_stride,
                               uint8_t* digests_dev) {
    return guarded([&] {
        MXEC_TRY(check_km(k, m));
        if (shard_size == 0) return set_error(MXEC_E_EMPTY_SHARD, mxec_strerror(MXEC_E_EMPTY_SHARD));
        if (n_obj == 0) return MXEC_OK;
        if (!data || !parity) return set_error(MXEC_E_INVALID_ARG, "null base pointer");
        DevScope ds;
        MXEC_TRY(ds.open(ctx, dev));
        hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the HIP null stream
        uint32_t off = 0;
        std::vector<uint64_t> len(static_cast<size_t>(k + m), shard_size);
        for (int j = 0; j < k; ++j)
            if (data_len) len[size_t(j)] = std::min<uint64_t>(data_len[j], shard_size);
        std::vector<const uint8_t*> in(static_cast<size_t>(n_obj * k));
        std::vector<uint8_t*> out(static_cast<size_t>(n_obj * m));
        std::vector<RsObject> objs(static_cast<size_t>(n_obj));
        for (uint64_t o = 0; o < n_obj; ++o) {
            for (int j = 0; j < k; ++j) in[o * k + j] = data + o * data_obj_stride + j * data_shard_stride;
            for (int i = 0; i < m; ++i) out[o * m + i] = parity + o * parity_obj_stride + i * parity_shard_stride;
            objs[o] = RsObject{&in[o * k], len.data(), &out[o * m], len.data() + k, 0};
        }
        MXEC_TRY(with_stable_coef(
            *ds.d, s, [&] { return encode_coef(*ds.d, k, m, &off); },
            [&] {
                for (auto& ob : objs) ob.coef_off = off;
                return run_rs(*ds.d, *ds.slot, s, shard_size, k, m, objs);
            }));
        if (digests_dev) {
            std::vector<const uint8_t*> ptrs;
            std::vector<uint64_t> lens;
            ptrs.reserve(size_t(n_obj * (k + m)));
            lens.reserve(ptrs.capacity());
            for (uint64_t o = 0; o < n_obj; ++o) {
                for (int j = 0; j < k; ++j) { ptrs.push_back(in[o * k + j]); lens.push_back(len[size_t(j)]); }
                for (int i = 0; i < m; ++i) { ptrs.push_back(out[o * m + i]); lens.push_back(shard_size); }
            }
            MXEC_TRY(run_sha(*ds.d, *ds.slot, s, ptrs, lens, digests_dev, nullptr, nullptr));
        }
        return MXEC_OK;
    });
}

int mxec_encode_batch_device(mxec_ctx* ctx, int dev, void* stream, const mxec_object* objs,
                             uint64_t n_obj, const uint8_t* const* data, const uint64_t* data_len,
                             uint8_t* const* parity, uint8_t* digests_dev) {
    return guarded([&] {
        if (n_obj == 0) return MXEC_OK;
        if (!objs || !data || !parity) return set_error(MXEC_E_INVALID_ARG, "null argument");
        DevScope ds;
        MXEC_TRY(ds.open(ctx, dev));
        hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the HIP null stream
        std::vector<uint64_t> dofs(static_cast<size_t>(n_obj)), pofs(static_cast<size_t>(n_obj));
        uint64_t dsum = 0, psum = 0;
        for (uint64_t o = 0; o < n_obj; ++o) {
            MXEC_TRY(check_km(objs[o].k, objs[o].m));
            if (objs[o].shard_size == 0) return set_error(MXEC_E_EMPTY_SHARD, mxec_strerror(MXEC_E_EMPTY_SHARD));
            dofs[o] = dsum;
            pofs[o] = psum;
            dsum += uint64_t(objs[o].k);
            psum += uint64_t(objs[o].m);
        }
        for (uint64_t i = 0; i < psum; ++i)
            if (!parity[i]) return set_error(MXEC_E_INVALID_ARG, "null parity pointer " + std::to_string(i));
        std::vector<uint64_t> dl(static_cast<size_t>(dsum)), pl(static_cast<size_t>(psum));
        for (uint64_t o = 0; o < n_obj; ++o) {
            for (int j = 0; j < objs[o].k; ++j) {
                const uint64_t idx = dofs[o] + uint64_t(j);
                dl[idx] = data_len ? std::min<uint64_t>(data_len[idx], objs[o].shard_size) : objs[o].shard_size;
            }
            for (int i = 0; i < objs[o].m; ++i) pl[pofs[o] + uint64_t(i)] = objs[o].shard_size;
        }
        for (uint64_t j = 0; j < dsum; ++j)
            if (!data[j] && dl[j]) return set_error(MXEC_E_INVALID_ARG, "null data pointer " + std::to_string(j));
        // One launch per parity count m: objects of every k and shard size
        // share it (run_rs_mixed; unaligned or m > 8: per (k, shard_size)).
        std::map<int, std::vector<RsMixedObject>> groups;
        MXEC_TRY(with_stable_coef(*ds.d, s, [&]() -> int {
            groups.clear();
            std::map<std::pair<int, int>, uint32_t> offs;
            for (uint64_t o = 0; o < n_obj; ++o) {
                const int k = objs[o].k, m = objs[o].m;
                auto it = offs.find({k, m});
                if (it == offs.end()) {
                    uint32_t off = 0;
                    MXEC_TRY(encode_coef(*ds.d, k, m, &off));
                    it = offs.emplace(std::make_pair(k, m), off).first;
                }
                groups[m].push_back(RsMixedObject{k, objs[o].shard_size,
                                                  RsObject{data + dofs[o], &dl[dofs[o]], parity + pofs[o],
                                                           &pl[pofs[o]], it->second}});
            }
            return MXEC_OK;
        }, [&] { return run_rs_mixed(*ds.d, *ds.slot, s, groups); }));
        if (digests_dev) {
            std::vector<const uint8_t*> ptrs;
            std::vector<uint64_t> lens;
            for (uint64_t o = 0; o < n_obj; ++o) {
                for (int j = 0; j < objs[o].k; ++j) { ptrs.push_back(data[dofs[o] + j]); lens.push_back(dl[dofs[o] + j]); }
                for (int i = 0; i < objs[o].m; ++i) { ptrs.push_back(parity[pofs[o] + i]); lens.push_back(objs[o].shard_size); }
            }
            MXEC_TRY(run_sha(*ds.d, *ds.slot, s, ptrs, lens, digests_dev, nullptr, nullptr));
        }
        return MXEC_OK;
    });
}

int mxec_reconstruct_strided_device(mxec_ctx* ctx, int dev, void* stream, int k, int m,
                                    uint64_t shard_size, uint64_t n_obj, uint8_t* shards,
                                    uint64_t obj_stride, uint64_t shard_stride,
                                    const uint64_t* shard_len, uint8_t* present,
                                    const uint8_t* expected_sha_dev, uint32_t flags,
                                    int32_t* status_out) {
    return guarded([&] {
        int rc = rs_check(k, m);
        if (rc) return set_error(rc, std::string("RS init error: ") + mxec_strerror(rc));
        if (shard_size == 0) return set_error(MXEC_E_EMPTY_SHARD, mxec_strerror(MXEC_E_EMPTY_SHARD));
        if (n_obj == 0) return MXEC_OK;
        if (!shards || !present) return set_error(MXEC_E_INVALID_ARG, "null argument");
        const int total = k + m;
        DevScope ds;
        MXEC_TRY(ds.open(ctx, dev));
        Slot& slot = *ds.slot;
        hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the HIP null stream
        std::vector<uint64_t> len(static_cast<size_t>(total));
        for (int i = 0; i < total; ++i)
            len[size_t(i)] = shard_len ? std::min<uint64_t>(shard_len[i], shard_size) : shard_size;
        auto shard_ptr = [&](uint64_t o, int i) { return shards + o * obj_stride + uint64_t(i) * shard_stride; };
        const bool data_only = (flags & MXEC_F_DATA_ONLY) != 0;
        std::vector<int32_t> st(static_cast<size_t>(n_obj), MXEC_OK);
        std::vector<uint8_t*> sp(static_cast<size_t>(n_obj * total));
        std::vector<BatchObj> bo(static_cast<size_t>(n_obj));
        for (uint64_t o = 0; o < n_obj; ++o) {
            for (int i = 0; i < total; ++i) sp[o * total + i] = shard_ptr(o, i);
            bo[o] = BatchObj{k, m, shard_size, &sp[o * total], len.data(), present + o * total};
        }
        // Rebuild `objs` from the present mask as it stands (rebuild_batch).
        auto rebuild = [&](const std::vector<uint64_t>& objs) -> int {
            return rebuild_batch(*ds.d, slot, s, data_only, bo, objs, st);
        };
        std::vector<uint64_t> all(static_cast<size_t>(n_obj));
        for (uint64_t o = 0; o < n_obj; ++o) all[o] = o;
        bool rebuilt = false;
        if (expected_sha_dev) {
            std::vector<const uint8_t*> ptrs;
            std::vector<uint64_t> lens;
            std::vector<uint64_t> idx;
            for (uint64_t o = 0; o < n_obj; ++o)
                for (int i = 0; i < total; ++i)
                    if (present[o * total + i]) {
                        ptrs.push_back(shard_ptr(o, i));
                        lens.push_back(len[size_t(i)]);
                        idx.push_back(o * total + i);
                    }
            if (!ptrs.empty() && !sha_combines(*ds.d, ptrs.size())) {
                // A batch that fills the chip: its own launch on `stream`,
                // digests compared on the device (the verify kernel compares
                // message t against expected[idx[t]]), n flags read back.
                MXEC_TRY(slot.digests.grow(ptrs.size()));
                auto* ok = static_cast<uint8_t*>(slot.digests.p);
                const uint32_t* tmo = nullptr;
                MXEC_TRY(run_sha(*ds.d, slot, s, ptrs, lens, nullptr, expected_sha_dev, ok, &idx, nullptr, 0, &tmo));
                const size_t fo = (ptrs.size() + 15) & ~size_t(15);
                MXEC_TRY(slot.hdig.grow(fo + 16));
                auto* hflag = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(slot.hdig.p) + fo);
                *hflag = 0;
                MXEC_HIP(hipMemcpyAsync(slot.hdig.p, ok, ptrs.size(), hipMemcpyDeviceToHost, s));
                if (tmo) MXEC_HIP(hipMemcpyAsync(hflag, tmo, 4, hipMemcpyDeviceToHost, s));
                MXEC_TRY(slot_wait(*ds.slot, s));
                if (*hflag != 0)
                    return set_error(MXEC_E_DEVICE, "SHA-256 stream kernel: a wave timed out waiting for its predecessor segment");
                const auto* okh = static_cast<const uint8_t*>(slot.hdig.p);
                for (size_t t = 0; t < idx.size(); ++t)
                    if (!okh[t]) present[idx[t]] = 0;
            } else if (!ptrs.empty()) {
                // A small batch: hashed by the device's combiner together with
                // every concurrent caller's verification (combiner.cpp), once
                // the work queued on `stream` has produced the shards; digests
                // compared on the host.  The combined launch waits for that
                // work on the device (an event recorded here), not the host.
                //
                // Speculative rebuild: the decode from the present mask as
                // given is queued right behind that event, so it runs beside
                // the hash instead of after it (the hash is a VALU-bound
                // chain, the decode an HBM stream).  It reads only present
                // shards and writes only missing ones, which the hash does not
                // read.  Objects whose digests all match keep it -- exactly
                // what verify-then-rebuild produces; an object with a
                // mismatch is rebuilt again from its original mask minus the
                // mismatched shards, over the same output shards, in stream
                // order (chunk_reader.rs:176-211 semantics).  An object that
                // ends up short of k shards may have its missing shards
                // overwritten by the speculative decode.
                const size_t ne = size_t(n_obj) * size_t(total) * 32;
                MXEC_TRY(slot.hdig.grow(ne));
                MXEC_HIP(hipMemcpyAsync(slot.hdig.p, expected_sha_dev, ne, hipMemcpyDeviceToHost, s));
                if (!slot.ready_ev) MXEC_HIP(hipEventCreateWithFlags(&slot.ready_ev, hipEventDisableTiming));
                MXEC_HIP(hipEventRecord(slot.ready_ev, s));
                const std::vector<uint8_t> orig(present, present + n_obj * uint64_t(total));
                // Queued by the combiner's leader right after the hash launch,
                // so the host work of the plans does not hold back the hash
                // (or this caller's arrival with it).
                const std::function<int()> spec = [&] { return rebuild(all); };
                rebuilt = true;
                std::vector<uint8_t> dig(ptrs.size() * 32);
                if (int hrc = sha256_combined(*ds.d, slot, s, ptrs, lens, dig.data(), slot.ready_ev, &spec)) {
                    // No verdict: the mask goes back as it came (the speculative
                    // rebuild may already have marked shards present).
                    const std::string msg = last_error();
                    std::memcpy(present, orig.data(), orig.size());
                    (void)slot_wait(*ds.slot, s);  // the speculative decode, if queued
                    return set_error(hrc, msg);
                }
                MXEC_TRY(slot_wait(*ds.slot, s));  // the digest copy (long done), the speculative decode
                const auto* exph = static_cast<const uint8_t*>(slot.hdig.p);
                std::vector<uint64_t> redo;
                for (size_t t = 0; t < idx.size(); ++t) {
                    if (std::memcmp(&dig[t * 32], exph + idx[t] * 32, 32) == 0) continue;
                    const uint64_t o = idx[t] / uint64_t(total);
                    if (redo.empty() || redo.back() != o) {
                        redo.push_back(o);  // idx ascends: objects arrive in order
                        std::memcpy(present + o * total, &orig[o * total], size_t(total));
                    }
                }
                for (size_t t = 0; t < idx.size(); ++t)
                    if (std::memcmp(&dig[t * 32], exph + idx[t] * 32, 32) != 0) present[idx[t]] = 0;
                MXEC_TRY(rebuild(redo));
            }
        }
        if (!rebuilt) MXEC_TRY(rebuild(all));
        int first_err = MXEC_OK;
        for (uint64_t o = 0; o < n_obj; ++o) {
            if (status_out) status_out[o] = st[o];
            if (st[o] != MXEC_OK && first_err == MXEC_OK) {
                int np = 0;
                for (int i = 0; i < total; ++i) np += present[o * total + i] != 0;
                first_err = st[o];
                set_error(first_err, too_few_msg(np, k, total));
            }
        }
        return first_err;
    });
}

int mxec_reconstruct_batch_device(mxec_ctx* ctx, int dev, void* stream, const mxec_object* objs,
                                  uint64_t n_obj, uint8_t* const* shards, const uint64_t* shard_len,
                                  uint8_t* present, const uint8_t* expected_sha_dev, uint32_t flags,
                                  int32_t* status_out) {
    return guarded([&] {
        if (n_obj == 0) return MXEC_OK;
        if (!objs || !shards || !present) return set_error(MXEC_E_INVALID_ARG, "null argument");
        std::vector<uint64_t> first(static_cast<size_t>(n_obj));
        uint64_t sum = 0;
        for (uint64_t o = 0; o < n_obj; ++o) {
            if (int rc = rs_check(objs[o].k, objs[o].m))
                return set_error(rc, std::string("RS init error: ") + mxec_strerror(rc));
            if (objs[o].shard_size == 0) return set_error(MXEC_E_EMPTY_SHARD, mxec_strerror(MXEC_E_EMPTY_SHARD));
            first[o] = sum;
            sum += uint64_t(objs[o].k + objs[o].m);
        }
        DevScope ds;
        MXEC_TRY(ds.open(ctx, dev));
        Slot& slot = *ds.slot;
        hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the HIP null stream
        // Every shard pointer is needed: present ones are read, missing ones
        // are where the rebuilt bytes go (a NULL would fault the device).
        for (uint64_t g = 0; g < sum; ++g)
            if (!shards[g]) return set_error(MXEC_E_INVALID_ARG, "null shard pointer " + std::to_string(g));
        std::vector<uint64_t> len(static_cast<size_t>(sum));
        std::vector<BatchObj> bo(static_cast<size_t>(n_obj));
        for (uint64_t o = 0; o < n_obj; ++o) {
            const uint64_t S = objs[o].shard_size;
            for (int i = 0; i < objs[o].k + objs[o].m; ++i) {
                const uint64_t g = first[o] + uint64_t(i);
                len[g] = shard_len ? std::min<uint64_t>(shard_len[g], S) : S;
            }
            bo[o] = BatchObj{objs[o].k, objs[o].m, S, shards + first[o], &len[first[o]], present + first[o]};
        }
        if (expected_sha_dev) {
            // Verify every present shard in one launch on `stream` (digests
            // compared on the device against expected[global shard index]),
            // read the flags back; a mismatch is an erasure
            // (chunk_reader.rs:176-196).
            std::vector<const uint8_t*> ptrs;
            std::vector<uint64_t> lens, idx;
            for (uint64_t g = 0; g < sum; ++g)
                if (present[g]) {
                    ptrs.push_back(shards[g]);
                    lens.push_back(len[g]);
                    idx.push_back(g);
                }
            if (!ptrs.empty()) {
                MXEC_TRY(slot.digests.grow(ptrs.size()));
                auto* ok = static_cast<uint8_t*>(slot.digests.p);
                const uint32_t* tmo = nullptr;
                MXEC_TRY(run_sha(*ds.d, slot, s, ptrs, lens, nullptr, expected_sha_dev, ok, &idx, nullptr, 0, &tmo));
                const size_t fo = (ptrs.size() + 15) & ~size_t(15);
                MXEC_TRY(slot.hdig.grow(fo + 16));
                auto* hflag = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(slot.hdig.p) + fo);
                *hflag = 0;
                MXEC_HIP(hipMemcpyAsync(slot.hdig.p, ok, ptrs.size(), hipMemcpyDeviceToHost, s));
                if (tmo) MXEC_HIP(hipMemcpyAsync(hflag, tmo, 4, hipMemcpyDeviceToHost, s));
                MXEC_TRY(slot_wait(slot, s));
                if (*hflag != 0)
                    return set_error(MXEC_E_DEVICE, "SHA-256 stream kernel: a wave timed out waiting for its predecessor segment");
                const auto* okh = static_cast<const uint8_t*>(slot.hdig.p);
                for (size_t t = 0; t < idx.size(); ++t)
                    if (!okh[t]) present[idx[t]] = 0;
            }
        }
        std::vector<int32_t> st(static_cast<size_t>(n_obj), MXEC_OK);
        std::vector<uint64_t> all(static_cast<size_t>(n_obj));
        for (uint64_t o = 0; o < n_obj; ++o) all[o] = o;
        MXEC_TRY(rebuild_batch(*ds.d, slot, s, (flags & MXEC_F_DATA_ONLY) != 0, bo, all, st));
        int first_err = MXEC_OK;
        for (uint64_t o = 0; o < n_obj; ++o) {
            if (status_out) status_out[o] = st[o];
            if (st[o] != MXEC_OK && first_err == MXEC_OK) {
                const int total = objs[o].k + objs[o].m;
                int np = 0;
                for (int i = 0; i < total; ++i) np += present[first[o] + uint64_t(i)] != 0;
                first_err = st[o];
                set_error(first_err, too_few_msg(np, objs[o].k, total));
            }
        }
        return first_err;
    });
}

int mxec_sha256_batch_device(mxec_ctx* ctx, int dev, void* stream, const uint8_t* const* bufs,
                             const uint64_t* lens, uint64_t n, uint8_t* digests_dev) {
    return guarded([&] {
        if (n == 0) return MXEC_OK;
        if (!bufs || !lens || !digests_dev) return set_error(MXEC_E_INVALID_ARG, "null argument");
        for (uint64_t i = 0; i < n; ++i)
            if (!bufs[i]) return set_error(MXEC_E_INVALID_ARG, "null message pointer " + std::to_string(i));
        DevScope ds;
        MXEC_TRY(ds.open(ctx, dev));
        hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the HIP null stream
        std::vector<const uint8_t*> p(bufs, bufs + n);
        std::vector<uint64_t> l(lens, lens + n);
        return run_sha(*ds.d, *ds.slot, s, p, l, digests_dev, nullptr, nullptr);
    });
}

}  // extern "C"
