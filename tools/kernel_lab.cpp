// kernel_lab.cpp — measurement harness for the RS kernel on one MI355X.
//
// Calibrates the HBM ceiling with plain streaming kernels (copy, read-only,
// write-only, and the RS access pattern with the GF math removed: read k
// shards, write m shards) and sweeps the interior RS kernel's knobs
// (RsVariant) on the BASELINE shapes.  Development tool, not product; prints
// one JSON object per measurement.
//
//   make -C tools && tools/kernel_lab [n_obj_cfg2]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../maxio_amd/csrc/gf256.hpp"
#include "../maxio_amd/csrc/kernels.hpp"

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) d[i] = s[i];
}
__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
    u32x4 acc = {0, 0, 0, 0};
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) acc ^= s[i];
    if (acc.x == 0x12345678u) d[0] = acc;  // keep the loads alive
}
__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ d, uint64_t n) {
    const u32x4 v = {1, 2, 3, 4};
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) d[i] = v;
}
// Read ceilings by load form: four independent nontemporal 16-byte loads per
// lane per step, and LDS-DMA (global_load_lds_dwordx4, 16 KiB per wave in
// flight; AUX 2 = nontemporal).
__global__ __launch_bounds__(256) void k_read_nt4(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
    u32x4 acc = {0, 0, 0, 0};
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i + 3 * stride < n; i += 4 * stride) {
        const u32x4 a = __builtin_nontemporal_load(s + i), b = __builtin_nontemporal_load(s + i + stride);
        const u32x4 c = __builtin_nontemporal_load(s + i + 2 * stride), e = __builtin_nontemporal_load(s + i + 3 * stride);
        acc ^= a ^ b ^ c ^ e;
    }
    if (acc.x == 0x12345678u) d[0] = acc;
}
template <int AUX>
__global__ __launch_bounds__(256) void k_read_glds(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
    __shared__ u32x4 buf[4][16][64];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t chunks = n / 1024, nw = uint64_t(gridDim.x) * 4;
    for (uint64_t c = blockIdx.x * 4ull + wave; c < chunks; c += nw) {
        const u32x4* src = s + c * 1024 + lane;
#pragma unroll
        for (int q = 0; q < 16; ++q)
            __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(src + q * 64),
                                             (void __attribute__((address_space(3)))*)&buf[wave][q][0], 16, 0, AUX);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (d && buf[wave][0][lane].x == 0x12345678u) d[0] = buf[wave][1][lane];
}
__global__ __launch_bounds__(256) void k_write_nt(u32x4* __restrict__ d, uint64_t n) {
    const u32x4 v = {1, 2, 3, 4};
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256)
        __builtin_nontemporal_store(v, d + i);
}
// Copy with four independent nontemporal 16-byte loads in flight per lane.
__global__ __launch_bounds__(256) void k_copy_nt4(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i + 3 * stride < n; i += 4 * stride) {
        const u32x4 a = __builtin_nontemporal_load(s + i), b = __builtin_nontemporal_load(s + i + stride);
        const u32x4 c = __builtin_nontemporal_load(s + i + 2 * stride), e = __builtin_nontemporal_load(s + i + 3 * stride);
        __builtin_nontemporal_store(a, d + i);
        __builtin_nontemporal_store(b, d + i + stride);
        __builtin_nontemporal_store(c, d + i + 2 * stride);
        __builtin_nontemporal_store(e, d + i + 3 * stride);
    }
}
// The RS fast kernel's exact access pattern without the GF math: tile =
// 256 lanes x 16 B x 4 vectors of every shard, 4 inputs x 4 vectors of
// nontemporal loads in flight, XOR, then 2 outputs x 4 vectors of nt stores.
__global__ __launch_bounds__(256) void k_pattern_tile(const uint8_t* __restrict__ data, uint8_t* __restrict__ par,
                                                      uint64_t S, uint64_t n_obj) {
    constexpr uint64_t kTile = 256 * 16 * 4;
    const uint64_t tpo = S / kTile, n_tiles = tpo * n_obj;
    for (uint64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        const uint64_t o = t / tpo, base = (t - o * tpo) * kTile + threadIdx.x * 16;
        u32x4 x[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int v = 0; v < 4; ++v)
                x[j][v] = __builtin_nontemporal_load(
                    reinterpret_cast<const u32x4*>(data + (o * 4 + j) * S + base + v * 4096));
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const u32x4 p = x[0][v] ^ x[1][v] ^ x[2][v] ^ x[3][v];
            __builtin_nontemporal_store(p, reinterpret_cast<u32x4*>(par + (o * 2) * S + base + v * 4096));
            __builtin_nontemporal_store(p + 1u, reinterpret_cast<u32x4*>(par + (o * 2 + 1) * S + base + v * 4096));
        }
    }
}
// The same 4-read : 2-write pattern with the reads as LDS-DMA (nontemporal
// policy) into a per-wave D-stage ring.  A wave owns a contiguous run of
// `run` 1-KiB column blocks of one object (pointers stay in SGPRs); each
// iteration issues the 4 loads of block t+D-1, waits for block t with the
// constant count vmcnt(6(D-1)) (every iteration issues 4 loads + 2 stores and
// the counter retires in issue order), XORs it out of LDS and stores.
template <int D>
__global__ __launch_bounds__(64) void k_pattern_glds(const uint8_t* __restrict__ data, uint8_t* __restrict__ par,
                                                     uint64_t S, uint64_t n_obj, uint32_t run) {
    __shared__ u32x4 ring[D][4][64];
    const uint32_t lane = threadIdx.x;
    const uint64_t bpo = S / 1024, runs_per_obj = bpo / run, n_runs = runs_per_obj * n_obj;
    for (uint64_t r = blockIdx.x; r < n_runs; r += gridDim.x) {
        const uint64_t o = r / runs_per_obj, b0 = (r - o * runs_per_obj) * run;
        const uint8_t* in0 = data + (o * 4) * S + lane * 16;
        uint8_t* out0 = par + (o * 2) * S + lane * 16;
        auto issue = [&](uint64_t b, int slot) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_global_load_lds(
                    (const void __attribute__((address_space(1)))*)(in0 + j * S + b * 1024),
                    (void __attribute__((address_space(3)))*)&ring[slot][j][0], 16, 0, 2);
        };
#pragma unroll
        for (int d = 0; d < D - 1; ++d) issue(b0 + d, d);
        for (uint32_t t = 0; t < run; ++t) {
            const uint64_t b = b0 + t;
            if (t + D - 1 < run) {
                issue(b + D - 1, int((t + D - 1) % D));
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * (D - 1)) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const int slot = int(t % D);
            const u32x4 p = ring[slot][0][lane] ^ ring[slot][1][lane] ^ ring[slot][2][lane] ^ ring[slot][3][lane];
            __builtin_nontemporal_store(p, reinterpret_cast<u32x4*>(out0 + b * 1024));
            __builtin_nontemporal_store(p + 1u, reinterpret_cast<u32x4*>(out0 + S + b * 1024));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}
// RS access pattern without the math: object o, 16-B column c: read k shards,
// write m shards (XOR of inputs), same layout as the bench.
__global__ __launch_bounds__(256) void k_pattern(const uint8_t* __restrict__ data, uint8_t* __restrict__ par,
                                                 uint32_t k, uint32_t m, uint64_t S, uint64_t n_obj) {
    const uint64_t vec_per_shard = S / 16;
    const uint64_t total = n_obj * vec_per_shard;
    for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < total; t += uint64_t(gridDim.x) * 256) {
        const uint64_t o = t / vec_per_shard, c = t - o * vec_per_shard;
        u32x4 acc = {0, 0, 0, 0};
        for (uint32_t j = 0; j < k; ++j) acc ^= reinterpret_cast<const u32x4*>(data + (o * k + j) * S)[c];
        for (uint32_t i = 0; i < m; ++i) reinterpret_cast<u32x4*>(par + (o * m + i) * S)[c] = acc + i;
    }
}

__global__ __launch_bounds__(256) void k_diff(const u32x4* __restrict__ a, const u32x4* __restrict__ b, uint64_t n,
                                             unsigned long long* bad) {
    unsigned long long c = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) {
        const u32x4 x = a[i] ^ b[i];
        c += (x.x | x.y | x.z | x.w) != 0;
    }
    if (c) atomicAdd(bad, c);
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    template <class F>
    double median_ms(F f, int reps = 7) {
        f();
        CK(hipDeviceSynchronize());
        std::vector<double> t;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(a, 0));
            f();
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        return t[t.size() / 2];
    }
};

struct Shape {
    int k, r;
    uint64_t S, n;
};

// Device descriptors for a strided batch: in = data shard j of object o,
// out = parity i of object o.
struct Batch {
    mxec::RsArgs a{};
    void* mem = nullptr;
    Batch(const uint8_t* data, uint8_t* par, Shape sh, const std::vector<uint32_t>& table, uint32_t** coef_dev) {
        std::vector<const uint8_t*> ip(sh.n * sh.k);
        std::vector<uint8_t*> op(sh.n * sh.r);
        std::vector<uint64_t> il(sh.n * sh.k, sh.S), ol(sh.n * sh.r, sh.S);
        std::vector<uint32_t> co(sh.n, 0);
        // MXEC_LAB_OM=1: the bench's object-major layout ([n][k+r][S + pad],
        // pad 2 MiB + 64 KiB for multi-MiB shards) from `data`; else data
        // [n][k][S] and parity [n][r][S] apart.
        const bool om = getenv("MXEC_LAB_OM") != nullptr;
        const uint64_t ss = sh.S + (sh.S >= (4u << 20) ? (2u << 20) + (64u << 10) : 0);
        for (uint64_t o = 0; o < sh.n; ++o) {
            for (int j = 0; j < sh.k; ++j)
                ip[o * sh.k + j] = om ? data + (o * (sh.k + sh.r) + j) * ss : data + (o * sh.k + j) * sh.S;
            for (int i = 0; i < sh.r; ++i)
                op[o * sh.r + i] = om ? const_cast<uint8_t*>(data) + (o * (sh.k + sh.r) + sh.k + i) * ss
                                      : par + (o * sh.r + i) * sh.S;
        }
        size_t bytes = ip.size() * 8 + op.size() * 8 + il.size() * 8 + ol.size() * 8 + co.size() * 4 + 64;
        CK(hipMalloc(&mem, bytes));
        char* p = static_cast<char*>(mem);
        auto put = [&](const void* src, size_t n) { CK(hipMemcpy(p, src, n, hipMemcpyHostToDevice)); char* r = p; p += (n + 15) & ~size_t(15); return r; };
        a.in_ptrs = reinterpret_cast<const uint8_t* const*>(put(ip.data(), ip.size() * 8));
        a.out_ptrs = reinterpret_cast<uint8_t* const*>(put(op.data(), op.size() * 8));
        a.in_len = reinterpret_cast<const uint64_t*>(put(il.data(), il.size() * 8));
        a.out_len = reinterpret_cast<const uint64_t*>(put(ol.data(), ol.size() * 8));
        a.coef_off = reinterpret_cast<const uint32_t*>(put(co.data(), co.size() * 4));
        CK(hipMalloc(coef_dev, table.size() * 4));
        CK(hipMemcpy(*coef_dev, table.data(), table.size() * 4, hipMemcpyHostToDevice));
        a.coef = *coef_dev;
        a.shard_size = sh.S;
        a.n_edge = 0;
        a.n_obj = uint32_t(sh.n);
        a.k = uint32_t(sh.k);
        a.r = uint32_t(sh.r);
        a.r_total = uint32_t(sh.r);
        a.row0 = 0;
        a.aligned = 1;
    }
    ~Batch() { (void)hipFree(mem); }
};

int main(int argc, char** argv) {
    const uint64_t n2 = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1024;
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    Timer tm;
    // One pool for everything: config 2 at n2 objects = n2 * 60 MiB.
    const uint64_t S2 = 10ull << 20;
    // (object-major mode: 10 MiB shards padded by 2 MiB + 64 KiB)
    const uint64_t pool = n2 * 6 * (getenv("MXEC_LAB_OM") ? S2 + (2u << 20) + (64u << 10) : S2);
    uint8_t* buf;
    CK(hipMalloc(&buf, pool));
    CK(hipMemset(buf, 0x5A, pool));
    // random-ish data (the RS math does not branch on data; DVFS might)
    hipLaunchKernelGGL(k_write, dim3(cus * 8), dim3(256), 0, 0, reinterpret_cast<u32x4*>(buf), pool / 16);
    CK(hipDeviceSynchronize());

    auto report = [](const char* what, const char* shape, double ms, double bytes) {
        std::printf("{\"what\": \"%s\", \"shape\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", what, shape, ms,
                    bytes / (ms * 1e-3) / 1e9);
        std::fflush(stdout);
    };

    // `kernel_lab N sha` runs the SHA-256 section only; `kernel_lab N hbm`
    // the load-form ceilings, the tile-order sweep and the SHA split form.
    const bool sha_only = argc > 2 && !std::strcmp(argv[2], "sha");
    const bool sha_big = argc > 2 && !std::strcmp(argv[2], "shabig");
    const bool hbm_only = argc > 2 && !std::strcmp(argv[2], "hbm");
    // `kernel_lab N ns`: every geometry of the north-star shape (k=8 m=4, 1 MiB)
    // against the 2:1 no-math pattern, two rounds.
    const bool ns_only = argc > 2 && !std::strcmp(argv[2], "ns");
    // ---- calibration ----
    if (hbm_only) {
        const uint64_t nvec = pool / 16, half = pool / 2 / 16;
        auto* s = reinterpret_cast<const u32x4*>(buf);
        auto* d = reinterpret_cast<u32x4*>(buf + pool / 2);
        for (int rep = 0; rep < 2; ++rep) {
            for (int bpc : {8, 16}) {
                char nm[64];
                std::snprintf(nm, sizeof nm, "read_bpc%d", bpc);
                double ms = tm.median_ms([&] { hipLaunchKernelGGL(k_read, dim3(cus * bpc), dim3(256), 0, 0, s, d, nvec); });
                report(nm, "pool", ms, 16.0 * nvec);
                std::snprintf(nm, sizeof nm, "read_nt4_bpc%d", bpc);
                ms = tm.median_ms([&] { hipLaunchKernelGGL(k_read_nt4, dim3(cus * bpc), dim3(256), 0, 0, s, d, nvec); });
                report(nm, "pool", ms, 16.0 * nvec);
            }
            for (int bpc : {2, 4}) {
                char nm[64];
                std::snprintf(nm, sizeof nm, "read_glds_bpc%d", bpc);
                double ms = tm.median_ms([&] { hipLaunchKernelGGL(k_read_glds<0>, dim3(cus * bpc), dim3(256), 0, 0, s, d, nvec); });
                report(nm, "pool", ms, 16.0 * nvec);
                std::snprintf(nm, sizeof nm, "read_glds_nt_bpc%d", bpc);
                ms = tm.median_ms([&] { hipLaunchKernelGGL(k_read_glds<2>, dim3(cus * bpc), dim3(256), 0, 0, s, d, nvec); });
                report(nm, "pool", ms, 16.0 * nvec);
            }
            for (int wpc : {8, 16, 32}) {
                for (uint32_t run : {16u, 64u}) {
                    char nm[96];
                    std::snprintf(nm, sizeof nm, "pattern_glds_d3_wpc%d_run%u", wpc, run);
                    double ms = tm.median_ms([&] { hipLaunchKernelGGL(k_pattern_glds<3>, dim3(cus * wpc), dim3(64), 0, 0, buf, buf + n2 * 4 * S2, S2, n2, run); });
                    report(nm, "k4m2 S10MiB", ms, double(n2) * 6 * S2);
                    std::snprintf(nm, sizeof nm, "pattern_glds_d5_wpc%d_run%u", wpc, run);
                    ms = tm.median_ms([&] { hipLaunchKernelGGL(k_pattern_glds<5>, dim3(cus * wpc), dim3(64), 0, 0, buf, buf + n2 * 4 * S2, S2, n2, run); });
                    report(nm, "k4m2 S10MiB", ms, double(n2) * 6 * S2);
                }
            }
            for (int bpc : {8, 16, 32}) {
                char nm[64];
                std::snprintf(nm, sizeof nm, "copy_nt4_bpc%d", bpc);
                double ms = tm.median_ms([&] { hipLaunchKernelGGL(k_copy_nt4, dim3(cus * bpc), dim3(256), 0, 0, s, d, half); });
                report(nm, "2x half pool", ms, 32.0 * half);
                std::snprintf(nm, sizeof nm, "pattern_tile_4r2w_bpc%d", bpc);
                ms = tm.median_ms([&] { hipLaunchKernelGGL(k_pattern_tile, dim3(cus * bpc), dim3(256), 0, 0, buf, buf + n2 * 4 * S2, S2, n2); });
                report(nm, "k4m2 S10MiB", ms, double(n2) * 6 * S2);
            }
            double ms = tm.median_ms([&] { hipLaunchKernelGGL(k_write, dim3(cus * 8), dim3(256), 0, 0, d, half); });
            report("write", "half pool", ms, 16.0 * half);
            ms = tm.median_ms([&] { hipLaunchKernelGGL(k_write_nt, dim3(cus * 8), dim3(256), 0, 0, d, half); });
            report("write_nt", "half pool", ms, 16.0 * half);
            ms = tm.median_ms([&] { hipLaunchKernelGGL(k_copy, dim3(cus * 16), dim3(256), 0, 0, s, d, half); });
            report("copy_bpc16", "2x half pool", ms, 32.0 * half);
        }
    }
    if (!sha_only && !hbm_only && !sha_big) {
        const uint64_t half = pool / 2 / 16;
        auto* s = reinterpret_cast<const u32x4*>(buf);
        auto* d = reinterpret_cast<u32x4*>(buf + pool / 2);
        for (int bpc : {4, 8, 16}) {
            char nm[64];
            std::snprintf(nm, sizeof nm, "copy_bpc%d", bpc);
            double ms = tm.median_ms([&] { hipLaunchKernelGGL(k_copy, dim3(cus * bpc), dim3(256), 0, 0, s, d, half); });
            report(nm, "2x half pool", ms, 2.0 * half * 16);
        }
        double ms = tm.median_ms([&] { hipLaunchKernelGGL(k_read, dim3(cus * 8), dim3(256), 0, 0, s, d, half * 2); });
        report("read", "pool", ms, 2.0 * half * 16);
        ms = tm.median_ms([&] { hipLaunchKernelGGL(k_write, dim3(cus * 8), dim3(256), 0, 0, d, half); });
        report("write", "half pool", ms, 1.0 * half * 16);
        ms = tm.median_ms([&] { hipLaunchKernelGGL(k_pattern, dim3(cus * 8), dim3(256), 0, 0, buf, buf + n2 * 4 * S2, 4u, 2u, S2, n2); });
        report("pattern_4r2w", "k4m2 S10MiB", ms, double(n2) * 6 * S2);
    }

    // ---- RS variants ----
    auto sweep = [&](Shape sh, const char* name, bool full) {
        auto mat = mxec::rs_matrix(sh.k, sh.r);
        mxec::GfMatrix rows(sh.r, sh.k);
        for (int i = 0; i < sh.r; ++i)
            for (int j = 0; j < sh.k; ++j) rows.at(i, j) = mat->at(sh.k + i, j);
        uint32_t* coef = nullptr;
        Batch b(buf, buf + sh.n * sh.k * sh.S, sh, mxec::coef_tables(rows), &coef);
        const double bytes = double(sh.n) * (sh.k + sh.r) * sh.S;
        std::vector<mxec::RsVariant> vs;
        if (hbm_only) {
            // (An LDS-DMA ring form of this kernel and a contiguous-run tile
            // order were measured here and dropped: profiles/r1_lab_rs_glds_variants.jsonl,
            // profiles/r1_lab_hbm_ceilings_tile_order.jsonl.)
            for (int bpc : {8, 16, 32}) vs.push_back(mxec::RsVariant{4, true, bpc});
        } else if (ns_only) {
            // V = 4: workgroups per CU of grid-stride, alternating, three
            // rounds; MXEC_LAB_MW=3 adds the R = 4 kernel compiled for 3
            // waves per SIMD (164 VGPRs against 173: measured 1.2-1.6 %
            // slower, profiles/r2_lab_ns_occupancy.jsonl)
            const bool mw = getenv("MXEC_LAB_MW") != nullptr;
            for (int rep = 0; rep < 3; ++rep)
                for (int bpc : {512, 1024}) {
                    vs.push_back(mxec::RsVariant{4, true, bpc, 0});
                    vs.push_back(mxec::RsVariant{2, true, bpc, 0});
                    if (mw) vs.push_back(mxec::RsVariant{4, true, bpc, 3});
                }
        } else if (full) {
            for (int v : {1, 2, 4})
                for (bool nt : {false, true})
                    for (int bpc : {4, 8, 16}) vs.push_back(mxec::RsVariant{v, nt, bpc});
        } else {
            for (int v : {1, 2, 4})
                for (bool nt : {false, true}) vs.push_back(mxec::RsVariant{v, nt, 8});
        }
        // Reference output of the default register kernel, for a bit-exact
        // check of every variant (hbm mode).
        uint8_t* par = buf + sh.n * sh.k * sh.S;
        const uint64_t par_bytes = sh.n * sh.r * sh.S;
        uint8_t* ref = nullptr;
        unsigned long long* bad = nullptr;
        const bool check = (hbm_only || ns_only) && !getenv("MXEC_LAB_OM");  // OM: parity is inside the data
        if (check) {
            CK(hipMalloc(&ref, par_bytes));
            CK(hipMalloc(&bad, 8));
            CK(mxec::launch_rs_apply_variant(b.a, cus, 0, mxec::RsVariant{4, true, 16}));
            CK(hipMemcpy(ref, par, par_bytes, hipMemcpyDeviceToDevice));
        }
        for (const auto& v : vs) {
            if (check) {
                CK(hipMemset(par, 0, par_bytes));
                CK(mxec::launch_rs_apply_variant(b.a, cus, 0, v));
                CK(hipMemset(bad, 0, 8));
                hipLaunchKernelGGL(k_diff, dim3(cus * 8), dim3(256), 0, 0, reinterpret_cast<const u32x4*>(par),
                                   reinterpret_cast<const u32x4*>(ref), par_bytes / 16, bad);
                unsigned long long nb = 0;
                CK(hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost));
                std::printf("{\"what\": \"check\", \"v\": %d, \"bpc\": %d, \"min_waves\": %d, \"bad16\": %llu}\n",
                            v.vecs, v.blocks_per_cu, v.min_waves, nb);
            }
            double ms = tm.median_ms([&] { CK(mxec::launch_rs_apply_variant(b.a, cus, 0, v)); });
            char nm[96];
            std::snprintf(nm, sizeof nm, "rs_v%d_nt%d_bpc%d_mw%d", v.vecs, int(v.nt), v.blocks_per_cu, v.min_waves);
            report(nm, name, ms, bytes);
        }
        (void)hipFree(coef);
        if (ref) (void)hipFree(ref);
        if (bad) (void)hipFree(bad);
    };
    // ---- SHA-256: one lane per message ----
    auto sha = [&](uint64_t n, uint64_t L, const char* name, int force = 0) {
        std::vector<const uint8_t*> ptrs(n);
        std::vector<uint64_t> lens(n, L);
        for (uint64_t i = 0; i < n; ++i) ptrs[i] = buf + i * L;
        void* d;
        CK(hipMalloc(&d, n * 8 * 2 + n * 32));
        CK(hipMemcpy(d, ptrs.data(), n * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(static_cast<char*>(d) + n * 8, lens.data(), n * 8, hipMemcpyHostToDevice));
        mxec::ShaArgs sa{};
        sa.ptrs = static_cast<const uint8_t* const*>(d);
        sa.lens = reinterpret_cast<const uint64_t*>(static_cast<char*>(d) + n * 8);
        sa.digests = static_cast<uint8_t*>(d) + n * 16;
        sa.n = uint32_t(n);
        sa.force = force;
        double ms = tm.median_ms([&] { CK(mxec::launch_sha256(sa, 0)); }, 3);
        report("sha256", name, ms, double(n) * L);
        std::printf("{\"what\": \"sha256_us_per_block\", \"shape\": \"%s\", \"us\": %.3f}\n", name,
                    ms * 1e3 / (L / 64.0));
        CK(hipFree(d));
    };
    if (sha_big) {
        // Many 1 MiB messages (combined GET verification): forms by batch size.
        for (uint64_t n : {16384ull, 49152ull, 65536ull, 81920ull}) {
            char nm[96];
            std::snprintf(nm, sizeof nm, "%llu x 1 MiB split form", (unsigned long long)n);
            sha(n, 1ull << 20, nm, 2);
            std::snprintf(nm, sizeof nm, "%llu x 1 MiB one-wave form", (unsigned long long)n);
            sha(n, 1ull << 20, nm, 1);
        }
        CK(hipFree(buf));
        return 0;
    }
    if (ns_only) {
        sweep(Shape{8, 4, 1ull << 20, n2 * 60 / 12}, "k8m4 S1MiB (north star)", true);
        sweep(Shape{4, 2, S2, n2}, "k4m2 S10MiB (cfg2)", true);
        sweep(Shape{10, 4, 1ull << 20, n2 * 60 / 14}, "k10m4 S1MiB (cfg4)", true);
        sweep(Shape{8, 2, 1ull << 20, 1024}, "k8r2 S1MiB x1024 (cfg3 decode)", true);
        CK(hipFree(buf));
        return 0;
    }
    if (hbm_only) {
        sweep(Shape{4, 2, S2, n2}, "k4m2 S10MiB (cfg2)", true);
        sweep(Shape{8, 4, 1ull << 20, n2 * 60 / 12}, "k8m4 S1MiB (north star)", true);
        sha(10240, 1ull << 20, "10240 x 1 MiB split form", 2);
        // (32 and 16 messages per wave of the split form measured 2.70 / 2.76
        // us per block against 1.82: profiles/r1_lab_sha_lanes_per_wave.jsonl.)
        CK(hipFree(buf));
        return 0;
    }
    sha(10240, 1ull << 20, "10240 x 1 MiB (cfg3 verify)");
    sha(10240, 1ull << 20, "10240 x 1 MiB split form", 2);
    sha(10240, 1ull << 20, "10240 x 1 MiB one-wave form", 1);
    sha(1024, 10ull << 20, "1024 x 10 MiB split form", 2);
    if (sha_only) {
        CK(hipFree(buf));
        return 0;
    }
    sha(6144, 10ull << 20, "6144 x 10 MiB (cfg2 put path)");
    sha(1024, 1ull << 20, "1024 x 1 MiB");
    sha(65536, 64ull << 10, "65536 x 64 KiB");
    sha(262144, 16ull << 10, "262144 x 16 KiB");

    sweep(Shape{4, 2, S2, n2}, "k4m2 S10MiB (cfg2)", true);
    sweep(Shape{8, 4, 1ull << 20, n2 * 60 / 12}, "k8m4 S1MiB (north star)", false);
    sweep(Shape{10, 4, 1ull << 20, n2 * 60 / 14}, "k10m4 S1MiB (cfg4)", false);
    sweep(Shape{8, 2, 1ull << 20, n2 * 60 / 10}, "k8r2 S1MiB (cfg3 decode)", false);
    CK(hipFree(buf));
    return 0;
}
