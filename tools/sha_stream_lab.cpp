// sha_stream_lab — the SHA-256 stream form (persistent waves over segments)
// against the split form on the same messages: digests compared, the work
// words (item counter, timeout code, per-group progress) dumped, and the
// big-batch timings (81 920 x 1 MiB etc.) beside the split / one-wave forms.
//
//   tools/sha_stream_lab check     small ragged batches, forced stream form
//   tools/sha_stream_lab big       timing: n x 1 MiB for n in 65536, 81920, 98304, 131072
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../maxio_amd/csrc/kernels.hpp"

#define CK(x)                                                                                       \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                           \
        }                                                                                           \
    } while (0)

namespace {

__global__ void fill_random(uint64_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) {
        uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
        x ^= x >> 31;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 29;
        p[i] = x;
    }
}

// Placement probe: every wave records HW_ID and XCC_ID, then stays resident
// ~`hold` s_memtime ticks so the dispatcher places the whole grid at once.
__global__ void placement(uint32_t* out, uint64_t hold) {
    const uint32_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    if ((threadIdx.x & 63) == 0) {
        out[2 * w] = hw;
        out[2 * w + 1] = xcc;
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < hold) __builtin_amdgcn_s_sleep(10);
}

struct Batch {
    uint8_t* data = nullptr;  // device, messages back to back (16-byte aligned starts)
    std::vector<const uint8_t*> ptrs;
    std::vector<uint64_t> lens;
    void* tables = nullptr;  // ptrs, lens
    uint8_t* dig = nullptr;
    uint32_t* work = nullptr;
    uint32_t* state = nullptr;
    int cus = 256;

    void make(const std::vector<uint64_t>& L, uint64_t seed, bool random = true) {
        uint64_t total = 0;
        for (uint64_t l : L) total += (l + 255) / 256 * 256 + 256;
        CK(hipMalloc(&data, total));
        if (random) {
            std::vector<uint8_t> h(total);
            uint64_t x = seed;
            for (auto& b : h) {
                x ^= x << 13;
                x ^= x >> 7;
                x ^= x << 17;
                b = uint8_t(x);
            }
            CK(hipMemcpy(data, h.data(), total, hipMemcpyHostToDevice));
        } else if (getenv("LAB_CONST")) {
            CK(hipMemset(data, 0x5A, total));  // constant bytes (lower switching activity)
        } else {
            hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(data), total / 8, seed);
            CK(hipDeviceSynchronize());
        }
        uint64_t o = 0;
        for (uint64_t l : L) {
            ptrs.push_back(data + o);
            lens.push_back(l);
            o += (l + 255) / 256 * 256 + 256;
        }
        const size_t n = L.size();
        CK(hipMalloc(&tables, n * 16));
        CK(hipMemcpy(tables, ptrs.data(), n * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(static_cast<char*>(tables) + n * 8, lens.data(), n * 8, hipMemcpyHostToDevice));
        CK(hipMalloc(&dig, n * 32));
        CK(hipMalloc(&work, 4 * (4 + (n + 63) / 64)));
        CK(hipMalloc(&state, 32 * n + 32 * 4096));  // + SHA_STREAM_DEBUG records  // + SHA_STREAM_DEBUG records
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    }
    mxec::ShaArgs args(int form) {
        const size_t n = lens.size();
        const bool wg4 = form == 4;  // stream form, four waves per workgroup
        if (wg4) form = 3;
        mxec::ShaArgs a{};
        a.ptrs = static_cast<const uint8_t* const*>(tables);
        a.lens = reinterpret_cast<const uint64_t*>(static_cast<char*>(tables) + n * 8);
        a.digests = dig;
        a.n = uint32_t(n);
        a.force = form;
        if (form == 3) {
            const uint64_t groups = (n + 63) / 64, simds = uint64_t(cus) * 4;
            uint64_t longest = 0;
            for (uint64_t l : lens) longest = l > longest ? l : longest;
            a.work = work;
            a.state = state;
            a.waves = uint32_t(simds);
            (void)groups;
            if (const char* e = getenv("LAB_WAVES")) a.waves = uint32_t(atoi(e));
            if (wg4) a.wg_waves = 4;
            a.seg_max = uint32_t(longest / 64 / mxec::kShaSegBlocks + 1);
        }
        return a;
    }
    double run(int form) {
        const size_t n = lens.size();
        CK(hipMemset(work, 0, 4 * (4 + (n + 63) / 64)));
        CK(hipMemset(dig, 0, n * 32));
        CK(hipMemset(state, 0, 32 * n + 32 * 4096));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a, 0));
        CK(mxec::launch_sha256(args(form), 0));
        CK(hipGetLastError());
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms;
    }
    std::vector<uint8_t> digests() {
        std::vector<uint8_t> h(lens.size() * 32);
        CK(hipMemcpy(h.data(), dig, h.size(), hipMemcpyDeviceToHost));
        return h;
    }
    std::vector<uint32_t> work_words() {
        std::vector<uint32_t> h(4 + (lens.size() + 63) / 64);
        CK(hipMemcpy(h.data(), work, h.size() * 4, hipMemcpyDeviceToHost));
        return h;
    }
    void free_all() {
        (void)hipFree(data);
        (void)hipFree(tables);
        (void)hipFree(dig);
        (void)hipFree(work);
        (void)hipFree(state);
    }
};

int check(const char* name, const std::vector<uint64_t>& L) {
    Batch b;
    b.make(L, 0x6D6178696Full + L.size());
    const double ms_split = b.run(2);
    const auto ref = b.digests();
    const double ms_one = b.run(1);
    const double ms = b.run(3);
    std::printf("{\"case\": \"%s\", \"ms_split\": %.3f, \"ms_one\": %.3f}\n", name, ms_split, ms_one);
    const auto got = b.digests();
    const auto w = b.work_words();
    size_t bad = 0, first = SIZE_MAX;
    for (size_t i = 0; i < L.size(); ++i)
        if (std::memcmp(&ref[i * 32], &got[i * 32], 32)) {
            ++bad;
            if (first == SIZE_MAX) first = i;
        }
    std::string prog;
    for (size_t g = 0; g < w.size() - 4 && g < 16; ++g) prog += (g ? "," : "") + std::to_string(w[4 + g]);
    std::printf("{\"case\": \"%s\", \"n\": %zu, \"ms\": %.3f, \"items_taken\": %u, \"timeout\": %u, \"prog\": [%s], "
                "\"mismatch\": %zu, \"first_bad\": %lld}\n",
                name, L.size(), ms, w[0], w[1], prog.c_str(), bad, first == SIZE_MAX ? -1ll : (long long)first);
    {
        std::vector<uint32_t> dbg(8 * 64);
        CK(hipMemcpy(dbg.data(), b.state + L.size() * 8, dbg.size() * 4, hipMemcpyDeviceToHost));
        std::string d;
        const uint32_t t0 = dbg[4];
        for (int t = 0; t < 12; ++t)
            d += (t ? " | " : "") + std::to_string(dbg[8 * t]) + "/" + std::to_string(dbg[8 * t + 1]) + "/" +
                 std::to_string(dbg[8 * t + 2]) + "/" + std::to_string(dbg[8 * t + 3]) + " start " +
                 std::to_string(int(dbg[8 * t + 4] - t0)) + " waited " + std::to_string(int(dbg[8 * t + 6] - t0)) +
                 " loopdone " + std::to_string(int(dbg[8 * t + 7] - t0)) + " pub " + std::to_string(int(dbg[8 * t + 5] - t0));
        std::printf("{\"case\": \"%s\", \"items (taken 1+sg / waited / prog seen / published)\": \"%s\"}\n", name,
                    d.c_str());
    }
    // the same with four waves per workgroup
    b.run(4);
    const auto got4 = b.digests();
    const auto w4 = b.work_words();
    size_t bad4 = 0;
    for (size_t i = 0; i < L.size(); ++i) bad4 += std::memcmp(&ref[i * 32], &got4[i * 32], 32) != 0;
    std::printf("{\"case\": \"%s\", \"wg4_mismatch\": %zu, \"wg4_timeout\": %u}\n", name, bad4, w4[1]);
    std::fflush(stdout);
    b.free_all();
    return bad || w[1] || bad4 || w4[1] ? 1 : 0;
}

}  // namespace

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "check";
    int fails = 0;
    if (mode == "check") {
        const uint64_t SEG = 512 * 64;
        fails += check("one 1 MiB message", {1 << 20});
        fails += check("one message of 2 segments", {2 * SEG});
        fails += check("64 messages of 3 segments", std::vector<uint64_t>(64, 3 * SEG));
        std::vector<uint64_t> ragged = {0, 1, 55, 56, 63, 64, 119, 120, SEG - 64, SEG - 1, SEG, SEG + 1, SEG + 64,
                                        2 * SEG, 3 * SEG - 9, 1 << 20, (1 << 20) + 5, 5 * SEG + 100};
        uint64_t x = 7;
        for (int i = 0; i < 150; ++i) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            ragged.push_back((x >> 33) % (4 * SEG));
        }
        fails += check("ragged 168", ragged);
        fails += check("64 messages of 1 segment", std::vector<uint64_t>(64, SEG - 64));
        fails += check("2 messages of 2 segments", std::vector<uint64_t>(2, 2 * SEG));
        if (getenv("LAB_BIGCHECK")) fails += check("1100 groups x 2 segments", std::vector<uint64_t>(1100 * 64, 2 * SEG));
    } else if (mode == "place") {
        // Where do W persistent waves land (waves per SIMD), after nothing
        // and after an 8 GiB HBM write kernel?
        const uint32_t W = getenv("LAB_WAVES") ? uint32_t(atoi(getenv("LAB_WAVES"))) : 1024;
        uint32_t* out = nullptr;
        CK(hipMalloc(&out, 8 * 8192));
        uint64_t* junk = nullptr;
        const uint64_t jn = (8ull << 30) / 8;
        CK(hipMalloc(&junk, jn * 8));
        for (int per : {1, 4})
            for (int between : {0, 1, 0, 1}) {
                if (between) hipLaunchKernelGGL(fill_random, dim3(8192), dim3(256), 0, 0, junk, jn, 1ull);
                CK(hipMemset(out, 0xFF, 8 * 8192));
                hipLaunchKernelGGL(placement, dim3(W / per), dim3(64 * per), 0, 0, out, 2000000ull);
                CK(hipDeviceSynchronize());
                std::vector<uint32_t> h(2 * W);
                CK(hipMemcpy(h.data(), out, 8 * W, hipMemcpyDeviceToHost));
                std::map<uint64_t, int> simd, cu;
                for (uint32_t w = 0; w < W; ++w) {
                    const uint64_t key = (uint64_t(h[2 * w + 1] & 0xF) << 32) | (h[2 * w] & 0xFF30u);
                    ++simd[key];
                    ++cu[key & ~uint64_t(0x30)];
                }
                std::map<int, int> hist;
                for (auto& kv : simd) ++hist[kv.second];
                std::string hs;
                for (auto& kv : hist) hs += (hs.empty() ? "" : ", ") + std::to_string(kv.first) + " waves: " + std::to_string(kv.second);
                std::printf("{\"waves\": %u, \"per_wg\": %d, \"after_hbm_kernel\": %d, \"simds_used\": %zu, \"cus_used\": %zu, \"simds by waves\": \"%s\", \"hw0\": \"%08x\"}\n",
                            W, per, between, simd.size(), cu.size(), hs.c_str(), h[0]);
                std::fflush(stdout);
            }
        (void)hipFree(out);
        (void)hipFree(junk);
    } else if (mode == "repeat") {
        // n x 1 MiB stream-form launches back to back; LAB_BETWEEN=1 puts an
        // 8 GiB HBM write kernel between launches (as config 3c's decodes).
        const uint64_t n = getenv("LAB_N") ? strtoull(getenv("LAB_N"), nullptr, 10) : 81920;
        Batch b;
        b.make(std::vector<uint64_t>(n, 1 << 20), n, false);
        uint64_t* junk = nullptr;
        const uint64_t jn = (8ull << 30) / 8;
        const bool between = getenv("LAB_BETWEEN") != nullptr;
        if (between) CK(hipMalloc(&junk, jn * 8));
        for (int r = 0; r < 8; ++r) {
            if (between) {
                hipLaunchKernelGGL(fill_random, dim3(8192), dim3(256), 0, 0, junk, jn, uint64_t(r));
                CK(hipDeviceSynchronize());
            }
            const double ms = b.run(getenv("LAB_FORM") ? atoi(getenv("LAB_FORM")) : 3);
            std::printf("{\"repeat\": %d, \"n\": %llu, \"between\": %d, \"ms\": %.3f, \"timeout\": %u}\n", r,
                        (unsigned long long)n, int(between), ms, b.work_words()[1]);
            std::fflush(stdout);
        }
        if (junk) (void)hipFree(junk);
        b.free_all();
    } else {
        std::vector<uint64_t> sizes = {20480, 32768, 40960, 51200, 65536, 81920, 98304, 131072};
        if (const char* e = getenv("LAB_SIZES")) {
            sizes.clear();
            for (const char* q = e; *q;) {
                sizes.push_back(strtoull(q, const_cast<char**>(&q), 10));
                if (*q == ',') ++q;
            }
        }
        for (uint64_t n : sizes) {
            Batch b;
            b.make(std::vector<uint64_t>(n, 1 << 20), n, false);
            for (int form : {2, 1, 3, 4}) {
                b.run(form);  // warm
                const double ms = b.run(form);
                const auto w = b.work_words();
                std::printf("{\"n\": %llu, \"form\": \"%s\", \"ms\": %.3f, \"GBps_hashed\": %.1f, \"timeout\": %u}\n",
                            (unsigned long long)n, form == 1 ? "one" : form == 2 ? "split" : form == 3 ? "stream" : "stream_wg4", ms,
                            double(n) * (1 << 20) / (ms * 1e-3) / 1e9, form >= 3 ? w[1] : 0u);
                std::fflush(stdout);
            }
            b.free_all();
        }
    }
    return fails ? 1 : 0;
}
