// gcm_lab — times gcm_frames_kernel variants (compile-time knobs, see
// Makefile) on N synthetic objects of 40 MiB: where does the time go?
// Keys/tables are random (timing only; parity lives in tests/).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../maxio_amd/csrc/gcm_kernel.hip"

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

int main(int argc, char** argv) {
    const uint64_t n_obj = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 64;
    const char* tag = argc > 2 ? argv[2] : "default";
    const uint64_t size = 40ull << 20, fs = 65536, nf = size / fs, fl = fs + 28;
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t *pt, *fr;
    CK(hipMalloc(&pt, n_obj * size));
    CK(hipMalloc(&fr, n_obj * nf * fl));
    CK(hipMemset(pt, 0x37, n_obj * size));
    std::mt19937 rng(1);
    std::vector<uint32_t> te(1024);
    for (auto& v : te) v = rng();
    std::vector<mxec::GcmKey> keys(n_obj);
    for (auto& k : keys) {
        uint32_t* w = reinterpret_cast<uint32_t*>(&k);
        for (size_t i = 0; i < sizeof(k) / 4; ++i) w[i] = rng();
    }
    std::vector<mxec::GcmFrame> frames;
    for (uint64_t o = 0; o < n_obj; ++o)
        for (uint64_t f = 0; f < nf; ++f) {
            mxec::GcmFrame x{};
            uint8_t* base = fr + (o * nf + f) * fl;
            x.in = pt + o * size + f * fs;
            x.out = base + 12;
            x.hdr = base;
            x.tag = base + 12 + fs;
            x.aad = nullptr;
            x.aad_len = 0;
            x.index = f;
            x.len = uint32_t(fs);
            x.key = uint32_t(o);
            x.prefix_be = 0x01020304u;
            frames.push_back(x);
        }
    void *dte, *dkeys, *dfr;
    CK(hipMalloc(&dte, te.size() * 4));
    CK(hipMalloc(&dkeys, keys.size() * sizeof(mxec::GcmKey)));
    CK(hipMalloc(&dfr, frames.size() * sizeof(mxec::GcmFrame)));
    CK(hipMemcpy(dte, te.data(), te.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dkeys, keys.data(), keys.size() * sizeof(mxec::GcmKey), hipMemcpyHostToDevice));
    CK(hipMemcpy(dfr, frames.data(), frames.size() * sizeof(mxec::GcmFrame), hipMemcpyHostToDevice));
    mxec::GcmArgs a{};
    a.te = static_cast<const uint32_t*>(dte);
    a.keys = static_cast<const mxec::GcmKey*>(dkeys);
    a.frames = static_cast<const mxec::GcmFrame*>(dfr);
    a.n_frames = frames.size();
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(mxec::launch_gcm_frames(a, false, cus, 0));
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(e0, 0));
        CK(mxec::launch_gcm_frames(a, false, cus, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const double m = ms[ms.size() / 2];
    std::printf("{\"what\": \"gcm_lab\", \"variant\": \"%s\", \"objects\": %lu, \"ms\": %.3f, \"GiBps\": %.1f}\n", tag,
                (unsigned long)n_obj, m, n_obj * double(size) / (m * 1e-3) / (1 << 30));
    return 0;
}
