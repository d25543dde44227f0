// h2d_lab: host -> device upload of GET-sized requests (8 x 1 MiB from
// pageable host memory) by T threads at once, each on its own stream:
//   pageable  hipMemcpyAsync straight from the pageable buffers (HIP stages)
//   pinned    memcpy into a per-thread pinned pair of 8 MiB pieces, one DMA
//             per piece, double-buffered with events
// Prints per-mode aggregate GiB/s and mean per-request latency.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char** argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 64;
    const int reqs = argc > 2 ? atoi(argv[2]) : 8;  // per thread
    const size_t chunk = 1 << 20, nchunk = 8, piece = 8 << 20;
    for (int mode = 0; mode < 2; ++mode) {
        std::vector<std::thread> th;
        std::vector<double> lat(T, 0);
        const auto t0 = std::chrono::steady_clock::now();
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                hipStream_t s;
                CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
                void* dev;
                CK(hipMalloc(&dev, chunk * nchunk));
                std::vector<std::vector<uint8_t>> host(nchunk, std::vector<uint8_t>(chunk, uint8_t(t)));
                void* pin[2];
                hipEvent_t ev[2];
                for (int b = 0; b < 2; ++b) {
                    CK(hipHostMalloc(&pin[b], piece, hipHostMallocDefault));
                    CK(hipEventCreateWithFlags(&ev[b], hipEventDisableTiming));
                }
                for (int r = 0; r < reqs + 1; ++r) {
                    const auto a = std::chrono::steady_clock::now();
                    if (mode == 0) {
                        for (size_t c = 0; c < nchunk; ++c)
                            CK(hipMemcpyAsync((uint8_t*)dev + c * chunk, host[c].data(), chunk, hipMemcpyHostToDevice, s));
                    } else {
                        // all 8 MiB fit one piece here; the lab still alternates buffers
                        const int b = r & 1;
                        CK(hipEventSynchronize(ev[b]));
                        for (size_t c = 0; c < nchunk; ++c) memcpy((uint8_t*)pin[b] + c * chunk, host[c].data(), chunk);
                        CK(hipMemcpyAsync(dev, pin[b], chunk * nchunk, hipMemcpyHostToDevice, s));
                        CK(hipEventRecord(ev[b], s));
                    }
                    CK(hipStreamSynchronize(s));
                    if (r) lat[t] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
                }
                for (int b = 0; b < 2; ++b) { CK(hipHostFree(pin[b])); CK(hipEventDestroy(ev[b])); }
                CK(hipFree(dev));
                CK(hipStreamDestroy(s));
            });
        for (auto& x : th) x.join();
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        double ml = 0;
        for (double x : lat) ml += x;
        ml /= double(T) * reqs;
        printf("{\"mode\": \"%s\", \"threads\": %d, \"GiBps_incl_setup\": %.2f, \"ms_per_8MiB_request\": %.3f}\n",
               mode ? "pinned" : "pageable", T, double(T) * (reqs + 1) * chunk * nchunk / el / (1 << 30), ml);
        fflush(stdout);
    }
    return 0;
}
