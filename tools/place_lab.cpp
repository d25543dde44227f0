// place_lab: why does a lone split-form SHA-256 workgroup (one consumer wave
// + one producer wave, a barrier per block) take 1.7 us per block on one
// launch and 3 us on the next?  Two candidates: the two waves landing on one
// SIMD (sharing its issue slot), or the shader clock dropping under a light
// load.  Each wave of a 2-wave workgroup runs a dependent VALU chain with a
// barrier per step (the split kernel's shape) and records HW_ID (SIMD / CU /
// SE), shader-clock cycles (s_memtime) and wall time (s_memrealtime, 100 MHz).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

struct Rec {
    unsigned hwid0, hwid1, xcc;
    unsigned long long c0, c1, r0, r1;
};

__global__ __launch_bounds__(128) void chain(Rec* out, unsigned steps, unsigned ops0, unsigned ops1, unsigned* sink) {
    const unsigned wave = threadIdx.x >> 6;
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (15 << 11));
    __syncthreads();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    unsigned x = threadIdx.x * 2654435761u, y = x ^ 0x9e3779b9u;
    const unsigned ops = wave ? ops1 : ops0;
    for (unsigned s = 0; s < steps; ++s) {
        for (unsigned k = 0; k < ops; k += 4) {
            x = __builtin_amdgcn_alignbit(x, x, 7) + y;
            y = __builtin_amdgcn_alignbit(y, y, 13) ^ x;
            x += y;
            y ^= x;
        }
        __syncthreads();
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        Rec* r = out + blockIdx.x;
        if (wave == 0) { r->hwid0 = hw; r->xcc = xcc; r->c0 = c0; r->r0 = r0; r->c1 = c1; r->r1 = r1; }
        else r->hwid1 = hw;
    }
    if (x == 0x12345678u && y == 1) sink[0] = x;
}

int main(int argc, char** argv) {
    const unsigned steps = argc > 1 ? atoi(argv[1]) : 4096;
    const int launches = argc > 2 ? atoi(argv[2]) : 12;
    const unsigned ops0 = 900, ops1 = 400;
    Rec* d;
    unsigned* sink;
    hipMalloc(&d, sizeof(Rec) * 4096);
    hipMalloc(&sink, 4);
    std::vector<Rec> h(4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int nwg : {1, 1, 8, 64, 512}) {
        for (int l = 0; l < launches; ++l) {
            hipEventRecord(e0);
            chain<<<nwg, 128>>>(d, steps, ops0, ops1, sink);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(h.data(), d, sizeof(Rec) * nwg, hipMemcpyDeviceToHost);
            int same = 0;
            double fmin = 1e9, fmax = 0;
            for (int i = 0; i < nwg; ++i) {
                const Rec& r = h[i];
                if (((r.hwid0 >> 4) & 3) == ((r.hwid1 >> 4) & 3)) ++same;
                const double f = double(r.c1 - r.c0) / (double(r.r1 - r.r0) / 100.0);  // MHz
                fmin = f < fmin ? f : fmin;
                fmax = f > fmax ? f : fmax;
            }
            const Rec& r = h[0];
            printf("wg=%3d launch=%2d ms=%.3f us/step=%.3f same_simd=%d/%d simd0=%u simd1=%u cu=%u se=%u xcc=%u clk_MHz=[%.0f,%.0f]\n",
                   nwg, l, ms, ms * 1e3 / steps, same, nwg, (r.hwid0 >> 4) & 3, (r.hwid1 >> 4) & 3,
                   (r.hwid0 >> 8) & 15, (r.hwid0 >> 13) & 7, r.xcc & 15, fmin, fmax);
            fflush(stdout);
        }
    }
    return 0;
}
