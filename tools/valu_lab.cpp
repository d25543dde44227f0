// valu_lab: dependent-issue latency vs issue rate of one wave64 on one SIMD
// (what bounds a serial hash chain).  Kernels run a loop of 32 VALU ops:
//   dep1  one chain (every op depends on the previous)
//   dep2 / dep4 / dep8  2 / 4 / 8 interleaved independent chains
// for each op kind (v_add_u32, v_alignbit_b32, v_bitop3_b32, v_add3_u32),
// one workgroup of one wave; cycles per op from s_memtime (core clock).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CH, int KIND>
__global__ __launch_bounds__(64) void chain(unsigned* out, int iters, unsigned long long* cyc) {
    unsigned x[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = threadIdx.x + c;
    unsigned y = threadIdx.x * 77u + 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int o = 0; o < 32 / CH; ++o)
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                if (KIND == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                if (KIND == 1) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(x[c]));
                if (KIND == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(x[c]) : "v"(y));
                if (KIND == 3) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x[c]) : "v"(y));
            }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += x[c];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int CH, int KIND>
void run(unsigned* out, unsigned long long* d, const char* name) {
    const int iters = 4096;
    unsigned long long c = 0;
    for (int rep = 0; rep < 3; ++rep) {
        chain<CH, KIND><<<1, 64>>>(out, iters, d);
        (void)hipMemcpy(&c, d, 8, hipMemcpyDeviceToHost);
    }
    printf("{\"op\": \"%s\", \"chains\": %d, \"cycles_per_op\": %.2f}\n", name, CH, double(c) / (iters * 32.0));
}

int chip_main();

int main(int argc, char** argv) {
    if (argc > 1 && argv[1][0] == 'c') return chip_main();  // valu_lab chip
    unsigned* out;
    unsigned long long* d;
    (void)hipMalloc(&out, 256);
    (void)hipMalloc(&d, 8);
#define K(k, n) run<1, k>(out, d, n); run<2, k>(out, d, n); run<4, k>(out, d, n); run<8, k>(out, d, n);
    K(0, "v_add_u32") K(1, "v_alignbit_b32") K(2, "v_bitop3_b32") K(3, "v_add3_u32")
    return 0;
}

// ---- chip-wide issue rate: how many int32 lane-ops per second the SIMDs
// sustain with 1, 2, 4 or 8 waves each (8 independent chains per wave).
// Sets the INT32-VALU roofline of the SHA-256 kernels (bench.py).
template <int KIND>
__global__ __launch_bounds__(256) void thru(unsigned* out, int iters) {
    unsigned x[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) x[c] = threadIdx.x + c * 0x9E3779B9u + blockIdx.x;
    const unsigned y = threadIdx.x * 77u + 1;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int o = 0; o < 4; ++o)
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                if (KIND == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                if (KIND == 1) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(x[c]));
                if (KIND == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(x[c]) : "v"(y));
                if (KIND == 3) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x[c]) : "v"(y));
                if (KIND == 4) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(x[c]) : "v"(y));
            }
    }
    unsigned s = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) s ^= x[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int KIND>
void chip(const char* name, int cus) {
    const int iters = 20000;
    unsigned* out;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int wps : {1, 2, 4, 8}) {
        const int blocks = cus * wps;  // 256-thread blocks: 4 waves, one per SIMD
        (void)hipMalloc(&out, size_t(blocks) * 256 * 4);
        thru<KIND><<<blocks, 256>>>(out, iters);
        (void)hipEventRecord(a);
        thru<KIND><<<blocks, 256>>>(out, iters);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        const double lane_ops = double(blocks) * 256 * iters * 32;
        printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"chip_lane_ops_T_per_s\": %.2f, \"ms\": %.3f}\n", name,
               wps, lane_ops / (ms * 1e-3) / 1e12, ms);
        (void)hipFree(out);
    }
}

int chip_main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    chip<0>("v_add_u32", cus);
    chip<1>("v_alignbit_b32", cus);
    chip<2>("v_bitop3_b32", cus);
    chip<3>("v_add3_u32", cus);
    chip<4>("v_perm_b32", cus);
    return 0;
}
