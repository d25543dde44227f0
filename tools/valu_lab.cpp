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

int main() {
    unsigned* out;
    unsigned long long* d;
    (void)hipMalloc(&out, 256);
    (void)hipMalloc(&d, 8);
#define K(k, n) run<1, k>(out, d, n); run<2, k>(out, d, n); run<4, k>(out, d, n); run<8, k>(out, d, n);
    K(0, "v_add_u32") K(1, "v_alignbit_b32") K(2, "v_bitop3_b32") K(3, "v_add3_u32")
    return 0;
}
