// place_lab2: where the two waves of each workgroup of a full-chip
// split-form SHA launch land.  1280 workgroups x 128 threads with 32 KiB of
// LDS each (the split kernel's footprint: five per CU), a ~2 ms busy loop so
// all are resident together; per wave HW_ID (SIMD, CU, SH, SE) and XCC_ID.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(128) void busy(unsigned* out, unsigned iters) {
    __shared__ unsigned pad[8192];  // 32 KiB
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (15 << 11));
    pad[threadIdx.x] = threadIdx.x;
    __syncthreads();
    unsigned x = pad[(threadIdx.x * 7) & 127];
    for (unsigned i = 0; i < iters; ++i) x = __builtin_amdgcn_alignbit(x, x, 7) + i;
    if ((threadIdx.x & 63) == 0) {
        out[blockIdx.x * 4 + (threadIdx.x >> 6) * 2] = hw;
        out[blockIdx.x * 4 + (threadIdx.x >> 6) * 2 + 1] = xcc;
    }
    if (x == 0x1234567u) pad[0] = x;
}

int main() {
    const int nwg = 1280;
    unsigned* d;
    (void)hipMalloc(&d, nwg * 16);
    busy<<<nwg, 128>>>(d, 200000);
    (void)hipDeviceSynchronize();
    std::vector<unsigned> h(nwg * 4);
    (void)hipMemcpy(h.data(), d, nwg * 16, hipMemcpyDeviceToHost);
    for (int b = 0; b < nwg; ++b)
        printf("%d %u %u %u %u\n", b, h[b * 4], h[b * 4 + 1], h[b * 4 + 2], h[b * 4 + 3]);
    return 0;
}
