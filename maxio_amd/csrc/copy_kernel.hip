// copy_kernel.hip — host <-> device copies by CU waves, for the host
// pipeline (pipeline.cpp) and the single-request calls when their copies
// must not queue behind other users of the SDMA engines (MXEC_PIPE_COPY:
// reconstruct batches under the default `auto`, every batch under `waves`).
//
// The caller's page-locked buffers from mxec_host_alloc are mapped into the
// GPU's address space at their host address, so a wave can load from /
// store to them over PCIe like any global memory.  The host cuts a batch of
// copies into blocks of at most kCopyBlock bytes; a grid-stride loop walks
// the blocks, each lane moving 16-byte vectors with four in flight (plain
// loads of host memory; nontemporal stores into HBM, nontemporal loads of
// HBM and plain stores into host memory for the download).  A block whose
// two ends sit at the same offset modulo 16 moves its ragged head and tail
// bytewise and the rest as vectors; the host sends segments whose ends
// differ modulo 16 by SDMA (copy_phase_ok), so the byte loop is a fallback.
#include "kernels.hpp"

namespace mxec {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kThreads = 256;

template <bool kToHost>
__global__ __launch_bounds__(kThreads) void copy_blocks(const CopyBlk* __restrict__ blks, uint64_t n) {
    for (uint64_t b = blockIdx.x; b < n; b += gridDim.x) {
        const CopyBlk k = blks[b];
        const uint8_t* src = reinterpret_cast<const uint8_t*>(k.src);
        uint8_t* dst = reinterpret_cast<uint8_t*>(k.dst);
        if (((k.src ^ k.dst) & 15) == 0) {
            // Same phase modulo 16 on both sides: the ragged head and tail
            // (< 16 bytes each) by single lanes, the aligned middle as
            // 16-byte vectors -- a short last chunk or a caller pointer at an
            // odd offset costs two bytes' loops, not a byte loop over the block.
            const uint64_t head = std::min<uint64_t>((16 - (k.src & 15)) & 15, k.len);
            if (threadIdx.x < head) dst[threadIdx.x] = src[threadIdx.x];
            const u32x4* s = reinterpret_cast<const u32x4*>(src + head);
            u32x4* d = reinterpret_cast<u32x4*>(dst + head);
            const uint64_t nv = (k.len - head) / 16;
            uint64_t i = threadIdx.x;
            for (; i + 3 * kThreads < nv; i += 4 * kThreads) {
                u32x4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    v[u] = kToHost ? __builtin_nontemporal_load(s + i + u * kThreads) : s[i + u * kThreads];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (kToHost) d[i + u * kThreads] = v[u];
                    else __builtin_nontemporal_store(v[u], d + i + u * kThreads);
                }
            }
            for (; i < nv; i += kThreads) {
                const u32x4 v = kToHost ? __builtin_nontemporal_load(s + i) : s[i];
                if (kToHost) d[i] = v;
                else __builtin_nontemporal_store(v, d + i);
            }
            const uint64_t done = head + nv * 16;
            if (threadIdx.x < k.len - done) dst[done + threadIdx.x] = src[done + threadIdx.x];
        } else {
            // Different phases (the host side sends such segments by SDMA
            // instead, copy_phase_ok; kept for completeness).
            for (uint64_t i = threadIdx.x; i < k.len; i += kThreads) dst[i] = src[i];
        }
    }
}

}  // namespace

hipError_t launch_copy_blocks(const CopyBlk* blks, uint64_t n, bool to_host, uint32_t grid, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (grid == 0 || grid > n) grid = uint32_t(n < (uint64_t(1) << 31) ? n : (uint64_t(1) << 31));
    if (to_host) hipLaunchKernelGGL(copy_blocks<true>, dim3(grid), dim3(kThreads), 0, s, blks, n);
    else hipLaunchKernelGGL(copy_blocks<false>, dim3(grid), dim3(kThreads), 0, s, blks, n);
    return hipGetLastError();
}

}  // namespace mxec
