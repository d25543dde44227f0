// probe_kernel.hip — HBM calibration streams for bench.py (libmaxio_probe.so).
//
// Not part of the storage ABI: these are the denominators bench.py prints
// beside the RS kernel's roofline fraction ("what this box's HBM gives a plain
// stream of the same shape"), measured with the same load / store forms the
// RS kernel uses — nontemporal global_load_dwordx4 with four 16-byte loads in
// flight per lane, nontemporal stores, 16 workgroups of 256 lanes per CU
// (mxprobe_set_stream_wpc changes it: the RS kernel's 512 reads faster),
// grid-stride.
//
//   mxprobe_copy       read n bytes, write n bytes             (1:1)
//   mxprobe_copy_float4  the same with the guide's float4 copy: plain loads
//                      and stores, one element per lane, no grid-stride
//   mxprobe_read2_write1  read 2n bytes (two sources), write n (2:1, the
//                      encode stream of k=4 m=2 and k=8 m=4)
//   mxprobe_read       read n bytes                            (read-only)
//   mxprobe_write      write n bytes (policy 0 nontemporal, 1 plain)
//   mxprobe_rs_pattern the RS kernel's own access pattern with the GF math
//                      replaced by XOR: object-major [n][k][S] in,
//                      [n][m][S] out, tiles of 256 lanes x 16 B x 4 vectors,
//                      4 inputs x 4 vectors of loads in flight, 512 WG per CU
//                      (the ceiling the RS kernel is measured against)
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void probe_copy(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const u32x4 a = __builtin_nontemporal_load(s + i), b = __builtin_nontemporal_load(s + i + stride);
        const u32x4 c = __builtin_nontemporal_load(s + i + 2 * stride), e = __builtin_nontemporal_load(s + i + 3 * stride);
        __builtin_nontemporal_store(a, d + i);
        __builtin_nontemporal_store(b, d + i + stride);
        __builtin_nontemporal_store(c, d + i + 2 * stride);
        __builtin_nontemporal_store(e, d + i + 3 * stride);
    }
    for (; i < n; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}

// The guide's float4 copy (MI355X_MICROARCH.md: 6.29 TB/s measured): one
// 16-byte element per lane, plain (temporal) loads and stores, one
// workgroup per 256 elements, no grid-stride loop.
__global__ __launch_bounds__(256) void probe_copy_float4(const float4* __restrict__ s, float4* __restrict__ d, uint64_t n) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i < n) d[i] = s[i];
}

__global__ __launch_bounds__(256) void probe_read2_write1(const u32x4* __restrict__ s0, const u32x4* __restrict__ s1,
                                                          u32x4* __restrict__ d, uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    for (; i + stride < n; i += 2 * stride) {
        const u32x4 a = __builtin_nontemporal_load(s0 + i), b = __builtin_nontemporal_load(s0 + i + stride);
        const u32x4 c = __builtin_nontemporal_load(s1 + i), e = __builtin_nontemporal_load(s1 + i + stride);
        __builtin_nontemporal_store(a ^ c, d + i);
        __builtin_nontemporal_store(b ^ e, d + i + stride);
    }
    for (; i < n; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(s0 + i) ^ __builtin_nontemporal_load(s1 + i), d + i);
}

__global__ __launch_bounds__(256) void probe_read(const u32x4* __restrict__ s, u32x4* __restrict__ sink, uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    u32x4 acc = {0, 0, 0, 0};
    uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const u32x4 a = __builtin_nontemporal_load(s + i), b = __builtin_nontemporal_load(s + i + stride);
        const u32x4 c = __builtin_nontemporal_load(s + i + 2 * stride), e = __builtin_nontemporal_load(s + i + 3 * stride);
        acc ^= a ^ b ^ c ^ e;
    }
    for (; i < n; i += stride) acc ^= __builtin_nontemporal_load(s + i);
    if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u) sink[0] = acc;  // keeps the loads; never true for the probe's data
}

// Store policies of the write probes (gfx950 cache-policy bits on a vector
// global_store_dwordx4): 0 nt, 1 plain, 2 sc1, 3 sc0 sc1, 4 sc1 nt.  Plain /
// nt keep the line in the XCD's L2, sc1 / sc0 sc1 drop it
// (MI355X_MICROARCH.md, memory-model table).
typedef u32x4 __attribute__((address_space(1)))* g4ptr;
template <int P>
__device__ __forceinline__ void store_p(u32x4* d, u32x4 v) {
    g4ptr g = (g4ptr)(d);
    if constexpr (P == 0) __builtin_nontemporal_store(v, g);
    else if constexpr (P == 1) *g = v;
    else if constexpr (P == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(g), "v"(v) : "memory");
    else if constexpr (P == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(g), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(g), "v"(v) : "memory");
}

template <int P>
__global__ __launch_bounds__(256) void probe_write(u32x4* __restrict__ d, uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    const u32x4 v = {blockIdx.x, threadIdx.x, 0x5A5A5A5Au, 0xA5A5A5A5u};
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += stride) store_p<P>(d + i, v);
}

template <int R, int P = 0>
__global__ __launch_bounds__(256) void probe_pattern(const uint8_t* __restrict__ data, uint8_t* __restrict__ par,
                                                     uint32_t k, uint64_t S, uint64_t n_obj, uint64_t dstride,
                                                     uint64_t pstride, uint64_t sstride) {
    constexpr uint64_t kTile = 256 * 16 * 4;
    const uint64_t tpo = S / kTile, n_tiles = tpo * n_obj;
    for (uint64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        const uint64_t o = t / tpo, base = (t - o * tpo) * kTile + threadIdx.x * 16;
        u32x4 acc[4][R];
#pragma unroll
        for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int i = 0; i < R; ++i) acc[v][i] = u32x4{0, 0, 0, 0};
        for (uint32_t j = 0; j < k; j += 4) {
            u32x4 x[4][4];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                for (int v = 0; v < 4; ++v)
                    x[jj][v] = __builtin_nontemporal_load(
                        reinterpret_cast<const u32x4*>(data + o * dstride + (j + jj) * sstride + base + v * 4096));
#pragma unroll
            for (int v = 0; v < 4; ++v)
#pragma unroll
                for (int i = 0; i < R; ++i) acc[v][i] ^= (x[0][v] ^ x[1][v]) + (x[2][v] ^ x[3][v]) * (i + 1u);
        }
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
            for (int v = 0; v < 4; ++v)
                store_p<P>(reinterpret_cast<u32x4*>(par + o * pstride + i * sstride + base + v * 4096), acc[v][i]);
    }
}

// The RS pattern (m = 2) with each workgroup's parity held back in LDS over
// G consecutive tiles of one object and then stored as G x 16 KiB runs per
// parity shard (do longer store bursts recover the ~12 %
// the 2:1 read / write mix costs?).  LDS: G x 2 x 16 KiB per workgroup
// (G = 2: 64 KiB, two workgroups per CU; G = 4: 128 KiB, one).
template <int G>
__global__ __launch_bounds__(256) void probe_pattern_lds(const uint8_t* __restrict__ data, uint8_t* __restrict__ par,
                                                         uint32_t k, uint64_t S, uint64_t n_obj, uint64_t ostride,
                                                         uint64_t sstride) {
    constexpr int R = 2;
    constexpr uint64_t kTile = 256 * 16 * 4;
    __shared__ u32x4 held[G][R][4][256];
    const uint64_t tpo = S / kTile, spo = tpo / G, n_super = spo * n_obj;
    for (uint64_t t = blockIdx.x; t < n_super; t += gridDim.x) {
        const uint64_t o = t / spo, t0 = (t - o * spo) * G;
#pragma unroll 1
        for (int g = 0; g < G; ++g) {
            const uint64_t base = (t0 + g) * kTile + threadIdx.x * 16;
            u32x4 acc[4][R];
#pragma unroll
            for (int v = 0; v < 4; ++v)
#pragma unroll
                for (int i = 0; i < R; ++i) acc[v][i] = u32x4{0, 0, 0, 0};
            for (uint32_t j = 0; j < k; j += 4) {
                u32x4 x[4][4];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                    for (int v = 0; v < 4; ++v)
                        x[jj][v] = __builtin_nontemporal_load(
                            reinterpret_cast<const u32x4*>(data + o * ostride + (j + jj) * sstride + base + v * 4096));
#pragma unroll
                for (int v = 0; v < 4; ++v)
#pragma unroll
                    for (int i = 0; i < R; ++i) acc[v][i] ^= (x[0][v] ^ x[1][v]) + (x[2][v] ^ x[3][v]) * (i + 1u);
            }
#pragma unroll
            for (int v = 0; v < 4; ++v)
#pragma unroll
                for (int i = 0; i < R; ++i) held[g][i][v][threadIdx.x] = acc[v][i];
        }
        // Each lane stores back what it computed (same addresses as the plain
        // pattern), shard after shard, G tiles in a row.
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int v = 0; v < 4; ++v)
                    __builtin_nontemporal_store(
                        held[g][i][v][threadIdx.x],
                        reinterpret_cast<u32x4*>(par + o * ostride + i * sstride + (t0 + g) * kTile +
                                                 threadIdx.x * 16 + v * 4096));
    }
}

// The RS tile schedule split into its halves (the placement lab's
// diagnosis): READ only loads the k data shards of every tile (folded into a
// sink store that never fires), WRITE only stores the R parity shards.
template <int R, bool READ, bool WRITE>
__global__ __launch_bounds__(256) void probe_pattern_part(const uint8_t* __restrict__ data, uint8_t* __restrict__ par,
                                                          uint32_t k, uint64_t S, uint64_t n_obj, uint64_t ostride,
                                                          uint64_t sstride, u32x4* __restrict__ sink) {
    constexpr uint64_t kTile = 256 * 16 * 4;
    const uint64_t tpo = S / kTile, n_tiles = tpo * n_obj;
    u32x4 any = {0, 0, 0, 0};
    for (uint64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        const uint64_t o = t / tpo, base = (t - o * tpo) * kTile + threadIdx.x * 16;
        u32x4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
        if constexpr (READ) {
            for (uint32_t j = 0; j < k; j += 4) {
                u32x4 x[4][4];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                    for (int v = 0; v < 4; ++v)
                        x[jj][v] = __builtin_nontemporal_load(
                            reinterpret_cast<const u32x4*>(data + o * ostride + (j + jj) * sstride + base + v * 4096));
#pragma unroll
                for (int v = 0; v < 4; ++v) acc[v] ^= (x[0][v] ^ x[1][v]) + (x[2][v] ^ x[3][v]);
            }
        } else {
#pragma unroll
            for (int v = 0; v < 4; ++v) acc[v] = u32x4{uint32_t(t), uint32_t(v), 0x5A5A5A5Au, 0xA5A5A5A5u};
        }
        if constexpr (WRITE) {
#pragma unroll
            for (int i = 0; i < R; ++i)
#pragma unroll
                for (int v = 0; v < 4; ++v)
                    store_p<0>(reinterpret_cast<u32x4*>(par + o * ostride + i * sstride + base + v * 4096),
                               acc[v] + uint32_t(i));
        } else {
#pragma unroll
            for (int v = 0; v < 4; ++v) any ^= acc[v];
        }
    }
    if (!WRITE && any.x == 0x12345678u && any.y == 0x9abcdef0u) sink[0] = any;
}

// The RS pattern (k = 4, m = 2) in time-divided phases: every workgroup
// reads G tiles' data shards (parity kept in registers) only while the
// chip-wide 100 MHz clock is in the first `rwin` ticks of each `period`, and
// stores the parity only in the rest, so HBM sees read bursts and write
// bursts instead of a steady 2:1 mix (is the mixing penalty avoidable?).
// period == 0: no gating (the same kernel, unphased).  Lab probe only.
__device__ __forceinline__ uint64_t rt_ticks() { return __builtin_amdgcn_s_memrealtime(); }
template <int G>
__global__ __launch_bounds__(256) void probe_phased(const uint8_t* __restrict__ data, uint8_t* __restrict__ par,
                                                    uint64_t S, uint64_t n_obj, uint64_t ostride, uint64_t sstride,
                                                    uint32_t period, uint32_t rwin) {
    constexpr uint64_t kTile = 256 * 16 * 4;
    const uint64_t tpo = S / kTile, n_tiles = tpo * n_obj;
    for (uint64_t t0 = uint64_t(blockIdx.x) * G; t0 < n_tiles; t0 += uint64_t(gridDim.x) * G) {
        if (period) {
            while (rt_ticks() % period >= rwin) __builtin_amdgcn_s_sleep(1);
        }
        u32x4 out[G][2][4];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint64_t t = t0 + g < n_tiles ? t0 + g : t0;
            const uint64_t o = t / tpo, base = (t - o * tpo) * kTile + threadIdx.x * 16;
            u32x4 x[4][4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int v = 0; v < 4; ++v)
                    x[j][v] = __builtin_nontemporal_load(
                        reinterpret_cast<const u32x4*>(data + o * ostride + j * sstride + base + v * 4096));
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                out[g][0][v] = (x[0][v] ^ x[1][v]) + (x[2][v] ^ x[3][v]);
                out[g][1][v] = (x[0][v] + x[1][v]) ^ (x[2][v] + x[3][v]);
            }
        }
        if (period) {
            while (rt_ticks() % period < rwin) __builtin_amdgcn_s_sleep(1);
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            if (t0 + g >= n_tiles) break;
            const uint64_t t = t0 + g, o = t / tpo, base = (t - o * tpo) * kTile + threadIdx.x * 16;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int v = 0; v < 4; ++v)
                    store_p<0>(reinterpret_cast<u32x4*>(par + o * ostride + i * sstride + base + v * 4096), out[g][i][v]);
        }
    }
}

// The RS access pattern at the float4 copy's granularity: one 16-byte column
// of one object per lane (XOR for the GF math), plain loads and stores, one
// workgroup per 256 columns -- the schedule with the least state per lane
// (the placement lab's second denominator).
template <int R>
__global__ __launch_bounds__(256) void probe_rs_float4(const uint8_t* __restrict__ data, uint8_t* __restrict__ par,
                                                       uint32_t k, uint64_t cols, uint64_t n_obj, uint64_t dstride,
                                                       uint64_t pstride, uint64_t sstride) {
    const uint64_t g = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    if (g >= cols * n_obj) return;
    const uint64_t o = g / cols, c = (g - o * cols) * 16;
    u32x4 acc[R];
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = u32x4{0, 0, 0, 0};
    for (uint32_t j = 0; j < k; ++j) {
        const u32x4 x = *reinterpret_cast<const u32x4*>(data + o * dstride + j * sstride + c);
#pragma unroll
        for (int i = 0; i < R; ++i) acc[i] ^= x * (i + j + 1u);
    }
#pragma unroll
    for (int i = 0; i < R; ++i) *reinterpret_cast<u32x4*>(par + o * pstride + i * sstride + c) = acc[i];
}

// Host <-> device copy by CU waves instead of the SDMA engines: each lane
// moves 16-byte vectors, four in flight, grid-stride over the range (the
// host side is page-locked memory mapped into the GPU's address space).
__global__ __launch_bounds__(256) void probe_copy_waves(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const u32x4 a = __builtin_nontemporal_load(s + i), b = __builtin_nontemporal_load(s + i + stride);
        const u32x4 c = __builtin_nontemporal_load(s + i + 2 * stride), e = __builtin_nontemporal_load(s + i + 3 * stride);
        __builtin_nontemporal_store(a, d + i);
        __builtin_nontemporal_store(b, d + i + stride);
        __builtin_nontemporal_store(c, d + i + 2 * stride);
        __builtin_nontemporal_store(e, d + i + 3 * stride);
    }
    for (; i < n; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}

int g_stream_wpc = 16;  // workgroups per CU of the plain stream probes (mxprobe_set_stream_wpc)

int cus() {
    int dev = 0, n = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n;
}
int grid() { return cus() * g_stream_wpc; }

}  // namespace

// Sizes in bytes, multiples of 16; pointers 16-byte aligned.  Enqueued on
// `stream`; returns a hipError_t.
extern "C" int mxprobe_copy(void* dst, const void* src, uint64_t bytes, void* stream) {
    if ((bytes & 15) || (reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15)
        return int(hipErrorInvalidValue);
    hipLaunchKernelGGL(probe_copy, dim3(grid()), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<const u32x4*>(src), static_cast<u32x4*>(dst), bytes / 16);
    return int(hipGetLastError());
}

// The guide's float4 copy over `bytes` (multiple of 16, at most 2^40).
extern "C" int mxprobe_copy_float4(void* dst, const void* src, uint64_t bytes, void* stream) {
    if ((bytes & 15) || bytes > (uint64_t(1) << 40) || (reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15)
        return int(hipErrorInvalidValue);
    const uint64_t n = bytes / 16, blocks = (n + 255) / 256;
    if (blocks == 0) return 0;
    hipLaunchKernelGGL(probe_copy_float4, dim3(uint32_t(blocks)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<const float4*>(src), static_cast<float4*>(dst), n);
    return int(hipGetLastError());
}

extern "C" int mxprobe_read2_write1(void* dst, const void* src0, const void* src1, uint64_t bytes, void* stream) {
    if ((bytes & 15) ||
        (reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src0) | reinterpret_cast<uintptr_t>(src1)) & 15)
        return int(hipErrorInvalidValue);
    hipLaunchKernelGGL(probe_read2_write1, dim3(grid()), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<const u32x4*>(src0), static_cast<const u32x4*>(src1), static_cast<u32x4*>(dst),
                       bytes / 16);
    return int(hipGetLastError());
}

extern "C" int mxprobe_read(const void* src, uint64_t bytes, void* sink16, void* stream) {
    if ((bytes & 15) || (reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(sink16)) & 15)
        return int(hipErrorInvalidValue);
    hipLaunchKernelGGL(probe_read, dim3(grid()), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<const u32x4*>(src), static_cast<u32x4*>(sink16), bytes / 16);
    return int(hipGetLastError());
}

extern "C" int mxprobe_write(void* dst, uint64_t bytes, int policy, void* stream) {
    if ((bytes & 15) || (reinterpret_cast<uintptr_t>(dst) & 15) || policy < 0 || policy > 4)
        return int(hipErrorInvalidValue);
    hipStream_t s = static_cast<hipStream_t>(stream);
    u32x4* d = static_cast<u32x4*>(dst);
    switch (policy) {
        case 0: hipLaunchKernelGGL(probe_write<0>, dim3(grid()), dim3(256), 0, s, d, bytes / 16); break;
        case 1: hipLaunchKernelGGL(probe_write<1>, dim3(grid()), dim3(256), 0, s, d, bytes / 16); break;
        case 2: hipLaunchKernelGGL(probe_write<2>, dim3(grid()), dim3(256), 0, s, d, bytes / 16); break;
        case 3: hipLaunchKernelGGL(probe_write<3>, dim3(grid()), dim3(256), 0, s, d, bytes / 16); break;
        default: hipLaunchKernelGGL(probe_write<4>, dim3(grid()), dim3(256), 0, s, d, bytes / 16); break;
    }
    return int(hipGetLastError());
}

// k a multiple of 4, m in {1, 2, 4}, S a multiple of 16 KiB; object o's
// shard j at data + o * data_obj_stride + j * shard_stride (parity likewise):
// [n][k][S] / [n][m][S] with strides k*S / m*S and S, or one object-major
// [n][k+m][shard_stride] buffer with both object strides (k+m)*shard_stride.
extern "C" int mxprobe_rs_pattern_strided(const void* data, void* parity, uint32_t k, uint32_t m, uint64_t S,
                                          uint64_t n_obj, uint64_t data_obj_stride, uint64_t parity_obj_stride,
                                          uint64_t shard_stride, void* stream) {
    if (k == 0 || (k & 3) || S == 0 || (S % 16384) ||
        ((reinterpret_cast<uintptr_t>(data) | reinterpret_cast<uintptr_t>(parity)) & 15))
        return int(hipErrorInvalidValue);
    const dim3 g(uint32_t(cus() * (m <= 2 ? 1024 : 512))), b(256);  // as the RS kernel (rs_default_variant)
    const auto* in = static_cast<const uint8_t*>(data);
    auto* out = static_cast<uint8_t*>(parity);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t ds = data_obj_stride, ps = parity_obj_stride, ss = shard_stride;
    if (m == 1) hipLaunchKernelGGL(probe_pattern<1>, g, b, 0, s, in, out, k, S, n_obj, ds, ps, ss);
    else if (m == 2) hipLaunchKernelGGL(probe_pattern<2>, g, b, 0, s, in, out, k, S, n_obj, ds, ps, ss);
    else if (m == 4) hipLaunchKernelGGL(probe_pattern<4>, g, b, 0, s, in, out, k, S, n_obj, ds, ps, ss);
    else return int(hipErrorInvalidValue);
    return int(hipGetLastError());
}

extern "C" int mxprobe_rs_pattern(const void* data, void* parity, uint32_t k, uint32_t m, uint64_t S, uint64_t n_obj,
                                  void* stream) {
    return mxprobe_rs_pattern_strided(data, parity, k, m, S, n_obj, uint64_t(k) * S, uint64_t(m) * S, S, stream);
}

// The halves of the RS pattern over an object-major batch (one buffer,
// object stride `obj_stride`, shard stride `shard_stride`, m = 2, k a
// multiple of 4, S a multiple of 16 KiB): part 0 reads the k data shards
// only, part 1 writes the m parity shards only, part 2 both (the pattern).
// Grid as the RS kernel at m <= 2 (1024 per CU).  sink: 16 bytes of device
// memory (never written in practice).
extern "C" int mxprobe_rs_pattern_part(const void* data, void* parity, uint32_t k, uint64_t S, uint64_t n_obj,
                                       uint64_t obj_stride, uint64_t shard_stride, int part, void* sink,
                                       void* stream) {
    if (k == 0 || (k & 3) || S == 0 || (S % 16384) || part < 0 || part > 2 ||
        ((reinterpret_cast<uintptr_t>(data) | reinterpret_cast<uintptr_t>(parity) |
          reinterpret_cast<uintptr_t>(sink)) & 15))
        return int(hipErrorInvalidValue);
    const dim3 g(uint32_t(cus() * 1024)), b(256);
    const auto* in = static_cast<const uint8_t*>(data);
    auto* out = static_cast<uint8_t*>(parity);
    auto* sk = static_cast<u32x4*>(sink);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (part == 0) hipLaunchKernelGGL((probe_pattern_part<2, true, false>), g, b, 0, s, in, out, k, S, n_obj, obj_stride, shard_stride, sk);
    else if (part == 1) hipLaunchKernelGGL((probe_pattern_part<2, false, true>), g, b, 0, s, in, out, k, S, n_obj, obj_stride, shard_stride, sk);
    else hipLaunchKernelGGL((probe_pattern_part<2, true, true>), g, b, 0, s, in, out, k, S, n_obj, obj_stride, shard_stride, sk);
    return int(hipGetLastError());
}

// probe_pattern_lds over an object-major batch (m = 2, k a multiple of 4,
// S a multiple of G x 16 KiB; parity at data + k * shard_stride of each
// object), `wpc` workgroups per CU.
extern "C" int mxprobe_rs_pattern_lds(const void* data, void* parity, uint32_t k, uint64_t S, uint64_t n_obj,
                                      uint64_t obj_stride, uint64_t shard_stride, int G, int wpc, void* stream) {
    if (k == 0 || (k & 3) || S == 0 || (G != 2 && G != 4) || (S % (uint64_t(G) * 16384)) || wpc < 1 ||
        wpc > 4096 || ((reinterpret_cast<uintptr_t>(data) | reinterpret_cast<uintptr_t>(parity)) & 15) ||
        static_cast<const uint8_t*>(parity) != static_cast<const uint8_t*>(data) + uint64_t(k) * shard_stride)
        return int(hipErrorInvalidValue);
    const dim3 g(uint32_t(cus() * wpc)), b(256);
    const auto* in = static_cast<const uint8_t*>(data);
    auto* out = static_cast<uint8_t*>(parity);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (G == 2) hipLaunchKernelGGL(probe_pattern_lds<2>, g, b, 0, s, in, out, k, S, n_obj, obj_stride, shard_stride);
    else hipLaunchKernelGGL(probe_pattern_lds<4>, g, b, 0, s, in, out, k, S, n_obj, obj_stride, shard_stride);
    return int(hipGetLastError());
}

// probe_phased over an object-major k = 4, m = 2 batch: `wpc` workgroups per
// CU, G in {1, 2, 4} tiles per phase, period / rwin in 10 ns ticks (period 0:
// ungated).
extern "C" int mxprobe_rs_phased(const void* data, void* parity, uint64_t S, uint64_t n_obj, uint64_t obj_stride,
                                 uint64_t shard_stride, int G, int wpc, uint32_t period, uint32_t rwin, void* stream) {
    if (S == 0 || (S % 16384) || wpc < 1 || wpc > 4096 || (period && rwin >= period) ||
        ((reinterpret_cast<uintptr_t>(data) | reinterpret_cast<uintptr_t>(parity)) & 15))
        return int(hipErrorInvalidValue);
    const dim3 g(uint32_t(cus() * wpc)), b(256);
    const auto* in = static_cast<const uint8_t*>(data);
    auto* out = static_cast<uint8_t*>(parity);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (G == 1) hipLaunchKernelGGL(probe_phased<1>, g, b, 0, s, in, out, S, n_obj, obj_stride, shard_stride, period, rwin);
    else if (G == 2) hipLaunchKernelGGL(probe_phased<2>, g, b, 0, s, in, out, S, n_obj, obj_stride, shard_stride, period, rwin);
    else if (G == 4) hipLaunchKernelGGL(probe_phased<4>, g, b, 0, s, in, out, S, n_obj, obj_stride, shard_stride, period, rwin);
    else return int(hipErrorInvalidValue);
    return int(hipGetLastError());
}

// probe_rs_float4 over the same strided layout (m in {1, 2, 4}, S % 16 == 0).
extern "C" int mxprobe_rs_float4_strided(const void* data, void* parity, uint32_t k, uint32_t m, uint64_t S,
                                         uint64_t n_obj, uint64_t data_obj_stride, uint64_t parity_obj_stride,
                                         uint64_t shard_stride, void* stream) {
    if (k == 0 || S == 0 || (S % 16) || ((reinterpret_cast<uintptr_t>(data) | reinterpret_cast<uintptr_t>(parity)) & 15))
        return int(hipErrorInvalidValue);
    const uint64_t cols = S / 16, blocks = (cols * n_obj + 255) / 256;
    if (blocks >= (uint64_t(1) << 32)) return int(hipErrorInvalidValue);
    const auto* in = static_cast<const uint8_t*>(data);
    auto* out = static_cast<uint8_t*>(parity);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 g{uint32_t(blocks), 1, 1}, b{256, 1, 1};
    const uint64_t ds = data_obj_stride, ps = parity_obj_stride, ss = shard_stride;
    if (m == 1) hipLaunchKernelGGL(probe_rs_float4<1>, g, b, 0, s, in, out, k, cols, n_obj, ds, ps, ss);
    else if (m == 2) hipLaunchKernelGGL(probe_rs_float4<2>, g, b, 0, s, in, out, k, cols, n_obj, ds, ps, ss);
    else if (m == 4) hipLaunchKernelGGL(probe_rs_float4<4>, g, b, 0, s, in, out, k, cols, n_obj, ds, ps, ss);
    else return int(hipErrorInvalidValue);
    return int(hipGetLastError());
}

// The RS pattern at m = 2 with store policy `policy` (store_p above), for the
// write-policy lab (tools/region_lab.py --policies); same geometry as
// mxprobe_rs_pattern_strided.
extern "C" int mxprobe_rs_pattern_policy(const void* data, void* parity, uint32_t k, uint64_t S, uint64_t n_obj,
                                         uint64_t obj_stride, uint64_t shard_stride, int policy, void* stream) {
    if (k == 0 || (k & 3) || S == 0 || (S % 16384) || policy < 0 || policy > 4 ||
        ((reinterpret_cast<uintptr_t>(data) | reinterpret_cast<uintptr_t>(parity)) & 15))
        return int(hipErrorInvalidValue);
    const dim3 g(uint32_t(cus() * 512)), b(256);
    const auto* in = static_cast<const uint8_t*>(data);
    auto* out = static_cast<uint8_t*>(parity);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t os = obj_stride, ss = shard_stride;
    switch (policy) {
        case 0: hipLaunchKernelGGL((probe_pattern<2, 0>), g, b, 0, s, in, out, k, S, n_obj, os, os, ss); break;
        case 1: hipLaunchKernelGGL((probe_pattern<2, 1>), g, b, 0, s, in, out, k, S, n_obj, os, os, ss); break;
        case 2: hipLaunchKernelGGL((probe_pattern<2, 2>), g, b, 0, s, in, out, k, S, n_obj, os, os, ss); break;
        case 3: hipLaunchKernelGGL((probe_pattern<2, 3>), g, b, 0, s, in, out, k, S, n_obj, os, os, ss); break;
        default: hipLaunchKernelGGL((probe_pattern<2, 4>), g, b, 0, s, in, out, k, S, n_obj, os, os, ss); break;
    }
    return int(hipGetLastError());
}

// probe_copy_waves over `bytes` (multiple of 16) with `blocks` workgroups of
// 256 lanes: host -> device or device -> host by CU loads / stores.
extern "C" int mxprobe_copy_waves(void* dst, const void* src, uint64_t bytes, int blocks, void* stream) {
    if ((bytes & 15) || blocks < 1 || ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15))
        return int(hipErrorInvalidValue);
    hipLaunchKernelGGL(probe_copy_waves, dim3(uint32_t(blocks)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<const u32x4*>(src), static_cast<u32x4*>(dst), bytes / 16);
    return int(hipGetLastError());
}

// Workgroups per CU of the copy / read / read2_write1 / write probes (1-4096).
extern "C" int mxprobe_set_stream_wpc(int wpc) {
    if (wpc < 1 || wpc > 4096) return int(hipErrorInvalidValue);
    g_stream_wpc = wpc;
    return 0;
}
