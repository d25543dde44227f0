// sha_step_lab: cycles per step of SHA-256 step programs on one wave64
// (can a message split over four lanes beat the lag pair
// form's 9 VALU per step?).  Every variant runs 64 steps per block with the
// product's dependency structure (an 8-slot ring, the new value of step t
// feeding step t + 1), per-lane operands loaded from memory so nothing folds,
// and times itself with s_memtime (core clock).  Variants:
//   9   the product's lag pair step (sha256_kernel.hip compress_lag): 3
//       v_alignbit, v_bitop3 XOR3, selector, Ch, v_xad, v_add_dpp, v_add3
//   9x2 the same step for two independent messages interleaved in each lane
//       (18 VALU per step): what the chain leaves of the wave's issue rate
//   8q  the best four-lane step found: 3 v_alignbit, XOR3, Ch
//       (one table), v_add3, v_xad, and the sum across lanes as a
//       v_add_dpp ON the chain (x' = v + swap(v))
//   7   the pair step without the H preparation (no v_xad, no v_add_dpp):
//       a floor no two-side form reaches (the other side's d and K + W must
//       enter somewhere)
//   6   the E side alone (no selector either): the one-table floor
// Launch: `waves` waves of one workgroup (1: one SIMD; 4: one per SIMD;
// 8: two per SIMD).
//   sha_step_lab [blocks]   -> one JSON line per (variant, waves)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) {
    return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);
}
#define QDPP(x, ctrl) uint32_t(__builtin_amdgcn_update_dpp(0, int(x), (ctrl), 0xF, 0xF, true))
constexpr int kSwap = 0xB1;  // quad_perm [1, 0, 3, 2]

__device__ __forceinline__ uint32_t xad(uint32_t x, uint32_t m, uint32_t c) {
    uint32_t r = (x ^ m) + c;
    asm("" : "+v"(r));
    return r;
}

struct Lane {
    uint32_t sh1, sh2, sh3, ma;
};

// One block of the product's lag step (compress_lag's loop).
__device__ __forceinline__ void block9(uint32_t (&x)[8], const u32x4 (&v)[16], const Lane& q) {
    uint32_t H = QDPP(x[7], kSwap) + xad(x[5], q.ma, v[0][0]);
    uint32_t xc = xad(x[6], q.ma, v[0][1]);
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        const uint32_t X0 = x[t & 7], X1 = x[(t + 7) & 7], X2 = x[(t + 6) & 7];
        const uint32_t S = xor3(rotr(X0, q.sh1), rotr(X0, q.sh2), rotr(X0, q.sh3));
        const uint32_t sel = __builtin_amdgcn_bitop3_b32(X0, X1, q.ma, 0xD2);
        uint32_t Hn = QDPP(X0, kSwap) + xc;
        asm("" : "+v"(Hn));
        const int u = (t + 2) & 63;
        xc = xad(X1, q.ma, v[u >> 2][u & 3]);
        x[(t + 1) & 7] = S + bsel(sel, X1, X2) + H;
        H = Hn;
    }
}

__device__ __forceinline__ void block8q(uint32_t (&x)[8], const u32x4 (&v)[16], const Lane& q) {
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        const uint32_t X0 = x[t & 7], X1 = x[(t + 7) & 7], X2 = x[(t + 6) & 7], X3 = x[(t + 5) & 7];
        const uint32_t S = xor3(rotr(X0, q.sh1), rotr(X0, q.sh2), rotr(X0, q.sh3));
        const uint32_t xc = xad(X3, q.ma, v[t >> 2][t & 3]);
        uint32_t V = S + bsel(X0, X1, X2) + xc;
        asm("" : "+v"(V));  // one v_add3, then the cross-lane sum on the chain
        uint32_t Xn = V + QDPP(V, kSwap);
        asm("" : "+v"(Xn));
        x[(t + 1) & 7] = Xn;
    }
}

__device__ __forceinline__ void block7(uint32_t (&x)[8], const u32x4 (&v)[16], const Lane& q) {
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        const uint32_t X0 = x[t & 7], X1 = x[(t + 7) & 7], X2 = x[(t + 6) & 7];
        const uint32_t S = xor3(rotr(X0, q.sh1), rotr(X0, q.sh2), rotr(X0, q.sh3));
        const uint32_t sel = __builtin_amdgcn_bitop3_b32(X0, X1, q.ma, 0xD2);
        x[(t + 1) & 7] = S + bsel(sel, X1, X2) + v[t >> 2][t & 3];
    }
}

__device__ __forceinline__ void block6(uint32_t (&x)[8], const u32x4 (&v)[16], const Lane& q) {
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        const uint32_t X0 = x[t & 7], X1 = x[(t + 7) & 7], X2 = x[(t + 6) & 7];
        const uint32_t S = xor3(rotr(X0, q.sh1), rotr(X0, q.sh2), rotr(X0, q.sh3));
        x[(t + 1) & 7] = S + bsel(X0, X1, X2) + v[t >> 2][t & 3];
    }
}

template <int VAR>
__global__ __launch_bounds__(512) void step_lab(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int blocks,
                                               unsigned long long* __restrict__ cyc) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Lane q;
    q.sh1 = in[lane & 1 ? 1 : 0];
    q.sh2 = in[lane & 1 ? 3 : 2];
    q.sh3 = in[lane & 1 ? 5 : 4];
    q.ma = in[6 + (lane & 1)];
    u32x4 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = u32x4{in[8 + i * 4], in[9 + i * 4], in[10 + i * 4], in[11 + i * 4]} + lane;
    uint32_t x[8], y[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        x[i] = in[72 + i] ^ threadIdx.x;
        y[i] = in[80 + i] ^ threadIdx.x;
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int b = 0; b < blocks; ++b) {
        if constexpr (VAR == 9) block9(x, v, q);
        if constexpr (VAR == 18) {  // two messages interleaved: the compiler schedules both chains together
            block9(x, v, q);
            block9(y, v, q);
        }
        if constexpr (VAR == 8) block8q(x, v, q);
        if constexpr (VAR == 7) block7(x, v, q);
        if constexpr (VAR == 6) block6(x, v, q);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i] + y[i];
    out[threadIdx.x] = s;
    if (lane == 0) cyc[wave] = t1 - t0;
}

template <int VAR>
void run(const uint32_t* in, uint32_t* out, unsigned long long* cyc, int blocks, int waves, const char* name,
         double ops) {
    unsigned long long h[8] = {};
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(step_lab<VAR>, dim3(1), dim3(64 * waves), 0, 0, in, out, blocks, cyc);
        (void)hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    }
    double worst = 0;
    for (int w = 0; w < waves; ++w) worst = double(h[w]) > worst ? double(h[w]) : worst;
    const double steps = double(blocks) * 64.0;  // 9x2: both messages advance one step
    printf("{\"variant\": \"%s\", \"waves\": %d, \"valu_per_step\": %.0f, \"cycles_per_step\": %.2f, "
           "\"cycles_per_valu\": %.2f}\n",
           name, waves, ops, worst / steps, worst / steps / ops);
    fflush(stdout);
}

}  // namespace

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 2048;
    uint32_t hin[96];
    const uint32_t sh[6] = {6, 2, 11, 13, 25, 22};
    for (int i = 0; i < 6; ++i) hin[i] = sh[i];
    hin[6] = 0;
    hin[7] = ~0u;
    for (int i = 8; i < 96; ++i) hin[i] = 0x9E3779B9u * uint32_t(i);
    uint32_t *in, *out;
    unsigned long long* cyc;
    (void)hipMalloc(&in, sizeof hin);
    (void)hipMalloc(&out, 512 * 4);
    (void)hipMalloc(&cyc, 8 * 8);
    (void)hipMemcpy(in, hin, sizeof hin, hipMemcpyHostToDevice);
    for (int waves : {1, 4, 8}) {
        run<9>(in, out, cyc, blocks, waves, "9 lag pair (product)", 9);
        run<18>(in, out, cyc, blocks, waves, "9x2 two messages per lane", 18);
        run<8>(in, out, cyc, blocks, waves, "8q four-lane, dpp on chain", 8);
        run<7>(in, out, cyc, blocks, waves, "7 pair without H prep", 7);
        run<6>(in, out, cyc, blocks, waves, "6 one side, one table", 6);
    }
    return 0;
}
