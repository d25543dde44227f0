// sha256_kernel.hip — batched SHA-256 (FIPS 180-4) for gfx950.
//
// Replaces Sha256::digest (sha2 0.10.9) at filesystem.rs:1070 (write_chunk),
// :1131 (parity shards) and chunk_reader.rs:108 / :184 (verify on read).
//
// SHA-256 of one message is a serial chain of 64-byte compressions, so the
// parallelism is across messages, plus what a round's two halves offer.  The
// 64 rounds are fully unrolled, rotates are v_alignbit_b32, Σ/σ XOR3, Ch and
// Maj are one v_bitop3_b32 each (14 VALU per round on one lane).  Forms, by
// batch size: the lag quad form (up to 48 messages per CU: a producer wave
// computes K + W, each message's e-side and a-side rounds run on two lanes of
// a consumer wave, the a-side two rounds behind, 9 VALU per step; the default
// latency form, with a piece mode that carries chains across launches), the
// same-round quad form (lab A/B), the split (producer / consumer) form with
// one lane per message, one wave per 64 messages, and the persistent stream
// form for batches of more groups than the chip has SIMDs (below).  Per
// message the work is a VALU-latency chain (see DESIGN.md for the roofline),
// not HBM-bound.
#include <cstdlib>
#include <cstring>

#include "hash_device.hpp"
#include "kernels.hpp"

namespace mxec {
namespace {

using namespace hashdev;

// Wave priority of the hash waves.  A hash wave issues one VALU every ~4.5
// cycles for tens of ms; decode waves sharing its SIMD (the speculative
// rebuild beside the combined hash, capi.cpp) should take the remaining
// issue slots rather than stretch the chain.
__device__ __forceinline__ void sha_priority(uint32_t prio) {
    if (prio >= 3) __builtin_amdgcn_s_setprio(3);
    else if (prio == 2) __builtin_amdgcn_s_setprio(2);
    else if (prio == 1) __builtin_amdgcn_s_setprio(1);
}

__global__ __launch_bounds__(64) void sha256_kernel(const uint8_t* const* __restrict__ ptrs,
                                                    const uint64_t* __restrict__ lens,
                                                    uint8_t* __restrict__ digests,
                                                    const uint8_t* __restrict__ expected,
                                                    const uint64_t* __restrict__ exp_idx,
                                                    uint8_t* __restrict__ ok, uint32_t n, uint32_t prio) {
    sha_priority(prio);
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = ptrs[i];
    const uint64_t len = lens[i];
    const uint64_t nfull = len / 64;
    uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                      0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    uint32_t w[16];
    if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
        u32x4 cur[4], nxt[4];
        if (nfull) load_block(p, cur);
        for (uint64_t b = 0; b < nfull; ++b) {
            if (b + 1 < nfull) load_block(p + 64 * (b + 1), nxt);
            block_words(cur, w);
            compress(st, w);
#pragma unroll
            for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
        }
    } else {
        for (uint64_t b = 0; b < nfull; ++b) {
            const uint8_t* q = p + 64 * b;
#pragma unroll
            for (int t = 0; t < 16; ++t)
                w[t] = uint32_t(q[4 * t]) << 24 | uint32_t(q[4 * t + 1]) << 16 |
                       uint32_t(q[4 * t + 2]) << 8 | uint32_t(q[4 * t + 3]);
            compress(st, w);
        }
    }
    const uint32_t rem = uint32_t(len - nfull * 64);
    const uint8_t* tp = p + nfull * 64;
    const int nblk = (rem + 9 <= 64) ? 1 : 2;
    const uint64_t bits = len * 8;
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = tail_word(tp, rem, t, nblk, bits);
    compress(st, w);
    if (nblk == 2) {
#pragma unroll
        for (int t = 0; t < 16; ++t) w[t] = tail_word(tp, rem, 16 + t, nblk, bits);
        compress(st, w);
    }
    bool match = true;
    const uint64_t ei = exp_idx ? exp_idx[i] : i;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const uint32_t be = bswap(st[t]);
        if (digests) reinterpret_cast<uint32_t*>(digests + 32 * uint64_t(i))[t] = be;
        if (expected) match &= reinterpret_cast<const uint32_t*>(expected + 32 * ei)[t] == be;
    }
    if (ok) ok[i] = match ? 1 : 0;
}

// ---------------------------------------------------------------------------
// Split form for latency-bound batches (fewer messages than SIMD slots).
//
// One wave issues at most one VALU instruction every ~4 cycles, so a lone
// message's time per block is its instruction count.  The message schedule
// (W[16..63]) depends only on the message bytes, not on the state, so a
// second wave of the same workgroup computes K[t] + W[t] for block b+1 into
// LDS while the first wave runs the 64 rounds of block b: the serial wave's
// stream drops from ~1500 to ~950 instructions per block.  LDS is
// double-buffered, laid out [buf][t/4][lane] x 16 B so each ds_read_b128 /
// ds_write_b128 is 64 consecutive 16-byte slots (conflict-free).
// ---------------------------------------------------------------------------

// Ch as one v_bitop3 (0xCA = e ? f : g); t1 = (h + kw + Ch) + S1.
#define SHA_RNDKW(a, b, c, d, e, f, g, h, kw)                                       \
    do {                                                                            \
        const uint32_t hk = h + (kw) + __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);  \
        const uint32_t t1 = hk + SHA_S1(e);                                         \
        d += t1;                                                                    \
        h = t1 + SHA_S0(a) + maj(a, b, c);                                          \
    } while (0)

#define SHA_4RKW(v)                                  \
    SHA_RNDKW(a, b, c, d, e, f, g, h, (v).x);        \
    SHA_RNDKW(h, a, b, c, d, e, f, g, (v).y);        \
    SHA_RNDKW(g, h, a, b, c, d, e, f, (v).z);        \
    SHA_RNDKW(f, g, h, a, b, c, d, e, (v).w)

#define SHA_4RKW2(v)                                 \
    SHA_RNDKW(e, f, g, h, a, b, c, d, (v).x);        \
    SHA_RNDKW(d, e, f, g, h, a, b, c, (v).y);        \
    SHA_RNDKW(c, d, e, f, g, h, a, b, (v).z);        \
    SHA_RNDKW(b, c, d, e, f, g, h, a, (v).w)

// 64 rounds with K[t] + W[t] already in registers (v[q] = words 4q..4q+3).
__device__ __forceinline__ void compress_regs(uint32_t (&st)[8], const u32x4 (&v)[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int q = 0; q < 16; q += 2) {
        SHA_4RKW(v[q]);
        SHA_4RKW2(v[q + 1]);
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// The K + W of one block from LDS (kwl[q * ROW] = words 4q..4q+3).
template <int ROW = 64>
__device__ __forceinline__ void load_kw(const u32x4* kwl, u32x4 (&v)[16]) {
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = kwl[q * ROW];
}

#ifdef MXEC_LAB
// 64 rounds reading K + W from LDS: all 16 reads issued up front so their
// latency overlaps the first rounds (the split form's two-buffer ring, lab).
__device__ __forceinline__ void compress_kw(uint32_t (&st)[8], const u32x4* kwl) {
    u32x4 v[16];
    load_kw(kwl, v);
    compress_regs(st, v);
}
#endif

__constant__ uint32_t kK256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

// Producer: K + W of one block (w = its 16 big-endian words) into LDS.
template <int ROW = 64>
__device__ __forceinline__ void schedule_kw(uint32_t (&w)[16], u32x4* dst) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        uint32_t o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = 4 * q + u;
#ifndef MXEC_LAB_SHA_NOSCHED
            if (t >= 16) SHA_W(t);
#endif
            o[u] = w[t & 15] + kK256[t];
        }
        dst[q * ROW] = u32x4{o[0], o[1], o[2], o[3]};
    }
}

// Producer with two lanes per message (the lag pair form's producer waves):
// lane L = lane & 1 of the pair computes the schedule words of parity L --
// W[2s + L] at pair step s = 8 .. 31 -- so a producer wave issues ~350 VALU
// per block instead of the one-lane form's ~570 and, at two producer waves
// per workgroup, stays well ahead of the consumers (whose ~600 VALU per
// block are the chain; with one producer wave the two were neck and neck and
// the barriers cost the difference).  W[t] = σ1(W[t-2]) + W[t-7] +
// σ0(W[t-15]) + W[t-16]: t - 2 and t - 16 have the lane's own parity, t - 7
// and t - 15 the other's.  Own words sit in A[k] = W[2k + L]; the other
// parity in B, lane 0: B[k] = W[2k + 1], lane 1: B[k] = W[2k + 2], so that
//   W[2s + L] = A[s] + σ1(A[s - 1]) + B[s - 4] + σ0(B[s])   (indices mod 8)
// reads the same registers in both lanes.  After step s the pair swaps one
// word by DPP: lane 0 sends its W[2s], lane 1 its W[2s - 1] (the value of
// the step before: a v_cndmask picks which), and both store what arrives in
// B[s - 1].  Each lane writes K + W of its own words into the message's LDS
// column (rows of four words: components L and L + 2).  kown[k] = K[2k + L].
// The K + W ring's barriers (producer and consumer sides).  Diagnostic
// build `make nosync` (MXEC_LAB_SHA_NOSYNC): none at all -- every wave runs
// its loop unsynchronised (wrong digests, same work), so the form's block
// time without the barriers and the waits behind them.
#ifdef MXEC_LAB_SHA_NOSYNC
#define KW_SYNC() ((void)0)
#else
#define KW_SYNC() __syncthreads()
#endif

#define QDPP_SWAP(x) uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0xB1, 0xF, 0xF, true))  // quad_perm [1,0,3,2]

template <int ROW>
__device__ __forceinline__ void schedule_kw_pair(const uint32_t (&w)[16], bool odd, const uint32_t (&kown)[32],
                                                 uint32_t* col) {
    uint32_t A[8], B[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        A[k] = odd ? w[2 * k + 1] : w[2 * k];
        B[k] = k < 7 ? (odd ? w[2 * k + 2] : w[2 * k + 1]) : w[15];  // lane 1's B[7] (W[16]) arrives at step 8
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        col[q * ROW * 4] = A[2 * q] + kown[2 * q];
        col[q * ROW * 4 + 2] = A[2 * q + 1] + kown[2 * q + 1];
    }
#pragma unroll
    for (int s = 8; s < 32; ++s) {
        const uint32_t x = A[s & 7] + SHA_s1(A[(s - 1) & 7]) + B[(s - 4) & 7] + SHA_s0(B[s & 7]);
        const uint32_t prev = A[(s - 1) & 7];
        A[s & 7] = x;
        if (s < 31) B[(s - 1) & 7] = QDPP_SWAP(odd ? prev : x);
        if (s & 1) {  // row (s - 1) / 2 has both of this lane's words
            const int q = s >> 1;
            col[q * ROW * 4] = prev + kown[s - 1];
            col[q * ROW * 4 + 2] = x + kown[s];
        }
    }
}

__device__ __forceinline__ void message_words(const uint8_t* p, bool aligned, uint32_t (&w)[16]) {
    if (aligned) {
        u32x4 blk[4];
        load_block(p, blk);
        block_words(blk, w);
    } else {
        // Global, not flat, byte loads: a pending flat load makes the
        // compiler drain vmcnt to 0 before every later use of a load result,
        // which would also wait out the producer's prefetch ring.
        typedef const uint8_t __attribute__((address_space(1)))* gbyte;
        const gbyte q = (gbyte)(p);
#pragma unroll
        for (int t = 0; t < 16; ++t)
            w[t] = uint32_t(q[4 * t]) << 24 | uint32_t(q[4 * t + 1]) << 16 |
                   uint32_t(q[4 * t + 2]) << 8 | uint32_t(q[4 * t + 3]);
    }
}

constexpr int kShaPrefetch = 4;
__device__ __forceinline__ uint64_t min_u64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// The producer wave of the split and quad forms: K + W of blocks 0 .. nmax-1
// of the wave's 64 messages (one per lane; `live` lanes with `nfull` full
// blocks each) into the NB-buffer LDS ring kw[NB][16][ROW] at column `lane`.
// Blocks 0 .. NB-2 are written before a first barrier, block b + NB - 1
// before the barrier that opens block b: 1 + nmax barriers in all, which the
// consumer waves match.
// PAIR2: two lanes per message (schedule_kw_pair; lane & 1 = the parity,
// `col` = the message's LDS column); otherwise one lane per message in column
// `lane` (schedule_kw).
// With PAIR2 a producer wave holds half of the workgroup's messages, so the
// workgroup-wide facts come from the caller: `wg_donor`, a message of nmax
// blocks (the re-read target of lanes without blocks), and `wg_aligned`,
// whether every message of the workgroup is 16-byte aligned.
template <int NB, int ROW, bool PAIR2 = false>
__device__ __forceinline__ void kw_producer(u32x4* kw, uint32_t lane, bool live, const uint8_t* p,
                                            uint64_t nfull, uint64_t nmax, bool aligned, uint32_t col = 0,
                                            const uint8_t* wg_donor = nullptr, bool wg_aligned = true) {
    constexpr int AHEAD = NB - 1;  // blocks the producer runs ahead of the consumer
    constexpr int BUF = 16 * ROW;  // u32x4 per buffer
    uint32_t w[16];
    const bool odd = (lane & 1) != 0;
    uint32_t kown[32];  // K[2k + parity] (PAIR2)
    if constexpr (PAIR2) {
#pragma unroll
        for (int k = 0; k < 32; ++k) kown[k] = odd ? kK256[2 * k + 1] : kK256[2 * k];
    }
    auto schedule = [&](uint32_t buf) {
        if constexpr (PAIR2)
            schedule_kw_pair<ROW>(w, odd, kown, reinterpret_cast<uint32_t*>(kw + buf * BUF + col) + (odd ? 1 : 0));
        else
            schedule_kw<ROW>(w, kw + buf * BUF + lane);
    };
    if (PAIR2 ? wg_aligned : __all(!live || nfull == 0 || aligned)) {
        // Every message 16-byte aligned: the raw bytes of the next
        // kShaPrefetch blocks stay in flight across the barriers in a
        // register ring indexed at compile time (the loop is unrolled by the
        // ring size), so the producer's step is the schedule alone.  One
        // block ahead was not enough for a lone workgroup: with the chip
        // otherwise idle a load's round trip can outlast a 1.8 us step, and
        // the consumer then waited at the barrier (29-52 ms for one 1 MiB
        // message, run to run).  Every load is unconditional -- lanes past
        // their last block re-read it, lanes without one read a donor lane's
        // -- because a load under a branch makes the compiler's wait before
        // the next use drain every load in flight (it cannot count the ones
        // that may have been skipped).  Blocks at or past nmax are scheduled
        // into buffers nobody reads as a real block.
        const uint8_t* dp = wg_donor;
        if constexpr (!PAIR2) {
            const uint64_t donor_mask = __ballot(nfull == nmax);
            const int donor = __ffsll((unsigned long long)donor_mask) - 1;
            dp = reinterpret_cast<const uint8_t*>(__shfl(reinterpret_cast<uintptr_t>(p), donor));
        }
        const bool own = live && nfull > 0;
        const uint8_t* ps = own ? p : dp;
        const uint64_t last = (own ? nfull : nmax) - 1;  // nmax > 0 when the loop runs
        u32x4 ring[kShaPrefetch][4];
        if (nmax > 0) {
            u32x4 blk[AHEAD][4];
#pragma unroll
            for (int j = 0; j < AHEAD; ++j) load_block(ps + 64 * min_u64(j, last), blk[j]);
#pragma unroll
            for (int j = 0; j < kShaPrefetch; ++j) load_block(ps + 64 * min_u64(j + AHEAD, last), ring[j]);
#pragma unroll
            for (int j = 0; j < AHEAD; ++j) {
                block_words(blk[j], w);
                schedule(uint32_t(j));
            }
        }
        KW_SYNC();
        // Whole groups of kShaPrefetch steps, then the rest: an exit in the
        // middle of a group would join the loop's back edge with fewer loads
        // issued, and the waits at the top would drain the ring again.
        uint32_t wb = AHEAD % NB;  // buffer of block b + AHEAD
        uint64_t b0 = 0;
        for (; b0 + kShaPrefetch <= nmax; b0 += kShaPrefetch) {
#pragma unroll
            for (int j = 0; j < kShaPrefetch; ++j) {
                const uint64_t b = b0 + j;
                // ring[j] holds block b + AHEAD (or a clamped re-read nobody
                // consumes: lanes compress only blocks below their nfull).
                block_words(ring[j], w);
                load_block(ps + 64 * min_u64(b + AHEAD + kShaPrefetch, last), ring[j]);
                schedule(wb);
                wb = wb + 1 == NB ? 0 : wb + 1;
                KW_SYNC();
            }
        }
#pragma unroll
        for (int j = 0; j < kShaPrefetch - 1; ++j) {  // the ring already holds these blocks
            if (b0 + j < nmax) {
                block_words(ring[j], w);
                schedule(wb);
                wb = wb + 1 == NB ? 0 : wb + 1;
                KW_SYNC();
            }
        }
    } else {
        // An unaligned message in the wave: byte loads, one block at a time.
#pragma unroll
        for (int j = 0; j < AHEAD; ++j)
            if (uint64_t(j) < nfull) {
                message_words(p + 64 * j, aligned, w);
                schedule(uint32_t(j));
            }
        KW_SYNC();
        uint32_t wb = AHEAD % NB;
        for (uint64_t b = 0; b < nmax; ++b) {
            if (b + AHEAD < nfull) {
                message_words(p + 64 * (b + AHEAD), aligned, w);
                schedule(wb);
            }
            wb = wb + 1 == NB ? 0 : wb + 1;
            KW_SYNC();
        }
    }
}

// NB = 3 (default): the producer runs two blocks ahead, so the consumer
// issues block b+1's 16 LDS reads right after the barrier that opens block b
// and runs block b's rounds from registers: no read latency at the top of a
// block and one wait per block instead of one per four rounds.  NB = 2 is
// the earlier one-ahead form (MXEC_SHA_SPLIT_BUFS=2, lab).  Buffer of block
// b: b % NB; 16 KiB each.
template <int NB>
__global__ __launch_bounds__(128) void sha256_split_kernel(const uint8_t* const* __restrict__ ptrs,
                                                           const uint64_t* __restrict__ lens,
                                                           uint8_t* __restrict__ digests,
                                                           const uint8_t* __restrict__ expected,
                                                           const uint64_t* __restrict__ exp_idx,
                                                           uint8_t* __restrict__ ok, uint32_t n, uint32_t prio) {
    static_assert(NB == 2 || NB == 3, "two or three K+W buffers");
    sha_priority(prio);
    __shared__ u32x4 kw[NB][16][64];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * 64 + lane;
    const bool live = i < n;
    const uint8_t* p = live ? ptrs[i] : nullptr;
    const uint64_t len = live ? lens[i] : 0;
    const uint64_t nfull = len / 64;
    const bool aligned = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
    // Both waves serve the same 64 messages, so this trip count is the same
    // in both and every barrier below is reached by both.
    uint64_t nmax = nfull;
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        const uint64_t o = __shfl_xor(nmax, s);
        nmax = o > nmax ? o : nmax;
    }
    // Equal in every lane now; say so, so the loops below branch on scalars
    // (a divergent loop exit would make every prefetch load conditional).
    nmax = (uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(nmax >> 32))) << 32) |
           __builtin_amdgcn_readfirstlane(uint32_t(nmax));
    uint32_t w[16];
    uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                      0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    // The two roles run separate loops with one barrier per block each plus
    // one before the first (the trip counts match, so the barriers pair up).
    if (wave == 0) {
        KW_SYNC();
        if constexpr (NB == 2) {
#ifdef MXEC_LAB
            for (uint64_t b = 0; b < nmax; ++b) {
                if (b < nfull) compress_kw(st, &kw[b & 1][0][lane]);
                KW_SYNC();
            }
#endif
        } else {
            // Blocks 0 and 1 were written before the first barrier; block
            // b+1 before the barrier that opens block b.  Two register sets
            // swap roles every block (the loop is unrolled by two), and the
            // reads of a block past the last land in registers nobody uses.
            u32x4 cur[16], nxt[16];
            load_kw(&kw[0][0][lane], cur);
            // Retire these reads here: otherwise the loop's first wait, sized
            // for 32 reads in flight on entry, also stalls every later block
            // on its just-issued prefetch (lgkmcnt counts to 15).
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
            uint32_t rb = 1;  // buffer of the block after the current one
            for (uint64_t b = 0; b < nmax; b += 2) {
                load_kw(&kw[rb][0][lane], nxt);
                if (b < nfull) compress_regs(st, cur);
                KW_SYNC();
                rb = rb == 2 ? 0 : rb + 1;
                if (b + 1 >= nmax) break;
                load_kw(&kw[rb][0][lane], cur);
                if (b + 1 < nfull) compress_regs(st, nxt);
                KW_SYNC();
                rb = rb == 2 ? 0 : rb + 1;
            }
        }
    } else {
        kw_producer<NB, 64>(&kw[0][0][0], lane, live, p, nfull, nmax, aligned);
    }
    if (wave == 1 || !live) return;
    const uint32_t rem = uint32_t(len - nfull * 64);
    const uint8_t* tp = p + nfull * 64;
    const int nblk = (rem + 9 <= 64) ? 1 : 2;
    const uint64_t bits = len * 8;
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = tail_word(tp, rem, t, nblk, bits);
    compress(st, w);
    if (nblk == 2) {
#pragma unroll
        for (int t = 0; t < 16; ++t) w[t] = tail_word(tp, rem, 16 + t, nblk, bits);
        compress(st, w);
    }
    bool match = true;
    const uint64_t ei = exp_idx ? exp_idx[i] : i;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const uint32_t be = bswap(st[t]);
        if (digests) reinterpret_cast<uint32_t*>(digests + 32 * uint64_t(i))[t] = be;
        if (expected) match &= reinterpret_cast<const uint32_t*>(expected + 32 * ei)[t] == be;
    }
    if (ok) ok[i] = match ? 1 : 0;
}

// ---------------------------------------------------------------------------
// Quad form for latency-bound batches (at most 48 messages per CU).
//
// The split form's consumer sits on the one-lane floor: 14 VALU per round
// (Σ1, Ch, Σ0, Maj, the adds), issued one every ~4.4 cycles by one wave.
// Here four lanes of a consumer wave serve one message, and the e-side and
// a-side halves of a round run as the SAME instructions in two lanes with
// per-lane operands:
//   lane E (4j):       X = e, rotations 6/11/25 -> Σ1(e); Ch(e, f, g)
//   lane A (4j + 1):   X = a, rotations 2/13/22 -> Σ0(a); Maj(a, b, c)
//   lanes 4j + 2, + 3: all zero (the zero source of the DPP reads below).
// Maj(a, b, c) = Ch(~(a ^ b), b, c), so one v_bitop3 makes the selector
// (e in lane E, ~(a ^ b) in lane A) and one more is Ch in both lanes.  With
// H = h + d + K + W in lane E and -d in lane A,
//   P  = Σ + Ch + H       is d + T1 = e' in lane E and T2 - d in lane A;
//   X' = P + P[lane E]    (one v_add_u32 with a quad_perm DPP source)
// is e' in lane E (its DPP source is a zero lane) and T1 + T2 = a' in lane A.
// The next round's H is X[t-2] + X[t-2][lane A] (h + d in lane E, d in lane
// A: DPP again), then one v_xad_u32: xor with a per-lane mask (all ones in
// lane A: ~d + 1 = -d) plus the K + W word (K + W in lane E, 1 in lane A, 0
// in the zero lanes).  10 VALU per round instead of 14; the idle lanes cost
// nothing, the chain being bound by the wave's issue rate.
//
// A workgroup is one producer wave (the split form's, kw_producer: K + W of
// 48 messages, one per lane) and three consumer waves of 16 messages each,
// so each wave has a SIMD of its own.  K + W rows are kQuadRow columns wide:
// 0..47 the producer's, 64 all zero and 65 all one, so every consumer lane
// reads its word at the same row offset from its own column.  The padded
// tail (1 or 2 blocks) runs in lane E after the main loop, one-lane form.
// ---------------------------------------------------------------------------
constexpr int kQuadRow = 66;  // u32x4 per K + W row: 64 producer lanes, zeros, ones

#define QDPP(x, ctrl) uint32_t(__builtin_amdgcn_update_dpp(0, int(x), (ctrl), 0xF, 0xF, true))
#ifdef MXEC_LAB
constexpr int kQuadFromE = 0xA2;   // quad_perm [2, 0, 2, 2]: lane A reads lane E, the rest a zero lane
constexpr int kQuadFromA = 0xA9;   // quad_perm [1, 2, 2, 2]: lane E reads lane A, the rest a zero lane
#endif
constexpr int kQuadBcastA = 0x55;  // quad_perm [1, 1, 1, 1]
constexpr int kPairBcastA = 0xF5;  // quad_perm [1, 1, 3, 3]: each message's lane A to its lane E

struct QuadLane {
    uint32_t sh1, sh2, sh3;  // rotations: Σ1's in lane E, Σ0's in lane A
    uint32_t ma;             // all ones in lane A (selector ~(a ^ b); negated d), else 0
};

#ifdef MXEC_LAB
// One block.  s[0..3] = (e, f, g, h) in lane E, (a, b, c, d) in lane A, zero
// in the zero lanes; v = the block's K + W rows as this lane reads them.
__device__ __forceinline__ void compress_quad(uint32_t (&s)[4], const u32x4 (&v)[16], const QuadLane& q) {
    uint32_t x[4];  // x[t & 3] = X[t]; X[-1], X[-2], X[-3] = s[1], s[2], s[3]
    x[0] = s[0];
    x[3] = s[1];
    x[2] = s[2];
    x[1] = s[3];
    uint32_t h = ((x[1] + QDPP(x[1], kQuadFromA)) ^ q.ma) + v[0].x;
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        const uint32_t X0 = x[t & 3], X1 = x[(t + 3) & 3], X2 = x[(t + 2) & 3];
        const uint32_t S = xor3(rotr(X0, q.sh1), rotr(X0, q.sh2), rotr(X0, q.sh3));
        const uint32_t sel = __builtin_amdgcn_bitop3_b32(X0, X1, q.ma, 0xD2);  // X0 ^ (~X1 & ma)
        const uint32_t P = S + bsel(sel, X1, X2) + h;
        if (t < 63) h = ((X2 + QDPP(X2, kQuadFromA)) ^ q.ma) + v[(t + 1) >> 2][(t + 1) & 3];
        x[(t + 1) & 3] = P + QDPP(P, kQuadFromE);
    }
    s[0] += x[0];
    s[1] += x[3];
    s[2] += x[2];
    s[3] += x[1];
}
#endif

// Lag variant (the auto quad form; MXEC_SHA_FORM=lag pins it).  Above, lane A's
// a' = T1 + T2 needs lane E's T1 of the same round, so a DPP add sits on
// every round's critical path (X -> rotations -> xor3 -> add3 -> DPP add ->
// X'): the rounds measured ~54 cycles for 10 VALU.  Here lane A runs
// TWO rounds behind lane E (tools/sha_lag_model.py is the lane-level model,
// checked against hashlib):
//   step t, lane E:  e[t+1] = Σ1(e[t]) + Ch(e[t], e[t-1], e[t-2]) + H,
//                    H = e[t-3] + a[t-3] + K[t] + W[t]         (h + d + K + W)
//   step t, lane A:  a[t-1] = Σ0(a[t-2]) + Maj(a[t-2], a[t-3], a[t-4]) + H,
//                    H = T1[t-2] = e[t-1] - a[t-5]
// With the history in an 8-slot ring x[t & 7] (X0 newest), the cross-lane
// operand of BOTH lanes is the other lane's X1 (a[t-3] for lane E, e[t-1]
// for lane A): one DPP swap of a value written a step earlier, off the
// chain.  A step is 3 alignbit + xor3 + selector + Ch + v_xad (X3 ^ mask +
// c) + v_add_dpp + add3 = 9 VALU, chain X -> alignbit -> xor3 -> add3 -> X'.
// A block is 66 steps (lane A's last two rounds run beside two unused lane-E
// values); lane A's first two outputs are forced to the known b and a, and
// lane A keeps its state rotated as (c, d, a, b) so both lanes load the ring
// from, and mostly add back, the same slots.  Lanes 2 and 3 of a quad swap
// among themselves and compute nothing anyone reads.
constexpr int kLagSwap = 0xB1;  // quad_perm [1, 0, 3, 2]

// (X3 ^ ma) + c as one v_xad: left free, the compiler sums X3 ^ ma, c and a
// v_mov_dpp with an add3 (10 VALU per step instead of 9).
__device__ __forceinline__ uint32_t lag_xc(uint32_t x3, uint32_t ma, uint32_t c) {
    uint32_t r = (x3 ^ ma) + c;
    asm("" : "+v"(r));
    return r;
}

// The step's order is the compiler's: r1 H' r2 r3 sel xc S ch P, with H'
// the NEXT step's H (DPP of this step's X0, which is step t+1's X1) and xc
// the xad of the step after that.  A lone wave issues independent VALU at
// ~5-5.8 cycles (tools/valu_lab.cpp), so 9 per step at ~46 cycles is that
// floor; a hand order spacing every on-chain pair two slots apart, held
// with sched_barriers, measured 1.48 us per block against 1.265
// (profiles/r3/sha_lag/ab_order.jsonl).
//
// `at(t)` runs at the top of step t (the caller's K + W reads for the next
// block, spread over the block: sha256_quad_kernel LDG).
struct NoStep {
    __device__ __forceinline__ void operator()(int) const {}
};
template <class AT = NoStep>
__device__ __forceinline__ void compress_lag(uint32_t (&s)[4], const u32x4 (&v)[16], const QuadLane& q,
                                             const AT& at = AT()) {
    const bool is_a = q.ma != 0;
    const uint32_t one = q.ma & 1;  // c after lane E's rounds: 1 in lane A (-X3 = ~X3 + 1), 0 elsewhere
    uint32_t x[8];
    x[0] = s[0];
    x[7] = s[1];
    x[6] = s[2];
    x[5] = s[3];
    // Step t finds its H ready and leaves H[t+1] (DPP of its own X0,
    // which is step t+1's X1) and xc[t+2] (X3 of step t+2 is step t's
    // X1) for the steps after it.
    uint32_t H = QDPP(x[7], kLagSwap) + lag_xc(x[5], q.ma, v[0][0]);
    uint32_t xc = lag_xc(x[6], q.ma, v[0][1]);
#pragma unroll
    for (int t = 0; t < 66; ++t) {
        at(t);
        const uint32_t X0 = x[t & 7], X1 = x[(t + 7) & 7], X2 = x[(t + 6) & 7];
        const uint32_t S = xor3(rotr(X0, q.sh1), rotr(X0, q.sh2), rotr(X0, q.sh3));
        const uint32_t sel = __builtin_amdgcn_bitop3_b32(X0, X1, q.ma, 0xD2);  // X0 ^ (~X1 & ma)
        uint32_t Hn = QDPP(X0, kLagSwap) + xc;
        asm("" : "+v"(Hn));  // one v_add_u32_dpp (not reassociated into the add3)
        const int u = t + 2;
        xc = lag_xc(X1, q.ma, u < 64 ? v[u >> 2][u & 3] : one);
        uint32_t P = S + bsel(sel, X1, X2) + H;
        if (t == 0) P = is_a ? s[3] : P;  // b = a[-1]
        if (t == 1) P = is_a ? s[2] : P;  // a = a[0]
        x[(t + 1) & 7] = P;
        H = Hn;
    }
    // Lane E: e[64], e[63], e[62], e[61] in x[0], x[7], x[6], x[5];
    // lane A: a[62], a[61], a[64], a[63] in x[0], x[7], x[2], x[1].
    s[0] += x[0];
    s[1] += x[7];
    s[2] += is_a ? x[2] : x[6];
    s[3] += is_a ? x[1] : x[5];
}

// LAG: compress_lag (default) or the same-round compress_quad (lab A/B).
// PAIR (lag only; MXEC_SHA_FORM=lagpair, lab): two messages per quad -- the
// lag form needs no zero lanes, so lanes 4j+2 / 4j+3 run a second message's
// E and A sides -- and a workgroup is the producer wave (64 messages) plus two
// consumer waves of 32: 64 messages per workgroup of three waves.
// P2 (PAIR only; the auto form): two producer waves of 32 messages, two
// lanes per message (schedule_kw_pair), waves 0-1; consumers waves 2-3: a
// workgroup of four waves, one per SIMD.
// LDG (lag forms): the next block's 16 ds_read_b128 of K + W go out in LDG
// groups spread over the current block -- group g at the top of step
// 64 g / LDG -- instead of all 16 right after the barrier.  A wave may hold
// at most 15 LDS instructions in flight (lgkmcnt is 4 bits), so the 16th
// read of a burst waited for the first to come back, and the in-order wave
// issued no VALU meanwhile (round 5: ~260 cycles per block above the step
// lab's 66 x 37.4).
template <bool LAG, bool PAIR = false, bool P2 = false, int LDG = 1>
__global__ __launch_bounds__(256) void sha256_quad_kernel(const uint8_t* const* __restrict__ ptrs,
                                                         const uint64_t* __restrict__ lens,
                                                         uint8_t* __restrict__ digests,
                                                         const uint8_t* __restrict__ expected,
                                                         const uint64_t* __restrict__ exp_idx,
                                                         uint8_t* __restrict__ ok, uint32_t n, uint32_t prio,
                                                         ShaPiece pc) {
    static_assert(LAG || !PAIR, "two messages per quad needs the lag form (no zero lanes)");
    static_assert(PAIR || !P2, "two producer waves serve the two-messages-per-quad consumers");
    constexpr uint32_t PW = P2 ? 2 : 1;  // producer waves
    constexpr int NB = 3, BUF = 16 * kQuadRow;
    constexpr uint32_t MSGS = PAIR ? 64 : kShaQuadMsgs;  // messages per workgroup
    sha_priority(prio);
    __shared__ u32x4 kw[NB][16][kQuadRow];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x < NB * 16 * 2) {  // the constant columns; the first barrier publishes them
        const uint32_t r = threadIdx.x >> 1, c = threadIdx.x & 1;
        kw[r / 16][r % 16][64 + c] = u32x4{c, c, c, c};
    }
    const uint32_t base = blockIdx.x * MSGS;
    // Every wave derives the same trip count from the workgroup's messages
    // (one per lane below kShaQuadMsgs), so the barriers pair up.
    const uint32_t pi = base + lane;
    const bool plive = lane < MSGS && pi < n;
    const uint8_t* pp = plive ? ptrs[pi] : nullptr;
    const uint64_t pfull = plive ? lens[pi] / 64 : 0;
    uint64_t nmax = pfull;
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        const uint64_t o = __shfl_xor(nmax, s);
        nmax = o > nmax ? o : nmax;
    }
    nmax = (uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(nmax >> 32))) << 32) |
           __builtin_amdgcn_readfirstlane(uint32_t(nmax));
    if constexpr (P2) {
        if (wave < PW) {  // producer wave `wave`: messages 32 * wave + lane / 2, two lanes each
            // The workgroup-wide donor and alignment, from the one-lane-per-
            // message view (pi = base + lane) every wave holds.
            const uint64_t dmask = __ballot(plive && pfull == nmax);
            const int dl = dmask ? __ffsll((unsigned long long)dmask) - 1 : 0;
            const uint8_t* wdonor = reinterpret_cast<const uint8_t*>(__shfl(reinterpret_cast<uintptr_t>(pp), dl));
            const bool waligned = __all(!plive || pfull == 0 || (reinterpret_cast<uintptr_t>(pp) & 15) == 0);
            const uint32_t mi = wave * 32 + (lane >> 1), qi = base + mi;
            const bool qlive = qi < n;
            const uint8_t* qp = qlive ? ptrs[qi] : nullptr;
            const uint64_t qfull = qlive ? lens[qi] / 64 : 0;
            kw_producer<NB, kQuadRow, true>(&kw[0][0][0], lane, qlive, qp, qfull, nmax,
                                            (reinterpret_cast<uintptr_t>(qp) & 15) == 0, mi, wdonor, waligned);
            return;
        }
    } else if (wave == 0) {
        kw_producer<NB, kQuadRow>(&kw[0][0][0], lane, plive, pp, pfull, nmax,
                                  (reinterpret_cast<uintptr_t>(pp) & 15) == 0);
        return;
    }
    const uint32_t role = PAIR ? lane & 1 : lane & 3;
    const uint32_t ml = PAIR ? (wave - PW) * 32 + (lane >> 1) : (wave - 1) * 16 + (lane >> 2);
    const uint32_t i = base + ml;
    const bool live = i < n;
    const uint8_t* p = live ? ptrs[i] : nullptr;
    const uint64_t len = live ? lens[i] : 0;
    const uint64_t nfull = len / 64;
    QuadLane q;
    q.sh1 = role == 0 ? 6 : 2;
    q.sh2 = role == 0 ? 11 : 13;
    q.sh3 = role == 0 ? 25 : 22;
    q.ma = role == 1 ? ~0u : 0u;
    // Piece mode: the launch's message i is state slot pc.slot[i] (digest,
    // ok and running state are indexed by the slot).
    const uint32_t slot = live && pc.state ? pc.slot[i] : i;
    uint32_t s[4] = {0, 0, 0, 0};
    if (live && pc.state && pc.resume && role < 2) {  // continue the chain (a..h in state[slot])
        const uint32_t* sv = pc.state + 8 * uint64_t(slot);
        if (role == 0) {
            s[0] = sv[4]; s[1] = sv[5]; s[2] = sv[6]; s[3] = sv[7];
        } else if (LAG) {  // (c, d, a, b)
            s[0] = sv[2]; s[1] = sv[3]; s[2] = sv[0]; s[3] = sv[1];
        } else {
            s[0] = sv[0]; s[1] = sv[1]; s[2] = sv[2]; s[3] = sv[3];
        }
    } else if (role == 0) {
        s[0] = 0x510e527fu; s[1] = 0x9b05688cu; s[2] = 0x1f83d9abu; s[3] = 0x5be0cd19u;
    } else if (role == 1 && LAG) {  // (c, d, a, b)
        s[0] = 0x3c6ef372u; s[1] = 0xa54ff53au; s[2] = 0x6a09e667u; s[3] = 0xbb67ae85u;
    } else if (role == 1) {
        s[0] = 0x6a09e667u; s[1] = 0xbb67ae85u; s[2] = 0x3c6ef372u; s[3] = 0xa54ff53au;
    }
    const u32x4* kcol = &kw[0][0][role == 0 ? ml : role == 1 ? 65 : 64];
    // As the split form's NB = 3 consumer: block b + 1's reads go out right
    // after the barrier that opens block b, block b runs from registers.
    KW_SYNC();
    u32x4 cur[16], nxt[16];
    load_kw<kQuadRow>(kcol, cur);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    static_assert(LDG == 1 || LDG == 2 || LDG == 4 || LDG == 15, "K + W read groups: 1, 2, 4 or 15 + 1");
    // LDG 15: rows 0-14 after the barrier, row 15 at the top of step 2 (a
    // burst of 15 fits lgkmcnt; the 16th no longer waits for the first).
    constexpr int NG = LDG == 15 ? 2 : LDG;  // read groups
    constexpr int RPG = 16 / NG;             // rows per read group (LDG 1, 2, 4)
    // Group g's rows of the block in ring buffer `buf` into `dst`.
    auto rows = [&](u32x4 (&dst)[16], uint32_t buf, int g) {
        const int r0 = LDG == 15 ? (g ? 15 : 0) : g * RPG, r1 = LDG == 15 ? (g ? 16 : 15) : (g + 1) * RPG;
#pragma unroll
        for (int r = r0; r < r1; ++r) dst[r] = kcol[buf * BUF + r * kQuadRow];
    };
    auto at_step = [&](u32x4 (&dst)[16], uint32_t buf, int t) {
        if constexpr (LDG == 15) {
            if (t == 2) rows(dst, buf, 1);
        } else if (LDG > 1 && t > 0 && t < 64 && t % (64 / LDG) == 0) {
            rows(dst, buf, t / (64 / LDG));
        }
    };
    uint32_t rb = 1;
    for (uint64_t b = 0; b < nmax; b += 2) {
        rows(nxt, rb, 0);
        if (b < nfull) {
#ifdef MXEC_LAB
            if constexpr (!LAG) {
                for (int g = 1; g < NG; ++g) rows(nxt, rb, g);
                compress_quad(s, cur, q);
            } else
#endif
            compress_lag(s, cur, q, [&](int t) { at_step(nxt, rb, t); });
        }  // a lane past its message's blocks never reads K + W again: no reads here
        KW_SYNC();
        rb = rb == 2 ? 0 : rb + 1;
        if (b + 1 >= nmax) break;
        rows(cur, rb, 0);
        if (b + 1 < nfull) {
#ifdef MXEC_LAB
            if constexpr (!LAG) {
                for (int g = 1; g < NG; ++g) rows(cur, rb, g);
                compress_quad(s, nxt, q);
            } else
#endif
            compress_lag(s, nxt, q, [&](int t) { at_step(cur, rb, t); });
        }  // a lane past its message's blocks never reads K + W again: no reads here
        KW_SYNC();
        rb = rb == 2 ? 0 : rb + 1;
    }
    // Lane E takes (a, b, c, d) from lane A and finishes alone: padded tail,
    // digest, expected-digest check.  (The lag form's lane A holds
    // (c, d, a, b).)
    uint32_t st[8];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        st[t] = QDPP(s[LAG ? (t + 2) & 3 : t], PAIR ? kPairBcastA : kQuadBcastA);
        st[4 + t] = s[t];
    }
    if (role != 0 || !live) return;
    const uint64_t total = pc.state ? pc.total[i] : len;
    if (total == kShaNotFinal) {  // mid-message piece: the running state goes back
        uint32_t* sv = pc.state + 8 * uint64_t(slot);
#pragma unroll
        for (int t = 0; t < 8; ++t) sv[t] = st[t];
        return;
    }
    const uint32_t rem = uint32_t(len - nfull * 64);
    const uint8_t* tp = p + nfull * 64;
    const int nblk = (rem + 9 <= 64) ? 1 : 2;
    const uint64_t bits = total * 8;
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = tail_word(tp, rem, t, nblk, bits);
    compress(st, w);
    if (nblk == 2) {
#pragma unroll
        for (int t = 0; t < 16; ++t) w[t] = tail_word(tp, rem, 16 + t, nblk, bits);
        compress(st, w);
    }
    bool match = true;
    const uint64_t ei = exp_idx ? exp_idx[slot] : slot;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const uint32_t be = bswap(st[t]);
        if (digests) reinterpret_cast<uint32_t*>(digests + 32 * uint64_t(slot))[t] = be;
        if (expected) match &= reinterpret_cast<const uint32_t*>(expected + 32 * ei)[t] == be;
    }
    if (ok) ok[slot] = match ? 1 : 0;
}

// ---------------------------------------------------------------------------
// Stream form for batches with more 64-message groups than 3/4 of the chip's
// SIMDs (e.g. config 3c: eight concurrent 10 240-chunk verifications = 1 280
// groups on 1 024 SIMDs).  Whole-chain scheduling ends with the SIMDs that
// hold two groups running at half speed while the rest idle (81 920 x 1 MiB:
// 78-96 ms split form vs 53 for 65 536).  Here a group's chain is cut into
// segments of kShaSegBlocks blocks; persistent waves (one per SIMD, four per
// workgroup so each lands on its own SIMD) take (group, segment) items from a
// counter in segment-major order, so a SIMD that finishes early takes the next
// segment of some other group and the load evens out to within one segment.
//
// Hand-off between the waves that run consecutive segments of a group
// (MI355X_MICROARCH.md, visibility; cdna_hip_programming.md Guideline 16,
// recipe R1): each lane stores its 8 state words with agent-scope relaxed
// atomic stores (write-through), the wave drains them (vmcnt(0)), then every
// lane stores the same value to the group's progress word (agent-scope
// relaxed); the next wave polls that word with all lanes (relaxed, s_sleep,
// bounded), then one agent acquire, then the lanes read the state with
// agent-scope loads.  Item t's predecessor is item t - groups, taken earlier
// by a resident wave, so every wait ends; a wave that still waits 4 s
// (s_memrealtime) gives up, leaves kShaStreamTimeout in work[1] and every
// other wave drains the queue without hashing (the host checks the word).
// ---------------------------------------------------------------------------
typedef uint32_t __attribute__((address_space(1))) gu32;

// A wait gives up after this many ticks of the 100 MHz s_memrealtime clock
// (4 s): a predecessor segment takes ~1.4 ms, so only a fault gets there.
#ifndef SHA_STREAM_WAIT_TICKS
#define SHA_STREAM_WAIT_TICKS (400ull * 1000 * 1000)
#endif
// Lab builds (tools/sha_stream_lab) define SHA_STREAM_DEBUG: per item, eight
// words after the n x 8 state words record (taken, waited ok, progress word
// seen, published, and s_memtime / 16 at start, publish, wait end, loop end).
#ifdef SHA_STREAM_DEBUG
#define SHA_DBG(t, k, v) (state_p[uint64_t(n) * 8 + uint64_t(t) * 8 + (k)] = (v))
#else
#define SHA_DBG(t, k, v) ((void)0)
#endif

__device__ __forceinline__ uint32_t prog_read(gu32* prog) {
    return __hip_atomic_load(prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave-uniform wait: every lane polls the same word (one request per
// instruction) and the exit test is on scalars, so no divergent loop sits
// inside a lane-0 branch.  (A lane-0-only spin loop let the compiler's
// control-flow structurizer fold the previous item's lane-0 publish into the
// next item's wait region: a wave with two or more live lanes then held its
// publish until its own next wait timed out — measured in
// tools/sha_stream_lab, profiles/r2_sha_stream_lab.txt.)
__device__ __forceinline__ bool stream_wait(gu32* prog, uint32_t want, gu32* tmo) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t spins = 0;; ++spins) {
        if (uint32_t(__builtin_amdgcn_readfirstlane(prog_read(prog))) == want) return true;
        if ((spins & 63) == 0) {
            if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0)
                return false;
            if (__builtin_amdgcn_s_memrealtime() - t0 > SHA_STREAM_WAIT_TICKS) {
                __hip_atomic_store(tmo, kShaStreamTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

__global__ __launch_bounds__(256) void sha256_stream_kernel(const uint8_t* const* __restrict__ ptrs,
                                                           const uint64_t* __restrict__ lens,
                                                           uint8_t* __restrict__ digests,
                                                           const uint8_t* __restrict__ expected,
                                                           const uint64_t* __restrict__ exp_idx,
                                                           uint8_t* __restrict__ ok, uint32_t n,
                                                           uint32_t* work_p, uint32_t* state_p,
                                                           uint32_t seg_max, uint32_t prio) {
    sha_priority(prio);
    gu32* work = (gu32*)(work_p);
    gu32* state = (gu32*)(state_p);
    const uint32_t lane = threadIdx.x & 63;  // every wave of a workgroup works alone
    const uint32_t groups = (n + 63) / 64;
    // The host (ops.cpp run_sha) picks this form only when n_items plus one
    // overshoot take per wave stays below 2^32, so the item counter never
    // wraps back onto item 0.
    const uint64_t n_items = uint64_t(groups) * seg_max;
    for (;;) {
        uint32_t t = 0;
        if (lane == 0) t = __hip_atomic_fetch_add(work, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t = __builtin_amdgcn_readfirstlane(t);
        if (uint64_t(t) >= n_items) break;
        const uint32_t sg = t / groups, g = t - sg * groups;
        const uint32_t i = g * 64 + lane;
        const bool live = i < n;
        const uint8_t* p = live ? ptrs[i] : nullptr;
        const uint64_t len = live ? lens[i] : 0;
        const uint64_t nfull = len / 64;
        const uint32_t last = uint32_t(nfull / kShaSegBlocks);  // the segment holding this lane's tail
        uint32_t segs = last;
#pragma unroll
        for (int x = 32; x >= 1; x >>= 1) segs = max(segs, uint32_t(__shfl_xor(int(segs), x)));
        segs = __builtin_amdgcn_readfirstlane(segs) + 1;
        if (sg >= segs) continue;  // this group has no such segment
        gu32* prog = work + 4 + g;
        if (lane == 0) SHA_DBG(t, 0, 1u + sg);
        if (lane == 0) SHA_DBG(t, 4, uint32_t(__builtin_amdgcn_s_memtime() >> 4));
        if (sg > 0) {
            const bool okw = stream_wait(prog, sg, work + 1);
            if (lane == 0) SHA_DBG(t, 1, okw ? 1u : 0u);
            if (lane == 0) SHA_DBG(t, 6, uint32_t(__builtin_amdgcn_s_memtime() >> 4));
            if (lane == 0) SHA_DBG(t, 2, prog_read(prog));
            if (!okw) continue;  // timed out: drain
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        } else if (__hip_atomic_load(work + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
            continue;  // another wave timed out: drain without hashing
        }
        uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                          0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
        gu32* my = state + uint64_t(live ? i : 0) * 8;
        if (sg > 0 && live && sg <= last) {
#pragma unroll
            for (int w = 0; w < 8; ++w) st[w] = __hip_atomic_load(my + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // Blocks [b0, b1) of this segment; the trip count is the wave's
        // longest, loads are unconditional (clamped to a block the lane
        // owns, or a donor lane's) so the prefetch is never drained by a
        // branch, and a lane compresses only its own blocks.
        const uint64_t b0 = uint64_t(sg) * kShaSegBlocks;
        const uint64_t b1 = sg <= last ? min(b0 + kShaSegBlocks, nfull) : b0;
        uint32_t cnt = uint32_t(b1 > b0 ? b1 - b0 : 0), cmax = cnt;
#pragma unroll
        for (int x = 32; x >= 1; x >>= 1) cmax = max(cmax, uint32_t(__shfl_xor(int(cmax), x)));
        cmax = __builtin_amdgcn_readfirstlane(cmax);
        if (cmax > 0) {
            const uint64_t dmask = __ballot(cnt == cmax);
            const int donor = __ffsll((unsigned long long)dmask) - 1;
            const uint8_t* dp = reinterpret_cast<const uint8_t*>(__shfl(reinterpret_cast<uintptr_t>(p), donor));
            const uint64_t db0 = uint64_t(__shfl(int64_t(b0), donor));
            const bool own = cnt > 0;
            const uint8_t* base = own ? p + 64 * b0 : dp + 64 * db0;
            const uint32_t lastb = (own ? cnt : cmax) - 1;
            u32x4 cur[4], nxt[4];
            load_block(base, cur);
            uint32_t w[16];
            for (uint32_t b = 0; b < cmax; ++b) {
                load_block(base + 64 * uint64_t(min(b + 1, lastb)), nxt);
                if (b < cnt) {
                    block_words(cur, w);
                    compress(st, w);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
            }
        }
        if (lane == 0) SHA_DBG(t, 7, uint32_t(__builtin_amdgcn_s_memtime() >> 4));
        if (live && sg == last) {
            // Padding blocks, digest, expected-digest check (as the other forms).
            const uint32_t rem = uint32_t(len - nfull * 64);
            const uint8_t* tp = p + nfull * 64;
            const int nblk = (rem + 9 <= 64) ? 1 : 2;
            const uint64_t bits = len * 8;
            uint32_t w[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) w[q] = tail_word(tp, rem, q, nblk, bits);
            compress(st, w);
            if (nblk == 2) {
#pragma unroll
                for (int q = 0; q < 16; ++q) w[q] = tail_word(tp, rem, 16 + q, nblk, bits);
                compress(st, w);
            }
            bool match = true;
            const uint64_t ei = exp_idx ? exp_idx[i] : i;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint32_t be = bswap(st[q]);
                if (digests) reinterpret_cast<uint32_t*>(digests + 32 * uint64_t(i))[q] = be;
                if (expected) match &= reinterpret_cast<const uint32_t*>(expected + 32 * ei)[q] == be;
            }
            if (ok) ok[i] = match ? 1 : 0;
        } else if (live && sg < last) {
#pragma unroll
            for (int q = 0; q < 8; ++q) __hip_atomic_store(my + q, st[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (sg + 1 < segs) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every lane's state stores have landed
            if (lane == 0) SHA_DBG(t, 5, uint32_t(__builtin_amdgcn_s_memtime() >> 4));
            // Every lane, the same word and value: no divergent region.  The
            // release orders the state stores before the hand-off in the
            // memory model (the reader's acquire fence pairs with it), not
            // only through the vmcnt drain above.
            __hip_atomic_store(prog, sg + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            if (lane == 0) SHA_DBG(t, 3, sg + 1);
        }
    }
}

}  // namespace

// Messages at or below this count run the split (two waves per 64 messages)
// form: while its waves fit about one per SIMD, a message's latency is the
// kernel's time; above it, one wave per 64 messages (or the stream form,
// chosen by the caller) keeps every SIMD doing rounds.  Up to 3/4 of a
// group per SIMD the split form still led (40 960 x 1 MiB: 42.8 ms vs 51.2
// one-wave, 44.9 stream); at 51 200 the stream form led (44.8 vs 53.9 split;
// profiles/r2_sha_stream_lab_sizes.jsonl).
constexpr uint32_t kSplitMaxMessages = 256 * 4 * 64 * 3 / 4;

// The quad form the auto choice takes (up to kShaLagMsgs per CU): 4 =
// same-round, 5 = lag, 6 = lag with two messages per quad.  6 against 5 on
// config 3's 10 240 x 1 MiB: 20.72 vs 20.89 ms; at 16 000 messages (past 5's
// 48 per CU) 20.93 ms against the split form's 27.5 (profiles/r3/sha_lag/).
// Forms 4 and 5 and the split form's two-buffer ring exist in lab builds
// only (`make lab`, -DMXEC_LAB).
constexpr int kShaQuadAuto = 6;
// K + W read groups of the auto form's consumers (sha256_quad_kernel LDG;
// lab builds A/B it with MXEC_SHA_LDG=1|2|4|15).  Spreading the next block's
// reads over the block lost: 10 240 x 1 MiB took
// 22.0 ms with two groups and 22.4 with four against 19.6 with all 16 reads
// after the barrier, on one box in interleaved fresh processes
// (profiles/r6/sha_ldg_ab.jsonl), and 15 after the barrier with the 16th at
// step 2 (same 605 VALU) took 21.7 against 19.7 (sha_ldg15_ab_r6ag.jsonl):
// one read among the chain's VALU costs far more than the burst's wait.
constexpr int kShaLdg = 1;

#ifdef MXEC_LAB
// MXEC_SHA_SPLIT_BUFS=2: the split form's one-ahead K+W ring (lab A/B; read
// per launch), default 3.
int split_bufs() {
    const char* e = getenv("MXEC_SHA_SPLIT_BUFS");
    return e && atoi(e) == 2 ? 2 : 3;
}

// MXEC_SHA_PRIO=0..3 (lab A/B; read per launch), default 3.
uint32_t sha_prio() {
    const char* e = getenv("MXEC_SHA_PRIO");
    return e ? uint32_t(atoi(e)) : 3u;
}
#else
constexpr int split_bufs() { return 3; }
constexpr uint32_t sha_prio() { return 3u; }
#endif

hipError_t launch_sha256(const ShaArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    const uint32_t blocks = (a.n + 63) / 64;
    int form = a.force;
    if (form == 0) {
        // Auto: the lag pair form while its workgroups fit one per CU, then
        // split, then one wave per 64 messages.  (The host pins a form
        // through a.force: MXEC_SHA_FORM, read into the context's knobs.)
        const uint64_t n_cus = a.n_cus ? a.n_cus : 256;
#ifdef MXEC_LAB
        // Lab builds: MXEC_SHA_FORM=quad|lag selects the lab quad forms.
        const char* env = getenv("MXEC_SHA_FORM");
        if (env && !strcmp(env, "quad")) form = 4;
        else if (env && !strcmp(env, "lag")) form = 5;
        else
#endif
        form = a.n <= kShaLagMsgs * n_cus ? kShaQuadAuto : a.n <= kSplitMaxMessages ? 2 : 1;
    }
    if (a.piece.state && form != 4 && form != 5 && form != 6) return hipErrorInvalidValue;  // piece mode: quad forms
#ifdef MXEC_LAB
    if (form == 4 || form == 5) {  // 4: the same-round quad, 5: the lag quad (lab A/B)
        const dim3 grid((a.n + kShaQuadMsgs - 1) / kShaQuadMsgs);
        hipLaunchKernelGGL(form == 5 ? sha256_quad_kernel<true> : sha256_quad_kernel<false>, grid, dim3(256), 0, s,
                           a.ptrs, a.lens, a.digests, a.expected, a.exp_idx, a.ok, a.n, sha_prio(), a.piece);
        return hipGetLastError();
    }
#else
    if (form == 4 || form == 5) return hipErrorInvalidValue;
#endif
    if (form == 6) {  // the lag quad, two messages per quad, two producer waves (the auto form)
#ifdef MXEC_LAB
        if (const char* e = getenv("MXEC_SHA_PRODUCERS"); e && atoi(e) == 1) {  // lab A/B: one producer wave
            hipLaunchKernelGGL((sha256_quad_kernel<true, true, false>), dim3((a.n + 63) / 64), dim3(192), 0, s, a.ptrs,
                               a.lens, a.digests, a.expected, a.exp_idx, a.ok, a.n, sha_prio(), a.piece);
            return hipGetLastError();
        }
#endif
#ifdef MXEC_LAB
        if (const char* e = getenv("MXEC_SHA_LDG"); e && atoi(e) != kShaLdg) {  // lab A/B: K + W read groups
            const int g = atoi(e);
            auto* kern = g == 1    ? &sha256_quad_kernel<true, true, true, 1>
                         : g == 2  ? &sha256_quad_kernel<true, true, true, 2>
                         : g == 15 ? &sha256_quad_kernel<true, true, true, 15>
                                   : &sha256_quad_kernel<true, true, true, 4>;
            hipLaunchKernelGGL(kern, dim3((a.n + 63) / 64), dim3(256), 0, s, a.ptrs, a.lens, a.digests, a.expected,
                               a.exp_idx, a.ok, a.n, sha_prio(), a.piece);
            return hipGetLastError();
        }
#endif
        hipLaunchKernelGGL((sha256_quad_kernel<true, true, true, kShaLdg>), dim3((a.n + 63) / 64), dim3(256), 0, s,
                           a.ptrs, a.lens, a.digests, a.expected, a.exp_idx, a.ok, a.n, sha_prio(), a.piece);
        return hipGetLastError();
    }
    if (form == 3) {
        const uint32_t per = a.wg_waves ? a.wg_waves : 1;
        if (!a.work || !a.state || a.waves == 0 || a.seg_max == 0 || per > 4 || a.waves % per) return hipErrorInvalidValue;
        hipLaunchKernelGGL(sha256_stream_kernel, dim3(a.waves / per), dim3(64 * per), 0, s, a.ptrs, a.lens, a.digests,
                           a.expected, a.exp_idx, a.ok, a.n, a.work, a.state, a.seg_max, sha_prio());
        return hipGetLastError();
    }
    const bool split = form == 2;
#ifdef MXEC_LAB
    if (split && split_bufs() == 2)
        hipLaunchKernelGGL(sha256_split_kernel<2>, dim3(blocks), dim3(128), 0, s, a.ptrs, a.lens,
                           a.digests, a.expected, a.exp_idx, a.ok, a.n, sha_prio());
    else
#endif
    if (split)
        hipLaunchKernelGGL(sha256_split_kernel<3>, dim3(blocks), dim3(128), 0, s, a.ptrs, a.lens,
                           a.digests, a.expected, a.exp_idx, a.ok, a.n, sha_prio());
    else
        hipLaunchKernelGGL(sha256_kernel, dim3(blocks), dim3(64), 0, s, a.ptrs, a.lens, a.digests,
                           a.expected, a.exp_idx, a.ok, a.n, sha_prio());
    return hipGetLastError();
}

}  // namespace mxec
