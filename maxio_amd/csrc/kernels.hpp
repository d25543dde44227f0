// kernels.hpp — launch interface of the gfx950 kernels (rs_kernel.hip,
// sha256_kernel.hip).  Host code builds the descriptor tables in device
// memory and calls these launchers on a HIP stream.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mxec {

// One launch applies an r x k GF(2^8) matrix to a batch of objects that share
// (k, r, shard_size):  out[o][i][b] = XOR_j coef(o)[i][j] * in[o][j][b].
// Bytes of input j at or beyond in_len[o][j] read as zero (the crate's
// zero padding, filesystem.rs:1111 / chunk_reader.rs:192); output i is written
// for b < out_len[o][i] only.
struct alignas(16) RsTileRec {  // one tile of a grouped launch (below)
    uint32_t obj;    // its object
    uint32_t k;      // the object's input count
    uint32_t in0;    // the object's first entry in in_ptrs / in_len
    uint32_t local;  // the tile's index within the object
};
struct RsArgs {
    const uint8_t* const* in_ptrs;  // [n_obj][k]
    uint8_t* const* out_ptrs;       // [n_obj][r_total]; this launch writes rows
                                    //   [row0, row0 + r)
    const uint64_t* in_len;         // [n_obj][k]
    const uint64_t* out_len;        // [n_obj][r_total]
    const uint32_t* coef;           // tables, [j][i][8] per matrix (gf256.hpp)
    const uint32_t* coef_off;       // [n_obj] dword offset of object's table
    const uint64_t* edge_list;      // [n_edge] object << 32 | tile: every tile
                                    //   of an unaligned launch (edge kernel)
    uint64_t n_edge;
    uint64_t edge_tile_bytes;       // tile size the list was built for
    uint64_t shard_size;
    uint32_t n_obj, k, r, r_total, row0;
    uint32_t aligned;               // all pointers 16-byte aligned (else every
                                    //   tile is in the edge list)
    // Grouped launch (objects of different k and shard size sharing r, every
    // pointer aligned, r_total == r <= 8): when `tiles` is set, launch tile t
    // is tiles[t] — its object, that object's k and first input entry, and
    // the tile's index within the object.  k and shard_size above are then
    // unused.
    const RsTileRec* tiles = nullptr;
    uint64_t n_tiles = 0;
    // Multi-r grouped launch (tiles set): objects of every r <= kMultiR in
    // one grid; tiles[t].k holds k | r << 16, object o's outputs are
    // out_ptrs / out_len [o * kMultiR, o * kMultiR + r), its coefficient
    // table rows r apart.  r, r_total and row0 above are unused.
    uint32_t multi = 0;
    // Uniform launches: workgroups per CU chosen by the caller (the grid
    // tuner, ops.cpp); 0 = rs_default_variant's.
    uint32_t blocks_per_cu = 0;
    // Every launch form: at most this many workgroups (0: no cap).  Tests
    // (mxec_open_test rs_grid_cap) shrink the grid so each workgroup walks many tiles.
    uint32_t max_blocks = 0;
};
constexpr uint32_t kMultiR = 4;

// Tuning knobs of the interior kernel (tools/kernel_lab.cpp sweeps them).
struct RsVariant {
    int vecs = 2;           // 16-byte column vectors per lane per tile (1, 2, 4)
    bool nt = false;        // nontemporal loads / stores
    int blocks_per_cu = 8;  // grid = n_cus * blocks_per_cu (grid-stride)
    int min_waves = 0;      // 3: compile for >= 3 waves per SIMD (<= 168 VGPRs; V = 4, nt)
    bool load_nt = true;    // with nt: false = plain loads, nontemporal stores (V = 4, R <= 4; lab)
    bool store_nt = true;   // with nt: false = nontemporal loads, plain stores (V = 4, R <= 4; lab)
    int group = 4;          // inputs loaded per step; 8 with V = 2, R = 3..4 (lab)
};

// Uniform launches, or grouped ones (a.tiles set: rs_group_variant, aligned).
hipError_t launch_rs_apply(const RsArgs& a, int n_cus, hipStream_t s);
hipError_t launch_rs_apply_variant(const RsArgs& a, int n_cus, hipStream_t s, const RsVariant& v);
// Geometry the default launch uses for a given total row count, and its tile.
RsVariant rs_default_variant(uint32_t r_total);
// Geometry of grouped launches (a.tiles set) for r rows.
RsVariant rs_group_variant(uint32_t r);
uint64_t rs_tile_bytes(const RsVariant& v);

// SHA-256 over n messages, one lane per message.  If `expected` is set the
// kernel also writes ok[i] = (digest == expected[i]).
// Piece mode of the quad forms (the host pipeline hashes every chunk piece by
// piece while later pieces still upload): launch message i is the next piece
// of the chain kept in state slot slot[i].  With resume the chain continues
// from state[slot] (else from the IV).  total[i] == kShaNotFinal: the piece
// ends mid-message (a multiple of 64 bytes) and the running state goes back
// to state[slot]; otherwise it is the last piece of a total[i]-byte message,
// padded and finished into digests[slot] (ok[slot] against
// expected[exp_idx ? exp_idx[slot] : slot]).
constexpr uint64_t kShaNotFinal = ~uint64_t(0);
struct ShaPiece {
    uint32_t* state = nullptr;        // [slots][8] (a..h); null: whole messages
    const uint32_t* slot = nullptr;   // [n]
    const uint64_t* total = nullptr;  // [n]
    uint32_t resume = 0;
};

struct ShaArgs {
    const uint8_t* const* ptrs;  // [n]
    const uint64_t* lens;        // [n]
    uint8_t* digests;            // [n][32] (may be null when only ok is wanted)
    const uint8_t* expected;     // [*][32] or null
    const uint64_t* exp_idx;     // [n]: message i compares expected[exp_idx[i]]
                                 //   (null: expected[i])
    uint8_t* ok;                 // [n] or null
    uint32_t n;
    int force = 0;               // 0 auto, 1 one wave per 64 messages, 2 split,
                                 // 3 stream (needs the fields below), 4 quad,
                                 // 5 lag quad
    uint32_t n_cus = 0;          // the device's CUs (auto form choice; 0: 256)
    // Stream form (batches of more 64-message groups than the chip has
    // SIMDs): persistent waves take (group, segment) items in segment-major
    // order; a group's running state is handed from segment to segment
    // through `state`.  Every message 16-byte aligned.
    uint32_t* work = nullptr;    // [4 + groups] zeroed before the launch:
                                 //   [0] next item, [1] timeout code, [4 + g] segments of group g done
    uint32_t* state = nullptr;   // [n][8]
    uint32_t waves = 0;          // persistent waves
    uint32_t wg_waves = 1;       // waves per workgroup (1 or 4; waves divisible by it)
    uint32_t seg_max = 0;        // segments of the longest message
    ShaPiece piece;              // piece mode (quad forms, force 4 or 5 only)
};
// Messages per workgroup of the quad form (three consumer waves of 16).
constexpr uint32_t kShaQuadMsgs = 48;
// Messages per workgroup of the lag quad form with two messages per quad
// (two consumer waves of 32): the auto latency form, one workgroup per CU.
constexpr uint32_t kShaLagMsgs = 64;
// A chain's pace per 64-byte block on the MI355X (us), for host-side
// estimates of a launch's length (combiner.cpp): the lag pair form the auto
// choice takes up to kShaLagMsgs per CU (config 3: 19.1 ms for 16 384
// blocks, two producer waves since round 5), the split / one-wave forms
// beyond (29 ms per 1 MiB chunk).
constexpr double kShaLagUsPerBlock = 1.17;
constexpr double kShaSplitUsPerBlock = 1.8;
// Blocks per stream-form segment (32 KiB of each message).
constexpr uint32_t kShaSegBlocks = 512;
// Timeout code the stream form leaves in work[1] when a wave gave up
// waiting for a predecessor segment (the digests are then incomplete).
constexpr uint32_t kShaStreamTimeout = 0x5AA5u;

hipError_t launch_sha256(const ShaArgs& a, hipStream_t s);

// ---- PUT body digests (digest_kernel.hip) -----------------------------------
enum : uint32_t { kBodyMd5 = 0, kBodySha1 = 1, kBodySha256 = 2 };
struct BodyHashArgs {
    const uint8_t* const* ptrs;  // [n] device pointers
    const uint64_t* lens;        // [n]
    const uint32_t* algs;        // [gridDim.y] kBody* per launch row
    uint8_t* out;                // [n] records of out_stride bytes
    uint64_t out_stride;
    uint32_t off_md5, off_sha1, off_sha256;
    uint32_t n;
};
hipError_t launch_body_hash(const BodyHashArgs& a, uint32_t n_algs, hipStream_t s);

// Per-polynomial constants (reflected domain), built on the host.
struct CrcTables {
    uint32_t poly;
    uint32_t slice[16][256];      // slice[k][b] = raw CRC of byte b followed by 15-k zero bytes
    uint32_t shift4k[4][256];     // byte k of v -> (v's byte k) * x^(8*4096)
    uint32_t shift_tile[4][256];  // same for x^(8*crc_tile_bytes())
    uint32_t lane_shift[256];     // x^(8*16*(255-L))
    uint32_t tile_pow[64];        // x^(8*TILE*2^j)
    uint32_t byte_pow[64];        // x^(8*2^j)
};
struct CrcBody {
    const uint8_t* base;   // floor16(p): 16-byte aligned
    const uint8_t* tail;   // last partial unit (tail_len < 16 bytes)
    uint64_t len;          // body length
    uint64_t tile0;        // first tile in the launch's tile space
    uint64_t n_tiles;
    uint64_t pad_units;    // leading virtual zero units of the first tile
    uint32_t head_skip;    // bytes of unit 0 before p
    uint32_t tail_len;
    uint32_t prev;         // running CRC to continue (crc32c_append); 0 = fresh
    uint32_t _pad;
};
struct CrcArgs {
    const CrcTables* tables;
    const CrcBody* bodies;  // [n_bodies], tile0 ascending
    const uint32_t* tile_body;  // [n_tiles] body of each tile
    uint32_t* tile_crc;     // [n_tiles] scratch
    uint8_t* out;           // finished CRC of body b at out + b * out_stride
    uint64_t out_stride;
    uint64_t n_tiles;
    uint32_t n_bodies;
};
uint64_t crc_tile_bytes();
hipError_t launch_crc(const CrcArgs& a, int n_cus, hipStream_t s);

// ---- encrypt-then-EC frames (gcm_kernel.hip) ----------------------------------
// Per object (data key): AES-256 round keys as big-endian words, H^1..H^256
// and the 4-bit position table of H^256 (htab[p][v] = (v at nibble p) * H^256).
typedef uint32_t gcm_u32x4 __attribute__((ext_vector_type(4)));
struct GcmKey {
    uint32_t rk[60];
    gcm_u32x4 hpow[256];     // hpow[e - 1] = H^e
    gcm_u32x4 htab[32][16];
};
struct GcmFrame {
    const uint8_t* in;       // payload in (plaintext / ciphertext)
    uint8_t* out;            // payload out
    uint8_t* hdr;            // encrypt: 12-byte nonce written here; decrypt: stored nonce
    uint8_t* tag;            // encrypt: tag written here; decrypt: stored tag
    const uint8_t* aad;      // aad_len bytes (may be null when aad_len == 0)
    uint64_t index;          // chunk index of this frame
    uint32_t len;            // payload bytes (<= frame size)
    uint32_t aad_len;
    uint32_t key;            // index into keys
    uint32_t prefix_be;      // nonce prefix as a big-endian word (encrypt)
};
struct GcmArgs {
    const uint32_t* te;      // Te0..Te3, 4 x 256 words
    const GcmKey* keys;
    const GcmFrame* frames;  // frames of one object are consecutive
    int32_t* status;         // decrypt: 0 ok, 1 tag mismatch, 2 index mismatch
    uint64_t n_frames;
};
hipError_t launch_gcm_frames(const GcmArgs& a, bool decrypt, int n_cus, hipStream_t s);

// ---- host <-> device copies by CU waves (copy_kernel.hip) ---------------------
// One block of a copy batch: len bytes from src to dst (one side host memory
// mapped into the GPU's address space, the other HBM).  The table itself may
// sit in mapped host memory.
struct alignas(16) CopyBlk {
    uint64_t dst, src, len, pad;
};
constexpr uint64_t kCopyBlock = uint64_t(256) << 10;  // bytes per block (at most)
hipError_t launch_copy_blocks(const CopyBlk* blks, uint64_t n, bool to_host, uint32_t grid, hipStream_t s);
// Whether a host <-> device segment suits the wave copy: both ends at the
// same offset modulo 16 (then only its head and tail bytes go bytewise).
inline bool copy_phase_ok(const void* host, const void* dev) {
    return ((reinterpret_cast<uintptr_t>(host) ^ reinterpret_cast<uintptr_t>(dev)) & 15) == 0;
}

}  // namespace mxec
