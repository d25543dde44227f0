/*
 * maxio_ec.h — C ABI of the MI355X erasure-coding backend for MaxIO's
 * chunked-EC storage path (src/storage, reference v0.3.2).
 *
 * Plain C: pointers, sizes and int return codes; no C++ types, no torch types,
 * no exceptions cross this boundary.  Every call is reentrant and thread-safe
 * (tokio workers may call concurrently); each device has its own queues.
 * Results are deterministic and independent of the device count.
 *
 * What each entry point replaces in the reference (file:line under the
 * reference checkout; the crates are reed-solomon-erasure 6.0.0 and sha2 0.10.9,
 * Cargo.lock:1462-1473 and :1778-1786):
 *
 *   mxec_rs_check            ReedSolomon::new(k, m) argument errors
 *                            (called at filesystem.rs:1121, chunk_reader.rs:168)
 *   mxec_rs_parity_matrix    the matrix ReedSolomon::new builds (build_matrix)
 *   mxec_sha256_batch        Sha256::digest at filesystem.rs:1070 (write_chunk),
 *                            :1131 (parity), chunk_reader.rs:108 and :184 (verify)
 *   mxec_encode              FilesystemStorage::compute_and_write_parity,
 *                            filesystem.rs:1084-1145 (guard :1095, pad :1108-1113,
 *                            encode :1121-1124, parity digest :1131) plus the data
 *                            digests of write_chunk :1062-1080 — minus the file I/O
 *   mxec_reconstruct         try_reconstruct_data_chunk, chunk_reader.rs:157-226
 *                            (verify :176-196, count :199-208, reconstruct :211,
 *                            truncate :216-222) — minus the file I/O
 *   mxec_*_batch_host        many mxec_encode / mxec_reconstruct calls at once
 *                            from host memory, pipelined over every device
 *   mxec_*_device            the same two operations over device-resident
 *                            batches (objects of any k and chunk size that share
 *                            the output count share one launch)
 *   mxec_write_chunk,
 *   mxec_compute_and_write_parity,
 *   mxec_try_reconstruct_data_chunk,
 *   mxec_put_object_chunked  the file-level functions themselves, writing the
 *                            same `{key}.ec/{index:06}` files and manifest.json
 *                            (filesystem.rs:686-828, 1062-1145; chunk_reader.rs:87-226)
 *   mxec_reader_*            VerifiedChunkReader (chunk_reader.rs:35-85, 228-276)
 *   mxec_body_sums*          the PUT body digests: Md5 ETag + ChecksumHasher
 *                            (filesystem.rs:28-63, 700-725, 775-777)
 *   mxec_frames_*            FrameEncryptor / FrameDecryptor (storage/crypto.rs)
 *                            and the frame AAD builders (filesystem.rs:112-163)
 */
#ifndef MAXIO_EC_H
#define MAXIO_EC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes -------------------------------------------------------
 * -1..-13 mirror reed_solomon_erasure::Error variants one for one; -14 is the
 * crate's SingularMatrix (matrix.rs); the rest are MaxIO's own guards and this
 * library's device / argument failures. */
#define MXEC_OK 0
#define MXEC_E_TOO_FEW_SHARDS (-1)
#define MXEC_E_TOO_MANY_SHARDS (-2)
#define MXEC_E_TOO_FEW_DATA_SHARDS (-3)
#define MXEC_E_TOO_MANY_DATA_SHARDS (-4)
#define MXEC_E_TOO_FEW_PARITY_SHARDS (-5)
#define MXEC_E_TOO_MANY_PARITY_SHARDS (-6)
#define MXEC_E_TOO_FEW_BUFFER_SHARDS (-7)
#define MXEC_E_TOO_MANY_BUFFER_SHARDS (-8)
#define MXEC_E_INCORRECT_SHARD_SIZE (-9)
#define MXEC_E_TOO_FEW_SHARDS_PRESENT (-10)
#define MXEC_E_EMPTY_SHARD (-11)
#define MXEC_E_INVALID_SHARD_FLAGS (-12)
#define MXEC_E_INVALID_INDEX (-13)
#define MXEC_E_SINGULAR_MATRIX (-14)
#define MXEC_E_TOO_MANY_SHARDS_255 (-20) /* filesystem.rs:1095-1102 k+m>255 */
#define MXEC_E_INVALID_ARG (-21)
#define MXEC_E_DEVICE (-30)
#define MXEC_E_OOM (-31)
#define MXEC_E_NO_DEVICE (-32)
#define MXEC_E_IO (-40)              /* StorageError::Io / io::Error */
#define MXEC_E_INTEGRITY (-41)       /* size or checksum mismatch (InvalidData) */
#define MXEC_E_JSON (-42)            /* StorageError::Json */

/* ---- flags ---------------------------------------------------------------- */
#define MXEC_F_DATA_ONLY 0x1u /* reconstruct: rebuild missing data shards only
                                 (crate reconstruct_data) */

typedef struct mxec_ctx mxec_ctx;

/* ---- library / context ---------------------------------------------------- */
const char* mxec_version(void);
const char* mxec_strerror(int code);
/* Last error message of the calling thread (never NULL). */
const char* mxec_last_error(void);
/* Number of visible HIP devices (0 on a host without a GPU). */
int mxec_device_count(void);
/* device_mask: bit d selects HIP device d; 0 selects every visible device.
 * streams_per_device: HIP streams (and staging rings) per device, >= 1.
 * Returns NULL if no device can be opened (see mxec_last_error). */
mxec_ctx* mxec_open(uint32_t device_mask, int streams_per_device);
/* TEST-ONLY open: as mxec_open, plus settings that exist to drive code paths
 * on a one-GPU test box.  They are never read from the environment, so a
 * production host cannot turn them on by accident.
 *   logical_devices:  open every selected GPU this many times (1..8), each
 *                     copy a separate device with its own streams, arenas,
 *                     combiner and pipeline (the multi-device paths);
 *   rs_grid_cap:      cap every RS launch at this many workgroups (0: off),
 *                     so each workgroup walks many tiles of its grid-stride loop;
 *   coef_arena_bytes: bytes per half of each device's coefficient-table arena
 *                     (0: 64 MiB), small enough that tests recycle it. */
mxec_ctx* mxec_open_test(uint32_t device_mask, int streams_per_device, int logical_devices, uint32_t rs_grid_cap,
                         uint64_t coef_arena_bytes);
void mxec_close(mxec_ctx* ctx);
int mxec_ctx_device_count(const mxec_ctx* ctx);
/* HIP device id of the ctx's i-th device. */
int mxec_ctx_device_id(const mxec_ctx* ctx, int i);
/* Runtime statistics of ctx device i: SHA-256 verification launches run by
 * the device's combiner (concurrent small requests share one launch) and the
 * messages they hashed. */
int mxec_ctx_combiner_stats(mxec_ctx* ctx, int i, uint64_t* launches, uint64_t* messages);
/* Host-batch pipeline (mxec_{encode,reconstruct}_batch_host) counters of ctx
 * device `dev` since the context opened, into out[0 .. n): the copies it
 * issued (1D SDMA DMAs, 2D SDMA DMAs -- the PUT's piece copies -- and their
 * rows, CU-wave copy blocks), the upload brackets MXEC_PIPE_COPY=auto timed
 * and how many ran below its SDMA floor (the rest of those calls' uploads,
 * and the device's for 2 s, copied by waves), the piece-major verified
 * reconstruct waves and the verification groups they ran as, the last timed
 * upload bracket's SDMA rate in MB/s, the same three for downloads
 * (brackets timed, below the floor, last rate), the host-batch calls run on
 * the device and how many of them started while another was in flight, the
 * verified GET's speculative piece rebuilds and the objects it rebuilt
 * again after a verdict, and the host waits that paced a shared call's
 * enqueue.  Returns how many counters were
 * written (min(n, MXEC_PIPE_STAT_COUNT)), or an error.  Diagnostics (tests). */
#define MXEC_PIPE_STAT_COPIES_1D 0
#define MXEC_PIPE_STAT_COPIES_2D 1
#define MXEC_PIPE_STAT_ROWS_2D 2
#define MXEC_PIPE_STAT_WAVE_BLOCKS 3
#define MXEC_PIPE_STAT_SDMA_CHECKS 4
#define MXEC_PIPE_STAT_SDMA_SLOW 5
#define MXEC_PIPE_STAT_VERIFY_WAVES 6
#define MXEC_PIPE_STAT_VERIFY_GROUPS 7
#define MXEC_PIPE_STAT_SDMA_LAST_MBPS 8
#define MXEC_PIPE_STAT_SDMA_DOWN_CHECKS 9
#define MXEC_PIPE_STAT_SDMA_DOWN_SLOW 10
#define MXEC_PIPE_STAT_SDMA_DOWN_LAST_MBPS 11
#define MXEC_PIPE_STAT_CALLS 12
#define MXEC_PIPE_STAT_CALLS_SHARED 13
#define MXEC_PIPE_STAT_SPEC_PIECES 14
#define MXEC_PIPE_STAT_SPEC_REDOS 15
#define MXEC_PIPE_STAT_PACE_WAITS 16
#define MXEC_PIPE_STAT_COUNT 17
int mxec_ctx_pipe_stats(mxec_ctx* ctx, int dev, uint64_t* out, int n);
/* Workgroups per CU the ctx's device `dev` runs large uniform RS launches of
 * (k inputs, m outputs, shard_size) at: the grid tuner times the first
 * launches of a shape at three grid sizes and keeps the fastest (which of
 * them wins depends on the box and on where the batch sits in HBM).  0 while
 * the shape is still being tuned; the default grid for shapes never launched
 * or too small to tune.  Diagnostics (the bench reports it). */
int mxec_ctx_rs_grid(mxec_ctx* ctx, int dev, int k, int m, uint64_t shard_size);
/* Coefficient-table arena statistics of ctx device `dev`: how often the
 * arena's two halves were recycled (a new generation reused the older half),
 * how many batches were queued again because their tables' half was
 * recycled before their launches were fenced, and how many recycles had to
 * wait for a fenced launch still running (fence_waits may be NULL).
 * Diagnostics (tests). */
int mxec_ctx_coef_stats(mxec_ctx* ctx, int dev, uint64_t* recycles, uint64_t* relaunches,
                        uint64_t* fence_waits);
/* Page-locked host memory for request bodies and GET buffers (the Axum body
 * MaxIO hands to a PUT, the buffer a GET fills).  Every host-pointer entry
 * point accepts any host memory; when a buffer comes from here, its bytes
 * move straight to and from the device (by DMA, or by the GPU's own waves
 * over PCIe, INTEGRATION.md MXEC_PIPE_COPY) instead of through the
 * library's pinned staging copy.  NULL on failure; free with
 * mxec_host_free. */
void* mxec_host_alloc(mxec_ctx* ctx, size_t bytes);
/* The same, on the NUMA node of the ctx's device `dev` (MXEC_HOST_NUMA or
 * not): on a host whose GPUs sit on two sockets, a request body meant for a
 * GPU goes on that GPU's socket, and the host batch calls deal an object to
 * a GPU on the node of its pages (pipeline.cpp deal_batch) -- the DMAs then
 * stay off the socket link.  Replaces nothing in the reference (MaxIO's
 * bodies are plain heap memory; filesystem.rs:686-828). */
void* mxec_host_alloc_device(mxec_ctx* ctx, int dev, size_t bytes);
void mxec_host_free(mxec_ctx* ctx, void* p);

/* HBM for a device-resident batch of n_obj objects of (k, m, shard_size),
 * laid out object-major: shard j of object o at
 * base + (o * (k + m) + j) * (*shard_stride), each object's parity after its
 * data -- the layout mxec_encode_strided_device / _reconstruct_strided_device
 * take with obj_stride = (k + m) * shard_stride.  The placement is measured:
 * up to two allocations (the second while the first is held) times two shard
 * strides, each timed by one encode over the whole candidate; the fastest is
 * kept (where a batch lies in HBM moves the encode by up to ~8 %, DESIGN.md
 * §7).  Transiently up to twice the batch's bytes.  probe_ms: NULL, or 4
 * floats receiving the candidates' times (allocation-major; -1 for a
 * candidate not tried).  NULL on failure (mxec_last_error).  Replaces nothing
 * in the reference: a long-lived process allocates its batch buffers once. */
void* mxec_batch_alloc(mxec_ctx* ctx, int dev, int k, int m, uint64_t shard_size,
                       uint64_t n_obj, uint64_t* shard_stride, float* probe_ms);
int mxec_batch_free(mxec_ctx* ctx, void* p);

/* ---- ReedSolomon::new ----------------------------------------------------- */
/* 0 if new(k, m) would succeed; otherwise the crate's error
 * (TooFewDataShards / TooFewParityShards / TooManyShards). */
int mxec_rs_check(int k, int m);
/* Writes the m x k parity rows of the crate's encoding matrix, row-major. */
int mxec_rs_parity_matrix(int k, int m, uint8_t* out);

/* ---- host-pointer entry points (the drop-in for one request) -------------- */
/* SHA-256 of n host buffers; out[i] = digest of bufs[i][0..lens[i]). */
int mxec_sha256_batch(mxec_ctx* ctx, const uint8_t* const* bufs,
                      const size_t* lens, size_t n, uint8_t (*out)[32]);

/* Encode one object: k data chunks (data_len[j] <= shard_size bytes, zero
 * padded to shard_size as filesystem.rs:1111 does), m parity outputs of
 * shard_size bytes each.  sha256_out, if not NULL, receives k+m digests:
 * data digests over the unpadded bytes (write_chunk :1070), parity digests over
 * the full shard (:1131).  data_len NULL means every chunk is shard_size. */
int mxec_encode(mxec_ctx* ctx, int k, int m, size_t shard_size,
                const uint8_t* const* data, const size_t* data_len,
                uint8_t* const* parity, uint8_t (*sha256_out)[32]);

/* Reconstruct one object, try_reconstruct_data_chunk semantics.
 * shards[i] (i < k+m) holds shard_len[i] bytes when present_inout[i] != 0;
 * for a missing shard it is the output buffer (shard_len[i] bytes; parity
 * shards use shard_size).  If expected_sha256 is not NULL every present shard
 * is hashed and a mismatch turns it into an erasure (:176-196), rebuilt into
 * the same buffer at shard_len[i] bytes.  Missing
 * shards are rebuilt (all of them, or data only with MXEC_F_DATA_ONLY);
 * present_inout[i] is 1 on return for every verified or rebuilt shard.
 * Fewer than k verified shards: MXEC_E_TOO_FEW_SHARDS_PRESENT, nothing is
 * written, and *n_present (if not NULL) holds the verified count. */
int mxec_reconstruct(mxec_ctx* ctx, int k, int m, size_t shard_size,
                     uint8_t* const* shards, const size_t* shard_len,
                     const uint8_t (*expected_sha256)[32],
                     uint8_t* present_inout, uint32_t flags, int* n_present);

/* ---- completion handles (non-blocking host calls) -------------------------
 * The *_async forms queue the blocking call of the same name on the
 * context's worker threads and return at once (MXEC_OK and *ticket set), or
 * return an argument error without a ticket.  Pointer arrays, digests to
 * compare and directory strings are copied at submission; data buffers and
 * out-parameters (parity, shards, present_inout, n_present, out, out_len)
 * must stay valid until the ticket completes.  A tokio caller registers
 * mxec_ticket_fd (an eventfd, readable once the call is done) with AsyncFd
 * and awaits it instead of parking a blocking-pool thread for the ~30 ms a
 * 1 MiB chunk's SHA-256 chain takes (chunk_reader.rs:244-249, main.rs:81). */
typedef struct mxec_ticket mxec_ticket;
/* eventfd that becomes readable when the call completes. */
int mxec_ticket_fd(const mxec_ticket* t);
/* 1 when complete, 0 while running (never blocks). */
int mxec_ticket_poll(mxec_ticket* t);
/* Blocks until complete; returns the call's status and sets the calling
 * thread's mxec_last_error to its message. */
int mxec_ticket_wait(mxec_ticket* t);
/* The failed call's message ("" on success or while running). */
const char* mxec_ticket_error(const mxec_ticket* t);
/* Waits for completion if needed, then frees the ticket and its fd. */
void mxec_ticket_free(mxec_ticket* t);
int mxec_sha256_batch_async(mxec_ctx* ctx, const uint8_t* const* bufs, const size_t* lens,
                            size_t n, uint8_t (*out)[32], mxec_ticket** ticket);
int mxec_encode_async(mxec_ctx* ctx, int k, int m, size_t shard_size,
                      const uint8_t* const* data, const size_t* data_len,
                      uint8_t* const* parity, uint8_t (*sha256_out)[32], mxec_ticket** ticket);
int mxec_reconstruct_async(mxec_ctx* ctx, int k, int m, size_t shard_size,
                           uint8_t* const* shards, const size_t* shard_len,
                           const uint8_t (*expected_sha256)[32], uint8_t* present_inout,
                           uint32_t flags, int* n_present, mxec_ticket** ticket);
int mxec_put_object_chunked_async(mxec_ctx* ctx, const char* ec_dir, uint64_t chunk_size,
                                  uint32_t parity_shards, const uint8_t* body, size_t len,
                                  mxec_ticket** ticket);
int mxec_get_object_chunked_async(mxec_ctx* ctx, const char* ec_dir, uint64_t offset,
                                  uint64_t length, uint8_t* out, uint64_t out_cap,
                                  uint64_t* out_len, mxec_ticket** ticket);

/* ---- device-resident batches ---------------------------------------------
 * All data pointers below are HIP device pointers on ctx device `dev`
 * (index into the ctx's devices).  `stream` is a hipStream_t of that device;
 * NULL is the HIP null (default) stream, as in other HIP libraries, so work
 * the caller queued there is ordered before ours.  Calls return after
 * enqueueing, except
 * mxec_reconstruct_strided_device and mxec_reconstruct_batch_device with
 * verification, which synchronise once to read the verdicts (the erasure
 * pattern picks the decode matrix). */

/* Uniform batch of n_obj objects, each k data + m parity shards of
 * shard_size bytes.  Object o, data shard j lives at
 * data + o*data_obj_stride + j*data_shard_stride (likewise parity).
 * data_len (host, k entries, NULL = shard_size) applies to every object.
 * digests_dev (device, n_obj*(k+m)*32, NULL = skip) gets the data then
 * parity digests of each object, object-major. */
int mxec_encode_strided_device(mxec_ctx* ctx, int dev, void* stream, int k,
                               int m, uint64_t shard_size, uint64_t n_obj,
                               const uint8_t* data, uint64_t data_obj_stride,
                               uint64_t data_shard_stride,
                               const uint64_t* data_len, uint8_t* parity,
                               uint64_t parity_obj_stride,
                               uint64_t parity_shard_stride,
                               uint8_t* digests_dev);

/* General batch: object o has k[o] data and m[o] parity shards of
 * shard_size[o] bytes; the pointer arrays are host arrays of device pointers,
 * concatenated over objects (sum k, sum m entries); data_len likewise (NULL =
 * full shards).  digests_dev: sum(k+m)*32 bytes, object-major, or NULL.
 * Objects with the same m share one kernel launch whatever their k and
 * shard size (16-byte aligned pointers, m <= 8; otherwise one launch per
 * (k, m, shard_size)). */
typedef struct mxec_object {
    int32_t k;
    int32_t m;
    uint64_t shard_size;
} mxec_object;
int mxec_encode_batch_device(mxec_ctx* ctx, int dev, void* stream,
                             const mxec_object* objs, uint64_t n_obj,
                             const uint8_t* const* data,
                             const uint64_t* data_len,
                             uint8_t* const* parity, uint8_t* digests_dev);

/* End-to-end PUT compute for many objects whose chunks are in HOST memory
 * (request bodies) — the batched form of mxec_encode.  Same array layout as
 * mxec_encode_batch_device but host pointers; digests (host, sum(k+m)) and
 * status_out (host, n_obj) may be NULL.  Objects are dealt over the ctx's
 * devices -- object o to device o mod D when every object has the same
 * (k, m, shard_size), balanced by bytes otherwise; per device, uploads
 * (direct from pinned memory, else via a pinned ring), RS + SHA-256 kernels
 * and downloads are pipelined on separate streams with the whole batch
 * resident in HBM.  Blocks until every
 * parity chunk and digest is in host memory.  Thread-safe: concurrent
 * calls (this one and mxec_reconstruct_batch_host, from any threads) share
 * each device -- up to MXEC_PIPE_LANES at once, their waves interleaved on
 * the device's four pipeline streams. */
int mxec_encode_batch_host(mxec_ctx* ctx, const mxec_object* objs,
                           uint64_t n_obj, const uint8_t* const* data,
                           const uint64_t* data_len, uint8_t* const* parity,
                           uint8_t (*digests)[32], int32_t* status_out);

/* End-to-end GET compute for many objects whose shards are in HOST memory
 * (the shard files as read from disk) -- the batched form of
 * mxec_reconstruct (try_reconstruct_data_chunk, chunk_reader.rs:157-226, per
 * object).  Same array layout as mxec_reconstruct_batch_device but host
 * pointers: shards (sum(k+m), object-major; a missing shard's pointer is the
 * buffer its rebuilt bytes go to), shard_len (NULL = shard_size), present
 * (in/out); expected_sha256 (host, sum(k+m) digests) or NULL to skip
 * verification; status_out (host, n_obj) may be NULL.  Objects are dealt
 * over the ctx's devices as mxec_encode_batch_host deals them; per device the
 * present shards go up (direct from pinned memory, else via a pinned ring),
 * are verified and rebuilt there, and only the rebuilt shards come back.  With
 * verification the missing shards are rebuilt piece by piece as the present
 * ones arrive, before the verdict (MXEC_GET_SPECULATE, default on), and an
 * object whose verdict drops a shard is rebuilt again from the verified
 * ones.  An object short of k verified shards gets
 * MXEC_E_TOO_FEW_SHARDS_PRESENT: its present shards' buffers are not written
 * and its missing shards' buffers are undefined (not written with
 * MXEC_GET_SPECULATE=0; the reference returns an error and no data,
 * chunk_reader.rs:203-206); the call returns the first such status.
 * Blocks until every rebuilt shard is in host memory.  Thread-safe, as
 * mxec_encode_batch_host. */
int mxec_reconstruct_batch_host(mxec_ctx* ctx, const mxec_object* objs,
                                uint64_t n_obj, uint8_t* const* shards,
                                const uint64_t* shard_len, uint8_t* present,
                                const uint8_t (*expected_sha256)[32],
                                uint32_t flags, int32_t* status_out);

/* Uniform reconstruct batch.  Object o, shard i (0 <= i < k+m) lives at
 * shards + o*obj_stride + i*shard_stride.  shard_len (host, k+m entries,
 * NULL = shard_size) is the byte length of shard i in every object.
 * present (host, n_obj*(k+m)) in/out as in mxec_reconstruct.
 * expected_sha_dev (device, n_obj*(k+m)*32) or NULL to skip verification.
 * status_out (host, n_obj, may be NULL): 0 or MXEC_E_TOO_FEW_SHARDS_PRESENT
 * per object; the call returns the first non-zero status.  With verification
 * the rebuild from the mask as given runs beside the hash (objects with a
 * digest mismatch are rebuilt again), so an object that fails may have had
 * its missing shards written. */
int mxec_reconstruct_strided_device(mxec_ctx* ctx, int dev, void* stream,
                                    int k, int m, uint64_t shard_size,
                                    uint64_t n_obj, uint8_t* shards,
                                    uint64_t obj_stride, uint64_t shard_stride,
                                    const uint64_t* shard_len, uint8_t* present,
                                    const uint8_t* expected_sha_dev,
                                    uint32_t flags, int32_t* status_out);

/* The completion-handle form (see mxec_ticket above): shard_len is copied at
 * submission; present and status_out must stay valid until the ticket
 * completes, and the shards are the caller's until then. */
int mxec_reconstruct_strided_device_async(mxec_ctx* ctx, int dev, void* stream,
                                          int k, int m, uint64_t shard_size,
                                          uint64_t n_obj, uint8_t* shards,
                                          uint64_t obj_stride, uint64_t shard_stride,
                                          const uint64_t* shard_len, uint8_t* present,
                                          const uint8_t* expected_sha_dev,
                                          uint32_t flags, int32_t* status_out,
                                          mxec_ticket** ticket);

/* Mixed reconstruct batch — the counterpart of mxec_encode_batch_device for
 * a stream of objects of different (k, m) and shard sizes (BASELINE
 * configs[4]; try_reconstruct_data_chunk, chunk_reader.rs:157-226, per
 * object).  shards (host array of device pointers, sum(k+m) entries,
 * object-major), shard_len (host, sum(k+m), NULL = shard_size) and present
 * (host, sum(k+m), in/out as in mxec_reconstruct) are concatenated over
 * objects; expected_sha_dev (device, sum(k+m)*32) or NULL to skip
 * verification; status_out (host, n_obj, may be NULL) as in
 * mxec_reconstruct_strided_device.  With verification the call synchronises
 * once to read the verdicts.  Objects of every shape that rebuild the same
 * number of shards share one kernel launch. */
int mxec_reconstruct_batch_device(mxec_ctx* ctx, int dev, void* stream,
                                  const mxec_object* objs, uint64_t n_obj,
                                  uint8_t* const* shards,
                                  const uint64_t* shard_len, uint8_t* present,
                                  const uint8_t* expected_sha_dev,
                                  uint32_t flags, int32_t* status_out);

/* The completion-handle form: objs, shards and shard_len are copied at
 * submission; present and status_out must stay valid until the ticket
 * completes, and the shards are the caller's until then. */
int mxec_reconstruct_batch_device_async(mxec_ctx* ctx, int dev, void* stream,
                                        const mxec_object* objs, uint64_t n_obj,
                                        uint8_t* const* shards,
                                        const uint64_t* shard_len,
                                        uint8_t* present,
                                        const uint8_t* expected_sha_dev,
                                        uint32_t flags, int32_t* status_out,
                                        mxec_ticket** ticket);

/* SHA-256 of n device buffers (host arrays of device pointers and lengths)
 * into digests_dev (device, n*32). */
int mxec_sha256_batch_device(mxec_ctx* ctx, int dev, void* stream,
                             const uint8_t* const* bufs, const uint64_t* lens,
                             uint64_t n, uint8_t* digests_dev);

/* ---- file-level path (src/storage/filesystem.rs, chunk_reader.rs) -------- */
/* ChunkInfo (mod.rs:182-189): kind 0 = data, 1 = parity. */
typedef struct mxec_chunk_info {
    uint32_t index;
    uint64_t size;
    char sha256[65]; /* lowercase hex + NUL, hex::encode(Sha256::digest) */
    uint8_t kind;
} mxec_chunk_info;

/* write_chunk (filesystem.rs:1062-1080): writes ec_dir/{index:06}. */
int mxec_write_chunk(mxec_ctx* ctx, const char* ec_dir, uint32_t index,
                     const uint8_t* data, size_t len, mxec_chunk_info* out);

/* compute_and_write_parity (filesystem.rs:1084-1145): re-reads the k data
 * chunk files named by data_chunks, encodes, writes ec_dir/{k+i:06}. */
int mxec_compute_and_write_parity(mxec_ctx* ctx, const char* ec_dir,
                                  uint64_t chunk_size, uint32_t parity_shards,
                                  const mxec_chunk_info* data_chunks, int k,
                                  mxec_chunk_info* parity_out);

/* put_object_chunked's chunking + manifest (filesystem.rs:686-773) for a
 * fully buffered body: chunks of chunk_size, empty body -> one empty chunk and
 * no parity, parity when parity_shards > 0 && len > 0, manifest.json written
 * with serde_json::to_string_pretty's layout. */
int mxec_put_object_chunked(mxec_ctx* ctx, const char* ec_dir,
                            uint64_t chunk_size, uint32_t parity_shards,
                            const uint8_t* body, size_t len);

/* ---- encrypt-then-EC frames (src/storage/crypto.rs, filesystem.rs:112-163) --
 * The object body is cut into frame_size (FRAME_CHUNK_SIZE = 65536) plaintext
 * frames; frame i is nonce(12) = prefix(4) || (first_index + i) as u64 LE,
 * then the AES-256-GCM ciphertext, then the 16-byte tag (crypto.rs:1-20,
 * 426-432).  The EC layer then chunks these bytes like any body.
 * aad: NULL with aad_len 0 (no_aad), or n_frames * aad_len bytes with frame
 * i's AAD at aad + i * aad_len (mxec_frame_aads builds the reference's
 * SHA-256(identity || index LE) AADs).                                      */
#define MXEC_FRAME_CHUNK_SIZE 65536u
#define MXEC_FRAME_OVERHEAD 28u
/* Bytes of the frame stream for plaintext_len bytes. */
uint64_t mxec_frames_len(uint64_t plaintext_len, uint32_t frame_size);
/* FrameEncryptor over a whole buffer; out receives mxec_frames_len bytes. */
int mxec_frames_encrypt(mxec_ctx* ctx, const uint8_t key[32], const uint8_t nonce_prefix[4],
                        uint64_t first_index, const uint8_t* aad, uint32_t aad_len,
                        uint32_t frame_size, const uint8_t* pt, uint64_t len,
                        uint8_t* out, uint64_t out_cap, uint64_t* out_len);
/* FrameDecryptor over a whole buffer: every frame's stored index and tag are
 * checked (MXEC_E_INTEGRITY with crypto.rs's messages: "frame index mismatch:
 * expected E, got G", "AES-GCM decryption failed: authentication error",
 * "truncated encrypted frame"); no plaintext is returned on failure. */
int mxec_frames_decrypt(mxec_ctx* ctx, const uint8_t key[32], uint64_t first_index,
                        const uint8_t* aad, uint32_t aad_len, uint32_t frame_size,
                        const uint8_t* frames, uint64_t frames_len, uint64_t plaintext_size,
                        uint8_t* out, uint64_t out_cap, uint64_t* out_len);
/* Device-resident batches: one launch over every frame of every job. */
typedef struct mxec_frames_job {
    const uint8_t* key;       /* host, 32 bytes */
    uint8_t nonce_prefix[4];  /* encrypt only */
    uint32_t frame_size;
    uint64_t first_index;
    const uint8_t* aad_dev;   /* device, n_frames * aad_len bytes, or NULL */
    uint32_t aad_len;
    uint32_t reserved;
    const uint8_t* in_dev;    /* encrypt: plaintext; decrypt: frame stream */
    uint64_t len;             /* plaintext bytes */
    uint8_t* out_dev;         /* encrypt: frame stream; decrypt: plaintext */
} mxec_frames_job;
int mxec_frames_encrypt_device(mxec_ctx* ctx, int dev, void* stream,
                               const mxec_frames_job* jobs, uint64_t n_jobs);
/* Synchronous; status_out[j] = 0 or MXEC_E_INTEGRITY per job. */
int mxec_frames_decrypt_device(mxec_ctx* ctx, int dev, void* stream,
                               const mxec_frames_job* jobs, uint64_t n_jobs,
                               int32_t* status_out);
/* build_frame_aad / build_part_aad (filesystem.rs:118-158): out[i] =
 * SHA-256(prefix || (first_index + i) as u64 LE), prefix = the identity bytes
 * (bucket 0 key 0 version 0, or "PART" 0 upload_id 0 part_le4 0). */
int mxec_frame_aads(mxec_ctx* ctx, const uint8_t* prefix, uint32_t prefix_len,
                    uint64_t first_index, uint64_t n_frames, uint8_t (*out)[32]);

/* ---- PUT body digests (filesystem.rs:28-63, 700-725, 775-777) -------------
 * Every PUT hashes the whole body with MD5 (the ETag, hex-encoded and quoted
 * by the caller) and, when the request names an algorithm, with the
 * ChecksumHasher (x-amz-checksum-*, base64 of the bytes below).              */
#define MXEC_SUM_MD5    0x01u
#define MXEC_SUM_CRC32  0x02u /* crc32fast::Hasher::finalize               */
#define MXEC_SUM_CRC32C 0x04u /* crc32c::crc32c_append(0, body)            */
#define MXEC_SUM_SHA1   0x08u
#define MXEC_SUM_SHA256 0x10u
typedef struct mxec_body_sums {
    uint8_t md5[16];
    uint32_t crc32;  /* the u32 value; to_be_bytes() before base64 */
    uint32_t crc32c;
    uint8_t sha1[20];
    uint8_t sha256[32];
} mxec_body_sums;    /* 76 bytes; fields not requested are left untouched */

/* Digests of n host bodies (one record each). */
int mxec_body_sums_batch(mxec_ctx* ctx, const uint8_t* const* bodies, const uint64_t* lens,
                         uint64_t n, uint32_t which, mxec_body_sums* out);
/* Device-resident bodies (host array of device pointers); out_dev is a device
 * array of n records, written asynchronously on `stream`. */
int mxec_body_sums_batch_device(mxec_ctx* ctx, int dev, void* stream,
                                const uint8_t* const* bodies_dev, const uint64_t* lens,
                                uint64_t n, uint32_t which, mxec_body_sums* out_dev);
/* put_object_chunked plus the body digests it computes on the way
 * (PutResult etag / checksum_value, filesystem.rs:775-777). */
int mxec_put_object_chunked_sums(mxec_ctx* ctx, const char* ec_dir,
                                 uint64_t chunk_size, uint32_t parity_shards,
                                 const uint8_t* body, size_t len, uint32_t which,
                                 mxec_body_sums* sums_out);

/* put_object_chunked_encrypted (filesystem.rs:835-1060) for a buffered body:
 * the plaintext becomes AES-256-GCM 64 KiB frames (first index 0, frame i's
 * AAD = SHA-256(aad_prefix || i LE) with aad_prefix = bucket 0 key 0
 * version 0, build_frame_aad :118-128), the frame stream is chunked, parity
 * added, and manifest.json records total_size = frame-stream bytes and
 * plaintext_size.  `which` / sums_out: the plaintext body digests as in
 * mxec_put_object_chunked_sums (0 / NULL to skip). */
int mxec_put_object_chunked_encrypted(mxec_ctx* ctx, const char* ec_dir,
                                      uint64_t chunk_size, uint32_t parity_shards,
                                      const uint8_t key[32], const uint8_t nonce_prefix[4],
                                      const uint8_t* aad_prefix, uint32_t aad_prefix_len,
                                      const uint8_t* body, size_t len, uint32_t which,
                                      mxec_body_sums* sums_out);

/* One part of a CompleteMultipartUpload (PartMeta, multipart.rs). */
typedef struct mxec_multipart_part {
    const char* path;      /* part file (upload_part wrote it flat)          */
    uint64_t size;         /* plaintext bytes of the part                    */
    uint8_t md5[16];       /* the part ETag as raw bytes                     */
    uint32_t part_number;
    uint8_t encrypted;     /* frames under the upload key (SSE multipart)    */
} mxec_multipart_part;

/* complete_multipart_chunked (filesystem.rs:1147-1310): parts concatenated,
 * re-chunked, parity, manifest.json; etag_out receives "<hex md5 of the
 * parts' raw MD5s>-<n_parts>" (unquoted, :1240-1244).  The composite
 * x-amz-checksum is mxec_body_sums_batch over the parts' raw checksums. */
int mxec_complete_multipart_chunked(mxec_ctx* ctx, const char* ec_dir,
                                    uint64_t chunk_size, uint32_t parity_shards,
                                    const mxec_multipart_part* parts, uint32_t n_parts,
                                    char etag_out[48]);

/* complete_multipart_chunked_encrypted (filesystem.rs:1315-1560): encrypted
 * parts are decrypted with upload_key (AADs of "PART" 0 upload_id 0
 * part_number_le4 0, :147-163), the recombined plaintext re-encrypted under
 * the object key as in mxec_put_object_chunked_encrypted, chunked, parity,
 * manifest with plaintext_size; the same ETag. */
int mxec_complete_multipart_chunked_encrypted(mxec_ctx* ctx, const char* ec_dir,
                                              uint64_t chunk_size, uint32_t parity_shards,
                                              const mxec_multipart_part* parts, uint32_t n_parts,
                                              const uint8_t upload_key[32], const char* upload_id,
                                              const uint8_t key[32], const uint8_t nonce_prefix[4],
                                              const uint8_t* aad_prefix, uint32_t aad_prefix_len,
                                              char etag_out[48]);


/* GET of a whole EC object (VerifiedChunkReader over manifest.json,
 * chunk_reader.rs:35-152): verified chunks, RS recovery of bad ones.
 * out must hold manifest total_size bytes; *out_len receives it.
 * offset/length select a range as with_range (:52-82); length UINT64_MAX = to
 * the end.  Chunks the range covers whole are read straight into out and
 * verified there, so out must not be touched by anyone else during the call;
 * on an error *out_len is the number of bytes served before the bad chunk
 * (the streaming reader's prefix) and the bytes of out past it are
 * unspecified. */
int mxec_get_object_chunked(mxec_ctx* ctx, const char* ec_dir, uint64_t offset,
                            uint64_t length, uint8_t* out, uint64_t out_cap,
                            uint64_t* out_len);

/* GET / ranged GET of an encrypt-then-EC object (filesystem.rs:1618-1630,
 * :1700-1725): the frames covering [offset, offset + length) of the
 * plaintext (FrameDecryptor::ciphertext_offset / for_range) are read through
 * the verified chunk reader, decrypted (AADs SHA-256(aad_prefix || i LE)) and
 * the range copied to out.  frame_size = the object's encryption chunk_size;
 * plaintext_size = ObjectMeta.size, or UINT64_MAX for the manifest's
 * plaintext_size; length UINT64_MAX = to the end. */
int mxec_get_object_chunked_encrypted(mxec_ctx* ctx, const char* ec_dir, const uint8_t key[32],
                                      const uint8_t* aad_prefix, uint32_t aad_prefix_len,
                                      uint32_t frame_size, uint64_t plaintext_size,
                                      uint64_t offset, uint64_t length, uint8_t* out,
                                      uint64_t out_cap, uint64_t* out_len);

/* VerifiedChunkReader (chunk_reader.rs:12-276) as a pull stream.
 * mxec_reader_open = new (:35-49) when offset == 0 and length == UINT64_MAX,
 * with_range (:52-82) otherwise.  mxec_reader_read = poll_read (:228-276):
 * returns bytes copied (> 0), 0 at the end, or a negative error code; chunks
 * are verified against the manifest (size + SHA-256) in GPU batches of up to
 * `batch_bytes` (0 = 64 MiB), bad chunks of a batch are rebuilt in one decode
 * when the manifest has parity, and an unrecoverable chunk fails the read
 * that reaches it — after every byte before it was served, as the reference
 * aborts mid-stream. */
typedef struct mxec_reader mxec_reader;
int mxec_reader_open(mxec_ctx* ctx, const char* ec_dir, uint64_t offset,
                     uint64_t length, uint64_t batch_bytes, mxec_reader** out);
int64_t mxec_reader_read(mxec_reader* r, uint8_t* buf, uint64_t cap);
void mxec_reader_close(mxec_reader* r);

/* try_reconstruct_data_chunk (chunk_reader.rs:157-226) over ec_dir's files and
 * manifest.json: out receives chunks[target].size bytes. */
int mxec_try_reconstruct_data_chunk(mxec_ctx* ctx, const char* ec_dir,
                                    uint32_t target, uint8_t* out,
                                    uint64_t out_cap, uint64_t* out_len);

#ifdef __cplusplus
}
#endif
#endif /* MAXIO_EC_H */
