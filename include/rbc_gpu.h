/*
 * rbc_gpu.h -- C ABI of the MI355X-native Reliable Broadcast data path.
 *
 * This is the drop-in boundary for joomanzi/cleisthenes' rbc package: the Go
 * handlers (rbc/rbc.go:47-66) and the pb layout (pb/message.proto:25-35) stay
 * unchanged; the three data-path functions and the third-party encoder they
 * hold are served from here through a thin cgo shim:
 *
 *   rbc/rbc.go:97-100  shard(enc, data) ([][]byte, error)     -> rbc_shard / rbc_shard_commit
 *   rbc/rbc.go:92-95   validateMessage(echo *EchoRequest) bool -> rbc_validate_message / rbc_validate_batch
 *   rbc/rbc.go:86-90   interpolate(rootHash, shards) ([]byte, error)
 *                                                             -> rbc_interpolate / rbc_interpolate_batch
 *   rbc/rbc.go:42      broadcast(VAL): needs root + per-shard branch (Merkle build)
 *                                                             -> rbc_shard_commit / rbc_dev_merkle_build
 *   rbc/rbc.go:20      enc reedsolomon.Encoder (klauspost v1.9.1, go.mod:10)
 *                                                             -> rbc_rs_* (New/Split/Encode/Verify/
 *                                                                Reconstruct/ReconstructData/Update/Join)
 *   (BASELINE north_star (5)) ACS output assembly over xGMI  -> rbc_comm_* + rbc_dev_allgather_roots
 *
 * Plain pointers and sizes only.  All functions return an int status
 * (RBC_OK = 0 or a negative RBC_ERR_*); rbc_strerror() names it.
 * Error values map 1:1 onto klauspost/reedsolomon v1.9.1's error variables
 * plus ROOT_MISMATCH (interpolate's Merkle recheck) and DEVICE.
 *
 * Frozen Merkle convention: leaf = SHA-256(shard, S bytes),
 * node = SHA-256(left || right), bottom row padded to a power of two with EMPTY
 * leaves that contribute no bytes.  A branch is d = ceil(log2 N) sibling digests
 * leaf -> root; the flat Go form (rbc/request.go:11 `Branch []byte`) omits the
 * level-0 sibling when it is empty ((index ^ 1) >= N), the device form keeps a
 * zero-filled 32-byte slot there ([N][d][32]).
 *
 * Thread safety: every entry point may be called from many threads (the Go
 * batcher's goroutines).  A context serialises its own submissions with a
 * mutex; device-resident (rbc_dev_*) calls on one context must be ordered on
 * one HIP stream (they share the context's decode workspace).
 */
#ifndef RBC_GPU_H
#define RBC_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RBC_ABI_VERSION 7

/* ---- status codes ------------------------------------------------------- */
#define RBC_OK 0
#define RBC_ERR_INV_SHARD_NUM (-1)        /* reedsolomon.ErrInvShardNum         */
#define RBC_ERR_MAX_SHARD_NUM (-2)        /* reedsolomon.ErrMaxShardNum         */
#define RBC_ERR_TOO_FEW_SHARDS (-3)       /* reedsolomon.ErrTooFewShards        */
#define RBC_ERR_SHARD_NO_DATA (-4)        /* reedsolomon.ErrShardNoData         */
#define RBC_ERR_SHARD_SIZE (-5)           /* reedsolomon.ErrShardSize           */
#define RBC_ERR_SHORT_DATA (-6)           /* reedsolomon.ErrShortData           */
#define RBC_ERR_RECONSTRUCT_REQUIRED (-7) /* reedsolomon.ErrReconstructRequired */
#define RBC_ERR_ROOT_MISMATCH (-8)        /* interpolate: Merkle root recheck   */
#define RBC_ERR_DEVICE (-9)               /* HIP / RCCL failure                 */
#define RBC_ERR_INVALID_ARG (-10)
#define RBC_ERR_SINGULAR (-11)            /* internal: singular sub-matrix      */
#define RBC_ERR_NO_COMM (-12)             /* multi-GPU call before rbc_comm_init */
#define RBC_ERR_INVALID_INPUT (-13)       /* reedsolomon.ErrInvalidInput (Update) */

const char *rbc_strerror(int status);
int rbc_abi_version(void);
/* The file this library was mapped from (dladdr + realpath), so a caller can
 * record which build it measured. */
int rbc_library_path(char *out, size_t cap);
int rbc_device_count(int *count);

/* ---- context: one (N, f) RBC geometry on one GPU ------------------------
 * rbc/rbc.go:9-20 keeps n, f and `enc` per RBC; N-2f data shards, 2f parity. */
typedef struct rbc_ctx rbc_ctx;
int rbc_ctx_create(int n, int f, int device, rbc_ctx **out);
void rbc_ctx_destroy(rbc_ctx *ctx);
int rbc_ctx_params(const rbc_ctx *ctx, int *k, int *p, int *depth);
int rbc_ctx_device(const rbc_ctx *ctx, int *device); /* ABI 7: the HIP device the context runs on */
/* klauspost buildMatrix(k, n) as used by this context: n*k bytes, row-major */
int rbc_ctx_encode_matrix(const rbc_ctx *ctx, uint8_t *out);
/* GF(2^8) codec behind encode / interpolate (same bytes either way):
 * RBC_CODEC_AUTO = additive FFT where this build has a specialised transform
 * for (n, k) (rbc_ctx_codec reports it), else the matrix kernel;
 * RBC_CODEC_MATRIX forces klauspost's encode-matrix product on the GPU. */
#define RBC_CODEC_AUTO 0
#define RBC_CODEC_MATRIX 1
#define RBC_CODEC_FFT 2
int rbc_ctx_set_codec(rbc_ctx *ctx, int codec);
int rbc_ctx_codec(const rbc_ctx *ctx, int *codec); /* effective: MATRIX or FFT */
/* Wave issue priority (0..3, the SIMD arbiter's s_setprio level) of this
 * context's commit-side kernels (encode, leaf hashing, tree build) and
 * receive-side kernels (ECHO verify, interpolate's hashing, root recheck,
 * digest).  Only matters when both sides run concurrently on two streams;
 * results are identical either way.  Default 0 / 0. */
int rbc_ctx_set_wave_priority(rbc_ctx *ctx, int commit_prio, int receive_prio);
/* Levels of interpolate's two GF transforms: the missing-data-row GEMV and
 * the FFT re-encode (the matrix codec's decode product takes the second).
 * -1 = the commit side's level (default), like the commit side's own
 * transform.  Which side they should side with depends on which stream
 * limits the pipelined step. */
int rbc_ctx_set_decode_priority(rbc_ctx *ctx, int gemv_prio, int reencode_prio);
/* Root recheck of rbc_dev_receive_step (interpolate's Merkle recheck,
 * rbc/rbc.go:86-90).  RBC_RECHECK_REUSE (default): hash only the subtrees
 * that hold no valid ECHO leaf and compare their roots with the received
 * branches (verified against the committed root), falling back to the whole
 * tree for an instance whose decode changed a valid row; RBC_RECHECK_FULL:
 * rehash the whole tree.  The statuses are the same either way (up to
 * SHA-256 collisions); rbc_dev_interpolate always rehashes the whole tree
 * (it has no branches). */
#define RBC_RECHECK_REUSE 0
#define RBC_RECHECK_FULL 1
int rbc_ctx_set_recheck(rbc_ctx *ctx, int mode);
/* Which ECHO-verify form rbc_dev_verify / rbc_dev_receive_step run for rows
 * of shard_len bytes (validateMessage, rbc/rbc.go:92-95): RBC_VERIFY_WALK,
 * the per-leaf branch walk fused into the row hashing, or
 * RBC_VERIFY_SHARED_PATH, leaf hashing then merkle_path_kernel (where the
 * walk's 2d compressions per row are a real share of the row's own; C4).
 * Both give the same valid[] bit for bit. */
#define RBC_VERIFY_WALK 0
#define RBC_VERIFY_SHARED_PATH 1
int rbc_ctx_verify_form(const rbc_ctx *ctx, uint32_t shard_len, int *form);

/* ---- device memory / streams / events (so a host runtime needs no other
 *      GPU library to drive the rbc_dev_* path) ---------------------------- */
int rbc_dev_malloc(int device, size_t bytes, void **ptr);
int rbc_dev_free(void *ptr);
int rbc_dev_memset(void *ptr, int value, size_t bytes);
int rbc_memcpy_h2d(void *dst, const void *src, size_t bytes);
int rbc_memcpy_d2h(void *dst, const void *src, size_t bytes);
int rbc_host_alloc(size_t bytes, void **ptr); /* pinned (hipHostMalloc) */
int rbc_host_free(void *ptr);
int rbc_stream_create(int device, void **stream);
/* high != 0: the device's greatest stream priority (its waves are dispatched
 * ahead of normal-priority streams' when both have work queued), else the least. */
int rbc_stream_create_priority(int device, int high, void **stream);
int rbc_stream_destroy(void *stream);
int rbc_stream_sync(void *stream);
int rbc_event_create(void **event);
int rbc_event_destroy(void *event);
int rbc_event_record(void *event, void *stream);
int rbc_event_elapsed_ms(void *start, void *stop, float *ms);
/* Make later work on `stream` wait for `event` (cross-stream pipelining). */
int rbc_stream_wait_event(void *stream, void *event);
int rbc_device_sync(int device);
/* hipMemGetInfo: free and total device memory in bytes (a host runtime sizes
 * its batches and in-flight buffer sets from it). */
int rbc_device_mem_info(int device, size_t *free_bytes, size_t *total_bytes);

/* ---- device-resident batch stages -----------------------------------------
 * All buffers are device memory laid out per DESIGN.md section 4; `stream` is a
 * hipStream_t (NULL = default).  `count` RBC instances per call.  Lengths are
 * per instance (device uint32 array) or, when that pointer is NULL, uniform.
 * shard_pitch % 64 == 0 and >= S_i; value rows must be readable for
 * round_up(k*S_i, 16) + 16 bytes (value_pitch >= that; contents past B_i are
 * ignored -- the Split zero pad is produced by masking).                    */

/* shard(): Split + Encode.  values [count][value_pitch] (B_i bytes used) ->
 * shards [count][n][shard_pitch] (data rows 0..k-1 + parity rows k..n-1;
 * bytes past S_i = ceil(B_i/k) zeroed). */
int rbc_dev_encode(rbc_ctx *ctx, void *stream, int count, const uint8_t *values, uint64_t value_pitch,
                   const uint32_t *value_lens, uint32_t uniform_value_len, uint8_t *shards,
                   uint32_t shard_pitch);
/* leaves [count][n][32] = SHA-256 of each shard's S_i bytes. */
int rbc_dev_leaves(rbc_ctx *ctx, void *stream, int count, const uint8_t *shards, uint32_t shard_pitch,
                   const uint32_t *shard_lens, uint32_t uniform_shard_len, uint8_t *leaves);
/* Merkle build: roots [count][32], branches [count][n][d][32] (nullable). */
int rbc_dev_merkle_build(rbc_ctx *ctx, void *stream, int count, const uint8_t *leaves, uint8_t *roots,
                         uint8_t *branches);
/* encode + leaves + Merkle build in one call (VAL construction). */
int rbc_dev_shard_commit(rbc_ctx *ctx, void *stream, int count, const uint8_t *values, uint64_t value_pitch,
                         const uint32_t *value_lens, uint32_t uniform_value_len, uint8_t *shards,
                         uint32_t shard_pitch, const uint32_t *shard_lens, uint8_t *leaves, uint8_t *roots,
                         uint8_t *branches);
/* ECHO-side validateMessage for every received (instance, shard j): hash
 * shard j, walk branch j, compare with roots[i].  valid[i][j] = present[i][j]
 * && ok (present nullable = all).  Only present shards are hashed (they are
 * compacted on the device first), so leaves [count][n][32] (nullable)
 * receives the hashes of the present shards for interpolate's recheck; the
 * slots of absent shards are left unspecified. */
int rbc_dev_verify(rbc_ctx *ctx, void *stream, int count, const uint8_t *shards, uint32_t shard_pitch,
                   const uint32_t *shard_lens, uint32_t uniform_shard_len, const uint8_t *branches,
                   const uint8_t *roots, const uint8_t *present, uint8_t *valid, uint8_t *leaves);
/* interpolate(): from the first k valid shards by index (klauspost rule)
 * regenerate every other position of the full re-encoding IN PLACE in
 * `shards`, recompute the Merkle root and compare with roots[i]; on success
 * write value = data shards 0..k-1 concatenated (k*S_i bytes, pad kept) to
 * values_out [count][value_pitch] (bytes past k*S_i are unspecified, and a
 * row is defined only where status[i] == RBC_OK) and the batch digest
 * SHA-256(leaf_0 || .. || leaf_{k-1}) to digests [count][32] (likewise
 * defined only where status[i] == RBC_OK).
 * status[i]: RBC_OK, RBC_ERR_TOO_FEW_SHARDS or RBC_ERR_ROOT_MISMATCH.
 * leaves_verified != 0: `leaves` already holds SHA-256 of the valid shards
 * (rbc_dev_verify output) and only regenerated rows are hashed; 0: all rows.
 * values_out == NULL (value_pitch ignored) is the row view: no value is
 * assembled, and the value is the k data rows shards[i][0..k-1][0..S_i) as
 * regenerated in place (a caller that copies per shard anyway -- the cgo
 * side -- saves the k*S_i read + write of the join). */
int rbc_dev_interpolate(rbc_ctx *ctx, void *stream, int count, uint8_t *shards, uint32_t shard_pitch,
                        const uint32_t *shard_lens, uint32_t uniform_shard_len, const uint8_t *valid,
                        uint8_t *leaves, int leaves_verified, const uint8_t *roots, uint8_t *values_out,
                        uint32_t value_pitch, uint8_t *digests, int32_t *status);
/* Pipelined receiver, one call per batch:
 * rbc_dev_receive_step(ctx, stream, cur, prev) hashes the received ECHO
 * shards of `cur` (validateMessage, rbc/rbc.go:92-95) AND the rows
 * interpolate regenerated for `prev` in ONE SHA launch, then runs prev's
 * Merkle root recheck + batch digest, then cur's decode (first-k-valid
 * prepare, missing-data GF, FFT re-encode + compare; the value join on the
 * context's aux stream).  Alone, prev's regen hashing is a latency-bound tail
 * (few long serial chains); beside cur's verify it fills the SIMDs.
 * `prev` must be the `cur` of the previous call on this context (NULL on the
 * first call); a last call with cur = NULL completes the final batch.  When a
 * call's work on `stream` is done, prev's valid / leaves / status /
 * values_out / digests are final and equal rbc_dev_verify followed by
 * rbc_dev_interpolate(leaves_verified = 1) on the same inputs (interpolate,
 * rbc/rbc.go:86-90); cur's buffers must stay untouched until the next call's
 * work is done.  While a batch is pending, rbc_dev_interpolate on
 * the same context returns RBC_ERR_INVALID_ARG (they share its decode
 * workspace).  All pointers are device memory; present may be NULL (all
 * received).  cur and prev may share no output buffer (shards, valid, leaves,
 * status, values_out, digests): RBC_ERR_INVALID_ARG.  A call rejected by its
 * argument checks enqueues nothing (prev stays pending); an error after
 * prev's work was enqueued still completes prev once the call's work on
 * `stream` is, and cur is then not pending (the next call passes prev = NULL). */
typedef struct rbc_rx_batch {
    int count;
    uint8_t *shards;             /* [count][n][shard_pitch], regenerated in place */
    uint32_t shard_pitch;
    const uint32_t *shard_lens;  /* S_i, or NULL: uniform_shard_len */
    uint32_t uniform_shard_len;
    const uint8_t *branches;     /* [count][n][d][32] */
    const uint8_t *roots;        /* [count][32] */
    const uint8_t *present;      /* [count][n] received ECHOs (nullable) */
    uint8_t *valid;              /* [count][n] out */
    uint8_t *leaves;             /* [count][n][32] out (own buffer per batch in flight) */
    uint8_t *values_out;         /* [count][value_pitch] out; NULL: row view (rbc_dev_interpolate) */
    uint32_t value_pitch;
    uint8_t *digests;            /* [count][32] out (nullable) */
    int32_t *status;             /* [count] out */
    /* ABI 6: != 0 when valid / leaves already hold rbc_dev_verify's output for
     * this batch's received ECHOs (e.g. run on the proposer's stream right
     * after the commit it depends on): the step then only decodes it as cur
     * (no compaction, no row hashing or path walk for it) and rehashes,
     * rechecks and digests it as prev as usual. */
    int verified;
} rbc_rx_batch;
/* Timing marks (each nullable, rbc_event_create events) recorded on `stream`:
 * hashed after the hashing launch (and cur's shared-path walk), decode_begin
 * after prev's recheck, decoded after cur's decode (prepare, missing-data GF,
 * FFT re-encode + compare), so a caller can time each part live.  ABI 4:
 * hash_begin right before the row-hashing launch (after cur's compaction) and
 * rows_hashed right after it, before the shared-path verify
 * (merkle_path_kernel, W = 256 at short rows) -- so each of the two kernels
 * has its own span; with the per-leaf walk rows_hashed and hashed coincide.
 * ABI 5: prev_released completes once nothing of this call reads prev's
 * shards, branches or roots any more (its recheck on `stream`, its digest and
 * a join from the previous call on the context's aux stream; recorded on the
 * aux stream, so `stream` does not wait for it): a producer may refill prev's
 * shard set from then on while cur's decode still runs.  Not recorded when
 * prev is NULL. */
typedef struct rbc_rx_marks {
    void *hashed;
    void *decode_begin;
    void *decoded;
    void *hash_begin;
    void *rows_hashed;
    void *prev_released;
} rbc_rx_marks;
int rbc_dev_receive_step(rbc_ctx *ctx, void *stream, const rbc_rx_batch *cur, const rbc_rx_batch *prev,
                         const rbc_rx_marks *marks);
/* Synthetic Byzantine input for tests/bench: shards[i][corrupt[i]][0] ^= 0x5a
 * for every i with corrupt[i] >= 0 (corrupt: device int32[count]). */
int rbc_dev_inject_faults(rbc_ctx *ctx, void *stream, int count, uint8_t *shards, uint32_t shard_pitch,
                          const int32_t *corrupt);

/* ---- host-memory batch API (the Go batcher's entry points) ----------------
 * Copies through pinned staging on the context's own stream.  Each call
 * returns a ticket; rbc_wait / rbc_poll complete it (no C->Go callbacks).
 * Caller buffers must stay valid until the ticket completes. */
/* shard() + Merkle commit for `count` proposals: values[i] (value_lens[i] bytes)
 * -> shards_out [count][n][shard_pitch] (S_i bytes per row used; when
 * shards_out is pinned and shard_pitch % 64 == 0 the rows come back whole in
 * one copy, bytes [S_i, shard_pitch) as zero),
 * shard_lens_out [count] (S_i), roots_out [count][32],
 * branches_out [count][n][d][32] (nullable). */
int rbc_shard_commit(rbc_ctx *ctx, int count, const uint8_t *const *values, const size_t *value_lens,
                     uint8_t *shards_out, size_t shard_pitch, uint32_t *shard_lens_out, uint8_t *roots_out,
                     uint8_t *branches_out, uint64_t *ticket);
/* validateMessage for `count` independent ECHO messages: shard i
 * (shard_lens[i] bytes), leaf index indices[i], flat branch (branch_lens[i]
 * bytes, Go form), root (32 bytes).  ok_out[i] = 1 valid / 0 invalid. */
int rbc_validate_batch(rbc_ctx *ctx, int count, const uint8_t *const *shards, const size_t *shard_lens,
                       const uint32_t *indices, const uint8_t *const *branches, const size_t *branch_lens,
                       const uint8_t *const *roots, uint8_t *ok_out, uint64_t *ticket);
/* rbc_validate_batch with the messages already laid out as the device reads
 * them -- for a caller that keeps its own pinned request rings (the batcher's
 * validate lane; a Go batcher over rbc_host_alloc memory).  Message i's shard
 * bytes are arena[offs[i] .. offs[i] + lens[i]) with offs[i] % 64 == 0 and the
 * arena readable to offs[i] + round_up(lens[i], 64); branches[i] is the
 * device form [depth][32] (a zero slot for an empty level-0 sibling); roots[i]
 * 32 bytes; idx[i] < n the sender's leaf index.  One DMA of arena[0,
 * arena_bytes), one launch, the verdicts into ok_out[count] (1 = valid).
 * Every host buffer must stay valid until the ticket completes; pinned
 * (rbc_host_alloc) memory gives direct DMA.  Replaces the per-message staging
 * of validateMessage (rbc/rbc.go:92-95) for coalesced ECHOs. */
int rbc_validate_packed(rbc_ctx *ctx, int count, const uint8_t *arena, size_t arena_bytes, const uint64_t *offs,
                        const uint32_t *lens, const uint8_t *idx, const uint8_t *branches, const uint8_t *roots,
                        uint8_t *ok_out, uint64_t *ticket);
/* ABI 6: rbc_validate_packed that also returns each message's leaf,
 * leaves_out[i] = SHA-256 of message i's shard bytes (32 B, nullable), so an
 * interpolate of the same shards need not hash them again
 * (rbc_interpolate_batch_verified).  Either form moves only the named bytes
 * over PCIe when the arena is pinned and the messages cover less than 3/4 of
 * it (a receiver's [count][n][pitch] ECHO buffer with offs at the received
 * rows), else the whole arena in one DMA. */
int rbc_validate_packed_leaves(rbc_ctx *ctx, int count, const uint8_t *arena, size_t arena_bytes,
                               const uint64_t *offs, const uint32_t *lens, const uint8_t *idx,
                               const uint8_t *branches, const uint8_t *roots, uint8_t *ok_out, uint8_t *leaves_out,
                               uint64_t *ticket);
/* ABI 7: rbc_validate_packed_leaves whose messages stay on the device: the
 * arena is moved into keep_dev (device memory, keep_bytes >= arena_bytes, e.g.
 * rbc_dev_malloc) instead of a launch buffer, so message i's bytes are
 * keep_dev[offs[i] .. offs[i] + lens[i]) once the ticket completes -- for an
 * interpolate of the same shards straight from device memory
 * (rbc_interpolate_batch_kept): the ECHO rows of the drop-in's
 * validateMessage -> interpolate sequence (rbc/rbc.go:92-95, 86-90) then
 * cross PCIe once.  The caller must not reuse keep_dev before the
 * interpolates that read it have completed. */
int rbc_validate_packed_keep(rbc_ctx *ctx, int count, const uint8_t *arena, size_t arena_bytes, const uint64_t *offs,
                             const uint32_t *lens, const uint8_t *idx, const uint8_t *branches, const uint8_t *roots,
                             uint8_t *ok_out, uint8_t *leaves_out, uint8_t *keep_dev, size_t keep_bytes,
                             uint64_t *ticket);
/* interpolate() for `count` instances: shards [count][n][shard_pitch] with
 * present [count][n] (0 = missing, the Go `len == 0`), shard_lens [count],
 * roots [count][32] -> values_out [count][value_pitch] (k*S_i bytes),
 * digests_out [count][32] (nullable), status_out [count].  Pinned values_out
 * comes back in one copy: every row but the last whole, bytes [k*S_i,
 * value_pitch) as zero. */
int rbc_interpolate_batch(rbc_ctx *ctx, int count, const uint8_t *shards, size_t shard_pitch,
                          const size_t *shard_lens, const uint8_t *present, const uint8_t *roots,
                          uint8_t *values_out, size_t value_pitch, uint8_t *digests_out, int32_t *status_out,
                          uint64_t *ticket);
/* ABI 6: rbc_interpolate_batch over shards that were already validated:
 * every present row (present[i][j] != 0) passed validateMessage and
 * leaves [count][n][32] holds its SHA-256 (rbc_validate_packed_leaves /
 * rbc_batcher_validate_leaf output; the slots of absent rows are ignored).
 * The device hashes only the rows interpolate regenerates or finds changed
 * (~2f of N instead of N), as rbc_dev_receive_step does; outputs and statuses
 * equal rbc_interpolate_batch's on the same shards when the leaves are the
 * present rows' true hashes (a wrong leaf is trusted: pass only leaves this
 * library computed for exactly these bytes).  leaves == NULL is
 * rbc_interpolate_batch. */
int rbc_interpolate_batch_verified(rbc_ctx *ctx, int count, const uint8_t *shards, size_t shard_pitch,
                                   const size_t *shard_lens, const uint8_t *present, const uint8_t *leaves,
                                   const uint8_t *roots, uint8_t *values_out, size_t value_pitch,
                                   uint8_t *digests_out, int32_t *status_out, uint64_t *ticket);
/* ABI 7: rbc_interpolate_batch_verified over rows that are already in device
 * memory (rbc_validate_packed_keep): rows [count][n] holds the device address
 * of shard j of instance i (NULL = missing), shard_lens[i] bytes each; leaves
 * [count][n][32] their SHA-256 (as rbc_interpolate_batch_verified; NULL
 * rehashes all N).  Outputs and statuses equal rbc_interpolate_batch_verified's
 * over the same bytes. */
int rbc_interpolate_batch_kept(rbc_ctx *ctx, int count, const uint8_t *const *rows, const size_t *shard_lens,
                               const uint8_t *leaves, const uint8_t *roots, uint8_t *values_out, size_t value_pitch,
                               uint8_t *digests_out, int32_t *status_out, uint64_t *ticket);
/* ABI 6: the receiver's whole batch in one submission, for a batching host
 * that holds each instance's received ECHOs together (validateMessage of
 * every present row, rbc/rbc.go:92-95, then interpolate of the ones that
 * validated, rbc/rbc.go:86-90): the present rows cross PCIe ONCE (from a
 * pinned, uniform-length buffer only those rows are read), are verified on
 * the device against branches [count][n][depth][32] (device form: a zero
 * slot for an empty level-0 sibling) and roots [count][32], and interpolate
 * reuses the leaves the verify computed.  valid_out [count][n] = present &&
 * the branch proves the row (the validateMessage verdicts); values_out /
 * digests_out / status_out as rbc_interpolate_batch over the valid rows. */
int rbc_receive_batch(rbc_ctx *ctx, int count, const uint8_t *shards, size_t shard_pitch, const size_t *shard_lens,
                      const uint8_t *present, const uint8_t *branches, const uint8_t *roots, uint8_t *valid_out,
                      uint8_t *values_out, size_t value_pitch, uint8_t *digests_out, int32_t *status_out,
                      uint64_t *ticket);
int rbc_wait(rbc_ctx *ctx, uint64_t ticket);
int rbc_poll(rbc_ctx *ctx, uint64_t ticket, int *done);

/* ---- single-call drop-ins (batch of one, synchronous) --------------------- */
/* shard(enc, data) + commit: shards_out n*S bytes (shard j at j*S),
 * *shard_len_out = S, root_out 32 B, branches_out n*d*32 B (nullable). */
int rbc_shard(rbc_ctx *ctx, const uint8_t *data, size_t len, uint8_t *shards_out, size_t shards_cap,
              size_t *shard_len_out, uint8_t *root_out, uint8_t *branches_out);
/* validateMessage(echo): *ok = 1 iff the branch proves shard at `index` under root. */
int rbc_validate_message(rbc_ctx *ctx, const uint8_t *root, const uint8_t *branch, size_t branch_len,
                         const uint8_t *shard, size_t shard_len, uint32_t index, int *ok);
/* interpolate(rootHash, shards): shards[j] with lens[j] (0 = missing);
 * value_out capacity k*S; *value_len = k*S; digest_out 32 B (nullable). */
int rbc_interpolate(rbc_ctx *ctx, const uint8_t *root, const uint8_t *const *shards, const size_t *lens,
                    uint8_t *value_out, size_t value_cap, size_t *value_len, uint8_t *digest_out);

/* ---- request batcher (north_star (4): many RBC instances per launch) -------
 * Thousands of per-instance RBC event loops (rbc/rbc.go:78, one goroutine
 * each) submit single requests from any thread; a worker coalesces them per
 * kind into one batched launch when max_batch are queued or the oldest has
 * waited max_wait_us.  Caller buffers stay valid until the ticket completes.
 * rbc_batcher_wait returns the request's own status (RBC_OK, klauspost error,
 * RBC_ERR_ROOT_MISMATCH, ...) and releases the ticket. */
typedef struct rbc_batcher rbc_batcher;
int rbc_batcher_create(rbc_ctx *ctx, int max_batch, int max_wait_us, rbc_batcher **out);
void rbc_batcher_destroy(rbc_batcher *b); /* drains pending requests first */
/* shard(): shards_out n*S (shard j at j*S), root 32 B, branches n*d*32 (device form, nullable) */
int rbc_batcher_shard(rbc_batcher *b, const uint8_t *data, size_t len, uint8_t *shards_out, size_t shards_cap,
                      size_t *shard_len_out, uint8_t *root_out, uint8_t *branches_out, uint64_t *ticket);
/* validateMessage(): *ok_out set when the ticket completes.  Validates have
 * their own lane: the calling thread copies the message into the open pinned
 * arena (device layout) and returns; an arena is launched through
 * rbc_validate_packed when it holds max_msgs messages or max_bytes of shards,
 * or its first message has waited max_wait_us (max_batch does not apply). */
int rbc_batcher_validate(rbc_batcher *b, const uint8_t *root, const uint8_t *branch, size_t branch_len,
                         const uint8_t *shard, size_t shard_len, uint32_t index, int *ok_out, uint64_t *ticket);
/* The validate lane's arena size (default 65,536 messages / 256 MiB of
 * shards, six arenas, four in flight); before the first validate only.
 * max_msgs < 2^20, 64 <= max_bytes <= 4 GiB - 64. */
int rbc_batcher_set_validate(rbc_batcher *b, int max_msgs, size_t max_bytes);
/* ABI 6: rbc_batcher_validate that also returns the shard's leaf
 * (leaf_out, 32 B, written when *ok_out == 1) for a later
 * rbc_batcher_interpolate_verified of the same shard.  rbc/rbc.go:88,93 are
 * both package-internal, so a cgo shim can keep the leaves per RBC instance
 * and the handlers stay unchanged. */
int rbc_batcher_validate_leaf(rbc_batcher *b, const uint8_t *root, const uint8_t *branch, size_t branch_len,
                              const uint8_t *shard, size_t shard_len, uint32_t index, int *ok_out, uint8_t *leaf_out,
                              uint64_t *ticket);
/* ABI 7: keep validated shards on the device for their instance's
 * interpolate.  With a ring of device_bytes (rbc_dev_malloc'ed on the
 * context's device; 0 turns keeping off, the default) every validate launch
 * moves its arena into the ring (rbc_validate_packed_keep) and indexes each
 * shard that validated by (root, index) with the caller's shard pointer and
 * length; rbc_batcher_interpolate(_verified) whose every present shard is
 * indexed -- the SAME pointer and length that was validated -- reads the rows
 * (and their leaves) on the device (rbc_interpolate_batch_kept), so the ECHO
 * rows cross PCIe once, as the Go handlers' validateMessage -> interpolate
 * sequence (rbc/rbc.go:92-95, 86-90) stays unchanged.  Any miss takes the
 * host path; results are the same either way provided the caller does not
 * modify a validated shard's bytes before its interpolate.  A launch whose
 * ring region is still read by an interpolate in flight is not kept.  Before
 * the first validate only. */
int rbc_batcher_set_keep(rbc_batcher *b, size_t device_bytes);
/* interpolates served from kept rows / from host memory, validate launches kept / not kept */
int rbc_batcher_keep_stats(rbc_batcher *b, uint64_t *kept_interps, uint64_t *host_interps, uint64_t *kept_launches,
                           uint64_t *unkept_launches);
/* interpolate(): shards/lens are n entries (lens[j] == 0: missing) */
int rbc_batcher_interpolate(rbc_batcher *b, const uint8_t *root, const uint8_t *const *shards, const size_t *lens,
                            uint8_t *value_out, size_t value_cap, size_t *value_len, uint8_t *digest_out,
                            uint64_t *ticket);
/* ABI 6: interpolate() of shards that passed rbc_batcher_validate_leaf:
 * leaves n*32 bytes, leaves[32j..] the leaf of shard j for every lens[j] != 0
 * (rbc_interpolate_batch_verified semantics: only regenerated rows are hashed). */
int rbc_batcher_interpolate_verified(rbc_batcher *b, const uint8_t *root, const uint8_t *const *shards,
                                     const size_t *lens, const uint8_t *leaves, uint8_t *value_out, size_t value_cap,
                                     size_t *value_len, uint8_t *digest_out, uint64_t *ticket);
int rbc_batcher_wait(rbc_batcher *b, uint64_t ticket);
int rbc_batcher_poll(rbc_batcher *b, uint64_t ticket, int *done);
int rbc_batcher_stats(rbc_batcher *b, uint64_t *batches, uint64_t *requests);

/* ---- reedsolomon.Encoder mirror (klauspost v1.9.1 semantics) ---------------
 * Shards are host buffers; lens[i] == 0 marks a missing shard (Go len 0).
 * Reconstruct writes missing shards into the caller's buffers (capacity >= the
 * shard size) and sets their lens; present shards are never modified. */
typedef struct rbc_rs rbc_rs;
int rbc_rs_new(int data_shards, int parity_shards, int device, rbc_rs **out); /* reedsolomon.New */
void rbc_rs_free(rbc_rs *rs);
int rbc_rs_encode(rbc_rs *rs, uint8_t *const *shards, const size_t *lens, int n_shards);
int rbc_rs_verify(rbc_rs *rs, const uint8_t *const *shards, const size_t *lens, int n_shards, int *ok);
int rbc_rs_reconstruct(rbc_rs *rs, uint8_t *const *shards, size_t *lens, int n_shards);
int rbc_rs_reconstruct_data(rbc_rs *rs, uint8_t *const *shards, size_t *lens, int n_shards);
/* Split: out receives n*per bytes (shard i at i*per); *per_shard = per. */
int rbc_rs_split(rbc_rs *rs, const uint8_t *data, size_t len, uint8_t *out, size_t out_cap, size_t *per_shard);
/* Update(shards, newDatashards): parity shards += M[k+r][c] * (old_c ^ new_c)
 * for every changed data shard c (new_lens[c] != 0).  As in Go, shards[c] is
 * left holding old_c ^ new_c.  Errors in Go's order: ErrTooFewShards
 * (n_shards != k+p or n_new != k: len(shards) != r.Shards,
 * len(newDatashards) != r.DataShards), checkShards on
 * both sets, ErrInvalidInput (a changed shard whose old shard is nil, or a
 * nil parity shard); a new shard of another size is ErrShardSize. */
int rbc_rs_update(rbc_rs *rs, uint8_t *const *shards, const size_t *lens, int n_shards,
                  const uint8_t *const *new_data, const size_t *new_lens, int n_new);
/* Join: first k shards, out_size bytes; a NULL shard pointer is Go `nil`. */
int rbc_rs_join(rbc_rs *rs, const uint8_t *const *shards, const size_t *lens, int n_shards, size_t out_size,
                uint8_t *dst);

/* ---- multi-GPU: RCCL all-gather of {root, digest} over xGMI ----------------
 * One process per GPU.  Rank 0 creates the id, the host runtime broadcasts
 * its 128 bytes, every rank calls rbc_comm_init.  gathered receives
 * [nranks][count][64] = {root[32], digest[32]} per instance (ACS output set). */
int rbc_comm_unique_id(uint8_t id_out[128]);
int rbc_comm_init(rbc_ctx *ctx, int nranks, int rank, const uint8_t id[128]);
int rbc_comm_destroy(rbc_ctx *ctx);
int rbc_dev_allgather_roots(rbc_ctx *ctx, void *stream, int count, const uint8_t *roots,
                            const uint8_t *digests, uint8_t *gathered);
/* Ragged shares (total % nranks != 0): every rank sends `slots` records
 * (slots = rbc_acs_max_share, the same on every rank); its own `count` <=
 * slots are packed on the device and the rest are zero.  The digest of an
 * instance with status[i] != 0 (interpolate failed; status nullable) is sent
 * as 32 zero bytes, so a record alone says whether the instance is in the ACS
 * output set.  gathered: [nranks][slots][64]. */
int rbc_dev_allgather_records(rbc_ctx *ctx, void *stream, int count, int slots, const uint8_t *roots,
                              const uint8_t *digests, const int32_t *status, uint8_t *gathered);
/* The communicator as RCCL reports it (ncclCommCount / ncclCommUserRank /
 * ncclGetVersion) and the files the RCCL and HIP runtimes were mapped from
 * (lib paths nullable; truncated to cap). */
int rbc_comm_info(rbc_ctx *ctx, int *nranks, int *rank, int *rccl_version, char *rccl_path, size_t rccl_cap,
                  int *hip_runtime_version, char *hip_path, size_t hip_cap);
/* PCI bus id of a device ("0000:xx:yy.z"), for host NUMA placement per rank. */
int rbc_device_pci_bus_id(int device, char *out, int cap);

/* ---- ACS output-set assembly (host only; the consumer of the all-gather) --
 * The reference's ACS is absent (honeybadger.go:19-21 TODO, sendBatch panics
 * at honeybadger.go:57-59): this is the part of it that turns the gathered
 * RBC outputs into the ordered epoch set.  Instances are partitioned over
 * ranks in contiguous blocks: rank r owns [r*total/nranks, (r+1)*total/nranks). */
int rbc_acs_partition(int total, int nranks, int rank, int *first, int *count);
int rbc_acs_max_share(int total, int nranks, int *slots);
/* gathered [nranks][slots][64] (rbc_dev_allgather_records output, on the
 * host) -> the instances with a non-zero digest, in instance order:
 * instances_out[m] = id, records_out [m][64] (nullable), *out_count = m.
 * Both outputs need room for `total` entries. */
int rbc_acs_assemble(const uint8_t *gathered, int nranks, int slots, int total, int32_t *instances_out,
                     uint8_t *records_out, int *out_count);

/* ---- test / bench utilities (synthetic inputs and result checks) ---------- */
/* dst [rows][pitch] (pitch % 16 == 0): 64-bit word w of local row i, global
 * row r = first_row + i, is splitmix64(seed * 0x9E3779B97F4A7C15 + r * pitch / 8
 * + w), little-endian (restated on the host by cleisthenes_amd.synth). */
int rbc_dev_fill_random(int device, void *stream, uint8_t *dst, uint64_t first_row, uint64_t rows, uint64_t pitch,
                        uint64_t seed);
/* *mismatch_dev (device uint32, zeroed first) = number of 16-byte chunks in
 * which the first len bytes of rows a[r] and b[r] differ, r < rows. */
int rbc_dev_count_mismatch(int device, void *stream, const uint8_t *a, uint64_t a_pitch, const uint8_t *b,
                           uint64_t b_pitch, uint64_t rows, uint64_t len, uint32_t *mismatch_dev);
/* The row-view form: *mismatch_dev = number of 16-byte chunks of data row j
 * (shards + i*inst_pitch + j*row_pitch, first min(16, S - 16q) bytes) that
 * differ from value bytes [j*S + 16q, ...) of values + i*value_pitch, where
 * value bytes at or past value_len compare as zero (the Split pad); i < count,
 * j < k.  value_pitch >= k*S + 16. */
int rbc_dev_count_mismatch_rows(int device, void *stream, const uint8_t *shards, uint64_t inst_pitch,
                                uint32_t row_pitch, int k, uint32_t shard_len, const uint8_t *values,
                                uint64_t value_pitch, uint32_t value_len, uint64_t count, uint32_t *mismatch_dev);
/* The receive guard's input: every row a receiver has to regenerate -- absent
 * (present[i][j] == 0; present nullable = none) or the Byzantine row
 * corrupt[i] >= 0 (corrupt nullable) -- is overwritten over its whole
 * row_pitch with seeded splitmix64 garbage, so that a decode which skipped a
 * row cannot pass on the proposer's intact bytes.  row_pitch % 16 == 0. */
int rbc_dev_poison_rows(int device, void *stream, uint8_t *shards, uint64_t inst_pitch, uint32_t row_pitch, int n,
                        const uint8_t *present, const int32_t *corrupt, uint64_t count, uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif /* RBC_GPU_H */
