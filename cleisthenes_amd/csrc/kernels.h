// kernels.h -- argument blocks and launchers of the batched RBC kernels
// (host side of kernels.hip).  Plain structs passed by value to the kernels.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "../../include/rbc_gpu.h"
#include "host_shared.h"

enum { GF_MODE_ENCODE = 0, GF_MODE_DECODE = 1 };

struct GfArgs {
    int count;                 // instances
    int tiles;                 // column tiles per instance (gf_rows: 16 * tpb bytes; gf_regen: set by its launcher)
    int rc;                    // rows per chunk (template)
    int tpb;                   // gf_rows: threads per block, 256 (4 KiB tiles); 0 = 256
    int wpt;                   // gf_regen: words per lane (set by rbc_launch_gf_regen)
    int R, K;                  // output rows, input rows per instance
    int mode;                  // GF_MODE_*
    const uint8_t *in;         // encode: values [I][value_pitch]; decode: shards [I][N][pitch]
    uint64_t in_inst_pitch;
    uint32_t in_row_pitch;     // decode only
    uint32_t in_inst_bytes;    // readable bytes per instance (buffer bound)
    uint8_t *out;              // shards [I][N][pitch]
    uint64_t out_inst_pitch;
    uint32_t out_row_pitch;
    uint8_t *copy;             // encode: data rows written through; decode: used rows copied (out != in)
    const uint32_t *lens;      // encode: B_i; decode: S_i (nullptr -> uniform_len)
    uint32_t uniform_len;
    const uint8_t *coef;       // R x K bytes (+ inst * coef_inst_stride)
    uint64_t coef_inst_stride;
    const uint8_t *in_idx;     // decode: [I][idx_stride] input row positions (K used)
    const uint8_t *out_idx;    // decode: [I][idx_stride2] output row positions (R regen)
    uint32_t idx_stride, idx_stride2;
    const int32_t *status;     // skip instances with status != 0 (nullable)
    // decode compare mode (nmiss != nullptr): output rows r >= nmiss[inst] are
    // present-and-verified shards; they are compared with the regenerated
    // bytes instead of re-hashed, and only a mismatching row is stored,
    // flagged and appended to the hash list
    const int32_t *nmiss;
    uint32_t *flags;           // [I][n]
    uint32_t *list;            // (inst << 8 | pos) rows to hash
    uint32_t *counter;
    int n;
    const int32_t *rcount;     // per-instance output row count (nullable -> R)
    int prio;                  // wave issue priority 0..3 (set_wave_prio)
};

struct ShaArgs {
    int count;
    int rows_per_inst;         // row slots per instance
    const uint8_t *rows;       // [I][N][row_pitch]
    uint64_t inst_pitch;
    uint32_t row_pitch;
    const uint32_t *lens;      // S_i (nullable)
    uint32_t uniform_len;
    const uint8_t *idx;        // optional row positions [I][idx_stride]
    uint32_t idx_stride;
    const int32_t *status;     // nullable
    uint8_t *leaves;           // [I][N][32] (nullable)
    uint64_t leaves_inst_pitch;
    int per_message;           // 1: each instance is one ECHO message (leaf index = idx[inst])
    const uint64_t *row_offs;  // per_message: message i's bytes at rows + row_offs[i] (nullable: i * inst_pitch)
    const uint32_t *list;      // list mode: rows (inst << 8 | pos), count in *list_count
    const uint32_t *list_count;
    // verify
    int n, depth;
    const uint8_t *branches;   // [I][N][d][32]
    uint64_t br_inst_pitch;
    const uint8_t *roots;      // [I][32]
    const uint8_t *present;    // [I][N] (nullable -> all present)
    uint8_t *valid;            // [I][N]
    int prio;                  // wave issue priority 0..3 (set_wave_prio)
};

struct MerkleArgs {
    int count, n, width, depth, k;
    const uint8_t *leaves;     // [I][N][32]
    uint64_t leaves_inst_pitch;
    uint8_t *roots;            // build: out; check: recomputed root out (nullable)
    uint8_t *branches;         // build: [I][N][d][32] (nullable)
    uint64_t br_inst_pitch;
    const uint8_t *expect_roots;  // check
    int32_t *status;           // check: in/out
    uint8_t *digests;          // check: [I][32] (nullable)
    int trees_per_block;       // set by rbc_launch_merkle
    int prio;                  // wave issue priority 0..3 (set_wave_prio)
    const uint8_t *only;       // check: [I] nonzero = recheck this instance, others untouched (nullable = all)
    int stop_m;                // build, set by rbc_launch_merkle: stop at the layer of stop_m nodes (0 = root)
};

// merkle_recheck_kernel: the receive step's root recheck over the nodes ECHO
// verify established
struct RecheckArgs {
    int count, n, width, depth;
    const uint8_t *leaves;     // [I][N][32]: verified leaves + the regenerated rows' hashes
    uint64_t leaves_inst_pitch;
    const uint8_t *branches;   // [I][N][d][32]: the received ECHO branches
    uint64_t br_inst_pitch;
    const uint8_t *valid;      // [I][N]
    const uint32_t *flags;     // [I][N]: valid rows the re-encoding changed (decode compare)
    const uint8_t *vroots;     // [I][32]: the roots the branches were verified against
    const uint8_t *expect_roots;  // [I][32]
    int32_t *status;           // in/out
    uint8_t *need_full;        // [I] out: 1 = leave the instance to the full recheck (merkle_kernel<true>, only)
    int inst_per_block;        // set by rbc_launch_recheck
    int prio;
};
hipError_t rbc_launch_recheck(const RecheckArgs &a, hipStream_t st);

// merkle_path_kernel: shared-path branch verification over precomputed leaves
struct PathArgs {
    int count, n, width, lg_width, depth;
    const uint8_t *leaves;     // [I][N][32]
    uint64_t leaves_inst_pitch;
    const uint8_t *branches;   // [I][N][d][32]
    uint64_t br_inst_pitch;
    const uint8_t *roots;      // [I][32]
    const uint8_t *present;    // [I][N] (nullable -> all present)
    const int32_t *status;     // nullable
    uint8_t *valid;            // [I][N]
    int inst_per_block;        // set by rbc_launch_merkle_path
    int prio;                  // wave issue priority 0..3 (set_wave_prio)
};

struct PrepArgs {
    int count, n, k;
    const uint8_t *valid;      // [I][valid_stride]
    uint32_t valid_stride;
    const uint8_t *M;          // encode matrix [n][k]
    uint8_t *used;             // [I][used_stride]   first k valid positions
    uint32_t used_stride;
    uint8_t *regen;            // [I][regen_stride]  the other n-k positions
    uint32_t regen_stride;
    uint8_t *dmat;             // [I][dmat_stride] = (n-k) x k decode matrix
    uint64_t dmat_stride;
    int32_t *status;           // out
    // compare mode: regen = [missing..., present-unused...], nmiss[i] = #missing,
    // missing rows appended to list, flags[i][*] zeroed
    int32_t *nmiss;
    uint32_t *flags;
    uint32_t *list;
    uint32_t *counter;
    // FFT codec: D covers only the missing data rows (rcount[i] of them, they
    // lead `regen`); cls[i][pos] = 0 skip / 1 store / 2 compare for pos >= k
    int fft;
    int32_t *rcount;
    uint8_t *cls;
    uint32_t cls_stride;
    const uint8_t *gf_exp;     // device exp[512] / log[256] tables (FFT prepare)
    const uint8_t *gf_log;
    int prio;                  // wave issue priority 0..3 (set_wave_prio)
};

struct JoinArgs {
    int count, k;
    uint32_t chunks;           // 16-byte chunks per instance (= value_pitch / 16)
    uint32_t blocks_per_inst;  // set by rbc_launch_join
    const uint8_t *shards;     // full codeword rows
    uint64_t inst_pitch;
    uint32_t row_pitch;
    uint32_t inst_bytes;       // readable bytes per instance
    const uint32_t *lens;      // S_i (nullable)
    uint32_t uniform_len;
    uint8_t *values;           // [I][value_pitch]
    uint32_t value_pitch;
    const int32_t *status;
    int prio;                  // wave issue priority 0..3 (set_wave_prio)
};

// rs_fft_kernel (rs_fft.hip): additive-FFT systematic encode, one lane per
// dword column of one instance
struct FftArgs {
    int count, n, k;
    int mode;                  // GF_MODE_ENCODE: values -> data + parity rows;
                               // GF_MODE_DECODE: data rows -> parity rows by class
    const uint8_t *values;     // encode: [I][value_pitch]
    uint32_t value_pitch;
    uint8_t *shards;           // [I][N][row_pitch]
    uint64_t inst_pitch;
    uint32_t row_pitch;
    const uint32_t *lens;      // encode: B_i, decode: S_i (nullable)
    uint32_t uniform_len;
    const int32_t *status;     // nullable
    // decode: per-position class [I][cls_stride] (0 skip, 1 store, 2 compare);
    // nullptr -> store every parity position
    const uint8_t *cls;
    uint32_t cls_stride;       // multiple of 4
    uint32_t *flags;           // [I][n]
    uint32_t *list;
    uint32_t *counter;
    int prio;                  // wave issue priority 0..3 (set_wave_prio)
    // decode, optional: also assemble interpolate's value from the k data rows
    // the kernel loads anyway -- join[i][0 .. k*S) = data rows 0..k-1 of S
    // bytes, zeros up to join_pitch (uniform S only, join_pitch - k*S < 256)
    uint8_t *join;
    uint32_t join_pitch;
};

// VAL / ECHO marshaling (wire.hip): message (i, j) = pb.Message bytes of
// the request for shard j of instance i, at out + (i*n + j)*out_pitch.
struct WireArgs {
    int count, n, depth, type;
    const uint8_t *shards;
    uint64_t inst_pitch;
    uint32_t row_pitch;
    const uint32_t *lens;  // per instance, or NULL: uniform_len
    uint32_t uniform_len;
    const uint8_t *branches;  // [count][n][depth][32]
    const uint8_t *roots;     // [count][32]
    uint8_t *out;
    uint64_t out_pitch;  // % 16 == 0
    uint32_t *out_lens;  // [count*n], nullable
};
hipError_t rbc_launch_marshal_val(const WireArgs &a, hipStream_t st);

hipError_t rbc_launch_rs_fft(const FftArgs &a, hipStream_t st);

int rbc_gf_pick_rc(int R, int rcmax);
hipError_t rbc_launch_gf_rows(const GfArgs &a, hipStream_t st);
// interpolate's missing data rows (FFT codec, gf_regen.hip): one wave per column tile of 256 * W
// bytes owns every row (W and the tiles chosen from the row length); needs rcount (row count <= R)
hipError_t rbc_launch_gf_regen(const GfArgs &a, hipStream_t st);
hipError_t rbc_launch_sha_rows(const ShaArgs &a, bool verify, hipStream_t st);
// receive step: v's rows (list or all; branch walk + verdict when v_walk) and
// r's listed regen rows in one launch (count <= 0 disables a side)
// zero0 / zero1 (nullable, 16 B each): counters one lane zeroes during the launch (receive step)
hipError_t rbc_launch_sha_rx(const ShaArgs &v, const ShaArgs &r, bool v_walk, hipStream_t st, uint4 *zero0 = nullptr,
                             uint4 *zero1 = nullptr);
hipError_t rbc_launch_merkle(const MerkleArgs &a, bool check, hipStream_t st);
hipError_t rbc_launch_merkle_path(const PathArgs &a, hipStream_t st);
hipError_t rbc_launch_decode_prepare(const PrepArgs &a, hipStream_t st);
hipError_t rbc_launch_digest(const uint8_t *leaves, uint64_t leaves_inst_pitch, int k, const int32_t *status,
                             uint8_t *digests, int count, hipStream_t st, int prio = 0);
hipError_t rbc_launch_join(const JoinArgs &a, hipStream_t st);
hipError_t rbc_launch_inject_faults(uint8_t *shards, uint64_t inst_pitch, uint32_t row_pitch,
                                    const int32_t *corrupt, int count, hipStream_t st);
// roots_src -> roots_dst (nullable): each instance's 32-B root copied on the way (receive step)
hipError_t rbc_launch_compact_present(const uint8_t *present, int n, int count, uint8_t *valid, uint32_t *list,
                                     uint32_t *counter, hipStream_t st, int prio = 0,
                                     const uint8_t *roots_src = nullptr, uint8_t *roots_dst = nullptr);
hipError_t rbc_launch_pack_records(const uint8_t *roots, const uint8_t *digests, const int32_t *status, int count,
                                   int slots, uint8_t *out, hipStream_t st);
hipError_t rbc_launch_fill_random(uint8_t *dst, uint64_t first_row, uint64_t rows, uint64_t pitch, uint64_t seed,
                                  hipStream_t st);
// present rows of a pinned host batch -> device rows (zero-copy reads), absent rows zeroed
hipError_t rbc_launch_gather_present(const uint8_t *host, uint64_t hpitch, uint32_t S, const uint8_t *present,
                                     uint8_t *dev, uint32_t dpitch, uint32_t rows, hipStream_t st);
// the messages of a pinned validate arena -> the same offsets of a device arena
// (zero-copy reads of bytes [offs[i], offs[i] + lens[i]) only; the rest untouched)
hipError_t rbc_launch_gather_msgs(const uint8_t *host, const uint64_t *offs, const uint32_t *lens, uint32_t count,
                                  uint8_t *dev, uint32_t avg_len, hipStream_t st);
// pinned host values (device array of their addresses) -> device value rows (zero-copy reads)
// rows [0, width) of src (src_pitch) into dst at dst_pitch, zeros to dst_pitch
hipError_t rbc_launch_pack_rows(const uint8_t *src, uint32_t src_pitch, uint8_t *dst, uint32_t dst_pitch,
                                uint32_t width, uint32_t rows, hipStream_t st);
// rows from device addresses (0 = absent), lens per instance of n rows
hipError_t rbc_launch_gather_ptrs(const uint64_t *ptrs, const uint32_t *lens, uint32_t n, uint8_t *dev,
                                  uint32_t dpitch, uint32_t rows, hipStream_t st);
hipError_t rbc_launch_gather_values(const uint64_t *ptrs, const uint32_t *lens, uint32_t count, uint8_t *dev,
                                    uint64_t vpitch, hipStream_t st);
hipError_t rbc_launch_count_mismatch(const uint8_t *a, uint64_t a_pitch, const uint8_t *b, uint64_t b_pitch,
                                     uint64_t rows, uint64_t len, uint32_t *counter, hipStream_t st);
hipError_t rbc_launch_count_mismatch_rows(const uint8_t *shards, uint64_t inst_pitch, uint32_t row_pitch, int k,
                                          uint32_t S, const uint8_t *values, uint64_t value_pitch, uint32_t B,
                                          uint64_t count, uint32_t *counter, hipStream_t st);
// receive-guard input: absent rows (present == 0) and corrupt[i] filled with seeded garbage
hipError_t rbc_launch_poison_rows(uint8_t *shards, uint64_t inst_pitch, uint32_t row_pitch, int n,
                                  const uint8_t *present, const int32_t *corrupt, uint64_t count, uint64_t seed,
                                  hipStream_t st);
