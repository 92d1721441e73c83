// kernels.hip -- batched RBC data-path kernels for MI355X (gfx950).
//
// Replaces, for thousands of RBC instances per launch, the work behind
//   shard()           rbc/rbc.go:97-100  (klauspost Split + Encode)
//   Merkle build      (VAL construction, rbc/rbc.go:42; docs/RBC-EN.md:31)
//   validateMessage() rbc/rbc.go:92-95   (ECHO branch verify)
//   interpolate()     rbc/rbc.go:86-90   (Reconstruct + re-encode + root recheck)
//
// HBM layout:
//   values   [I][value_pitch]            proposer input, B_i bytes used
//   shards   [I][N][shard_pitch]         shard_pitch % 64 == 0, >= S_i; bytes in
//                                        [S_i, pitch) are written as zero
//   leaves   [I][N][32]                  SHA-256(shard)
//   roots    [I][32]
//   branches [I][N][d][32]               level-0 slot zero when sibling empty
//   valid    [I][N] u8 ; status [I] i32 ; digests [I][32]
// No MFMA: GF(2^8) and SHA-256 are not dense contractions (north_star).
#include <algorithm>

#include "device_common.h"
#include "kernels.h"

using namespace rbcdev;

#include "buffer_io.h"

// ============================================================================
// gf_rows: out[r] = XOR_j coef[r][j] * in[j]   (klauspost codeSomeShards)
// One block = one instance x one 4 KiB column tile; each thread owns 16
// consecutive bytes (4 packed words) of every row.  Output rows are done in
// chunks of RC so the RC x 4 accumulators stay in VGPRs; the chunk's perm
// tables (RC x K x 20 B) live in LDS and are read by wave-uniform broadcast.
// Encode mode reads data row j straight out of the value bytes at j*S
// (Split), funnel-shifting unaligned rows, masks the zero pad, and writes the
// data rows through to shards[0..k) on the first chunk.
// ============================================================================
template <int RC, int TPB>
__global__ __launch_bounds__(TPB, (RC <= 21 ? 3 : 2)) void gf_rows_kernel(GfArgs a) {
    set_wave_prio(a.prio);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int KP = (a.K + 1) & ~1;
    uint4 *s_t01 = reinterpret_cast<uint4 *>(smem);
    uint32_t *s_t2 = reinterpret_cast<uint32_t *>(smem + (size_t)16 * RC * KP);
    uint8_t *s_in = reinterpret_cast<uint8_t *>(smem + (size_t)20 * RC * KP);
    uint8_t *s_out = s_in + 256;  // 256 = max positions

    // block -> (work item = instance x column tile, row chunk c).  The chunks
    // of one item are 8 block ids apart, i.e. dispatched to the same XCD under
    // round-robin placement, so the item's input rows are re-read from that
    // XCD's L2 (speed only; any placement is correct).
    const int chunks = a.R > 0 ? (a.R + RC - 1) / RC : 1;  // R == 0: Split copy only
    const int grp = blockIdx.x / (8 * chunks), rem = blockIdx.x - grp * 8 * chunks;
    const int c = rem >> 3;
    const int item = grp * 8 + (rem & 7);
    if (item >= a.count * a.tiles) return;
    const int inst = item / a.tiles;
    const int tile = item - inst * a.tiles;
    const int tid = threadIdx.x;
    if (a.status && a.status[inst] != 0) return;

    // shard length of this instance
    uint32_t S;
    uint32_t B = 0;
    if (a.mode == GF_MODE_ENCODE) {
        B = inst_len(a.lens, a.uniform_len, inst);
        S = (B + a.K - 1) / a.K;
    } else {
        S = inst_len(a.lens, a.uniform_len, inst);
    }
    const uint32_t tile_byte0 = (uint32_t)tile * (16u * TPB);  // TPB threads x 16 B
    if (tile_byte0 >= a.out_row_pitch) return;
    const uint32_t my_off = tile_byte0 + 16u * tid;      // byte offset inside a row
    const bool my_store = my_off < a.out_row_pitch;

    const uint8_t *in_inst = a.in + (size_t)inst * a.in_inst_pitch;
    uint8_t *out_inst = a.out + (size_t)inst * a.out_inst_pitch;
    const rsrc_t rin = make_rsrc(in_inst, a.in_inst_bytes);

    if (a.mode == GF_MODE_DECODE) {
        for (int t = tid; t < a.K; t += TPB) s_in[t] = a.in_idx[(size_t)inst * a.idx_stride + t];
        for (int t = tid; t < a.R; t += TPB) s_out[t] = a.out_idx[(size_t)inst * a.idx_stride2 + t];
    }

    // load 16 bytes of input row j for this thread (masked to the row)
    auto load_row = [&](int j) -> uint4 {
        if (j >= a.K) return make_uint4(0, 0, 0, 0);
        if (a.mode == GF_MODE_ENCODE) {
            const uint32_t row0 = (uint32_t)j * S;                   // Split: data[j*S : (j+1)*S]
            const int lim = (int)min(S, B > row0 ? B - row0 : 0u);  // bytes of this row that are data
            uint4 v = make_uint4(0, 0, 0, 0);
            if ((int)my_off < lim) {
                v = bload16(rin, row0 + my_off);  // unaligned when S % 16 != 0
                if ((int)my_off + 16 > lim) v = mask16(v, lim - (int)my_off);
            }
            return v;
        } else {
            // the row position is wave-uniform: row start in SGPRs (s_mul), not a per-lane v_mul_lo;
            // a lane past the pitch (never stored) loads a clamped column: the buffer range check
            // does not cover the scalar row offset, so the last row's overhang could leave the buffer
            return bload16s(rin, min(my_off, a.in_row_pitch - 16u), uniform(s_in[j]) * a.in_row_pitch);
        }
    };

    const int cmp_from = a.nmiss ? a.nmiss[inst] : 0x7fffffff;
    const int rlim = a.rcount ? min(a.rcount[inst], a.R) : a.R;  // block-uniform
    if (a.R > 0 && c * RC >= rlim) return;
    {
        const int r0 = c * RC;
        const int rows = min(RC, rlim - r0);
        for (int e = tid; e < RC * KP; e += TPB) {
            const int r = e / KP, j = e - r * KP;
            uint32_t cf = 0;
            if (r < rows && j < a.K)
                cf = a.coef[(size_t)inst * a.coef_inst_stride + (size_t)(r0 + r) * a.K + j];
            uint4 t01;
            uint32_t t2;
            gf_tables(cf, t01, t2);
            // layout [j][r] (t2 as {j even, j odd} pairs): the RC rows of one
            // input column are consecutive, so every LDS read in the hot loop
            // is one base VGPR plus a compile-time immediate offset
            s_t01[j * RC + r] = t01;
            s_t2[((j >> 1) * RC + r) * 2 + (j & 1)] = t2;
        }
        __syncthreads();

        uint32_t acc[RC][4];
#pragma unroll
        for (int r = 0; r < RC; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0;

        const bool do_copy = (c == 0) && a.copy && my_store;
        // one input pair (rows j, j+1) into all RC accumulators
        auto mac_pair = [&](int j, const uint4 &xa, const uint4 &xb) {
            if (do_copy) {
                const uint32_t pa = (a.mode == GF_MODE_ENCODE) ? (uint32_t)j : s_in[j];
                *reinterpret_cast<uint4 *>(a.copy + (size_t)inst * a.out_inst_pitch +
                                           (size_t)pa * a.out_row_pitch + my_off) = xa;
                if (j + 1 < a.K) {
                    const uint32_t pb = (a.mode == GF_MODE_ENCODE) ? (uint32_t)(j + 1) : s_in[j + 1];
                    *reinterpret_cast<uint4 *>(a.copy + (size_t)inst * a.out_inst_pitch +
                                               (size_t)pb * a.out_row_pitch + my_off) = xb;
                }
            }
            const GfSel sa0 = gf_sel(xa.x), sa1 = gf_sel(xa.y), sa2 = gf_sel(xa.z), sa3 = gf_sel(xa.w);
            const GfSel sb0 = gf_sel(xb.x), sb1 = gf_sel(xb.y), sb2 = gf_sel(xb.z), sb3 = gf_sel(xb.w);
#pragma unroll
            for (int r = 0; r < RC; ++r) {
                if (r >= rows) break;  // block-uniform: a short last chunk skips its padding rows
                const uint4 ta = s_t01[j * RC + r];
                const uint4 tb = s_t01[(j + 1) * RC + r];
                const uint2 t2 = *reinterpret_cast<const uint2 *>(&s_t2[((j >> 1) * RC + r) * 2]);
                acc[r][0] = xor3(acc[r][0], gf_mul4(ta, t2.x, sa0), gf_mul4(tb, t2.y, sb0));
                acc[r][1] = xor3(acc[r][1], gf_mul4(ta, t2.x, sa1), gf_mul4(tb, t2.y, sb1));
                acc[r][2] = xor3(acc[r][2], gf_mul4(ta, t2.x, sa2), gf_mul4(tb, t2.y, sb2));
                acc[r][3] = xor3(acc[r][3], gf_mul4(ta, t2.x, sa3), gf_mul4(tb, t2.y, sb3));
            }
        };
        // two buffers of an input pair each, every load issued one pair of
        // multiplies ahead of its use and no register rotation: the compiler's
        // wait at the loop top then covers loads issued a whole pair earlier
        uint4 a0 = load_row(0), a1 = load_row(1), b0, b1;
        for (int j = 0; j < KP; j += 4) {
            b0 = load_row(j + 2);
            b1 = load_row(j + 3);
            mac_pair(j, a0, a1);
            a0 = load_row(j + 4);
            a1 = load_row(j + 5);
            if (j + 2 < KP) mac_pair(j + 2, b0, b1);
        }
        if (my_store) {
            const int nvalid = (int)S - (int)my_off;  // zero the bytes past S
#pragma unroll
            for (int r = 0; r < RC; ++r) {
                if (r < rows) {
                    const uint32_t pos = (a.mode == GF_MODE_ENCODE) ? (uint32_t)(a.K + r0 + r) : s_out[r0 + r];
                    uint4 v = make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
                    if (nvalid < 16) v = mask16(v, nvalid);
                    uint4 *dst = reinterpret_cast<uint4 *>(out_inst + (size_t)pos * a.out_row_pitch + my_off);
                    if (cmp_from <= r0 + r) {
                        // valid shard that was not used: keep it unless the
                        // re-encoding differs, then overwrite and queue a re-hash
                        const uint4 o = *dst;
                        if (o.x != v.x || o.y != v.y || o.z != v.z || o.w != v.w) {
                            *dst = v;
                            if (atomicOr(&a.flags[(size_t)inst * a.n + pos], 1u) == 0u)
                                a.list[atomicAdd(a.counter, 1u)] = ((uint32_t)inst << 8) | pos;
                        }
                    } else {
                        *dst = v;
                    }
                }
            }
        }
    }
}

// ============================================================================
// sha_rows: leaf_j = SHA-256(shard_j) for a list of rows, one lane per row;
// VERIFY additionally walks the Merkle branch (validateMessage,
// rbc/rbc.go:92-95) and writes valid = present && (root' == root).
// ============================================================================
template <bool VERIFY>
// Occupancy of the SHA kernels: under the two-stream schedule both streams'
// SHA launches (2,048 waves each at C2) must be resident together, 4 waves
// per SIMD, so every kernel that hashes rows is held to <= 128 VGPRs
// (the verify walk then spills 36 B per lane, outside the block loop)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void sha_rows_kernel(ShaArgs a) {
    set_wave_prio(a.prio);
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    int inst, pos;
    if (a.list) {  // compacted (inst, pos) work list built on the device
        if (t >= (int)*a.list_count) return;
        const uint32_t e = a.list[t];
        inst = (int)(e >> 8);
        pos = (int)(e & 0xffu);
    } else {
        if (t >= a.count * a.rows_per_inst) return;
        inst = t / a.rows_per_inst;
        const int slot = t - inst * a.rows_per_inst;
        // per_message: every "instance" is one independent ECHO message whose
        // leaf index is idx[inst]; otherwise slot -> row position (idx optional)
        pos = a.idx ? (int)a.idx[(size_t)inst * a.idx_stride + slot] : slot;
    }
    if (a.status && a.status[inst] != 0) return;
    const int rowsel = a.per_message ? 0 : pos;
    const uint32_t S = inst_len(a.lens, a.uniform_len, inst);
    const uint8_t *row = a.row_offs ? a.rows + a.row_offs[inst]  // packed per-message arena (64-B aligned)
                                    : a.rows + (size_t)inst * a.inst_pitch + (size_t)rowsel * a.row_pitch;
    Sha256State s;
    sha256_row(row, S, s);
    uint32_t h[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) h[q] = s.h[q];
    if (a.leaves) store_digest(a.leaves + (size_t)inst * a.leaves_inst_pitch + 32u * rowsel, h);
    if (VERIFY) {
        const uint8_t *br = a.branches + (size_t)inst * a.br_inst_pitch + (size_t)rowsel * a.depth * 32u;
        uint32_t tix = (uint32_t)pos;
        for (int l = 0; l < a.depth; ++l, tix >>= 1) {
            const bool empty = (l == 0) && ((pos ^ 1) >= a.n);
            uint32_t o[8];
            if (empty) {
                sha256_node32(h, o);
            } else {
                // one node body with selected inputs (two inlined orderings
                // cost code size and registers)
                uint32_t sib[8], L[8], R[8];
                load_digest(br + 32u * l, sib);
                const bool right = (tix & 1u) != 0;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    L[q] = right ? sib[q] : h[q];
                    R[q] = right ? h[q] : sib[q];
                }
                sha256_node64(L, R, o);
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) h[q] = o[q];
        }
        uint32_t root[8];
        load_digest(a.roots + (size_t)inst * 32u, root);
        bool ok = true;
#pragma unroll
        for (int q = 0; q < 8; ++q) ok = ok && (h[q] == root[q]);
        const bool inrange = pos < a.n;
        if (a.per_message) {
            a.valid[inst] = (ok && inrange) ? 1 : 0;
        } else {
            const bool present = a.present ? a.present[(size_t)inst * a.n + pos] != 0 : true;
            a.valid[(size_t)inst * a.n + pos] = (ok && present) ? 1 : 0;
        }
    }
}

// Receive step (rbc_dev_receive_step): ONE launch hashes the received ECHO
// shards of batch t (list v, or every row when v.list is null; with
// v_walk the branch walk + verdict of sha_rows_kernel<true> follows) and the
// rows interpolate regenerated for batch t-1 (list r).  Separately, batch
// t-1's regen hashing is a latency-bound tail (42 rows x 1024 instances at
// C2 = 672 waves of 373 serial compressions for 1,024 SIMDs) and the
// verify 1,376 waves; together they are 2,048 waves, as full as the leaves.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void sha_rx_kernel(ShaArgs v, ShaArgs r, int v_walk,
                                                                                                   uint4 *zero0,
                                                                                                   uint4 *zero1) {
    set_wave_prio(v.prio);
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    // the receive step's list counters for the NEXT list builders (this call's
    // decode, the next call's compaction), which nothing here reads: zeroed
    // by one lane instead of two memset launches on the receiver's stream
    if (t == 0) {
        if (zero0) *zero0 = make_uint4(0u, 0u, 0u, 0u);
        if (zero1) *zero1 = make_uint4(0u, 0u, 0u, 0u);
    }
    const int nv = v.count <= 0 ? 0 : (v.list ? (int)*v.list_count : v.count * v.rows_per_inst);
    // r's rows start at the next whole wave after v's, so every wave is all-v
    // or all-r and the choice between the two argument blocks is scalar (the
    // selected pointers and pitches stay in SGPRs: no spills at 128 VGPRs)
    const int nv_pad = (nv + 63) & ~63;
    const bool isv = __builtin_amdgcn_readfirstlane(t & ~63) < nv_pad;
    int inst, pos;
    if (isv) {
        if (t >= nv) return;
        if (v.list) {
            const uint32_t e = v.list[t];
            inst = (int)(e >> 8);
            pos = (int)(e & 0xffu);
        } else {
            inst = t / v.rows_per_inst;
            pos = t - inst * v.rows_per_inst;
        }
    } else {
        t -= nv_pad;
        if (r.count <= 0 || t >= (int)*r.list_count) return;
        const uint32_t e = r.list[t];
        inst = (int)(e >> 8);
        pos = (int)(e & 0xffu);
        if (r.status && r.status[inst] != 0) return;
    }
    const uint8_t *rows = isv ? v.rows : r.rows;
    const uint64_t inst_pitch = isv ? v.inst_pitch : r.inst_pitch;
    const uint32_t row_pitch = isv ? v.row_pitch : r.row_pitch;
    const uint32_t S = isv ? inst_len(v.lens, v.uniform_len, inst) : inst_len(r.lens, r.uniform_len, inst);
    uint8_t *leaves = isv ? v.leaves : r.leaves;
    const uint64_t lpitch = isv ? v.leaves_inst_pitch : r.leaves_inst_pitch;
    Sha256State s;
    sha256_row(rows + (size_t)inst * inst_pitch + (size_t)pos * row_pitch, S, s);
    uint32_t h[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) h[q] = s.h[q];
    if (leaves) store_digest(leaves + (size_t)inst * lpitch + 32u * pos, h);
    if (isv && v_walk) {
        const uint8_t *br = v.branches + (size_t)inst * v.br_inst_pitch + (size_t)pos * v.depth * 32u;
        uint32_t tix = (uint32_t)pos;
        for (int l = 0; l < v.depth; ++l, tix >>= 1) {
            const bool empty = (l == 0) && ((pos ^ 1) >= v.n);
            uint32_t o[8];
            if (empty) {
                sha256_node32(h, o);
            } else {
                // one node body with selected inputs (two inlined orderings
                // cost code size and registers)
                uint32_t sib[8], L[8], R[8];
                load_digest(br + 32u * l, sib);
                const bool right = (tix & 1u) != 0;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    L[q] = right ? sib[q] : h[q];
                    R[q] = right ? h[q] : sib[q];
                }
                sha256_node64(L, R, o);
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) h[q] = o[q];
        }
        uint32_t root[8];
        load_digest(v.roots + (size_t)inst * 32u, root);
        bool ok = true;
#pragma unroll
        for (int q = 0; q < 8; ++q) ok = ok && (h[q] == root[q]);
        const bool present = v.present ? v.present[(size_t)inst * v.n + pos] != 0 : true;
        v.valid[(size_t)inst * v.n + pos] = (ok && present) ? 1 : 0;
    }
}

// Two rows per lane (rows 2t, 2t+1 of one instance, so one length), the
// compressions interleaved: the per-wave dependent chain halves its stalls
// (profiles/r01_sha_probe.txt: 6,071 SIMD clk per row-compression at one
// wave per SIMD vs 6,423 for one row per lane at two).  Launched for the
// full-instance grids (leaves, ECHO verify) when N is even; list mode and
// per-message verify keep sha_rows_kernel.
template <bool VERIFY>
__global__ __launch_bounds__(256) void sha_rows2_kernel(ShaArgs a) {
    set_wave_prio(a.prio);
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int half = a.rows_per_inst >> 1;
    if (t >= a.count * half) return;
    const int inst = t / half;
    const int slot = 2 * (t - inst * half);
    if (a.status && a.status[inst] != 0) return;
    int pos[2];
#pragma unroll
    for (int r = 0; r < 2; ++r)
        pos[r] = a.idx ? (int)a.idx[(size_t)inst * a.idx_stride + slot + r] : slot + r;
    const uint32_t S = inst_len(a.lens, a.uniform_len, inst);
    const uint8_t *base = a.rows + (size_t)inst * a.inst_pitch;
    Sha256State s[2];
    sha256_row2(base + (size_t)pos[0] * a.row_pitch, base + (size_t)pos[1] * a.row_pitch, S, s);
    uint32_t h[2][8];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int q = 0; q < 8; ++q) h[r][q] = s[r].h[q];
    if (a.leaves)
#pragma unroll
        for (int r = 0; r < 2; ++r) store_digest(a.leaves + (size_t)inst * a.leaves_inst_pitch + 32u * pos[r], h[r]);
    if (VERIFY) {
        // N even: every level-0 sibling exists (no empty padding leaf)
        const uint8_t *br[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) br[r] = a.branches + (size_t)inst * a.br_inst_pitch + (size_t)pos[r] * a.depth * 32u;
        for (int l = 0; l < a.depth; ++l) {
            uint32_t L[2][8], Rr[2][8], o[2][8];
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                uint32_t sib[8];
                load_digest(br[r] + 32u * l, sib);
                const bool right = ((uint32_t)pos[r] >> l) & 1u;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    L[r][q] = right ? sib[q] : h[r][q];
                    Rr[r][q] = right ? h[r][q] : sib[q];
                }
            }
            sha256_node64x2(L, Rr, o);
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int q = 0; q < 8; ++q) h[r][q] = o[r][q];
        }
        uint32_t root[8];
        load_digest(a.roots + (size_t)inst * 32u, root);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            bool ok = true;
#pragma unroll
            for (int q = 0; q < 8; ++q) ok = ok && (h[r][q] == root[q]);
            const bool present = a.present ? a.present[(size_t)inst * a.n + pos[r]] != 0 : true;
            a.valid[(size_t)inst * a.n + pos[r]] = (ok && present && pos[r] < a.n) ? 1 : 0;
        }
    }
}

// ============================================================================
// merkle: G trees per one-wave block.  BUILD writes root + all N branches;
// CHECK recomputes the root over the re-encoded leaves, compares it with the
// expected root (interpolate's recheck).  Node convention (frozen):
// H(L || R), empty padding leaves contribute no bytes.
// The node hashes of one level of all G trees are packed onto consecutive
// lanes, so the narrow upper levels of a tree share a pass instead of idling
// most lanes of one wave per tree (N = 256, G = 2: 6 instead of 9 passes per
// tree; N = 128, G = 2: 4.5 instead of 7).  One-wave blocks: a 256-thread
// form measured the same alone but slowed the bench's two-stream pipeline
// (it is the hardest block shape to place beside the other stream's kernels).  Only internal nodes live in LDS ([G][W][8] words,
// node i of tree g at g*W + i, i in [1, W)); the leaf level reads its children
// straight from the leaves in HBM.
// ============================================================================
template <bool CHECK>
__global__ __launch_bounds__(64) void merkle_kernel(MerkleArgs a) {
    set_wave_prio(a.prio);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *nodes = reinterpret_cast<uint32_t *>(smem);
    const int G = a.trees_per_block, W = a.width, n = a.n;
    const int inst0 = (int)blockIdx.x * G;
    const int tid = threadIdx.x;
    const int m_last = (!CHECK && a.stop_m) ? a.stop_m : 1;
    for (int m = W >> 1, lgm = a.depth - 1; m >= m_last; m >>= 1, --lgm) {
        for (int t = tid; t < G * m; t += 64) {
            const int g = t >> lgm, i = m + (t & (m - 1));
            const int inst = inst0 + g;
            if (inst >= a.count || (CHECK && a.only && !a.only[inst])) continue;
            const int lc = 2 * i, rc = lc + 1;
            // one compression body for every node form (fewer live registers):
            // H(L || R) = [L | R] + a constant pad block; H(L) (right child an
            // empty padding leaf) = [L | 0x80 .. | 256 bits]; H("") constant
            uint32_t w[16];
            bool two = true, none = false;
            if (lc >= W) {  // leaf level: children are leaves lc-W, rc-W (empty past n)
                const int jl = lc - W, jr = rc - W;
                const uint8_t *lv = a.leaves + (size_t)inst * a.leaves_inst_pitch;
                none = jl >= n;
                uint32_t l[8], r[8];
                load_digest(lv + 32u * (none ? 0 : jl), l);
                if (jr < n) load_digest(lv + 32u * jr, r);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    w[q] = l[q];
                    w[8 + q] = jr < n ? r[q] : 0u;
                }
                if (jr >= n) {
                    w[8] = 0x80000000u;
                    w[15] = 256u;
                    two = false;
                }
            } else {
                const uint32_t *nl = nodes + ((size_t)g * W + lc) * 8, *nr = nodes + ((size_t)g * W + rc) * 8;
#pragma unroll
                for (int q = 0; q < 8; ++q) { w[q] = nl[q]; w[8 + q] = nr[q]; }
            }
            uint32_t o[8];
            if (none) {
                sha256_empty(o);
            } else {
                Sha256State st;
                sha256_init(st);
                sha256_compress(st, w);
                if (two) {
#pragma unroll
                    for (int q = 0; q < 16; ++q) w[q] = 0;
                    w[0] = 0x80000000u;
                    w[15] = 512u;
                    sha256_compress(st, w);
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) o[q] = st.h[q];
            }
            uint32_t *dst = nodes + ((size_t)g * W + i) * 8;
#pragma unroll
            for (int q = 0; q < 8; ++q) dst[q] = o[q];
        }
        __syncthreads();
    }
    if (!CHECK && a.stop_m) {
        // W = 256, stopped at the layer of 32 nodes (level 3): merkle_top_kernel
        // finishes the tree.  Hand the layer over in the level-4..7 branch
        // slots of leaves 0..7 (1 KiB, node 32 + q at leaf q / 4, slot 4 + q % 4,
        // as words); merkle_top_kernel reads them before it writes those slots.
        for (int e = tid; e < G * 32; e += 64) {
            const int g = e >> 5, q = e & 31, inst = inst0 + g;
            if (inst >= a.count) continue;
            const uint32_t *nd = nodes + ((size_t)g * W + 32 + q) * 8;
            uint4 *dst = reinterpret_cast<uint4 *>(a.branches + (size_t)inst * a.br_inst_pitch +
                                                   ((size_t)(q >> 2) * a.depth + 4 + (q & 3)) * 32u);
            dst[0] = make_uint4(nd[0], nd[1], nd[2], nd[3]);
            dst[1] = make_uint4(nd[4], nd[5], nd[6], nd[7]);
        }
    }
    // roots: one thread per tree (W == 1: the root is leaf 0)
    for (int g = tid; g < G; g += 64) {
        const int inst = inst0 + g;
        if (!CHECK && a.stop_m) break;  // merkle_top_kernel writes them
        if (inst >= a.count || (CHECK && a.only && !a.only[inst])) continue;
        uint32_t root[8];
        if (W == 1) {
            load_digest(a.leaves + (size_t)inst * a.leaves_inst_pitch, root);
        } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) root[q] = nodes[((size_t)g * W + 1) * 8 + q];
        }
        if (!CHECK) {
            store_digest(a.roots + (size_t)inst * 32u, root);
        } else {
            if (a.status && a.status[inst] != 0) continue;
            uint32_t ex[8];
            load_digest(a.expect_roots + (size_t)inst * 32u, ex);
            bool ok = true;
#pragma unroll
            for (int q = 0; q < 8; ++q) ok = ok && (ex[q] == root[q]);
            if (a.status) a.status[inst] = ok ? 0 : RBC_ERR_ROOT_MISMATCH;
            if (a.roots) store_digest(a.roots + (size_t)inst * 32u, root);
        }
    }
    if (!CHECK && a.branches && a.depth > 0) {  // W == 1: no branch bytes
        // branch[j][l] = node ((W + j) >> l) ^ 1; one 16-byte half per item,
        // item e of a tree = (jl = j*lw + l, half) at e = 2*jl + half, so a
        // wave store covers 1 KiB of consecutive branch bytes (lw = depth) or
        // eight leaves' first 128-B lines (lw = 4).  jl advances by 32 per
        // pass: (j, l) step by (32 / lw, 32 % lw) with a carry, no integer
        // division inside the loop.
        // Level 0 siblings are leaves (zero slot when past n).
        // With stop_m (W = 256) only levels 0..3 are written here (lw = 4, the
        // first 128-B line of each leaf's branch); merkle_top_kernel writes 4..7.
        const int depth = a.depth, lw = a.stop_m ? 4 : depth, items = n * lw * 2;
        const int qd = 32 / lw, rd = 32 - qd * lw;
        const int half = tid & 1, j_0 = (tid >> 1) / lw, l_0 = (tid >> 1) - j_0 * lw;
        for (int g = 0; g < G; ++g) {
            const int inst = inst0 + g;
            if (inst >= a.count) break;
            int j = j_0, l = l_0;
            for (int e = tid; e < items; e += 64, j += qd, l += rd) {
                if (l >= lw) { l -= lw; ++j; }
                const int node = ((W + j) >> l) ^ 1;
                uint4 v = make_uint4(0, 0, 0, 0);
                if (l == 0) {
                    if (node - W < n)
                        v = *reinterpret_cast<const uint4 *>(a.leaves + (size_t)inst * a.leaves_inst_pitch +
                                                             32u * (node - W) + 16u * half);
                } else {
                    const uint32_t *nd = nodes + ((size_t)g * W + node) * 8 + 4 * half;
                    v = make_uint4(bswap32(nd[0]), bswap32(nd[1]), bswap32(nd[2]), bswap32(nd[3]));
                }
                *reinterpret_cast<uint4 *>(a.branches + (size_t)inst * a.br_inst_pitch +
                                           ((size_t)j * depth + l) * 32u + 16u * half) = v;
            }
        }
    }
}

// ============================================================================
// merkle_top: the top five layers (16, 8, 4, 2, 1 nodes) of W = 256 trees
// that merkle_kernel<false> stopped at the layer of 32 nodes, T trees per
// one-wave block.  Beside two trees in a wave those layers fill 32, 16, .. 2
// lanes of five passes; here T = 8 trees' layer fills 128, 64, .. 8 lanes of
// six passes for four times the trees.  Writes the roots and the branch
// levels 4..7 (the second 128-B line of each leaf's branch record), after
// reading the 32-node layer merkle_kernel left in those slots.
// ============================================================================
__global__ __launch_bounds__(64) void merkle_top_kernel(MerkleArgs a) {
    set_wave_prio(a.prio);
    constexpr int T = 8, M0 = 32, W = 256;
    __shared__ uint32_t nodes[T][2 * M0][8];  // heap index 1 .. 63 of each tree
    const int tid = threadIdx.x, inst0 = (int)blockIdx.x * T, d = a.depth;
    for (int e = tid; e < T * M0; e += 64) {
        const int g = e >> 5, q = e & 31, inst = inst0 + g;
        if (inst >= a.count) continue;
        const uint4 *src = reinterpret_cast<const uint4 *>(a.branches + (size_t)inst * a.br_inst_pitch +
                                                           ((size_t)(q >> 2) * d + 4 + (q & 3)) * 32u);
        const uint4 v0 = src[0], v1 = src[1];
        uint32_t *nd = nodes[g][M0 + q];
        nd[0] = v0.x; nd[1] = v0.y; nd[2] = v0.z; nd[3] = v0.w;
        nd[4] = v1.x; nd[5] = v1.y; nd[6] = v1.z; nd[7] = v1.w;
    }
    __syncthreads();
    for (int m = M0 / 2, lgm = 4; m >= 1; m >>= 1, --lgm) {
        for (int t = tid; t < T * m; t += 64) {
            const int g = t >> lgm, i = m + (t & (m - 1));
            if (inst0 + g >= a.count) continue;
            uint32_t o[8];
            sha256_node64(nodes[g][2 * i], nodes[g][2 * i + 1], o);
#pragma unroll
            for (int q = 0; q < 8; ++q) nodes[g][i][q] = o[q];
        }
        __syncthreads();
    }
    for (int g = tid; g < T; g += 64)
        if (inst0 + g < a.count) store_digest(a.roots + (size_t)(inst0 + g) * 32u, nodes[g][1]);
    // branch[j][l] = node ((W + j) >> l) ^ 1 for l = 4..7: item e = (j, l - 4, half)
    const int items = a.n * 4 * 2;
    for (int g = 0; g < T; ++g) {
        const int inst = inst0 + g;
        if (inst >= a.count) break;
        for (int e = tid; e < items; e += 64) {
            const int half = e & 1, j = e >> 3, l = 4 + ((e >> 1) & 3);
            const uint32_t *nd = nodes[g][((W + j) >> l) ^ 1] + 4 * half;
            *reinterpret_cast<uint4 *>(a.branches + (size_t)inst * a.br_inst_pitch + ((size_t)j * d + l) * 32u +
                                       16u * half) =
                make_uint4(bswap32(nd[0]), bswap32(nd[1]), bswap32(nd[2]), bswap32(nd[3]));
        }
    }
}

// ============================================================================
// merkle_recheck: interpolate's root recheck inside rbc_dev_receive_step,
// over the nodes ECHO verify already established (interpolate,
// rbc/rbc.go:86-90; validateMessage, rbc/rbc.go:92-95).
// Every valid ECHO leaf j was verified against the committed root R, so its
// leaf hash and every sibling in its branch are nodes of the committed tree C
// (collision resistance).  The re-encoding E equals C at every valid leaf the
// decode left unchanged (used rows are never rewritten; a valid unused row
// the re-encoding differs from is flagged).  Hence E's root equals R iff
// E(v) == C(v) at the root v of every MAXIMAL subtree that holds no valid
// leaf, and C(v) is the level-l entry of the branch of any valid leaf under
// v's sibling.  So only the nodes inside those subtrees are hashed (C4:
// ~15 of 255 per instance, C2 ~25 of 127) plus one 32-byte compare per
// subtree, instead of the whole tree; and R (copied when the branches were
// verified) must equal expect_roots[i] now.  An instance with a flagged row
// is left to the full recheck (need_full -> merkle_kernel<true>, `only`).
// The status equals the full recheck's on every input, up to SHA-256
// collisions (tests/test_gpu_parity.py: node-reuse vs full recheck).
// One-wave blocks of G instances: the node hashes of one level of all G
// instances are packed onto consecutive lanes (like merkle_kernel); LDS
// holds E of the hashed nodes ([G][W][8] words, heap index 1..W-1) and a
// has-valid byte per heap node ([G][2W], leaves at W..2W-1).
// ============================================================================
__global__ __launch_bounds__(64) void merkle_recheck_kernel(RecheckArgs a) {
    set_wave_prio(a.prio);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int G = a.inst_per_block, W = a.width, lgW = a.depth, n = a.n;
    uint32_t *E = reinterpret_cast<uint32_t *>(smem);
    uint8_t *hv = smem + (size_t)G * W * 32;
    uint16_t *task = reinterpret_cast<uint16_t *>(hv + (size_t)G * 2 * W);  // G * W / 2 entries at most
    __shared__ uint32_t s_state[64];  // per instance: bit 0 live, bit 1 a compare failed, bit 2 flagged row
    const int lane = threadIdx.x;
    const int inst0 = (int)blockIdx.x * G;
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int g = lane; g < G; g += 64) {
        const int inst = inst0 + g;
        s_state[g] = (inst < a.count && a.status[inst] == 0) ? 1u : 0u;
    }
    __syncthreads();
    // 1. leaves: has-valid = valid; a flagged (changed) valid row sends the instance to the full recheck
    for (int t = lane; t < G * W; t += 64) {
        const int g = t >> lgW, j = t & (W - 1), inst = inst0 + g;
        uint8_t v = 0;
        if ((s_state[g] & 1u) && j < n) {
            v = a.valid[(size_t)inst * n + j] != 0;
            if (v && a.flags[(size_t)inst * n + j]) atomicOr(&s_state[g], 4u);
        }
        hv[g * 2 * W + W + j] = v;
    }
    __syncthreads();
    // 2. has-valid up the tree (heap order: node i's children are 2i, 2i+1)
    for (int l = 1; l <= lgW; ++l) {
        const int m = W >> l;
        for (int t = lane; t < G * m; t += 64) {
            const int g = t >> (lgW - l), i = m + (t & (m - 1));
            uint8_t *h = hv + g * 2 * W;
            h[i] = h[2 * i] | h[2 * i + 1];
        }
        __syncthreads();
    }
    auto active = [&](int g) { return (s_state[g] & 5u) == 1u; };  // live, no flagged row
    // 3. E of every node that holds no valid leaf, level by level, the
    //    level's nodes of all G instances on consecutive lanes
    for (int l = 1; l < lgW; ++l) {
        const int m = W >> l;
        int total = 0;
        for (int t0 = 0; t0 < G * m; t0 += 64) {  // wave-uniform trip count
            const int t = t0 + lane;
            const int g = t >> (lgW - l), i = m + (t & (m - 1));
            const bool need = t < G * m && active(g) && !hv[g * 2 * W + i];
            const uint64_t bm = __ballot(need);
            if (need) task[total + __popcll(bm & below)] = (uint16_t)(g * 2 * W + i);
            total += __popcll(bm);
        }
        __syncthreads();
        if (total == 0) continue;  // wave-uniform: no hashing at this level
        for (int q = lane; q < total; q += 64) {
            const int gi = task[q], g = gi / (2 * W), i = gi - g * 2 * W;
            uint32_t o[8];
            if (l == 1) {  // children are leaves 2i - W, 2i + 1 - W (empty past n)
                const int jl = 2 * i - W, jr = jl + 1;
                const uint8_t *lv = a.leaves + (size_t)(inst0 + g) * a.leaves_inst_pitch;
                if (jl >= n) {
                    sha256_empty(o);
                } else {
                    uint32_t L[8];
                    load_digest(lv + 32u * jl, L);
                    if (jr < n) {
                        uint32_t R[8];
                        load_digest(lv + 32u * jr, R);
                        sha256_node64(L, R, o);
                    } else {
                        sha256_node32(L, o);
                    }
                }
            } else {
                uint32_t L[8], R[8];
                const uint32_t *nl = E + ((size_t)g * W + 2 * i) * 8, *nr = E + ((size_t)g * W + 2 * i + 1) * 8;
#pragma unroll
                for (int q2 = 0; q2 < 8; ++q2) { L[q2] = nl[q2]; R[q2] = nr[q2]; }
                sha256_node64(L, R, o);
            }
            uint32_t *dst = E + ((size_t)g * W + i) * 8;
#pragma unroll
            for (int q2 = 0; q2 < 8; ++q2) dst[q2] = o[q2];
        }
        __syncthreads();
    }
    // 4. compare the root v of every maximal valid-free subtree (level l < d)
    //    with the level-l branch entry of the first valid leaf under its
    //    sibling.  Only an empty LEAF (l == 0, j >= n) is skipped: the walk
    //    itself makes that sibling empty.  A padding node at l >= 1 is taken
    //    from the proposer's branch by the walk, so a Byzantine commitment can
    //    put any value there; it is compared like every other node (E holds
    //    the standard padding hash, step 3), as the full recheck would.
    for (int l = 0; l < lgW; ++l) {
        const int m = W >> l;
        for (int t = lane; t < G * m; t += 64) {
            const int g = t >> (lgW - l), i = m + (t & (m - 1));
            const uint8_t *h = hv + g * 2 * W;
            if (!active(g) || h[i] || !h[i >> 1] || (l == 0 && (i - m) >= n)) continue;
            int s = i ^ 1;
            while (s < W) s = h[2 * s] ? 2 * s : 2 * s + 1;  // first valid leaf under the sibling
            const int inst = inst0 + g, j = s - W;
            const uint4 *br = reinterpret_cast<const uint4 *>(a.branches + (size_t)inst * a.br_inst_pitch +
                                                              ((size_t)j * lgW + l) * 32u);
            const uint4 c0 = br[0], c1 = br[1];
            uint4 e0, e1;
            if (l == 0) {  // E = the regenerated row's leaf hash, raw bytes
                const uint4 *lf = reinterpret_cast<const uint4 *>(a.leaves + (size_t)inst * a.leaves_inst_pitch +
                                                                  32u * (i - W));
                e0 = lf[0];
                e1 = lf[1];
            } else {  // LDS holds the digest words; the branch holds their bytes
                const uint32_t *e = E + ((size_t)g * W + i) * 8;
                e0 = make_uint4(bswap32(e[0]), bswap32(e[1]), bswap32(e[2]), bswap32(e[3]));
                e1 = make_uint4(bswap32(e[4]), bswap32(e[5]), bswap32(e[6]), bswap32(e[7]));
            }
            const bool same = e0.x == c0.x && e0.y == c0.y && e0.z == c0.z && e0.w == c0.w && e1.x == c1.x &&
                              e1.y == c1.y && e1.z == c1.z && e1.w == c1.w;
            if (!same) atomicOr(&s_state[g], 2u);
        }
    }
    __syncthreads();
    // 5. status, or the hand-off to the full recheck
    for (int g = lane; g < G; g += 64) {
        const int inst = inst0 + g;
        if (inst >= a.count) continue;
        const uint32_t st = s_state[g];
        a.need_full[inst] = (st & 5u) == 5u ? 1 : 0;
        if ((st & 5u) != 1u) continue;
        const uint4 *x = reinterpret_cast<const uint4 *>(a.vroots + (size_t)inst * 32u);
        const uint4 *y = reinterpret_cast<const uint4 *>(a.expect_roots + (size_t)inst * 32u);
        const uint4 x0 = x[0], x1 = x[1], y0 = y[0], y1 = y[1];
        const bool root_same = x0.x == y0.x && x0.y == y0.y && x0.z == y0.z && x0.w == y0.w && x1.x == y1.x &&
                               x1.y == y1.y && x1.z == y1.z && x1.w == y1.w;
        a.status[inst] = (!(st & 2u) && root_same) ? 0 : RBC_ERR_ROOT_MISMATCH;
    }
}

// ============================================================================
// merkle_path: batched branch verification with shared paths (ECHO side of
// validateMessage, rbc/rbc.go:92-95, for all N shards of an instance).
// Leaf j's walk is h <- H(order_l(h, branch_j[l])) for l = 0..d-1 and it is
// valid iff the end equals the root.  Walks of leaves under one level-(l+1)
// node hash the SAME 64-byte input whenever their inputs agree -- the honest
// case -- so each level hashes every distinct input once: the group's first
// participating leaf (rep) owns one hash task, and any leaf whose input
// differs from the rep's owns one more (its own walk).  Each leaf then takes
// the digest of the task whose input equals its own, which is exactly the
// value its own walk would compute: the result is bit-identical to the
// per-leaf walk for every input, honest or not.  Per instance that is W-1
// node hashes plus one per divergent (leaf, level) instead of N*d.
// One wave per block: lane owns leaves s*64 + lane (s < W/64), or 64/W
// instances share the wave when W < 64; the hash tasks of a level are packed
// onto consecutive lanes.
// Leaves come from sha_rows_kernel<false>; this kernel writes valid[].
// ============================================================================
template <int L>
__global__ __launch_bounds__(64) void merkle_path_kernel(PathArgs a) {
    set_wave_prio(a.prio);
    // one wave per block; lane owns leaf positions p = s*64 + lane (s < L)
    __shared__ uint32_t s_pair[64 * L][17];  // +1 word: conflict-free rows; an owner's task
                                              // digest overwrites words 0..7 of its own row
    __shared__ uint8_t s_empty[64 * L];
    __shared__ uint16_t s_owner[64 * L];
    const int lane = threadIdx.x;
    const int W = a.width, lgW = a.lg_width;
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int jj[L], inst_s[L];
    bool ok_s[L], part[L];
    uint64_t pm[L];
    uint32_t x[L][8];
#pragma unroll
    for (int s = 0; s < L; ++s) {
        const int p = s * 64 + lane;
        const int g = p >> lgW;
        jj[s] = p & (W - 1);
        inst_s[s] = (int)blockIdx.x * a.inst_per_block + g;
        ok_s[s] = g < a.inst_per_block && inst_s[s] < a.count && !(a.status && a.status[inst_s[s]] != 0);
        part[s] = ok_s[s] && jj[s] < a.n && (!a.present || a.present[(size_t)inst_s[s] * a.n + jj[s]] != 0);
        pm[s] = __ballot(part[s]);
        if (part[s]) load_digest(a.leaves + (size_t)inst_s[s] * a.leaves_inst_pitch + 32u * jj[s], x[s]);
    }
    // participation masks by leaf word, read at a runtime word index: from
    // LDS (a select chain over pm[] became a scratch array in the 4-level form)
    __shared__ uint64_t s_pm[L];
    if (lane == 0) {
#pragma unroll
        for (int s = 0; s < L; ++s) s_pm[s] = pm[s];
    }
    __syncthreads();
    auto pmask = [&](int w) -> uint64_t { return s_pm[w]; };
    // At W = 256 (C4, d = 8) a leaf's branch levels 4q..4q+3 are one 128-B
    // line.  They are staged in LDS four levels at a time, every line of the
    // instance's participating leaves read once, whole, by 8 consecutive lanes
    // with 8 loads per lane in flight: the levels of a block are far apart in
    // time and the lines of the blocks in flight on an XCD outgrow its L2, so
    // loading one 32-B sibling per level read 1.34-2.74 GB per launch against
    // 0.80 GB of branches (round 3 and tools/gpu_runs/gpu_r04c.sh).  The
    // 32 KiB stage also holds the kernel at 3 blocks per CU, a residency that
    // measured fastest (gpu_r04c.sh).  Measured at C4 (GB/s): this form
    // 355.6 (gpu_r04j.sh); per-level loads at 3 / 4 / 8 blocks per CU 355-356,
    // 355-361, 355 (gpu_r04i.sh, gpu_r04j.sh); the stage waiting on every load
    // 336 (gpu_r04f.sh); the levels in VGPRs (332 per lane) 320 (gpu_r04d.sh);
    // two instances per wave 263 (gpu_r04g.sh).
    constexpr int QL = L == 4 ? 4 : 1;  // levels per stage (W = 256 only)
    constexpr int PPL = 2 * QL;  // 16-B pieces per leaf and stage
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint4 *s_stage = reinterpret_cast<uint4 *>(smem);  // [64 * L][PPL] x 16 B when QL > 1
    // the block's branches (the launcher keeps inst_per_block * pitch < 4 GiB)
    const rsrc_t rb = make_rsrc(a.branches + (size_t)blockIdx.x * a.inst_per_block * a.br_inst_pitch,
                                (uint32_t)((uint64_t)a.inst_per_block * a.br_inst_pitch));
    // ---- Speculative top levels (W = 256).  Levels 0 and 1 run exactly as
    // above (128 + 64 tasks fill the lanes); levels 2..7 would take one pass
    // each for 32, 16, .. 1 tasks.  Instead every node above level 2 is hashed
    // at once from the values the branches CLAIM for its children: claim(v)
    // at level l is the level-l branch entry of the first participating leaf
    // under v's sibling.  The instance is proven -- every participating leaf
    // valid -- when (i) all participating leaves under each level-l node v
    // (l >= 2) hold the same level-l entry, (ii) all of them reached the same
    // exact level-2 value X(v), equal to claim(v) where that exists, and (iii)
    // each node's hash equals its claim (the root at the top).  Then, by
    // induction over the levels, each leaf's own walk computes exactly these
    // hashes and ends at the root.  A child with no claim (no participant
    // under its sibling) takes its own task's hash instead: a later pass.
    // Anything else re-runs levels 2..7 exactly (the per-level form above),
    // so valid[] is bit-identical to the per-leaf walk for every input.
    constexpr bool SPEC = L == 4;
    constexpr int L0 = 2;                 // first speculative level
    int lo = 0, hi = SPEC ? L0 : a.depth;  // exact levels of this pass: [lo, hi)
    bool spec = SPEC, proven = false, sfail = false;
    // spec scratch in s_pair (no exact level runs meanwhile), in words:
    // claims [126][8] (raw bytes; level l at node v: row 128 - (256 >> (l-1)) + v),
    // X2 [64][8] at 1008, task hashes [63][8] at 1520, task done flags [63] at 2024
    uint32_t *s_raw = &s_pair[0][0];
    auto claim_row = [](int l, int v) { return 128 - (256 >> (l - 1)) + v; };
    auto task_of = [](int m, int v) { return 64 - (256 >> (m - 1)) + v; };  // node v at level m >= 3
    auto sub_mask = [&](int l, int v) -> uint64_t {  // participants under node (l, v), l <= 6
        const int p0 = v << l;
        const uint64_t m = pmask(p0 >> 6);
        return l >= 6 ? m : (m >> (p0 & 63)) & ((1ull << (1 << l)) - 1ull);
    };
    auto has = [&](int l, int v) -> bool {
        if (l <= 6) return sub_mask(l, v) != 0;
        uint64_t m = 0;
        for (int w = (v << l) >> 6; w < ((v + 1) << l) >> 6; ++w) m |= pmask(w);
        return m != 0;
    };
    auto rep_of = [&](int l, int v, int self) -> int {  // first participant under (l, v)
        if (l <= 6) return (v << l) + __builtin_ctzll(sub_mask(l, v));
        for (int w = (v << l) >> 6; w < ((v + 1) << l) >> 6; ++w) {
            const uint64_t m = pmask(w);
            if (m) return w * 64 + __builtin_ctzll(m);
        }
        return self;
    };
    auto eq8 = [](const uint4 &a0, const uint4 &a1, const uint4 &b0, const uint4 &b1) {
        return a0.x == b0.x && a0.y == b0.y && a0.z == b0.z && a0.w == b0.w && a1.x == b1.x && a1.y == b1.y &&
               a1.z == b1.z && a1.w == b1.w;
    };
    // the staged levels lq..lq+3: check (i) and publish the claims
    auto spec_collect = [&](int lq) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int l = lq + t;
            if (l < L0) continue;
#pragma unroll
            for (int s = 0; s < L; ++s) {
                if (!part[s]) continue;
                const int p = s * 64 + lane, v = p >> l, r = rep_of(l, v, p);
                const uint4 m0 = s_stage[p * PPL + 2 * t], m1 = s_stage[p * PPL + 2 * t + 1];
                if (r == p) {
                    uint4 *c = reinterpret_cast<uint4 *>(s_raw + 8 * claim_row(l, v ^ 1));
                    c[0] = m0;
                    c[1] = m1;
                } else {
                    sfail |= !eq8(m0, m1, s_stage[r * PPL + 2 * t], s_stage[r * PPL + 2 * t + 1]);
                }
            }
        }
        if (lq == 0) {  // each level-2 node's first participant publishes its exact value
#pragma unroll
            for (int s = 0; s < L; ++s) {
                const int p = s * 64 + lane;
                if (part[s] && rep_of(L0, p >> L0, p) == p)
#pragma unroll
                    for (int q = 0; q < 8; ++q) s_raw[1008 + 8 * (p >> L0) + q] = x[s][q];
            }
        }
    };
    auto claim_words = [&](int l, int v, uint32_t (&o)[8]) {
        load_digest(reinterpret_cast<const uint8_t *>(s_raw + 8 * claim_row(l, v)), o);
    };
    // checks (ii) and (iii), the node hashes of levels 3..8; true = not proven
    auto spec_finish = [&]() -> bool {
        uint32_t *s_done = s_raw + 2024;
        if (lane < 63) s_done[lane] = 0;
        __syncthreads();
#pragma unroll
        for (int s = 0; s < L; ++s) {
            if (!part[s]) continue;
            const uint32_t *X = s_raw + 1008 + 8 * ((s * 64 + lane) >> L0);
#pragma unroll
            for (int q = 0; q < 8; ++q) sfail |= x[s][q] != X[q];
        }
        // lane t: node P at level m (3..8), children 2P, 2P + 1 at level l
        const int t = lane;
        const int m = t < 32 ? 3 : t < 48 ? 4 : t < 56 ? 5 : t < 60 ? 6 : t < 62 ? 7 : 8;
        const int P = t - task_of(m, 0), l = m - 1;
        const bool h0 = t < 63 && has(l, 2 * P), h1 = t < 63 && has(l, 2 * P + 1);
        const bool active = h0 || h1;
        uint32_t in[2][8];
        int dep[2] = {-1, -1};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int c = 2 * P + k;
            const bool hc = k ? h1 : h0, hs = k ? h0 : h1;
#pragma unroll
            for (int q = 0; q < 8; ++q) in[k][q] = 0;
            if (!active) continue;
            if (l == L0 && hc) {
#pragma unroll
                for (int q = 0; q < 8; ++q) in[k][q] = s_raw[1008 + 8 * c + q];
                if (hs) {
                    uint32_t cl[8];
                    claim_words(l, c, cl);
#pragma unroll
                    for (int q = 0; q < 8; ++q) sfail |= cl[q] != in[k][q];
                }
            } else if (hs) {
                claim_words(l, c, in[k]);
            } else {
                dep[k] = task_of(l, c);
            }
        }
        bool done = false;
        uint32_t h[8];
        for (int it = 0; it < 8 - L0; ++it) {
            const bool ready = active && !done && dep[0] < 0 && dep[1] < 0;
            if (__ballot(ready) == 0) break;
            if (ready) {
                sha256_node64(in[0], in[1], h);
#pragma unroll
                for (int q = 0; q < 8; ++q) s_raw[1520 + 8 * t + q] = h[q];
                s_done[t] = 1;
                done = true;
            }
            __syncthreads();
            if (active && !done) {
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    if (dep[k] >= 0 && s_done[dep[k]]) {
#pragma unroll
                        for (int q = 0; q < 8; ++q) in[k][q] = s_raw[1520 + 8 * dep[k] + q];
                        dep[k] = -1;
                    }
                }
            }
            __syncthreads();
        }
        if (active && !done) sfail = true;
        if (done && (m == 8 || has(m, P ^ 1))) {
            uint32_t ref[8];
            if (m == 8) load_digest(a.roots + (size_t)inst_s[0] * 32u, ref);
            else claim_words(m, P, ref);
#pragma unroll
            for (int q = 0; q < 8; ++q) sfail |= h[q] != ref[q];
        }
        return __ballot(sfail) != 0;
    };
    for (int lq = 0; lq < a.depth; lq += QL) {
        if constexpr (QL > 1) {
            const int nl = min(QL, a.depth - lq);  // levels in this stage
            __syncthreads();                         // the previous stage's reads are done
            // batches of SB pieces per lane: every load of a batch in flight
            // before the first LDS write (one wait per batch, not per piece)
            constexpr int SB = 8;  // 16 measured the same (gpu_r04j.sh)
#pragma unroll 1
            for (int c0 = 0; c0 < L * PPL; c0 += SB) {
                uint4 v[SB];
#pragma unroll
                for (int u = 0; u < SB; ++u) {  // no branch: an idle piece reads past the buffer (0)
                    const int c = (c0 + u) * 64 + lane;
                    const int p = c / PPL, piece = c % PPL;
                    const bool on = piece < 2 * nl && ((pmask(p >> 6) >> (p & 63)) & 1ull);
                    const uint32_t off = (uint32_t)(p >> lgW) * (uint32_t)a.br_inst_pitch +
                                         ((uint32_t)(p & (W - 1)) * a.depth + lq) * 32u + 16u * piece;
                    v[u] = bload16(rb, on ? off : 0xfffffff0u);
                }
#pragma unroll
                for (int u = 0; u < SB; ++u) s_stage[(c0 + u) * 64 + lane] = v[u];
            }
            __syncthreads();
        }
    // one level of the stage (t a compile-time index)
    auto level = [&](auto tc) {
        constexpr int t = decltype(tc)::value;
        const int l = lq + t;
        if (l >= lo && l < hi) {  // wave-uniform
        // 1. each leaf's ordered input (left || right) for level l
#pragma unroll
        for (int s = 0; s < L; ++s) {
            if (!part[s]) continue;
            const int p = s * 64 + lane, j = jj[s];
            const bool empty = (l == 0) && ((j ^ 1) >= a.n);
            uint32_t sib[8];
            if (empty) {
#pragma unroll
                for (int q = 0; q < 8; ++q) sib[q] = 0u;
            } else if constexpr (QL > 1) {
                load_digest(reinterpret_cast<const uint8_t *>(s_stage + p * PPL + 2 * t), sib);
            } else {
                load_digest(a.branches + (size_t)inst_s[s] * a.br_inst_pitch + ((size_t)j * a.depth + l) * 32u, sib);
            }
            const bool right = (j >> l) & 1;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                s_pair[p][q] = right ? sib[q] : x[s][q];
                s_pair[p][8 + q] = right ? x[s][q] : sib[q];
            }
            s_empty[p] = empty ? 1 : 0;
        }
        __syncthreads();
        // 2. rep = first participating leaf of the level-(l+1) group; owners
        //    are reps and leaves whose input differs from their rep's
        int rep[L];
        bool owner[L];
        int total = 0, base[L];
        uint64_t om[L];
#pragma unroll
        for (int s = 0; s < L; ++s) {
            const int p = s * 64 + lane;
            rep[s] = p;
            owner[s] = false;
            if (part[s]) {
                const int gs = 2 << l;
                const int t0 = p & ~(gs - 1), t1 = t0 + gs;
                for (int w = t0 >> 6; w <= (t1 - 1) >> 6; ++w) {
                    uint64_t m = pmask(w);
                    const int lo = t0 - w * 64, hi = t1 - w * 64;
                    if (lo > 0) m &= ~0ull << lo;
                    if (hi < 64) m &= (1ull << hi) - 1ull;
                    if (m) { rep[s] = w * 64 + __builtin_ctzll(m); break; }
                }
                bool same = true;
                if (rep[s] != p) {
                    same = s_empty[p] == s_empty[rep[s]];
#pragma unroll
                    for (int q = 0; q < 16; ++q) same = same && (s_pair[p][q] == s_pair[rep[s]][q]);
                }
                owner[s] = (rep[s] == p) || !same;
            }
            om[s] = __ballot(owner[s]);
            base[s] = total;
            total += __popcll(om[s]);
        }
        // 3. number the hash tasks (owners) on consecutive lanes
#pragma unroll
        for (int s = 0; s < L; ++s)
            if (owner[s]) s_owner[base[s] + __popcll(om[s] & below)] = (uint16_t)(s * 64 + lane);
        __syncthreads();
        // 4. hash the tasks: one compression body for both node forms --
        //    H(L || R) = two blocks, the second constant; H(L) (empty level-0
        //    sibling) = one block [L | 0x80 .. | 256 bits]
        for (int i = lane; i < total; i += 64) {
            const int o = s_owner[i];
            const bool empty = s_empty[o] != 0;
            Sha256State st;
            sha256_init(st);
            uint32_t w[16];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                w[q] = s_pair[o][q];
                w[8 + q] = s_pair[o][8 + q];
            }
            if (empty) {
                w[8] = 0x80000000u;
                w[15] = 256u;
            }
            sha256_compress(st, w);
            if (!empty) {
#pragma unroll
                for (int q = 0; q < 16; ++q) w[q] = 0;
                w[0] = 0x80000000u;
                w[15] = 512u;
                sha256_compress(st, w);
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) s_pair[o][q] = st.h[q];
        }
        __syncthreads();
        // 5. every walk takes the digest of the task with its input (the
        //    rep's task unless it owns one)
#pragma unroll
        for (int s = 0; s < L; ++s) {
            if (!part[s]) continue;
            const int o = owner[s] ? s * 64 + lane : rep[s];
#pragma unroll
            for (int q = 0; q < 8; ++q) x[s][q] = s_pair[o][q];
        }
        __syncthreads();
        }
    };
    level(IntC<0>{});
    if constexpr (QL >= 2) level(IntC<1>{});
    if constexpr (QL == 4) {
        level(IntC<2>{});
        level(IntC<3>{});
    }
    if constexpr (SPEC) {
        if (spec) {  // wave-uniform
            spec_collect(lq);
            if (lq + QL >= a.depth) {
                spec = false;
                if (!spec_finish()) {
                    proven = true;
                    break;
                }
                lo = L0;  // not proven: levels 2..7 exactly, restaged from level 0
                hi = a.depth;
                lq = -QL;
            }
        }
    }
    }
#pragma unroll
    for (int s = 0; s < L; ++s) {
        if (!(ok_s[s] && jj[s] < a.n)) continue;
        bool ok = part[s] && proven;
        if (part[s] && !proven) {
            uint32_t root[8];
            load_digest(a.roots + (size_t)inst_s[s] * 32u, root);
            ok = true;
#pragma unroll
            for (int q = 0; q < 8; ++q) ok = ok && (x[s][q] == root[q]);
        }
        a.valid[(size_t)inst_s[s] * a.n + jj[s]] = ok ? 1 : 0;
    }
}

// ============================================================================
// digest: batch digest = SHA-256(leaf_0 || .. || leaf_{k-1}) of every
// instance that passed the root recheck, one lane per instance.  The message
// is the first 32k bytes of the instance's leaves; the last partial block is
// assembled from 16-byte reads inside that range only (no over-read).
// ============================================================================
__global__ __launch_bounds__(64) void digest_kernel(const uint8_t *leaves, uint64_t leaves_inst_pitch, int k,
                                                    const int32_t *status, uint8_t *digests, int count, int prio) {
    set_wave_prio(prio);
    const int inst = blockIdx.x * blockDim.x + threadIdx.x;
    if (inst >= count) return;
    if (status && status[inst] != 0) return;
    const uint8_t *msg = leaves + (size_t)inst * leaves_inst_pitch;
    const uint32_t len = 32u * (uint32_t)k;
    Sha256State s;
    sha256_init(s);
    uint32_t w[16];
    const uint32_t nfull = len >> 6;
    uint4 q[4];
    if (nfull) load_block_raw(msg, q);
    for (uint32_t b = 0; b < nfull; ++b) {
        bswap_block(q, w);
        if (b + 1 < nfull) load_block_raw(msg + 64u * (b + 1), q);
        sha256_compress(s, w);
    }
    // len % 64 is 0 or 32: tail = [32 bytes of leaf k-1 | 0x80 ...] or [0x80 ...]
    const uint32_t rem = len & 63u;
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = 0;
    if (rem) {
        const uint4 *v = reinterpret_cast<const uint4 *>(msg + 64u * nfull);
        const uint4 x0 = v[0], x1 = v[1];
        w[0] = bswap32(x0.x); w[1] = bswap32(x0.y); w[2] = bswap32(x0.z); w[3] = bswap32(x0.w);
        w[4] = bswap32(x1.x); w[5] = bswap32(x1.y); w[6] = bswap32(x1.z); w[7] = bswap32(x1.w);
        w[8] = 0x80000000u;
    } else {
        w[0] = 0x80000000u;
    }
    const uint64_t bits = (uint64_t)len * 8u;
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
    sha256_compress(s, w);
    uint32_t d[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) d[t] = s.h[t];
    store_digest(digests + (size_t)inst * 32u, d);
}

// ============================================================================
// decode_prepare: per instance, pick the first k valid shards by index
// (klauspost Reconstruct rule), invert the k x k sub-matrix of the encode
// matrix by Gauss-Jordan in LDS, and form D = M[regen] * inv so one GF pass
// regenerates every non-used position (data and parity) of the re-encoding.
// ============================================================================
__global__ __launch_bounds__(256) void decode_prepare_kernel(PrepArgs a) {
    set_wave_prio(a.prio);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int n = a.n, k = a.k;
    uint8_t *s_exp = smem;             // 512
    uint8_t *s_log = smem + 512;       // 256
    uint8_t *s_used = smem + 768;      // 256
    uint8_t *s_regen = smem + 1024;    // 256
    int *s_misc = reinterpret_cast<int *>(smem + 1536);  // 4 ints
    uint8_t *A = smem + 1552;          // 512: log w_u, log l(x_r)
    const int inst = blockIdx.x, tid = threadIdx.x;

    if (tid == 0) {
        s_log[0] = 0;
        int x = 1;
        for (int i = 0; i < 255; ++i) {
            s_exp[i] = (uint8_t)x;
            s_exp[i + 255] = (uint8_t)x;
            s_log[x] = (uint8_t)i;
            x <<= 1;
            if (x & 0x100) x ^= 0x11d;
        }
        s_exp[510] = s_exp[0];
        s_exp[511] = s_exp[1];
        // used = first k valid by index (klauspost rule); regen = the missing
        // positions first, then the valid-but-unused ones
        int nu = 0, nm = 0;
        const uint8_t *v = a.valid + (size_t)inst * a.valid_stride;
        for (int j = 0; j < n; ++j) {
            if (v[j] && nu < k) s_used[nu++] = (uint8_t)j;
            else if (!v[j]) s_regen[nm++] = (uint8_t)j;
        }
        int nr = nm;
        for (int j = 0, seen = 0; j < n; ++j)
            if (v[j] && seen++ >= k) s_regen[nr++] = (uint8_t)j;
        s_misc[0] = nu;
        s_misc[1] = nr;
        s_misc[2] = (a.counter && nu >= k) ? (int)atomicAdd(a.counter, (unsigned)nm) : 0;
        if (a.nmiss) a.nmiss[inst] = nm;
        s_misc[3] = nm;
    }
    __syncthreads();
    const int nu = s_misc[0], nr = s_misc[1];
    if (nu < k) {
        if (tid == 0) a.status[inst] = RBC_ERR_TOO_FEW_SHARDS;
        return;
    }
    if (a.counter) {
        const int base = s_misc[2], nm = s_misc[3];
        for (int t = tid; t < nm; t += 256) a.list[base + t] = ((uint32_t)inst << 8) | s_regen[t];
        for (int t = tid; t < n; t += 256) a.flags[(size_t)inst * n + t] = 0;
    }
    for (int t = tid; t < k; t += 256) a.used[(size_t)inst * a.used_stride + t] = s_used[t];
    for (int t = tid; t < nr; t += 256) a.regen[(size_t)inst * a.regen_stride + t] = s_regen[t];
    // D[r][u] = L_u(x_r): the Lagrange basis of U at every regenerated
    // position (data or parity).  klauspost's matrix is an evaluation code, so
    // this equals M[regen] * inv(M[U]) exactly -- no k x k
    // inversion.  Logs mod 255; x_a ^ x_b != 0 for distinct positions.
    uint8_t *s_lw = A;          // k: log w_u
    uint8_t *s_ll = A + 256;    // nr: log l(x_r)
    for (int u = tid; u < k; u += 256) {
        const uint32_t xu = s_used[u];
        uint32_t acc = 0;
        for (int v = 0; v < k; ++v)
            if (v != u) acc += s_log[xu ^ s_used[v]];
        s_lw[u] = (uint8_t)((255u * 255u - acc) % 255u);
    }
    for (int r = tid; r < nr; r += 256) {
        const uint32_t xr = s_regen[r];
        uint32_t acc = 0;
        for (int v = 0; v < k; ++v) acc += s_log[xr ^ s_used[v]];
        s_ll[r] = (uint8_t)(acc % 255u);
    }
    __syncthreads();
    uint8_t *D = a.dmat + (size_t)inst * a.dmat_stride;
    const int lane = tid & 63, wv = tid >> 6;
    for (int r = wv; r < nr; r += 4) {
        const uint32_t xr = s_regen[r], lr = s_ll[r] + 255u;
        for (int u = lane; u < k; u += 64)
            D[(size_t)r * k + u] = s_exp[(s_lw[u] + lr - s_log[xr ^ s_used[u]]) % 255u];
    }
    if (tid == 0) a.status[inst] = 0;
}

// ============================================================================
// decode_prepare_fft: the FFT codec's interpolate plan.  With U = the first k
// valid positions (klauspost's Reconstruct rule) = every present data row D_p
// plus the first m valid parity rows P_u (m = #missing data rows D_m), the
// missing data rows are x_{D_m} = D s_U with D the m x k Lagrange matrix of
// U at D_m (below; equal to [A^-1 M[P_u][D_p] | A^-1], A = M[P_u][D_m]).
// Parity positions are then re-encoded by rs_fft_kernel from the completed
// data half; cls[pos] tells it what to do per position.
// ============================================================================
__global__ __launch_bounds__(256) void decode_prepare_fft_kernel(PrepArgs a, const uint8_t *exp_tab,
                                                                  const uint8_t *log_tab) {
    set_wave_prio(a.prio);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int n = a.n, k = a.k;
    uint8_t *s_exp = smem;           // 512
    uint8_t *s_log = smem + 512;     // 256
    uint8_t *s_used = smem + 768;    // 256: U in index order
    uint8_t *s_miss = smem + 1024;   // 256: missing positions in index order
    int *s_misc = reinterpret_cast<int *>(smem + 1280);  // 8 ints
    int *s_wcnt = reinterpret_cast<int *>(smem + 1568);  // 12 ints: per-wave counts
    const int inst = blockIdx.x, tid = threadIdx.x;
    for (int t = tid; t < 512; t += 256) s_exp[t] = exp_tab[t];
    s_log[tid] = log_tab[tid];
    // used = the first k valid positions, missing = the invalid ones, both in
    // index order: block-wide ranks from wave ballots (n <= 256 = blockDim)
    {
        const int lane = tid & 63, w = tid >> 6;
        const bool in = tid < n;
        const bool ok = in && a.valid[(size_t)inst * a.valid_stride + tid] != 0;
        const bool miss = in && !ok;
        const uint64_t bo = __ballot(ok), bm = __ballot(miss), bd = __ballot(miss && tid < k);
        const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
        if (lane == 0) {
            s_wcnt[w] = __popcll(bo);
            s_wcnt[4 + w] = __popcll(bm);
            s_wcnt[8 + w] = __popcll(bd);
        }
        __syncthreads();
        int rok = __popcll(bo & below), rmiss = __popcll(bm & below);
        int tok = 0, tmiss = 0, tmd = 0;
        for (int q = 0; q < 4; ++q) {
            if (q < w) {
                rok += s_wcnt[q];
                rmiss += s_wcnt[4 + q];
            }
            tok += s_wcnt[q];
            tmiss += s_wcnt[4 + q];
            tmd += s_wcnt[8 + q];
        }
        const bool used = ok && rok < k;
        if (used) s_used[rok] = (uint8_t)tid;
        if (miss) s_miss[rmiss] = (uint8_t)tid;
        if (in)
            a.cls[(size_t)inst * a.cls_stride + tid] =
                (tid < k || used) ? 0 : (miss ? 1 : (a.counter ? 2 : 1));
        if (tid == 0) {
            const int nu = tok < k ? tok : k;
            s_misc[0] = nu;
            s_misc[1] = tmd;
            s_misc[2] = (a.counter && nu >= k) ? (int)atomicAdd(a.counter, (unsigned)tmiss) : 0;
            s_misc[3] = tmiss;
            if (a.nmiss) a.nmiss[inst] = tmiss;
            a.rcount[inst] = tmd;
        }
    }
    __syncthreads();
    const int nu = s_misc[0], m = s_misc[1];
    if (nu < k) {
        if (tid == 0) a.status[inst] = RBC_ERR_TOO_FEW_SHARDS;
        return;
    }
    if (a.counter) {
        const int base = s_misc[2], nm = s_misc[3];
        for (int t = tid; t < nm; t += 256) a.list[base + t] = ((uint32_t)inst << 8) | s_miss[t];
        for (int t = tid; t < n; t += 256) a.flags[(size_t)inst * n + t] = 0;
    }
    for (int t = tid; t < k; t += 256) a.used[(size_t)inst * a.used_stride + t] = s_used[t];
    for (int t = tid; t < m; t += 256) a.regen[(size_t)inst * a.regen_stride + t] = s_miss[t];
    if (m == 0) {
        if (tid == 0) a.status[inst] = 0;
        return;
    }
    // D[r][u] = L_u(x_r): the Lagrange basis of U evaluated at the missing
    // data position x_r.  klauspost's code is an evaluation code (shard r =
    // P(r), deg P < k, the labels 0..N-1 as field elements), so the map from
    // the k values at U to the missing values is unique and this IS
    // [A^-1 M[P_u][D_p] | A^-1] -- with no inversion, no pivoting and no
    // barrier per pivot.  In logs (mod 255; x_a ^ x_b != 0 for distinct
    // positions, so every operand is nonzero):
    //   log w_u   = -sum_{v in U, v != u} log(x_u ^ x_v)     (barycentric weight)
    //   log l(x_r) =  sum_{v in U}        log(x_r ^ x_v)     (x_r not in U)
    //   D[r][u]   = exp(log w_u + log l(x_r) - log(x_r ^ x_u))
    uint8_t *s_lw = smem + 1616;        // k: log w_u
    uint8_t *s_ll = s_lw + 256;         // m: log l(x_r)
    for (int u = tid; u < k; u += 256) {
        const uint32_t xu = s_used[u];
        uint32_t acc = 0;
        for (int v = 0; v < k; ++v)
            if (v != u) acc += s_log[xu ^ s_used[v]];
        s_lw[u] = (uint8_t)((255u * 255u - acc) % 255u);
    }
    for (int r = tid; r < m; r += 256) {
        const uint32_t xr = s_miss[r];
        uint32_t acc = 0;
        for (int v = 0; v < k; ++v) acc += s_log[xr ^ s_used[v]];
        s_ll[r] = (uint8_t)(acc % 255u);
    }
    __syncthreads();
    uint8_t *D = a.dmat + (size_t)inst * a.dmat_stride;
    const int lane = tid & 63, wv = tid >> 6;
    for (int r = wv; r < m; r += 4) {
        const uint32_t xr = s_miss[r], lr = s_ll[r] + 255u;
        for (int u = lane; u < k; u += 64) {
            const uint32_t e = (s_lw[u] + lr - s_log[xr ^ s_used[u]]) % 255u;
            D[(size_t)r * k + u] = s_exp[e];
        }
    }
    if (tid == 0) a.status[inst] = 0;
}

// ============================================================================
// join: value = data shards 0..k-1 concatenated (k*S bytes, pad kept).  One
// block covers JOIN_U x 256 aligned 16-byte output chunks of ONE instance
// (blockIdx.x = inst * blocks_per_inst + tile, a scalar division); a chunk may
// straddle two rows.  The row index o / S comes from a float reciprocal with a
// +-1 correction (o < 2^32, j < 256: the estimate is never further off), and
// all loads of a thread are issued before its stores.
// ============================================================================
constexpr int JOIN_U = 4;
__global__ __launch_bounds__(256) void join_kernel(JoinArgs a) {
    set_wave_prio(a.prio);
    const int inst = (int)(blockIdx.x / a.blocks_per_inst);
    const uint32_t tile = blockIdx.x - (uint32_t)inst * a.blocks_per_inst;
    if (a.status && a.status[inst] != 0) return;
    const uint32_t S = inst_len(a.lens, a.uniform_len, inst);
    const uint32_t total = S * (uint32_t)a.k;
    uint8_t *vrow = a.values + (size_t)inst * a.value_pitch;
    const uint8_t *rows = a.shards + (size_t)inst * a.inst_pitch;
    const rsrc_t r = make_rsrc(rows, a.inst_bytes);
    uint4 v[JOIN_U];
    if (S >= 16) {
        const float invS = 1.0f / (float)S;
#pragma unroll
        for (int u = 0; u < JOIN_U; ++u) {
            const uint32_t o = ((tile * JOIN_U + u) * 256u + threadIdx.x) * 16u;
            v[u] = make_uint4(0, 0, 0, 0);
            if (o >= total) continue;
            uint32_t j0 = (uint32_t)((float)o * invS);
            int32_t s0 = (int32_t)(o - j0 * S);
            if (s0 < 0) { --j0; s0 += (int32_t)S; }
            if (s0 >= (int32_t)S) { ++j0; s0 -= (int32_t)S; }
            v[u] = bload16(r, j0 * a.row_pitch + (uint32_t)s0);
            const int c0 = (int)min(16u, S - (uint32_t)s0);
            if (c0 < 16) {
                // bytes c0..15 come from the start of row j0+1: read the 16 bytes
                // that END at row j0+1 byte 16-c0, then blend by byte mask
                uint4 w = make_uint4(0, 0, 0, 0);
                if (j0 + 1 < (uint32_t)a.k) w = bload16(r, (j0 + 1) * a.row_pitch - (uint32_t)c0);
                const uint4 m = mask16(make_uint4(~0u, ~0u, ~0u, ~0u), c0);
                v[u].x = (v[u].x & m.x) | (w.x & ~m.x);
                v[u].y = (v[u].y & m.y) | (w.y & ~m.y);
                v[u].z = (v[u].z & m.z) | (w.z & ~m.z);
                v[u].w = (v[u].w & m.w) | (w.w & ~m.w);
            }
            if (o + 16u > total) v[u] = mask16(v[u], (int)(total - o));
        }
    } else {
        // tiny shards: byte path
#pragma unroll
        for (int u = 0; u < JOIN_U; ++u) {
            const uint32_t o = ((tile * JOIN_U + u) * 256u + threadIdx.x) * 16u;
            uint32_t w[4] = {0, 0, 0, 0};
            for (int b = 0; b < 16; ++b) {
                const uint32_t g = o + b;
                if (g >= total) break;
                const uint32_t j = g / S, off = g - j * S;
                const uint32_t byte = rows[(size_t)j * a.row_pitch + off];
                w[b >> 2] |= byte << (8 * (b & 3));
            }
            v[u] = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
#pragma unroll
    for (int u = 0; u < JOIN_U; ++u) {
        const uint32_t o = ((tile * JOIN_U + u) * 256u + threadIdx.x) * 16u;
        if (o < a.value_pitch) *reinterpret_cast<uint4 *>(vrow + o) = v[u];
    }
}

// Synthetic Byzantine faults (bench/test input generation only): flip one
// byte of shard corrupt[i] of instance i.
__global__ void inject_faults_kernel(uint8_t *shards, uint64_t inst_pitch, uint32_t row_pitch,
                                     const int32_t *corrupt, int count) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const int j = corrupt[i];
    if (j >= 0) shards[(size_t)i * inst_pitch + (size_t)j * row_pitch] ^= 0x5a;
}

// ============================================================================
// compact_present: the (inst, pos) list of the ECHO shards that were actually
// received (present[i][pos] != 0), for the ECHO verify to hash only those
// (validateMessage runs per received message, rbc/rbc.go:92-95); absent rows
// get valid = 0 here.  A 256-thread block handles 16 instances, one wave per
// instance at a time; the block reserves its list range with ONE global
// atomic (one per instance serialised 16k atomics on one address at C4:
// 0.19 ms), and the rows of an instance stay contiguous in the list.
// ============================================================================
constexpr int COMPACT_IPB = 16;
__global__ __launch_bounds__(256) void compact_present_kernel(const uint8_t *present, int n, int count,
                                                              uint8_t *valid, uint32_t *list, uint32_t *counter,
                                                              int prio, const uint8_t *roots_src, uint8_t *roots_dst) {
    set_wave_prio(prio);
    __shared__ uint32_t s_cnt[COMPACT_IPB];
    __shared__ uint32_t s_base;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int inst0 = blockIdx.x * COMPACT_IPB;
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    bool p[COMPACT_IPB / 4][4];
    uint64_t m[COMPACT_IPB / 4][4];
#pragma unroll
    for (int q = 0; q < COMPACT_IPB / 4; ++q) {  // wave w owns instances inst0 + 4q + w
        const int inst = inst0 + 4 * q + w;
        int total = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int pos = c * 64 + lane;
            p[q][c] = inst < count && pos < n && present[(size_t)inst * n + pos] != 0;
            m[q][c] = __ballot(p[q][c]);
            total += __popcll(m[q][c]);
            if (inst < count && pos < n && !p[q][c]) valid[(size_t)inst * n + pos] = 0;
        }
        if (lane == 0) s_cnt[4 * q + w] = (uint32_t)total;
        // the receive step keeps the roots the branches are verified against
        // (merkle_recheck_kernel's vroots): a copy here instead of a separate
        // D2D copy launch on the receiver's critical path
        if (roots_dst && inst < count && lane < 8)
            reinterpret_cast<uint32_t *>(roots_dst)[(size_t)inst * 8 + lane] =
                reinterpret_cast<const uint32_t *>(roots_src)[(size_t)inst * 8 + lane];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int i = 0; i < COMPACT_IPB; ++i) t += s_cnt[i];
        s_base = t ? atomicAdd(counter, t) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < COMPACT_IPB / 4; ++q) {
        const int slot = 4 * q + w, inst = inst0 + slot;
        uint32_t off = s_base;
        for (int i = 0; i < slot; ++i) off += s_cnt[i];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (p[q][c]) list[off + __popcll(m[q][c] & below)] = ((uint32_t)inst << 8) | (uint32_t)(c * 64 + lane);
            off += __popcll(m[q][c]);
        }
    }
}

// ============================================================================
// ACS records (rbc_dev_allgather_records): [slots][64] = {root, digest} per
// instance, zero past `count`; the digest of an instance whose interpolate
// failed (status != 0) is all-zero, so the record says on its own whether
// the instance is in the output set.  One thread per 16-byte quarter.
// ============================================================================
__global__ void pack_records_kernel(const uint8_t *roots, const uint8_t *digests, const int32_t *status, int count,
                                    int slots, uint8_t *out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= slots * 4) return;
    const int i = t >> 2, q = t & 3;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (i < count) {
        const bool ok = !status || status[i] == 0;
        if (q < 2) v = *reinterpret_cast<const uint4 *>(roots + (size_t)i * 32 + 16 * q);
        else if (digests && ok) v = *reinterpret_cast<const uint4 *>(digests + (size_t)i * 32 + 16 * (q - 2));
    }
    *reinterpret_cast<uint4 *>(out + (size_t)i * 64 + 16 * q) = v;
}

// ============================================================================
// Synthetic input (bench / tests): row r (global index first_row + local
// row), 64-bit word w of a [rows][pitch] buffer =
// splitmix64(seed * golden + r * (pitch / 8) + w), little-endian.
// The host restates the same function (cleisthenes_amd.synth) to rebuild
// any row for the oracle check, so multi-GiB inputs never cross PCIe.
// ============================================================================
RBC_DEV uint64_t splitmix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void fill_random_kernel(uint8_t *dst, uint64_t first_row, uint64_t rows,
                                                          uint64_t pitch, uint64_t seed) {
    const uint64_t chunks = pitch / 16;  // pitch % 16 == 0
    const uint64_t total = rows * chunks;
    const uint64_t base = seed * 0x9E3779B97F4A7C15ull + first_row * (pitch / 8);
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < total;
         c += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = c / chunks, q = c - r * chunks;
        const uint64_t w0 = base + r * (pitch / 8) + 2 * q;
        const uint64_t a = splitmix64(w0), b = splitmix64(w0 + 1);
        *reinterpret_cast<uint4 *>(dst + r * pitch + 16 * q) =
            make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    }
}

// Count the 16-byte chunks where rows of a and b differ in their first `len`
// bytes (both pitches % 16 == 0, 16-byte aligned bases).
__global__ __launch_bounds__(256) void count_mismatch_kernel(const uint8_t *a, uint64_t a_pitch, const uint8_t *b,
                                                             uint64_t b_pitch, uint64_t rows, uint64_t len,
                                                             uint32_t *counter) {
    const uint64_t chunks = (len + 15) / 16;
    const uint64_t total = rows * chunks;
    uint32_t bad = 0;
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < total;
         c += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = c / chunks, q = c - r * chunks;
        uint4 x = *reinterpret_cast<const uint4 *>(a + r * a_pitch + 16 * q);
        uint4 y = *reinterpret_cast<const uint4 *>(b + r * b_pitch + 16 * q);
        const int nv = (int)min((uint64_t)16, len - 16 * q);
        if (nv < 16) {
            x = mask16(x, nv);
            y = mask16(y, nv);
        }
        bad += (x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w) ? 1u : 0u;
    }
    if (bad) atomicAdd(counter, bad);
}

// The row-view value check (interpolate with values_out == NULL leaves the
// value as the k data rows of the shard set): count the 16-byte chunks of data
// row j of each instance whose first min(16, S - 16q) bytes differ from the
// value bytes at j*S + 16q, where value bytes at or past B compare as zero
// (klauspost Split's pad).  The value side is read unaligned (gfx950 buffer
// loads take any byte offset).
__global__ __launch_bounds__(256) void count_mismatch_rows_kernel(const uint8_t *shards, uint64_t inst_pitch,
                                                                  uint32_t row_pitch, int k, uint32_t S,
                                                                  const uint8_t *values, uint64_t value_pitch,
                                                                  uint32_t B, uint64_t count, uint32_t *counter) {
    const uint64_t chunks = (S + 15) / 16, per_inst = (uint64_t)k * chunks, total = count * per_inst;
    uint32_t bad = 0;
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < total;
         c += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = c / per_inst, rem = c - i * per_inst, j = rem / chunks, q = rem - j * chunks;
        uint4 x = *reinterpret_cast<const uint4 *>(shards + i * inst_pitch + j * row_pitch + 16 * q);
        const uint32_t off = (uint32_t)(j * S + 16 * q);
        uint4 y = bload16(make_rsrc(values + i * value_pitch, (uint32_t)value_pitch), off);
        const int nrow = (int)min((uint64_t)16, S - 16 * q);
        const int nval = min(nrow, (int)B - (int)off);
        x = mask16(x, nrow);
        y = mask16(y, nval);
        bad += (x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w) ? 1u : 0u;
    }
    if (bad) atomicAdd(counter, bad);
}

// The receive guard's input (bench / tests): every row a receiver must
// regenerate -- absent (present[i][j] == 0) or the one Byzantine row
// corrupt[i] -- is overwritten across its whole pitch with splitmix64 bytes
// keyed by (seed, instance, row), so only interpolate's regeneration can put
// the committed bytes back.  One 16-byte chunk per thread, grid-stride.
__global__ __launch_bounds__(256) void poison_rows_kernel(uint8_t *shards, uint64_t inst_pitch, uint32_t row_pitch,
                                                          int n, const uint8_t *present, const int32_t *corrupt,
                                                          uint64_t count, uint64_t seed) {
    const uint64_t chunks = row_pitch / 16, per_inst = (uint64_t)n * chunks, total = count * per_inst;
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < total;
         c += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = c / per_inst, rem = c - i * per_inst, j = rem / chunks, q = rem - j * chunks;
        const bool gone = (present && present[i * n + j] == 0) || (corrupt && corrupt[i] == (int32_t)j);
        if (!gone) continue;
        const uint64_t w0 = seed * 0x9E3779B97F4A7C15ull + ((i * (uint64_t)n + j) << 24) + 2 * q;
        const uint64_t a = splitmix64(w0), b = splitmix64(w0 + 1);
        *reinterpret_cast<uint4 *>(shards + i * inst_pitch + j * row_pitch + 16 * q) =
            make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    }
}

// Host batch API, receiver side: move only the PRESENT shard rows of a pinned
// caller batch into the device rows, reading the host memory directly over
// PCIe (zero-copy; measured at the DMA engine's rate, tools/probes/
// zerocopy_probe.hip).  Bytes [S, dpitch) of a present row and every absent
// row are written as zero.  One WAVE per row (r = instance * N + row), 1 KiB
// per pass: C4's 384-B rows used to leave 232 of a 256-thread block idle
// (the C4 host-fed receive ran at 10 GB/s); the 64 four-wave blocks of the
// grid keep 256 rows' reads in flight and leave the CUs to the other slots'
// kernels.  The host read is bounded to the row's S bytes.
RBC_DEV void row_gather16(const uint8_t *row, uint32_t S, uint4 *dst, uint32_t chunks, uint32_t lane) {
    const rsrc_t src = make_rsrc(row, S);
    for (uint32_t c = lane; c < chunks; c += 64) {
        const int nv = (int)S - (int)(16u * c);
        uint4 v = make_uint4(0, 0, 0, 0);
        if (nv >= 16) {
            v = bload16(src, 16u * c);
        } else if (nv > 0) {
            // a 16-byte buffer load that crosses num_records returns zero as a
            // whole: the row's last bytes are read one by one (never past S)
            uint32_t w[4] = {0u, 0u, 0u, 0u};
            for (int b = 0; b < nv; ++b) w[b >> 2] |= (uint32_t)row[16u * c + b] << (8 * (b & 3));
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        dst[c] = v;
    }
}

__global__ __launch_bounds__(256) void gather_present_kernel(const uint8_t *host, uint64_t hpitch, uint32_t S,
                                                             const uint8_t *present, uint8_t *dev, uint32_t dpitch,
                                                             uint32_t rows) {
    const uint32_t lane = threadIdx.x & 63u, waves = gridDim.x * (blockDim.x >> 6);
    const uint32_t chunks = dpitch / 16;
    for (uint32_t r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < rows; r += waves) {
        uint4 *dst = reinterpret_cast<uint4 *>(dev + (size_t)r * dpitch);
        if (!present[r]) {
            for (uint32_t c = lane; c < chunks; c += 64) dst[c] = make_uint4(0, 0, 0, 0);
            continue;
        }
        row_gather16(host + (size_t)r * hpitch, S, dst, chunks, lane);
    }
}

// Validate lane over a SPARSE pinned arena (rbc_validate_packed): a receiver
// whose ECHO rows sit at their leaf positions in a [count][N][pitch] buffer
// names only the received rows (offs), so only those bytes cross PCIe instead
// of one DMA of the whole arena.  Same zero-copy read as gather_present, one
// wave per message; the device copy keeps the host offsets (the SHA kernel
// reads rows by offs), and bytes past a message's length inside its last 64-B
// block are written as zero (sha256_row masks them anyway).  offs / lens are
// device copies.
__global__ __launch_bounds__(256) void gather_msgs_kernel(const uint8_t *host, const uint64_t *offs,
                                                          const uint32_t *lens, uint32_t count, uint8_t *dev) {
    const uint32_t lane = threadIdx.x & 63u, waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t m = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); m < count; m += waves) {
        const uint64_t off = offs[m];
        const uint32_t S = lens[m];
        row_gather16(host + off, S, reinterpret_cast<uint4 *>(dev + off), (S + 15) / 16, lane);
    }
}

// Host batch API, proposer side: many short pinned values (C4: 16,384 x 64 KiB
// per epoch) gathered into the device value rows by one launch over a device
// array of their host addresses, instead of one DMA call per value (~4 us of
// host time each).  One wave per value; bytes past lens[i] are left as they
// are (the encode masks the Split pad).
__global__ __launch_bounds__(256) void gather_values_kernel(const uint64_t *ptrs, const uint32_t *lens,
                                                            uint32_t count, uint8_t *dev, uint64_t vpitch) {
    const uint32_t lane = threadIdx.x & 63u, waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < count; i += waves)
        row_gather16(reinterpret_cast<const uint8_t *>(ptrs[i]), lens[i],
                     reinterpret_cast<uint4 *>(dev + (size_t)i * vpitch), (lens[i] + 15) / 16, lane);
}

// Interpolate over rows a validate left in device memory
// (rbc_interpolate_batch_kept): row r of the [count][n] batch is read from
// ptrs[r] (lens[r / n] bytes; 0 = an absent row, written as zeros) into
// dev + r * dpitch, zero-padded to dpitch.  One wave per row, HBM to HBM.
__global__ __launch_bounds__(256) void gather_ptrs_kernel(const uint64_t *ptrs, const uint32_t *lens, uint32_t n,
                                                          uint8_t *dev, uint32_t dpitch, uint32_t rows) {
    const uint32_t lane = threadIdx.x & 63u, waves = gridDim.x * (blockDim.x >> 6);
    const uint32_t chunks = dpitch / 16;
    for (uint32_t r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < rows; r += waves) {
        uint4 *dst = reinterpret_cast<uint4 *>(dev + (size_t)r * dpitch);
        const uint64_t src = ptrs[r];
        if (!src) {
            for (uint32_t c = lane; c < chunks; c += 64) dst[c] = make_uint4(0, 0, 0, 0);
            continue;
        }
        row_gather16(reinterpret_cast<const uint8_t *>(src), lens[r / n], dst, chunks, lane);
    }
}

// ============================================================================
// launchers
// ============================================================================
// Waves in flight for a zero-copy gather of rows of about S bytes: each wave
// moves one row per round trip over PCIe, so 256 waves keep the read queue
// full for long rows (C2: 23.8 KB); short rows (C4: 763 B) need more waves for
// the same bytes in flight (C4 host-fed validate 30 -> 54 GB/s, fused receive
// 13 -> 16, profiles/r06ac/).
static uint32_t gather_blocks(uint32_t rows, uint32_t S) {
    const uint32_t cap = S < 4096 ? 64 * std::min<uint32_t>(16u, (4096u + S - 1) / std::max(S, 1u)) : 64u;
    return std::min((rows + 3) / 4, cap);
}

// Values into the caller's row pitch on the device (host batch API): dst row
// r = src row r [0, width), zeros up to dst_pitch; one thread per dst dword,
// byte loads (dst rows need not be aligned).
__global__ __launch_bounds__(256) void pack_rows_kernel(const uint8_t *src, uint32_t src_pitch, uint8_t *dst,
                                                        uint32_t dst_pitch, uint32_t width, uint32_t total) {
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < (total + 3) / 4; w += gridDim.x * blockDim.x) {
        uint32_t v = 0;
        for (uint32_t b = 0; b < 4; ++b) {
            const uint32_t o = 4 * w + b;
            if (o >= total) break;
            const uint32_t r = o / dst_pitch, c = o - r * dst_pitch;
            if (c < width) v |= (uint32_t)src[(size_t)r * src_pitch + c] << (8 * b);
        }
        if (4 * w + 4 <= total) {
            reinterpret_cast<uint32_t *>(dst)[w] = v;
        } else {
            for (uint32_t b = 0; 4 * w + b < total; ++b) dst[4 * w + b] = (uint8_t)(v >> (8 * b));
        }
    }
}

hipError_t rbc_launch_pack_rows(const uint8_t *src, uint32_t src_pitch, uint8_t *dst, uint32_t dst_pitch,
                                uint32_t width, uint32_t rows, hipStream_t st) {
    const uint64_t total = (uint64_t)dst_pitch * rows;
    if (rows == 0 || total == 0) return hipSuccess;
    if (total >= 0xffffffffULL || width > dst_pitch || width > src_pitch || ((uintptr_t)dst % 4))
        return hipErrorInvalidValue;
    const uint32_t words = (uint32_t)((total + 3) / 4);
    hipLaunchKernelGGL(pack_rows_kernel, dim3(std::min<uint32_t>((words + 255) / 256, 8192u)), dim3(256), 0, st, src,
                       src_pitch, dst, dst_pitch, width, (uint32_t)total);
    return hipGetLastError();
}

hipError_t rbc_launch_gather_ptrs(const uint64_t *ptrs, const uint32_t *lens, uint32_t n, uint8_t *dev,
                                  uint32_t dpitch, uint32_t rows, hipStream_t st) {
    if (rows == 0) return hipSuccess;
    if (dpitch % 16 || n == 0) return hipErrorInvalidValue;
    const uint32_t blocks = std::min((rows + 3) / 4, 2048u);  // device rows: fill the chip, not a PCIe queue
    hipLaunchKernelGGL(gather_ptrs_kernel, dim3(blocks), dim3(256), 0, st, ptrs, lens, n, dev, dpitch, rows);
    return hipGetLastError();
}
hipError_t rbc_launch_gather_values(const uint64_t *ptrs, const uint32_t *lens, uint32_t count, uint8_t *dev,
                                    uint64_t vpitch, hipStream_t st) {
    if (count == 0) return hipSuccess;
    if (vpitch % 16) return hipErrorInvalidValue;
    const uint32_t blocks = std::min((count + 3) / 4, 64u);
    hipLaunchKernelGGL(gather_values_kernel, dim3(blocks), dim3(256), 0, st, ptrs, lens, count, dev, vpitch);
    return hipGetLastError();
}
hipError_t rbc_launch_gather_msgs(const uint8_t *host, const uint64_t *offs, const uint32_t *lens, uint32_t count,
                                  uint8_t *dev, uint32_t avg_len, hipStream_t st) {
    if (count == 0) return hipSuccess;
    const uint32_t blocks = gather_blocks(count, avg_len);  // as gather_present
    hipLaunchKernelGGL(gather_msgs_kernel, dim3(blocks), dim3(256), 0, st, host, offs, lens, count, dev);
    return hipGetLastError();
}

hipError_t rbc_launch_compact_present(const uint8_t *present, int n, int count, uint8_t *valid, uint32_t *list,
                                     uint32_t *counter, hipStream_t st, int prio, const uint8_t *roots_src,
                                     uint8_t *roots_dst) {
    if (count <= 0) return hipSuccess;
    if (n > 256) return hipErrorInvalidValue;
    hipLaunchKernelGGL(compact_present_kernel, dim3((count + COMPACT_IPB - 1) / COMPACT_IPB), dim3(256), 0, st,
                       present, n, count, valid, list, counter, prio, roots_src, roots_dst);
    return hipGetLastError();
}

hipError_t rbc_launch_pack_records(const uint8_t *roots, const uint8_t *digests, const int32_t *status, int count,
                                   int slots, uint8_t *out, hipStream_t st) {
    if (slots <= 0) return hipSuccess;
    hipLaunchKernelGGL(pack_records_kernel, dim3((slots * 4 + 255) / 256), dim3(256), 0, st, roots, digests, status,
                       count, slots, out);
    return hipGetLastError();
}

hipError_t rbc_launch_fill_random(uint8_t *dst, uint64_t first_row, uint64_t rows, uint64_t pitch, uint64_t seed,
                                  hipStream_t st) {
    if (rows == 0 || pitch == 0) return hipSuccess;
    if (pitch % 16) return hipErrorInvalidValue;
    hipLaunchKernelGGL(fill_random_kernel, dim3(8192), dim3(256), 0, st, dst, first_row, rows, pitch, seed);
    return hipGetLastError();
}

hipError_t rbc_launch_gather_present(const uint8_t *host, uint64_t hpitch, uint32_t S, const uint8_t *present,
                                     uint8_t *dev, uint32_t dpitch, uint32_t rows, hipStream_t st) {
    if (rows == 0) return hipSuccess;
    if (dpitch % 16 || S > dpitch) return hipErrorInvalidValue;
    const uint32_t blocks = gather_blocks(rows, S);  // one wave per row
    hipLaunchKernelGGL(gather_present_kernel, dim3(blocks), dim3(256), 0, st, host, hpitch, S, present, dev, dpitch,
                       rows);
    return hipGetLastError();
}

hipError_t rbc_launch_count_mismatch(const uint8_t *a, uint64_t a_pitch, const uint8_t *b, uint64_t b_pitch,
                                     uint64_t rows, uint64_t len, uint32_t *counter, hipStream_t st) {
    if (rows == 0 || len == 0) return hipSuccess;
    if (a_pitch % 16 || b_pitch % 16 || len > a_pitch || len > b_pitch || ((uintptr_t)a | (uintptr_t)b) % 16)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(count_mismatch_kernel, dim3(8192), dim3(256), 0, st, a, a_pitch, b, b_pitch, rows, len,
                       counter);
    return hipGetLastError();
}
hipError_t rbc_launch_count_mismatch_rows(const uint8_t *shards, uint64_t inst_pitch, uint32_t row_pitch, int k,
                                          uint32_t S, const uint8_t *values, uint64_t value_pitch, uint32_t B,
                                          uint64_t count, uint32_t *counter, hipStream_t st) {
    if (count == 0 || k <= 0 || S == 0) return hipSuccess;
    if (row_pitch % 16 || inst_pitch % 16 || ((uintptr_t)shards % 16) || S > row_pitch ||
        value_pitch < (uint64_t)k * S + 16 || value_pitch > 0x7fffffffull || B > (uint64_t)k * S)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(count_mismatch_rows_kernel, dim3(8192), dim3(256), 0, st, shards, inst_pitch, row_pitch, k, S,
                       values, value_pitch, B, count, counter);
    return hipGetLastError();
}
hipError_t rbc_launch_poison_rows(uint8_t *shards, uint64_t inst_pitch, uint32_t row_pitch, int n,
                                  const uint8_t *present, const int32_t *corrupt, uint64_t count, uint64_t seed,
                                  hipStream_t st) {
    if (count == 0 || n <= 0 || row_pitch == 0) return hipSuccess;
    if (row_pitch % 16 || inst_pitch % 16 || ((uintptr_t)shards % 16) || (uint64_t)n * row_pitch > inst_pitch)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(poison_rows_kernel, dim3(8192), dim3(256), 0, st, shards, inst_pitch, row_pitch, n, present,
                       corrupt, count, seed);
    return hipGetLastError();
}

template <int RC, int TPB = 256>
static hipError_t launch_gf_rc(const GfArgs &a, hipStream_t st) {
    const int KP = (a.K + 1) & ~1;
    const size_t lds = (size_t)20 * RC * KP + 512;
    const int chunks = a.R > 0 ? (a.R + RC - 1) / RC : 1;
    const long items = (long)a.count * a.tiles;
    dim3 grid((unsigned)(((items + 7) / 8) * 8 * chunks));
    hipLaunchKernelGGL((gf_rows_kernel<RC, TPB>), grid, dim3(TPB), lds, st, a);
    return hipGetLastError();
}

static const int kRC[] = {1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
                          18, 19, 20, 21, 22, 23, 24, 26, 28, 30, 32, 36, 40, 42, 44, 48};

int rbc_gf_pick_rc(int R, int rcmax) {
    // fewest chunks of <= rcmax rows, then the smallest instantiated RC covering them
    if (R <= 0) return 1;
    if (rcmax < 1) rcmax = 1;
    if (rcmax > 48) rcmax = 48;
    const int chunks = (R + rcmax - 1) / rcmax;
    const int want = (R + chunks - 1) / chunks;
    for (int rc : kRC)
        if (rc >= want) return rc;
    return 48;
}

hipError_t rbc_launch_gf_rows(const GfArgs &a, hipStream_t st) {
    if (a.count <= 0 || (a.R <= 0 && !a.copy)) return hipSuccess;
    if (a.tpb != 0 && a.tpb != 256) return hipErrorInvalidValue;
    switch (a.rc) {
#define RBC_RC_CASE(x) case x: return launch_gf_rc<x>(a, st);
        RBC_RC_CASE(1) RBC_RC_CASE(2) RBC_RC_CASE(3) RBC_RC_CASE(4) RBC_RC_CASE(5) RBC_RC_CASE(6)
        RBC_RC_CASE(7) RBC_RC_CASE(8) RBC_RC_CASE(9) RBC_RC_CASE(10) RBC_RC_CASE(11) RBC_RC_CASE(12)
        RBC_RC_CASE(13) RBC_RC_CASE(14) RBC_RC_CASE(15) RBC_RC_CASE(16) RBC_RC_CASE(17) RBC_RC_CASE(18)
        RBC_RC_CASE(19) RBC_RC_CASE(20) RBC_RC_CASE(21) RBC_RC_CASE(22) RBC_RC_CASE(23) RBC_RC_CASE(24)
        RBC_RC_CASE(26) RBC_RC_CASE(28) RBC_RC_CASE(30) RBC_RC_CASE(32) RBC_RC_CASE(36) RBC_RC_CASE(40)
        RBC_RC_CASE(42) RBC_RC_CASE(44) RBC_RC_CASE(48)
#undef RBC_RC_CASE
        default: return hipErrorInvalidValue;
    }
}

hipError_t rbc_launch_sha_rows(const ShaArgs &a, bool verify, hipStream_t st) {
    const long total = (long)a.count * a.rows_per_inst;
    if (total <= 0) return hipSuccess;
    // Measured (MI355X, bench): two rows per lane wins only where its ILP hits
    // the branch walk's short, cache-resident compressions and waves are
    // plentiful -- C4 verify 5.47 -> 4.51 ms (4 M rows) -- and loses wherever
    // the leaf hashing streams HBM at ~1 wave per SIMD (C2 leaves 1.93 -> 2.13,
    // C2 verify 1.99 -> 2.18, C4 leaves 2.15 -> 2.38): it halves the waves
    // that hide load latency.  So: verify only, from 4 waves per SIMD of
    // one-row work.
    constexpr int tpb2 = 256;
    const bool two = verify && !a.list && !a.per_message && a.rows_per_inst % 2 == 0 && a.n % 2 == 0 &&
                     total >= 4L * 64 * 1024;
    if (two) {
        dim3 g2((unsigned)((total / 2 + tpb2 - 1) / tpb2));
        if (verify) hipLaunchKernelGGL(sha_rows2_kernel<true>, g2, dim3(tpb2), 0, st, a);
        else hipLaunchKernelGGL(sha_rows2_kernel<false>, g2, dim3(tpb2), 0, st, a);
        return hipGetLastError();
    }
    // 256-thread blocks: the per-SIMD SHA rate hardly grows past one wave, so
    // the kernel's time is set by the SIMD that holds the most waves, and
    // 4-wave blocks spread them evenly (C2 leaves alone: 2.07 ms; one-wave
    // blocks 2.97, 128-thread 3.05; tools/gpu_r02shatpb.sh)
    // (under round 3's pipeline too: one-wave / 128-thread blocks for the
    // leaf hashing give C2 497-503 against 529-532 GB/s, C1 374-392 against
    // 469-477; tools/gpu_runs/gpu_r03ze.sh)
    dim3 grid((unsigned)((total + 255) / 256));
    if (verify) hipLaunchKernelGGL(sha_rows_kernel<true>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(sha_rows_kernel<false>, grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t rbc_launch_sha_rx(const ShaArgs &v, const ShaArgs &r, bool v_walk, hipStream_t st, uint4 *zero0,
                             uint4 *zero1) {
    const long total = (v.count > 0 ? ((long)v.count * v.rows_per_inst + 63) / 64 * 64 : 0) +
                       (r.count > 0 ? (long)r.count * r.rows_per_inst : 0);
    if (total <= 0) {  // no rows: the counters still have to be zero for their next users
        for (uint4 *z : {zero0, zero1})
            if (z) {
                const hipError_t e = hipMemsetAsync(z, 0, sizeof(uint4), st);
                if (e != hipSuccess) return e;
            }
        return hipSuccess;
    }
    if ((v.count > 0 && (!v.rows || (v_walk && (!v.valid || !v.roots)))) || (r.count > 0 && (!r.list || !r.list_count)))
        return hipErrorInvalidValue;
    // one-wave blocks: 4.78-4.82 ms per C2 receive step against 5.03 with
    // 256-thread blocks (tools/gpu_r02tpb.sh); in round 3's pipeline, C2
    // 526-531 GB/s against 477-486 (256) and 439-447 (128), C1 and C4 within
    // 3 % (tools/gpu_runs/gpu_r03y.sh)
    constexpr int tpb = 64;
    hipLaunchKernelGGL(sha_rx_kernel, dim3((unsigned)((total + tpb - 1) / tpb)), dim3(tpb), 0, st, v, r, v_walk ? 1 : 0,
                       zero0, zero1);
    return hipGetLastError();
}

hipError_t rbc_launch_merkle_path(const PathArgs &a, hipStream_t st) {
    if (a.count <= 0) return hipSuccess;
    if (a.width < 1 || a.width > 256 || (1 << a.lg_width) != a.width || a.depth != a.lg_width || a.n > a.width)
        return hipErrorInvalidValue;
    // One wave per block: an instance's leaves (L = W / 64 per lane), or
    // 64 / W instances when W < 64.  Measured (C4, MI355X): 256-thread blocks
    // (one leaf per thread) kept only 3 blocks per CU resident at 152 VGPRs,
    // mostly idle at the level barriers (path 1.34 ms); 1024-thread blocks
    // were slower still (70 KB of LDS per block).
    PathArgs b = a;
    const int L = a.width > 64 ? a.width / 64 : 1;
    b.inst_per_block = a.width >= 64 ? 1 : 64 / a.width;
    if (L == 4 && a.br_inst_pitch > 0xffffffffull)
        return hipErrorInvalidValue;  // the stage's buffer descriptor spans an instance's branches
    const dim3 grid((unsigned)((a.count + b.inst_per_block - 1) / b.inst_per_block));
    // W = 256 (C4): 32 KiB of dynamic LDS stage four branch levels of every
    // leaf (see the kernel); with the 18 KiB of its static LDS, 3 blocks per CU.
    if (L == 4) hipLaunchKernelGGL(merkle_path_kernel<4>, grid, dim3(64), (size_t)64 * 4 * 128, st, b);
    else if (L == 2) hipLaunchKernelGGL(merkle_path_kernel<2>, grid, dim3(64), 0, st, b);
    else hipLaunchKernelGGL(merkle_path_kernel<1>, grid, dim3(64), 0, st, b);
    return hipGetLastError();
}

hipError_t rbc_launch_merkle(const MerkleArgs &a, bool check, hipStream_t st) {
    if (a.count <= 0) return hipSuccess;
    if (a.width < 1 || a.width > 1024 || (a.width & (a.width - 1)) || (1 << a.depth) != a.width)
        return hipErrorInvalidValue;
    MerkleArgs b = a;
    // up to 512 / W trees per block (<= 64), but keep >= 512 blocks so that a
    // small batch still spreads over every CU (C2 and C4: 2 trees per block)
    // (C4, W = 256, measured: 1 tree per block 0.68 ms, 2 trees 0.63, 4 trees 0.95;
    // in the pipelined step 4 trees per block equal to 2 at C2 and C4, gpu_r04l.sh)
    int g = a.width >= 512 ? 1 : (512 / a.width < 64 ? 512 / a.width : 64);
    while (g > 1 && (a.count + g - 1) / g < 512) g >>= 1;
    b.trees_per_block = g;
    // W = 256 builds with branches: the top five layers in merkle_top_kernel
    // (C4: build VALU 265 -> 158 + 35 M, the step 370.9-371.0 -> 376.7-378.6 GB/s, gpu_r04t.sh)
    b.stop_m = (!check && a.width == 256 && a.depth == 8 && a.branches && a.n > 128) ? 32 : 0;
    const size_t lds = (size_t)b.trees_per_block * a.width * 32;  // 16 KiB at most
    const unsigned blocks = (unsigned)((a.count + b.trees_per_block - 1) / b.trees_per_block);
    if (check) hipLaunchKernelGGL(merkle_kernel<true>, dim3(blocks), dim3(64), lds, st, b);
    else hipLaunchKernelGGL(merkle_kernel<false>, dim3(blocks), dim3(64), lds, st, b);
    if (b.stop_m) {
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(merkle_top_kernel, dim3((unsigned)((a.count + 7) / 8)), dim3(64), 0, st, b);
    }
    return hipGetLastError();
}

hipError_t rbc_launch_recheck(const RecheckArgs &a, hipStream_t st) {
    if (a.count <= 0) return hipSuccess;
    if (a.width < 2 || a.width > 256 || (a.width & (a.width - 1)) || (1 << a.depth) != a.width)
        return hipErrorInvalidValue;
    RecheckArgs b = a;
    // G instances per one-wave block: 512 / W leaves' worth (16 KiB of node
    // LDS), but >= 512 blocks so that a small batch still spreads over the CUs
    int g = std::min(512 / a.width, 64);
    while (g > 1 && (a.count + g - 1) / g < 512) g >>= 1;
    b.inst_per_block = g;
    const size_t lds = (size_t)g * a.width * 32 + (size_t)g * 2 * a.width + (size_t)g * a.width;
    const unsigned blocks = (unsigned)((a.count + g - 1) / g);
    hipLaunchKernelGGL(merkle_recheck_kernel, dim3(blocks), dim3(64), lds, st, b);
    return hipGetLastError();
}

hipError_t rbc_launch_digest(const uint8_t *leaves, uint64_t leaves_inst_pitch, int k, const int32_t *status,
                             uint8_t *digests, int count, hipStream_t st, int prio) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(digest_kernel, dim3((count + 63) / 64), dim3(64), 0, st, leaves, leaves_inst_pitch, k, status,
                       digests, count, prio);
    return hipGetLastError();
}

hipError_t rbc_launch_decode_prepare(const PrepArgs &a, hipStream_t st) {
    if (a.count <= 0) return hipSuccess;
    if (a.fft) {
        const size_t lds = 1616 + 512;  // tables, U / missing lists, counts, log w_u, log l(x_r)
        hipLaunchKernelGGL(decode_prepare_fft_kernel, dim3(a.count), dim3(256), lds, st, a, a.gf_exp, a.gf_log);
        return hipGetLastError();
    }
    PrepArgs b = a;
    const size_t lds = 1552 + 512;
    hipLaunchKernelGGL(decode_prepare_kernel, dim3(a.count), dim3(256), lds, st, b);
    return hipGetLastError();
}

hipError_t rbc_launch_join(const JoinArgs &a, hipStream_t st) {
    if (a.count <= 0 || a.chunks == 0) return hipSuccess;
    JoinArgs b = a;
    b.blocks_per_inst = (a.chunks + 256u * JOIN_U - 1) / (256u * JOIN_U);
    const uint64_t blocks = (uint64_t)a.count * b.blocks_per_inst;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(join_kernel, dim3((unsigned)blocks), dim3(256), 0, st, b);
    return hipGetLastError();
}

hipError_t rbc_launch_inject_faults(uint8_t *shards, uint64_t inst_pitch, uint32_t row_pitch,
                                    const int32_t *corrupt, int count, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(inject_faults_kernel, dim3((count + 255) / 256), dim3(256), 0, st, shards, inst_pitch,
                       row_pitch, corrupt, count);
    return hipGetLastError();
}
