// gf_regen.hip -- interpolate's missing-data-row GEMV for the FFT codec
// (its own translation unit: the kernel is instantiated per row count, and
// compiles in parallel with kernels.hip).
#include <algorithm>

#include "buffer_io.h"
#include "kernels.h"

using namespace rbcdev;

// ============================================================================
// gf_regen: interpolate's missing data rows with the FFT codec (decode mode,
// no compare / copy): out[r] = XOR_j D[r][j] * in[j] for the rcount[i] <= R
// missing rows of each instance (klauspost codeSomeShards, the missing-data
// half of Reconstruct).
//
// One block per (instance, group of NT column tiles); a tile is 64 lanes x W
// words and belongs to one wave, which accumulates ALL of the instance's m
// rows over it (passes of at most RC rows).  So every input byte is read
// from HBM once, by the one wave that owns its column, and the byte
// selectors of an input word are computed once and shared by every row.
// Round 3 split the rows of one tile over the waves of a block instead: each
// wave read the same k input rows, shared only through the caches as far as
// the waves stayed in step -- PMC reads 1.25x (C2) / 1.69x (C4) of k*S
// (profiles/r04c_*).  The NT waves of a block use the same coefficients, so
// the five perm tables of each (row, input) are built once per block, JC
// inputs at a time, by all of its lanes into one of two LDS buffers: one
// barrier per chunk (a wave reaches the barrier of chunk c only after its
// MACs of chunk c-1, so building c+1 into the other buffer never overwrites
// tables in use).  The MAC loop reads them by wave-uniform broadcast at a
// VGPR base plus immediates.  The pass body is instantiated per row count
// (1..RC): straight-line, no per-row exit (that costs ~2x the registers).
// ============================================================================
template <int W>
struct GfVec {
    uint32_t v[W];
};
// f(IntC<rows>{}) for a runtime rows in [I, MAX]
template <int I, int MAX, class F>
__device__ __forceinline__ void dispatch_rows(int rows, F &&f) {
    if constexpr (I <= MAX) {
        if (rows == I) f(IntC<I>{});
        else dispatch_rows<I + 1, MAX>(rows, f);
    }
}

template <int W, int RC, int JC, int NT, int WPE>
__global__ __launch_bounds__(64 * NT) __attribute__((amdgpu_waves_per_eu(WPE))) void gf_regen_kernel(GfArgs a) {
    static_assert(JC % 4 == 0, "two input pairs per trip");
    static_assert(W >= 1 && W <= 4, "1 to 4 words per lane");
    set_wave_prio(a.prio);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = (int)uniform(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    const int groups = (a.tiles + NT - 1) / NT;
    const int inst = (int)blockIdx.x / groups;
    const int tile = ((int)blockIdx.x - inst * groups) * NT + wave;
    if (inst >= a.count) return;
    if (a.status && a.status[inst] != 0) return;  // block-uniform, before any barrier
    const int m = min(a.rcount[inst], a.R);
    if (m <= 0) return;
    const uint32_t pitch = a.out_row_pitch;
    // a wave past the last tile still builds tables and meets the barriers
    const bool live = tile < a.tiles && (uint32_t)tile * (256u * W) < pitch;
    const uint32_t my_off = (uint32_t)tile * (256u * W) + 4u * W * (uint32_t)lane;
    // lanes past the pitch load a clamped column (never stored): the buffer
    // range check does not cover the scalar row offset
    const uint32_t ld_off = min(my_off, pitch - 4u * W);
    const uint32_t S = inst_len(a.lens, a.uniform_len, inst);
    const int K = a.K;
    const int KP = (K + 3) & ~3;
    constexpr uint32_t T01_B = 16u * RC * JC, T2_B = 8u * RC * (JC / 2), BUF_B = T01_B + T2_B;
    uint32_t *s_off = reinterpret_cast<uint32_t *>(smem + 2 * BUF_B);
    const uint8_t *in_inst = a.in + (size_t)inst * a.in_inst_pitch;
    uint8_t *out_inst = a.out + (size_t)inst * a.out_inst_pitch;
    const rsrc_t rin = make_rsrc(in_inst, a.in_inst_bytes);
    const rsrc_t rout = make_rsrc(out_inst, (uint32_t)a.out_inst_pitch);
    const uint8_t *idx = a.in_idx + (size_t)inst * a.idx_stride;
    // input row starts; the prefetch past K reads row 0 (never accumulated)
    for (int t = (int)threadIdx.x; t < KP + 8; t += 64 * NT)
        s_off[t] = (t < K ? (uint32_t)idx[t] : 0u) * a.in_row_pitch;
    __syncthreads();
    const uint8_t *coef = a.coef + (size_t)inst * a.coef_inst_stride;
    const uint8_t *oidx = a.out_idx + (size_t)inst * a.idx_stride2;

    auto load_row = [&](int j) -> GfVec<W> {
        const uint32_t so = uniform(s_off[j]);
        GfVec<W> x;
        if constexpr (W == 4) {
            auto v = __builtin_amdgcn_raw_buffer_load_b128(rin, (int)ld_off, (int)so, 0);
            x.v[0] = v[0]; x.v[1] = v[1]; x.v[2] = v[2]; x.v[3] = v[3];
        } else if constexpr (W == 3) {
            auto v = __builtin_amdgcn_raw_buffer_load_b96(rin, (int)ld_off, (int)so, 0);
            x.v[0] = v[0]; x.v[1] = v[1]; x.v[2] = v[2];
        } else if constexpr (W == 2) {
            auto v = __builtin_amdgcn_raw_buffer_load_b64(rin, (int)ld_off, (int)so, 0);
            x.v[0] = v[0]; x.v[1] = v[1];
        } else {
            x.v[0] = __builtin_amdgcn_raw_buffer_load_b32(rin, (int)ld_off, (int)so, 0);
        }
        return x;
    };

    auto pass = [&](auto rgc, int r0) {
        constexpr int RG = decltype(rgc)::value;
        // the thread id through an opaque copy: otherwise LLVM hoists every
        // row count's thread-derived table addresses out of the pass to the
        // kernel entry, where RC sets of them stay live and spill (round 3's
        // form spilled 116 B of scratch per lane: its dirty lines were ~1x
        // the missing rows' bytes of extra HBM writes and reads, PMC r04b)
        int tid = (int)threadIdx.x;
        asm volatile("" : "+v"(tid));
        uint32_t acc[RG][W];
#pragma unroll
        for (int r = 0; r < RG; ++r)
#pragma unroll
            for (int w = 0; w < W; ++w) acc[r][w] = 0;
        // tables of inputs [j0, j0 + JC) for the RG rows into buffer `buf`,
        // layout [j][r] (t2 as {j even, j odd} pairs), zero past K; the
        // block's threads take consecutive rows of one input (adjacent 16-B
        // LDS stores)
        auto build = [&](int j0, int buf) {
            uint4 *t01s = reinterpret_cast<uint4 *>(smem + buf * BUF_B);
            uint32_t *t2s = reinterpret_cast<uint32_t *>(smem + buf * BUF_B + T01_B);
            for (int e = tid; e < RG * JC; e += 64 * NT) {
                const int jl = e / RG, r = e - jl * RG, j = j0 + jl;
                const uint32_t cf = j < K ? coef[(size_t)(r0 + r) * K + j] : 0u;
                uint4 t01;
                uint32_t t2;
                gf_tables(cf, t01, t2);
                t01s[jl * RC + r] = t01;
                t2s[((jl >> 1) * RC + r) * 2 + (jl & 1)] = t2;
            }
        };
        auto mac_pair = [&](int buf, int jl, const GfVec<W> &xa, const GfVec<W> &xb) {
            GfSel sa[W], sb[W];
#pragma unroll
            for (int w = 0; w < W; ++w) {
                sa[w] = gf_sel(xa.v[w]);
                sb[w] = gf_sel(xb.v[w]);
            }
            uint32_t o01 = (uint32_t)buf * BUF_B + (uint32_t)jl * (16u * RC);
            uint32_t o2 = (uint32_t)buf * BUF_B + T01_B + (uint32_t)(jl >> 1) * (8u * RC);
            asm volatile("" : "+v"(o01), "+v"(o2));  // VGPR base: no per-read v_mov of an SGPR address
            const unsigned char *p01 = smem + o01;
            const unsigned char *p2 = smem + o2;
#pragma unroll
            for (int r = 0; r < RG; ++r) {
                const uint4 ta = *reinterpret_cast<const uint4 *>(p01 + 16 * r);
                const uint4 tb = *reinterpret_cast<const uint4 *>(p01 + 16 * (RC + r));
                const uint2 t2 = *reinterpret_cast<const uint2 *>(p2 + 8 * r);
#pragma unroll
                for (int w = 0; w < W; ++w)
                    acc[r][w] = xor3(acc[r][w], gf_mul4(ta, t2.x, sa[w]), gf_mul4(tb, t2.y, sb[w]));
            }
        };
        // two buffers of an input pair each, every load issued one pair of
        // multiplies ahead of its use (see gf_rows_kernel)
        GfVec<W> a0{}, a1{}, b0{}, b1{};
        if (live) {
            a0 = load_row(0);
            a1 = load_row(1);
        }
        for (int j = 0; j < KP; j += 4) {
            const int jl = j % JC, buf = (j / JC) & 1;  // JC % 4 == 0: a chunk starts at a trip
            if (jl == 0) {
                build(j, buf);
                __syncthreads();
            }
            if (live) {
                b0 = load_row(j + 2);
                b1 = load_row(j + 3);
                mac_pair(buf, jl, a0, a1);
                a0 = load_row(j + 4);
                a1 = load_row(j + 5);
                mac_pair(buf, jl + 2, b0, b1);
            }
        }
        if (!live) return;
        // one dwordx4 / x2 / x1 store per lane and row; zero the bytes past
        // S, never write past the pitch (a multiple of 4 * W: whole lanes)
        const int nvalid = (int)S - (int)my_off;
        if (my_off < pitch) {
#pragma unroll
            for (int r = 0; r < RG; ++r) {
                const uint32_t so = uniform((uint32_t)oidx[r0 + r] * pitch);
                uint32_t v[W];
#pragma unroll
                for (int w = 0; w < W; ++w) v[w] = acc[r][w] & keep_bytes(nvalid - 4 * w);
                if constexpr (W == 4) {
                    __builtin_amdgcn_raw_buffer_store_b128(u32x4{v[0], v[1], v[2], v[3]}, rout, (int)my_off, (int)so, 0);
                } else if constexpr (W == 3) {
                    if (my_off + 12u <= pitch) {
                        __builtin_amdgcn_raw_buffer_store_b96(u32x3{v[0], v[1], v[2]}, rout, (int)my_off, (int)so, 0);
                    } else {  // the last tile's lane that straddles the pitch (pitch % 12 != 0)
#pragma unroll
                        for (int w = 0; w < 3; ++w)
                            if (my_off + 4u * w < pitch)
                                __builtin_amdgcn_raw_buffer_store_b32(v[w], rout, (int)(my_off + 4u * w), (int)so, 0);
                    }
                } else if constexpr (W == 2) {
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2{v[0], v[1]}, rout, (int)my_off, (int)so, 0);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b32(v[0], rout, (int)my_off, (int)so, 0);
                }
            }
        }
    };
    static_assert(RC <= 48, "up to 48 rows a pass");
    for (int r0 = 0; r0 < m; r0 += RC) {
        const int rows = min(RC, m - r0);  // block-uniform
        dispatch_rows<1, RC>(rows, [&](auto rgc) { pass(rgc, r0); });
        __syncthreads();  // the next pass's first build reuses buffer 0
    }
}

hipError_t rbc_launch_gf_regen(const GfArgs &a, hipStream_t st) {
    if (a.count <= 0 || a.R <= 0) return hipSuccess;
    if (a.mode != GF_MODE_DECODE || !a.rcount || a.nmiss || a.copy || a.K < 1 || a.K > 248 || a.out_row_pitch % 4u)
        return hipErrorInvalidValue;
    // one wave per column tile owns every missing row: 512-B tiles (8 B per
    // lane), or 256 B (4 B per lane) for rows of at most 2 KiB, where they keep
    // the lanes busy (C4: S = 763 -> 3 tiles, 99 %)
    const uint32_t S = a.lens ? a.out_row_pitch : a.uniform_len;
    // (C4's 768-B row as ONE tile of 12 B per lane, a wave owning the whole
    // instance at 167 VGPRs: 308-312 against 320 GB/s, tools/gpu_runs/gpu_r04e.sh)
    const int W = S <= 2048 ? 1 : 2;
    GfArgs b = a;
    b.wpt = W;
    b.tiles = (int)((a.out_row_pitch + 256u * W - 1) / (256u * W));
    constexpr int JC = 16;  // inputs per table chunk; 8 measured the same at C2 and C4 (gpu_r04i.sh)
    const int KP = (a.K + 3) & ~3;
    auto go = [&](auto kern, int RC, int NT) {
        const uint64_t blocks = (uint64_t)b.count * ((b.tiles + NT - 1) / NT);
        if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
        const size_t lds = 2 * (size_t)24 * RC * JC + 4 * (size_t)(KP + 8);
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(64 * NT), lds, st, b);
        return hipGetLastError();
    };
    if (W == 1)  // short rows (C4: S = 763, 3 tiles of 256 B; m ~ 29 +- 4 of k = 86 in one pass)
        return go(gf_regen_kernel<1, 40, JC, 3, 4>, 40, 3);
    // long rows (C1-C3: m ~ 7-15 of k = 22-44): 512-B tiles, four to a block
    return go(gf_regen_kernel<2, 24, JC, 4, 4>, 24, 4);
}

