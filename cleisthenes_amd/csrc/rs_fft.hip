// rs_fft.hip -- Reed-Solomon systematic encode over GF(2^8)/0x11D by additive
// FFT, for gfx950.  Bit-identical to klauspost/reedsolomon v1.9.1's matrix
// code (held at rbc/rbc.go:20; shard() at rbc/rbc.go:97-100) because it
// computes the same linear map:
//
//   klauspost's M = V * inv(V[:k]), V[r][c] = r^c, so shard r is P(r) for the
//   unique P with deg P < k and P(j) = data_j (j < k), evaluated at the field
//   elements with integer labels 0..N-1.  Those labels form the GF(2)-subspace
//   V_n = span{1, 2, .., 2^(n-1)}, the domain of the Lin-Chung-Han additive FFT
//   in the novel polynomial basis X_i = prod_{j in bits(i)} W_j, where
//   W_j = s_j / s_j(2^j) and s_j is the vanishing polynomial of V_j.  deg P < k
//   iff the novel coefficients vanish from index k on, so
//     coeffs  = solve(n, 0, data, k)   (only power-of-two IFFT/FFT blocks)
//     shards  = FFT(coeffs) at the positions [k, N)
//   Model and op counts: tests/fft_model.py (checked against the oracle by
//   tests/test_fft_model.py).
//
// Every butterfly constant W_j(lambda) is a compile-time constant, so the
// whole transform unrolls into straight-line VALU code: a constant multiply of
// 4 packed bytes is three v_perm_b32 lookups into literal 8-entry tables
// (the CDNA analogue of PSHUFB split-nibble tables), the add is v_bitop3 xor3.
// One lane owns one dword column of every row of one instance; the rows live
// in VGPRs for the whole transform (no LDS).  At N=128, k=44: 462 constant
// multiplies + ~550 xors per column instead of the matrix's 3,696 MACs.
//
// Modes: ENCODE reads data row j straight from the value bytes at j*S (Split,
// zero pad by masking) and writes data + parity rows; DECODE reads the k data
// rows of an already completed data half (interpolate: the missing data rows
// are regenerated first by gf_regen_kernel) and writes the parity positions by
// class: 0 skip (used), 1 store (missing), 2 compare (valid but unused: store,
// flag and queue for re-hash only if the re-encoding differs).
#include <utility>

#include "device_common.h"
#include "kernels.h"

using namespace rbcdev;

namespace lch {

constexpr uint32_t gmul(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1u) r ^= a;
        b >>= 1;
        a <<= 1;
        if (a & 0x100u) a ^= 0x11du;
    }
    return r;
}
constexpr uint32_t ginv(uint32_t a) {
    uint32_t r = 1, e = 254;  // a^254 = a^-1
    while (e) {
        if (e & 1u) r = gmul(r, a);
        a = gmul(a, a);
        e >>= 1;
    }
    return r;
}
// s_j(x): vanishing polynomial of V_j = span{1..2^(j-1)}; linearized, so
// s_{j+1}(x) = s_j(x) * (s_j(x) + s_j(2^j)).
constexpr uint32_t s_eval(int j, uint32_t x) {
    if (j == 0) return x;
    const uint32_t a = s_eval(j - 1, x);
    return gmul(a, a ^ s_eval(j - 1, 1u << (j - 1)));
}
// butterfly constant of layer j on coset lambda: W_j(lambda)
constexpr uint32_t twiddle(int j, uint32_t lam) { return gmul(s_eval(j, lam), ginv(s_eval(j, 1u << j))); }

struct Tab {
    uint32_t t0lo, t0hi, t1lo, t1hi, t2;
};
constexpr Tab make_tab(uint32_t c) {
    uint32_t m[8] = {};
    m[0] = c;
    for (int i = 1; i < 8; ++i) m[i] = gmul(m[i - 1], 2);
    Tab t{};
    t.t0lo = (m[0] << 8) | (m[1] << 16) | ((m[0] ^ m[1]) << 24);
    t.t0hi = m[2] | ((m[2] ^ m[0]) << 8) | ((m[2] ^ m[1]) << 16) | ((m[2] ^ m[1] ^ m[0]) << 24);
    t.t1lo = (m[3] << 8) | (m[4] << 16) | ((m[3] ^ m[4]) << 24);
    t.t1hi = m[5] | ((m[5] ^ m[3]) << 8) | ((m[5] ^ m[4]) << 16) | ((m[5] ^ m[4] ^ m[3]) << 24);
    t.t2 = (m[6] << 8) | (m[7] << 16) | ((m[6] ^ m[7]) << 24);
    return t;
}

// Per-group table registers.  gfx950 VOP3 reads one scalar operand, so one
// half of each 8-entry table must sit in a VGPR; all butterflies of one
// (layer, coset) group share the constant, so the two halves are
// materialised once per group (volatile: never CSE'd into a kernel-long
// register, which would cost occupancy) and the other half plus t2 ride in
// SGPRs.
struct TR {
    uint32_t lo0, lo1;
};
template <uint32_t C>
RBC_DEV TR tab_regs() {
    TR r{0u, 0u};
    if constexpr (C > 1) {
        constexpr Tab t = make_tab(C);
        asm volatile("v_mov_b32 %0, %1" : "=v"(r.lo0) : "i"(t.t0lo));
        asm volatile("v_mov_b32 %0, %1" : "=v"(r.lo1) : "i"(t.t1lo));
    }
    return r;
}

// a + C*x for 4 packed bytes (C compile-time, tables from tab_regs<C>())
template <uint32_t C>
RBC_DEV uint32_t mac(uint32_t a, uint32_t x, const TR &r) {
    if constexpr (C == 0) {
        return a;
    } else if constexpr (C == 1) {
        return a ^ x;
    } else {
        constexpr Tab t = make_tab(C);
        const uint32_t p0 = perm(t.t0hi, r.lo0, x & 0x07070707u);
        const uint32_t p1 = perm(t.t1hi, r.lo1, (x >> 3) & 0x07070707u);
        const uint32_t p2 = perm(t.t2, t.t2, (x >> 6) & 0x03030303u);
        return xor3(a, p0, p1) ^ p2;
    }
}

template <int B, int E, class F>
RBC_DEV void sfor(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + 1, E>(f);
    }
}

constexpr int cmin(int a, int b) { return a < b ? a : b; }
constexpr int cmax(int a, int b) { return a > b ? a : b; }

template <int V>
using IC = std::integral_constant<int, V>;

constexpr int SB = 4;  // sub-transforms of >= 2^SB rows are scheduled one after the other

// All 2^M evaluations on coset LAM + V_M, in place, of the polynomial whose
// novel coefficients are v[OFF .. OFF+2^M) (rows >= NZ are zero, never read).
template <int M, int LAM, int OFF, int NZ, int R>
RBC_DEV void fft_full(uint32_t (&v)[R]) {
    if constexpr (NZ <= 0) {
        sfor<0, (1 << M)>([&](auto I) { v[OFF + decltype(I)::value] = 0u; });
    } else if constexpr (M > 0) {
        constexpr int H = 1 << (M - 1);
        constexpr uint32_t w = twiddle(M - 1, LAM);
        constexpr int NZA = cmin(NZ, H), NZB = cmax(NZ - H, 0);
        const TR tr = NZB > 0 ? tab_regs<w>() : TR{0u, 0u};
        sfor<0, H>([&](auto I) {
            constexpr int i = decltype(I)::value;
            if constexpr (i < NZB) {
                const uint32_t a = v[OFF + i], b = v[OFF + H + i];
                const uint32_t a2 = mac<w>(a, b, tr);
                v[OFF + i] = a2;
                v[OFF + H + i] = a2 ^ b;
            } else if constexpr (i < NZA) {
                v[OFF + H + i] = v[OFF + i];  // b == 0
            }
        });
        fft_full<M - 1, LAM, OFF, NZA>(v);
        fft_full<M - 1, LAM + H, OFF + H, NZA>(v);
    }
}

// Evaluations on coset LAM + V_M of the polynomial whose novel coefficients are
// v[OFF .. OFF+2^M) (rows >= NZ are zero and never read).  Only the outputs
// with local index in [LO, HI) are needed.  Sub-transforms of size 2^G are
// completed in place and handed over as a group, st(IC<lam>, IC<off>, IC<lo>,
// IC<hi>): outputs v[off + lo .. off + hi) are the evaluations at lam + i --
// so a sink can batch its memory traffic per group.
template <int G, int M, int LAM, int OFF, int NZ, int LO, int HI, int R, class ST>
RBC_DEV void fft(uint32_t (&v)[R], ST &st) {
    if constexpr (LO >= HI) {
        return;
    } else if constexpr (M <= G) {
        fft_full<M, LAM, OFF, NZ>(v);
        st(IC<LAM>{}, IC<OFF>{}, IC<LO>{}, IC<HI>{});
    } else {
        constexpr int H = 1 << (M - 1);
        constexpr uint32_t w = twiddle(M - 1, LAM);
        constexpr int NZA = cmin(NZ, H), NZB = cmax(NZ - H, 0);
        constexpr bool needA = LO < H, needB = HI > H;
        constexpr uint32_t wt = needA ? w : (w ^ 1u);  // needB only: b' = a + (w+1) b
        const TR tr = NZB > 0 ? tab_regs<wt>() : TR{0u, 0u};
        sfor<0, H>([&](auto I) {
            constexpr int i = decltype(I)::value;
            if constexpr (i < NZB) {
                const uint32_t a = v[OFF + i], b = v[OFF + H + i];
                if constexpr (needA && needB) {
                    const uint32_t a2 = mac<wt>(a, b, tr);
                    v[OFF + i] = a2;
                    v[OFF + H + i] = a2 ^ b;
                } else if constexpr (needA) {
                    v[OFF + i] = mac<wt>(a, b, tr);
                } else {
                    v[OFF + H + i] = mac<wt>(a, b, tr);  // a + (w+1) b
                }
            } else if constexpr (i < NZA && needB) {
                v[OFF + H + i] = v[OFF + i];  // b == 0
            }
        });
        if constexpr (needA) fft<G, M - 1, LAM, OFF, NZA, LO, cmin(HI, H)>(v, st);
        // keep the scheduler from interleaving the two independent halves
        // (that would double the live rows and halve occupancy)
        if constexpr (needA && needB && M >= SB) __builtin_amdgcn_sched_barrier(0);
        if constexpr (needB) fft<G, M - 1, LAM + H, OFF + H, NZA, cmax(LO - H, 0), HI - H>(v, st);
    }
}

// Inverse transform on coset LAM + V_M, in place (all 2^M rows known).
template <int M, int LAM, int OFF, int R>
RBC_DEV void ifft(uint32_t (&v)[R]) {
    if constexpr (M > 0) {
        constexpr int H = 1 << (M - 1);
        ifft<M - 1, LAM, OFF>(v);
        ifft<M - 1, LAM + H, OFF + H>(v);
        constexpr uint32_t w = twiddle(M - 1, LAM);
        const TR tr = tab_regs<w>();
        sfor<0, H>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const uint32_t b = v[OFF + i] ^ v[OFF + H + i];
            v[OFF + H + i] = b;
            v[OFF + i] = mac<w>(v[OFF + i], b, tr);
        });
    }
}

// Rows v[OFF .. OFF+T) hold the evaluations at the first T points of
// LAM + V_M of a polynomial with novel-coefficient support [0, T); on return
// they hold those coefficients (rows [T, 2^M) are zero by construction).
template <int M, int LAM, int OFF, int T, int R>
RBC_DEV void solve(uint32_t (&v)[R]) {
    constexpr int SZ = 1 << M;
    if constexpr (T == SZ) {
        ifft<M, LAM, OFF>(v);
    } else if constexpr (T <= SZ / 2) {
        solve<M - 1, LAM, OFF, T>(v);
    } else {
        constexpr int H = SZ / 2, TP = T - H;
        constexpr uint32_t w = twiddle(M - 1, LAM);
        ifft<M - 1, LAM, OFF>(v);  // g = P0 + w P1
        // d = vals[H..T) - FFT_{LAM+H}(g)[0..TP) = FFT_{LAM+H}(P1)[0..TP)
        uint32_t g[H];
        sfor<0, H>([&](auto I) { g[decltype(I)::value] = v[OFF + decltype(I)::value]; });
        auto sub = [&](auto Lam, auto Off, auto Lo, auto Hi) {
            sfor<decltype(Lo)::value, decltype(Hi)::value>([&](auto I) {
                constexpr int i = decltype(I)::value;
                v[OFF + H + decltype(Lam)::value - (LAM + H) + i] ^= g[decltype(Off)::value + i];
            });
        };
        fft<0, M - 1, LAM + H, 0, H, 0, TP>(g, sub);
        solve<M - 1, LAM + H, OFF + H, TP>(v);  // P1
        const TR tr = tab_regs<w>();
        sfor<0, TP>([&](auto I) {              // P0 = g + w P1
            constexpr int i = decltype(I)::value;
            v[OFF + i] = mac<w>(v[OFF + i], v[OFF + H + i], tr);
        });
    }
}

}  // namespace lch

namespace {

RBC_DEV uint32_t keep_bytes4(int nv) { return nv >= 4 ? 0xffffffffu : (nv <= 0 ? 0u : ((1u << (8 * nv)) - 1u)); }

template <int LOGW, int K, int N, int MODE>
// waves_per_eu(2): at N=256 the decode variant otherwise takes 256 VGPRs + 25
// AGPRs (one wave per SIMD); with the hint it fits 256 with no scratch
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void rs_fft_kernel(FftArgs a) {
    set_wave_prio(a.prio);
    constexpr int W = 1 << LOGW;
    constexpr int G = 3;   // encode: outputs are stored in groups of 2^G rows
    constexpr int GD = 2;  // decode: compare-pipeline group (VGPRs: 1 -> 143, 2 -> 157, 3 -> 181)
    static_assert(K >= 1 && K <= N && N <= W && 2 * N > W, "geometry");
    // XCD-aware tile order: the dispatcher deals workgroups round-robin over
    // the 8 XCDs (linear id % 8), so neighbouring column tiles of one instance
    // would land on different L2s.  Encode reads data row j at j*S, which is
    // not line aligned: a 256-B tile touches 3 lines, 2 of them shared with
    // its neighbours.  Remapping linear id L -> (L % 8) * (T8 / 8) + L / 8
    // gives each XCD a contiguous run of tiles, so the shared lines hit in
    // that XCD's L2 instead of being fetched twice from HBM.  Decode too: its
    // fused join stores row j at j*S, so neighbouring tiles (and row j's end
    // and row j+1's start) share value lines, merged in one L2 this way
    // (C1 / C2 / C3 +1-3 %, profiles/r06r/).
    uint32_t tile_x = blockIdx.x, tile_y = blockIdx.y;
    {
        const uint32_t gx = gridDim.x, total = gx * gridDim.y, t8 = total & ~7u;
        uint32_t lin = blockIdx.y * gx + blockIdx.x;
        if (lin < t8) lin = (lin & 7u) * (t8 >> 3) + (lin >> 3);
        tile_y = lin / gx;
        tile_x = lin - tile_y * gx;
    }
    const int col = (int)tile_x * 64 + threadIdx.x;  // dword column inside the row
    const int inst = (int)tile_y;
    if (inst >= a.count) return;
    if (a.status && a.status[inst] != 0) return;
    const uint32_t off = 4u * (uint32_t)col;
    if (off >= a.row_pitch) return;
    uint32_t S, B = 0;
    if constexpr (MODE == GF_MODE_ENCODE) {
        B = a.lens ? a.lens[inst] : a.uniform_len;
        S = (B + K - 1) / K;
    } else {
        S = a.lens ? a.lens[inst] : a.uniform_len;
    }
    const uint32_t keep = keep_bytes4((int)S - (int)off);  // bytes past S are zero
    // every row access is base(SGPR) + off(one VGPR) + row*pitch(SGPR): one
    // VGPR of addressing for all N rows instead of a 64-bit pointer per row
    uint8_t *shards = a.shards + (size_t)inst * a.inst_pitch;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(shards, (short)0, (int)a.inst_pitch, 0x00020000);
    const int pitch = (int)a.row_pitch;
    auto row_store = [&](int pos, uint32_t x) { __builtin_amdgcn_raw_buffer_store_b32(x, rs, (int)off, pos * pitch, 0); };
    auto row_load = [&](int pos) -> uint32_t { return __builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, pos * pitch, 0); };

    uint32_t v[W];
    if constexpr (MODE == GF_MODE_ENCODE) {
        const uint8_t *val = a.values + (size_t)inst * a.value_pitch;
        const auto rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(val), (short)0, (int)a.value_pitch,
                                                           0x00020000);
        // all K loads issued back to back, unconditionally (out-of-range
        // reads return 0 through the buffer descriptor); the Split zero pad
        // is applied by masking afterwards.  Unaligned dword reads are fine
        // on gfx950.
        lch::sfor<0, K>([&](auto J) {
            constexpr int j = decltype(J)::value;
            v[j] = __builtin_amdgcn_raw_buffer_load_b32(rv, (int)off, (int)((uint32_t)j * S), 0);
        });
        lch::sfor<0, K>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const uint32_t row0 = (uint32_t)j * S;  // Split: data[j*S : (j+1)*S]
            if (row0 + S <= B) {                    // wave-uniform: a full data row
                v[j] &= keep;
            } else {                                // the rows carrying the zero pad
                const int lim = (int)(B > row0 ? B - row0 : 0u);
                v[j] &= keep_bytes4(lim - (int)off);
            }
            // materialise the masked row: otherwise the AND is folded into
            // the first butterfly (v_bitop3) and the raw row plus its mask
            // stay live through the transform (+44 VGPRs)
            asm volatile("" : "+v"(v[j]));
            row_store(j, v[j]);
        });
    } else {
        lch::sfor<0, K>([&](auto J) { v[decltype(J)::value] = row_load(decltype(J)::value); });
        if (a.join) {
            // interpolate's value (rbc/rbc.go:88) straight from the loaded rows:
            // data row j at j*S, dword stores at byte offsets that need not be
            // aligned, the lane that straddles S writes its bytes one by one;
            // tile 0 zeroes the value's tail up to join_pitch.  The buffer
            // descriptor bounds every store to the instance's value row.
            const auto rj = __builtin_amdgcn_make_buffer_rsrc(a.join + (size_t)inst * a.join_pitch, (short)0,
                                                              (int)a.join_pitch, 0x00020000);
            const int nb = (int)S - (int)off;  // this lane's valid bytes per row
            lch::sfor<0, K>([&](auto J) {
                constexpr int j = decltype(J)::value;
                const int so = (int)((uint32_t)j * S);
                if (nb >= 4) {
                    __builtin_amdgcn_raw_buffer_store_b32(v[j], rj, (int)off, so, 0);
                } else if (nb > 0) {
                    for (int b = 0; b < nb; ++b)
                        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v[j] >> (8 * b)), rj, (int)off + b, so, 0);
                }
            });
            if (tile_x == 0) {
                const uint32_t end = (uint32_t)K * S;
                for (int b = 0; b < 4; ++b) {
                    const uint32_t o = end + 4u * threadIdx.x + (uint32_t)b;
                    if (o < a.join_pitch) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)0, rj, (int)o, 0, 0);
                }
            }
        }
    }

    lch::solve<LOGW, 0, 0, K>(v);
    // opaque phase boundary: without it LLVM fuses xor chains of the final
    // transform with solve's and keeps raw input rows live to the end
    // (N=128 encode: 191 -> 127 VGPRs, 2 -> 4 waves per SIMD)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wunused-lambda-capture"  // the capture is needed (asm operand)
    lch::sfor<0, K>([&v](auto J) { asm volatile("" : "+v"(v[decltype(J)::value])); });
#pragma clang diagnostic pop

    if constexpr (MODE == GF_MODE_ENCODE) {
        auto st = [&](auto Lam, auto Off, auto Lo, auto Hi) {
            lch::sfor<decltype(Lo)::value, decltype(Hi)::value>([&](auto I) {
                constexpr int i = decltype(I)::value, pos = decltype(Lam)::value + i;
                // no `& keep`: every input byte past S was masked to zero on
                // load, and the transform is column-wise linear
                if constexpr (pos >= K && pos < N) row_store(pos, v[decltype(Off)::value + i]);
            });
        };
        lch::fft<G, LOGW, 0, 0, K, K, N>(v, st);
    } else {
        const uint32_t *cls = reinterpret_cast<const uint32_t *>(a.cls + (size_t)inst * a.cls_stride);
        // Software pipeline over output groups: the compare loads of group g
        // are in flight while group g-1 is compared and stored, so the HBM
        // latency of a compare read is paid once per kernel, not per group.
        constexpr int GS = 1 << GD;
        uint32_t px[GS], pold[GS], pc[GS];
        int ppos = 0, pcnt = 0;
        auto flush = [&]() {
            lch::sfor<0, GS>([&](auto I) {
                constexpr int i = decltype(I)::value;
                if (i < pcnt) {  // wave-uniform
                    const int pos = ppos + i;
                    if (pc[i] == 1u) {
                        row_store(pos, px[i]);
                    } else if (pc[i] == 2u && pold[i] != px[i]) {
                        row_store(pos, px[i]);
                        if (a.flags && atomicOr(&a.flags[(size_t)inst * N + pos], 1u) == 0u)
                            a.list[atomicAdd(a.counter, 1u)] = ((uint32_t)inst << 8) | (uint32_t)pos;
                    }
                }
            });
        };
        auto st = [&](auto Lam, auto Off, auto Lo, auto Hi) {
            constexpr int lam = decltype(Lam)::value, o = decltype(Off)::value;
            constexpr int lo = lch::cmax(decltype(Lo)::value, K - lam), hi = lch::cmin(decltype(Hi)::value, N - lam);
            if constexpr (lo < hi) {
                uint32_t c[hi - lo], old[hi - lo];
                // class lookups + the compare loads of this group
                lch::sfor<lo, hi>([&](auto I) {
                    constexpr int i = decltype(I)::value, pos = lam + i;
                    c[i - lo] = (cls[pos >> 2] >> (8 * (pos & 3))) & 0xffu;  // wave-uniform
                    old[i - lo] = 0;
                    if (c[i - lo] == 2u) old[i - lo] = row_load(pos);
                });
                flush();  // the previous group, while these loads fly
                lch::sfor<lo, hi>([&](auto I) {
                    constexpr int i = decltype(I)::value;
                    px[i - lo] = v[o + i] & keep;
                    pold[i - lo] = old[i - lo];
                    pc[i - lo] = c[i - lo];
                });
                ppos = lam + lo;
                pcnt = hi - lo;
            }
        };
        lch::fft<GD, LOGW, 0, 0, K, K, N>(v, st);
        flush();
    }
}

template <int LOGW, int K, int N>
hipError_t launch_fft(const FftArgs &a, hipStream_t st) {
    dim3 grid((a.row_pitch / 4 + 63) / 64, (unsigned)a.count);
    if (a.mode == GF_MODE_ENCODE)
        hipLaunchKernelGGL((rs_fft_kernel<LOGW, K, N, GF_MODE_ENCODE>), grid, dim3(64), 0, st, a);
    else
        hipLaunchKernelGGL((rs_fft_kernel<LOGW, K, N, GF_MODE_DECODE>), grid, dim3(64), 0, st, a);
    return hipGetLastError();
}

}  // namespace

hipError_t rbc_launch_rs_fft(const FftArgs &a, hipStream_t st) {
    if (a.count <= 0) return hipSuccess;
    if (a.row_pitch % 4) return hipErrorInvalidValue;
#define RBC_FFT_CASE(lw, kk, nn) \
    if (a.n == nn && a.k == kk) return launch_fft<lw, kk, nn>(a, st);
    RBC_FFT_GEOMS(RBC_FFT_CASE)
#undef RBC_FFT_CASE
    return hipErrorInvalidValue;
}
