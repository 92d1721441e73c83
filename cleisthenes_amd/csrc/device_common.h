// device_common.h -- gfx950 (CDNA4) device helpers for the RBC data path.
//
// SHA-256 (FIPS 180-4; Go crypto/sha256, the hash the rbc package's Merkle
// commitment uses per BASELINE.json north_star) and GF(2^8)/0x11D
// (klauspost/reedsolomon v1.9.1 galois.go, held at rbc/rbc.go:20) written
// directly for the CDNA4 VALU:
//   * rotates are v_alignbit_b32, the 3-input XORs of Sigma/sigma and of the
//     GF accumulation are gfx950's v_bitop3_b32 (truth table 0x96),
//     Ch is v_bfi_b32;
//   * GF(2^8) constant multiply of 4 packed bytes is three v_perm_b32 byte
//     lookups into 8-entry tables (bits 0-2, 3-5, 6-7 of each byte) -- the
//     CDNA analogue of the PSHUFB split-nibble kernel klauspost ships for
//     amd64, with one VALU op per 4 bytes per table instead of per-byte LDS
//     lookups.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RBC_DEV __device__ __forceinline__

// Wave issue priority (s_setprio, 0..3) from a kernel argument: the SIMD's
// instruction arbiter prefers higher-priority waves.  Two streams of
// VALU-bound kernels share every SIMD under the bench's pipeline; raising
// the waves of the stream on the critical path lets its dependent SHA
// chains issue as if alone while the other stream fills the gaps.
// `p` is a kernel argument, so the branch is uniform (scalar).
RBC_DEV void set_wave_prio(int p) {
    if (p == 1) __builtin_amdgcn_s_setprio(1);
    else if (p == 2) __builtin_amdgcn_s_setprio(2);
    else if (p >= 3) __builtin_amdgcn_s_setprio(3);
}

namespace rbcdev {

RBC_DEV uint32_t rotr(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
RBC_DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
RBC_DEV uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x00010203u); }
RBC_DEV uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) { return __builtin_amdgcn_perm(hi, lo, sel); }

__constant__ static const uint32_t kSHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

struct Sha256State {
    uint32_t h[8];
};

RBC_DEV void sha256_init(Sha256State &s) {
    s.h[0] = 0x6a09e667u; s.h[1] = 0xbb67ae85u; s.h[2] = 0x3c6ef372u; s.h[3] = 0xa54ff53au;
    s.h[4] = 0x510e527fu; s.h[5] = 0x9b05688cu; s.h[6] = 0x1f83d9abu; s.h[7] = 0x5be0cd19u;
}

// One compression, message words already big-endian-decoded.  Fully
// unrolled: the K constants and (for constant padding blocks) the whole
// message schedule fold at compile time.
RBC_DEV void sha256_compress(Sha256State &s, uint32_t (&w)[16]) {
    uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3];
    uint32_t e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
            w[i & 15] = wi;
        }
        const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        const uint32_t ch = (e & f) ^ (~e & g);
        const uint32_t t1 = h + S1 + ch + kSHA_K[i] + wi;
        const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        const uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xe8);  // Maj (symmetric)
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + S0 + mj;
    }
    s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
    s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

// R independent compressions interleaved round by round.  One wave alone
// issues a dependent VALU chain at ~8.7 clk per instruction
// (profiles/r01_valu_probe.txt); R chains per lane hide that latency without
// needing more waves per SIMD (profiles/r01_sha_probe.txt: rows/lane=2).
// Rotating registers: at round i, a..h live in v[(0-i)&7] .. v[(7-i)&7].
template <int R>
RBC_DEV void sha256_compress_n(Sha256State (&s)[R], uint32_t (&w)[R][16]) {
    uint32_t v[R][8];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int q = 0; q < 8; ++q) v[r][q] = s[r].h[q];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint32_t wi;
            if (i < 16) {
                wi = w[r][i];
            } else {
                const uint32_t w15 = w[r][(i - 15) & 15], w2 = w[r][(i - 2) & 15];
                const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
                const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
                wi = w[r][i & 15] + s0 + w[r][(i - 7) & 15] + s1;
                w[r][i & 15] = wi;
            }
            uint32_t &a = v[r][(0 - i) & 7], &b = v[r][(1 - i) & 7], &c = v[r][(2 - i) & 7];
            uint32_t &d = v[r][(3 - i) & 7], &e = v[r][(4 - i) & 7], &f = v[r][(5 - i) & 7];
            uint32_t &g = v[r][(6 - i) & 7], &h = v[r][(7 - i) & 7];
            const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
            const uint32_t ch = (e & f) ^ (~e & g);
            const uint32_t t1 = h + S1 + ch + kSHA_K[i] + wi;
            const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
            const uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xe8);
            d = d + t1;        // becomes e of round i+1
            h = t1 + S0 + mj;  // becomes a of round i+1
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int q = 0; q < 8; ++q) s[r].h[q] += v[r][q];
}

// Load 64 bytes (16-byte aligned) and decode to big-endian words.
RBC_DEV void load_block_be(const uint8_t *p, uint32_t (&w)[16]) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const uint4 v = q[t];
        w[4 * t + 0] = bswap32(v.x);
        w[4 * t + 1] = bswap32(v.y);
        w[4 * t + 2] = bswap32(v.z);
        w[4 * t + 3] = bswap32(v.w);
    }
}

// SHA-256 of `len` bytes at a 16-byte-aligned row whose storage is readable
// up to round_up(len, 64) (the shard pitch guarantees it).  Byte-exact: the
// bytes past `len` inside the last block are masked, never hashed.
RBC_DEV void bswap_block(const uint4 (&q)[4], uint32_t (&w)[16]) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        w[4 * t + 0] = bswap32(q[t].x);
        w[4 * t + 1] = bswap32(q[t].y);
        w[4 * t + 2] = bswap32(q[t].z);
        w[4 * t + 3] = bswap32(q[t].w);
    }
}
RBC_DEV void load_block_raw(const uint8_t *p, uint4 (&q)[4]) {
    const uint4 *v = reinterpret_cast<const uint4 *>(p);
#pragma unroll
    for (int t = 0; t < 4; ++t) q[t] = v[t];
}

RBC_DEV void sha256_row(const uint8_t *row, uint32_t len, Sha256State &s) {
    sha256_init(s);
    const uint32_t nfull = len >> 6;
    uint32_t w[16];
    // software pipeline: block b+1's loads are in flight while block b is
    // compressed (a compression is ~1.4k VALU ops, longer than an HBM miss).
    // (Two blocks per iteration with ping-pong buffers drops 9 VALU per
    // compression and is ~2 % faster alone, but takes the leaf kernel from 108
    // to 124 VGPRs and the two-stream bench from 479-485 to 454-459 GB/s:
    // tools/gpu_runs/gpu_r02unroll.sh.)
    // (Without the prefetch the leaf kernel needs 95 VGPRs instead of 108,
    // and the bench drops from 489-498 to 469-477 GB/s: tools/gpu_runs/gpu_r02pf.sh.)
    uint4 q[4];
    if (nfull) load_block_raw(row, q);
    for (uint32_t b = 0; b < nfull; ++b) {
        bswap_block(q, w);
        if (b + 1 < nfull) load_block_raw(row + 64u * (b + 1), q);
        sha256_compress(s, w);
    }

    const uint32_t rem = len & 63u;
    if (rem) {
        load_block_be(row + 64u * nfull, w);
    } else {
#pragma unroll
        for (int t = 0; t < 16; ++t) w[t] = 0;
    }
    // keep bytes < rem, put 0x80 at rem, zero the rest
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const int nb = (int)rem - 4 * t;  // valid bytes in this word
        uint32_t v = w[t];
        if (nb >= 4) {
        } else if (nb <= 0) {
            v = (nb == 0) ? 0x80000000u : 0u;
        } else {
            const uint32_t keep = 0xffffffffu << (32 - 8 * nb);
            v = (v & keep) | (0x80u << (24 - 8 * nb));
        }
        w[t] = v;
    }
    const uint64_t bits = (uint64_t)len * 8u;
    if (rem <= 55u) {
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
        sha256_compress(s, w);
    } else {
        sha256_compress(s, w);
#pragma unroll
        for (int t = 0; t < 14; ++t) w[t] = 0;
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
        sha256_compress(s, w);
    }
}

// Last data block of a `len`-byte message (tail words already in w): keep
// the len % 64 message bytes, append 0x80, zero the rest.
RBC_DEV void sha256_pad_tail(uint32_t (&w)[16], uint32_t len) {
    const uint32_t rem = len & 63u;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const int nb = (int)rem - 4 * t;
        uint32_t v = w[t];
        if (nb >= 4) {
        } else if (nb <= 0) {
            v = (nb == 0) ? 0x80000000u : 0u;
        } else {
            const uint32_t keep = 0xffffffffu << (32 - 8 * nb);
            v = (v & keep) | (0x80u << (24 - 8 * nb));
        }
        w[t] = v;
    }
}

// Two rows of the same length hashed by one lane, compressions interleaved.
RBC_DEV void sha256_row2(const uint8_t *row0, const uint8_t *row1, uint32_t len, Sha256State (&s)[2]) {
    sha256_init(s[0]);
    sha256_init(s[1]);
    const uint32_t nfull = len >> 6;
    uint32_t w[2][16];
    uint4 q0[4], q1[4];
    if (nfull) {
        load_block_raw(row0, q0);
        load_block_raw(row1, q1);
    }
    for (uint32_t b = 0; b < nfull; ++b) {
        bswap_block(q0, w[0]);
        bswap_block(q1, w[1]);
        if (b + 1 < nfull) {
            load_block_raw(row0 + 64u * (b + 1), q0);
            load_block_raw(row1 + 64u * (b + 1), q1);
        }
        sha256_compress_n<2>(s, w);
    }
    const uint32_t rem = len & 63u;
    if (rem) {
        load_block_be(row0 + 64u * nfull, w[0]);
        load_block_be(row1 + 64u * nfull, w[1]);
    } else {
#pragma unroll
        for (int t = 0; t < 16; ++t) w[0][t] = w[1][t] = 0;
    }
    sha256_pad_tail(w[0], len);
    sha256_pad_tail(w[1], len);
    const uint64_t bits = (uint64_t)len * 8u;
    if (rem > 55u) {
        sha256_compress_n<2>(s, w);
#pragma unroll
        for (int t = 0; t < 14; ++t) w[0][t] = w[1][t] = 0;
    }
    w[0][14] = w[1][14] = (uint32_t)(bits >> 32);
    w[0][15] = w[1][15] = (uint32_t)bits;
    sha256_compress_n<2>(s, w);
}

// Two Merkle nodes H(l_r || r_r) at once (second block's schedule constant).
RBC_DEV void sha256_node64x2(const uint32_t (&l)[2][8], const uint32_t (&rr)[2][8], uint32_t (&out)[2][8]) {
    Sha256State s[2];
    sha256_init(s[0]);
    sha256_init(s[1]);
    uint32_t w[2][16];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int t = 0; t < 8; ++t) { w[r][t] = l[r][t]; w[r][8 + t] = rr[r][t]; }
    sha256_compress_n<2>(s, w);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
#pragma unroll
        for (int t = 0; t < 16; ++t) w[r][t] = 0;
        w[r][0] = 0x80000000u;
        w[r][15] = 512u;
    }
    sha256_compress_n<2>(s, w);
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int t = 0; t < 8; ++t) out[r][t] = s[r].h[t];
}

// SHA-256 over the concatenation of two 32-byte digests (Merkle node,
// HBBFT convention: H(left || right)).  Second block's schedule is constant.
RBC_DEV void sha256_node64(const uint32_t (&l)[8], const uint32_t (&r)[8], uint32_t (&out)[8]) {
    Sha256State s;
    sha256_init(s);
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 8; ++t) { w[t] = l[t]; w[8 + t] = r[t]; }
    sha256_compress(s, w);
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = 0;
    w[0] = 0x80000000u;
    w[15] = 512u;
    sha256_compress(s, w);
#pragma unroll
    for (int t = 0; t < 8; ++t) out[t] = s.h[t];
}

// SHA-256 of a single 32-byte digest (node whose right child is an empty
// padding leaf).
RBC_DEV void sha256_node32(const uint32_t (&l)[8], uint32_t (&out)[8]) {
    Sha256State s;
    sha256_init(s);
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 8; ++t) w[t] = l[t];
    w[8] = 0x80000000u;
#pragma unroll
    for (int t = 9; t < 15; ++t) w[t] = 0;
    w[15] = 256u;
    sha256_compress(s, w);
#pragma unroll
    for (int t = 0; t < 8; ++t) out[t] = s.h[t];
}

// SHA-256("") -- node whose both children are empty padding leaves.
RBC_DEV void sha256_empty(uint32_t (&out)[8]) {
    out[0] = 0xe3b0c442u; out[1] = 0x98fc1c14u; out[2] = 0x9afbf4c8u; out[3] = 0x996fb924u;
    out[4] = 0x27ae41e4u; out[5] = 0x649b934cu; out[6] = 0xa495991bu; out[7] = 0x7852b855u;
}

// Digest <-> bytes in memory (standard SHA-256 output byte order).
RBC_DEV void store_digest(uint8_t *dst, const uint32_t (&h)[8]) {
    uint4 *q = reinterpret_cast<uint4 *>(dst);
    q[0] = make_uint4(bswap32(h[0]), bswap32(h[1]), bswap32(h[2]), bswap32(h[3]));
    q[1] = make_uint4(bswap32(h[4]), bswap32(h[5]), bswap32(h[6]), bswap32(h[7]));
}
RBC_DEV void load_digest(const uint8_t *src, uint32_t (&h)[8]) {
    const uint4 *q = reinterpret_cast<const uint4 *>(src);
    const uint4 a = q[0], b = q[1];
    h[0] = bswap32(a.x); h[1] = bswap32(a.y); h[2] = bswap32(a.z); h[3] = bswap32(a.w);
    h[4] = bswap32(b.x); h[5] = bswap32(b.y); h[6] = bswap32(b.z); h[7] = bswap32(b.w);
}

// ---------------------------------------------------------------- GF(2^8)
// xtime over 0x11D for a single byte held in a uint32.
RBC_DEV uint32_t gf_xtime(uint32_t v) { return ((v << 1) ^ ((v & 0x80u) ? 0x1du : 0u)) & 0xffu; }

// Expand coefficient c into the 5 perm tables used by gf_mul4:
//   t0lo/t0hi: c*{0..7}, t1lo/t1hi: c*{0,8,..,56}, t2: c*{0,64,128,192}.
RBC_DEV void gf_tables(uint32_t c, uint4 &t01, uint32_t &t2) {
    uint32_t m[8];
    m[0] = c & 0xffu;
#pragma unroll
    for (int i = 1; i < 8; ++i) m[i] = gf_xtime(m[i - 1]);
    const uint32_t t0lo = (m[0] << 8) | (m[1] << 16) | ((m[0] ^ m[1]) << 24);
    const uint32_t t0hi = m[2] | ((m[2] ^ m[0]) << 8) | ((m[2] ^ m[1]) << 16) | ((m[2] ^ m[1] ^ m[0]) << 24);
    const uint32_t t1lo = (m[3] << 8) | (m[4] << 16) | ((m[3] ^ m[4]) << 24);
    const uint32_t t1hi = m[5] | ((m[5] ^ m[3]) << 8) | ((m[5] ^ m[4]) << 16) | ((m[5] ^ m[4] ^ m[3]) << 24);
    t01 = make_uint4(t0lo, t0hi, t1lo, t1hi);
    t2 = (m[6] << 8) | (m[7] << 16) | ((m[6] ^ m[7]) << 24);
}

// Byte selectors of a data word (shared by every coefficient applied to it).
struct GfSel {
    uint32_t s0, s1, s2;
};
RBC_DEV GfSel gf_sel(uint32_t x) {
    GfSel s;
    s.s0 = x & 0x07070707u;
    s.s1 = (x >> 3) & 0x07070707u;
    s.s2 = (x >> 6) & 0x03030303u;
    return s;
}
// c * x for 4 packed bytes, as three byte-permute lookups (XOR of the parts
// is folded into the caller's accumulation).
RBC_DEV uint32_t gf_mul4(const uint4 &t01, uint32_t t2, const GfSel &s) {
    return xor3(perm(t01.y, t01.x, s.s0), perm(t01.w, t01.z, s.s1), perm(t2, t2, s.s2));
}

}  // namespace rbcdev
