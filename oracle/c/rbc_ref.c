/*
 * rbc_ref.c -- C restatement of the Cleisthenes RBC data path.
 * TEST INFRASTRUCTURE ONLY (oracle + CPU baseline).  The product path
 * (cleisthenes_amd/csrc, librbc_gpu.so) never links or calls this file.
 *
 * It restates, for speed, exactly what oracle/rbc_oracle.py restates:
 *   - klauspost/reedsolomon v1.9.1 (go.mod:10; held at rbc/rbc.go:20):
 *     GF(2^8)/0x11D, buildMatrix = vandermonde * top^-1, Split/Encode,
 *     Reconstruct "first k present by index" -- galMulSlice as the AVX2
 *     split-nibble VPSHUFB kernel klauspost ships for amd64.
 *   - crypto/sha256 (FIPS 180-4), SHA-NI when the CPU has it.
 *   - the frozen HBBFT Merkle spec (leaf = H(shard), node = H(L||R), empty
 *     padding leaves), validateMessage (rbc/rbc.go:92-95) and interpolate
 *     (rbc/rbc.go:86-90) with a full re-encode + root recheck.
 * It is checked against oracle/rbc_oracle.py (itself pinned by klauspost's
 * own test vectors) in tests/test_oracle.py.
 */
#define _GNU_SOURCE
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ GF */
static uint8_t EXP_[512], LOG_[256], MUL_[256][256];
static uint8_t TLO_[256][16], THI_[256][16];
static int gf_ready = 0;
static pthread_once_t gf_once = PTHREAD_ONCE_INIT;

static void gf_init_once(void) {
    int x = 1;
    for (int i = 0; i < 255; i++) {
        EXP_[i] = (uint8_t)x;
        LOG_[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 512; i++) EXP_[i] = EXP_[i - 255];
    for (int a = 0; a < 256; a++)
        for (int b = 0; b < 256; b++)
            MUL_[a][b] = (a && b) ? EXP_[(LOG_[a] + LOG_[b]) % 255] : 0;
    for (int c = 0; c < 256; c++)
        for (int i = 0; i < 16; i++) {
            TLO_[c][i] = MUL_[c][i];
            THI_[c][i] = MUL_[c][i << 4];
        }
    gf_ready = 1;
}
static void gf_init(void) { pthread_once(&gf_once, gf_init_once); }

uint8_t rbcref_gal_mul(uint8_t a, uint8_t b) { gf_init(); return MUL_[a][b]; }

static uint8_t gal_div(uint8_t a, uint8_t b) {
    if (!a) return 0;
    int r = (int)LOG_[a] - (int)LOG_[b];
    if (r < 0) r += 255;
    return EXP_[r];
}
static uint8_t gal_exp(uint8_t a, int n) {
    if (n == 0) return 1;
    if (a == 0) return 0;
    return EXP_[(LOG_[a] * n) % 255];
}

/* Gauss-Jordan inverse of an n x n matrix (klauspost matrix.Invert). */
int rbcref_invert(int n, const uint8_t *m, uint8_t *out) {
    gf_init();
    int w = 2 * n;
    uint8_t *work = (uint8_t *)calloc((size_t)n * w, 1);
    if (!work) return -10;
    for (int r = 0; r < n; r++) {
        memcpy(work + r * w, m + r * n, n);
        work[r * w + n + r] = 1;
    }
    for (int r = 0; r < n; r++) {
        if (work[r * w + r] == 0) {
            for (int b = r + 1; b < n; b++)
                if (work[b * w + r]) {
                    for (int c = 0; c < w; c++) {
                        uint8_t t = work[r * w + c];
                        work[r * w + c] = work[b * w + c];
                        work[b * w + c] = t;
                    }
                    break;
                }
        }
        if (work[r * w + r] == 0) { free(work); return -11; }
        if (work[r * w + r] != 1) {
            uint8_t s = gal_div(1, work[r * w + r]);
            for (int c = 0; c < w; c++) work[r * w + c] = MUL_[s][work[r * w + c]];
        }
        for (int b = 0; b < n; b++) {
            if (b == r) continue;
            uint8_t s = work[b * w + r];
            if (s)
                for (int c = 0; c < w; c++) work[b * w + c] ^= MUL_[s][work[r * w + c]];
        }
    }
    for (int r = 0; r < n; r++) memcpy(out + r * n, work + r * w + n, n);
    free(work);
    return 0;
}

/* buildMatrix(k, n): vandermonde(n, k) * inverse(top k x k).  out: n*k. */
int rbcref_encode_matrix(int k, int n, uint8_t *out) {
    gf_init();
    if (k <= 0 || n < k) return -1;
    if (n > 256) return -2;
    uint8_t *vm = (uint8_t *)malloc((size_t)n * k), *inv = (uint8_t *)malloc((size_t)k * k);
    for (int r = 0; r < n; r++)
        for (int c = 0; c < k; c++) vm[r * k + c] = gal_exp((uint8_t)r, c);
    int rc = rbcref_invert(k, vm, inv);
    if (rc) { free(vm); free(inv); return rc; }
    for (int r = 0; r < n; r++)
        for (int c = 0; c < k; c++) {
            uint8_t acc = 0;
            for (int i = 0; i < k; i++) acc ^= MUL_[vm[r * k + i]][inv[i * k + c]];
            out[r * k + c] = acc;
        }
    free(vm);
    free(inv);
    return 0;
}

/* galMulSliceXor: out ^= c * in, AVX2 split-nibble (klauspost amd64). */
__attribute__((target("avx2"))) static void mul_xor_avx2(uint8_t c, const uint8_t *in, uint8_t *out,
                                                          size_t n) {
    const __m256i lo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)TLO_[c]));
    const __m256i hi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)THI_[c]));
    const __m256i msk = _mm256_set1_epi8(0x0f);
    size_t i = 0;
    for (; i + 32 <= n; i += 32) {
        __m256i x = _mm256_loadu_si256((const __m256i *)(in + i));
        __m256i l = _mm256_and_si256(x, msk);
        __m256i h = _mm256_and_si256(_mm256_srli_epi64(x, 4), msk);
        __m256i r = _mm256_xor_si256(_mm256_shuffle_epi8(lo, l), _mm256_shuffle_epi8(hi, h));
        _mm256_storeu_si256((__m256i *)(out + i),
                            _mm256_xor_si256(_mm256_loadu_si256((const __m256i *)(out + i)), r));
    }
    for (; i < n; i++) out[i] ^= MUL_[c][in[i]];
}
static void mul_xor_scalar(uint8_t c, const uint8_t *in, uint8_t *out, size_t n) {
    const uint8_t *t = MUL_[c];
    for (size_t i = 0; i < n; i++) out[i] ^= t[in[i]];
}
static int have_avx2 = -1, have_sha = -1;
static void cpu_detect(void) {
    if (have_avx2 < 0) {
        __builtin_cpu_init();
        have_avx2 = __builtin_cpu_supports("avx2") ? 1 : 0;
        unsigned a, b, c, d;
        __asm__ volatile("cpuid" : "=a"(a), "=b"(b), "=c"(c), "=d"(d) : "a"(7), "c"(0));
        have_sha = ((b >> 29) & 1) && __builtin_cpu_supports("sse4.1");
    }
}
int rbcref_cpu_features(void) { cpu_detect(); return have_avx2 | (have_sha << 1); }
static int force_scalar = 0;
void rbcref_force_scalar(int on) { force_scalar = on; }

static void mul_xor(uint8_t c, const uint8_t *in, uint8_t *out, size_t n) {
    if (c == 0) return;
    if (have_avx2 && !force_scalar) mul_xor_avx2(c, in, out, n);
    else mul_xor_scalar(c, in, out, n);
}

/* out[r] = XOR_j coef[r*K + j] * in[j] over len bytes (codeSomeShards),
 * processed in column chunks so the k inputs stay cache resident. */
void rbcref_gf_rows(int R, int K, const uint8_t *coef, const uint8_t *const *in,
                    uint8_t *const *out, size_t len) {
    gf_init();
    cpu_detect();
    const size_t CH = 8192;
    for (size_t o = 0; o < len; o += CH) {
        size_t n = len - o < CH ? len - o : CH;
        for (int r = 0; r < R; r++) {
            memset(out[r] + o, 0, n);
            for (int j = 0; j < K; j++) mul_xor(coef[r * K + j], in[j] + o, out[r] + o, n);
        }
    }
}

/* -------------------------------------------------------------- SHA-256 */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
static const uint32_t H0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                               0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha_blocks_scalar(uint32_t st[8], const uint8_t *p, size_t nblk) {
    while (nblk--) {
        uint32_t w[64];
        for (int i = 0; i < 16; i++)
            w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 |
                   (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
        for (int i = 16; i < 64; i++) {
            uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
            uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
        for (int i = 0; i < 64; i++) {
            uint32_t S1 = ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25);
            uint32_t ch = (e & f) ^ (~e & g);
            uint32_t t1 = h + S1 + ch + K256[i] + w[i];
            uint32_t S0 = ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22);
            uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
            uint32_t t2 = S0 + mj;
            h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        st[0] += a; st[1] += b; st[2] += c; st[3] += d;
        st[4] += e; st[5] += f; st[6] += g; st[7] += h;
        p += 64;
    }
}

__attribute__((target("sha,sse4.1,ssse3"))) static void sha_blocks_ni(uint32_t st[8], const uint8_t *p,
                                                                     size_t nblk) {
    const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i TMP = _mm_loadu_si128((const __m128i *)&st[0]);
    __m128i S1 = _mm_loadu_si128((const __m128i *)&st[4]);
    TMP = _mm_shuffle_epi32(TMP, 0xB1);
    S1 = _mm_shuffle_epi32(S1, 0x1B);
    __m128i S0 = _mm_alignr_epi8(TMP, S1, 8);
    S1 = _mm_blend_epi16(S1, TMP, 0xF0);
    while (nblk--) {
        __m128i A = S0, C = S1, W[4], msg;
        for (int i = 0; i < 16; i++) {
            if (i < 4) W[i] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 16 * i)), MASK);
            msg = _mm_add_epi32(W[i & 3], _mm_loadu_si128((const __m128i *)&K256[4 * i]));
            S1 = _mm_sha256rnds2_epu32(S1, S0, msg);
            if (i >= 3 && i < 15) {  /* next schedule group, before W[i-1] gets msg1 */
                __m128i t = _mm_alignr_epi8(W[i & 3], W[(i - 1) & 3], 4);
                W[(i + 1) & 3] = _mm_sha256msg2_epu32(_mm_add_epi32(W[(i + 1) & 3], t), W[i & 3]);
            }
            msg = _mm_shuffle_epi32(msg, 0x0E);
            S0 = _mm_sha256rnds2_epu32(S0, S1, msg);
            if (i >= 1 && i <= 12) W[(i - 1) & 3] = _mm_sha256msg1_epu32(W[(i - 1) & 3], W[i & 3]);
        }
        S0 = _mm_add_epi32(S0, A);
        S1 = _mm_add_epi32(S1, C);
        p += 64;
    }
    TMP = _mm_shuffle_epi32(S0, 0x1B);
    S1 = _mm_shuffle_epi32(S1, 0xB1);
    S0 = _mm_blend_epi16(TMP, S1, 0xF0);
    S1 = _mm_alignr_epi8(S1, TMP, 8);
    _mm_storeu_si128((__m128i *)&st[0], S0);
    _mm_storeu_si128((__m128i *)&st[4], S1);
}

static void sha_blocks(uint32_t st[8], const uint8_t *p, size_t nblk) {
    if (have_sha && !force_scalar) sha_blocks_ni(st, p, nblk);
    else sha_blocks_scalar(st, p, nblk);
}

void rbcref_sha256(const uint8_t *p, size_t n, uint8_t out[32]) {
    cpu_detect();
    uint32_t st[8];
    memcpy(st, H0, sizeof st);
    size_t full = n / 64;
    sha_blocks(st, p, full);
    uint8_t tail[128];
    size_t rem = n - full * 64;
    memset(tail, 0, sizeof tail);
    memcpy(tail, p + full * 64, rem);
    tail[rem] = 0x80;
    size_t tb = (rem + 9 <= 64) ? 1 : 2;
    uint64_t bits = (uint64_t)n * 8;
    for (int i = 0; i < 8; i++) tail[tb * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha_blocks(st, tail, tb);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = st[i] >> 24;
        out[4 * i + 1] = st[i] >> 16;
        out[4 * i + 2] = st[i] >> 8;
        out[4 * i + 3] = st[i];
    }
}

/* --------------------------------------------------------------- Merkle */
static int tree_width(int n) { int w = 1; while (w < n) w <<= 1; return w; }
static int tree_depth(int n) { int w = tree_width(n), d = 0; while ((1 << d) < w) d++; return d; }
int rbcref_tree_depth(int n) { return tree_depth(n); }

/* nodes: 2W slots of 32 bytes; len[] 0 or 32 (empty padding leaves). */
static void tree_build(int n, const uint8_t *leaves, uint8_t *nodes, uint8_t *len) {
    int w = tree_width(n);
    for (int j = 0; j < w; j++) {
        if (j < n) { memcpy(nodes + 32 * (w + j), leaves + 32 * j, 32); len[w + j] = 32; }
        else { memset(nodes + 32 * (w + j), 0, 32); len[w + j] = 0; }
    }
    for (int i = w - 1; i >= 1; i--) {
        uint8_t buf[64];
        int l = len[2 * i], r = len[2 * i + 1];
        memcpy(buf, nodes + 32 * (2 * i), l);
        memcpy(buf + l, nodes + 32 * (2 * i + 1), r);
        rbcref_sha256(buf, l + r, nodes + 32 * i);
        len[i] = 32;
    }
}

/* root (32) and branches [n][d][32] (empty level-0 sibling zero-filled). */
void rbcref_merkle_from_leaves(int n, const uint8_t *leaves, uint8_t *root, uint8_t *branches) {
    int w = tree_width(n), d = tree_depth(n);
    uint8_t *nodes = (uint8_t *)malloc((size_t)64 * w);
    uint8_t *len = (uint8_t *)malloc((size_t)2 * w);
    tree_build(n, leaves, nodes, len);
    memcpy(root, nodes + 32, 32);
    if (branches)
        for (int j = 0; j < n; j++) {
            int t = w + j;
            for (int l = 0; l < d; l++, t >>= 1) memcpy(branches + ((size_t)j * d + l) * 32, nodes + 32 * (t ^ 1), 32);
        }
    free(nodes);
    free(len);
}

/* branch walk from a known leaf digest (the verify half of validateMessage) */
static int merkle_walk(int n, const uint8_t leaf[32], uint32_t index, const uint8_t *branch, const uint8_t *root) {
    if ((int)index >= n) return 0;
    int d = tree_depth(n);
    uint8_t h[32], buf[64];
    memcpy(h, leaf, 32);
    uint32_t t = index;
    for (int l = 0; l < d; l++, t >>= 1) {
        int empty = (l == 0) && ((int)(index ^ 1) >= n);
        const uint8_t *br = branch + 32 * l;
        if (empty) {
            rbcref_sha256(h, 32, h);
        } else if (t & 1) {
            memcpy(buf, br, 32); memcpy(buf + 32, h, 32); rbcref_sha256(buf, 64, h);
        } else {
            memcpy(buf, h, 32); memcpy(buf + 32, br, 32); rbcref_sha256(buf, 64, h);
        }
    }
    return memcmp(h, root, 32) == 0;
}

int rbcref_merkle_verify(int n, const uint8_t *shard, size_t S, uint32_t index, const uint8_t *branch,
                         const uint8_t *root) {
    uint8_t h[32];
    if ((int)index >= n) return 0;
    rbcref_sha256(shard, S, h);
    return merkle_walk(n, h, index, branch, root);
}

/* klauspost builds the encode matrix once in New(); cache it per (k, n) so
 * the CPU baseline does not rebuild it for every instance. */
static pthread_mutex_t mat_mu = PTHREAD_MUTEX_INITIALIZER;
static struct { int k, n; uint8_t *m; } mat_cache[16];
static const uint8_t *cached_matrix(int k, int n) {
    pthread_mutex_lock(&mat_mu);
    for (int i = 0; i < 16; i++)
        if (mat_cache[i].m && mat_cache[i].k == k && mat_cache[i].n == n) {
            pthread_mutex_unlock(&mat_mu);
            return mat_cache[i].m;
        }
    int slot = 0;
    while (slot < 16 && mat_cache[slot].m) slot++;
    if (slot == 16) { free(mat_cache[0].m); mat_cache[0].m = NULL; slot = 0; }
    uint8_t *m = (uint8_t *)malloc((size_t)n * k);
    rbcref_encode_matrix(k, n, m);
    mat_cache[slot].k = k; mat_cache[slot].n = n; mat_cache[slot].m = m;
    pthread_mutex_unlock(&mat_mu);
    return m;
}

/* ------------------------------------------------------------ RBC path */
/* shard(enc, data) + Merkle commit: value (B bytes) -> shards [n][pitch],
 * root, branches [n][d][32], leaves [n][32] (optional). */
int rbcref_encode_commit(int n, int f, const uint8_t *value, size_t B, uint8_t *shards, size_t pitch,
                         uint8_t *root, uint8_t *branches, uint8_t *leaves_out) {
    gf_init();
    int k = n - 2 * f, p = 2 * f;
    if (k <= 0 || p < 0) return -1;
    if (n > 256) return -2;
    if (B == 0) return -6;
    size_t S = (B + k - 1) / k;
    if (pitch < S) return -10;
    const uint8_t *m = cached_matrix(k, n);
    for (int j = 0; j < k; j++) {
        uint8_t *dst = shards + (size_t)j * pitch;
        size_t off = (size_t)j * S;
        size_t have = off < B ? (B - off < S ? B - off : S) : 0;
        memcpy(dst, value + off, have);
        memset(dst + have, 0, S - have);
    }
    const uint8_t **in = (const uint8_t **)malloc(sizeof(void *) * k);
    uint8_t **out = (uint8_t **)malloc(sizeof(void *) * (p ? p : 1));
    for (int j = 0; j < k; j++) in[j] = shards + (size_t)j * pitch;
    for (int r = 0; r < p; r++) out[r] = shards + (size_t)(k + r) * pitch;
    rbcref_gf_rows(p, k, m + (size_t)k * k, in, out, S);
    uint8_t *lv = leaves_out ? leaves_out : (uint8_t *)malloc((size_t)32 * n);
    for (int j = 0; j < n; j++) rbcref_sha256(shards + (size_t)j * pitch, S, lv + 32 * j);
    rbcref_merkle_from_leaves(n, lv, root, branches);
    if (!leaves_out) free(lv);
    free(in); free(out);
    return 0;
}

/* interpolate(rootHash, shards): valid[j] != 0 marks a present shard.
 * value_out: k*S bytes; digest_out: 32 bytes.  0 ok, -3 too few, -8 root mismatch. */
int rbcref_interpolate(int n, int f, const uint8_t *shards, size_t pitch, size_t S, const uint8_t *valid,
                       const uint8_t *root, uint8_t *value_out, uint8_t *digest_out) {
    gf_init();
    int k = n - 2 * f, p = 2 * f;
    if (k <= 0 || n > 256) return -1;
    int used[256], regen[256], nu = 0, nr = 0;
    for (int j = 0; j < n; j++) {
        if (valid[j] && nu < k) used[nu++] = j;
        else regen[nr++] = j;
    }
    if (nu < k) return -3;
    (void)p;
    const uint8_t *m = cached_matrix(k, n);
    uint8_t *sub = (uint8_t *)malloc((size_t)k * k),
            *inv = (uint8_t *)malloc((size_t)k * k), *dm = (uint8_t *)malloc((size_t)(nr ? nr : 1) * k);
    for (int r = 0; r < k; r++) memcpy(sub + r * k, m + (size_t)used[r] * k, k);
    int rc = rbcref_invert(k, sub, inv);
    if (rc) { free(sub); free(inv); free(dm); return rc; }
    /* D = M[regen] * inv : regenerated shard = D row . used shards */
    for (int r = 0; r < nr; r++)
        for (int c = 0; c < k; c++) {
            uint8_t acc = 0;
            for (int i = 0; i < k; i++) acc ^= MUL_[m[(size_t)regen[r] * k + i]][inv[i * k + c]];
            dm[r * k + c] = acc;
        }
    uint8_t *full = (uint8_t *)malloc((size_t)n * S);
    const uint8_t **in = (const uint8_t **)malloc(sizeof(void *) * k);
    uint8_t **out = (uint8_t **)malloc(sizeof(void *) * (nr ? nr : 1));
    for (int i = 0; i < k; i++) {
        in[i] = shards + (size_t)used[i] * pitch;
        memcpy(full + (size_t)used[i] * S, in[i], S);
    }
    for (int r = 0; r < nr; r++) out[r] = full + (size_t)regen[r] * S;
    rbcref_gf_rows(nr, k, dm, in, out, S);
    uint8_t *lv = (uint8_t *)malloc((size_t)32 * n), r2[32];
    for (int j = 0; j < n; j++) rbcref_sha256(full + (size_t)j * S, S, lv + 32 * j);
    rbcref_merkle_from_leaves(n, lv, r2, NULL);
    int ok = memcmp(r2, root, 32) == 0;
    if (ok) {
        if (value_out) memcpy(value_out, full, (size_t)k * S);
        if (digest_out) rbcref_sha256(lv, (size_t)32 * k, digest_out);
    }
    free(lv); free(full); free(in); free(out); free(sub); free(inv); free(dm);
    return ok ? 0 : -8;
}

/* interpolate() as the GPU path runs it: the first k valid shards decode the
 * rest (Lagrange/inverse D as above); a valid-but-unused shard that equals its
 * re-encoding keeps the leaf its ECHO was verified with (leaves_in[j]), every
 * other regenerated row is hashed.  Same result as rbcref_interpolate, which
 * re-hashes all n rows. */
int rbcref_interpolate_leaves(int n, int f, const uint8_t *shards, size_t pitch, size_t S, const uint8_t *valid,
                              const uint8_t *leaves_in, const uint8_t *root, uint8_t *value_out,
                              uint8_t *digest_out) {
    gf_init();
    int k = n - 2 * f;
    if (k <= 0 || n > 256) return -1;
    int used[256], regen[256], nu = 0, nr = 0;
    for (int j = 0; j < n; j++) {
        if (valid[j] && nu < k) used[nu++] = j;
        else regen[nr++] = j;
    }
    if (nu < k) return -3;
    const uint8_t *m = cached_matrix(k, n);
    uint8_t *sub = (uint8_t *)malloc((size_t)k * k),
            *inv = (uint8_t *)malloc((size_t)k * k), *dm = (uint8_t *)malloc((size_t)(nr ? nr : 1) * k);
    for (int r = 0; r < k; r++) memcpy(sub + r * k, m + (size_t)used[r] * k, k);
    int rc = rbcref_invert(k, sub, inv);
    if (rc) { free(sub); free(inv); free(dm); return rc; }
    for (int r = 0; r < nr; r++)
        for (int c = 0; c < k; c++) {
            uint8_t acc = 0;
            for (int i = 0; i < k; i++) acc ^= MUL_[m[(size_t)regen[r] * k + i]][inv[i * k + c]];
            dm[r * k + c] = acc;
        }
    uint8_t *full = (uint8_t *)malloc((size_t)n * S);
    const uint8_t **in = (const uint8_t **)malloc(sizeof(void *) * k);
    uint8_t **out = (uint8_t **)malloc(sizeof(void *) * (nr ? nr : 1));
    for (int i = 0; i < k; i++) {
        in[i] = shards + (size_t)used[i] * pitch;
        memcpy(full + (size_t)used[i] * S, in[i], S);
    }
    for (int r = 0; r < nr; r++) out[r] = full + (size_t)regen[r] * S;
    rbcref_gf_rows(nr, k, dm, in, out, S);
    uint8_t *lv = (uint8_t *)malloc((size_t)32 * n), r2[32];
    for (int i = 0; i < k; i++) memcpy(lv + 32 * used[i], leaves_in + 32 * used[i], 32);
    for (int r = 0; r < nr; r++) {
        const int j = regen[r];
        if (valid[j] && memcmp(full + (size_t)j * S, shards + (size_t)j * pitch, S) == 0)
            memcpy(lv + 32 * j, leaves_in + 32 * j, 32);
        else
            rbcref_sha256(full + (size_t)j * S, S, lv + 32 * j);
    }
    rbcref_merkle_from_leaves(n, lv, r2, NULL);
    int ok = memcmp(r2, root, 32) == 0;
    if (ok) {
        if (value_out) memcpy(value_out, full, (size_t)k * S);
        if (digest_out) rbcref_sha256(lv, (size_t)32 * k, digest_out);
    }
    free(lv); free(full); free(in); free(out); free(sub); free(inv); free(dm);
    return ok ? 0 : -8;
}

/* ------------------------------------------------- CPU baseline pipeline */
/* One "step" per instance, the same work bench.py's GPU step does:
 * encode+commit -> (corrupt) -> verify all N echoes -> interpolate from the
 * first k valid of a present subset -> value + digest. */
typedef struct {
    int n, f, first, count, nvals;
    size_t B;
    const uint8_t *values;      /* nvals x B; instance i uses value i % nvals */
    const uint8_t *present;     /* count x n */
    const int32_t *corrupt;     /* count: shard index to corrupt or -1 */
    int status_sum;
    double enc_secs, dec_secs;  /* this thread's encode+commit / verify+decode time */
} job_t;

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void *pipeline_worker(void *arg) {
    job_t *jb = (job_t *)arg;
    int n = jb->n, f = jb->f, k = n - 2 * f, d = tree_depth(n);
    size_t S = (jb->B + k - 1) / k, pitch = (S + 63) & ~(size_t)63;
    uint8_t *shards = (uint8_t *)malloc((size_t)n * pitch);
    uint8_t *br = (uint8_t *)malloc((size_t)n * (d ? d : 1) * 32);
    uint8_t *value = (uint8_t *)malloc((size_t)k * S);
    uint8_t *lv = (uint8_t *)malloc((size_t)32 * n);
    uint8_t root[32], dig[32], valid[256];
    for (int i = 0; i < jb->count; i++) {
        const int vi = (jb->first + i) % jb->nvals;
        const double t0 = now_s();
        rbcref_encode_commit(n, f, jb->values + (size_t)vi * jb->B, jb->B, shards, pitch, root, br, NULL);
        const double t1 = now_s();
        int cj = jb->corrupt[i];
        if (cj >= 0) shards[(size_t)cj * pitch] ^= 0x5a;
        /* validateMessage for every present ECHO, keeping its leaf digest */
        for (int j = 0; j < n; j++) {
            valid[j] = 0;
            if (!jb->present[(size_t)i * n + j]) continue;
            rbcref_sha256(shards + (size_t)j * pitch, S, lv + 32 * j);
            valid[j] = (uint8_t)merkle_walk(n, lv + 32 * j, j, br + (size_t)j * d * 32, root);
        }
        int rc = rbcref_interpolate_leaves(n, f, shards, pitch, S, valid, lv, root, value, dig);
        jb->status_sum += rc;
        if (cj >= 0) shards[(size_t)cj * pitch] ^= 0x5a;
        const double t2 = now_s();
        jb->enc_secs += t1 - t0;
        jb->dec_secs += t2 - t1;
    }
    free(shards); free(br); free(value); free(lv);
    return NULL;
}

/* Returns wall seconds for `count` instances split over `threads`. */
double rbcref_pipeline2(int n, int f, int count, size_t B, int threads, const uint8_t *values, int nvals,
                        const uint8_t *present, const int32_t *corrupt, int *status_sum, double *enc_secs,
                        double *dec_secs);
double rbcref_pipeline(int n, int f, int count, size_t B, int threads, const uint8_t *values, int nvals,
                       const uint8_t *present, const int32_t *corrupt, int *status_sum) {
    return rbcref_pipeline2(n, f, count, B, threads, values, nvals, present, corrupt, status_sum, NULL, NULL);
}

/* ... and the summed per-thread time of each phase (encode+commit,
 * verify+decode), so phase rates are bytes * threads / phase seconds. */
double rbcref_pipeline2(int n, int f, int count, size_t B, int threads, const uint8_t *values, int nvals,
                        const uint8_t *present, const int32_t *corrupt, int *status_sum, double *enc_secs,
                        double *dec_secs) {
    gf_init();
    cpu_detect();
    if (threads < 1) threads = 1;
    if (threads > count) threads = count;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    job_t jobs[256];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    int per = count / threads, extra = count % threads, first = 0;
    for (int t = 0; t < threads; t++) {
        int c = per + (t < extra);
        jobs[t] = (job_t){n, f, first, c, nvals, B, values, present + (size_t)first * n, corrupt + first, 0, 0, 0};
        pthread_create(&th[t], NULL, pipeline_worker, &jobs[t]);
        first += c;
    }
    int s = 0;
    double es = 0, ds = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        s += jobs[t].status_sum;
        es += jobs[t].enc_secs;
        ds += jobs[t].dec_secs;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (status_sum) *status_sum = s;
    if (enc_secs) *enc_secs = es;
    if (dec_secs) *dec_secs = ds;
    return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}

/* validateMessage (rbc/rbc.go:92-95) for `count` ECHO messages on `threads`
 * host threads (SHA-NI where present): message m verifies shard j[m] of
 * instance inst[m] against its branch and root, from a committed set of
 * shards [ninst][n][S], branches [ninst][n][d][32], roots [ninst][32].  The
 * batcher's CPU baseline (bench.py cpu_baseline leg).  Returns wall seconds. */
typedef struct {
    int n, d, first, count;
    size_t S;
    const uint8_t *shards, *branches, *roots;
    const int32_t *inst, *j;
    uint8_t *ok;
} vjob_t;

static void *verify_worker(void *arg) {
    vjob_t *jb = (vjob_t *)arg;
    for (int m = jb->first; m < jb->first + jb->count; m++) {
        const size_t i = (size_t)jb->inst[m], j = (size_t)jb->j[m];
        jb->ok[m] = (uint8_t)rbcref_merkle_verify(jb->n, jb->shards + (i * jb->n + j) * jb->S, jb->S, (uint32_t)j,
                                                  jb->branches + (i * jb->n + j) * jb->d * 32, jb->roots + 32 * i);
    }
    return NULL;
}

double rbcref_verify_many(int n, size_t S, const uint8_t *shards, const uint8_t *branches, const uint8_t *roots,
                          int count, const int32_t *inst, const int32_t *j, int threads, uint8_t *ok) {
    cpu_detect();
    if (threads < 1) threads = 1;
    if (threads > count) threads = count;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    vjob_t jobs[256];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    int per = count / threads, extra = count % threads, first = 0;
    for (int t = 0; t < threads; t++) {
        int c = per + (t < extra);
        jobs[t] = (vjob_t){n, tree_depth(n), first, c, S, shards, branches, roots, inst, j, ok};
        pthread_create(&th[t], NULL, verify_worker, &jobs[t]);
        first += c;
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}
