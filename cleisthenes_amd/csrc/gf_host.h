// gf_host.h -- host-side GF(2^8) matrix construction for the encode matrix.
//
// klauspost/reedsolomon v1.9.1 (go.mod:10, held by rbc/rbc.go:20):
//   galois.go  : GF(2^8), generating polynomial 29 (0x11D), generator 2,
//                galExp(a, 0) = 1, galExp(0, n>0) = 0
//   matrix.go  : vandermonde(rows, cols)[r][c] = galExp(r, c); Invert by
//                Gauss-Jordan
//   reedsolomon.go buildMatrix(k, n) = vandermonde(n, k) * inverse(top k x k)
// Built once per context on the host (n*k <= 64 KiB) and uploaded; the
// per-instance decode matrices are built on the GPU (decode_prepare_kernel).
#pragma once
#include <stdint.h>

#include <vector>

namespace rbchost {

struct Gf {
    uint8_t exp[512];
    uint8_t log[256];
    Gf() {
        int x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = (uint8_t)x;
            log[x] = (uint8_t)i;
            x <<= 1;
            if (x & 0x100) x ^= 0x11d;
        }
        for (int i = 255; i < 512; ++i) exp[i] = exp[i - 255];
        log[0] = 0;
    }
    uint8_t mul(uint8_t a, uint8_t b) const { return (a && b) ? exp[log[a] + log[b]] : 0; }
    uint8_t div(uint8_t a, uint8_t b) const {
        if (!a) return 0;
        int r = (int)log[a] - (int)log[b];
        if (r < 0) r += 255;
        return exp[r];
    }
    uint8_t pow(uint8_t a, int n) const {
        if (n == 0) return 1;
        if (a == 0) return 0;
        return exp[(log[a] * n) % 255];
    }
};

inline const Gf &gf() {
    static const Gf g;
    return g;
}

// Gauss-Jordan inverse, n x n row-major.  Returns false if singular.
inline bool invert(int n, const uint8_t *m, uint8_t *out) {
    const Gf &g = gf();
    const int w = 2 * n;
    std::vector<uint8_t> a((size_t)n * w, 0);
    for (int r = 0; r < n; ++r) {
        for (int c = 0; c < n; ++c) a[(size_t)r * w + c] = m[(size_t)r * n + c];
        a[(size_t)r * w + n + r] = 1;
    }
    for (int r = 0; r < n; ++r) {
        if (a[(size_t)r * w + r] == 0) {
            int b = r + 1;
            while (b < n && a[(size_t)b * w + r] == 0) ++b;
            if (b == n) return false;
            for (int c = 0; c < w; ++c) std::swap(a[(size_t)r * w + c], a[(size_t)b * w + c]);
        }
        const uint8_t s = g.div(1, a[(size_t)r * w + r]);
        for (int c = 0; c < w; ++c) a[(size_t)r * w + c] = g.mul(s, a[(size_t)r * w + c]);
        for (int b = 0; b < n; ++b) {
            if (b == r) continue;
            const uint8_t f = a[(size_t)b * w + r];
            if (!f) continue;
            for (int c = 0; c < w; ++c) a[(size_t)b * w + c] ^= g.mul(f, a[(size_t)r * w + c]);
        }
    }
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) out[(size_t)r * n + c] = a[(size_t)r * w + n + c];
    return true;
}

// buildMatrix(k, n): n x k, rows 0..k-1 identity, rows k..n-1 parity.
inline bool build_matrix(int k, int n, std::vector<uint8_t> &out) {
    const Gf &g = gf();
    std::vector<uint8_t> vm((size_t)n * k), inv((size_t)k * k);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c) vm[(size_t)r * k + c] = g.pow((uint8_t)r, c);
    if (!invert(k, vm.data(), inv.data())) return false;
    out.assign((size_t)n * k, 0);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c) {
            uint8_t acc = 0;
            for (int i = 0; i < k; ++i) acc ^= g.mul(vm[(size_t)r * k + i], inv[(size_t)i * k + c]);
            out[(size_t)r * k + c] = acc;
        }
    return true;
}

}  // namespace rbchost
