// host_shared.h -- host-side facts shared by the HIP launchers and the host
// runtime (capi.cpp), kept in a header so a host-only build of the runtime
// (the sanitizer build in tests/test_sanitizers.py) needs no HIP compiler.
#pragma once
#include <stddef.h>
#include <stdint.h>

// Geometries with a specialised additive-FFT transform (rs_fft.hip): N = 3f+1
// (the BFT maximum f) for the benchmark sizes, as X(log2 N, k, N).  Other
// (N, k) use gf_rows_kernel.
#define RBC_FFT_GEOMS(X) \
    X(2, 2, 4)           \
    X(4, 6, 16)          \
    X(6, 22, 64)         \
    X(7, 44, 128)        \
    X(8, 86, 256)

inline bool rbc_fft_supported(int n, int k) {
#define RBC_FFT_SUP(lw, kk, nn) \
    if (n == nn && k == kk) return true;
    RBC_FFT_GEOMS(RBC_FFT_SUP)
#undef RBC_FFT_SUP
    return false;
}

// Bytes of the pb.Message of a VAL (type 0) / ECHO (1) request for shard
// `index` of S bytes with a depth-`depth` branch: the host mirror of the
// marshal kernel's layout().total (wire.hip), for sizing out_pitch.
inline size_t rbc_val_message_bytes(int n, int depth, uint32_t S, uint32_t index, int type) {
    auto b64 = [](uint64_t x) { return (x + 2) / 3 * 4; };
    auto vl = [](uint64_t v) {
        uint64_t l = 1;
        while (v >= 0x80) {
            v >>= 7;
            ++l;
        }
        return l;
    };
    const bool empty0 = depth > 0 && (int)(index ^ 1u) >= n;
    const uint64_t br = 32u * (uint64_t)(depth - (empty0 ? 1 : 0));
    const uint64_t J = br ? 84 + b64(br) + b64(S) : 86 + b64(S);
    const uint64_t R = 1 + vl(J) + J + (type ? 2 : 0);
    return (size_t)(1 + vl(R) + R);
}
