// gf_probe.hip -- register-resident cost of one radix-16 additive-FFT block
// (4 layers, 32 butterflies, compile-time twiddles) in the product's packed
// form and in a bit-sliced form, to price the bit-sliced transform
//  with measured numbers.
//
//   packed : one lane holds one dword (4 byte-columns) of 16 rows; a constant
//            multiply-add is lch::mac (3 v_perm table lookups + selectors +
//            xor3), exactly the code rs_fft_kernel runs.
//   sliced : one lane holds 8 bit-planes (32 byte-columns) of 16 rows, 128
//            VGPRs; a constant multiply-add is its 8x8 GF(2) matrix unrolled
//            into an XOR network (bitop3 xor3 chains, no tables).
//   sliced+T: the same, with the byte -> bit-plane transposition of every row
//            before the block and back after it (3 swap-move stages, 12
//            swap-moves per 32 bytes each way), as a one-pass kernel would pay.
//
// Reported: SIMD clk per wave of radix-16 blocks over 32 byte-columns per
// lane (x 16 rows) = wall clk x SIMDs / wave-blocks, i.e. throughput at the
// occupancy the register count allows (packed: 8 blocks of 4 columns = one
// 32-column block).  tools/isa_mix.py-style static counts: llvm-objdump.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I cleisthenes_amd/csrc tools/gf_probe.hip -o tools/gf_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../cleisthenes_amd/csrc/rs_fft.hip"

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int ITER = 256;
constexpr int LAM = 16;  // coset of the block (non-trivial twiddles on every layer)

namespace probe {

using lch::sfor;

// a += C * b over 8 bit-planes: plane j of C*b is the XOR of the planes i of b
// whose basis image C*x^i has bit j set
template <uint32_t C>
__device__ __forceinline__ void smac(uint32_t (&a)[8], const uint32_t (&b)[8]) {
    if constexpr (C == 1) {
        sfor<0, 8>([&](auto J) { a[decltype(J)::value] ^= b[decltype(J)::value]; });
    } else if constexpr (C > 1) {
        // two new terms per v_bitop3 xor3 (LLVM leaves a plain chain of v_xor)
        sfor<0, 8>([&](auto J) {
            constexpr int j = decltype(J)::value;
            uint32_t acc = a[j], pend = 0;
            bool have = false;  // folded at compile time
            sfor<0, 8>([&](auto I) {
                constexpr int i = decltype(I)::value;
                if constexpr ((lch::gmul(C, 1u << i) >> j) & 1u) {
                    if (have) acc = xor3(acc, pend, b[i]);
                    else pend = b[i];
                    have = !have;
                }
            });
            a[j] = have ? acc ^ pend : acc;
        });
    }
}

// lch::fft_full over bit-sliced rows (all 2^M rows present)
template <int M, int LAM_, int OFF, int R>
__device__ __forceinline__ void sfft(uint32_t (&p)[R][8]) {
    if constexpr (M > 0) {
        constexpr int H = 1 << (M - 1);
        constexpr uint32_t w = lch::twiddle(M - 1, LAM_);
        sfor<0, H>([&](auto I) {
            constexpr int i = decltype(I)::value;
            smac<w>(p[OFF + i], p[OFF + H + i]);                                            // a' = a + w b
            sfor<0, 8>([&](auto J) { p[OFF + H + i][decltype(J)::value] ^= p[OFF + i][decltype(J)::value]; });  // b' = a' + b
        });
        sfft<M - 1, LAM_, OFF>(p);
        sfft<M - 1, LAM_ + H, OFF + H>(p);
    }
}

__device__ __forceinline__ void swapmove(uint32_t &a, uint32_t &b, int s, uint32_t m) {
    const uint32_t t = ((a >> s) ^ b) & m;
    b ^= t;
    a ^= t << s;
}

// 32 bytes (8 dwords) <-> 8 bit-planes: an 8x8 bit transpose per byte lane
// (an involution, so the same stages invert it)
__device__ __forceinline__ void transpose8(uint32_t (&x)[8]) {
    sfor<0, 4>([&](auto I) { swapmove(x[decltype(I)::value], x[decltype(I)::value + 4], 4, 0x0f0f0f0fu); });
    sfor<0, 2>([&](auto I) {
        swapmove(x[decltype(I)::value], x[decltype(I)::value + 2], 2, 0x33333333u);
        swapmove(x[decltype(I)::value + 4], x[decltype(I)::value + 6], 2, 0x33333333u);
    });
    sfor<0, 4>([&](auto I) { swapmove(x[2 * decltype(I)::value], x[2 * decltype(I)::value + 1], 1, 0x55555555u); });
}

}  // namespace probe

__global__ __launch_bounds__(256) void packed_kernel(uint32_t *out, uint32_t seed) {
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = seed * (i + 7) ^ threadIdx.x;
    for (int it = 0; it < ITER; ++it) {
        lch::fft_full<4, LAM, 0, 16>(v);
        asm volatile("" : "+v"(v[0]));
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) r ^= v[i];
    if (r == 0x12345678u) out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <bool TRANSPOSE>
__global__ __launch_bounds__(256) void sliced_kernel(uint32_t *out, uint32_t seed) {
    uint32_t p[16][8];
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) p[i][j] = seed * (8 * i + j + 7) ^ threadIdx.x;
    for (int it = 0; it < ITER; ++it) {
        if constexpr (TRANSPOSE) {
#pragma unroll
            for (int i = 0; i < 16; ++i) probe::transpose8(p[i]);
        }
        probe::sfft<4, LAM, 0>(p);
        if constexpr (TRANSPOSE) {
#pragma unroll
            for (int i = 0; i < 16; ++i) probe::transpose8(p[i]);
        }
        asm volatile("" : "+v"(p[0][0]));
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) r ^= p[i][j];
    if (r == 0x12345678u) out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// host check: the sliced block computes the packed block's bytes
__global__ void check_kernel(uint32_t *bad) {
    const uint32_t t = threadIdx.x;
    uint32_t v[8][16], p[16][8];
    for (int c = 0; c < 8; ++c)
        for (int i = 0; i < 16; ++i) v[c][i] = (t * 2654435761u) ^ (0x9e3779b9u * (uint32_t)(16 * c + i + 1));
    for (int i = 0; i < 16; ++i)
        for (int c = 0; c < 8; ++c) p[i][c] = v[c][i];
    for (int c = 0; c < 8; ++c) lch::fft_full<4, LAM, 0, 16>(v[c]);
    for (int i = 0; i < 16; ++i) probe::transpose8(p[i]);
    probe::sfft<4, LAM, 0>(p);
    for (int i = 0; i < 16; ++i) probe::transpose8(p[i]);
    uint32_t nbad = 0;
    for (int i = 0; i < 16; ++i)
        for (int c = 0; c < 8; ++c) nbad += p[i][c] != v[c][i];
    if (nbad) atomicAdd(bad, nbad);
}

template <class F>
double time_ms(F launch) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    launch();
    CHECK(hipEventRecord(a));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return ms / reps;
}

int main(int argc, char **argv) {
    const double ghz = argc > 1 ? atof(argv[1]) : 2.4;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount, simds = 4 * cus;
    uint32_t *d, *bad;
    CHECK(hipMalloc(&d, (size_t)cus * 16 * 256 * 4));
    CHECK(hipMalloc(&bad, 4));
    CHECK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(check_kernel, dim3(1), dim3(64), 0, 0, bad);
    uint32_t nbad = 0;
    CHECK(hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost));
    printf("sliced == packed bytes: %s (%u mismatching dwords)\n", nbad ? "NO" : "yes", nbad);
    const int blocks = cus * 16;  // 16 waves per CU: as many as the registers allow
    const double lanes = (double)blocks * 256 * ITER;
    struct R {
        const char *name;
        double ms, cols_per_lane;
    } rs[3] = {
        {"packed (lch::mac, 4 byte-columns per lane)",
         time_ms([&] { hipLaunchKernelGGL(packed_kernel, dim3(blocks), dim3(256), 0, 0, d, 7u); }), 4},
        {"sliced (XOR networks, 32 byte-columns per lane)",
         time_ms([&] { hipLaunchKernelGGL(sliced_kernel<false>, dim3(blocks), dim3(256), 0, 0, d, 7u); }), 32},
        {"sliced + transposes in and out",
         time_ms([&] { hipLaunchKernelGGL(sliced_kernel<true>, dim3(blocks), dim3(256), 0, 0, d, 7u); }), 32},
    };
    printf("clock assumed %.2f GHz, %d SIMDs, radix-16 block = 4 layers x 8 butterflies over 16 rows\n", ghz, simds);
    double base = 0;
    for (auto &r : rs) {
        // SIMD clk per wave of radix-16 blocks, normalised to 32 byte-columns per lane
        const double clk = r.ms * 1e-3 * ghz * 1e9 * simds / (lanes / 64) * (32.0 / r.cols_per_lane);
        if (base == 0) base = clk;
        printf("%-50s %8.3f ms  %8.1f SIMD clk per wave-block of 32 columns  (%.2fx of packed)\n", r.name, r.ms, clk,
               clk / base);
    }
    CHECK(hipFree(d));
    CHECK(hipFree(bad));
    return nbad ? 1 : 0;
}
