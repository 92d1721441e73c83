// sha_probe.hip -- cycles per SHA-256 compression (register-resident, no
// memory traffic) at 1..8 waves per SIMD, for the compression the data-path
// kernels use (device_common.h) and for ILP-2 (two interleaved rows per lane).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/sha_probe.hip -o tools/sha_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../cleisthenes_amd/csrc/device_common.h"

using namespace rbcdev;

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int ITER = 64;

template <int ROWS>
__global__ __launch_bounds__(256) void probe(uint32_t *out, uint32_t seed) {
    Sha256State s[ROWS];
    uint32_t w[ROWS][16];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
        sha256_init(s[r]);
#pragma unroll
        for (int i = 0; i < 16; ++i) w[r][i] = seed * (i + 1) + threadIdx.x + r;
    }
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            uint32_t m[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) m[i] = w[r][i] ^ s[r].h[i & 7];
            sha256_compress(s[r], m);
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int r = 0; r < ROWS; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc ^= s[r].h[i];
    if (acc == 0x12345678u) out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int ROWS>
void run(uint32_t *d, int cus, double ghz) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    printf("rows/lane=%d", ROWS);
    for (int wps = 1; wps <= 8; wps *= 2) {
        const int blocks = cus * wps;
        hipLaunchKernelGGL((probe<ROWS>), dim3(blocks), dim3(256), 0, 0, d, 7u);
        CHECK(hipEventRecord(a));
        const int reps = 5;
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((probe<ROWS>), dim3(blocks), dim3(256), 0, 0, d, 7u);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        const double cycles = ms / reps * 1e-3 * ghz * 1e9;
        // wave-compressions per SIMD = wps * ITER * ROWS
        printf("  w%d %.0f", wps, cycles / (wps * (double)ITER * ROWS));
    }
    printf("   (SIMD cycles per wave-compression)\n");
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
}

int main(int argc, char **argv) {
    const double ghz = argc > 1 ? atof(argv[1]) : 2.4;
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint32_t *d;
    CHECK(hipMalloc(&d, (size_t)cus * 8 * 256 * 4));
    run<1>(d, cus, ghz);
    run<2>(d, cus, ghz);
    CHECK(hipFree(d));
    return 0;
}
