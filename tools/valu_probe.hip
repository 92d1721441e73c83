// valu_probe.hip -- issue cost of the integer VALU instructions the SHA-256
// and GF(2^8) kernels are built from, at 1..8 waves per SIMD.
//
// Each lane runs CH independent chains (or one dependent chain) of a single
// instruction in inline asm, ITER times.  Reported: cycles per
// wave-instruction per SIMD = wall cycles / (waves per SIMD * instructions
// per wave), at the clock given on the command line (default 2.4 GHz).
// Build: hipcc -O3 --offload-arch=gfx950 tools/valu_probe.hip -o tools/valu_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CH 8
#define ITER 2048

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

template <int KIND>
__device__ __forceinline__ void op(uint32_t &v, uint32_t x, uint32_t y) {
    if (KIND == 0) asm volatile("v_alignbit_b32 %0, %0, %0, %1" : "+v"(v) : "v"(x));
    if (KIND == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v) : "v"(x), "v"(y));
    if (KIND == 2) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(v) : "v"(x), "v"(y));
    if (KIND == 3) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v) : "v"(x), "v"(y));
    if (KIND == 4) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v) : "v"(x));
    if (KIND == 5) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v) : "v"(x));
    if (KIND == 6) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v) : "v"(x), "v"(y));
    if (KIND == 7) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(v) : "v"(x), "v"(y));
    if (KIND == 8) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(v));
    if (KIND == 9) asm volatile("v_and_b32 %0, %0, %1" : "+v"(v) : "v"(x));
}

template <int KIND, bool DEP>
__global__ __launch_bounds__(256) void probe(uint32_t *out, uint32_t seed) {
    uint32_t v[CH];
    const uint32_t x = seed ^ threadIdx.x, y = seed * 3u + blockIdx.x;
#pragma unroll
    for (int i = 0; i < CH; ++i) v[i] = x + i;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i) op<KIND>(v[DEP ? 0 : i], x, y);
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < CH; ++i) r ^= v[i];
    if (r == 0x12345678u) out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

static const char *NAMES[] = {"alignbit", "bitop3", "add3", "perm", "xor", "add_u32", "fma_f32", "bfi", "lshr",
                              "and"};

template <int KIND, bool DEP>
void run(uint32_t *d, int cus, double ghz) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    printf("%-9s %s", NAMES[KIND], DEP ? "dep  " : "indep");
    for (int wps = 1; wps <= 8; wps *= 2) {
        const int blocks = cus * wps;  // 256 threads = one wave per SIMD per block
        hipLaunchKernelGGL((probe<KIND, DEP>), dim3(blocks), dim3(256), 0, 0, d, 7u);
        CHECK(hipEventRecord(a));
        const int reps = 5;
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((probe<KIND, DEP>), dim3(blocks), dim3(256), 0, 0, d, 7u);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        const double cycles = ms / reps * 1e-3 * ghz * 1e9;
        printf("  w%d %.2f", wps, cycles / (wps * (double)ITER * CH));
    }
    printf("   (cyc per wave-instr per SIMD)\n");
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
}

template <int KIND>
void both(uint32_t *d, int cus, double ghz) {
    run<KIND, false>(d, cus, ghz);
    run<KIND, true>(d, cus, ghz);
}

int main(int argc, char **argv) {
    const double ghz = argc > 1 ? atof(argv[1]) : 2.4;
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    printf("CUs=%d clockRate=%d kHz, assumed %.2f GHz\n", cus, p.clockRate, ghz);
    uint32_t *d;
    CHECK(hipMalloc(&d, (size_t)cus * 8 * 256 * 4));
    both<0>(d, cus, ghz);
    both<1>(d, cus, ghz);
    both<2>(d, cus, ghz);
    both<3>(d, cus, ghz);
    both<4>(d, cus, ghz);
    both<5>(d, cus, ghz);
    both<6>(d, cus, ghz);
    both<7>(d, cus, ghz);
    both<8>(d, cus, ghz);
    both<9>(d, cus, ghz);
    CHECK(hipFree(d));
    return 0;
}
