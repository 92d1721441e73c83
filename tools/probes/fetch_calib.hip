// fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE on gfx950 for the access
// widths this repository's kernels use, on byte counts known in advance
// (MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for 16-B-per-lane
// streaming reads, which it reports at 1/2).  Run under
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib
// and divide each dispatch's FETCH_SIZE (KiB) by the bytes it prints.
//   stream16 : 16 B per lane, contiguous, every byte of 1 GiB once
//   sparse32 : 32 B per lane at a 256-B lane stride (one 32-B piece of every
//              other 128-B line), as merkle_path_kernel reads one branch level
//   level<l> : four launches, l = 0..3, each reading bytes [32l, 32l + 32) of
//              every 256-B record: the same 128-B line four times, one level
//              per launch (merkle_path's levels 0..3 when nothing stays cached)
//   quad128  : the four levels' 128 B of every record in one launch (8 lanes
//              x 16 B per record): the same lines, each fetched once
// The buffer is 4 GiB, far past the 256 MiB last-level cache, so every pass
// misses on-die.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x)                                                              \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            return 1;                                                         \
        }                                                                     \
    } while (0)

__global__ void stream16(const uint4 *p, uint64_t n16, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;  // never true for the fill below; keeps the loads
}

// records of 256 B; read 32 B at byte `off` (+16 B pieces) of each
__global__ void strided32(const uint8_t *p, uint64_t records, uint32_t off, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < records;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 *q = reinterpret_cast<const uint4 *>(p + r * 256 + off);
        const uint4 a = q[0], b = q[1];
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// 8 lanes x 16 B cover bytes [0, 128) of one 256-B record
__global__ void quad128(const uint8_t *p, uint64_t records, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < records * 8;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = *reinterpret_cast<const uint4 *>(p + (t >> 3) * 256 + (t & 7) * 16);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const uint64_t bytes = 4ull << 30;
    uint8_t *buf = nullptr;
    uint32_t *sink = nullptr;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(buf, 0x5a, bytes));
    CHECK(hipDeviceSynchronize());
    const dim3 grid(8192), block(256);
    const uint64_t s_bytes = 1ull << 30;
    hipLaunchKernelGGL(stream16, grid, block, 0, 0, reinterpret_cast<const uint4 *>(buf), s_bytes / 16, sink);
    CHECK(hipDeviceSynchronize());
    printf("stream16  useful %llu B, 128-B lines %llu B\n", (unsigned long long)s_bytes, (unsigned long long)s_bytes);
    const uint64_t records = bytes / 256;
    hipLaunchKernelGGL(strided32, grid, block, 0, 0, buf, records, 0u, sink);
    CHECK(hipDeviceSynchronize());
    printf("sparse32  useful %llu B, 128-B lines %llu B\n", (unsigned long long)(records * 32),
           (unsigned long long)(records * 128));
    for (uint32_t l = 0; l < 4; ++l) {
        hipLaunchKernelGGL(strided32, grid, block, 0, 0, buf, records, 32u * l, sink);
        CHECK(hipDeviceSynchronize());
        printf("level%u    useful %llu B, 128-B lines %llu B\n", l, (unsigned long long)(records * 32),
               (unsigned long long)(records * 128));
    }
    hipLaunchKernelGGL(quad128, grid, block, 0, 0, buf, records, sink);
    CHECK(hipDeviceSynchronize());
    printf("quad128   useful %llu B, 128-B lines %llu B\n", (unsigned long long)(records * 128),
           (unsigned long long)(records * 128));
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    return 0;
}
