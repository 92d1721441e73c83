// Zero-copy bandwidth probe: a kernel reading pinned host memory (PCIe reads
// issued by the CUs) vs hipMemcpyAsync (SDMA), for the host batch API's
// present-rows-only H2D question.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void gather_rows(const uint4 *__restrict__ src, uint4 *__restrict__ dst, const unsigned *rows,
                            unsigned row16, unsigned nrows) {
    // one block per listed row; 16-byte chunks strided by the block
    const unsigned r = blockIdx.x;
    if (r >= nrows) return;
    const unsigned src_row = rows[r];
    const uint4 *s = src + (size_t)src_row * row16;
    uint4 *d = dst + (size_t)src_row * row16;
    for (unsigned i = threadIdx.x; i < row16; i += blockDim.x) d[i] = s[i];
}

int main() {
    const unsigned rows_total = 64 * 128, row_bytes = 23936, row16 = row_bytes / 16;
    const size_t bytes = (size_t)rows_total * row_bytes;
    void *h, *d;
    CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    CK(hipMalloc(&d, bytes));
    memset(h, 1, bytes);
    unsigned *list_h = (unsigned *)malloc(rows_total * 4), *list_d;
    CK(hipMalloc(&list_d, rows_total * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int frac = 3; frac >= 2; --frac) {  // all rows, then 2/3 of them
        unsigned n = 0;
        for (unsigned r = 0; r < rows_total; ++r)
            if (frac == 3 || r % 3 != 0) list_h[n++] = r;
        CK(hipMemcpy(list_d, list_h, n * 4, hipMemcpyHostToDevice));
        for (int tpb : {256, 512, 1024}) {
            hipLaunchKernelGGL(gather_rows, dim3(n), dim3(tpb), 0, 0, (const uint4 *)h, (uint4 *)d, list_d, row16, n);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a, 0));
            for (int it = 0; it < 5; ++it)
                hipLaunchKernelGGL(gather_rows, dim3(n), dim3(tpb), 0, 0, (const uint4 *)h, (uint4 *)d, list_d, row16, n);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("{\"probe\": \"kernel H2D gather\", \"rows\": %u, \"tpb\": %d, \"GBps\": %.2f, \"ms_per_batch\": %.3f}\n", n, tpb,
                   (double)n * row_bytes * 5 / (ms / 1e3) / 1e9, ms / 5);
        }
    }
    CK(hipEventRecord(a, 0));
    for (int it = 0; it < 5; ++it) CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"probe\": \"hipMemcpyAsync H2D\", \"GBps\": %.2f}\n", (double)bytes * 5 / (ms / 1e3) / 1e9);
    return 0;
}
