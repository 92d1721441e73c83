// duplex_probe.hip -- does host<->device traffic overlap both PCIe directions?
// The host-fed epoch (tools/host_bench.epoch) carried 27.9 GB/s in + 22.4 out
// at once, about the 55-57 GB/s one direction carries alone.  This times, on
// pinned memory (hipHostMalloc, 1 GiB each way):
//   sdma_h2d / sdma_d2h      hipMemcpyAsync alone
//   sdma_both                H2D on one stream || D2H on another
//   kread_h2d / kwrite_d2h   a kernel reading pinned host memory into HBM /
//                            writing HBM into pinned host memory (zero-copy)
//   kread+sdma_d2h           kernel reads || SDMA D2H
//   sdma_h2d+kwrite          SDMA H2D || kernel writes
//   kread+kwrite             both by kernels (two streams)
// One JSON line.  build: hipcc -O3 --offload-arch=gfx950 -o duplex_probe duplex_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

// grid-stride 16-B copy; `blocks` bounds the PCIe requests in flight
__global__ __launch_bounds__(256) void copy16(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

int main(int argc, char **argv) {
    const size_t bytes = (size_t)(argc > 1 ? atoi(argv[1]) : 1024) << 20;
    const int blocks = argc > 2 ? atoi(argv[2]) : 256;
    void *h_in, *h_out, *d_in, *d_out;
    CK(hipHostMalloc(&h_in, bytes, hipHostMallocDefault));
    CK(hipHostMalloc(&h_out, bytes, hipHostMallocDefault));
    CK(hipMalloc(&d_in, bytes));
    CK(hipMalloc(&d_out, bytes));
    for (size_t i = 0; i < bytes; i += 4096) ((char *)h_in)[i] = (char)i, ((char *)h_out)[i] = 0;
    CK(hipMemset(d_out, 1, bytes));
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    hipEvent_t e0, ea, eb;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&ea));
    CK(hipEventCreate(&eb));
    const size_t n16 = bytes / 16;
    // kinds: 0 none, 1 sdma h2d, 2 sdma d2h, 3 kernel read (h2d), 4 kernel write (d2h)
    auto issue = [&](int kind, hipStream_t s) {
        switch (kind) {
            case 1: CK(hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, s)); break;
            case 2: CK(hipMemcpyAsync(h_out, d_out, bytes, hipMemcpyDeviceToHost, s)); break;
            case 3: hipLaunchKernelGGL(copy16, dim3(blocks), dim3(256), 0, s, (const uint4 *)h_in, (uint4 *)d_in, n16); break;
            case 4: hipLaunchKernelGGL(copy16, dim3(blocks), dim3(256), 0, s, (const uint4 *)d_out, (uint4 *)h_out, n16); break;
            default: break;
        }
    };
    struct Case { const char *name; int ka, kb; };
    const Case cases[] = {{"sdma_h2d", 1, 0},       {"sdma_d2h", 2, 0},        {"sdma_both", 1, 2},
                          {"kread_h2d", 3, 0},      {"kwrite_d2h", 4, 0},      {"kread+sdma_d2h", 3, 2},
                          {"sdma_h2d+kwrite", 1, 4}, {"kread+kwrite", 3, 4}};
    printf("{\"bytes\": %zu, \"blocks\": %d", bytes, blocks);
    for (const Case &c : cases) {
        float best_a = 1e9f, best_b = 1e9f, best_all = 1e9f;
        for (int rep = 0; rep < 4; ++rep) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            CK(hipStreamWaitEvent(a, e0, 0));
            CK(hipStreamWaitEvent(b, e0, 0));
            issue(c.ka, a);
            issue(c.kb, b);
            CK(hipEventRecord(ea, a));
            CK(hipEventRecord(eb, b));
            CK(hipDeviceSynchronize());
            float ta = 0, tb = 0;
            CK(hipEventElapsedTime(&ta, e0, ea));
            CK(hipEventElapsedTime(&tb, e0, eb));
            if (rep) {  // the first repetition warms the mappings
                best_a = std::min(best_a, ta);
                best_b = std::min(best_b, tb);
                best_all = std::min(best_all, std::max(ta, c.kb ? tb : 0.f));
            }
        }
        const double gb = bytes / 1e9;
        printf(", \"%s\": {\"a_GBps\": %.2f", c.name, gb / (best_a / 1e3));
        if (c.kb) printf(", \"b_GBps\": %.2f, \"total_GBps\": %.2f", gb / (best_b / 1e3), 2 * gb / (best_all / 1e3));
        printf("}");
    }
    printf("}\n");
    return 0;
}
