// hip_stub.cpp -- a host-memory stand-in for the HIP runtime, RCCL and the
// kernel launchers, so that csrc/capi.cpp (the host runtime behind
// include/rbc_gpu.h: argument parsing, staging, tickets, ACS assembly, the
// Encoder mirror) can be built with a host compiler under ASan + UBSan and
// driven with random arguments (tests/cpp/capi_fuzz.cpp, tests/test_sanitizers.py).
//
// Test infrastructure only; nothing here is part of the product.
//  * Device memory is host memory (calloc), so every staging copy the runtime
//    makes is checked by ASan against the real allocation sizes.
//  * hipHostMalloc ranges are remembered, so hipPointerGetAttributes reports
//    pinned caller memory the way the runtime's zero-copy checks expect.
//  * Every launcher "runs" its kernel by touching (memset) exactly the output
//    ranges the real kernel writes for the arguments it was given, so an
//    undersized device or workspace buffer is an ASan report.
//  * Streams and events are dummies; every call completes at once.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <mutex>

#include "../../cleisthenes_amd/csrc/kernels.h"

namespace {
std::mutex mu;
std::map<const char *, size_t> pinned;  // hipHostMalloc'd ranges
std::map<const char *, size_t> devmem;  // hipMalloc'd ranges (reported as device memory)
struct Dummy {
    int x = 0;
};
void touch(void *p, size_t bytes) {
    if (p && bytes) memset(p, 0, bytes);
}
// a read the kernel makes (last byte of a range), kept by the compiler
template <class T>
void peek(const T *p, size_t i) {
    volatile T x = p[i];
    (void)x;
}
}  // namespace

extern "C" {
hipError_t hipGetDeviceCount(int *n) {
    *n = 1;
    return hipSuccess;
}
hipError_t hipSetDevice(int d) { return d == 0 ? hipSuccess : hipErrorInvalidDevice; }
hipError_t hipDeviceSynchronize() { return hipSuccess; }
hipError_t hipGetLastError() { return hipSuccess; }
hipError_t hipRuntimeGetVersion(int *v) {
    *v = 70200000;
    return hipSuccess;
}
hipError_t hipMemGetInfo(size_t *f, size_t *t) {
    *f = (size_t)1 << 34;
    *t = (size_t)1 << 35;
    return hipSuccess;
}
hipError_t hipDeviceGetPCIBusId(char *out, int len, int) {
    snprintf(out, len, "0000:00:00.0");
    return hipSuccess;
}
hipError_t hipDeviceGetStreamPriorityRange(int *least, int *greatest) {
    *least = 0;
    *greatest = -1;
    return hipSuccess;
}
hipError_t hipMalloc(void **p, size_t bytes) {
    *p = calloc(1, bytes ? bytes : 1);
    if (!*p) return hipErrorOutOfMemory;
    std::lock_guard<std::mutex> lk(mu);
    devmem[(const char *)*p] = bytes ? bytes : 1;
    return hipSuccess;
}
hipError_t hipFree(void *p) {
    {
        std::lock_guard<std::mutex> lk(mu);
        devmem.erase((const char *)p);
    }
    free(p);
    return hipSuccess;
}
hipError_t hipHostMalloc(void **p, size_t bytes, unsigned int) {
    *p = calloc(1, bytes ? bytes : 1);
    if (!*p) return hipErrorOutOfMemory;
    std::lock_guard<std::mutex> lk(mu);
    pinned[(const char *)*p] = bytes ? bytes : 1;
    return hipSuccess;
}
hipError_t hipHostFree(void *p) {
    {
        std::lock_guard<std::mutex> lk(mu);
        pinned.erase((const char *)p);
    }
    free(p);
    return hipSuccess;
}
hipError_t hipPointerGetAttributes(hipPointerAttribute_t *a, const void *p) {
    std::lock_guard<std::mutex> lk(mu);
    auto in = [p](std::map<const char *, size_t> &m) {
        auto it = m.upper_bound((const char *)p);
        if (it == m.begin()) return false;
        --it;
        return (const char *)p < it->first + it->second;
    };
    memset(a, 0, sizeof *a);
    if (in(pinned)) {
        a->type = hipMemoryTypeHost;
        a->devicePointer = const_cast<void *>(p);
        a->hostPointer = const_cast<void *>(p);
        return hipSuccess;
    }
    if (in(devmem)) {  // hipMalloc'd "device" memory
        a->type = hipMemoryTypeDevice;
        a->devicePointer = const_cast<void *>(p);
        return hipSuccess;
    }
    return hipErrorInvalidValue;
}
hipError_t hipMemcpy(void *d, const void *s, size_t n, hipMemcpyKind) {
    if (n) memcpy(d, s, n);
    return hipSuccess;
}
hipError_t hipMemcpyAsync(void *d, const void *s, size_t n, hipMemcpyKind k, hipStream_t) {
    return hipMemcpy(d, s, n, k);
}
hipError_t hipMemcpy2DAsync(void *d, size_t dp, const void *s, size_t sp, size_t w, size_t h, hipMemcpyKind,
                            hipStream_t) {
    for (size_t r = 0; r < h; ++r) memcpy((char *)d + r * dp, (const char *)s + r * sp, w);
    return hipSuccess;
}
hipError_t hipMemset(void *p, int v, size_t n) {
    if (n) memset(p, v, n);
    return hipSuccess;
}
hipError_t hipMemsetAsync(void *p, int v, size_t n, hipStream_t) { return hipMemset(p, v, n); }
hipError_t hipMemset2DAsync(void *p, size_t pitch, int v, size_t w, size_t h, hipStream_t) {
    for (size_t r = 0; r < h; ++r) memset((char *)p + r * pitch, v, w);
    return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned int) {
    *s = reinterpret_cast<hipStream_t>(new Dummy);
    return hipSuccess;
}
hipError_t hipStreamCreateWithPriority(hipStream_t *s, unsigned int f, int) { return hipStreamCreateWithFlags(s, f); }
hipError_t hipStreamDestroy(hipStream_t s) {
    delete reinterpret_cast<Dummy *>(s);
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned int) { return hipSuccess; }
hipError_t hipEventCreate(hipEvent_t *e) {
    *e = reinterpret_cast<hipEvent_t>(new Dummy);
    return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned int) { return hipEventCreate(e); }
hipError_t hipEventDestroy(hipEvent_t e) {
    delete reinterpret_cast<Dummy *>(e);
    return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventQuery(hipEvent_t) { return hipSuccess; }
hipError_t hipEventElapsedTime(float *ms, hipEvent_t, hipEvent_t) {
    *ms = 0.f;
    return hipSuccess;
}

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
    memset(id->internal, 7, sizeof id->internal);
    return ncclSuccess;
}
ncclResult_t ncclCommInitRank(ncclComm_t *c, int nranks, ncclUniqueId, int rank) {
    if (nranks != 1 || rank != 0) return ncclInvalidArgument;
    *c = reinterpret_cast<ncclComm_t>(new Dummy);
    return ncclSuccess;
}
ncclResult_t ncclCommDestroy(ncclComm_t c) {
    delete reinterpret_cast<Dummy *>(c);
    return ncclSuccess;
}
ncclResult_t ncclCommCount(const ncclComm_t, int *n) {
    *n = 1;
    return ncclSuccess;
}
ncclResult_t ncclCommUserRank(const ncclComm_t, int *r) {
    *r = 0;
    return ncclSuccess;
}
ncclResult_t ncclGetVersion(int *v) {
    *v = 22707;
    return ncclSuccess;
}
ncclResult_t ncclAllGather(const void *s, void *r, size_t n, ncclDataType_t, ncclComm_t, hipStream_t) {
    memmove(r, s, n);  // one rank
    return ncclSuccess;
}
}  // extern "C"

// ---- kernel launchers: touch exactly what the kernel writes
int rbc_gf_pick_rc(int R, int rcmax) {
    if (R <= 0) return 1;
    if (rcmax < 1) rcmax = 1;
    const int chunks = (R + rcmax - 1) / rcmax;
    return (R + chunks - 1) / chunks;
}
hipError_t rbc_launch_gf_rows(const GfArgs &a, hipStream_t) {
    if (a.count <= 0) return hipSuccess;
    for (int i = 0; i < a.count; ++i) {
        const uint8_t *oi = a.out_idx ? a.out_idx + (size_t)i * a.idx_stride2 : nullptr;
        for (int r = 0; r < a.R; ++r) {
            const uint32_t pos = oi ? oi[r] : (uint32_t)(a.K + r);
            touch(a.out + (size_t)i * a.out_inst_pitch + (size_t)pos * a.out_row_pitch, a.out_row_pitch);
        }
        if (a.in_idx) peek(a.in_idx, (size_t)i * a.idx_stride + (a.K - 1));
        if (a.coef) peek(a.coef, (size_t)i * a.coef_inst_stride + (size_t)a.R * a.K - 1);
    }
    return hipSuccess;
}
hipError_t rbc_launch_gf_regen(const GfArgs &a, hipStream_t st) {
    if (a.count > 0 && !a.rcount) return hipErrorInvalidValue;  // the launcher sets the column tiles itself
    return rbc_launch_gf_rows(a, st);  // same rows written, same inputs read
}
hipError_t rbc_launch_rs_fft(const FftArgs &a, hipStream_t) {
    if (a.count > 0) touch(a.shards, (size_t)a.count * a.inst_pitch);
    if (a.count > 0 && a.join) touch(a.join, (size_t)a.count * a.join_pitch);  // the fused value join
    return hipSuccess;
}
hipError_t rbc_launch_sha_rows(const ShaArgs &a, bool verify, hipStream_t) {
    if (a.count <= 0) return hipSuccess;
    if (a.leaves && !a.list && !a.per_message) touch(a.leaves, (size_t)a.count * a.leaves_inst_pitch);
    if (a.leaves && a.per_message) touch(a.leaves, (size_t)a.count * 32);
    if (verify && a.valid) touch(a.valid, (size_t)a.count * (a.per_message ? 1 : a.n));
    return hipSuccess;
}
hipError_t rbc_launch_sha_rx(const ShaArgs &v, const ShaArgs &r, bool v_walk, hipStream_t, uint4 *zero0, uint4 *zero1) {
    for (uint4 *z : {zero0, zero1})
        if (z) touch(z, sizeof(uint4));
    if (v.count > 0) {
        touch(v.leaves, (size_t)v.count * v.leaves_inst_pitch);
        if (v_walk) touch(v.valid, (size_t)v.count * v.n);
    }
    if (r.count > 0) touch(r.leaves, (size_t)r.count * r.leaves_inst_pitch);
    return hipSuccess;
}
hipError_t rbc_launch_recheck(const RecheckArgs &a, hipStream_t) {
    if (a.count <= 0) return hipSuccess;
    touch(a.status, (size_t)a.count * 4);
    touch(a.need_full, (size_t)a.count);
    return hipSuccess;
}
hipError_t rbc_launch_merkle(const MerkleArgs &a, bool check, hipStream_t) {
    if (a.count <= 0) return hipSuccess;
    if (!check) {
        touch(a.roots, (size_t)a.count * 32);
        touch(a.branches, (size_t)a.count * a.br_inst_pitch);
    } else {
        touch(a.status, (size_t)a.count * 4);
        peek(a.expect_roots, (size_t)a.count * 32 - 1);
    }
    return hipSuccess;
}
hipError_t rbc_launch_merkle_path(const PathArgs &a, hipStream_t) {
    if (a.count > 0) touch(a.valid, (size_t)a.count * a.n);
    return hipSuccess;
}
hipError_t rbc_launch_decode_prepare(const PrepArgs &a, hipStream_t) {
    if (a.count <= 0) return hipSuccess;
    touch(a.used, (size_t)a.count * a.used_stride);
    touch(a.regen, (size_t)a.count * a.regen_stride);
    touch(a.dmat, (size_t)a.count * a.dmat_stride);
    touch(a.status, (size_t)a.count * 4);
    if (a.nmiss) touch(a.nmiss, (size_t)a.count * 4);
    if (a.flags) touch(a.flags, (size_t)a.count * a.n * 4);
    if (a.fft) {
        touch(a.rcount, (size_t)a.count * 4);
        touch(a.cls, (size_t)a.count * a.cls_stride);
    }
    return hipSuccess;
}
hipError_t rbc_launch_digest(const uint8_t *leaves, uint64_t pitch, int k, const int32_t *, uint8_t *digests, int count,
                             hipStream_t, int) {
    if (count <= 0) return hipSuccess;
    peek(leaves, (size_t)(count - 1) * pitch + (size_t)k * 32 - 1);
    touch(digests, (size_t)count * 32);
    return hipSuccess;
}
hipError_t rbc_launch_join(const JoinArgs &a, hipStream_t) {
    if (a.count > 0) touch(a.values, (size_t)a.count * a.value_pitch);
    return hipSuccess;
}
hipError_t rbc_launch_inject_faults(uint8_t *shards, uint64_t inst_pitch, uint32_t row_pitch, const int32_t *corrupt,
                                    int count, hipStream_t) {
    for (int i = 0; i < count; ++i)
        if (corrupt[i] >= 0) shards[(size_t)i * inst_pitch + (size_t)corrupt[i] * row_pitch] ^= 0x5a;
    return hipSuccess;
}
hipError_t rbc_launch_compact_present(const uint8_t *present, int n, int count, uint8_t *valid, uint32_t *list,
                                      uint32_t *counter, hipStream_t, int, const uint8_t *roots_src,
                                      uint8_t *roots_dst) {
    if (count <= 0) return hipSuccess;
    peek(present, (size_t)count * n - 1);
    if (roots_dst) {
        peek(roots_src, (size_t)count * 32 - 1);
        touch(roots_dst, (size_t)count * 32);
    }
    touch(valid, (size_t)count * n);
    touch(list, (size_t)count * n * 4);
    touch(counter, 4);
    return hipSuccess;
}
hipError_t rbc_launch_pack_records(const uint8_t *, const uint8_t *, const int32_t *, int, int slots, uint8_t *out,
                                   hipStream_t) {
    touch(out, (size_t)slots * 64);
    return hipSuccess;
}
hipError_t rbc_launch_fill_random(uint8_t *dst, uint64_t, uint64_t rows, uint64_t pitch, uint64_t, hipStream_t) {
    touch(dst, rows * pitch);
    return hipSuccess;
}
hipError_t rbc_launch_gather_present(const uint8_t *host, uint64_t hpitch, uint32_t S, const uint8_t *present,
                                     uint8_t *dev, uint32_t dpitch, uint32_t rows, hipStream_t) {
    for (uint32_t r = 0; r < rows; ++r) {
        uint8_t *d = dev + (size_t)r * dpitch;
        touch(d, dpitch);
        if (present[r]) memcpy(d, host + (size_t)r * hpitch, S);
    }
    return hipSuccess;
}
hipError_t rbc_launch_gather_values(const uint64_t *ptrs, const uint32_t *lens, uint32_t count, uint8_t *dev,
                                    uint64_t vpitch, hipStream_t) {
    for (uint32_t i = 0; i < count; ++i) {  // whole 16-B chunks up to round_up(len, 16)
        touch(dev + (size_t)i * vpitch, (lens[i] + 15) / 16 * 16);
        memcpy(dev + (size_t)i * vpitch, reinterpret_cast<const void *>(ptrs[i]), lens[i]);
    }
    return hipSuccess;
}
hipError_t rbc_launch_gather_msgs(const uint8_t *host, const uint64_t *offs, const uint32_t *lens, uint32_t count,
                                  uint8_t *dev, uint32_t, hipStream_t) {
    for (uint32_t m = 0; m < count; ++m) {  // the kernel stores whole 16-B chunks up to round_up(len, 16)
        touch(dev + offs[m], (lens[m] + 15) / 16 * 16);
        memcpy(dev + offs[m], host + offs[m], lens[m]);
    }
    return hipSuccess;
}
hipError_t rbc_launch_pack_rows(const uint8_t *src, uint32_t src_pitch, uint8_t *dst, uint32_t dst_pitch,
                                uint32_t width, uint32_t rows, hipStream_t) {
    for (uint32_t r = 0; r < rows; ++r) {  // whole dst rows: zeros past width
        touch(dst + (size_t)r * dst_pitch, dst_pitch);
        memset(dst + (size_t)r * dst_pitch, 0, dst_pitch);
        memcpy(dst + (size_t)r * dst_pitch, src + (size_t)r * src_pitch, width);
    }
    return hipSuccess;
}
hipError_t rbc_launch_gather_ptrs(const uint64_t *ptrs, const uint32_t *lens, uint32_t n, uint8_t *dev,
                                  uint32_t dpitch, uint32_t rows, hipStream_t) {
    for (uint32_t r = 0; r < rows; ++r) {  // whole rows: zeros past lens[r / n] and for absent rows
        uint8_t *d = dev + (size_t)r * dpitch;
        touch(d, dpitch);
        memset(d, 0, dpitch);
        if (ptrs[r]) memcpy(d, reinterpret_cast<const void *>(ptrs[r]), lens[r / n]);
    }
    return hipSuccess;
}
hipError_t rbc_launch_count_mismatch(const uint8_t *, uint64_t, const uint8_t *, uint64_t, uint64_t, uint64_t,
                                     uint32_t *counter, hipStream_t) {
    touch(counter, 4);
    return hipSuccess;
}
hipError_t rbc_launch_count_mismatch_rows(const uint8_t *, uint64_t, uint32_t, int, uint32_t, const uint8_t *,
                                          uint64_t, uint32_t, uint64_t, uint32_t *counter, hipStream_t) {
    touch(counter, 4);
    return hipSuccess;
}
hipError_t rbc_launch_poison_rows(uint8_t *shards, uint64_t inst_pitch, uint32_t, int, const uint8_t *,
                                  const int32_t *, uint64_t count, uint64_t, hipStream_t) {
    touch(shards, count * inst_pitch);
    return hipSuccess;
}
hipError_t rbc_launch_marshal_val(const WireArgs &a, hipStream_t) {
    const size_t msgs = (size_t)a.count * a.n;
    if (msgs) touch(a.out, msgs * a.out_pitch);
    if (msgs && a.out_lens) touch(a.out_lens, msgs * 4);
    return hipSuccess;
}
