// capi.cpp -- C++ host runtime behind include/rbc_gpu.h.
//
// Mirrors, on the host side, the interfaces the reference's rbc package
// binds (rbc/rbc.go:20 `enc reedsolomon.Encoder`, shard/validateMessage/
// interpolate at rbc/rbc.go:86-100) and drives the batched HIP kernels in
// kernels.hip.  Argument checks and error values follow klauspost/reedsolomon
// v1.9.1 (reedsolomon.go: New, Split, Encode, Verify, Reconstruct, Join).
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <limits.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <string.h>

#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/rbc_gpu.h"
#include "../../include/rbc_protocol.h"
#include "gf_host.h"
#include "kernels.h"

namespace {

constexpr size_t kAlign = 64;
inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Rows per GF chunk (accumulators held in VGPRs) of the matrix codec.
constexpr int kGfRcMax = 21;

int tree_width(int n) {
    int w = 1;
    while (w < n) w <<= 1;
    return w;
}
int tree_depth(int n) {
    int w = tree_width(n), d = 0;
    while ((1 << d) < w) ++d;
    return d;
}

#define RBC_HIP(expr)                                  \
    do {                                               \
        hipError_t e_ = (expr);                        \
        if (e_ != hipSuccess) return RBC_ERR_DEVICE;   \
    } while (0)

// growable device / pinned buffer
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    bool pinned = false;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        release();
        size_t want = std::max(bytes, (size_t)256);
        hipError_t e = pinned ? hipHostMalloc(&p, want, hipHostMallocDefault) : hipMalloc(&p, want);
        if (e != hipSuccess) { p = nullptr; cap = 0; return e; }
        cap = want;
        return hipSuccess;
    }
    void release() {
        if (p) {
            if (pinned) (void)hipHostFree(p);
            else (void)hipFree(p);
        }
        p = nullptr;
        cap = 0;
    }
    template <class T> T *as() const { return reinterpret_cast<T *>(p); }
};

// Interpolate's decode workspace and its fork resources (aux stream for the
// value assembly beside the regen hashing).  One per independent stream of
// work: the context's device API has one, every host-API slot has its own.
struct Ws {
    DevBuf used, regen, dmat, nmiss, flags, list, counter, rcount, cls, vleaves, vlist;
    // receive step's node-reuse recheck: the roots each in-flight batch's
    // branches were verified against (two slots: cur and prev), and the
    // instances handed to the full recheck
    DevBuf vroot[2], need_full;
    // receive step's list counters (16 B each): V[2] the compaction of cur,
    // R[2] cur's regen list (decode) / prev's (hashing); parity flips per
    // call.  One lane of the hashing launch zeroes the next users' counters
    // (no memset launches on the receiver stream); v_clean tracks V[] on the host.
    DevBuf rxcnt;
    int rx_par = 0;
    bool rxcnt_init = false, v_clean[2] = {true, true};
    int rx_vslot = 0;           // slot of the pending batch's verified roots
    bool rx_vreuse = false;     // ... kept (the recheck mode when it was verified was REUSE)
    // fork the join onto an aux stream (device API); host-API slots keep one
    // stream each (their concurrency comes from the slots themselves, and
    // the box has GPU_MAX_HW_QUEUES = 4 hardware queues per process)
    bool fork = true;
    int rx_count = 0;           // receive_step: batch decoded by the last call, awaiting its rehash + check
    const uint8_t *rx_shards = nullptr;  // ... and its shard buffer (identity check of `prev`)
    hipStream_t aux = nullptr;  // created on first use
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_hashed = nullptr, ev_rel = nullptr;
    bool init() {
        return hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming) == hipSuccess &&
               hipEventCreateWithFlags(&ev_join, hipEventDisableTiming) == hipSuccess &&
               hipEventCreateWithFlags(&ev_hashed, hipEventDisableTiming) == hipSuccess &&
               hipEventCreateWithFlags(&ev_rel, hipEventDisableTiming) == hipSuccess;
    }
    void release() {
        for (DevBuf *b : {&used, &regen, &dmat, &nmiss, &flags, &list, &counter, &rcount, &cls, &vleaves, &vlist,
                          &vroot[0], &vroot[1], &need_full, &rxcnt})
            b->release();
        if (aux) (void)hipStreamDestroy(aux);
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        if (ev_join) (void)hipEventDestroy(ev_join);
        if (ev_hashed) (void)hipEventDestroy(ev_hashed);
        if (ev_rel) (void)hipEventDestroy(ev_rel);
        aux = nullptr;
        ev_fork = ev_join = ev_hashed = ev_rel = nullptr;
    }
};

// One in-flight host-API submission (the Go batcher's entry points): its own
// stream, device buffers, pinned staging both ways and decode workspace, so
// consecutive batches pipeline -- batch t+1 is staged and its H2D runs while
// batch t computes.  `finish` copies the pinned results into the caller's
// buffers at completion (rbc_wait / rbc_poll / slot reuse).
struct Slot {
    DevBuf d_values, d_shards, d_leaves, d_roots, d_branches, d_valid, d_status, d_digests, d_lens, d_slens, d_idx,
        d_offs, d_present, d_pack;
    DevBuf h_in{nullptr, 0, true}, h_out{nullptr, 0, true};
    Ws ws;
    hipStream_t stream = nullptr;
    hipStream_t dstream = nullptr;  // RBC_D2H_STREAM: the submission's D2H copies, gated on kdone
    hipEvent_t done = nullptr;
    // recorded after the submission's kernels, before its deferred D2H: a
    // waiter enqueues the D2H only once the kernels are done, so the copy
    // engine (one queue, served in enqueue order) never holds a later
    // submission's H2D behind a D2H that still waits on kernels
    hipEvent_t kdone = nullptr;
    uint64_t ticket = 0;
    bool busy = false;
    std::function<int()> finish;
    // Device-to-host copies of a submission, enqueued only when the NEXT
    // submission has enqueued its host-to-device copies (or at wait / poll):
    // the copy engine serves the streams' copies in enqueue order, so a D2H
    // queued at submit time (it waits on this submission's kernels) would hold
    // the next submission's H2D behind it and serialise the slots.
    std::function<int(hipStream_t)> d2h;  // enqueues the D2H copies on the given stream
    int d2h_rc = 0;
    void release() {
        for (DevBuf *b : {&d_values, &d_shards, &d_leaves, &d_roots, &d_branches, &d_valid, &d_status, &d_digests,
                          &d_lens, &d_slens, &d_idx, &d_offs, &d_present, &d_pack, &h_in, &h_out})
            b->release();
        ws.release();
        if (stream) (void)hipStreamDestroy(stream);
        if (dstream) (void)hipStreamDestroy(dstream);
        if (done) (void)hipEventDestroy(done);
        if (kdone) (void)hipEventDestroy(kdone);
        stream = nullptr;
        dstream = nullptr;
        done = nullptr;
        kdone = nullptr;
    }
};

// host-API submissions in flight per context: the batcher keeps 4 launches
// in flight (tools/batcher_bench.cpp), and the box has 4 hardware queues
#ifndef RBC_D2H_STREAM
#define RBC_D2H_STREAM 0
#endif
#ifndef RBC_HOST_SLOTS
#define RBC_HOST_SLOTS 4
#endif
constexpr int kHostSlots = RBC_HOST_SLOTS;

}  // namespace

struct rbc_ctx {
    int n = 0, f = 0, k = 0, p = 0, depth = 0, width = 0, device = 0;
    bool fft = false;              // additive-FFT codec active (rs_fft.hip)
    // wave issue priorities (s_setprio 0..3) of the commit-side kernels
    // (encode, leaves, tree build) and the receive-side ones (verify,
    // interpolate); rbc_ctx_set_wave_priority, default 0
    int tx_prio = 0, rx_prio = 0;
    // interpolate's two GF transforms (missing-data GEMV, FFT re-encode):
    // rbc_ctx_set_decode_priority, default -1 = the commit side's level, like
    // the commit side's own transform
    int gemv_prio_ = -1, reencode_prio_ = -1;
    // the receive step's root recheck: RBC_RECHECK_REUSE (default: over the
    // nodes ECHO verify established) or RBC_RECHECK_FULL (the whole tree)
    int recheck = RBC_RECHECK_REUSE;
    int gemv_prio() const { return gemv_prio_ < 0 ? tx_prio : gemv_prio_; }
    int reencode_prio() const { return reencode_prio_ < 0 ? tx_prio : reencode_prio_; }
    std::vector<uint8_t> h_M;      // n x k encode matrix
    uint8_t *d_M = nullptr;        // device copy; parity rows at d_M + k*k
    std::mutex mu;
    hipStream_t stream = nullptr;  // Encoder-mirror stream (created on first use)
    Ws ws;                         // interpolate workspace of the device API
    // host-API staging
    DevBuf d_values, d_shards, d_leaves, d_roots, d_branches, d_valid, d_status, d_digests, d_lens, d_slens,
        d_idx, d_present;
    DevBuf h_stage{nullptr, 0, true}, h_small{nullptr, 0, true};
    uint64_t next_ticket = 1;
    std::vector<std::unique_ptr<Slot>> slots;        // host-API pipeline
    std::unordered_map<uint64_t, int> retired;       // completed tickets not yet waited on
    // RCCL
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    DevBuf d_pack;
};

struct rbc_rs {
    rbc_ctx *ctx = nullptr;
};

namespace {

int ctx_create_kn(int n, int k, int device, rbc_ctx **out) {
    if (!out) return RBC_ERR_INVALID_ARG;
    *out = nullptr;
    if (k <= 0 || n - k < 0) return RBC_ERR_INV_SHARD_NUM;
    if (n > 256) return RBC_ERR_MAX_SHARD_NUM;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return RBC_ERR_DEVICE;
    rbc_ctx *c = new rbc_ctx();
    c->n = n;
    c->k = k;
    c->p = n - k;
    c->f = (n - k) / 2;
    c->width = tree_width(n);
    c->depth = tree_depth(n);
    c->device = device;
    c->fft = rbc_fft_supported(n, k);
    if (!rbchost::build_matrix(k, n, c->h_M)) { delete c; return RBC_ERR_SINGULAR; }
    // d_M = [n x k encode matrix | exp[512] | log[256]] (tables for decode_prepare_fft)
    std::vector<uint8_t> up(c->h_M);
    {
        const rbchost::Gf g;
        up.insert(up.end(), g.exp, g.exp + 512);
        up.insert(up.end(), g.log, g.log + 256);
    }
    if (hipSetDevice(device) != hipSuccess || hipMalloc(&c->d_M, up.size()) != hipSuccess ||
        hipMemcpy(c->d_M, up.data(), up.size(), hipMemcpyHostToDevice) != hipSuccess ||
        !c->ws.init()) {
        if (c->d_M) (void)hipFree(c->d_M);
        delete c;
        return RBC_ERR_DEVICE;
    }
    *out = c;
    return RBC_OK;
}

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// The context's own streams are created on first use (caller holds c->mu):
// a device-API caller that brings its own streams never spends hardware
// queues on them (GPU_MAX_HW_QUEUES is 4; streams beyond that share a queue
// and serialise).
hipStream_t host_stream(rbc_ctx *c) {
    if (!c->stream && hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) c->stream = nullptr;
    return c->stream;
}
hipStream_t aux_stream(Ws &w) {
    if (!w.aux && hipStreamCreateWithFlags(&w.aux, hipStreamNonBlocking) != hipSuccess) w.aux = nullptr;
    return w.aux;
}

// ------------------------------------------------------------ stage bodies
int stage_encode(rbc_ctx *c, hipStream_t st, int count, const uint8_t *values, uint64_t value_pitch,
                 const uint32_t *value_lens, uint32_t uniform_value_len, uint8_t *shards, uint32_t shard_pitch) {
    if (count < 0 || (count > 0 && (!values || !shards))) return RBC_ERR_INVALID_ARG;
    if (shard_pitch == 0 || shard_pitch % kAlign) return RBC_ERR_INVALID_ARG;
    if (!value_lens) {
        if (uniform_value_len == 0) return RBC_ERR_SHORT_DATA;
        const size_t S = (uniform_value_len + c->k - 1) / c->k;
        if (S > shard_pitch || value_pitch < round_up((size_t)c->k * S, 16) + 16) return RBC_ERR_INVALID_ARG;
    }
    if (value_pitch > 0x7fffffffULL || (uint64_t)c->n * shard_pitch > 0x7fffffffULL) return RBC_ERR_INVALID_ARG;
    if (count == 0) return RBC_OK;
    if (c->fft) {
        FftArgs a{};
        a.count = count;
        a.n = c->n;
        a.k = c->k;
        a.mode = GF_MODE_ENCODE;
        a.values = values;
        a.value_pitch = (uint32_t)value_pitch;
        a.shards = shards;
        a.inst_pitch = (uint64_t)c->n * shard_pitch;
        a.row_pitch = shard_pitch;
        a.lens = value_lens;
        a.uniform_len = uniform_value_len;
        a.prio = c->tx_prio;
        RBC_HIP(rbc_launch_rs_fft(a, st));
        return RBC_OK;
    }
    GfArgs g{};
    g.count = count;
    g.tiles = (int)((shard_pitch + 4095) / 4096);
    g.R = c->p;
    g.K = c->k;
    g.rc = rbc_gf_pick_rc(c->p > 0 ? c->p : 1, kGfRcMax);
    g.mode = GF_MODE_ENCODE;
    g.in = values;
    g.in_inst_pitch = value_pitch;
    g.in_inst_bytes = (uint32_t)value_pitch;
    g.out = shards;
    g.out_inst_pitch = (uint64_t)c->n * shard_pitch;
    g.out_row_pitch = shard_pitch;
    g.copy = shards;
    g.lens = value_lens;
    g.uniform_len = uniform_value_len;
    g.coef = c->d_M + (size_t)c->k * c->k;
    g.coef_inst_stride = 0;
    g.prio = c->tx_prio;
    RBC_HIP(rbc_launch_gf_rows(g, st));
    return RBC_OK;
}

int stage_leaves(rbc_ctx *c, hipStream_t st, int count, const uint8_t *shards, uint32_t shard_pitch,
                 const uint32_t *shard_lens, uint32_t uniform_shard_len, uint8_t *leaves) {
    if (count < 0 || (count > 0 && (!shards || !leaves))) return RBC_ERR_INVALID_ARG;
    if (shard_pitch % kAlign || (!shard_lens && (uniform_shard_len == 0 || uniform_shard_len > shard_pitch)))
        return RBC_ERR_INVALID_ARG;
    if (count == 0) return RBC_OK;
    ShaArgs a{};
    a.count = count;
    a.rows_per_inst = c->n;
    a.rows = shards;
    a.inst_pitch = (uint64_t)c->n * shard_pitch;
    a.row_pitch = shard_pitch;
    a.lens = shard_lens;
    a.uniform_len = uniform_shard_len;
    a.leaves = leaves;
    a.leaves_inst_pitch = (uint64_t)c->n * 32;
    a.n = c->n;
    a.depth = c->depth;
    a.prio = c->tx_prio;
    RBC_HIP(rbc_launch_sha_rows(a, false, st));
    return RBC_OK;
}

int stage_merkle_build(rbc_ctx *c, hipStream_t st, int count, const uint8_t *leaves, uint8_t *roots,
                       uint8_t *branches) {
    if (count < 0 || (count > 0 && (!leaves || !roots))) return RBC_ERR_INVALID_ARG;
    if (count == 0) return RBC_OK;
    MerkleArgs m{};
    m.count = count;
    m.n = c->n;
    m.width = c->width;
    m.depth = c->depth;
    m.k = c->k;
    m.leaves = leaves;
    m.leaves_inst_pitch = (uint64_t)c->n * 32;
    m.roots = roots;
    m.branches = c->depth > 0 ? branches : nullptr;
    m.br_inst_pitch = (uint64_t)c->n * c->depth * 32;
    m.prio = c->tx_prio;
    RBC_HIP(rbc_launch_merkle(m, false, st));
    return RBC_OK;
}

// ECHO verify's form: leaf hashes + the shared-path verify
// (merkle_path_kernel) where the per-leaf walk's 2d compressions per row are a
// real share of the leaf's ceil((S+9)/64) -- C4: 16 vs 13 -- and the per-leaf
// walk fused into the row hashing where they are not (C2: 14 vs 373).
static bool shared_path_verify(const rbc_ctx *c, const uint32_t *shard_lens, uint32_t uniform_shard_len) {
    const uint32_t blocks_per_row = shard_lens ? 0u : (uniform_shard_len + 9 + 63) / 64;
    return (shard_lens || 16u * (uint32_t)c->depth >= blocks_per_row) && c->depth >= 1 && c->width <= 256;
}

// wsp: a host-API slot's own workspace (its submission already holds c->mu);
// NULL: the context's, guarded by c->mu here (device API)
int stage_verify(rbc_ctx *c, hipStream_t st, int count, const uint8_t *shards, uint32_t shard_pitch,
                 const uint32_t *shard_lens, uint32_t uniform_shard_len, const uint8_t *branches,
                 const uint8_t *roots, const uint8_t *present, uint8_t *valid, uint8_t *leaves, Ws *wsp = nullptr) {
    if (count < 0 || (count > 0 && (!shards || !roots || !valid || (c->depth > 0 && !branches))))
        return RBC_ERR_INVALID_ARG;
    if (shard_pitch % kAlign || (!shard_lens && (uniform_shard_len == 0 || uniform_shard_len > shard_pitch)))
        return RBC_ERR_INVALID_ARG;
    if (count == 0) return RBC_OK;
    ShaArgs a{};
    a.count = count;
    a.rows_per_inst = c->n;
    a.rows = shards;
    a.inst_pitch = (uint64_t)c->n * shard_pitch;
    a.row_pitch = shard_pitch;
    a.lens = shard_lens;
    a.uniform_len = uniform_shard_len;
    a.leaves = leaves;
    a.leaves_inst_pitch = (uint64_t)c->n * 32;
    a.n = c->n;
    a.depth = c->depth;
    a.branches = branches;
    a.br_inst_pitch = (uint64_t)c->n * c->depth * 32;
    a.roots = roots;
    a.present = present;
    a.valid = valid;
    a.prio = c->rx_prio;
    // Shared-path verification: leaves, then one hash per
    // distinct branch-walk input.
    // The per-leaf walk costs 2d compressions per row on top of the leaf's
    // ceil((S+9)/64); the shared-path form pays off where that walk is a real
    // share (C4: 16 vs 13) and only adds a launch where it is not (C2: 14 vs
    // 373, measured equal alone and slower beside a second stream).
    const bool path_pays = shared_path_verify(c, shard_lens, uniform_shard_len);
    // Only the received ECHOs are validated (validateMessage runs per message):
    // with a present mask the shards to hash are compacted into a device list
    // first (N-f of N in the bench: a third fewer SHA rows than hashing all N).
    if (present && c->n <= 256) {
        uint32_t *vl = nullptr, *vc = nullptr;
        {
            std::unique_lock<std::mutex> lk(c->mu, std::defer_lock);
            if (!wsp) lk.lock();
            Ws &w = wsp ? *wsp : c->ws;
            RBC_HIP(w.vlist.ensure((size_t)count * c->n * 4 + 64));
            vl = w.vlist.as<uint32_t>();
            vc = vl + (size_t)count * c->n;
        }
        RBC_HIP(hipMemsetAsync(vc, 0, 4, st));
        RBC_HIP(rbc_launch_compact_present(present, c->n, count, valid, vl, vc, st, c->rx_prio));
        a.list = vl;
        a.list_count = vc;
    }
    if (path_pays) {
        uint8_t *lv = leaves;
        if (!lv) {
            std::unique_lock<std::mutex> lk(c->mu, std::defer_lock);
            if (!wsp) lk.lock();
            Ws &w = wsp ? *wsp : c->ws;
            RBC_HIP(w.vleaves.ensure((size_t)count * c->n * 32));
            lv = w.vleaves.as<uint8_t>();
        }
        a.leaves = lv;
        RBC_HIP(rbc_launch_sha_rows(a, false, st));
        PathArgs p{};
        p.count = count;
        p.n = c->n;
        p.width = c->width;
        p.lg_width = c->depth;
        p.depth = c->depth;
        p.leaves = lv;
        p.leaves_inst_pitch = (uint64_t)c->n * 32;
        p.branches = branches;
        p.br_inst_pitch = (uint64_t)c->n * c->depth * 32;
        p.roots = roots;
        p.present = present;
        p.valid = valid;
        p.prio = c->rx_prio;
        RBC_HIP(rbc_launch_merkle_path(p, st));
        return RBC_OK;
    }
    RBC_HIP(rbc_launch_sha_rows(a, true, st));
    return RBC_OK;
}

int ensure_ws(rbc_ctx *c, Ws &w, int count) {
    const size_t nr = (size_t)std::max(c->n - c->k, 1);
    RBC_HIP(w.used.ensure((size_t)count * c->k));
    RBC_HIP(w.regen.ensure((size_t)count * nr));
    RBC_HIP(w.dmat.ensure((size_t)count * nr * c->k));
    RBC_HIP(w.nmiss.ensure((size_t)count * 4));
    RBC_HIP(w.flags.ensure((size_t)count * c->n * 4));
    RBC_HIP(w.list.ensure((size_t)count * nr * 4));
    RBC_HIP(w.counter.ensure(16));
    RBC_HIP(w.rcount.ensure((size_t)count * 4));
    RBC_HIP(w.cls.ensure((size_t)count * round_up(c->n, 4)));
    return RBC_OK;
}

// decode_prepare + GF regeneration (in place), no hashing
// compare != 0: valid-but-unused rows are compared, not blindly rewritten,
// and the rows that need hashing are collected in ws_list
// values_out (optional): interpolate's joined value, assembled by the FFT
// re-encode from the data rows it loads (no separate join pass) where that
// applies -- the FFT codec, uniform S, a value row at most 256 B longer than
// k*S; *joined tells the caller whether it happened
// The FFT decode joins the value itself only for rows of at least this many
// bytes.  Short rows (C4: 763 B, 86 unaligned row stores per lane in the
// 256-VGPR decode) join faster as join_kernel on the receive step's aux
// stream, beside the recheck: C4 349 -> 361 GB/s, while C1 / C2 lose 4 % that
// way (profiles/r06am/).
constexpr uint32_t kFusedJoinMinS = 2048;
int stage_regenerate(rbc_ctx *c, Ws &w, hipStream_t st, int count, uint8_t *shards, uint32_t shard_pitch,
                     const uint32_t *shard_lens, uint32_t uniform_shard_len, const uint8_t *valid,
                     int32_t *status, int compare = 0, uint32_t *zeroed_counter = nullptr,
                     uint8_t *values_out = nullptr, uint32_t value_pitch = 0, bool *joined = nullptr) {
    if (joined) *joined = false;
    int rc = ensure_ws(c, w, count);
    if (rc) return rc;
    // the regen list's counter: the workspace's own (zeroed here), or one the
    // caller's stream has already zeroed (the receive step's R[])
    uint32_t *counter = zeroed_counter ? zeroed_counter : w.counter.as<uint32_t>();
    if (compare && !zeroed_counter) RBC_HIP(hipMemsetAsync(counter, 0, 16, st));
    const int nr = c->n - c->k;
    PrepArgs pa{};
    pa.count = count;
    pa.n = c->n;
    pa.k = c->k;
    pa.valid = valid;
    pa.valid_stride = (uint32_t)c->n;
    pa.M = c->d_M;
    pa.used = w.used.as<uint8_t>();
    pa.used_stride = (uint32_t)c->k;
    pa.regen = w.regen.as<uint8_t>();
    pa.regen_stride = (uint32_t)std::max(nr, 1);
    pa.dmat = w.dmat.as<uint8_t>();
    pa.dmat_stride = (uint64_t)std::max(nr, 1) * c->k;
    pa.status = status;
    pa.prio = c->rx_prio;
    if (compare) {
        pa.nmiss = w.nmiss.as<int32_t>();
        pa.flags = w.flags.as<uint32_t>();
        pa.list = w.list.as<uint32_t>();
        pa.counter = counter;
    }
    if (c->fft) {
        pa.fft = 1;
        pa.rcount = w.rcount.as<int32_t>();
        pa.cls = w.cls.as<uint8_t>();
        pa.cls_stride = (uint32_t)round_up(c->n, 4);
        pa.gf_exp = c->d_M + c->h_M.size();
        pa.gf_log = pa.gf_exp + 512;
    }
    RBC_HIP(rbc_launch_decode_prepare(pa, st));
    if (c->fft && nr > 0) {
        // 1) missing data rows: D (rcount[i] x k, per instance) times the used rows
        const int rmax = std::min(c->k, nr);
        GfArgs g{};
        g.count = count;
        g.R = rmax;
        g.K = c->k;
        // gf_regen_kernel's column tiles and block shape: rbc_launch_gf_regen (gf_regen.hip)
        g.mode = GF_MODE_DECODE;
        g.in = shards;
        g.in_inst_pitch = (uint64_t)c->n * shard_pitch;
        g.in_row_pitch = shard_pitch;
        g.in_inst_bytes = (uint32_t)((uint64_t)c->n * shard_pitch);
        g.out = shards;
        g.out_inst_pitch = (uint64_t)c->n * shard_pitch;
        g.out_row_pitch = shard_pitch;
        g.lens = shard_lens;
        g.uniform_len = uniform_shard_len;
        g.coef = pa.dmat;
        g.coef_inst_stride = pa.dmat_stride;
        g.in_idx = pa.used;
        g.out_idx = pa.regen;
        g.idx_stride = pa.used_stride;
        g.idx_stride2 = pa.regen_stride;
        g.status = status;
        g.rcount = pa.rcount;
        g.prio = c->gemv_prio();
        RBC_HIP(rbc_launch_gf_regen(g, st));
        // 2) parity positions: additive-FFT re-encode of the completed data half
        FftArgs a{};
        a.count = count;
        a.n = c->n;
        a.k = c->k;
        a.mode = GF_MODE_DECODE;
        a.shards = shards;
        a.inst_pitch = (uint64_t)c->n * shard_pitch;
        a.row_pitch = shard_pitch;
        a.lens = shard_lens;
        a.uniform_len = uniform_shard_len;
        a.status = status;
        a.cls = pa.cls;
        a.cls_stride = pa.cls_stride;
        if (compare) {
            a.flags = pa.flags;
            a.list = pa.list;
            a.counter = pa.counter;
        }
        a.prio = c->reencode_prio();
        // tile 0's lanes zero the value's tail, 4 B each, and only the lanes
        // with a column inside the row pitch run (rs_fft.hip): the tail must
        // fit min(256, shard_pitch) bytes, else the separate join zero-fills it
        if (values_out && joined && !shard_lens && uniform_shard_len >= kFusedJoinMinS &&
            value_pitch >= (uint64_t)c->k * uniform_shard_len &&
            value_pitch - (uint64_t)c->k * uniform_shard_len <= std::min<uint64_t>(256, shard_pitch)) {
            a.join = values_out;
            a.join_pitch = value_pitch;
            *joined = true;
        }
        RBC_HIP(rbc_launch_rs_fft(a, st));
    } else if (nr > 0) {
        GfArgs g{};
        g.count = count;
        g.tiles = (int)((shard_pitch + 4095) / 4096);
        g.R = nr;
        g.K = c->k;
        g.rc = rbc_gf_pick_rc(nr, kGfRcMax);
        g.mode = GF_MODE_DECODE;
        g.in = shards;
        g.in_inst_pitch = (uint64_t)c->n * shard_pitch;
        g.in_row_pitch = shard_pitch;
        g.in_inst_bytes = (uint32_t)((uint64_t)c->n * shard_pitch);
        g.out = shards;
        g.out_inst_pitch = (uint64_t)c->n * shard_pitch;
        g.out_row_pitch = shard_pitch;
        g.copy = nullptr;
        g.lens = shard_lens;
        g.uniform_len = uniform_shard_len;
        g.coef = pa.dmat;
        g.coef_inst_stride = pa.dmat_stride;
        g.in_idx = pa.used;
        g.out_idx = pa.regen;
        g.idx_stride = pa.used_stride;
        g.idx_stride2 = pa.regen_stride;
        g.status = status;
        if (compare) {
            g.nmiss = pa.nmiss;
            g.flags = pa.flags;
            g.list = pa.list;
            g.counter = pa.counter;
            g.n = c->n;
        }
        g.prio = c->reencode_prio();  // the matrix codec's one decode product
        RBC_HIP(rbc_launch_gf_rows(g, st));
    }
    return RBC_OK;
}

// On every exit after work was forked onto the aux stream, `st` waits for it,
// so a failing later launch never leaves the forked outputs unordered with
// the caller's stream.
struct JoinBack {
    Ws &w;
    hipStream_t st;
    bool armed = false;
    ~JoinBack() {
        if (!armed) return;
        (void)hipEventRecord(w.ev_join, w.aux);
        (void)hipStreamWaitEvent(st, w.ev_join, 0);
    }
};

int launch_join(rbc_ctx *c, hipStream_t js, int count, const uint8_t *shards, uint32_t shard_pitch,
                const uint32_t *shard_lens, uint32_t uniform_shard_len, uint8_t *values_out, uint32_t value_pitch,
                const int32_t *status) {
    JoinArgs j{};
    j.count = count;
    j.k = c->k;
    j.chunks = value_pitch / 16;
    j.shards = shards;
    j.inst_pitch = (uint64_t)c->n * shard_pitch;
    j.row_pitch = shard_pitch;
    j.inst_bytes = (uint32_t)((uint64_t)c->n * shard_pitch);
    j.lens = shard_lens;
    j.uniform_len = uniform_shard_len;
    j.values = values_out;
    j.value_pitch = value_pitch;
    j.status = status;
    j.prio = c->rx_prio;
    RBC_HIP(rbc_launch_join(j, js));
    return RBC_OK;
}

// interpolate: decode (prepare, missing-data GF, FFT re-encode + compare),
// value join, rehash of the regenerated rows, Merkle root recheck + batch
// digest.  values_out == NULL is the row-view form: no join, the value is the
// k data rows of `shards` (regenerated in place).  With w.fork the join
// (HBM-bound) runs on the aux stream beside the rehash (latency-bound, it
// under-fills the SIMDs) and the digest beside the recheck.
int stage_interpolate(rbc_ctx *c, Ws &w, hipStream_t st, int count, uint8_t *shards, uint32_t shard_pitch,
                      const uint32_t *shard_lens, uint32_t uniform_shard_len, const uint8_t *valid, uint8_t *leaves,
                      int leaves_verified, const uint8_t *roots, uint8_t *values_out, uint32_t value_pitch,
                      uint8_t *digests, int32_t *status) {
    if (count < 0 || (count > 0 && (!shards || !valid || !leaves || !roots || !status)))
        return RBC_ERR_INVALID_ARG;
    if (shard_pitch % kAlign || (values_out && value_pitch % 16)) return RBC_ERR_INVALID_ARG;
    if (!shard_lens && (uniform_shard_len == 0 || uniform_shard_len > shard_pitch ||
                        (values_out && value_pitch < (uint64_t)uniform_shard_len * c->k)))
        return RBC_ERR_INVALID_ARG;
    if ((uint64_t)c->n * shard_pitch > 0x7fffffffULL) return RBC_ERR_INVALID_ARG;
    if (count == 0) return RBC_OK;
    bool joined = false;
    int rc = stage_regenerate(c, w, st, count, shards, shard_pitch, shard_lens, uniform_shard_len, valid, status,
                              leaves_verified, nullptr, values_out, value_pitch, &joined);
    if (rc) return rc;
    JoinBack jb{w, st};
    if (w.fork && (values_out || digests) && !aux_stream(w)) return RBC_ERR_DEVICE;
    if (values_out && !joined) {
        hipStream_t js = st;
        if (w.fork) {
            RBC_HIP(hipEventRecord(w.ev_fork, st));
            RBC_HIP(hipStreamWaitEvent(w.aux, w.ev_fork, 0));
            jb.armed = true;
            js = w.aux;
        }
        rc = launch_join(c, js, count, shards, shard_pitch, shard_lens, uniform_shard_len, values_out, value_pitch,
                         status);
        if (rc) return rc;
    }
    const int nr = c->n - c->k;
    ShaArgs a{};
    a.count = count;
    a.rows = shards;
    a.inst_pitch = (uint64_t)c->n * shard_pitch;
    a.row_pitch = shard_pitch;
    a.lens = shard_lens;
    a.uniform_len = uniform_shard_len;
    a.status = status;
    a.leaves = leaves;
    a.leaves_inst_pitch = (uint64_t)c->n * 32;
    a.n = c->n;
    a.depth = c->depth;
    a.prio = c->rx_prio;
    if (leaves_verified) {
        // hash only the rows in the device-built list: every missing position
        // plus any valid-but-unused shard the re-encoding disagreed with
        a.rows_per_inst = nr;  // grid bound (count * nr entries at most)
        a.list = w.list.as<uint32_t>();
        a.list_count = w.counter.as<uint32_t>();
    } else {
        a.rows_per_inst = c->n;
    }
    if (a.rows_per_inst > 0) RBC_HIP(rbc_launch_sha_rows(a, false, st));
    MerkleArgs m{};
    m.count = count;
    m.n = c->n;
    m.width = c->width;
    m.depth = c->depth;
    m.k = c->k;
    m.leaves = leaves;
    m.leaves_inst_pitch = (uint64_t)c->n * 32;
    m.expect_roots = roots;
    m.status = status;
    m.prio = c->rx_prio;
    // the batch digest (one serial 23-compression chain per instance at C2)
    // needs only the data leaves: it runs on the aux stream beside the recheck
    hipStream_t ds = st;
    if (w.fork && digests) {
        RBC_HIP(hipEventRecord(w.ev_hashed, st));
        RBC_HIP(hipStreamWaitEvent(w.aux, w.ev_hashed, 0));
        jb.armed = true;
        ds = w.aux;
    }
    RBC_HIP(rbc_launch_merkle(m, true, st));
    if (digests)
        RBC_HIP(rbc_launch_digest(leaves, (uint64_t)c->n * 32, c->k, status, digests, count, ds, c->rx_prio));
    return RBC_OK;  // jb joins the aux stream back
}

// Pipelined receiver (rbc_dev_receive_step): cur's ECHO verify and prev's
// regen hashing share one SHA launch; prev's recheck + digest follow, then
// cur's decode.  The value join of cur runs on the aux stream and is waited
// for by the next call (with prev's digest), so a batch is final when the
// call that names it `prev` has run.
int check_rx_batch(rbc_ctx *c, const rbc_rx_batch *b) {
    if (b->count < 0) return RBC_ERR_INVALID_ARG;
    if (b->count == 0) return RBC_OK;
    if (!b->shards || !b->roots || !b->valid || !b->leaves || !b->status || (c->depth > 0 && !b->branches))
        return RBC_ERR_INVALID_ARG;
    if (b->shard_pitch % kAlign || (b->values_out && b->value_pitch % 16)) return RBC_ERR_INVALID_ARG;
    if (!b->shard_lens && (b->uniform_shard_len == 0 || b->uniform_shard_len > b->shard_pitch ||
                           (b->values_out && b->value_pitch < (uint64_t)b->uniform_shard_len * c->k)))
        return RBC_ERR_INVALID_ARG;
    if ((uint64_t)c->n * b->shard_pitch > 0x7fffffffULL) return RBC_ERR_INVALID_ARG;
    return RBC_OK;
}

// cur and prev are both in flight during a call: no output buffer may be shared
bool rx_alias(const rbc_rx_batch *a, const rbc_rx_batch *b) {
    auto same = [](const void *x, const void *y) { return x && x == y; };
    return same(a->shards, b->shards) || same(a->leaves, b->leaves) || same(a->status, b->status) ||
           same(a->valid, b->valid) || same(a->values_out, b->values_out) || same(a->digests, b->digests);
}

int stage_receive_step(rbc_ctx *c, hipStream_t st, const rbc_rx_batch *cur, const rbc_rx_batch *prev,
                       const rbc_rx_marks *marks) {
    Ws &w = c->ws;
    int rc;
    if (cur && (rc = check_rx_batch(c, cur))) return rc;
    if (prev && (rc = check_rx_batch(c, prev))) return rc;
    const bool hc = cur && cur->count > 0, hp = prev && prev->count > 0;
    // prev must be the batch whose decode the previous call left in the workspace
    if (hp != (w.rx_count > 0) || (hp && (prev->count != w.rx_count || prev->shards != w.rx_shards)))
        return RBC_ERR_INVALID_ARG;
    if (hc && hp && rx_alias(cur, prev)) return RBC_ERR_INVALID_ARG;
    if (!hc && !hp) return RBC_OK;
    if (!aux_stream(w)) return RBC_ERR_DEVICE;
    const int nr = c->n - c->k;
    ShaArgs v{}, r{};
    v.prio = c->rx_prio;  // the launch's wave priority (also when only prev's rows are hashed)
    bool v_walk = false, v_path = false;
    // list counters: cur's compaction V[par], cur's regen list R[par], prev's
    // regen list R[par ^ 1] (its decode ran in the previous call, whose parity
    // was par ^ 1); the hashing launch zeroes R[par] and V[par ^ 1]
    RBC_HIP(w.rxcnt.ensure(64));
    if (!w.rxcnt_init) {
        RBC_HIP(hipMemsetAsync(w.rxcnt.p, 0, 64, st));
        w.rxcnt_init = true;
        w.v_clean[0] = w.v_clean[1] = true;
    }
    const int par = w.rx_par;
    uint32_t *cnt = w.rxcnt.as<uint32_t>();
    uint32_t *v_cnt = cnt + 4 * par, *v_next = cnt + 4 * (par ^ 1), *r_cnt = cnt + 8 + 4 * par,
             *r_prev = cnt + 8 + 4 * (par ^ 1);
    // node-reuse recheck (merkle_recheck_kernel): keep the roots cur's branches
    // are verified against now, for cur's recheck in the next call
    const bool reuse = c->recheck == RBC_RECHECK_REUSE && c->depth >= 1 && c->width <= 256;
    const int cur_vslot = w.rx_vslot ^ (hp ? 1 : 0);
    bool roots_kept = false;
    if (hc && reuse) RBC_HIP(w.vroot[cur_vslot].ensure((size_t)cur->count * 32));
    const bool hv = hc && !cur->verified;  // cur's ECHOs still to verify in this step
    if (hv) {
        v.count = cur->count;
        v.rows_per_inst = c->n;
        v.rows = cur->shards;
        v.inst_pitch = (uint64_t)c->n * cur->shard_pitch;
        v.row_pitch = cur->shard_pitch;
        v.lens = cur->shard_lens;
        v.uniform_len = cur->uniform_shard_len;
        v.leaves = cur->leaves;
        v.leaves_inst_pitch = (uint64_t)c->n * 32;
        v.n = c->n;
        v.depth = c->depth;
        v.branches = cur->branches;
        v.br_inst_pitch = (uint64_t)c->n * c->depth * 32;
        v.roots = cur->roots;
        v.present = cur->present;
        v.valid = cur->valid;
        if (cur->present && c->n <= 256) {  // hash only the received shards (stage_verify)
            RBC_HIP(w.vlist.ensure((size_t)cur->count * c->n * 4 + 64));
            uint32_t *vl = w.vlist.as<uint32_t>();
            if (!w.v_clean[par]) RBC_HIP(hipMemsetAsync(v_cnt, 0, 4, st));  // after an error or a one-shot call
            RBC_HIP(rbc_launch_compact_present(cur->present, c->n, cur->count, cur->valid, vl, v_cnt, st, c->rx_prio,
                                               reuse ? cur->roots : nullptr,
                                               reuse ? w.vroot[cur_vslot].as<uint8_t>() : nullptr));
            w.v_clean[par] = false;
            roots_kept = reuse;
            v.list = vl;
            v.list_count = v_cnt;
        }
        // the shared-path verify where the branch walk is a real share (C4), as stage_verify
        v_path = shared_path_verify(c, cur->shard_lens, cur->uniform_shard_len);
        v_walk = !v_path;
    }
    if (hp && nr > 0) {
        r.count = prev->count;
        r.rows_per_inst = nr;
        r.rows = prev->shards;
        r.inst_pitch = (uint64_t)c->n * prev->shard_pitch;
        r.row_pitch = prev->shard_pitch;
        r.lens = prev->shard_lens;
        r.uniform_len = prev->uniform_shard_len;
        r.status = prev->status;
        r.leaves = prev->leaves;
        r.leaves_inst_pitch = (uint64_t)c->n * 32;
        r.list = w.list.as<uint32_t>();
        r.list_count = r_prev;
    }
    if (hc && reuse && !roots_kept)  // no compaction to carry the copy
        RBC_HIP(hipMemcpyAsync(w.vroot[cur_vslot].p, cur->roots, (size_t)cur->count * 32, hipMemcpyDeviceToDevice, st));
    if (marks && marks->hash_begin) RBC_HIP(hipEventRecord((hipEvent_t)marks->hash_begin, st));
    // (a verified cur leaves only prev's regen rows; with neither side the
    // launch still zeroes the next users' counters)
    RBC_HIP(rbc_launch_sha_rx(v, r, v_walk, st, reinterpret_cast<uint4 *>(r_cnt), reinterpret_cast<uint4 *>(v_next)));
    w.v_clean[par ^ 1] = true;
    if (marks && marks->rows_hashed) RBC_HIP(hipEventRecord((hipEvent_t)marks->rows_hashed, st));
    if (hv && v_path) {
        PathArgs p{};
        p.count = cur->count;
        p.n = c->n;
        p.width = c->width;
        p.lg_width = c->depth;
        p.depth = c->depth;
        p.leaves = cur->leaves;
        p.leaves_inst_pitch = (uint64_t)c->n * 32;
        p.branches = cur->branches;
        p.br_inst_pitch = (uint64_t)c->n * c->depth * 32;
        p.roots = cur->roots;
        p.present = cur->present;
        p.valid = cur->valid;
        p.prio = c->rx_prio;
        RBC_HIP(rbc_launch_merkle_path(p, st));
    }
    if (marks && marks->hashed) RBC_HIP(hipEventRecord((hipEvent_t)marks->hashed, st));
    // From here on prev's aux-stream work (its join from the previous call and
    // its digest) is joined back into `st` on every exit, errors included.
    struct PrevJoin {
        Ws &w;
        hipStream_t st;
        bool armed = false;
        ~PrevJoin() {
            if (armed) (void)hipStreamWaitEvent(st, w.ev_join, 0);
        }
    } pj{w, st};
    if (hp) {
        if (prev->digests) {  // beside the recheck, on the aux stream (after prev's join)
            RBC_HIP(hipEventRecord(w.ev_hashed, st));
            RBC_HIP(hipStreamWaitEvent(w.aux, w.ev_hashed, 0));
            RBC_HIP(rbc_launch_digest(prev->leaves, (uint64_t)c->n * 32, c->k, prev->status, prev->digests,
                                      prev->count, w.aux, c->rx_prio));
        }
        RBC_HIP(hipEventRecord(w.ev_join, w.aux));  // prev's join (+ digest) done
        pj.armed = true;
        MerkleArgs m{};
        m.count = prev->count;
        m.n = c->n;
        m.width = c->width;
        m.depth = c->depth;
        m.k = c->k;
        m.leaves = prev->leaves;
        m.leaves_inst_pitch = (uint64_t)c->n * 32;
        m.expect_roots = prev->roots;
        m.status = prev->status;
        m.prio = c->rx_prio;
        if (reuse && w.rx_vreuse) {
            // the nodes inside the valid-free subtrees only; an instance whose
            // decode changed a valid row goes on to the full recheck (m.only)
            RBC_HIP(w.need_full.ensure((size_t)prev->count));
            RecheckArgs ra{};
            ra.count = prev->count;
            ra.n = c->n;
            ra.width = c->width;
            ra.depth = c->depth;
            ra.leaves = prev->leaves;
            ra.leaves_inst_pitch = (uint64_t)c->n * 32;
            ra.branches = prev->branches;
            ra.br_inst_pitch = (uint64_t)c->n * c->depth * 32;
            ra.valid = prev->valid;
            ra.flags = w.flags.as<uint32_t>();
            ra.vroots = w.vroot[w.rx_vslot].as<uint8_t>();
            ra.expect_roots = prev->roots;
            ra.status = prev->status;
            ra.need_full = w.need_full.as<uint8_t>();
            ra.prio = c->rx_prio;
            RBC_HIP(rbc_launch_recheck(ra, st));
            m.only = ra.need_full;
        }
        RBC_HIP(rbc_launch_merkle(m, true, st));
        if (marks && marks->prev_released) {
            // the recheck was the last reader of prev's set on `st`; the aux
            // stream already holds prev's join and digest: the mark completes
            // after all three, and `st` goes on to cur's decode without waiting
            RBC_HIP(hipEventRecord(w.ev_rel, st));
            RBC_HIP(hipStreamWaitEvent(w.aux, w.ev_rel, 0));
            RBC_HIP(hipEventRecord((hipEvent_t)marks->prev_released, w.aux));
        }
    }
    w.rx_count = 0;  // prev is complete once this call's work on `st` is; cur is pending only on success
    if (hc) {
        if (marks && marks->decode_begin) RBC_HIP(hipEventRecord((hipEvent_t)marks->decode_begin, st));
        bool joined = false;
        rc = stage_regenerate(c, w, st, cur->count, cur->shards, cur->shard_pitch, cur->shard_lens,
                              cur->uniform_shard_len, cur->valid, cur->status, 1, r_cnt, cur->values_out,
                              cur->value_pitch, &joined);
        if (rc) return rc;
        if (marks && marks->decoded) RBC_HIP(hipEventRecord((hipEvent_t)marks->decoded, st));
        if (cur->values_out && !joined) {  // the row view (values_out NULL) has no join; the FFT decode joins
            RBC_HIP(hipEventRecord(w.ev_fork, st));
            RBC_HIP(hipStreamWaitEvent(w.aux, w.ev_fork, 0));
            rc = launch_join(c, w.aux, cur->count, cur->shards, cur->shard_pitch, cur->shard_lens,
                             cur->uniform_shard_len, cur->values_out, cur->value_pitch, cur->status);
            if (rc) return rc;
        }
        w.rx_count = cur->count;
        w.rx_shards = cur->shards;
        w.rx_vslot = cur_vslot;
        w.rx_vreuse = reuse;  // its verified roots were kept
    }
    w.rx_par ^= 1;  // the next call reads R[par] (cur's regen list) as its prev's
    return RBC_OK;  // pj: `st` waits for prev's join + digest
}

// klauspost checkShards / shardSize (reedsolomon.go)
int check_shards(const size_t *lens, int n, bool nilok, size_t *size_out) {
    size_t size = 0;
    for (int i = 0; i < n; ++i)
        if (lens[i]) { size = lens[i]; break; }
    if (size == 0) return RBC_ERR_SHARD_NO_DATA;
    for (int i = 0; i < n; ++i)
        if (lens[i] != size && (lens[i] != 0 || !nilok)) return RBC_ERR_SHARD_SIZE;
    *size_out = size;
    return RBC_OK;
}

// Regenerate on the GPU every non-used position of one codeword held in host
// buffers; copy back only the rows the caller asks for.
int host_reconstruct(rbc_ctx *c, uint8_t *const *shards, size_t *lens, int n_shards, bool data_only) {
    if (!shards || !lens) return RBC_ERR_INVALID_ARG;
    if (n_shards != c->n) return RBC_ERR_TOO_FEW_SHARDS;
    size_t S = 0;
    int rc = check_shards(lens, n_shards, true, &S);
    if (rc) return rc;
    int present = 0;
    for (int i = 0; i < c->n; ++i) {
        if (lens[i] && !shards[i]) return RBC_ERR_INVALID_ARG;  // a present shard needs its bytes
        present += lens[i] != 0;
    }
    if (present == c->n) return RBC_OK;
    if (present < c->k) return RBC_ERR_TOO_FEW_SHARDS;
    if (S > 0x7fffffffULL / (size_t)c->n) return RBC_ERR_INVALID_ARG;
    const size_t pitch = round_up(S, kAlign);
    std::lock_guard<std::mutex> lk(c->mu);
    RBC_HIP(hipSetDevice(c->device));
    RBC_HIP(c->d_shards.ensure((size_t)c->n * pitch));
    RBC_HIP(c->d_valid.ensure((size_t)c->n));
    RBC_HIP(c->d_status.ensure(sizeof(int32_t)));
    RBC_HIP(c->h_stage.ensure((size_t)c->n * pitch + c->n));
    uint8_t *stage = c->h_stage.as<uint8_t>();
    memset(stage, 0, (size_t)c->n * pitch + c->n);
    for (int i = 0; i < c->n; ++i) {
        if (lens[i]) memcpy(stage + (size_t)i * pitch, shards[i], S);
        stage[(size_t)c->n * pitch + i] = lens[i] ? 1 : 0;
    }
    hipStream_t st = host_stream(c);
    if (!st) return RBC_ERR_DEVICE;
    RBC_HIP(hipMemcpyAsync(c->d_shards.p, stage, (size_t)c->n * pitch, hipMemcpyHostToDevice, st));
    RBC_HIP(hipMemcpyAsync(c->d_valid.p, stage + (size_t)c->n * pitch, c->n, hipMemcpyHostToDevice, st));
    rc = stage_regenerate(c, c->ws, st, 1, c->d_shards.as<uint8_t>(), (uint32_t)pitch, nullptr, (uint32_t)S,
                          c->d_valid.as<uint8_t>(), c->d_status.as<int32_t>());
    if (rc) return rc;
    RBC_HIP(hipMemcpyAsync(stage, c->d_shards.p, (size_t)c->n * pitch, hipMemcpyDeviceToHost, st));
    int32_t status = 0;
    RBC_HIP(hipMemcpyAsync(&status, c->d_status.p, sizeof status, hipMemcpyDeviceToHost, st));
    RBC_HIP(hipStreamSynchronize(st));
    if (status) return status;
    const int last = data_only ? c->k : c->n;
    for (int i = 0; i < last; ++i) {
        if (lens[i]) continue;
        if (!shards[i]) return RBC_ERR_INVALID_ARG;
        memcpy(shards[i], stage + (size_t)i * pitch, S);
        lens[i] = S;
    }
    return RBC_OK;
}

}  // namespace

// =========================================================================
extern "C" {

const char *rbc_strerror(int s) {
    switch (s) {
        case RBC_OK: return "ok";
        case RBC_ERR_INV_SHARD_NUM: return "cannot create Encoder with zero or less data/parity shards";
        case RBC_ERR_MAX_SHARD_NUM: return "cannot create Encoder with more than 256 data+parity shards";
        case RBC_ERR_TOO_FEW_SHARDS: return "too few shards given";
        case RBC_ERR_SHARD_NO_DATA: return "no shard data";
        case RBC_ERR_SHARD_SIZE: return "shard sizes do not match";
        case RBC_ERR_SHORT_DATA: return "not enough data to fill the number of requested shards";
        case RBC_ERR_RECONSTRUCT_REQUIRED:
            return "reconstruction required as one or more required data shards are nil";
        case RBC_ERR_ROOT_MISMATCH: return "interpolated merkle root does not match the committed root";
        case RBC_ERR_DEVICE: return "HIP/RCCL device error";
        case RBC_ERR_INVALID_ARG: return "invalid argument";
        case RBC_ERR_SINGULAR: return "matrix is singular";
        case RBC_ERR_NO_COMM: return "multi-GPU communicator not initialised";
        case RBC_ERR_INVALID_INPUT: return "invalid input";
        case -20: return "malformed or out-of-protocol RBC message"; /* RBC_ERR_PROTOCOL */
        default: return "unknown rbc status";
    }
}

int rbc_abi_version(void) { return RBC_ABI_VERSION; }

int rbc_ctx_verify_form(const rbc_ctx *c, uint32_t shard_len, int *form) {
    if (!c || !form) return RBC_ERR_INVALID_ARG;
    *form = shared_path_verify(c, nullptr, shard_len) ? RBC_VERIFY_SHARED_PATH : RBC_VERIFY_WALK;
    return RBC_OK;
}

int rbc_ctx_set_recheck(rbc_ctx *c, int mode) {
    if (!c || (mode != RBC_RECHECK_REUSE && mode != RBC_RECHECK_FULL)) return RBC_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    c->recheck = mode;
    return RBC_OK;
}

int rbc_library_path(char *out, size_t cap) {
    if (!out || cap == 0) return RBC_ERR_INVALID_ARG;
    Dl_info info;
    if (!dladdr(reinterpret_cast<void *>(&rbc_library_path), &info) || !info.dli_fname) return RBC_ERR_INVALID_ARG;
    char real[PATH_MAX];
    const char *p = realpath(info.dli_fname, real) ? real : info.dli_fname;
    snprintf(out, cap, "%s", p);
    return RBC_OK;
}

int rbc_device_count(int *count) {
    if (!count) return RBC_ERR_INVALID_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return RBC_OK;
}

int rbc_ctx_create(int n, int f, int device, rbc_ctx **out) {
    if (f < 0 || n - 2 * f <= 0) return RBC_ERR_INV_SHARD_NUM;
    return ctx_create_kn(n, n - 2 * f, device, out);
}

void rbc_ctx_destroy(rbc_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    for (auto &sl : c->slots) {
        if (sl->busy && sl->d2h) {
            (void)sl->d2h(sl->stream);
            sl->d2h = nullptr;
            (void)hipEventRecord(sl->done, sl->stream);
        }
        if (sl->busy) (void)hipEventSynchronize(sl->done);
        sl->release();
    }
    c->ws.release();
    for (DevBuf *b : {&c->d_values, &c->d_shards, &c->d_leaves,
                      &c->d_roots, &c->d_branches, &c->d_valid, &c->d_status, &c->d_digests, &c->d_lens,
                      &c->d_slens, &c->d_idx, &c->d_present, &c->h_stage, &c->h_small, &c->d_pack})
        b->release();
    if (c->d_M) (void)hipFree(c->d_M);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int rbc_ctx_params(const rbc_ctx *c, int *k, int *p, int *depth) {
    if (!c) return RBC_ERR_INVALID_ARG;
    if (k) *k = c->k;
    if (p) *p = c->p;
    if (depth) *depth = c->depth;
    return RBC_OK;
}

int rbc_ctx_device(const rbc_ctx *c, int *device) {
    if (!c || !device) return RBC_ERR_INVALID_ARG;
    *device = c->device;
    return RBC_OK;
}

int rbc_ctx_set_wave_priority(rbc_ctx *c, int commit_prio, int receive_prio) {
    if (!c || commit_prio < 0 || commit_prio > 3 || receive_prio < 0 || receive_prio > 3) return RBC_ERR_INVALID_ARG;
    c->tx_prio = commit_prio;
    c->rx_prio = receive_prio;
    return RBC_OK;
}

int rbc_ctx_set_decode_priority(rbc_ctx *c, int gemv_prio, int reencode_prio) {
    if (!c || gemv_prio < -1 || gemv_prio > 3 || reencode_prio < -1 || reencode_prio > 3) return RBC_ERR_INVALID_ARG;
    c->gemv_prio_ = gemv_prio;
    c->reencode_prio_ = reencode_prio;
    return RBC_OK;
}

int rbc_ctx_set_codec(rbc_ctx *c, int codec) {
    if (!c) return RBC_ERR_INVALID_ARG;
    if (codec == RBC_CODEC_MATRIX) {
        c->fft = false;
    } else if (codec == RBC_CODEC_AUTO || codec == RBC_CODEC_FFT) {
        const bool ok = rbc_fft_supported(c->n, c->k);
        if (codec == RBC_CODEC_FFT && !ok) return RBC_ERR_INVALID_ARG;
        c->fft = ok;
    } else {
        return RBC_ERR_INVALID_ARG;
    }
    return RBC_OK;
}

int rbc_ctx_codec(const rbc_ctx *c, int *codec) {
    if (!c || !codec) return RBC_ERR_INVALID_ARG;
    *codec = c->fft ? RBC_CODEC_FFT : RBC_CODEC_MATRIX;
    return RBC_OK;
}

int rbc_ctx_encode_matrix(const rbc_ctx *c, uint8_t *out) {
    if (!c || !out) return RBC_ERR_INVALID_ARG;
    memcpy(out, c->h_M.data(), c->h_M.size());
    return RBC_OK;
}

// ---- memory / streams / events
int rbc_dev_malloc(int device, size_t bytes, void **ptr) {
    if (!ptr) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(device));
    RBC_HIP(hipMalloc(ptr, bytes ? bytes : 1));
    return RBC_OK;
}
int rbc_dev_free(void *ptr) { RBC_HIP(hipFree(ptr)); return RBC_OK; }
int rbc_dev_memset(void *ptr, int value, size_t bytes) { RBC_HIP(hipMemset(ptr, value, bytes)); return RBC_OK; }
int rbc_memcpy_h2d(void *dst, const void *src, size_t bytes) {
    RBC_HIP(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return RBC_OK;
}
int rbc_memcpy_d2h(void *dst, const void *src, size_t bytes) {
    RBC_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return RBC_OK;
}
int rbc_host_alloc(size_t bytes, void **ptr) {
    if (!ptr) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault));
    return RBC_OK;
}
int rbc_host_free(void *ptr) { RBC_HIP(hipHostFree(ptr)); return RBC_OK; }
int rbc_stream_create(int device, void **stream) {
    if (!stream) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(device));
    hipStream_t s;
    RBC_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = s;
    return RBC_OK;
}
int rbc_stream_create_priority(int device, int high, void **stream) {
    if (!stream) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(device));
    int least = 0, greatest = 0;
    RBC_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    hipStream_t s;
    RBC_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, high ? greatest : least));
    *stream = s;
    return RBC_OK;
}
int rbc_stream_destroy(void *stream) { RBC_HIP(hipStreamDestroy(as_stream(stream))); return RBC_OK; }
int rbc_stream_sync(void *stream) { RBC_HIP(hipStreamSynchronize(as_stream(stream))); return RBC_OK; }
int rbc_event_create(void **event) {
    if (!event) return RBC_ERR_INVALID_ARG;
    hipEvent_t e;
    RBC_HIP(hipEventCreate(&e));
    *event = e;
    return RBC_OK;
}
int rbc_event_destroy(void *event) { RBC_HIP(hipEventDestroy((hipEvent_t)event)); return RBC_OK; }
int rbc_event_record(void *event, void *stream) {
    RBC_HIP(hipEventRecord((hipEvent_t)event, as_stream(stream)));
    return RBC_OK;
}
int rbc_event_elapsed_ms(void *start, void *stop, float *ms) {
    if (!ms) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipEventSynchronize((hipEvent_t)stop));
    RBC_HIP(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
    return RBC_OK;
}
int rbc_stream_wait_event(void *stream, void *event) {
    if (!event) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipStreamWaitEvent(as_stream(stream), (hipEvent_t)event, 0));
    return RBC_OK;
}
int rbc_device_sync(int device) {
    RBC_HIP(hipSetDevice(device));
    RBC_HIP(hipDeviceSynchronize());
    return RBC_OK;
}

// ---- device-resident stages
int rbc_dev_encode(rbc_ctx *c, void *stream, int count, const uint8_t *values, uint64_t value_pitch,
                   const uint32_t *value_lens, uint32_t uniform_value_len, uint8_t *shards, uint32_t shard_pitch) {
    if (!c) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(c->device));
    return stage_encode(c, as_stream(stream), count, values, value_pitch, value_lens, uniform_value_len, shards,
                        shard_pitch);
}

int rbc_dev_leaves(rbc_ctx *c, void *stream, int count, const uint8_t *shards, uint32_t shard_pitch,
                   const uint32_t *shard_lens, uint32_t uniform_shard_len, uint8_t *leaves) {
    if (!c) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(c->device));
    return stage_leaves(c, as_stream(stream), count, shards, shard_pitch, shard_lens, uniform_shard_len, leaves);
}

int rbc_dev_merkle_build(rbc_ctx *c, void *stream, int count, const uint8_t *leaves, uint8_t *roots,
                         uint8_t *branches) {
    if (!c) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(c->device));
    return stage_merkle_build(c, as_stream(stream), count, leaves, roots, branches);
}

int rbc_dev_shard_commit(rbc_ctx *c, void *stream, int count, const uint8_t *values, uint64_t value_pitch,
                         const uint32_t *value_lens, uint32_t uniform_value_len, uint8_t *shards,
                         uint32_t shard_pitch, const uint32_t *shard_lens, uint8_t *leaves, uint8_t *roots,
                         uint8_t *branches) {
    if (!c) return RBC_ERR_INVALID_ARG;
    if (value_lens && !shard_lens) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(c->device));
    hipStream_t st = as_stream(stream);
    int rc = stage_encode(c, st, count, values, value_pitch, value_lens, uniform_value_len, shards, shard_pitch);
    if (rc) return rc;
    const uint32_t uS = value_lens ? 0u : (uniform_value_len + c->k - 1) / c->k;
    rc = stage_leaves(c, st, count, shards, shard_pitch, shard_lens, uS, leaves);
    if (rc) return rc;
    return stage_merkle_build(c, st, count, leaves, roots, branches);
}

int rbc_dev_verify(rbc_ctx *c, void *stream, int count, const uint8_t *shards, uint32_t shard_pitch,
                   const uint32_t *shard_lens, uint32_t uniform_shard_len, const uint8_t *branches,
                   const uint8_t *roots, const uint8_t *present, uint8_t *valid, uint8_t *leaves) {
    if (!c) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(c->device));
    return stage_verify(c, as_stream(stream), count, shards, shard_pitch, shard_lens, uniform_shard_len, branches,
                        roots, present, valid, leaves);
}

int rbc_dev_interpolate(rbc_ctx *c, void *stream, int count, uint8_t *shards, uint32_t shard_pitch,
                        const uint32_t *shard_lens, uint32_t uniform_shard_len, const uint8_t *valid,
                        uint8_t *leaves, int leaves_verified, const uint8_t *roots, uint8_t *values_out,
                        uint32_t value_pitch, uint8_t *digests, int32_t *status) {
    if (!c) return RBC_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);  // shared decode workspace
    // the workspace holds a receive-step batch's regen list until its next call
    if (c->ws.rx_count > 0) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(c->device));
    return stage_interpolate(c, c->ws, as_stream(stream), count, shards, shard_pitch, shard_lens, uniform_shard_len,
                             valid, leaves, leaves_verified, roots, values_out, value_pitch, digests, status);
}

int rbc_dev_receive_step(rbc_ctx *c, void *stream, const rbc_rx_batch *cur, const rbc_rx_batch *prev,
                         const rbc_rx_marks *marks) {
    if (!c) return RBC_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);  // shared decode workspace
    RBC_HIP(hipSetDevice(c->device));
    return stage_receive_step(c, as_stream(stream), cur, prev, marks);
}

size_t rbc_val_message_size(int n, uint32_t shard_len, uint32_t index, int type) {
    if (n < 1) return 0;
    int d = 0;
    while ((1 << d) < n) ++d;
    return rbc_val_message_bytes(n, d, shard_len, index, type);
}

int rbc_dev_marshal_val(rbc_ctx *c, void *stream, int count, int type, const uint8_t *shards,
                        uint32_t shard_pitch, const uint32_t *shard_lens, uint32_t uniform_shard_len,
                        const uint8_t *branches, const uint8_t *roots, uint8_t *out, uint64_t out_pitch,
                        uint32_t *out_lens) {
    if (!c || count < 0 || (type != 0 && type != 1) || out_pitch % 16 || shard_pitch % 4) return RBC_ERR_INVALID_ARG;
    if (count == 0) return RBC_OK;
    if (!shards || !roots || !out || (c->depth && !branches)) return RBC_ERR_INVALID_ARG;
    if (!shard_lens && (uniform_shard_len == 0 || uniform_shard_len > shard_pitch ||
                        out_pitch < rbc_val_message_bytes(c->n, c->depth, uniform_shard_len, 0, type)))
        return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(c->device));
    WireArgs a{};
    a.count = count;
    a.n = c->n;
    a.depth = c->depth;
    a.type = type;
    a.shards = shards;
    a.inst_pitch = (uint64_t)c->n * shard_pitch;
    a.row_pitch = shard_pitch;
    a.lens = shard_lens;
    a.uniform_len = uniform_shard_len;
    a.branches = branches;
    a.roots = roots;
    a.out = out;
    a.out_pitch = out_pitch;
    a.out_lens = out_lens;
    RBC_HIP(rbc_launch_marshal_val(a, as_stream(stream)));
    return RBC_OK;
}

int rbc_dev_inject_faults(rbc_ctx *c, void *stream, int count, uint8_t *shards, uint32_t shard_pitch,
                          const int32_t *corrupt) {
    if (!c || count < 0 || (count > 0 && (!shards || !corrupt))) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(c->device));
    RBC_HIP(rbc_launch_inject_faults(shards, (uint64_t)c->n * shard_pitch, shard_pitch, corrupt, count,
                                     as_stream(stream)));
    return RBC_OK;
}

// ---- host-memory batch API (pipelined through per-context slots)
extern "C++" {
namespace {

// Host-side staging copies run on several threads: one thread's memcpy
// (~10 GB/s) would otherwise bound the host path well below PCIe.
template <class F>
void parallel_for(int count, size_t bytes_per_item, F &&f) {
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    int nt = (int)std::min<size_t>(std::min<unsigned>(hw, 16u), (size_t)count * bytes_per_item / (4u << 20));
    nt = std::max(1, std::min(nt, count));
    if (nt == 1) {
        for (int i = 0; i < count; ++i) f(i);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(nt - 1);
    auto body = [&](int t) {
        for (int i = t; i < count; i += nt) f(i);
    };
    for (int t = 1; t < nt; ++t) th.emplace_back(body, t);
    body(0);
    for (auto &x : th) x.join();
}

// Enqueue a submission's deferred device-to-host copies and its completion
// event (see Slot::d2h).
void flush_d2h(Slot &s) {
    if (!s.d2h) return;
    s.d2h_rc = s.d2h(s.stream);
    s.d2h = nullptr;
    if (hipEventRecord(s.done, s.stream) != hipSuccess && !s.d2h_rc) s.d2h_rc = RBC_ERR_DEVICE;
}

// Free slot for the next submission: create one while fewer than
// kHostSlots exist, else reuse an idle one, else retire the oldest
// in-flight submission (its status is kept until the caller waits on it).
int retire(rbc_ctx *c, Slot &s) {
    int st = RBC_OK;
    flush_d2h(s);
    if (s.d2h_rc) st = s.d2h_rc;
    s.d2h_rc = 0;
    if (hipEventSynchronize(s.done) != hipSuccess) st = RBC_ERR_DEVICE;
    if (st == RBC_OK && s.finish) st = s.finish();
    s.finish = nullptr;
    s.busy = false;
    return st;
}

#ifndef RBC_BLOCKING_SYNC_EVENTS
#define RBC_BLOCKING_SYNC_EVENTS 1
#endif
constexpr unsigned kSlotEventSync = RBC_BLOCKING_SYNC_EVENTS ? hipEventBlockingSync : 0u;

Slot *acquire_slot(rbc_ctx *c) {
    for (auto &sl : c->slots)
        if (!sl->busy) return sl.get();
    if ((int)c->slots.size() < kHostSlots) {
        auto sl = std::make_unique<Slot>();
        if (hipStreamCreateWithFlags(&sl->stream, hipStreamNonBlocking) != hipSuccess ||
            (RBC_D2H_STREAM && hipStreamCreateWithFlags(&sl->dstream, hipStreamNonBlocking) != hipSuccess) ||
            // blocking-sync events: a host-API waiter (the batcher's completer, a
            // goroutine's cgo call) sleeps instead of spinning a core the
            // submitting threads need for their staging copies
            hipEventCreateWithFlags(&sl->done, hipEventDisableTiming | kSlotEventSync) != hipSuccess ||
            hipEventCreateWithFlags(&sl->kdone, hipEventDisableTiming | kSlotEventSync) != hipSuccess ||
            !sl->ws.init()) {
            sl->release();
            return nullptr;
        }
        sl->ws.fork = false;
        c->slots.push_back(std::move(sl));
        return c->slots.back().get();
    }
    Slot *old = nullptr;
    for (auto &sl : c->slots)
        if (!old || sl->ticket < old->ticket) old = sl.get();
    c->retired[old->ticket] = retire(c, *old);
    return old;
}

// Seal a submission: record its completion event and hand out a ticket, or
// (ticket == NULL) complete it before returning.  With `d2h` the submission's
// device-to-host copies are deferred (Slot::d2h); the other slots' deferred
// copies are enqueued now, behind this submission's host-to-device copies.
int submit(rbc_ctx *c, Slot &s, uint64_t *ticket, std::function<int()> finish,
           std::function<int(hipStream_t)> d2h = nullptr) {
    s.finish = std::move(finish);
    for (auto &o : c->slots)
        if (o.get() != &s && o->busy) flush_d2h(*o);
    s.d2h_rc = 0;
#ifndef RBC_DEFER_D2H
#define RBC_DEFER_D2H 1
#endif
    if (RBC_D2H_STREAM && d2h) {
        // the D2H copies go on the slot's own copy stream at once, behind an
        // event wait on its kernels: nothing waits in front of the next
        // submission's H2D on the compute stream, and no host call has to
        // enqueue them later
        const int rc = hipEventRecord(s.kdone, s.stream) != hipSuccess ||
                               hipStreamWaitEvent(s.dstream, s.kdone, 0) != hipSuccess
                           ? RBC_ERR_DEVICE
                           : d2h(s.dstream);
        if (rc || hipEventRecord(s.done, s.dstream) != hipSuccess) {
            s.finish = nullptr;
            return rc ? rc : RBC_ERR_DEVICE;
        }
    } else if (RBC_DEFER_D2H && d2h && ticket) {
        if (hipEventRecord(s.kdone, s.stream) != hipSuccess) {
            s.finish = nullptr;
            return RBC_ERR_DEVICE;
        }
        s.d2h = std::move(d2h);
    } else {
        const int rc = d2h ? d2h(s.stream) : RBC_OK;
        if (rc || hipEventRecord(s.done, s.stream) != hipSuccess) {
            s.finish = nullptr;
            return rc ? rc : RBC_ERR_DEVICE;
        }
    }
    s.ticket = c->next_ticket++;
    s.busy = true;
    if (!ticket) return retire(c, s);
    *ticket = s.ticket;
    return RBC_OK;
}

}  // namespace
}  // extern "C++"

// Caller memory that is already pinned (rbc_host_alloc / hipHostMalloc /
// hipHostRegister) is copied to and from directly: no staging memcpy.  A Go
// batcher that keeps its request and result rings in rbc_host_alloc memory
// gets the PCIe-only path.
static bool host_pinned(const void *p, size_t bytes) {
    if (!p) return false;
    for (const void *q : {p, (const void *)((const uint8_t *)p + (bytes ? bytes - 1 : 0))}) {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, q) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (a.type != hipMemoryTypeHost) return false;
    }
    return true;
}

// [p, p + bytes) readable by a kernel: device memory, or pinned host memory
// mapped at the same address (both ends checked: one attribute query each)
static bool device_readable(const void *p, size_t bytes) {
    if (!p) return false;
    for (const void *q : {p, (const void *)((const uint8_t *)p + (bytes ? bytes - 1 : 0))}) {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, q) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (a.type == hipMemoryTypeDevice) continue;
        if (a.type == hipMemoryTypeHost && a.devicePointer == q) continue;
        return false;
    }
    return true;
}

// The device address of pinned caller memory when it is the host address itself
// (hipHostMalloc / rbc_host_alloc under unified addressing), else NULL: a
// kernel may then read it directly over PCIe.
inline int n_of(const rbc_ctx *c) { return c->n; }
#ifndef RBC_ZERO_COPY_READS
#define RBC_ZERO_COPY_READS 1
#endif
static const uint8_t *host_zero_copy(const void *p, size_t bytes) {
    if (!RBC_ZERO_COPY_READS || !host_pinned(p, bytes)) return nullptr;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return a.devicePointer == p ? static_cast<const uint8_t *>(p) : nullptr;
}

// Every value in pinned memory?  *zc: also each readable zero-copy at its own
// address (two attribute queries per value, as host_pinned).
static bool values_pinned(const uint8_t *const *values, const size_t *lens, int count, bool *zc) {
    *zc = RBC_ZERO_COPY_READS != 0;
    for (int i = 0; i < count; ++i) {
        for (int e = 0; e < 2; ++e) {
            const void *q = values[i] + (e ? lens[i] - 1 : 0);
            hipPointerAttribute_t a;
            if (hipPointerGetAttributes(&a, q) != hipSuccess) {
                (void)hipGetLastError();
                return false;
            }
            if (a.type != hipMemoryTypeHost) return false;
            if (!e && a.devicePointer != q) *zc = false;
        }
    }
    return true;
}

// The pinned values of a shard_commit submission into the device value rows:
// one DMA per value, or -- many short values, all readable zero-copy -- one
// gather launch over their addresses (host time per DMA call dominated C4's
// 16,384-value epoch).  `lens` ([2*count] u32, pinned staging) is uploaded
// here when the gather needs it; `ptr_stage` has room for count addresses.
static int upload_pinned_values(Slot &s, hipStream_t st, int count, const uint8_t *const *values,
                                const size_t *value_lens, size_t vpitch, bool zc, uint32_t *lens,
                                uint64_t *ptr_stage) {
    size_t total = 0;
    for (int i = 0; i < count; ++i) total += value_lens[i];
    if (zc && count >= 64 && total / count < ((size_t)256 << 10)) {
        for (int i = 0; i < count; ++i) ptr_stage[i] = (uint64_t)(uintptr_t)values[i];
        RBC_HIP(s.d_offs.ensure((size_t)count * 8));
        RBC_HIP(hipMemcpyAsync(s.d_offs.p, ptr_stage, (size_t)count * 8, hipMemcpyHostToDevice, st));
        RBC_HIP(hipMemcpyAsync(s.d_lens.p, lens, (size_t)count * 4, hipMemcpyHostToDevice, st));
        RBC_HIP(rbc_launch_gather_values(s.d_offs.as<uint64_t>(), s.d_lens.as<uint32_t>(), (uint32_t)count,
                                         s.d_values.as<uint8_t>(), vpitch, st));
        return RBC_OK;
    }
    for (int i = 0; i < count; ++i)
        RBC_HIP(hipMemcpyAsync(s.d_values.as<uint8_t>() + (size_t)i * vpitch, values[i], value_lens[i],
                               hipMemcpyHostToDevice, st));
    return RBC_OK;
}

int rbc_shard_commit(rbc_ctx *c, int count, const uint8_t *const *values, const size_t *value_lens,
                     uint8_t *shards_out, size_t shard_pitch, uint32_t *shard_lens_out, uint8_t *roots_out,
                     uint8_t *branches_out, uint64_t *ticket) {
    if (!c || count < 0 || (count > 0 && (!values || !value_lens || !shards_out || !roots_out)))
        return RBC_ERR_INVALID_ARG;
    if (count == 0) { if (ticket) *ticket = 0; return RBC_OK; }
    size_t Smax = 0;
    for (int i = 0; i < count; ++i) {
        if (value_lens[i] == 0) return RBC_ERR_SHORT_DATA;  // Split: len(data) == 0
        if (!values[i]) return RBC_ERR_INVALID_ARG;
        Smax = std::max(Smax, (value_lens[i] + c->k - 1) / c->k);
    }
    if (shard_pitch < Smax) return RBC_ERR_INVALID_ARG;
    // pinned output whose pitch the device rows can take: the device rows use
    // it and the shards come back in ONE plain copy (pitch-to-pitch 2-D copies
    // of many short rows ran at 0.1 GB/s at C4, and odd pitches off the copy
    // engine's fast path); else whole HBM lines per row
    const bool sh_direct = host_pinned(shards_out, ((size_t)count * c->n - 1) * shard_pitch + Smax);
    const bool sh_flat = sh_direct && shard_pitch % kAlign == 0 && shard_pitch <= 0x7fffffffULL / c->n &&
                         host_pinned(shards_out, (size_t)count * c->n * shard_pitch);  // the flat copy's extent
    const size_t dpitch = sh_flat ? shard_pitch : round_up(Smax, 128);
    const size_t vpitch = round_up((size_t)c->k * Smax + 32, kAlign);
    if (vpitch > 0x7fffffffULL || (size_t)c->n * dpitch > 0x7fffffffULL) return RBC_ERR_INVALID_ARG;
    const int d = c->depth, n = c->n;
    const size_t sh_bytes = (size_t)count * n * dpitch, br_bytes = (size_t)count * n * std::max(d, 1) * 32;
    std::lock_guard<std::mutex> lk(c->mu);
    RBC_HIP(hipSetDevice(c->device));
    Slot *sp = acquire_slot(c);
    if (!sp) return RBC_ERR_DEVICE;
    Slot &s = *sp;
    hipStream_t st = s.stream;
    RBC_HIP(s.d_values.ensure((size_t)count * vpitch));
    RBC_HIP(s.d_shards.ensure(sh_bytes));
    RBC_HIP(s.d_leaves.ensure((size_t)count * n * 32));
    RBC_HIP(s.d_roots.ensure((size_t)count * 32));
    RBC_HIP(s.d_branches.ensure(br_bytes));
    RBC_HIP(s.d_lens.ensure((size_t)count * 8));
    // pinned staging only for what is not already pinned caller memory
    bool zc = false;
    const bool in_direct = values_pinned(values, value_lens, count, &zc);
    const size_t in_stage = in_direct ? 0 : (size_t)count * vpitch;
    const bool rt_direct = host_pinned(roots_out, (size_t)count * 32);
    const size_t br_out = (size_t)count * n * d * 32;
    const bool br_direct = branches_out && d > 0 && host_pinned(branches_out, br_out);
    RBC_HIP(s.h_in.ensure(in_stage + (size_t)count * 8 + (in_direct ? (size_t)count * 8 : 0)));
    RBC_HIP(s.h_out.ensure((sh_direct ? 0 : sh_bytes) + (size_t)count * 32 + br_bytes));
    uint8_t *stage = s.h_in.as<uint8_t>();
    uint32_t *lens = reinterpret_cast<uint32_t *>(stage + in_stage);
    if (in_direct) {
        // the encode kernel masks the Split pad (bytes past len are never used)
        for (int i = 0; i < count; ++i) {
            lens[i] = (uint32_t)value_lens[i];
            lens[count + i] = (uint32_t)((value_lens[i] + c->k - 1) / c->k);
        }
        const int rc = upload_pinned_values(s, st, count, values, value_lens, vpitch, zc, lens,
                                            reinterpret_cast<uint64_t *>(stage + in_stage + (size_t)count * 8));
        if (rc) return rc;
    } else {
        parallel_for(count, vpitch, [&](int i) {
            memcpy(stage + (size_t)i * vpitch, values[i], value_lens[i]);
            memset(stage + (size_t)i * vpitch + value_lens[i], 0, vpitch - value_lens[i]);
            lens[i] = (uint32_t)value_lens[i];
            lens[count + i] = (uint32_t)((value_lens[i] + c->k - 1) / c->k);
        });
        RBC_HIP(hipMemcpyAsync(s.d_values.p, stage, (size_t)count * vpitch, hipMemcpyHostToDevice, st));
    }
    RBC_HIP(hipMemcpyAsync(s.d_lens.p, lens, (size_t)count * 8, hipMemcpyHostToDevice, st));
    const uint32_t *d_vlens = s.d_lens.as<uint32_t>(), *d_slens = d_vlens + count;
    int rc = stage_encode(c, st, count, s.d_values.as<uint8_t>(), vpitch, d_vlens, 0, s.d_shards.as<uint8_t>(),
                          (uint32_t)dpitch);
    if (!rc) rc = stage_leaves(c, st, count, s.d_shards.as<uint8_t>(), (uint32_t)dpitch, d_slens, 0,
                               s.d_leaves.as<uint8_t>());
    if (!rc) rc = stage_merkle_build(c, st, count, s.d_leaves.as<uint8_t>(), s.d_roots.as<uint8_t>(),
                                     s.d_branches.as<uint8_t>());
    if (rc) return rc;
    uint8_t *o_sh = s.h_out.as<uint8_t>(), *o_rt = o_sh + (sh_direct ? 0 : sh_bytes),
            *o_br = o_rt + (size_t)count * 32;
    void *d_sh = s.d_shards.p, *d_rt = s.d_roots.p, *d_br = s.d_branches.p;
    auto d2h = [=](hipStream_t cs) -> int {
        if (sh_direct && dpitch == shard_pitch)  // every row whole: bytes [S_i, pitch) come back zero
            RBC_HIP(hipMemcpyAsync(shards_out, d_sh, sh_bytes, hipMemcpyDeviceToHost, cs));
        else if (sh_direct)  // Smax bytes per row: the device rows are zero past S_i
            RBC_HIP(hipMemcpy2DAsync(shards_out, shard_pitch, d_sh, dpitch, Smax, (size_t)count * n,
                                     hipMemcpyDeviceToHost, cs));
        else
            RBC_HIP(hipMemcpyAsync(o_sh, d_sh, sh_bytes, hipMemcpyDeviceToHost, cs));
        RBC_HIP(hipMemcpyAsync(rt_direct ? roots_out : o_rt, d_rt, (size_t)count * 32, hipMemcpyDeviceToHost, cs));
        if (branches_out && d > 0)
            RBC_HIP(hipMemcpyAsync(br_direct ? branches_out : o_br, d_br, br_bytes, hipMemcpyDeviceToHost, cs));
        return RBC_OK;
    };
    return submit(c, s, ticket, [=]() {
        parallel_for(count, sh_direct ? 0 : (size_t)n * Smax, [&](int i) {
            const size_t S = lens[count + i];
            if (!sh_direct)
                for (int j = 0; j < n; ++j)
                    memcpy(shards_out + ((size_t)i * n + j) * shard_pitch, o_sh + ((size_t)i * n + j) * dpitch, Smax);
            if (shard_lens_out) shard_lens_out[i] = (uint32_t)S;
        });
        if (!rt_direct) memcpy(roots_out, o_rt, (size_t)count * 32);
        if (branches_out && d > 0 && !br_direct) memcpy(branches_out, o_br, br_out);
        return RBC_OK;
    }, d2h);
}

// VAL hand-off: shard + commit on the device, marshal the
// N per-recipient pb.Message VALs there (marshal_val_kernel) and move the
// whole batch of finished messages to the caller's ring in one D2H.
int rbc_shard_commit_val(rbc_ctx *c, int count, const uint8_t *const *values, const size_t *value_lens,
                         uint8_t *msgs, size_t msg_pitch, uint32_t *msg_lens, uint8_t *roots_out,
                         uint64_t *ticket) {
    if (!c || count < 0 || (count > 0 && (!values || !value_lens || !msgs || !msg_lens))) return RBC_ERR_INVALID_ARG;
    if (count == 0) { if (ticket) *ticket = 0; return RBC_OK; }
    size_t Smax = 0;
    for (int i = 0; i < count; ++i) {
        if (value_lens[i] == 0) return RBC_ERR_SHORT_DATA;  // Split: len(data) == 0
        if (!values[i]) return RBC_ERR_INVALID_ARG;
        Smax = std::max(Smax, (value_lens[i] + c->k - 1) / c->k);
    }
    const int d = c->depth, n = c->n;
    const size_t need = round_up(std::max(rbc_val_message_bytes(n, d, (uint32_t)Smax, 0, RBC_MSG_VAL),
                                          rbc_val_message_bytes(n, d, (uint32_t)Smax, (uint32_t)(n - 1),
                                                                RBC_MSG_VAL)),
                                 16);
    if (msg_pitch < need || msg_pitch % 16) return RBC_ERR_INVALID_ARG;
    const size_t dpitch = round_up(Smax, 128);
    const size_t vpitch = round_up((size_t)c->k * Smax + 32, kAlign);
    if (vpitch > 0x7fffffffULL || (size_t)n * dpitch > 0x7fffffffULL) return RBC_ERR_INVALID_ARG;
    const size_t sh_bytes = (size_t)count * n * dpitch, br_bytes = (size_t)count * n * std::max(d, 1) * 32;
    const size_t msg_bytes = (size_t)count * n * msg_pitch;
    std::lock_guard<std::mutex> lk(c->mu);
    RBC_HIP(hipSetDevice(c->device));
    Slot *sp = acquire_slot(c);
    if (!sp) return RBC_ERR_DEVICE;
    Slot &s = *sp;
    hipStream_t st = s.stream;
    RBC_HIP(s.d_values.ensure((size_t)count * vpitch));
    RBC_HIP(s.d_shards.ensure(sh_bytes + msg_bytes));  // shards, then the messages
    RBC_HIP(s.d_leaves.ensure((size_t)count * n * 32));
    RBC_HIP(s.d_roots.ensure((size_t)count * 32));
    RBC_HIP(s.d_branches.ensure(br_bytes));
    RBC_HIP(s.d_lens.ensure((size_t)count * 8 + (size_t)count * n * 4));
    RBC_HIP(s.h_in.ensure((size_t)count * vpitch + (size_t)count * 16));
    uint8_t *stage = s.h_in.as<uint8_t>();
    uint32_t *lens = reinterpret_cast<uint32_t *>(stage + (size_t)count * vpitch);
    bool zc = false;
    const bool in_direct = values_pinned(values, value_lens, count, &zc);
    if (in_direct) {  // pinned values: one DMA each (or one gather), the encode kernel masks the Split pad
        for (int i = 0; i < count; ++i) {
            lens[i] = (uint32_t)value_lens[i];
            lens[count + i] = (uint32_t)((value_lens[i] + c->k - 1) / c->k);
        }
        const int rc = upload_pinned_values(s, st, count, values, value_lens, vpitch, zc, lens,
                                            reinterpret_cast<uint64_t *>(lens + 2 * (size_t)count));
        if (rc) return rc;
    } else {
        parallel_for(count, vpitch, [&](int i) {
            memcpy(stage + (size_t)i * vpitch, values[i], value_lens[i]);
            memset(stage + (size_t)i * vpitch + value_lens[i], 0, vpitch - value_lens[i]);
            lens[i] = (uint32_t)value_lens[i];
            lens[count + i] = (uint32_t)((value_lens[i] + c->k - 1) / c->k);
        });
        RBC_HIP(hipMemcpyAsync(s.d_values.p, stage, (size_t)count * vpitch, hipMemcpyHostToDevice, st));
    }
    RBC_HIP(hipMemcpyAsync(s.d_lens.p, lens, (size_t)count * 8, hipMemcpyHostToDevice, st));
    const uint32_t *d_vlens = s.d_lens.as<uint32_t>(), *d_slens = d_vlens + count;
    uint32_t *d_mlens = s.d_lens.as<uint32_t>() + 2 * (size_t)count;
    uint8_t *d_sh = s.d_shards.as<uint8_t>(), *d_msgs = d_sh + sh_bytes;
    int rc = stage_encode(c, st, count, s.d_values.as<uint8_t>(), vpitch, d_vlens, 0, d_sh, (uint32_t)dpitch);
    if (!rc) rc = stage_leaves(c, st, count, d_sh, (uint32_t)dpitch, d_slens, 0, s.d_leaves.as<uint8_t>());
    if (!rc) rc = stage_merkle_build(c, st, count, s.d_leaves.as<uint8_t>(), s.d_roots.as<uint8_t>(),
                                     s.d_branches.as<uint8_t>());
    if (rc) return rc;
    WireArgs a{};
    a.count = count;
    a.n = n;
    a.depth = d;
    a.type = RBC_MSG_VAL;
    a.shards = d_sh;
    a.inst_pitch = (uint64_t)n * dpitch;
    a.row_pitch = (uint32_t)dpitch;
    a.lens = d_slens;
    a.branches = s.d_branches.as<uint8_t>();
    a.roots = s.d_roots.as<uint8_t>();
    a.out = d_msgs;
    a.out_pitch = msg_pitch;
    a.out_lens = d_mlens;
    RBC_HIP(rbc_launch_marshal_val(a, st));
    // one D2H of the finished messages: straight into a pinned ring, else
    // through HIP's staging (pageable); deferred behind the next submission's H2D
    void *d_rt = s.d_roots.p;
    auto d2h = [=](hipStream_t cs) -> int {
        RBC_HIP(hipMemcpyAsync(msgs, d_msgs, msg_bytes, hipMemcpyDeviceToHost, cs));
        RBC_HIP(hipMemcpyAsync(msg_lens, d_mlens, (size_t)count * n * 4, hipMemcpyDeviceToHost, cs));
        if (roots_out) RBC_HIP(hipMemcpyAsync(roots_out, d_rt, (size_t)count * 32, hipMemcpyDeviceToHost, cs));
        return RBC_OK;
    };
    return submit(c, s, ticket, []() { return RBC_OK; }, d2h);
}

int rbc_validate_batch(rbc_ctx *c, int count, const uint8_t *const *shards, const size_t *shard_lens,
                       const uint32_t *indices, const uint8_t *const *branches, const size_t *branch_lens,
                       const uint8_t *const *roots, uint8_t *ok_out, uint64_t *ticket) {
    if (!c || count < 0 ||
        (count > 0 && (!shards || !shard_lens || !indices || !branches || !branch_lens || !roots || !ok_out)))
        return RBC_ERR_INVALID_ARG;
    if (count == 0) { if (ticket) *ticket = 0; return RBC_OK; }
    const int d = c->depth;
    size_t Smax = 1;
    for (int i = 0; i < count; ++i) Smax = std::max(Smax, shard_lens[i]);
    const size_t pitch = round_up(Smax, kAlign);
    const size_t bslot = (size_t)std::max(d, 1) * 32;
    if ((size_t)count * pitch > 0x7fffffffULL) return RBC_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    RBC_HIP(hipSetDevice(c->device));
    Slot *sp = acquire_slot(c);
    if (!sp) return RBC_ERR_DEVICE;
    Slot &s = *sp;
    hipStream_t st = s.stream;
    const size_t stage_bytes = (size_t)count * (pitch + bslot + 32 + 4 + 1);
    RBC_HIP(s.h_in.ensure(stage_bytes));
    RBC_HIP(s.h_out.ensure((size_t)count * 2));
    RBC_HIP(s.d_shards.ensure((size_t)count * pitch));
    RBC_HIP(s.d_branches.ensure((size_t)count * bslot));
    RBC_HIP(s.d_roots.ensure((size_t)count * 32));
    RBC_HIP(s.d_slens.ensure((size_t)count * 4));
    RBC_HIP(s.d_idx.ensure((size_t)count));
    RBC_HIP(s.d_valid.ensure((size_t)count));
    uint8_t *sh = s.h_in.as<uint8_t>();
    uint8_t *br = sh + (size_t)count * pitch;
    uint8_t *rt = br + (size_t)count * bslot;
    uint32_t *ln = reinterpret_cast<uint32_t *>(rt + (size_t)count * 32);
    uint8_t *ix = reinterpret_cast<uint8_t *>(ln + count);
    uint8_t *shape_ok = s.h_out.as<uint8_t>() + count;  // host-side shape verdicts
    // No blanket zeroing: the kernel reads a row only up to its length (the
    // bytes past it inside the last 64-byte block are masked), and a
    // malformed entry hashes one staged byte whose verdict is discarded.
    parallel_for(count, pitch, [&](int i) {
        const uint32_t j = indices[i];
        // unflatten the Go-form branch (the empty level-0 sibling is omitted)
        const bool empty0 = d > 0 && (j ^ 1u) >= (uint32_t)c->n;
        const size_t want = (size_t)32 * (d - (empty0 ? 1 : 0));
        shape_ok[i] = 1;
        if (j >= (uint32_t)c->n || branch_lens[i] != want || shard_lens[i] == 0 || !shards[i] || !roots[i] ||
            (want && !branches[i])) {
            shape_ok[i] = 0;
            ln[i] = 1;
            ix[i] = 0;
            memset(sh + (size_t)i * pitch, 0, 64);
            memset(br + (size_t)i * bslot, 0, bslot);
            memset(rt + 32 * i, 0, 32);
            return;
        }
        memcpy(sh + (size_t)i * pitch, shards[i], shard_lens[i]);
        size_t off = 0;
        for (int l = 0; l < d; ++l) {
            if (l == 0 && empty0) {
                memset(br + (size_t)i * bslot, 0, 32);  // the device form keeps a zero level-0 slot
                continue;
            }
            memcpy(br + (size_t)i * bslot + 32 * l, branches[i] + off, 32);
            off += 32;
        }
        memcpy(rt + 32 * i, roots[i], 32);
        ln[i] = (uint32_t)shard_lens[i];
        ix[i] = (uint8_t)j;
    });
    RBC_HIP(hipMemcpyAsync(s.d_shards.p, sh, (size_t)count * pitch, hipMemcpyHostToDevice, st));
    RBC_HIP(hipMemcpyAsync(s.d_branches.p, br, (size_t)count * bslot, hipMemcpyHostToDevice, st));
    RBC_HIP(hipMemcpyAsync(s.d_roots.p, rt, (size_t)count * 32, hipMemcpyHostToDevice, st));
    RBC_HIP(hipMemcpyAsync(s.d_slens.p, ln, (size_t)count * 4, hipMemcpyHostToDevice, st));
    RBC_HIP(hipMemcpyAsync(s.d_idx.p, ix, (size_t)count, hipMemcpyHostToDevice, st));
    ShaArgs a{};
    a.count = count;
    a.rows_per_inst = 1;
    a.rows = s.d_shards.as<uint8_t>();
    a.inst_pitch = pitch;
    a.row_pitch = 0;
    a.lens = s.d_slens.as<uint32_t>();
    a.idx = s.d_idx.as<uint8_t>();
    a.idx_stride = 1;
    a.per_message = 1;
    a.n = c->n;
    a.depth = d;
    a.branches = s.d_branches.as<uint8_t>();
    a.br_inst_pitch = bslot;
    a.roots = s.d_roots.as<uint8_t>();
    a.valid = s.d_valid.as<uint8_t>();
    RBC_HIP(rbc_launch_sha_rows(a, true, st));
    uint8_t *o_ok = s.h_out.as<uint8_t>();
    RBC_HIP(hipMemcpyAsync(o_ok, s.d_valid.p, (size_t)count, hipMemcpyDeviceToHost, st));
    return submit(c, s, ticket, [=]() {
        for (int i = 0; i < count; ++i) ok_out[i] = shape_ok[i] ? o_ok[i] : 0;
        return RBC_OK;
    });
}

// The packed form of rbc_validate_batch: the caller (the batcher's validate
// lane, or a Go batcher with its own rbc_host_alloc rings) has already laid the
// messages out as the device reads them, so this is one DMA of the shard arena,
// the metadata, one launch and a deferred D2H of the verdicts -- no per-message
// staging copy on the submitting thread.
int rbc_validate_packed(rbc_ctx *c, int count, const uint8_t *arena, size_t arena_bytes, const uint64_t *offs,
                        const uint32_t *lens, const uint8_t *idx, const uint8_t *branches, const uint8_t *roots,
                        uint8_t *ok_out, uint64_t *ticket) {
    return rbc_validate_packed_leaves(c, count, arena, arena_bytes, offs, lens, idx, branches, roots, ok_out, nullptr,
                                      ticket);
}

static int validate_packed(rbc_ctx *c, int count, const uint8_t *arena, size_t arena_bytes, const uint64_t *offs,
                           const uint32_t *lens, const uint8_t *idx, const uint8_t *branches, const uint8_t *roots,
                           uint8_t *ok_out, uint8_t *leaves_out, uint8_t *keep_dev, size_t keep_bytes,
                           uint64_t *ticket);

int rbc_validate_packed_leaves(rbc_ctx *c, int count, const uint8_t *arena, size_t arena_bytes, const uint64_t *offs,
                               const uint32_t *lens, const uint8_t *idx, const uint8_t *branches, const uint8_t *roots,
                               uint8_t *ok_out, uint8_t *leaves_out, uint64_t *ticket) {
    return validate_packed(c, count, arena, arena_bytes, offs, lens, idx, branches, roots, ok_out, leaves_out, nullptr,
                           0, ticket);
}

// The messages land in the caller's device buffer instead of the slot's and
// stay there: an interpolate of the same shards reads them on the device
// (rbc_interpolate_batch_kept), so the ECHO rows cross PCIe once.
int rbc_validate_packed_keep(rbc_ctx *c, int count, const uint8_t *arena, size_t arena_bytes, const uint64_t *offs,
                             const uint32_t *lens, const uint8_t *idx, const uint8_t *branches, const uint8_t *roots,
                             uint8_t *ok_out, uint8_t *leaves_out, uint8_t *keep_dev, size_t keep_bytes,
                             uint64_t *ticket) {
    if (count > 0 && (!keep_dev || keep_bytes < arena_bytes || !device_readable(keep_dev, arena_bytes)))
        return RBC_ERR_INVALID_ARG;
    return validate_packed(c, count, arena, arena_bytes, offs, lens, idx, branches, roots, ok_out, leaves_out,
                           keep_dev, keep_bytes, ticket);
}

static int validate_packed(rbc_ctx *c, int count, const uint8_t *arena, size_t arena_bytes, const uint64_t *offs,
                           const uint32_t *lens, const uint8_t *idx, const uint8_t *branches, const uint8_t *roots,
                           uint8_t *ok_out, uint8_t *leaves_out, uint8_t *keep_dev, size_t keep_bytes,
                           uint64_t *ticket) {
    (void)keep_bytes;
    if (!c || count < 0 ||
        (count > 0 && (!arena || !arena_bytes || !offs || !lens || !idx || !branches || !roots || !ok_out)))
        return RBC_ERR_INVALID_ARG;
    if (count == 0) { if (ticket) *ticket = 0; return RBC_OK; }
    // every message's 64-B blocks must lie inside the arena (the kernel reads
    // whole blocks) and its leaf index inside the tree
    size_t named = 0;  // arena bytes the messages cover
    for (int i = 0; i < count; ++i) {
        if (offs[i] % 64 || lens[i] == 0 || offs[i] > arena_bytes ||
            round_up((size_t)lens[i], 64) > arena_bytes - offs[i] || idx[i] >= c->n)  // no wrap-around
            return RBC_ERR_INVALID_ARG;
        named += round_up((size_t)lens[i], 64);
    }
    const int d = c->depth;
    const size_t bslot = (size_t)std::max(d, 1) * 32;
    // a sparse arena in pinned memory (a receiver's [count][N][pitch] ECHO
    // buffer naming only the received rows): gather the named bytes over PCIe
    // instead of moving the whole arena
    const uint8_t *zc = named < arena_bytes / 4 * 3 ? host_zero_copy(arena, arena_bytes) : nullptr;
    std::lock_guard<std::mutex> lk(c->mu);
    RBC_HIP(hipSetDevice(c->device));
    Slot *sp = acquire_slot(c);
    if (!sp) return RBC_ERR_DEVICE;
    Slot &s = *sp;
    hipStream_t st = s.stream;
    if (!keep_dev) RBC_HIP(s.d_shards.ensure(arena_bytes));
    uint8_t *d_arena = keep_dev ? keep_dev : s.d_shards.as<uint8_t>();
    RBC_HIP(s.d_branches.ensure((size_t)count * bslot));
    RBC_HIP(s.d_roots.ensure((size_t)count * 32));
    RBC_HIP(s.d_slens.ensure((size_t)count * 4));
    RBC_HIP(s.d_idx.ensure((size_t)count));
    RBC_HIP(s.d_offs.ensure((size_t)count * 8));
    RBC_HIP(s.d_valid.ensure((size_t)count));
    if (leaves_out) RBC_HIP(s.d_leaves.ensure((size_t)count * 32));
    RBC_HIP(hipMemcpyAsync(s.d_offs.p, offs, (size_t)count * 8, hipMemcpyHostToDevice, st));
    RBC_HIP(hipMemcpyAsync(s.d_slens.p, lens, (size_t)count * 4, hipMemcpyHostToDevice, st));
    if (zc)
        RBC_HIP(rbc_launch_gather_msgs(zc, s.d_offs.as<uint64_t>(), s.d_slens.as<uint32_t>(), (uint32_t)count,
                                       d_arena, (uint32_t)std::min<size_t>(named / count, 0xffffffffu), st));
    else
        RBC_HIP(hipMemcpyAsync(d_arena, arena, arena_bytes, hipMemcpyHostToDevice, st));
    RBC_HIP(hipMemcpyAsync(s.d_idx.p, idx, (size_t)count, hipMemcpyHostToDevice, st));
    RBC_HIP(hipMemcpyAsync(s.d_branches.p, branches, (size_t)count * bslot, hipMemcpyHostToDevice, st));
    RBC_HIP(hipMemcpyAsync(s.d_roots.p, roots, (size_t)count * 32, hipMemcpyHostToDevice, st));
    ShaArgs a{};
    a.count = count;
    a.rows_per_inst = 1;
    a.rows = d_arena;
    a.row_offs = s.d_offs.as<uint64_t>();
    a.lens = s.d_slens.as<uint32_t>();
    a.idx = s.d_idx.as<uint8_t>();
    a.idx_stride = 1;
    a.per_message = 1;
    a.n = c->n;
    a.depth = d;
    a.branches = s.d_branches.as<uint8_t>();
    a.br_inst_pitch = bslot;
    a.roots = s.d_roots.as<uint8_t>();
    a.valid = s.d_valid.as<uint8_t>();
    a.prio = c->rx_prio;
    if (leaves_out) {  // the message's SHA-256 leaf, [count][32] (interpolate_batch_verified reuses it)
        a.leaves = s.d_leaves.as<uint8_t>();
        a.leaves_inst_pitch = 32;
    }
    RBC_HIP(rbc_launch_sha_rows(a, true, st));
    void *d_valid = s.d_valid.p, *d_lv = s.d_leaves.p;
    auto d2h = [=](hipStream_t cs) -> int {  // behind the next submission's H2D (Slot::d2h)
        RBC_HIP(hipMemcpyAsync(ok_out, d_valid, (size_t)count, hipMemcpyDeviceToHost, cs));
        if (leaves_out) RBC_HIP(hipMemcpyAsync(leaves_out, d_lv, (size_t)count * 32, hipMemcpyDeviceToHost, cs));
        return RBC_OK;
    };
    return submit(c, s, ticket, []() { return RBC_OK; }, d2h);
}

static int host_receive(rbc_ctx *c, int count, const uint8_t *shards, size_t shard_pitch, const size_t *shard_lens,
                        const uint8_t *present, const uint8_t *leaves, const uint8_t *branches, const uint8_t *roots,
                        uint8_t *valid_out, uint8_t *values_out, size_t value_pitch, uint8_t *digests_out,
                        int32_t *status_out, uint64_t *ticket, const uint8_t *const *dev_rows = nullptr);

int rbc_interpolate_batch(rbc_ctx *c, int count, const uint8_t *shards, size_t shard_pitch,
                          const size_t *shard_lens, const uint8_t *present, const uint8_t *roots,
                          uint8_t *values_out, size_t value_pitch, uint8_t *digests_out, int32_t *status_out,
                          uint64_t *ticket) {
    return rbc_interpolate_batch_verified(c, count, shards, shard_pitch, shard_lens, present, nullptr, roots,
                                          values_out, value_pitch, digests_out, status_out, ticket);
}

// leaves != NULL: the present rows were validated (rbc_validate_packed_leaves
// / the batcher's validate lane) and leaves[i][j] holds their SHA-256, so the
// device hashes only the rows interpolate regenerates (or finds changed) --
// as rbc_dev_receive_step does -- instead of all N
int rbc_interpolate_batch_verified(rbc_ctx *c, int count, const uint8_t *shards, size_t shard_pitch,
                                   const size_t *shard_lens, const uint8_t *present, const uint8_t *leaves,
                                   const uint8_t *roots, uint8_t *values_out, size_t value_pitch,
                                   uint8_t *digests_out, int32_t *status_out, uint64_t *ticket) {
    return host_receive(c, count, shards, shard_pitch, shard_lens, present, leaves, nullptr, roots, nullptr,
                        values_out, value_pitch, digests_out, status_out, ticket);
}

// Rows a rbc_validate_packed_keep left on the device: a device gather
// assembles the batch, nothing of the shards crosses PCIe again.
int rbc_interpolate_batch_kept(rbc_ctx *c, int count, const uint8_t *const *rows, const size_t *shard_lens,
                               const uint8_t *leaves, const uint8_t *roots, uint8_t *values_out, size_t value_pitch,
                               uint8_t *digests_out, int32_t *status_out, uint64_t *ticket) {
    if (!c || (count > 0 && (!rows || !shard_lens))) return RBC_ERR_INVALID_ARG;
    // every instance's first and last row must be memory a kernel can read (a pageable host
    // address would fault the gather): one attribute query at each end
    for (int i = 0; i < count; ++i) {
        const uint8_t *const *r = rows + (size_t)i * c->n;
        int lo = 0, hi = c->n - 1;
        while (lo < c->n && !r[lo]) ++lo;
        while (hi >= 0 && !r[hi]) --hi;
        if (lo <= hi && (!device_readable(r[lo], shard_lens[i]) || !device_readable(r[hi], shard_lens[i])))
            return RBC_ERR_INVALID_ARG;
    }
    return host_receive(c, count, nullptr, 0, shard_lens, nullptr, leaves, nullptr, roots, nullptr, values_out,
                        value_pitch, digests_out, status_out, ticket, rows);
}

int rbc_receive_batch(rbc_ctx *c, int count, const uint8_t *shards, size_t shard_pitch, const size_t *shard_lens,
                      const uint8_t *present, const uint8_t *branches, const uint8_t *roots, uint8_t *valid_out,
                      uint8_t *values_out, size_t value_pitch, uint8_t *digests_out, int32_t *status_out,
                      uint64_t *ticket) {
    if (count > 0 && (!branches || !valid_out)) return RBC_ERR_INVALID_ARG;
    return host_receive(c, count, shards, shard_pitch, shard_lens, present, nullptr, branches, roots, valid_out,
                        values_out, value_pitch, digests_out, status_out, ticket);
}

// The host-memory receiver behind rbc_interpolate_batch(_verified) and
// rbc_receive_batch: the present rows cross PCIe once; with `branches` the
// ECHO verify (validateMessage of every present row) runs on the device
// first and interpolate reuses its leaves; with `leaves` the caller verified
// them; with neither interpolate rehashes all N rows.
static int host_receive(rbc_ctx *c, int count, const uint8_t *shards, size_t shard_pitch, const size_t *shard_lens,
                        const uint8_t *present, const uint8_t *leaves, const uint8_t *branches, const uint8_t *roots,
                        uint8_t *valid_out, uint8_t *values_out, size_t value_pitch, uint8_t *digests_out,
                        int32_t *status_out, uint64_t *ticket, const uint8_t *const *dev_rows) {
    if (!c || count < 0 ||
        (count > 0 && (!shard_lens || !roots || !values_out || !status_out ||
                       (!dev_rows && (!shards || !present)))))
        return RBC_ERR_INVALID_ARG;
    if (count == 0) { if (ticket) *ticket = 0; return RBC_OK; }
    size_t Smax = 1;
    for (int i = 0; i < count; ++i) {
        if (shard_lens[i] > (dev_rows ? (size_t)0xffffffffu : shard_pitch)) return RBC_ERR_INVALID_ARG;
        Smax = std::max(Smax, shard_lens[i]);
    }
    if (value_pitch < (size_t)c->k * Smax) return RBC_ERR_INVALID_ARG;
    // direct H2D of a pinned, uniform-length batch; pinned staging only for
    // what is not already pinned caller memory
    bool uniform = true;
    for (int i = 0; i < count && uniform; ++i) uniform = shard_lens[i] == Smax;
    const bool in_direct = !dev_rows && uniform && host_pinned(shards, ((size_t)count * n_of(c) - 1) * shard_pitch + Smax);
    const uint8_t *zc = in_direct ? host_zero_copy(shards, ((size_t)count * n_of(c) - 1) * shard_pitch + Smax)
                                  : nullptr;
    // a pinned batch whose pitch the device rows can take moves in ONE plain
    // copy (a pitched 2-D copy runs as a blit kernel)
    const bool flat = in_direct && !zc && shard_pitch % kAlign == 0 &&
                      host_pinned(shards, (size_t)count * n_of(c) * shard_pitch);  // the flat copy's extent
    const size_t dpitch = flat ? shard_pitch : round_up(Smax, 128);
    const size_t vpitch = round_up((size_t)c->k * Smax, 16);
    if ((size_t)c->n * dpitch > 0x7fffffffULL || vpitch > 0x7fffffffULL) return RBC_ERR_INVALID_ARG;
    const int n = c->n, k = c->k, d = c->depth;
    const size_t sh_bytes = (size_t)count * n * dpitch;
    const size_t br_bytes = (size_t)count * n * std::max(d, 1) * 32;
    std::lock_guard<std::mutex> lk(c->mu);
    RBC_HIP(hipSetDevice(c->device));
    Slot *sp = acquire_slot(c);
    if (!sp) return RBC_ERR_DEVICE;
    Slot &s = *sp;
    hipStream_t st = s.stream;
    RBC_HIP(s.d_shards.ensure(sh_bytes));
    RBC_HIP(s.d_valid.ensure((size_t)count * n));
    if (branches) {
        RBC_HIP(s.d_present.ensure((size_t)count * n));
        RBC_HIP(s.d_branches.ensure(br_bytes));
    }
    // the present mask on the device: interpolate's valid mask itself, or
    // (with `branches`) the verify's input, which writes valid
    uint8_t *d_pres = branches ? s.d_present.as<uint8_t>() : s.d_valid.as<uint8_t>();
    RBC_HIP(s.d_leaves.ensure((size_t)count * n * 32));
    RBC_HIP(s.d_roots.ensure((size_t)count * 32));
    RBC_HIP(s.d_values.ensure((size_t)count * vpitch));
    RBC_HIP(s.d_digests.ensure((size_t)count * 32));
    RBC_HIP(s.d_status.ensure((size_t)count * 4));
    RBC_HIP(s.d_slens.ensure((size_t)count * 4));
    const bool out_direct = host_pinned(values_out, (size_t)(count - 1) * value_pitch + (size_t)k * Smax);
    // device rows: the [count][n] table of their addresses instead of a shard staging block
    const size_t in_stage = dev_rows ? (size_t)count * n * 8 : in_direct ? 0 : sh_bytes,
                 out_stage = out_direct ? 0 : (size_t)count * vpitch;
    RBC_HIP(s.h_in.ensure(in_stage + (size_t)count * (n + 32 + 4)));
    RBC_HIP(s.h_out.ensure(out_stage + (size_t)count * (32 + 4)));
    // [shard staging][lens u32][roots][present]: the u32 lens stay aligned for any n
    uint8_t *i_sh = s.h_in.as<uint8_t>();
    uint32_t *ln = reinterpret_cast<uint32_t *>(i_sh + in_stage);
    uint8_t *i_rt = reinterpret_cast<uint8_t *>(ln + count), *i_pr = i_rt + (size_t)count * 32;
    // present mask first: the zero-copy gather reads it
    if (dev_rows)
        for (size_t r = 0; r < (size_t)count * n; ++r) i_pr[r] = dev_rows[r] != nullptr;
    else
        memcpy(i_pr, present, (size_t)count * n);
    RBC_HIP(hipMemcpyAsync(d_pres, i_pr, (size_t)count * n, hipMemcpyHostToDevice, st));
    if (dev_rows) {  // device to device: one wave per row, zero past S_i and for absent rows
        uint64_t *tab = reinterpret_cast<uint64_t *>(i_sh);
        for (size_t r = 0; r < (size_t)count * n; ++r) tab[r] = (uint64_t)(uintptr_t)dev_rows[r];
        for (int i = 0; i < count; ++i) ln[i] = (uint32_t)shard_lens[i];
        RBC_HIP(s.d_offs.ensure((size_t)count * n * 8));
        RBC_HIP(hipMemcpyAsync(s.d_offs.p, tab, (size_t)count * n * 8, hipMemcpyHostToDevice, st));
        RBC_HIP(hipMemcpyAsync(s.d_slens.p, ln, (size_t)count * 4, hipMemcpyHostToDevice, st));
        RBC_HIP(rbc_launch_gather_ptrs(s.d_offs.as<uint64_t>(), s.d_slens.as<uint32_t>(), (uint32_t)n,
                                       s.d_shards.as<uint8_t>(), (uint32_t)dpitch, (uint32_t)(count * n), st));
    } else if (zc) {
        // only the received rows cross PCIe (N-f of N at the bench shape)
        for (int i = 0; i < count; ++i) ln[i] = (uint32_t)shard_lens[i];
        RBC_HIP(rbc_launch_gather_present(zc, shard_pitch, (uint32_t)Smax, d_pres, s.d_shards.as<uint8_t>(),
                                          (uint32_t)dpitch, (uint32_t)(count * n), st));
    } else if (flat) {  // every row, one copy; bytes past S must be zero on the device
        for (int i = 0; i < count; ++i) ln[i] = (uint32_t)shard_lens[i];
        RBC_HIP(hipMemcpyAsync(s.d_shards.p, shards, sh_bytes, hipMemcpyHostToDevice, st));
        if (dpitch > Smax)
            RBC_HIP(hipMemset2DAsync(s.d_shards.as<uint8_t>() + Smax, dpitch, 0, dpitch - Smax, (size_t)count * n, st));
    } else if (in_direct) {  // bytes past S must arrive as zero: the rows are zeroed on the device first
        for (int i = 0; i < count; ++i) ln[i] = (uint32_t)shard_lens[i];
        if (dpitch > Smax) RBC_HIP(hipMemsetAsync(s.d_shards.p, 0, sh_bytes, st));
        RBC_HIP(hipMemcpy2DAsync(s.d_shards.p, dpitch, shards, shard_pitch, Smax, (size_t)count * n,
                                 hipMemcpyHostToDevice, st));
    } else {
        parallel_for(count, (size_t)n * dpitch, [&](int i) {
            ln[i] = (uint32_t)shard_lens[i];
            for (int j = 0; j < n; ++j) {
                uint8_t *dst = i_sh + ((size_t)i * n + j) * dpitch;
                const uint8_t *src = shards + ((size_t)i * n + j) * shard_pitch;
                memcpy(dst, src, shard_lens[i]);
                memset(dst + shard_lens[i], 0, dpitch - shard_lens[i]);
            }
        });
        RBC_HIP(hipMemcpyAsync(s.d_shards.p, i_sh, sh_bytes, hipMemcpyHostToDevice, st));
    }
    memcpy(i_rt, roots, (size_t)count * 32);
    RBC_HIP(hipMemcpyAsync(s.d_roots.p, i_rt, (size_t)count * 32, hipMemcpyHostToDevice, st));
    RBC_HIP(hipMemcpyAsync(s.d_slens.p, ln, (size_t)count * 4, hipMemcpyHostToDevice, st));
    if (leaves)  // 32 B per row (1/744 of a C2 row): the whole [count][n][32] block in one copy
        RBC_HIP(hipMemcpyAsync(s.d_leaves.p, leaves, (size_t)count * n * 32, hipMemcpyHostToDevice, st));
    int rc = RBC_OK;
    if (branches) {  // validateMessage of every present row on the device, its leaves kept for interpolate
        RBC_HIP(hipMemcpyAsync(s.d_branches.p, branches, br_bytes, hipMemcpyHostToDevice, st));
        rc = stage_verify(c, st, count, s.d_shards.as<uint8_t>(), (uint32_t)dpitch, s.d_slens.as<uint32_t>(), 0,
                          s.d_branches.as<uint8_t>(), s.d_roots.as<uint8_t>(), d_pres, s.d_valid.as<uint8_t>(),
                          s.d_leaves.as<uint8_t>(), &s.ws);
        if (rc) return rc;
    }
    // ragged batch: bytes past k*S_i of a value row are returned as zero
    RBC_HIP(hipMemsetAsync(s.d_values.p, 0, (size_t)count * vpitch, st));
    rc = stage_interpolate(c, s.ws, st, count, s.d_shards.as<uint8_t>(), (uint32_t)dpitch,
                               s.d_slens.as<uint32_t>(), 0, s.d_valid.as<uint8_t>(), s.d_leaves.as<uint8_t>(),
                               (leaves || branches) ? 1 : 0,
                               s.d_roots.as<uint8_t>(), s.d_values.as<uint8_t>(), (uint32_t)vpitch,
                               s.d_digests.as<uint8_t>(), s.d_status.as<int32_t>());
    if (rc) return rc;
    uint8_t *o_val = s.h_out.as<uint8_t>(), *o_dig = o_val + out_stage;
    int32_t *o_st = reinterpret_cast<int32_t *>(o_dig + (size_t)count * 32);
    // pinned values at another pitch: the rows repacked to it on the device, then ONE copy
    // (a pitched D2H runs as one DMA per row: 2,048 of them per C4 sub-batch, ~11 us each)
    const uint64_t packed = (uint64_t)(count - 1) * value_pitch + (uint64_t)k * Smax;
    const bool pack = out_direct && value_pitch != vpitch && (uint64_t)count * value_pitch < 0xffffffffULL;
    if (pack) {
        RBC_HIP(s.d_pack.ensure((size_t)count * value_pitch));
        RBC_HIP(rbc_launch_pack_rows(s.d_values.as<uint8_t>(), (uint32_t)vpitch, s.d_pack.as<uint8_t>(),
                                     (uint32_t)value_pitch, (uint32_t)(k * Smax), (uint32_t)count, st));
    }
    void *d_val = pack ? s.d_pack.p : s.d_values.p, *d_dig = s.d_digests.p, *d_st = s.d_status.p,
         *d_vd = s.d_valid.p;
    auto d2h = [=](hipStream_t cs) -> int {
        if (valid_out) RBC_HIP(hipMemcpyAsync(valid_out, d_vd, (size_t)count * n, hipMemcpyDeviceToHost, cs));
        if (out_direct && (value_pitch == vpitch || pack))  // one contiguous DMA
            RBC_HIP(hipMemcpyAsync(values_out, d_val, (size_t)packed, hipMemcpyDeviceToHost, cs));
        else if (out_direct)
            RBC_HIP(hipMemcpy2DAsync(values_out, value_pitch, d_val, vpitch, (size_t)k * Smax, (size_t)count,
                                     hipMemcpyDeviceToHost, cs));
        else
            RBC_HIP(hipMemcpyAsync(o_val, d_val, (size_t)count * vpitch, hipMemcpyDeviceToHost, cs));
        RBC_HIP(hipMemcpyAsync(o_dig, d_dig, (size_t)count * 32, hipMemcpyDeviceToHost, cs));
        RBC_HIP(hipMemcpyAsync(o_st, d_st, (size_t)count * 4, hipMemcpyDeviceToHost, cs));
        return RBC_OK;
    };
    return submit(c, s, ticket, [=]() {
        memcpy(status_out, o_st, (size_t)count * 4);
        if (!out_direct)
            parallel_for(count, (size_t)k * Smax, [&](int i) {
                memcpy(values_out + (size_t)i * value_pitch, o_val + (size_t)i * vpitch, (size_t)k * Smax);
            });
        if (digests_out) memcpy(digests_out, o_dig, (size_t)count * 32);
        return RBC_OK;
    }, d2h);
}

// A ticket completes (its outputs land in the caller's buffers) in rbc_wait,
// in an rbc_poll that finds it done, or when its slot is needed again.
int rbc_wait(rbc_ctx *c, uint64_t ticket) {
    if (!c || ticket == 0) return RBC_ERR_INVALID_ARG;
    std::unique_lock<std::mutex> lk(c->mu);
    if (ticket >= c->next_ticket) return RBC_ERR_INVALID_ARG;
    (void)hipSetDevice(c->device);
    // Wait for the submission's completion event WITHOUT the context lock, so
    // other threads keep submitting (the batcher's validate lane launches
    // while its completer waits); then retire it under the lock -- unless
    // another thread retired it meanwhile (its status is then in `retired`).
    // A D2H still deferred is enqueued only after the kernels it follows are
    // done (Slot::kdone): enqueued earlier it would wait on them at the head
    // of the copy engine's queue, in front of the next submission's H2D.
    auto find = [&]() -> Slot * {
        for (auto &sl : c->slots)
            if (sl->busy && sl->ticket == ticket) return sl.get();
        return nullptr;
    };
    // (an event of a slot retired and reused meanwhile only waits longer; the
    // ticket's status is then in `retired`)
    if (Slot *s = find()) {
        if (s->d2h) {
            const hipEvent_t kd = s->kdone;
            lk.unlock();
            (void)hipEventSynchronize(kd);
            lk.lock();
            s = find();
            if (s) flush_d2h(*s);
        }
        if (s) {
            const hipEvent_t ev = s->done;
            lk.unlock();
            (void)hipEventSynchronize(ev);
            lk.lock();
            if ((s = find())) return retire(c, *s);
        }
    }
    auto it = c->retired.find(ticket);
    if (it == c->retired.end()) return RBC_OK;  // completed and already collected
    const int st = it->second;
    c->retired.erase(it);
    return st;
}

int rbc_poll(rbc_ctx *c, uint64_t ticket, int *done) {
    if (!c || !done || ticket == 0) return RBC_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (ticket >= c->next_ticket) return RBC_ERR_INVALID_ARG;
    *done = 1;
    for (auto &sl : c->slots)
        if (sl->busy && sl->ticket == ticket) {
            if (sl->d2h) {  // kernels still running: not done, and the D2H stays deferred (Slot::kdone)
                const hipError_t k = hipEventQuery(sl->kdone);
                if (k == hipErrorNotReady) {
                    *done = 0;
                    return RBC_OK;
                }
            }
            flush_d2h(*sl);  // nothing completes while its copies are unqueued
            const hipError_t q = hipEventQuery(sl->done);
            if (q == hipErrorNotReady) {
                *done = 0;
                return RBC_OK;
            }
            c->retired[ticket] = retire(c, *sl);  // outputs are in place; status kept for rbc_wait
            return RBC_OK;
        }
    return RBC_OK;
}

// ---- single-call drop-ins
int rbc_shard(rbc_ctx *c, const uint8_t *data, size_t len, uint8_t *shards_out, size_t shards_cap,
              size_t *shard_len_out, uint8_t *root_out, uint8_t *branches_out) {
    if (!c || !shards_out || !root_out) return RBC_ERR_INVALID_ARG;
    if (len == 0) return RBC_ERR_SHORT_DATA;
    if (!data) return RBC_ERR_INVALID_ARG;
    const size_t S = (len + c->k - 1) / c->k;
    if (shards_cap < (size_t)c->n * S) return RBC_ERR_INVALID_ARG;
    uint32_t slen = 0;
    int rc = rbc_shard_commit(c, 1, &data, &len, shards_out, S, &slen, root_out, branches_out, nullptr);
    if (rc) return rc;
    if (shard_len_out) *shard_len_out = slen;
    return RBC_OK;
}

int rbc_validate_message(rbc_ctx *c, const uint8_t *root, const uint8_t *branch, size_t branch_len,
                         const uint8_t *shard, size_t shard_len, uint32_t index, int *ok) {
    if (!c || !ok || !root) return RBC_ERR_INVALID_ARG;
    *ok = 0;
    if (!shard || shard_len == 0) return RBC_OK;
    uint8_t r = 0;
    int rc = rbc_validate_batch(c, 1, &shard, &shard_len, &index, &branch, &branch_len, &root, &r, nullptr);
    if (rc) return rc;
    *ok = r;
    return RBC_OK;
}

// Single-call interpolate: each present shard is copied once, from the
// caller's pointer straight into the slot's pinned staging row (no
// intermediate buffer), and the value comes back through pinned memory.
int rbc_interpolate(rbc_ctx *c, const uint8_t *root, const uint8_t *const *shards, const size_t *lens,
                    uint8_t *value_out, size_t value_cap, size_t *value_len, uint8_t *digest_out) {
    if (!c || !root || !shards || !lens || !value_out) return RBC_ERR_INVALID_ARG;
    size_t S = 0;
    int rc = check_shards(lens, c->n, true, &S);
    if (rc) return rc;
    int present = 0;
    for (int i = 0; i < c->n; ++i) {
        present += lens[i] != 0;
        if (lens[i] && !shards[i]) return RBC_ERR_INVALID_ARG;
    }
    if (present < c->k) return RBC_ERR_TOO_FEW_SHARDS;  // rbc/rbc.go:87
    if (value_cap < (size_t)c->k * S) return RBC_ERR_INVALID_ARG;
    const int n = c->n, k = c->k;
    const size_t dpitch = round_up(S, 128), vpitch = round_up((size_t)k * S, 16);
    if ((size_t)n * dpitch > 0x7fffffffULL || vpitch > 0x7fffffffULL) return RBC_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    RBC_HIP(hipSetDevice(c->device));
    Slot *sp = acquire_slot(c);
    if (!sp) return RBC_ERR_DEVICE;
    Slot &s = *sp;
    hipStream_t st = s.stream;
    const size_t sh_bytes = (size_t)n * dpitch;
    RBC_HIP(s.d_shards.ensure(sh_bytes));
    const size_t npad = round_up((size_t)n, 64);  // root after the present flags, 64-B aligned
    RBC_HIP(s.d_valid.ensure(npad + 32));
    RBC_HIP(s.d_leaves.ensure((size_t)n * 32));
    RBC_HIP(s.d_values.ensure(vpitch));
    RBC_HIP(s.d_digests.ensure(32));
    RBC_HIP(s.d_status.ensure(4));
    RBC_HIP(s.h_in.ensure(sh_bytes + npad + 32));
    RBC_HIP(s.h_out.ensure(vpitch + 32 + 4));
    uint8_t *i_sh = s.h_in.as<uint8_t>(), *i_pr = i_sh + sh_bytes, *i_rt = i_pr + npad;
    memset(i_pr, 0, npad);
    for (int j = 0; j < n; ++j) {
        uint8_t *dst = i_sh + (size_t)j * dpitch;
        if (lens[j]) {
            memcpy(dst, shards[j], S);
            memset(dst + S, 0, dpitch - S);
        } else {
            memset(dst, 0, dpitch);
        }
        i_pr[j] = lens[j] ? 1 : 0;
    }
    memcpy(i_rt, root, 32);
    RBC_HIP(hipMemcpyAsync(s.d_shards.p, i_sh, sh_bytes, hipMemcpyHostToDevice, st));
    RBC_HIP(hipMemcpyAsync(s.d_valid.p, i_pr, npad + 32, hipMemcpyHostToDevice, st));  // present + root
    const uint8_t *d_root = s.d_valid.as<uint8_t>() + npad;
    rc = stage_interpolate(c, s.ws, st, 1, s.d_shards.as<uint8_t>(), (uint32_t)dpitch, nullptr, (uint32_t)S,
                           s.d_valid.as<uint8_t>(), s.d_leaves.as<uint8_t>(), 0, d_root, s.d_values.as<uint8_t>(),
                           (uint32_t)vpitch, s.d_digests.as<uint8_t>(), s.d_status.as<int32_t>());
    if (rc) return rc;
    uint8_t *o_val = s.h_out.as<uint8_t>(), *o_dig = o_val + vpitch;
    int32_t *o_st = reinterpret_cast<int32_t *>(o_dig + 32);
    RBC_HIP(hipMemcpyAsync(o_val, s.d_values.p, vpitch, hipMemcpyDeviceToHost, st));
    RBC_HIP(hipMemcpyAsync(o_dig, s.d_digests.p, 32, hipMemcpyDeviceToHost, st));
    RBC_HIP(hipMemcpyAsync(o_st, s.d_status.p, 4, hipMemcpyDeviceToHost, st));
    int32_t status = 0;
    rc = submit(c, s, nullptr, [&]() {
        status = *o_st;
        if (!status) {
            memcpy(value_out, o_val, (size_t)k * S);
            if (digest_out) memcpy(digest_out, o_dig, 32);
        }
        return RBC_OK;
    });
    if (rc) return rc;
    if (status) return status;
    if (value_len) *value_len = (size_t)k * S;
    return RBC_OK;
}

// ---- reedsolomon.Encoder mirror
int rbc_rs_new(int data_shards, int parity_shards, int device, rbc_rs **out) {
    if (!out) return RBC_ERR_INVALID_ARG;
    *out = nullptr;
    if (data_shards <= 0 || parity_shards < 0) return RBC_ERR_INV_SHARD_NUM;
    if (data_shards + parity_shards > 256) return RBC_ERR_MAX_SHARD_NUM;
    rbc_ctx *c = nullptr;
    int rc = ctx_create_kn(data_shards + parity_shards, data_shards, device, &c);
    if (rc) return rc;
    *out = new rbc_rs{c};
    return RBC_OK;
}

void rbc_rs_free(rbc_rs *rs) {
    if (!rs) return;
    rbc_ctx_destroy(rs->ctx);
    delete rs;
}

static int rs_parity(rbc_ctx *c, const uint8_t *const *shards, size_t S, std::vector<uint8_t> &parity) {
    // parity of the data shards, computed by the GPU encode kernel
    const size_t dpitch = round_up(S, kAlign);
    const size_t vpitch = round_up((size_t)c->k * S + 32, kAlign);
    if (vpitch > 0x7fffffffULL || (size_t)c->n * dpitch > 0x7fffffffULL) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(c->device));
    hipStream_t st = host_stream(c);
    if (!st) return RBC_ERR_DEVICE;
    RBC_HIP(c->h_stage.ensure(std::max(vpitch, (size_t)c->n * dpitch)));
    RBC_HIP(c->d_values.ensure(vpitch));
    RBC_HIP(c->d_shards.ensure((size_t)c->n * dpitch));
    uint8_t *stage = c->h_stage.as<uint8_t>();
    memset(stage, 0, vpitch);
    for (int j = 0; j < c->k; ++j) memcpy(stage + (size_t)j * S, shards[j], S);
    RBC_HIP(hipMemcpyAsync(c->d_values.p, stage, vpitch, hipMemcpyHostToDevice, st));
    int rc = stage_encode(c, st, 1, c->d_values.as<uint8_t>(), vpitch, nullptr, (uint32_t)((size_t)c->k * S),
                          c->d_shards.as<uint8_t>(), (uint32_t)dpitch);
    if (rc) return rc;
    parity.assign((size_t)c->p * S, 0);
    if (c->p > 0)
        RBC_HIP(hipMemcpy2DAsync(parity.data(), S, c->d_shards.as<uint8_t>() + (size_t)c->k * dpitch, dpitch, S,
                                 c->p, hipMemcpyDeviceToHost, st));
    RBC_HIP(hipStreamSynchronize(st));
    return RBC_OK;
}

int rbc_rs_encode(rbc_rs *rs, uint8_t *const *shards, const size_t *lens, int n_shards) {
    if (!rs || !shards || !lens) return RBC_ERR_INVALID_ARG;
    rbc_ctx *c = rs->ctx;
    if (n_shards != c->n) return RBC_ERR_TOO_FEW_SHARDS;
    size_t S = 0;
    int rc = check_shards(lens, n_shards, false, &S);
    if (rc) return rc;
    for (int i = 0; i < c->n; ++i)
        if (!shards[i]) return RBC_ERR_INVALID_ARG;
    std::vector<uint8_t> parity;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        rc = rs_parity(c, shards, S, parity);
    }
    if (rc) return rc;
    for (int r = 0; r < c->p; ++r) memcpy(shards[c->k + r], parity.data() + (size_t)r * S, S);
    return RBC_OK;
}

int rbc_rs_verify(rbc_rs *rs, const uint8_t *const *shards, const size_t *lens, int n_shards, int *ok) {
    if (!rs || !shards || !lens || !ok) return RBC_ERR_INVALID_ARG;
    rbc_ctx *c = rs->ctx;
    *ok = 0;
    if (n_shards != c->n) return RBC_ERR_TOO_FEW_SHARDS;
    size_t S = 0;
    int rc = check_shards(lens, n_shards, false, &S);
    if (rc) return rc;
    for (int i = 0; i < c->n; ++i)
        if (!shards[i]) return RBC_ERR_INVALID_ARG;
    std::vector<uint8_t> parity;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        rc = rs_parity(c, shards, S, parity);
    }
    if (rc) return rc;
    int good = 1;
    for (int r = 0; r < c->p && good; ++r) good = memcmp(shards[c->k + r], parity.data() + (size_t)r * S, S) == 0;
    *ok = good;
    return RBC_OK;
}

// klauspost v1.9.1 Update / updateParityShards (reedsolomon.go): for every
// changed data shard c (new_lens[c] != 0), delta = old ^ new is left in
// shards[c] (Go's sliceXor(in, oldin) writes into oldin) and every parity
// shard gains M[k+r][c] * delta.  The GF(2^8) product runs on the GPU
// (gf_rows, one launch for all changed shards); the xors are host memory ops.
int rbc_rs_update(rbc_rs *rs, uint8_t *const *shards, const size_t *lens, int n_shards,
                  const uint8_t *const *new_data, const size_t *new_lens, int n_new) {
    if (!rs || !shards || !lens || !new_data || !new_lens) return RBC_ERR_INVALID_ARG;
    rbc_ctx *c = rs->ctx;
    // Go: len(shards) != r.Shards, len(newDatashards) != r.DataShards -> ErrTooFewShards
    if (n_shards != c->n) return RBC_ERR_TOO_FEW_SHARDS;
    if (n_new != c->k) return RBC_ERR_TOO_FEW_SHARDS;
    size_t S = 0, S2 = 0;
    int rc = check_shards(lens, n_shards, true, &S);
    if (rc) return rc;
    rc = check_shards(new_lens, n_new, true, &S2);
    if (rc) return rc;
    for (int i = 0; i < n_new; ++i)
        if (new_lens[i] && !lens[i]) return RBC_ERR_INVALID_INPUT;
    for (int r = c->k; r < c->n; ++r)
        if (!lens[r]) return RBC_ERR_INVALID_INPUT;
    std::vector<int> changed;
    for (int j = 0; j < c->k; ++j)
        if (new_lens[j]) changed.push_back(j);
    if (changed.empty() || c->p == 0) return RBC_OK;
    if (S2 != S) return RBC_ERR_SHARD_SIZE;  // Go would index past the shorter slice
    for (int j : changed)
        if (!shards[j] || !new_data[j]) return RBC_ERR_INVALID_ARG;
    for (int r = c->k; r < c->n; ++r)
        if (!shards[r]) return RBC_ERR_INVALID_ARG;
    const int K = (int)changed.size(), P = c->p;
    const size_t pitch = round_up(S, kAlign);
    if ((size_t)(K + P) * pitch > 0x7fffffffULL) return RBC_ERR_INVALID_ARG;
    // delta rows (host xor, written back into the caller's old data shards)
    for (int j : changed)
        for (size_t x = 0; x < S; ++x) shards[j][x] ^= new_data[j][x];
    std::lock_guard<std::mutex> lk(c->mu);
    RBC_HIP(hipSetDevice(c->device));
    hipStream_t st = host_stream(c);
    if (!st) return RBC_ERR_DEVICE;
    const size_t rows_bytes = (size_t)(K + P) * pitch, meta = (size_t)P * K + 512;
    RBC_HIP(c->h_stage.ensure(rows_bytes + meta));
    RBC_HIP(c->d_shards.ensure(rows_bytes));
    RBC_HIP(c->d_values.ensure(meta));
    uint8_t *stage = c->h_stage.as<uint8_t>();
    memset(stage, 0, (size_t)K * pitch);
    for (int t = 0; t < K; ++t) memcpy(stage + (size_t)t * pitch, shards[changed[t]], S);
    uint8_t *coef = stage + rows_bytes, *in_idx = coef + (size_t)P * K, *out_idx = in_idx + 256;
    for (int r = 0; r < P; ++r)
        for (int t = 0; t < K; ++t) coef[(size_t)r * K + t] = c->h_M[(size_t)(c->k + r) * c->k + changed[t]];
    for (int t = 0; t < K; ++t) in_idx[t] = (uint8_t)t;
    for (int r = 0; r < P; ++r) out_idx[r] = (uint8_t)(K + r);
    RBC_HIP(hipMemcpyAsync(c->d_shards.p, stage, (size_t)K * pitch, hipMemcpyHostToDevice, st));
    RBC_HIP(hipMemcpyAsync(c->d_values.p, coef, meta, hipMemcpyHostToDevice, st));
    const uint8_t *d_coef = c->d_values.as<uint8_t>();
    GfArgs g{};
    g.count = 1;
    g.tiles = (int)((pitch + 4095) / 4096);
    g.R = P;
    g.K = K;
    g.rc = rbc_gf_pick_rc(P, kGfRcMax);
    g.mode = GF_MODE_DECODE;
    g.in = c->d_shards.as<uint8_t>();
    g.in_inst_pitch = rows_bytes;
    g.in_row_pitch = (uint32_t)pitch;
    g.in_inst_bytes = (uint32_t)rows_bytes;
    g.out = c->d_shards.as<uint8_t>();
    g.out_inst_pitch = rows_bytes;
    g.out_row_pitch = (uint32_t)pitch;
    g.uniform_len = (uint32_t)S;
    g.coef = d_coef;
    g.in_idx = d_coef + (size_t)P * K;
    g.out_idx = g.in_idx + 256;
    g.idx_stride = (uint32_t)K;
    g.idx_stride2 = (uint32_t)P;
    RBC_HIP(rbc_launch_gf_rows(g, st));
    RBC_HIP(hipMemcpy2DAsync(stage, S, c->d_shards.as<uint8_t>() + (size_t)K * pitch, pitch, S, P,
                             hipMemcpyDeviceToHost, st));
    RBC_HIP(hipStreamSynchronize(st));
    for (int r = 0; r < P; ++r) {
        uint8_t *dst = shards[c->k + r];
        const uint8_t *d = stage + (size_t)r * S;
        for (size_t x = 0; x < S; ++x) dst[x] ^= d[x];
    }
    return RBC_OK;
}

int rbc_rs_reconstruct(rbc_rs *rs, uint8_t *const *shards, size_t *lens, int n_shards) {
    if (!rs) return RBC_ERR_INVALID_ARG;
    return host_reconstruct(rs->ctx, shards, lens, n_shards, false);
}

int rbc_rs_reconstruct_data(rbc_rs *rs, uint8_t *const *shards, size_t *lens, int n_shards) {
    if (!rs) return RBC_ERR_INVALID_ARG;
    return host_reconstruct(rs->ctx, shards, lens, n_shards, true);
}

int rbc_rs_split(rbc_rs *rs, const uint8_t *data, size_t len, uint8_t *out, size_t out_cap, size_t *per_shard) {
    if (!rs || !out || !per_shard) return RBC_ERR_INVALID_ARG;
    rbc_ctx *c = rs->ctx;
    if (len == 0) return RBC_ERR_SHORT_DATA;
    if (!data) return RBC_ERR_INVALID_ARG;
    const size_t per = (len + c->k - 1) / c->k;
    if (out_cap < (size_t)c->n * per) return RBC_ERR_INVALID_ARG;
    memcpy(out, data, len);
    memset(out + len, 0, (size_t)c->n * per - len);
    *per_shard = per;
    return RBC_OK;
}

int rbc_rs_join(rbc_rs *rs, const uint8_t *const *shards, const size_t *lens, int n_shards, size_t out_size,
                uint8_t *dst) {
    if (!rs || !shards || !lens || (!dst && out_size)) return RBC_ERR_INVALID_ARG;
    rbc_ctx *c = rs->ctx;
    if (n_shards < c->k) return RBC_ERR_TOO_FEW_SHARDS;
    size_t size = 0;
    for (int i = 0; i < c->k; ++i) {
        if (!shards[i]) return RBC_ERR_RECONSTRUCT_REQUIRED;
        size += lens[i];
        if (size >= out_size) break;
    }
    if (size < out_size) return RBC_ERR_SHORT_DATA;
    size_t write = out_size, off = 0;
    for (int i = 0; i < c->k && write; ++i) {
        const size_t w = std::min(write, lens[i]);
        memcpy(dst + off, shards[i], w);
        off += w;
        write -= w;
    }
    return RBC_OK;
}

// ---- multi-GPU
int rbc_comm_unique_id(uint8_t id_out[128]) {
    if (!id_out) return RBC_ERR_INVALID_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return RBC_ERR_DEVICE;
    memcpy(id_out, id.internal, 128);
    return RBC_OK;
}

int rbc_comm_init(rbc_ctx *c, int nranks, int rank, const uint8_t id[128]) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return RBC_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    RBC_HIP(hipSetDevice(c->device));
    if (c->comm) { (void)ncclCommDestroy(c->comm); c->comm = nullptr; }
    ncclUniqueId uid;
    memcpy(uid.internal, id, 128);
    if (ncclCommInitRank(&c->comm, nranks, uid, rank) != ncclSuccess) { c->comm = nullptr; return RBC_ERR_DEVICE; }
    c->nranks = nranks;
    c->rank = rank;
    return RBC_OK;
}

int rbc_comm_destroy(rbc_ctx *c) {
    if (!c) return RBC_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    c->comm = nullptr;
    c->nranks = 1;
    c->rank = 0;
    return RBC_OK;
}

int rbc_dev_allgather_roots(rbc_ctx *c, void *stream, int count, const uint8_t *roots, const uint8_t *digests,
                            uint8_t *gathered) {
    if (!c || count < 0 || (count > 0 && (!roots || !gathered))) return RBC_ERR_INVALID_ARG;
    if (!c->comm) return RBC_ERR_NO_COMM;
    if (count == 0) return RBC_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    RBC_HIP(hipSetDevice(c->device));
    hipStream_t st = as_stream(stream);
    RBC_HIP(c->d_pack.ensure((size_t)count * 64));
    RBC_HIP(hipMemcpy2DAsync(c->d_pack.p, 64, roots, 32, 32, count, hipMemcpyDeviceToDevice, st));
    if (digests)
        RBC_HIP(hipMemcpy2DAsync(c->d_pack.as<uint8_t>() + 32, 64, digests, 32, 32, count, hipMemcpyDeviceToDevice,
                                 st));
    else
        RBC_HIP(hipMemset2DAsync(c->d_pack.as<uint8_t>() + 32, 64, 0, 32, count, st));
    if (ncclAllGather(c->d_pack.p, gathered, (size_t)count * 64, ncclUint8, c->comm, st) != ncclSuccess)
        return RBC_ERR_DEVICE;
    return RBC_OK;
}

int rbc_dev_allgather_records(rbc_ctx *c, void *stream, int count, int slots, const uint8_t *roots,
                              const uint8_t *digests, const int32_t *status, uint8_t *gathered) {
    if (!c || count < 0 || slots < count || (count > 0 && !roots) || (slots > 0 && !gathered))
        return RBC_ERR_INVALID_ARG;
    if (!c->comm) return RBC_ERR_NO_COMM;
    if (slots == 0) return RBC_OK;  // every rank passes the same slots: all skip together
    std::lock_guard<std::mutex> lk(c->mu);
    RBC_HIP(hipSetDevice(c->device));
    hipStream_t st = as_stream(stream);
    RBC_HIP(c->d_pack.ensure((size_t)slots * 64));
    RBC_HIP(rbc_launch_pack_records(roots, digests, status, count, slots, c->d_pack.as<uint8_t>(), st));
    if (ncclAllGather(c->d_pack.p, gathered, (size_t)slots * 64, ncclUint8, c->comm, st) != ncclSuccess)
        return RBC_ERR_DEVICE;
    return RBC_OK;
}

static void copy_path(const void *sym, char *out, size_t cap) {
    if (!out || cap == 0) return;
    out[0] = 0;
    Dl_info info;
    if (!dladdr(sym, &info) || !info.dli_fname) return;
    char buf[PATH_MAX];
    const char *p = realpath(info.dli_fname, buf) ? buf : info.dli_fname;
    snprintf(out, cap, "%s", p);
}

int rbc_comm_info(rbc_ctx *c, int *nranks, int *rank, int *rccl_version, char *rccl_path, size_t rccl_cap,
                  int *hip_runtime_version, char *hip_path, size_t hip_cap) {
    if (!c) return RBC_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (rccl_version && ncclGetVersion(rccl_version) != ncclSuccess) return RBC_ERR_DEVICE;
    if (hip_runtime_version && hipRuntimeGetVersion(hip_runtime_version) != hipSuccess) return RBC_ERR_DEVICE;
    copy_path(reinterpret_cast<const void *>(&ncclAllGather), rccl_path, rccl_cap);
    copy_path(reinterpret_cast<const void *>(&hipDeviceSynchronize), hip_path, hip_cap);
    if (nranks || rank) {
        if (!c->comm) return RBC_ERR_NO_COMM;
        int nr = 0, r = 0;
        if (ncclCommCount(c->comm, &nr) != ncclSuccess || ncclCommUserRank(c->comm, &r) != ncclSuccess)
            return RBC_ERR_DEVICE;
        if (nranks) *nranks = nr;
        if (rank) *rank = r;
    }
    return RBC_OK;
}

int rbc_device_mem_info(int device, size_t *free_bytes, size_t *total_bytes) {
    if (!free_bytes || !total_bytes) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(device));
    RBC_HIP(hipMemGetInfo(free_bytes, total_bytes));
    return RBC_OK;
}

int rbc_device_pci_bus_id(int device, char *out, int cap) {
    if (!out || cap < 13) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipDeviceGetPCIBusId(out, cap, device));
    return RBC_OK;
}

// ---- ACS output-set assembly (host)
int rbc_acs_partition(int total, int nranks, int rank, int *first, int *count) {
    if (total < 0 || nranks < 1 || rank < 0 || rank >= nranks || !first || !count) return RBC_ERR_INVALID_ARG;
    const int64_t a = (int64_t)rank * total / nranks, b = (int64_t)(rank + 1) * total / nranks;
    *first = (int)a;
    *count = (int)(b - a);
    return RBC_OK;
}

int rbc_acs_max_share(int total, int nranks, int *slots) {
    if (total < 0 || nranks < 1 || !slots) return RBC_ERR_INVALID_ARG;
    *slots = (int)(((int64_t)total + nranks - 1) / nranks);  // = the largest contiguous share
    return RBC_OK;
}

int rbc_acs_assemble(const uint8_t *gathered, int nranks, int slots, int total, int32_t *instances_out,
                     uint8_t *records_out, int *out_count) {
    if (!out_count || nranks < 1 || slots < 0 || total < 0 || (total > 0 && (!gathered || !instances_out)))
        return RBC_ERR_INVALID_ARG;
    int m = 0;
    for (int r = 0; r < nranks; ++r) {
        int first = 0, cnt = 0;
        rbc_acs_partition(total, nranks, r, &first, &cnt);
        if (cnt > slots) return RBC_ERR_INVALID_ARG;  // gather buffer smaller than a share
        for (int t = 0; t < cnt; ++t) {
            const uint8_t *rec = gathered + ((size_t)r * slots + t) * 64;
            uint8_t any = 0;
            for (int q = 32; q < 64; ++q) any |= rec[q];
            if (!any) continue;  // zero digest: interpolate failed, not in the set
            instances_out[m] = first + t;
            if (records_out) memcpy(records_out + (size_t)m * 64, rec, 64);
            ++m;
        }
    }
    *out_count = m;
    return RBC_OK;
}

// ---- test / bench utilities
int rbc_dev_fill_random(int device, void *stream, uint8_t *dst, uint64_t first_row, uint64_t rows, uint64_t pitch,
                        uint64_t seed) {
    if ((!dst && rows) || pitch % 16) return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(device));
    RBC_HIP(rbc_launch_fill_random(dst, first_row, rows, pitch, seed, as_stream(stream)));
    return RBC_OK;
}

int rbc_dev_count_mismatch(int device, void *stream, const uint8_t *a, uint64_t a_pitch, const uint8_t *b,
                           uint64_t b_pitch, uint64_t rows, uint64_t len, uint32_t *mismatch_dev) {
    if (!mismatch_dev || (rows && len && (!a || !b))) return RBC_ERR_INVALID_ARG;
    if (a_pitch % 16 || b_pitch % 16 || len > a_pitch || len > b_pitch || ((uintptr_t)a | (uintptr_t)b) % 16)
        return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(device));
    hipStream_t st = as_stream(stream);
    RBC_HIP(hipMemsetAsync(mismatch_dev, 0, sizeof(uint32_t), st));
    RBC_HIP(rbc_launch_count_mismatch(a, a_pitch, b, b_pitch, rows, len, mismatch_dev, st));
    return RBC_OK;
}

int rbc_dev_count_mismatch_rows(int device, void *stream, const uint8_t *shards, uint64_t inst_pitch,
                                uint32_t row_pitch, int k, uint32_t shard_len, const uint8_t *values,
                                uint64_t value_pitch, uint32_t value_len, uint64_t count, uint32_t *mismatch_dev) {
    if (!mismatch_dev || k <= 0 || (count && (!shards || !values))) return RBC_ERR_INVALID_ARG;
    if (row_pitch % 16 || inst_pitch % 16 || (uintptr_t)shards % 16 || shard_len > row_pitch ||
        value_pitch < (uint64_t)k * shard_len + 16 || value_pitch > 0x7fffffffULL ||
        value_len > (uint64_t)k * shard_len || (uint64_t)k * row_pitch > inst_pitch)
        return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(device));
    hipStream_t st = as_stream(stream);
    RBC_HIP(hipMemsetAsync(mismatch_dev, 0, sizeof(uint32_t), st));
    RBC_HIP(rbc_launch_count_mismatch_rows(shards, inst_pitch, row_pitch, k, shard_len, values, value_pitch, value_len,
                                           count, mismatch_dev, st));
    return RBC_OK;
}

int rbc_dev_poison_rows(int device, void *stream, uint8_t *shards, uint64_t inst_pitch, uint32_t row_pitch, int n,
                        const uint8_t *present, const int32_t *corrupt, uint64_t count, uint64_t seed) {
    if (n <= 0 || (count && !shards) || row_pitch % 16 || inst_pitch % 16 || (uintptr_t)shards % 16 ||
        (uint64_t)n * row_pitch > inst_pitch)
        return RBC_ERR_INVALID_ARG;
    RBC_HIP(hipSetDevice(device));
    RBC_HIP(rbc_launch_poison_rows(shards, inst_pitch, row_pitch, n, present, corrupt, count, seed,
                                   as_stream(stream)));
    return RBC_OK;
}

}  // extern "C"
