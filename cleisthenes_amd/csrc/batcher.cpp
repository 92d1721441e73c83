// batcher.cpp -- request coalescing for the RBC data path (C++ host runtime).
//
// Each RBC instance in the reference runs its own goroutine event loop
// (rbc/rbc.go:78 run(), channels at rbc/rbc.go:31-33), so shard /
// validateMessage / interpolate calls arrive one at a time from thousands of
// goroutines.  The GPU only pays off when many instances share a launch
// (BASELINE north_star (4)).  A batcher accepts single-instance requests from
// any number of threads, coalesces them per kind into one batched call
// (rbc_shard_commit / rbc_validate_batch / rbc_interpolate_batch) when
// `max_batch` requests are queued or the oldest has waited `max_wait_us`,
// and completes per-request tickets; callers block in rbc_batcher_wait or
// poll (no C -> Go callbacks).  Caller buffers must stay valid until their
// ticket completes (the cgo shim keeps the Go slices alive until then).
// Launches are submitted asynchronously (the context's host-API slots), so
// while batch t runs on the GPU the worker already stages batch t+1.  The
// batch-shaped shard / value buffers are pinned (rbc_host_alloc) and pooled,
// so the C API moves them with direct DMA (or the zero-copy gather of the
// present rows) instead of staging them once more.
//
// validateMessage has its own lane (round 5): it is called once per ECHO --
// N-f per instance per node, 88 k per C2 epoch of 1,024 instances -- so the
// per-request work must not funnel through one thread.  The CALLING thread
// reserves a slot in the open pinned arena (a short critical section), copies
// its shard, branch and root there in the device layout, and leaves; a lane
// worker seals the arena when it is full or its first message has waited
// max_wait_us and hands it to rbc_validate_packed (one DMA, one launch), up to
// kVInflight arenas in flight.  Results land in the callers' ok_out, tickets
// complete in arena order.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/rbc_gpu.h"

namespace {

// K_INTERPV: interpolate with the validate lane's leaves (rbc_batcher_interpolate_verified);
// K_INTERPK: interpolate whose every present shard the lane kept on the device (rbc_batcher_set_keep)
enum Kind { K_SHARD = 0, K_VALIDATE = 1, K_INTERP = 2, K_INTERPV = 3, K_INTERPK = 4 };
constexpr int kKinds = 5;

struct Req {
    uint64_t ticket;
    Kind kind;
    std::chrono::steady_clock::time_point t0;
    // shard
    const uint8_t *data = nullptr;
    size_t len = 0;
    uint8_t *shards_out = nullptr;
    size_t shards_cap = 0;
    size_t *shard_len_out = nullptr;
    uint8_t *root_out = nullptr;
    uint8_t *branches_out = nullptr;
    // interpolate
    const uint8_t *root = nullptr;
    std::vector<const uint8_t *> in_shards;
    std::vector<size_t> in_lens;
    uint8_t *value_out = nullptr;
    size_t value_cap = 0;
    size_t *value_len = nullptr;
    uint8_t *digest_out = nullptr;
    const uint8_t *leaves = nullptr;  // K_INTERPV: n x 32, the leaves of the present shards
    // K_INTERPK: the kept rows' device addresses (n, NULL = absent), their
    // leaves (n x 32) and the keep regions they pin until the launch completes
    std::vector<uint64_t> dev_rows;
    std::vector<uint8_t> kleaves;
    std::vector<uint64_t> kgens;
};

// Per-request copies between the callers' buffers and a launch's pinned
// buffers run on several threads once a batch moves more than a few MiB (one
// thread's memcpy, ~10 GB/s, would bound the coalescer far below PCIe).
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

// Growable pinned host buffer (rbc_host_alloc), reused across launches.
struct Pinned {
    uint8_t *p = nullptr;
    size_t cap = 0;
    uint8_t *ensure(size_t bytes) {
        if (bytes <= cap && p) return p;
        if (p) rbc_host_free(p);
        p = nullptr;
        cap = 0;
        void *q = nullptr;
        if (rbc_host_alloc(std::max<size_t>(bytes, 256), &q) != RBC_OK) return nullptr;
        p = static_cast<uint8_t *>(q);
        cap = std::max<size_t>(bytes, 256);
        return p;
    }
    ~Pinned() {
        if (p) rbc_host_free(p);
    }
};

// The pinned buffers of one launch: shards, roots, branches / values.
struct PinnedSet {
    Pinned shards, roots, br, values, leaves;
};

// One arena of the validate lane: the messages of one launch in the layout
// rbc_validate_packed reads (shard bytes at 64-B aligned offsets, device-form
// branches, roots, leaf indices), the verdicts, and the callers' ok_out.
struct VBuf {
    enum State { FREE, OPEN, SEALED, INFLIGHT };
    Pinned arena, meta;
    uint64_t *offs = nullptr;
    uint32_t *lens = nullptr;
    uint8_t *roots = nullptr, *br = nullptr, *idx = nullptr, *ok = nullptr, *shape = nullptr, *lv = nullptr;
    std::vector<int *> out;
    std::vector<uint8_t *> lout;     // callers' leaf_out (rbc_batcher_validate_leaf), nullable
    std::vector<const uint8_t *> hostp;  // callers' shard pointers (the keep index's identity check)
    uint8_t *keep_dev = nullptr;     // this launch's region of the keep ring (NULL: not kept)
    uint64_t keep_gen = 0;
    std::atomic<bool> any_leaf{false};  // some slot asked for its leaf (set before the caller's pend add)
    int cap = 0;                     // messages the meta block holds
    // Copies done, then at seal time + (kSealed - count): == kSealed exactly
    // when the arena is sealed and every reserved slot copied.  One atomic
    // add per message (the caller's, after its copy); only the returned values
    // are used, so a caller touches nothing of the arena after it (by then the
    // arena may already be launched, completed and reopened).
    static constexpr int64_t kSealed = (int64_t)1 << 40;
    alignas(64) std::atomic<int64_t> pend{0};
    // Reservations: ONE atomic add per message of (1 << 40 | bytes) to `word`
    // (slot = old count, offset = old bytes).  A reservation whose slot is
    // < cap but whose bytes do not fit leaves a hole (its slot is launched as
    // an empty message).  Sealing adds kBump to the count so later adds fail;
    // count / bytes below are the final values the seal takes from `word`.
    static constexpr uint64_t kCountOne = (uint64_t)1 << 40, kBytesMask = kCountOne - 1;
    static constexpr uint64_t kBump = (uint64_t)1 << 62;
    alignas(64) std::atomic<uint64_t> word{0};
    alignas(64) int count = 0;       // slots launched (final at the seal)
    size_t bytes = 0;                // arena bytes launched (final at the seal)
    uint64_t seen = 0;               // the launcher's last sample of the slot count (quiet detection)
    std::chrono::steady_clock::time_point t0, t_seen;  // opening / when `seen` last changed
    alignas(64) uint64_t gen = 0;    // launch generation (tickets complete in this order)
    State state = FREE;              // under vmu
    uint64_t ticket = 0;
    int rc = RBC_OK;
    bool layout(int msgs, int bslot) {  // the meta block for `msgs` messages
        const size_t per = 8 + 4 + 32 + (size_t)bslot + 3 + 32;
        if (!meta.ensure((size_t)msgs * per)) return false;
        uint8_t *p = meta.p;
        offs = reinterpret_cast<uint64_t *>(p);
        lens = reinterpret_cast<uint32_t *>(p + (size_t)msgs * 8);
        roots = p + (size_t)msgs * 12;
        br = roots + (size_t)msgs * 32;
        idx = br + (size_t)msgs * bslot;
        ok = idx + msgs;
        shape = ok + msgs;
        lv = shape + msgs;  // [msgs][32] leaves (only when a slot asked for one)
        cap = msgs;
        out.assign(msgs, nullptr);
        lout.assign(msgs, nullptr);
        hostp.assign(msgs, nullptr);
        return true;
    }
};
constexpr uint64_t kVTicket = 1ull << 63;  // validate-lane tickets: kVTicket | gen << 20 | slot
constexpr int kVSlotBits = 20;

// Device-resident ECHO rows (ABI 7, rbc_batcher_set_keep).  Each validate
// launch moves its arena into the next region of a device ring instead of a
// launch buffer (rbc_validate_packed_keep); every message that validated is
// indexed by (root, leaf index) with the caller's shard pointer and length and
// its leaf.  An interpolate whose every present shard is indexed -- the same
// pointer and length the caller validated -- reads the rows on the device
// (rbc_interpolate_batch_kept): the drop-in's ECHO rows then cross PCIe once.
// A region is reused only when nothing uses it (its validate has completed
// and no interpolate that reads it is in flight); when the next region is
// still in use the launch is simply not kept, and an interpolate that misses
// any shard takes the host path: keeping never changes a result.
struct KeepKey {
    uint8_t root[32];
    uint32_t idx;
    bool operator==(const KeepKey &o) const { return idx == o.idx && !memcmp(root, o.root, 32); }
};
struct KeepKeyHash {
    size_t operator()(const KeepKey &k) const {  // roots are SHA-256 digests: 8 of their bytes spread well
        uint64_t h;
        memcpy(&h, k.root, 8);
        return (size_t)(h ^ ((uint64_t)k.idx * 0x9e3779b97f4a7c15ull));
    }
};
struct KeepEntry {
    uint64_t gen;           // the region's generation when inserted
    const uint8_t *dev;     // the row on the device
    const uint8_t *host;    // the caller's shard pointer at validate time
    size_t len;
    uint8_t leaf[32];
};
struct KeepStore {
    std::mutex mu;
    uint8_t *dev = nullptr;
    size_t cap = 0, head = 0;
    struct Region {
        size_t off, len;
        uint64_t gen;
        int users;  // the validate writing it (until it completes) + interpolates reading it
        std::vector<KeepKey> keys;
    };
    std::deque<Region> regions;  // allocation order: generations ascending
    uint64_t next_gen = 1;
    std::unordered_map<KeepKey, KeepEntry, KeepKeyHash> map;
    uint64_t kept_interps = 0, host_interps = 0, kept_launches = 0, unkept_launches = 0;
    Region *find(uint64_t gen) {
        auto it = std::lower_bound(regions.begin(), regions.end(), gen,
                                   [](const Region &r, uint64_t g) { return r.gen < g; });
        return it != regions.end() && it->gen == gen ? &*it : nullptr;
    }
    void drop(Region &r) {  // forget the region's rows (those not re-inserted since)
        for (const KeepKey &k : r.keys) {
            auto it = map.find(k);
            if (it != map.end() && it->second.gen == r.gen) map.erase(it);
        }
    }
    // A region of `need` bytes for a launch, or 0 when the ring has no free
    // room at its head (the launch is then not kept).
    uint64_t alloc(size_t need, uint8_t **where) {
        std::lock_guard<std::mutex> lk(mu);
        need = (need + 255) / 256 * 256;
        if (!dev) return 0;
        if (need > cap) {
            unkept_launches++;
            return 0;
        }
        const size_t pos = head + need <= cap ? head : 0;
        for (const Region &r : regions)
            if (r.off < pos + need && pos < r.off + r.len && r.users > 0) {
                unkept_launches++;
                return 0;
            }
        for (auto it = regions.begin(); it != regions.end();) {
            if (it->off < pos + need && pos < it->off + it->len) {
                drop(*it);
                it = regions.erase(it);
            } else {
                ++it;
            }
        }
        regions.push_back(Region{pos, need, next_gen, 1, {}});
        head = pos + need;
        *where = dev + pos;
        kept_launches++;
        return next_gen++;
    }
    void release(uint64_t gen) {  // under mu
        if (Region *r = find(gen)) r->users--;
    }
};

}  // namespace

struct rbc_batcher {
    rbc_ctx *ctx = nullptr;
    int n = 0, k = 0, depth = 0;
    int max_batch = 256;
    int max_wait_us = 200;
    std::mutex mu;
    std::condition_variable cv_work;
    std::deque<Req> q[kKinds];
    // Completed tickets -> status, sharded by ticket so that the callers'
    // waits and polls (one per request, from many threads) and the worker's
    // completions contend per shard, not on the queue lock, and a finished
    // launch wakes only the waiters of the shards it touched.
    static constexpr int kShards = 64;
    struct DoneShard {
        std::mutex mu;
        std::condition_variable cv;
        std::unordered_map<uint64_t, int> done;
    };
    DoneShard shard[kShards];
    std::atomic<uint64_t> next{1};
    bool stop = false;
    uint64_t batches = 0, requests = 0;
    std::thread worker;

    // validate lane (see the file comment)
    // six arenas, four launches in flight (the context's host slots); with a
    // launch running, an arena is sealed once it holds kVTarget bytes (each
    // launch pays the SHA chain's fixed ~1 ms: 16 MiB arenas four deep keep
    // the H2D copy engine, ~55 GB/s, busy) or when arrivals pause
    static constexpr int kVBufs = 6, kVInflight = 4;
    static constexpr size_t kVTarget = (size_t)16 << 20;
    int v_max_msgs = 65536;
    size_t v_max_bytes = (size_t)256 << 20;
    int bslot = 32;
    alignas(64) std::atomic<VBuf *> v_open{nullptr};  // the arena reservations go to
    alignas(64) std::mutex vmu;             // everything below (own cache line: off the spinlock's)
    std::condition_variable v_work;         // launcher: a seal, a finished copy, a free launch slot
    std::condition_variable v_fl;           // completer: a launch
    std::condition_variable v_free;         // clients: a free arena
    std::condition_variable v_done;         // clients: a completed generation
    std::unique_ptr<VBuf> vb[kVBufs];
    std::deque<VBuf *> v_sealed, v_flight;  // generation order
    uint64_t v_next_gen = 1, v_next_launch = 1;
    std::atomic<uint64_t> v_done_gen{0};
    std::atomic<bool> v_any_failed{false};
    std::unordered_map<uint64_t, int> v_failed;  // generations whose launch failed
    uint64_t v_batches = 0, v_requests = 0;
    bool v_stop = false, v_launcher_done = false;
    std::thread v_worker, v_completer;
    int v_reserve(size_t need, VBuf **B, int *slot, size_t *off);
    bool v_seal(VBuf *B);
    void v_push_sealed(VBuf *B);
    void v_launch(VBuf *B);
    void v_complete(VBuf *B);
    void v_run();
    void v_finish_run();

    void run();
    std::mutex pool_mu;
    std::vector<std::unique_ptr<PinnedSet>> pool;  // under pool_mu (worker takes, completer returns)
    // the coalescer's launches in flight, completed in order by their own
    // thread: the copies out of batch t overlap the copies into batch t+1
    std::mutex cmu;
    std::condition_variable c_cv, c_space;
    std::deque<std::unique_ptr<struct Pending>> cq;
    bool c_stop = false;
    std::thread completer;
    void c_run();

    KeepStore keep;                     // rbc_batcher_set_keep
    std::atomic<bool> keep_on{false};
    bool keep_lookup(const uint8_t *root, const uint8_t *const *shards, const size_t *lens, Req &r);

    std::unique_ptr<struct Pending> submit(Kind kind, std::vector<Req> &&batch);
    void finish(struct Pending &p);
};

namespace {

inline size_t round_up64(size_t x) { return (x + 63) / 64 * 64; }

// spin-wait hint of v_reserve's retry (host code a cgo build links on any ISA)
inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#elif defined(__aarch64__)
    asm volatile("yield");
#else
    std::this_thread::yield();
#endif
}

int check_shards_sizes(const std::vector<size_t> &lens, size_t *S) {
    size_t size = 0;
    for (size_t l : lens)
        if (l) { size = l; break; }
    if (!size) return RBC_ERR_SHARD_NO_DATA;
    for (size_t l : lens)
        if (l && l != size) return RBC_ERR_SHARD_SIZE;
    *S = size;
    return RBC_OK;
}

}  // namespace

// One coalesced launch in flight: the requests it serves, the batch-shaped
// buffers the C API reads at submit and fills at completion, its ticket.
struct Pending {
    Kind kind;
    std::vector<Req> reqs;
    std::vector<int> st;         // per-request status (argument checks at submit)
    uint64_t ticket = 0;
    int rc = RBC_OK;             // submit status
    size_t Smax = 1;
    std::vector<int> idx;        // interpolate: requests in the batch
    std::vector<size_t> lens;
    std::vector<uint8_t> present, digests;
    std::vector<uint32_t> slens;
    std::vector<int32_t> status;
    std::unique_ptr<PinnedSet> pin;  // shards / roots / branches / values of this launch
    uint8_t *shards = nullptr, *roots = nullptr, *br = nullptr, *values = nullptr;
};

std::unique_ptr<Pending> rbc_batcher::submit(Kind kind, std::vector<Req> &&batch) {
    auto P = std::make_unique<Pending>();
    P->kind = kind;
    P->reqs = std::move(batch);
    const int count = (int)P->reqs.size();
    P->st.assign(count, RBC_OK);
    std::vector<Req> &b = P->reqs;
    {
        std::lock_guard<std::mutex> lk(pool_mu);
        if (pool.empty()) {
            P->pin = std::make_unique<PinnedSet>();
        } else {
            P->pin = std::move(pool.back());
            pool.pop_back();
        }
    }
    if (kind == K_SHARD) {
        std::vector<const uint8_t *> vals(count);
        P->lens.resize(count);
        for (int i = 0; i < count; ++i) {
            vals[i] = b[i].data;
            P->lens[i] = b[i].len;
            P->Smax = std::max(P->Smax, (b[i].len + k - 1) / k);
        }
        P->shards = P->pin->shards.ensure((size_t)count * n * P->Smax);
        P->roots = P->pin->roots.ensure((size_t)count * 32);
        P->br = P->pin->br.ensure((size_t)count * n * std::max(depth, 1) * 32);
        P->slens.resize(count);
        P->rc = (!P->shards || !P->roots || !P->br)
                    ? RBC_ERR_DEVICE
                    : rbc_shard_commit(ctx, count, vals.data(), P->lens.data(), P->shards, P->Smax, P->slens.data(),
                                       P->roots, P->br, &P->ticket);
    } else {
        // interpolate: klauspost argument checks per request, then one batch
        // over the requests that pass them
        std::vector<size_t> S(count, 0);
        for (int i = 0; i < count; ++i) {
            Req &r = b[i];
            int present = 0;
            for (size_t l : r.in_lens) present += l != 0;
            int rc = check_shards_sizes(r.in_lens, &S[i]);
            if (!rc && present < k) rc = RBC_ERR_TOO_FEW_SHARDS;
            if (!rc && r.value_cap < (size_t)k * S[i]) rc = RBC_ERR_INVALID_ARG;
            if (rc) P->st[i] = rc;
            else P->idx.push_back(i);
        }
        const int m = (int)P->idx.size();
        if (m) {
            for (int i : P->idx) P->Smax = std::max(P->Smax, S[i]);
            const size_t Smax = P->Smax;
            // absent rows stay as they are (never read: the present mask
            // rules them out); a present row is zero-padded to Smax
            const bool kept = kind == K_INTERPK;
            P->shards = kept ? nullptr : P->pin->shards.ensure((size_t)m * n * Smax);
            P->roots = P->pin->roots.ensure((size_t)m * 32);
            P->values = P->pin->values.ensure((size_t)m * k * Smax);
            uint8_t *lv = kind != K_INTERP ? P->pin->leaves.ensure((size_t)m * n * 32) : nullptr;
            P->present.assign((size_t)m * n, 0);
            P->digests.resize((size_t)m * 32);
            P->lens.resize(m);
            P->status.assign(m, 0);
            if ((!kept && !P->shards) || !P->roots || !P->values || (kind != K_INTERP && !lv)) {
                P->rc = RBC_ERR_DEVICE;
                return P;
            }
            for (int t = 0; t < m; ++t) P->lens[t] = S[P->idx[t]];
            if (kept) {  // the rows are on the device: their addresses and leaves, no shard bytes
                std::vector<const uint8_t *> rows((size_t)m * n, nullptr);
                for (int t = 0; t < m; ++t) {
                    Req &r = b[P->idx[t]];
                    for (int j = 0; j < n; ++j)
                        if (r.in_lens[j]) rows[(size_t)t * n + j] = reinterpret_cast<const uint8_t *>(r.dev_rows[j]);
                    memcpy(lv + (size_t)t * n * 32, r.kleaves.data(), (size_t)n * 32);
                    memcpy(P->roots + (size_t)t * 32, r.root, 32);
                }
                P->rc = rbc_interpolate_batch_kept(ctx, m, rows.data(), P->lens.data(), lv, P->roots, P->values,
                                                   (size_t)k * Smax, P->digests.data(), P->status.data(), &P->ticket);
                return P;
            }
            parallel_for(m, (size_t)n * Smax, [&](int t) {
                Req &r = b[P->idx[t]];
                for (int j = 0; j < n; ++j)
                    if (r.in_lens[j]) {
                        uint8_t *row = P->shards + ((size_t)t * n + j) * Smax;
                        memcpy(row, r.in_shards[j], P->lens[t]);
                        if (P->lens[t] < Smax) memset(row + P->lens[t], 0, Smax - P->lens[t]);
                        P->present[(size_t)t * n + j] = 1;
                        if (lv) memcpy(lv + ((size_t)t * n + j) * 32, r.leaves + (size_t)j * 32, 32);
                    }
                memcpy(P->roots + (size_t)t * 32, r.root, 32);
            });
            P->rc = rbc_interpolate_batch_verified(ctx, m, P->shards, Smax, P->lens.data(), P->present.data(), lv,
                                                   P->roots, P->values, (size_t)k * Smax, P->digests.data(),
                                                   P->status.data(), &P->ticket);
        }
    }
    return P;
}

void rbc_batcher::finish(Pending &P) {
    int rc = P.rc;
    if (!rc && P.ticket) rc = rbc_wait(ctx, P.ticket);
    const int count = (int)P.reqs.size();
    std::vector<Req> &b = P.reqs;
    if (P.kind == K_SHARD) {
        parallel_for(count, (size_t)n * P.Smax, [&](int i) {
            Req &r = b[i];
            if (rc) { P.st[i] = rc; return; }
            const size_t S = P.slens[i];
            if (r.shards_cap < (size_t)n * S) { P.st[i] = RBC_ERR_INVALID_ARG; return; }
            for (int j = 0; j < n; ++j)
                memcpy(r.shards_out + (size_t)j * S, P.shards + ((size_t)i * n + j) * P.Smax, S);
            if (r.shard_len_out) *r.shard_len_out = S;
            memcpy(r.root_out, P.roots + (size_t)i * 32, 32);
            if (r.branches_out && depth)
                memcpy(r.branches_out, P.br + (size_t)i * n * depth * 32, (size_t)n * depth * 32);
        });
    } else {
        parallel_for((int)P.idx.size(), (size_t)k * P.Smax, [&](int t) {
            Req &r = b[P.idx[t]];
            const int s = rc ? rc : P.status[t];
            P.st[P.idx[t]] = s;
            if (s) return;
            memcpy(r.value_out, P.values + (size_t)t * k * P.Smax, (size_t)k * P.lens[t]);
            if (r.value_len) *r.value_len = (size_t)k * P.lens[t];
            if (r.digest_out) memcpy(r.digest_out, P.digests.data() + (size_t)t * 32, 32);
        });
    }
    if (P.kind == K_INTERPK) {  // the launch no longer reads its keep regions
        std::lock_guard<std::mutex> lk(keep.mu);
        for (const Req &r : b)
            for (uint64_t g : r.kgens) keep.release(g);
    }
    if (P.pin) {  // the launch is complete: its buffers are free
        std::lock_guard<std::mutex> lk(pool_mu);
        pool.push_back(std::move(P.pin));
    }
    {  // count the launch before any of its requests reads as done: a client
       // that saw its last request complete then sees it in rbc_batcher_stats
        std::lock_guard<std::mutex> lk(mu);
        batches++;
        requests += count;
    }
    uint64_t touched = 0;  // bit per shard
    for (int i = 0; i < count; ++i) {
        const int sh = (int)(b[i].ticket % kShards);
        std::lock_guard<std::mutex> lk(shard[sh].mu);
        shard[sh].done[b[i].ticket] = P.st[i];
        touched |= 1ull << sh;
    }
    for (int sh = 0; sh < kShards; ++sh)
        if (touched >> sh & 1) shard[sh].cv.notify_all();
}

// Worker: coalesce and submit asynchronously; the completer thread (c_run)
// completes launches in order.  Up to depth_max launches are in flight (the
// context has as many host slots), so the host-side staging of batch t+1
// overlaps the GPU work of batch t and the copies out of batch t-1.
void rbc_batcher::run() {
    // launches in flight: 4 (41 vs 27 GB/s of shard + commit through the
    // coalescer at 2); the context has as many host slots
    constexpr size_t depth_max = 4;
    std::unique_lock<std::mutex> lk(mu);
    while (true) {
        // pick the kind whose queue is full, or whose oldest request is due
        const auto now = std::chrono::steady_clock::now();
        int pick = -1;
        auto earliest = now + std::chrono::hours(1);
        for (int kd = 0; kd < kKinds; ++kd) {
            if (q[kd].empty()) continue;
            const auto due = q[kd].front().t0 + std::chrono::microseconds(max_wait_us);
            if ((int)q[kd].size() >= max_batch || due <= now || stop) { pick = kd; break; }
            earliest = std::min(earliest, due);
        }
        if (pick < 0) {
            if (stop) break;  // every queue drained
            cv_work.wait_until(lk, earliest);
            continue;
        }
        // take the requests in O(1) under the lock (the whole queue when it
        // fits one launch), and move them into the batch outside it, so that
        // the submitting threads are not held up
        std::deque<Req> taken;
        if ((int)q[pick].size() <= max_batch) {
            taken.swap(q[pick]);
        } else {
            for (int i = 0; i < max_batch; ++i) {
                taken.push_back(std::move(q[pick].front()));
                q[pick].pop_front();
            }
        }
        lk.unlock();
        std::vector<Req> batch;
        batch.reserve(taken.size());
        for (auto &r : taken) batch.push_back(std::move(r));
        {  // a free launch slot first: a submission never waits inside the context for one
            std::unique_lock<std::mutex> cl(cmu);
            c_space.wait(cl, [&] { return cq.size() < depth_max; });
        }
        auto P = submit((Kind)pick, std::move(batch));
        {
            std::lock_guard<std::mutex> cl(cmu);
            cq.push_back(std::move(P));
        }
        c_cv.notify_one();
        lk.lock();
    }
    lk.unlock();
    {
        std::lock_guard<std::mutex> cl(cmu);
        c_stop = true;  // the completer drains cq and exits
    }
    c_cv.notify_one();
}

// Completer: the oldest launch's rbc_wait and copies out, in submission order
// (it stays at the head of cq, counted as in flight, until it is done).
void rbc_batcher::c_run() {
    std::unique_lock<std::mutex> cl(cmu);
    for (;;) {
        c_cv.wait(cl, [&] { return !cq.empty() || c_stop; });
        if (cq.empty()) return;
        Pending *P = cq.front().get();
        cl.unlock();
        finish(*P);
        cl.lock();
        cq.pop_front();
        c_space.notify_all();
    }
}

// ---- validate lane ----------------------------------------------------------

// Seal B if it is still the open arena: take it out of v_open, fix its final
// count / bytes with one add of kBump (every later reservation fails and
// retries), credit the slots nobody will copy into pend, and hand it to the
// launcher in generation order.  False if another caller sealed it first.
bool rbc_batcher::v_seal(VBuf *B) {
    VBuf *expect = B;
    if (!v_open.compare_exchange_strong(expect, nullptr)) return false;
    const uint64_t w = B->word.fetch_add(VBuf::kBump);
    B->count = (int)std::min<uint64_t>(w >> 40, (uint64_t)B->cap);
    B->bytes = std::min<uint64_t>(w & VBuf::kBytesMask, B->arena.cap);
    v_push_sealed(B);
    return true;
}

void rbc_batcher::v_push_sealed(VBuf *B) {
    std::lock_guard<std::mutex> lk(vmu);
    B->state = VBuf::SEALED;
    B->pend.fetch_add(VBuf::kSealed - B->count);
    auto it = v_sealed.begin();
    while (it != v_sealed.end() && (*it)->gen < B->gen) ++it;
    v_sealed.insert(it, B);
    v_work.notify_one();
}

// A slot for one message of `need` arena bytes: one atomic add on the open
// arena; opening a free arena under vmu (this message in slot 0) when none is.
int rbc_batcher::v_reserve(size_t need, VBuf **out, int *slot, size_t *off) {
    for (;;) {
        VBuf *B = v_open.load();
        if (B) {
            const uint64_t w = B->word.fetch_add(VBuf::kCountOne | need);
            const uint64_t oc = w >> 40, ob = w & VBuf::kBytesMask;
            if (oc >= (uint64_t)B->cap) {  // sealed, or full and being sealed: the next arena
                cpu_relax();
                continue;
            }
            if (ob + need <= B->arena.cap) {
                *out = B;
                *slot = (int)oc;
                *off = ob;
                if (oc + 1 == (uint64_t)B->cap) v_seal(B);  // the last slot
                else if (ob < kVTarget && ob + need >= kVTarget) v_work.notify_one();  // a hint; the launcher also polls
                return RBC_OK;
            }
            // no room for these bytes: slot oc is launched as an empty message
            B->out[oc] = nullptr;
            B->lout[oc] = nullptr;
            B->offs[oc] = 0;
            B->lens[oc] = 1;
            B->idx[oc] = 0;
            B->shape[oc] = 0;
            memset(B->br + (size_t)oc * bslot, 0, bslot);
            memset(B->roots + oc * 32, 0, 32);
            if (B->pend.fetch_add(1) + 1 == VBuf::kSealed) {
                std::lock_guard<std::mutex> lk(vmu);
                v_work.notify_one();
            }
            v_seal(B);
            continue;
        }
        std::unique_lock<std::mutex> lk(vmu);
        if (v_open.load()) continue;  // another caller opened one meanwhile
        VBuf *f = nullptr;
        for (;;) {
            for (auto &x : vb)
                if (x->state == VBuf::FREE) { f = x.get(); break; }
            if (f || v_stop) break;
            v_free.wait(lk);  // every arena is filling, sealed or in flight
        }
        if (!f) return RBC_ERR_INVALID_ARG;  // the batcher is being destroyed
        if (v_open.load()) continue;
        // an arena's buffers are allocated once, before it is first published,
        // and never moved (a caller holding a stale arena pointer only ever
        // reads them); messages larger than an arena take the direct path
        if (f->cap != v_max_msgs && !f->layout(v_max_msgs, bslot)) return RBC_ERR_DEVICE;
        if (!f->arena.ensure(v_max_bytes)) return RBC_ERR_DEVICE;
        // open f with this message in slot 0, so the launcher, woken here
        // under vmu, always finds a non-empty arena to time
        f->state = VBuf::OPEN;
        f->gen = v_next_gen++;
        f->count = 0;
        f->bytes = 0;
        f->pend.store(0);
        f->word.store(VBuf::kCountOne | need);
        f->rc = RBC_OK;
        f->ticket = 0;
        f->any_leaf.store(false);
        f->t0 = f->t_seen = std::chrono::steady_clock::now();  // max_wait runs from the first message
        f->seen = 1;
        *out = f;
        *slot = 0;
        *off = 0;
        if (f->cap == 1) {  // full at once
            f->count = 1;
            f->bytes = need;
            lk.unlock();
            v_push_sealed(f);
            return RBC_OK;
        }
        v_open.store(f);
        v_work.notify_one();
        return RBC_OK;
    }
}

void rbc_batcher::v_launch(VBuf *B) {
    B->keep_dev = nullptr;
    B->keep_gen = B->count && keep_on.load() ? keep.alloc(B->bytes, &B->keep_dev) : 0;
    if (B->keep_gen)  // the arena moves into its keep region, the leaves come back for the index
        B->rc = rbc_validate_packed_keep(ctx, B->count, B->arena.p, B->bytes, B->offs, B->lens, B->idx, B->br,
                                         B->roots, B->ok, B->lv, B->keep_dev, (B->bytes + 255) / 256 * 256,
                                         &B->ticket);
    else
        B->rc = B->count ? rbc_validate_packed_leaves(ctx, B->count, B->arena.p, B->bytes, B->offs, B->lens, B->idx,
                                                      B->br, B->roots, B->ok, B->any_leaf.load() ? B->lv : nullptr,
                                                      &B->ticket)
                         : RBC_OK;
    if (B->rc) B->ticket = 0;
}

void rbc_batcher::v_complete(VBuf *B) {
    int rc = B->rc;
    if (!rc && B->ticket) rc = rbc_wait(ctx, B->ticket);
    int real = 0;
    if (B->keep_gen) {  // index the rows that validated, then the launch no longer uses its region
        std::lock_guard<std::mutex> lk(keep.mu);
        KeepStore::Region *R = keep.find(B->keep_gen);
        for (int i = 0; R && !rc && i < B->count; ++i)
            if (B->out[i] && B->shape[i] && B->ok[i] && B->hostp[i]) {
                KeepKey key;
                memcpy(key.root, B->roots + (size_t)i * 32, 32);
                key.idx = B->idx[i];
                KeepEntry &e = keep.map[key];
                e.gen = B->keep_gen;
                e.dev = B->keep_dev + B->offs[i];
                e.host = B->hostp[i];
                e.len = B->lens[i];
                memcpy(e.leaf, B->lv + (size_t)i * 32, 32);
                R->keys.push_back(key);
            }
        keep.release(B->keep_gen);
    }
    for (int i = 0; i < B->count; ++i)
        if (B->out[i]) {  // holes have no caller
            const int ok = (!rc && B->shape[i]) ? B->ok[i] : 0;
            if (ok && B->lout[i]) memcpy(B->lout[i], B->lv + (size_t)i * 32, 32);
            *B->out[i] = ok;
            ++real;
        }
    std::lock_guard<std::mutex> lk(vmu);
    if (rc) {
        v_failed[B->gen] = rc;
        v_any_failed.store(true);
    }
    v_done_gen.store(B->gen);
    v_batches += real > 0;
    v_requests += real;
    v_flight.pop_front();  // B: the completer takes launches in order
    B->state = VBuf::FREE;
    v_free.notify_all();
    v_done.notify_all();
    v_work.notify_one();  // a launch slot is free
}

// Lane launcher: seal the open arena when its first message has waited
// max_wait_us and the lane is idle; with launches running, once it holds
// kVTarget bytes, or when no message has arrived for max_wait_us either (an
// arena sealed right after a completion, before the callers refill it, would
// launch only the stragglers).  Launch sealed arenas whose copies are
// complete, in generation order, at most kVInflight deep.
void rbc_batcher::v_run() {
    std::unique_lock<std::mutex> lk(vmu);
    for (;;) {
        const auto now = std::chrono::steady_clock::now();
        const int queued = (int)(v_flight.size() + v_sealed.size());
        const bool slot_free = queued < kVInflight;
        const auto mw = std::chrono::microseconds(max_wait_us);
        std::chrono::steady_clock::time_point wake{};
        VBuf *O = v_open.load();
        bool open_pending = false;
        if (O) {
            const uint64_t w = O->word.load();
            const uint64_t cnt = std::min<uint64_t>(w >> 40, (uint64_t)O->cap), bytes = w & VBuf::kBytesMask;
            // arrivals are sampled here (no per-message timestamp): `seen` moves when the count has
            if (cnt != O->seen) {
                O->seen = cnt;
                O->t_seen = now;
            }
            // idle lane: max_wait from the first message; busy: at least max_wait old and
            // max_wait / 4 without an arrival (a full max_wait of quiet cost 1 k outstanding
            // validates 11 -> 14 GB/s, tools/gpu_runs/gpu_r05v.sh), or kVTarget bytes
            wake = queued == 0 ? O->t0 + mw : std::max(O->t0 + mw, O->t_seen + mw / 4);
            const bool big = bytes >= kVTarget && O->t0 + mw <= now;
            if (v_stop || (slot_free && (wake <= now || big))) {
                lk.unlock();
                v_seal(O);
                lk.lock();
                continue;
            }
            open_pending = true;
        }
        VBuf *F = v_sealed.empty() ? nullptr : v_sealed.front();
        if (F && F->gen == v_next_launch && F->pend.load() == VBuf::kSealed && (int)v_flight.size() < kVInflight) {
            v_sealed.pop_front();
            v_next_launch++;
            F->state = VBuf::INFLIGHT;
            lk.unlock();
            v_launch(F);
            lk.lock();
            v_flight.push_back(F);
            v_fl.notify_one();
            continue;
        }
        if (v_stop && !v_open.load() && v_sealed.empty()) {
            v_launcher_done = true;  // everything launched: the completer drains v_flight and exits
            v_fl.notify_one();
            return;
        }
        if (open_pending && slot_free) v_work.wait_until(lk, wake);
        else v_work.wait(lk);
    }
}

// Lane completer: waits for the oldest launch (rbc_wait does not hold the
// context while it waits, so the launcher keeps submitting) and completes it.
void rbc_batcher::v_finish_run() {
    std::unique_lock<std::mutex> lk(vmu);
    for (;;) {
        if (!v_flight.empty()) {
            VBuf *B = v_flight.front();
            lk.unlock();
            v_complete(B);
            lk.lock();
            continue;
        }
        if (v_launcher_done) return;
        v_fl.wait(lk);
    }
}

// An interpolate request whose every present shard the lane kept (same
// caller pointer and length): its rows' device addresses and leaves, and a
// use of each region they lie in (released when the launch completes) --
// under the store lock, so no region it names can be reused before then.
bool rbc_batcher::keep_lookup(const uint8_t *root, const uint8_t *const *shards, const size_t *lens, Req &r) {
    if (!keep_on.load()) return false;
    std::lock_guard<std::mutex> lk(keep.mu);
    r.dev_rows.assign(n, 0);
    r.kleaves.assign((size_t)n * 32, 0);
    r.kgens.clear();
    KeepKey key;
    memcpy(key.root, root, 32);
    int present = 0;
    for (int j = 0; j < n; ++j) {
        if (!lens[j]) continue;
        key.idx = (uint32_t)j;
        const auto it = keep.map.find(key);
        if (it == keep.map.end() || it->second.host != shards[j] || it->second.len != lens[j]) {
            keep.host_interps++;
            return false;
        }
        r.dev_rows[j] = (uint64_t)(uintptr_t)it->second.dev;
        memcpy(r.kleaves.data() + (size_t)j * 32, it->second.leaf, 32);
        if (std::find(r.kgens.begin(), r.kgens.end(), it->second.gen) == r.kgens.end())
            r.kgens.push_back(it->second.gen);
        ++present;
    }
    if (!present) return false;
    for (uint64_t g : r.kgens)
        if (KeepStore::Region *R = keep.find(g)) R->users++;
    keep.kept_interps++;
    return true;
}

namespace {
uint64_t enqueue(rbc_batcher *b, Req &&r) {
    std::lock_guard<std::mutex> lk(b->mu);
    r.ticket = b->next++;
    r.t0 = std::chrono::steady_clock::now();
    const uint64_t t = r.ticket;
    const Kind kd = r.kind;
    b->q[kd].push_back(std::move(r));
    if ((int)b->q[kd].size() >= b->max_batch || b->q[kd].size() == 1) b->cv_work.notify_one();
    return t;
}
}  // namespace

extern "C" {

int rbc_batcher_create(rbc_ctx *ctx, int max_batch, int max_wait_us, rbc_batcher **out) {
    if (!ctx || !out || max_batch < 1 || max_wait_us < 0) return RBC_ERR_INVALID_ARG;
    rbc_batcher *b = new rbc_batcher();
    b->ctx = ctx;
    int k = 0, p = 0, d = 0;
    rbc_ctx_params(ctx, &k, &p, &d);
    b->k = k;
    b->n = k + p;
    b->depth = d;
    b->max_batch = max_batch;
    b->max_wait_us = max_wait_us;
    b->bslot = std::max(d, 1) * 32;
    for (auto &x : b->vb) x = std::make_unique<VBuf>();
    b->worker = std::thread([b] { b->run(); });
    b->completer = std::thread([b] { b->c_run(); });
    b->v_worker = std::thread([b] { b->v_run(); });
    b->v_completer = std::thread([b] { b->v_finish_run(); });
    *out = b;
    return RBC_OK;
}

int rbc_batcher_set_validate(rbc_batcher *b, int max_msgs, size_t max_bytes) {
    // a message's length travels as uint32 (rbc_validate_packed): arenas stay below 4 GiB
    if (!b || max_msgs < 1 || max_msgs >= (1 << kVSlotBits) || max_bytes < 64 || max_bytes > ((size_t)1 << 32) - 64)
        return RBC_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->vmu);
    if (b->v_next_gen != 1) return RBC_ERR_INVALID_ARG;  // before the first validate only
    b->v_max_msgs = max_msgs;
    b->v_max_bytes = max_bytes;
    return RBC_OK;
}

int rbc_batcher_set_keep(rbc_batcher *b, size_t device_bytes) {
    if (!b) return RBC_ERR_INVALID_ARG;
    {
        std::lock_guard<std::mutex> lk(b->vmu);
        if (b->v_next_gen != 1) return RBC_ERR_INVALID_ARG;  // before the first validate only
    }
    std::lock_guard<std::mutex> lk(b->keep.mu);
    if (b->keep.dev) {
        rbc_dev_free(b->keep.dev);
        b->keep.dev = nullptr;
        b->keep.cap = 0;
    }
    b->keep_on.store(false);
    if (!device_bytes) return RBC_OK;
    int dev = 0;
    void *p = nullptr;
    if (rbc_ctx_device(b->ctx, &dev) != RBC_OK || rbc_dev_malloc(dev, device_bytes, &p) != RBC_OK)
        return RBC_ERR_DEVICE;
    b->keep.dev = static_cast<uint8_t *>(p);
    b->keep.cap = device_bytes;
    b->keep.head = 0;
    b->keep_on.store(true);
    return RBC_OK;
}

int rbc_batcher_keep_stats(rbc_batcher *b, uint64_t *kept_interps, uint64_t *host_interps, uint64_t *kept_launches,
                           uint64_t *unkept_launches) {
    if (!b) return RBC_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->keep.mu);
    if (kept_interps) *kept_interps = b->keep.kept_interps;
    if (host_interps) *host_interps = b->keep.host_interps;
    if (kept_launches) *kept_launches = b->keep.kept_launches;
    if (unkept_launches) *unkept_launches = b->keep.unkept_launches;
    return RBC_OK;
}

void rbc_batcher_destroy(rbc_batcher *b) {
    if (!b) return;
    {
        std::lock_guard<std::mutex> lk(b->mu);
        b->stop = true;  // drains every queue before the worker exits
    }
    b->cv_work.notify_all();
    if (b->worker.joinable()) b->worker.join();
    if (b->completer.joinable()) b->completer.join();  // the worker's last launches completed
    {
        std::lock_guard<std::mutex> lk(b->vmu);
        b->v_stop = true;  // the lane drains too
    }
    b->v_work.notify_all();
    b->v_free.notify_all();
    if (b->v_worker.joinable()) b->v_worker.join();
    if (b->v_completer.joinable()) b->v_completer.join();
    if (b->keep.dev) rbc_dev_free(b->keep.dev);  // every launch that used it has completed
    delete b;
}

int rbc_batcher_shard(rbc_batcher *b, const uint8_t *data, size_t len, uint8_t *shards_out, size_t shards_cap,
                      size_t *shard_len_out, uint8_t *root_out, uint8_t *branches_out, uint64_t *ticket) {
    if (!b || !ticket || !shards_out || !root_out) return RBC_ERR_INVALID_ARG;
    if (len == 0) return RBC_ERR_SHORT_DATA;
    if (!data) return RBC_ERR_INVALID_ARG;
    Req r;
    r.kind = K_SHARD;
    r.data = data;
    r.len = len;
    r.shards_out = shards_out;
    r.shards_cap = shards_cap;
    r.shard_len_out = shard_len_out;
    r.root_out = root_out;
    r.branches_out = branches_out;
    *ticket = enqueue(b, std::move(r));
    return RBC_OK;
}

int rbc_batcher_validate(rbc_batcher *b, const uint8_t *root, const uint8_t *branch, size_t branch_len,
                         const uint8_t *shard, size_t shard_len, uint32_t index, int *ok_out, uint64_t *ticket) {
    return rbc_batcher_validate_leaf(b, root, branch, branch_len, shard, shard_len, index, ok_out, nullptr, ticket);
}

int rbc_batcher_validate_leaf(rbc_batcher *b, const uint8_t *root, const uint8_t *branch, size_t branch_len,
                              const uint8_t *shard, size_t shard_len, uint32_t index, int *ok_out, uint8_t *leaf_out,
                              uint64_t *ticket) {
    if (!b || !ticket || !ok_out || !root) return RBC_ERR_INVALID_ARG;
    *ok_out = 0;
    const int n = b->n, d = b->depth;
    // the Go-form branch omits an empty level-0 sibling (rbc_validate_batch's shape rule)
    const bool empty0 = d > 0 && (index ^ 1u) >= (uint32_t)n;
    const size_t want = (size_t)32 * (d - (empty0 ? 1 : 0));
    const bool shape_ok = index < (uint32_t)n && branch_len == want && shard_len != 0 && shard && (!want || branch);
    const size_t need = shape_ok ? (shard_len + 63) / 64 * 64 : 64;
    if (need > b->v_max_bytes) {  // larger than an arena: validated on this thread, complete at return
        uint8_t ok = 0;
        const uint8_t *sh = shard, *bp = branch, *rp = root;
        const int rc = rbc_validate_batch(b->ctx, 1, &sh, &shard_len, &index, &bp, &branch_len, &rp, &ok, nullptr);
        if (rc) return rc;
        if (ok && leaf_out) {  // the leaf of a message larger than an arena: a packed launch of one
            uint8_t *tmp = nullptr;
            void *q = nullptr;
            if (rbc_host_alloc(round_up64(shard_len) + 64, &q) != RBC_OK) return RBC_ERR_DEVICE;
            tmp = static_cast<uint8_t *>(q);
            memcpy(tmp, shard, shard_len);
            uint8_t brd[32 * 8] = {0}, okp = 0;
            const int n = b->n, d = b->depth;
            const bool e0 = d > 0 && (index ^ 1u) >= (uint32_t)n;
            for (int l = 0, o = 0; l < d; ++l)
                if (!(l == 0 && e0)) { memcpy(brd + 32 * l, branch + o, 32); o += 32; }
            const uint64_t off0 = 0;
            const uint32_t ln = (uint32_t)shard_len;
            const uint8_t ix = (uint8_t)index;
            int rc2 = rbc_validate_packed_leaves(b->ctx, 1, tmp, round_up64(shard_len), &off0, &ln, &ix, brd, root,
                                                 &okp, leaf_out, nullptr);
            rbc_host_free(tmp);
            if (rc2) return rc2;
        }
        *ok_out = ok;
        *ticket = kVTicket | 1;  // generation 0: already complete
        std::lock_guard<std::mutex> lk(b->vmu);
        b->v_batches++;
        b->v_requests++;
        return RBC_OK;
    }
    VBuf *B = nullptr;
    int slot = 0;
    size_t off = 0;
    const int rc = b->v_reserve(need, &B, &slot, &off);
    if (rc) return rc;
    // the copy runs on the calling thread, outside the lock
    uint8_t *row = B->arena.p + off, *br = B->br + (size_t)slot * b->bslot;
    B->out[slot] = ok_out;
    B->lout[slot] = leaf_out;
    B->hostp[slot] = shape_ok ? shard : nullptr;
    if (leaf_out && !B->any_leaf.load(std::memory_order_relaxed))
        B->any_leaf.store(true);  // before this slot's pend add: the launch sees it
    B->offs[slot] = off;
    B->shape[slot] = shape_ok;
    if (shape_ok) {
        memcpy(row, shard, shard_len);
        B->lens[slot] = (uint32_t)shard_len;
        B->idx[slot] = (uint8_t)index;
        size_t o = 0;
        for (int l = 0; l < d; ++l) {
            if (l == 0 && empty0) {
                memset(br, 0, 32);  // the device form keeps a zero level-0 slot
                continue;
            }
            memcpy(br + 32 * l, branch + o, 32);
            o += 32;
        }
        if (d == 0) memset(br, 0, 32);
        memcpy(B->roots + (size_t)slot * 32, root, 32);
    } else {  // hashed as one zero byte; the verdict is discarded (0)
        memset(row, 0, 64);
        B->lens[slot] = 1;
        B->idx[slot] = 0;
        memset(br, 0, b->bslot);
        memset(B->roots + (size_t)slot * 32, 0, 32);
    }
    *ticket = kVTicket | (B->gen << kVSlotBits) | (uint64_t)slot;  // gen is stable until this slot completes
    // the last copy of a sealed arena wakes the launcher (either it sees
    // this copy when it checks, or this update sees the seal)
    if (B->pend.fetch_add(1) + 1 == VBuf::kSealed) {
        std::lock_guard<std::mutex> lk(b->vmu);
        b->v_work.notify_one();
    }
    return RBC_OK;
}

int rbc_batcher_interpolate(rbc_batcher *b, const uint8_t *root, const uint8_t *const *shards, const size_t *lens,
                            uint8_t *value_out, size_t value_cap, size_t *value_len, uint8_t *digest_out,
                            uint64_t *ticket) {
    if (!b || !ticket || !root || !shards || !lens || !value_out) return RBC_ERR_INVALID_ARG;
    Req r;
    r.kind = b->keep_lookup(root, shards, lens, r) ? K_INTERPK : K_INTERP;
    r.root = root;
    r.in_shards.assign(shards, shards + b->n);
    r.in_lens.assign(lens, lens + b->n);
    r.value_out = value_out;
    r.value_cap = value_cap;
    r.value_len = value_len;
    r.digest_out = digest_out;
    *ticket = enqueue(b, std::move(r));
    return RBC_OK;
}

int rbc_batcher_interpolate_verified(rbc_batcher *b, const uint8_t *root, const uint8_t *const *shards,
                                     const size_t *lens, const uint8_t *leaves, uint8_t *value_out, size_t value_cap,
                                     size_t *value_len, uint8_t *digest_out, uint64_t *ticket) {
    if (!b || !ticket || !root || !shards || !lens || !value_out || !leaves) return RBC_ERR_INVALID_ARG;
    Req r;
    r.kind = b->keep_lookup(root, shards, lens, r) ? K_INTERPK : K_INTERPV;
    r.root = root;
    r.in_shards.assign(shards, shards + b->n);
    r.in_lens.assign(lens, lens + b->n);
    r.leaves = leaves;
    r.value_out = value_out;
    r.value_cap = value_cap;
    r.value_len = value_len;
    r.digest_out = digest_out;
    *ticket = enqueue(b, std::move(r));
    return RBC_OK;
}

int rbc_batcher_wait(rbc_batcher *b, uint64_t ticket) {
    if (!b) return RBC_ERR_INVALID_ARG;
    if (ticket & kVTicket) {  // validate lane: complete when its arena's generation is
        const uint64_t gen = (ticket & ~kVTicket) >> kVSlotBits;
        if (gen == 0) return RBC_OK;  // validated at submission (larger than an arena)
        if (b->v_done_gen.load() >= gen && !b->v_any_failed.load()) return RBC_OK;  // no lock
        std::unique_lock<std::mutex> lk(b->vmu);
        if (gen == 0 || gen >= b->v_next_gen) return RBC_ERR_INVALID_ARG;
        b->v_done.wait(lk, [&] { return b->v_done_gen.load() >= gen; });
        const auto it = b->v_failed.find(gen);
        return it == b->v_failed.end() ? RBC_OK : it->second;
    }
    if (ticket == 0 || ticket >= b->next.load()) return RBC_ERR_INVALID_ARG;
    auto &sh = b->shard[ticket % rbc_batcher::kShards];
    std::unique_lock<std::mutex> lk(sh.mu);
    if (!sh.done.count(ticket)) {
        b->cv_work.notify_one();  // a waiter: the worker re-checks what is due
        sh.cv.wait(lk, [&] { return sh.done.count(ticket) != 0; });
    }
    const auto it = sh.done.find(ticket);
    const int s = it->second;
    sh.done.erase(it);
    return s;
}

int rbc_batcher_poll(rbc_batcher *b, uint64_t ticket, int *done_out) {
    if (!b || !done_out) return RBC_ERR_INVALID_ARG;
    if (ticket & kVTicket) {
        const uint64_t gen = (ticket & ~kVTicket) >> kVSlotBits;
        std::lock_guard<std::mutex> lk(b->vmu);
        if (gen >= b->v_next_gen) return RBC_ERR_INVALID_ARG;
        *done_out = gen == 0 || b->v_done_gen.load() >= gen;
        return RBC_OK;
    }
    if (ticket == 0 || ticket >= b->next.load()) return RBC_ERR_INVALID_ARG;
    auto &sh = b->shard[ticket % rbc_batcher::kShards];
    std::lock_guard<std::mutex> lk(sh.mu);
    *done_out = sh.done.count(ticket) != 0;
    return RBC_OK;
}

int rbc_batcher_stats(rbc_batcher *b, uint64_t *batches, uint64_t *requests) {
    if (!b) return RBC_ERR_INVALID_ARG;
    std::scoped_lock lk(b->mu, b->vmu);
    if (batches) *batches = b->batches + b->v_batches;
    if (requests) *requests = b->requests + b->v_requests;
    return RBC_OK;
}

}  // extern "C"
