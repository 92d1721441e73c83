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

enum Kind { K_SHARD = 0, K_VALIDATE = 1, K_INTERP = 2 };

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
    // validate
    const uint8_t *root = nullptr;
    const uint8_t *branch = nullptr;
    size_t branch_len = 0;
    const uint8_t *shard = nullptr;
    size_t shard_len = 0;
    uint32_t index = 0;
    int *ok_out = nullptr;
    // interpolate
    std::vector<const uint8_t *> in_shards;
    std::vector<size_t> in_lens;
    uint8_t *value_out = nullptr;
    size_t value_cap = 0;
    size_t *value_len = nullptr;
    uint8_t *digest_out = nullptr;
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
    Pinned shards, roots, br, values;
};

}  // namespace

struct rbc_batcher {
    rbc_ctx *ctx = nullptr;
    int n = 0, k = 0, depth = 0;
    int max_batch = 256;
    int max_wait_us = 200;
    std::mutex mu;
    std::condition_variable cv_work;
    std::deque<Req> q[3];
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

    void run();
    std::vector<std::unique_ptr<PinnedSet>> pool;  // worker thread only

    std::unique_ptr<struct Pending> submit(Kind kind, std::vector<Req> &&batch);
    void finish(struct Pending &p);
};

namespace {

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
    std::vector<uint8_t> ok, present, digests;
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
    if (pool.empty()) {
        P->pin = std::make_unique<PinnedSet>();
    } else {
        P->pin = std::move(pool.back());
        pool.pop_back();
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
    } else if (kind == K_VALIDATE) {
        std::vector<const uint8_t *> sh(count), brs(count), rts(count);
        std::vector<size_t> sl(count), bl(count);
        std::vector<uint32_t> ix(count);
        P->ok.assign(count, 0);
        for (int i = 0; i < count; ++i) {
            sh[i] = b[i].shard;
            sl[i] = b[i].shard_len;
            brs[i] = b[i].branch;
            bl[i] = b[i].branch_len;
            rts[i] = b[i].root;
            ix[i] = b[i].index;
        }
        P->rc = rbc_validate_batch(ctx, count, sh.data(), sl.data(), ix.data(), brs.data(), bl.data(), rts.data(),
                                   P->ok.data(), &P->ticket);
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
            P->shards = P->pin->shards.ensure((size_t)m * n * Smax);
            P->roots = P->pin->roots.ensure((size_t)m * 32);
            P->values = P->pin->values.ensure((size_t)m * k * Smax);
            P->present.assign((size_t)m * n, 0);
            P->digests.resize((size_t)m * 32);
            P->lens.resize(m);
            P->status.assign(m, 0);
            if (!P->shards || !P->roots || !P->values) {
                P->rc = RBC_ERR_DEVICE;
                return P;
            }
            for (int t = 0; t < m; ++t) P->lens[t] = S[P->idx[t]];
            parallel_for(m, (size_t)n * Smax, [&](int t) {
                Req &r = b[P->idx[t]];
                for (int j = 0; j < n; ++j)
                    if (r.in_lens[j]) {
                        uint8_t *row = P->shards + ((size_t)t * n + j) * Smax;
                        memcpy(row, r.in_shards[j], P->lens[t]);
                        if (P->lens[t] < Smax) memset(row + P->lens[t], 0, Smax - P->lens[t]);
                        P->present[(size_t)t * n + j] = 1;
                    }
                memcpy(P->roots + (size_t)t * 32, r.root, 32);
            });
            P->rc = rbc_interpolate_batch(ctx, m, P->shards, Smax, P->lens.data(), P->present.data(), P->roots,
                                          P->values, (size_t)k * Smax, P->digests.data(), P->status.data(),
                                          &P->ticket);
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
    } else if (P.kind == K_VALIDATE) {
        for (int i = 0; i < count; ++i) {
            if (rc) P.st[i] = rc;
            else *b[i].ok_out = P.ok[i];
        }
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
    if (P.pin) pool.push_back(std::move(P.pin));  // the launch is complete: its buffers are free
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

// Worker: coalesce, submit asynchronously, and complete launches in order.
// Up to `depth` launches are in flight, so the host-side staging of batch
// t+1 overlaps the GPU work (and copies) of batch t.
void rbc_batcher::run() {
    std::deque<std::unique_ptr<Pending>> inflight;
    // launches in flight: 4 (41 vs 27 GB/s of shard + commit through the
    // coalescer at 2); the context has as many host slots
    constexpr size_t depth_max = 4;
    std::unique_lock<std::mutex> lk(mu);
    while (true) {
        // pick the kind whose queue is full, or whose oldest request is due
        const auto now = std::chrono::steady_clock::now();
        int pick = -1;
        auto earliest = now + std::chrono::hours(1);
        for (int kd = 0; kd < 3; ++kd) {
            if (q[kd].empty()) continue;
            const auto due = q[kd].front().t0 + std::chrono::microseconds(max_wait_us);
            if ((int)q[kd].size() >= max_batch || due <= now || stop) { pick = kd; break; }
            earliest = std::min(earliest, due);
        }
        if (pick < 0) {
            if (!inflight.empty()) {  // nothing new is due: complete what runs
                lk.unlock();
                finish(*inflight.front());
                inflight.pop_front();
                lk.lock();
                continue;
            }
            if (stop) return;
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
        inflight.push_back(submit((Kind)pick, std::move(batch)));
        if (inflight.size() >= depth_max) {
            finish(*inflight.front());
            inflight.pop_front();
        }
        lk.lock();
    }
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
    b->worker = std::thread([b] { b->run(); });
    *out = b;
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
    if (!b || !ticket || !ok_out || !root) return RBC_ERR_INVALID_ARG;
    *ok_out = 0;
    Req r;
    r.kind = K_VALIDATE;
    r.root = root;
    r.branch = branch;
    r.branch_len = branch_len;
    r.shard = shard;
    r.shard_len = shard_len;
    r.index = index;
    r.ok_out = ok_out;
    *ticket = enqueue(b, std::move(r));
    return RBC_OK;
}

int rbc_batcher_interpolate(rbc_batcher *b, const uint8_t *root, const uint8_t *const *shards, const size_t *lens,
                            uint8_t *value_out, size_t value_cap, size_t *value_len, uint8_t *digest_out,
                            uint64_t *ticket) {
    if (!b || !ticket || !root || !shards || !lens || !value_out) return RBC_ERR_INVALID_ARG;
    Req r;
    r.kind = K_INTERP;
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

int rbc_batcher_wait(rbc_batcher *b, uint64_t ticket) {
    if (!b) return RBC_ERR_INVALID_ARG;
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
    if (ticket == 0 || ticket >= b->next.load()) return RBC_ERR_INVALID_ARG;
    auto &sh = b->shard[ticket % rbc_batcher::kShards];
    std::lock_guard<std::mutex> lk(sh.mu);
    *done_out = sh.done.count(ticket) != 0;
    return RBC_OK;
}

int rbc_batcher_stats(rbc_batcher *b, uint64_t *batches, uint64_t *requests) {
    if (!b) return RBC_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(b->mu);
    if (batches) *batches = b->batches;
    if (requests) *requests = b->requests;
    return RBC_OK;
}

}  // extern "C"
