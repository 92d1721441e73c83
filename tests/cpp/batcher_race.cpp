// batcher_race.cpp -- race / memory checking of the request batcher
// (csrc/batcher.cpp) on the CPU, for SURVEY 5's "race detection" row.
//
// The batcher is built unchanged and linked against a stand-in for the
// context's host batch API (rbc_shard_commit / rbc_validate_batch /
// rbc_interpolate_batch / rbc_wait, include/rbc_gpu.h) that computes with the
// C oracle (oracle/c/rbc_ref.c) on one thread per ticket and finishes when
// rbc_wait joins it.  That is the contract the real API gives the batcher:
// caller buffers are read and written at some point between submit and the
// ticket's completion.  So a batcher that touched a launch's buffers (or
// reused its pinned set) before rbc_wait returned, or completed a request
// before its results were copied, races with that thread -- ThreadSanitizer
// reports it, and the result checks below catch what it does to the bytes.
//
// Many client threads submit a seeded random mix of shard / validate /
// interpolate requests (well-formed and malformed) and complete them by wait
// or poll in random order; every result is compared with a direct oracle
// call.  Built twice by tests/test_sanitizers.py: -fsanitize=thread (with
// ROCm's clang, whose TSan runtime intercepts pthread_cond_clockwait -- the
// gcc 11 one does not and reports std::condition_variable::wait_until as a
// double lock) and -fsanitize=address,undefined (g++).  Test infrastructure only (CPU, no GPU).
//   run: batcher_race [threads] [requests_per_thread]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "../../include/rbc_gpu.h"

extern "C" {
int rbcref_encode_commit(int n, int f, const uint8_t *value, size_t B, uint8_t *shards, size_t pitch,
                         uint8_t *root, uint8_t *branches, uint8_t *leaves_out);
int rbcref_interpolate(int n, int f, const uint8_t *shards, size_t pitch, size_t S, const uint8_t *valid,
                       const uint8_t *root, uint8_t *value_out, uint8_t *digest_out);
int rbcref_merkle_verify(int n, const uint8_t *shard, size_t S, uint32_t index, const uint8_t *branch,
                         const uint8_t *root);
int rbcref_tree_depth(int n);
}

// ------------------------------------------------ stand-in context (oracle)
struct rbc_ctx {
    int n, f, k, d;
    std::mutex mu;
    uint64_t next = 1;
    std::map<uint64_t, std::pair<std::thread, std::shared_ptr<int>>> inflight;
};

namespace {

uint64_t launch(rbc_ctx *c, std::function<int()> work) {
    auto rc = std::make_shared<int>(0);
    std::lock_guard<std::mutex> lk(c->mu);
    const uint64_t t = c->next++;
    c->inflight.emplace(t, std::make_pair(std::thread([rc, work] { *rc = work(); }), rc));
    return t;
}

// Go flat branch -> the oracle's [d][32] form (zero slot for an empty level-0 sibling)
bool unflatten(int n, int d, uint32_t j, const uint8_t *br, size_t len, uint8_t *out) {
    const bool empty0 = (j ^ 1u) >= (uint32_t)n;
    const size_t want = (size_t)(d - (empty0 && d > 0)) * 32;
    if (len != want) return false;
    if (empty0 && d > 0) {
        memset(out, 0, 32);
        memcpy(out + 32, br, len);
    } else {
        memcpy(out, br, len);
    }
    return true;
}

}  // namespace

extern "C" {

int rbc_ctx_params(const rbc_ctx *c, int *k, int *p, int *depth) {
    if (k) *k = c->k;
    if (p) *p = c->n - c->k;
    if (depth) *depth = c->d;
    return RBC_OK;
}

int rbc_host_alloc(size_t bytes, void **ptr) {
    *ptr = malloc(bytes);
    return *ptr ? RBC_OK : RBC_ERR_DEVICE;
}

int rbc_host_free(void *ptr) {
    free(ptr);
    return RBC_OK;
}

int rbc_shard_commit(rbc_ctx *c, int count, const uint8_t *const *values, const size_t *value_lens,
                     uint8_t *shards_out, size_t pitch, uint32_t *slens, uint8_t *roots, uint8_t *branches,
                     uint64_t *ticket) {
    for (int i = 0; i < count; ++i)
        if (!value_lens[i] || (value_lens[i] + c->k - 1) / c->k > pitch) return RBC_ERR_INVALID_ARG;
    // like the real API: the pointer and length arrays are read at submit,
    // the bytes they point to at some point before completion
    std::vector<const uint8_t *> vp(values, values + count);
    std::vector<size_t> vl(value_lens, value_lens + count);
    *ticket = launch(c, [=] {
        for (int i = 0; i < count; ++i) {
            slens[i] = (uint32_t)((vl[i] + c->k - 1) / c->k);
            const int rc = rbcref_encode_commit(c->n, c->f, vp[i], vl[i],
                                                shards_out + (size_t)i * c->n * pitch, pitch, roots + 32 * i,
                                                branches + (size_t)i * c->n * c->d * 32, nullptr);
            if (rc) return RBC_ERR_DEVICE;
        }
        return RBC_OK;
    });
    return RBC_OK;
}

int rbc_validate_batch(rbc_ctx *c, int count, const uint8_t *const *shards, const size_t *shard_lens,
                       const uint32_t *indices, const uint8_t *const *branches, const size_t *branch_lens,
                       const uint8_t *const *roots, uint8_t *ok_out, uint64_t *ticket) {
    std::vector<const uint8_t *> sp(shards, shards + count), bp(branches, branches + count),
        rp(roots, roots + count);
    std::vector<size_t> sl(shard_lens, shard_lens + count), bl(branch_lens, branch_lens + count);
    std::vector<uint32_t> ix(indices, indices + count);
    auto work = [=] {
        std::vector<uint8_t> br((size_t)std::max(c->d, 1) * 32);
        for (int i = 0; i < count; ++i)
            ok_out[i] = sl[i] && ix[i] < (uint32_t)c->n &&
                        unflatten(c->n, c->d, ix[i], bp[i], bl[i], br.data()) &&
                        rbcref_merkle_verify(c->n, sp[i], sl[i], ix[i], br.data(), rp[i]);
        return RBC_OK;
    };
    if (!ticket) return work();  // a NULL ticket: synchronous, as the real API
    *ticket = launch(c, work);
    return RBC_OK;
}

int rbc_validate_packed(rbc_ctx *c, int count, const uint8_t *arena, size_t arena_bytes, const uint64_t *offs,
                        const uint32_t *lens, const uint8_t *idx, const uint8_t *branches, const uint8_t *roots,
                        uint8_t *ok_out, uint64_t *ticket) {
    // the real API's argument checks, then the arena read at some point before completion
    for (int i = 0; i < count; ++i)
        if (offs[i] % 64 || !lens[i] || offs[i] + (lens[i] + 63) / 64 * 64 > arena_bytes || idx[i] >= c->n)
            return RBC_ERR_INVALID_ARG;
    const size_t bslot = (size_t)std::max(c->d, 1) * 32;
    *ticket = launch(c, [=] {
        for (int i = 0; i < count; ++i)
            ok_out[i] = rbcref_merkle_verify(c->n, arena + offs[i], lens[i], idx[i], branches + i * bslot,
                                             roots + 32 * i);
        return RBC_OK;
    });
    return RBC_OK;
}

int rbc_interpolate_batch(rbc_ctx *c, int count, const uint8_t *shards, size_t pitch, const size_t *shard_lens,
                          const uint8_t *present, const uint8_t *roots, uint8_t *values_out, size_t value_pitch,
                          uint8_t *digests_out, int32_t *status_out, uint64_t *ticket) {
    for (int i = 0; i < count; ++i)
        if (shard_lens[i] > pitch || (size_t)c->k * shard_lens[i] > value_pitch) return RBC_ERR_INVALID_ARG;
    std::vector<size_t> sl(shard_lens, shard_lens + count);
    *ticket = launch(c, [=] {
        for (int i = 0; i < count; ++i)
            status_out[i] = rbcref_interpolate(c->n, c->f, shards + (size_t)i * c->n * pitch, pitch, sl[i],
                                               present + (size_t)i * c->n, roots + 32 * i,
                                               values_out + (size_t)i * value_pitch,
                                               digests_out ? digests_out + 32 * i : nullptr);
        return RBC_OK;
    });
    return RBC_OK;
}

int rbc_wait(rbc_ctx *c, uint64_t ticket) {
    std::thread th;
    std::shared_ptr<int> rc;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        auto it = c->inflight.find(ticket);
        if (it == c->inflight.end()) return RBC_ERR_INVALID_ARG;
        th = std::move(it->second.first);
        rc = it->second.second;
        c->inflight.erase(it);
    }
    th.join();
    return *rc;
}

}  // extern "C"

// ---------------------------------------------------------------- driver
namespace {

struct Commit {  // one proposal committed by the oracle
    std::vector<uint8_t> value, shards, branches;  // shards [n][S]; branches [n][d][32]
    size_t S = 0;
    uint8_t root[32];
};

Commit commit(int n, int f, std::vector<uint8_t> v) {
    Commit cm;
    const int k = n - 2 * f, d = rbcref_tree_depth(n);
    cm.S = (v.size() + k - 1) / k;
    cm.shards.resize((size_t)n * cm.S);
    cm.branches.resize((size_t)n * d * 32);
    if (rbcref_encode_commit(n, f, v.data(), v.size(), cm.shards.data(), cm.S, cm.root, cm.branches.data(),
                             nullptr))
        abort();
    cm.value = std::move(v);
    return cm;
}

std::vector<uint8_t> flat_branch(int n, int d, const Commit &cm, uint32_t j) {
    std::vector<uint8_t> out;
    for (int l = 0; l < d; ++l) {
        if (l == 0 && (j ^ 1u) >= (uint32_t)n) continue;
        const uint8_t *p = cm.branches.data() + ((size_t)j * d + l) * 32;
        out.insert(out.end(), p, p + 32);
    }
    return out;
}

std::atomic<int> failures{0};

#define EXPECT(cond, ...)                           \
    do {                                            \
        if (!(cond)) {                              \
            fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);           \
            fprintf(stderr, "\n");                  \
            ++failures;                             \
        }                                           \
    } while (0)

// One outstanding request: the buffers it owns and how to check them.
struct Outstanding {
    uint64_t ticket = 0;
    int want_status = 0;
    std::function<void()> check;
    // owned buffers (stable addresses: heap vectors held by this object)
    std::vector<uint8_t> in, shards, root, branches, value, digest, brflat, shard;
    std::vector<std::vector<uint8_t>> rows;
    std::vector<const uint8_t *> ptrs;
    std::vector<size_t> lens;
    size_t out_len = 0;
    int ok = -1;
};

void client(rbc_batcher *bt, int n, int f, int id, int reqs, const std::vector<Commit> *pool) {
    const int k = n - 2 * f, d = rbcref_tree_depth(n);
    std::mt19937_64 rng(0x9e3779b97f4a7c15ull * (id + 1));
    auto rnd = [&](int lo, int hi) { return (int)(lo + rng() % (uint64_t)(hi - lo + 1)); };
    std::vector<std::unique_ptr<Outstanding>> live;
    auto complete = [&](Outstanding &o) {
        int rc;
        if (rnd(0, 1)) {
            int done = 0;
            while (rbc_batcher_poll(bt, o.ticket, &done) == RBC_OK && !done) std::this_thread::yield();
            rc = rbc_batcher_wait(bt, o.ticket);
        } else {
            rc = rbc_batcher_wait(bt, o.ticket);
        }
        EXPECT(rc == o.want_status, "client %d ticket %llu: status %d, want %d", id,
               (unsigned long long)o.ticket, rc, o.want_status);
        if (rc == RBC_OK && o.check) o.check();
    };
    for (int r = 0; r < reqs; ++r) {
        auto o = std::make_unique<Outstanding>();
        Outstanding &O = *o;
        const int kind = rnd(0, 2);
        const Commit &cm = (*pool)[rng() % pool->size()];
        uint64_t t = 0;
        if (kind == 0) {  // shard + commit of a fresh value
            O.in.resize(rnd(1, 5000));
            for (auto &c : O.in) c = (uint8_t)rng();
            const Commit want = commit(n, f, O.in);
            const bool small = rnd(0, 9) == 0;  // output buffer one byte short
            O.shards.resize((size_t)n * want.S - (small ? 1 : 0));
            O.root.resize(32);
            O.branches.resize((size_t)n * d * 32);
            O.want_status = small ? RBC_ERR_INVALID_ARG : RBC_OK;
            EXPECT(rbc_batcher_shard(bt, O.in.data(), O.in.size(), O.shards.data(), O.shards.size(), &O.out_len,
                                     O.root.data(), O.branches.data(), &t) == RBC_OK, "shard submit");
            O.check = [&O, want] {
                EXPECT(O.out_len == want.S && O.shards == want.shards && !memcmp(O.root.data(), want.root, 32) &&
                           O.branches == want.branches, "shard result differs from the oracle");
            };
        } else if (kind == 1) {  // validateMessage of one ECHO, maybe tampered
            const uint32_t j = (uint32_t)rnd(0, n - 1);
            O.shard.assign(cm.shards.begin() + (size_t)j * cm.S, cm.shards.begin() + (size_t)(j + 1) * cm.S);
            O.brflat = flat_branch(n, d, cm, j);
            O.root.assign(cm.root, cm.root + 32);
            const int tamper = rnd(0, 4);  // 0 shard, 1 branch, 2 root, 3-4 none
            if (tamper == 0) O.shard[rng() % O.shard.size()] ^= 1 << rnd(0, 7);
            if (tamper == 1 && !O.brflat.empty()) O.brflat[rng() % O.brflat.size()] ^= 0x80;
            if (tamper == 2) O.root[rnd(0, 31)] ^= 0x01;
            const bool expect = tamper >= 3 || (tamper == 1 && O.brflat.empty());
            O.want_status = RBC_OK;
            EXPECT(rbc_batcher_validate(bt, O.root.data(), O.brflat.data(), O.brflat.size(), O.shard.data(),
                                        O.shard.size(), j, &O.ok, &t) == RBC_OK, "validate submit");
            O.check = [&O, expect] { EXPECT(O.ok == (int)expect, "validate ok=%d want %d", O.ok, (int)expect); };
        } else {  // interpolate from a random present subset, maybe one shard corrupted
            O.rows.resize(n);
            O.ptrs.assign(n, nullptr);
            O.lens.assign(n, 0);
            std::vector<uint8_t> valid(n, 0);
            const int have = rnd(k - 1, n);
            std::vector<int> perm(n);
            for (int j = 0; j < n; ++j) perm[j] = j;
            std::shuffle(perm.begin(), perm.end(), rng);
            for (int q = 0; q < have; ++q) valid[perm[q]] = 1;
            const int bad = rnd(0, 3) == 0 ? perm[rnd(0, std::max(have - 1, 0))] : -1;
            const bool ragged = rnd(0, 15) == 0 && have >= 2;
            std::vector<uint8_t> flat((size_t)n * cm.S, 0);
            for (int j = 0; j < n; ++j) {
                if (!valid[j]) continue;
                O.rows[j].assign(cm.shards.begin() + (size_t)j * cm.S, cm.shards.begin() + (size_t)(j + 1) * cm.S);
                if (j == bad) O.rows[j][0] ^= 0x5a;
                memcpy(flat.data() + (size_t)j * cm.S, O.rows[j].data(), cm.S);
                O.ptrs[j] = O.rows[j].data();
                O.lens[j] = cm.S;
            }
            if (ragged) O.lens[perm[0]] = cm.S + 1;  // klauspost ErrShardSize
            O.root.assign(cm.root, cm.root + 32);
            const bool small = rnd(0, 15) == 0;
            O.value.resize((size_t)k * cm.S - (small ? 1 : 0));
            O.digest.resize(32);
            std::vector<uint8_t> want_value((size_t)k * cm.S), want_digest(32);
            int want = have < k ? RBC_ERR_TOO_FEW_SHARDS
                                : rbcref_interpolate(n, f, flat.data(), cm.S, cm.S, valid.data(), cm.root,
                                                     want_value.data(), want_digest.data());
            if (ragged) want = RBC_ERR_SHARD_SIZE;
            else if (small && have >= k) want = RBC_ERR_INVALID_ARG;
            O.want_status = want;
            EXPECT(rbc_batcher_interpolate(bt, O.root.data(), O.ptrs.data(), O.lens.data(), O.value.data(),
                                           O.value.size(), &O.out_len, O.digest.data(), &t) == RBC_OK,
                   "interpolate submit");
            O.check = [&O, want_value, want_digest] {
                EXPECT(O.out_len == want_value.size() && O.value == want_value && O.digest == want_digest,
                       "interpolate result differs from the oracle");
            };
        }
        O.ticket = t;
        live.push_back(std::move(o));
        // keep a few requests outstanding; complete a random one at times
        while (!live.empty() && (live.size() > 6 || rnd(0, 2) == 0)) {
            const size_t i = rng() % live.size();
            complete(*live[i]);
            live.erase(live.begin() + i);
        }
    }
    std::shuffle(live.begin(), live.end(), rng);
    for (auto &o : live) complete(*o);
}

}  // namespace

int main(int argc, char **argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 12;
    const int R = argc > 2 ? atoi(argv[2]) : 150;
    const int geo[][2] = {{4, 1}, {7, 2}, {16, 5}};
    for (auto &g : geo) {
        const int n = g[0], f = g[1];
        rbc_ctx ctx;
        ctx.n = n;
        ctx.f = f;
        ctx.k = n - 2 * f;
        ctx.d = rbcref_tree_depth(n);
        std::vector<Commit> pool;
        std::mt19937_64 rng(n);
        for (int i = 0; i < 8; ++i) {
            std::vector<uint8_t> v(1 + rng() % 3000);
            for (auto &c : v) c = (uint8_t)rng();
            pool.push_back(commit(n, f, std::move(v)));
        }
        for (const int max_batch : {1, 5, 64}) {
            rbc_batcher *bt = nullptr;
            if (rbc_batcher_create(&ctx, max_batch, 300, &bt) != RBC_OK) return 2;
            // small validate arenas: sealed by count, by bytes, and grown for one large message
            if (rbc_batcher_set_validate(bt, max_batch, max_batch == 64 ? 1024 : 4096) != RBC_OK) return 2;  // 1 KiB: larger shards take the direct path
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t) th.emplace_back(client, bt, n, f, t, R, &pool);
            for (auto &x : th) x.join();
            uint64_t nb = 0, nr = 0;
            rbc_batcher_stats(bt, &nb, &nr);
            EXPECT(nr == (uint64_t)T * R, "batcher served %llu of %d requests", (unsigned long long)nr, T * R);
            rbc_batcher_destroy(bt);
            printf("n=%d f=%d max_batch=%d: %llu requests in %llu launches\n", n, f, max_batch,
                   (unsigned long long)nr, (unsigned long long)nb);
        }
        if (!ctx.inflight.empty()) {
            fprintf(stderr, "FAIL: %zu launches never waited\n", ctx.inflight.size());
            ++failures;
        }
    }
    if (failures) {
        printf("FAILED %d\n", failures.load());
        return 1;
    }
    printf("ok\n");
    return 0;
}
