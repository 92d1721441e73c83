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
int rbcref_interpolate_leaves(int n, int f, const uint8_t *shards, size_t pitch, size_t S, const uint8_t *valid,
                              const uint8_t *leaves, const uint8_t *root, uint8_t *value_out, uint8_t *digest_out);
int rbcref_tree_depth(int n);
void rbcref_sha256(const uint8_t *p, size_t n, uint8_t out[32]);
}

// Failure injection of the validate lane's launches: when
// g_fail_mod > 0, the packed launch number q (1-based, launch order) fails
// at completion when q % g_fail_mod == 0 -- the arena of generation q, since
// the lane launches one arena per generation in order.
static std::atomic<int> g_fail_mod{0}, g_packed_calls{0};

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

int rbc_ctx_device(const rbc_ctx *, int *device) {
    *device = 0;
    return RBC_OK;
}

// "device" memory of the stand-in: host memory the launch threads read
int rbc_dev_malloc(int, size_t bytes, void **ptr) {
    *ptr = malloc(bytes);
    return *ptr ? RBC_OK : RBC_ERR_DEVICE;
}

int rbc_dev_free(void *ptr) {
    free(ptr);
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

int rbc_validate_packed_leaves(rbc_ctx *c, int count, const uint8_t *arena, size_t arena_bytes, const uint64_t *offs,
                               const uint32_t *lens, const uint8_t *idx, const uint8_t *branches, const uint8_t *roots,
                               uint8_t *ok_out, uint8_t *leaves_out, uint64_t *ticket) {
    // the real API's argument checks, then the arena read at some point before completion
    for (int i = 0; i < count; ++i)
        if (offs[i] % 64 || !lens[i] || offs[i] + (lens[i] + 63) / 64 * 64 > arena_bytes || idx[i] >= c->n)
            return RBC_ERR_INVALID_ARG;
    const size_t bslot = (size_t)std::max(c->d, 1) * 32;
    const int q = ticket ? ++g_packed_calls : 0, mod = g_fail_mod.load();  // (a synchronous call is no lane launch)
    const bool fail = mod > 0 && q > 0 && q % mod == 0;
    auto work = [=] {
        if (fail) {  // a failed launch writes nothing (a device error before the D2H)
            return RBC_ERR_DEVICE;
        }
        for (int i = 0; i < count; ++i) {
            ok_out[i] = rbcref_merkle_verify(c->n, arena + offs[i], lens[i], idx[i], branches + i * bslot,
                                             roots + 32 * i);
            if (leaves_out) rbcref_sha256(arena + offs[i], lens[i], leaves_out + 32 * (size_t)i);
        }
        return RBC_OK;
    };
    if (!ticket) return work();  // a NULL ticket: synchronous, as the real API
    *ticket = launch(c, work);
    return RBC_OK;
}

// ABI 7: the arena moves into keep_dev (as the device copy would) and is
// verified from there
int rbc_validate_packed_keep(rbc_ctx *c, int count, const uint8_t *arena, size_t arena_bytes, const uint64_t *offs,
                             const uint32_t *lens, const uint8_t *idx, const uint8_t *branches, const uint8_t *roots,
                             uint8_t *ok_out, uint8_t *leaves_out, uint8_t *keep_dev, size_t keep_bytes,
                             uint64_t *ticket) {
    if (!keep_dev || keep_bytes < arena_bytes) return RBC_ERR_INVALID_ARG;
    for (int i = 0; i < count; ++i)
        if (offs[i] % 64 || !lens[i] || offs[i] + (lens[i] + 63) / 64 * 64 > arena_bytes || idx[i] >= c->n)
            return RBC_ERR_INVALID_ARG;
    const size_t bslot = (size_t)std::max(c->d, 1) * 32;
    *ticket = launch(c, [=] {
        memcpy(keep_dev, arena, arena_bytes);
        for (int i = 0; i < count; ++i) {
            ok_out[i] = rbcref_merkle_verify(c->n, keep_dev + offs[i], lens[i], idx[i], branches + i * bslot,
                                             roots + 32 * i);
            if (leaves_out) rbcref_sha256(keep_dev + offs[i], lens[i], leaves_out + 32 * (size_t)i);
        }
        return RBC_OK;
    });
    return RBC_OK;
}

// ABI 7: rows read from the kept "device" addresses at some point before completion
int rbc_interpolate_batch_kept(rbc_ctx *c, int count, const uint8_t *const *rows, const size_t *shard_lens,
                               const uint8_t *leaves, const uint8_t *roots, uint8_t *values_out, size_t value_pitch,
                               uint8_t *digests_out, int32_t *status_out, uint64_t *ticket) {
    for (int i = 0; i < count; ++i)
        if ((size_t)c->k * shard_lens[i] > value_pitch) return RBC_ERR_INVALID_ARG;
    std::vector<const uint8_t *> rp(rows, rows + (size_t)count * c->n);
    std::vector<size_t> sl(shard_lens, shard_lens + count);
    *ticket = launch(c, [=] {
        for (int i = 0; i < count; ++i) {
            const size_t S = sl[i];
            std::vector<uint8_t> flat((size_t)c->n * S, 0), valid(c->n, 0);
            for (int j = 0; j < c->n; ++j)
                if (const uint8_t *r = rp[(size_t)i * c->n + j]) {
                    memcpy(flat.data() + (size_t)j * S, r, S);
                    valid[j] = 1;
                }
            status_out[i] =
                leaves ? rbcref_interpolate_leaves(c->n, c->f, flat.data(), S, S, valid.data(),
                                                   leaves + (size_t)i * c->n * 32, roots + 32 * i,
                                                   values_out + (size_t)i * value_pitch,
                                                   digests_out ? digests_out + 32 * i : nullptr)
                       : rbcref_interpolate(c->n, c->f, flat.data(), S, S, valid.data(), roots + 32 * i,
                                            values_out + (size_t)i * value_pitch,
                                            digests_out ? digests_out + 32 * i : nullptr);
        }
        return RBC_OK;
    });
    return RBC_OK;
}

int rbc_interpolate_batch_verified(rbc_ctx *c, int count, const uint8_t *shards, size_t pitch,
                                   const size_t *shard_lens, const uint8_t *present, const uint8_t *leaves,
                                   const uint8_t *roots, uint8_t *values_out, size_t value_pitch,
                                   uint8_t *digests_out, int32_t *status_out, uint64_t *ticket) {
    for (int i = 0; i < count; ++i)
        if (shard_lens[i] > pitch || (size_t)c->k * shard_lens[i] > value_pitch) return RBC_ERR_INVALID_ARG;
    std::vector<size_t> sl(shard_lens, shard_lens + count);
    *ticket = launch(c, [=] {
        for (int i = 0; i < count; ++i)
            status_out[i] =
                leaves ? rbcref_interpolate_leaves(c->n, c->f, shards + (size_t)i * c->n * pitch, pitch, sl[i],
                                                   present + (size_t)i * c->n, leaves + (size_t)i * c->n * 32,
                                                   roots + 32 * i, values_out + (size_t)i * value_pitch,
                                                   digests_out ? digests_out + 32 * i : nullptr)
                       : rbcref_interpolate(c->n, c->f, shards + (size_t)i * c->n * pitch, pitch, sl[i],
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
            if (rnd(0, 1)) {  // with the leaf (ABI 6)
                O.digest.assign(32, 0);
                EXPECT(rbc_batcher_validate_leaf(bt, O.root.data(), O.brflat.data(), O.brflat.size(), O.shard.data(),
                                                 O.shard.size(), j, &O.ok, O.digest.data(), &t) == RBC_OK,
                       "validate_leaf submit");
                O.check = [&O, expect] {
                    EXPECT(O.ok == (int)expect, "validate ok=%d want %d", O.ok, (int)expect);
                    uint8_t want[32];
                    rbcref_sha256(O.shard.data(), O.shard.size(), want);
                    if (O.ok == 1) EXPECT(!memcmp(want, O.digest.data(), 32), "validate leaf differs");
                };
            } else {
                EXPECT(rbc_batcher_validate(bt, O.root.data(), O.brflat.data(), O.brflat.size(), O.shard.data(),
                                            O.shard.size(), j, &O.ok, &t) == RBC_OK, "validate submit");
                O.check = [&O, expect] { EXPECT(O.ok == (int)expect, "validate ok=%d want %d", O.ok, (int)expect); };
            }
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
            const bool verified = rnd(0, 1) != 0;  // the present rows' leaves handed in (ABI 6)
            O.in.assign((size_t)n * 32, 0);
            for (int j = 0; j < n; ++j)
                if (valid[j]) rbcref_sha256(flat.data() + (size_t)j * cm.S, cm.S, O.in.data() + (size_t)j * 32);
            int want = have < k ? RBC_ERR_TOO_FEW_SHARDS
                       : verified ? rbcref_interpolate_leaves(n, f, flat.data(), cm.S, cm.S, valid.data(), O.in.data(),
                                                              cm.root, want_value.data(), want_digest.data())
                                  : rbcref_interpolate(n, f, flat.data(), cm.S, cm.S, valid.data(), cm.root,
                                                       want_value.data(), want_digest.data());
            if (ragged) want = RBC_ERR_SHARD_SIZE;
            else if (small && have >= k) want = RBC_ERR_INVALID_ARG;
            O.want_status = want;
            if (verified)
                EXPECT(rbc_batcher_interpolate_verified(bt, O.root.data(), O.ptrs.data(), O.lens.data(), O.in.data(),
                                                        O.value.data(), O.value.size(), &O.out_len, O.digest.data(),
                                                        &t) == RBC_OK, "interpolate_verified submit");
            else
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

// failed validate launches.  Every 3rd packed launch fails in the
// stand-in: rbc_batcher_wait must return the error for exactly the tickets of
// that launch's arena (generation g: ticket = 1 << 63 | g << 20 | slot),
// ok_out must stay 0 for them, and rbc_batcher_poll must report them done.
// Leaves are requested for every other message and must be the oracle's
// SHA-256 of the shard wherever the verdict is 1.
void failed_launches(int n, int f, const std::vector<Commit> &pool, int T, int R) {
    const int d = rbcref_tree_depth(n);
    rbc_ctx ctx;
    ctx.n = n;
    ctx.f = f;
    ctx.k = n - 2 * f;
    ctx.d = d;
    g_fail_mod = 3;
    g_packed_calls = 0;
    rbc_batcher *bt = nullptr;
    if (rbc_batcher_create(&ctx, 8, 200, &bt) != RBC_OK || rbc_batcher_set_validate(bt, 7, 1 << 16) != RBC_OK) abort();
    std::atomic<int> failed_seen{0}, ok_seen{0};
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            std::mt19937_64 rng(77 + t);
            for (int r = 0; r < R; ++r) {
                const Commit &cm = pool[rng() % pool.size()];
                const uint32_t j = (uint32_t)(rng() % n);
                std::vector<uint8_t> shard(cm.shards.begin() + (size_t)j * cm.S,
                                           cm.shards.begin() + (size_t)(j + 1) * cm.S);
                std::vector<uint8_t> br = flat_branch(n, d, cm, j), leaf(32, 0xEE);
                int ok = -1;
                uint64_t tk = 0;
                const bool want_leaf = (r & 1) != 0;
                EXPECT(rbc_batcher_validate_leaf(bt, cm.root, br.data(), br.size(), shard.data(), shard.size(), j, &ok,
                                                 want_leaf ? leaf.data() : nullptr, &tk) == RBC_OK, "submit");
                const uint64_t gen = (tk & ~(1ull << 63)) >> 20;
                const int rc = rbc_batcher_wait(bt, tk);
                int done = 0;
                EXPECT(rbc_batcher_poll(bt, tk, &done) == RBC_OK && done == 1, "poll after wait");
                const bool fails = gen > 0 && gen % 3 == 0;
                EXPECT(rc == (fails ? RBC_ERR_DEVICE : RBC_OK), "gen %llu rc %d", (unsigned long long)gen, rc);
                EXPECT(ok == (fails ? 0 : 1), "gen %llu ok %d", (unsigned long long)gen, ok);
                if (want_leaf && ok == 1) {
                    uint8_t want[32];
                    rbcref_sha256(shard.data(), shard.size(), want);
                    EXPECT(!memcmp(want, leaf.data(), 32), "leaf differs from the oracle's SHA-256");
                }
                (fails ? failed_seen : ok_seen)++;
            }
        });
    for (auto &x : th) x.join();
    rbc_batcher_destroy(bt);
    g_fail_mod = 0;
    EXPECT(failed_seen > 0 && ok_seen > 0, "failure injection: %d failed, %d ok", failed_seen.load(), ok_seen.load());
    printf("n=%d f=%d failed launches: %d requests failed, %d ok\n", n, f, failed_seen.load(), ok_seen.load());
}

// rbc_batcher_destroy with requests still outstanding (open,
// sealed and in-flight arenas; queued shard / interpolate requests) drains
// them: after it returns every request's outputs are final.
void destroy_outstanding(int n, int f, const std::vector<Commit> &pool, int T, int R) {
    const int k = n - 2 * f, d = rbcref_tree_depth(n);
    rbc_ctx ctx;
    ctx.n = n;
    ctx.f = f;
    ctx.k = k;
    ctx.d = d;
    rbc_batcher *bt = nullptr;
    if (rbc_batcher_create(&ctx, 16, 5000, &bt) != RBC_OK || rbc_batcher_set_validate(bt, 11, 1 << 16) != RBC_OK)
        abort();
    struct Item {
        int kind;
        const Commit *cm;
        uint32_t j;
        int ok = -1;
        std::vector<uint8_t> shard, br, leaf, value, digest, out, root, brs;
        std::vector<const uint8_t *> ptrs;
        std::vector<size_t> lens;
        size_t out_len = 0;
    };
    std::vector<std::vector<std::unique_ptr<Item>>> items(T);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            std::mt19937_64 rng(991 + t);
            for (int r = 0; r < R; ++r) {
                auto it = std::make_unique<Item>();
                Item &I = *it;
                I.kind = (int)(rng() % 3);
                I.cm = &pool[rng() % pool.size()];
                uint64_t tk = 0;
                if (I.kind == 0) {
                    I.j = (uint32_t)(rng() % n);
                    I.shard.assign(I.cm->shards.begin() + (size_t)I.j * I.cm->S,
                                   I.cm->shards.begin() + (size_t)(I.j + 1) * I.cm->S);
                    I.br = flat_branch(n, d, *I.cm, I.j);
                    I.leaf.assign(32, 0);
                    EXPECT(rbc_batcher_validate_leaf(bt, I.cm->root, I.br.data(), I.br.size(), I.shard.data(),
                                                     I.shard.size(), I.j, &I.ok, I.leaf.data(), &tk) == RBC_OK, "v");
                } else if (I.kind == 1) {
                    I.out.resize((size_t)n * I.cm->S);
                    I.root.resize(32);
                    I.brs.resize((size_t)n * d * 32);
                    EXPECT(rbc_batcher_shard(bt, I.cm->value.data(), I.cm->value.size(), I.out.data(), I.out.size(),
                                             &I.out_len, I.root.data(), I.brs.data(), &tk) == RBC_OK, "s");
                } else {
                    I.ptrs.assign(n, nullptr);
                    I.lens.assign(n, 0);
                    for (int j = 0; j < n; ++j)
                        if (j % 3 != 1 || j < k) {  // at least k present
                            I.ptrs[j] = I.cm->shards.data() + (size_t)j * I.cm->S;
                            I.lens[j] = I.cm->S;
                        }
                    I.value.resize((size_t)k * I.cm->S);
                    I.digest.resize(32);
                    EXPECT(rbc_batcher_interpolate(bt, I.cm->root, I.ptrs.data(), I.lens.data(), I.value.data(),
                                                   I.value.size(), &I.out_len, I.digest.data(), &tk) == RBC_OK, "i");
                }
                items[t].push_back(std::move(it));  // never waited: destroy must drain it
            }
        });
    for (auto &x : th) x.join();
    rbc_batcher_destroy(bt);
    int n_checked = 0;
    for (auto &v : items)
        for (auto &it : v) {
            Item &I = *it;
            if (I.kind == 0) {
                uint8_t want[32];
                rbcref_sha256(I.shard.data(), I.shard.size(), want);
                EXPECT(I.ok == 1 && !memcmp(want, I.leaf.data(), 32), "validate not drained: ok=%d", I.ok);
            } else if (I.kind == 1) {
                EXPECT(I.out_len == I.cm->S && I.out == I.cm->shards && !memcmp(I.root.data(), I.cm->root, 32),
                       "shard not drained");
            } else {
                EXPECT(I.out_len == (size_t)k * I.cm->S && !memcmp(I.value.data(), I.cm->value.data(),
                                                                    I.cm->value.size()), "interpolate not drained");
            }
            ++n_checked;
        }
    printf("n=%d f=%d destroy with %d requests outstanding: all drained\n", n, f, n_checked);
}

// ABI 7, rbc_batcher_set_keep: each client runs RBC instances of its own
// (fresh values), validates every ECHO (some tampered) and interpolates the
// ones that validated -- the Go handlers' sequence.  A keep ring of a few
// arenas wraps many times, so launches are kept and not kept and regions are
// recycled while other clients' interpolates pin theirs; every 4th
// interpolate passes copies of the validated shards (another pointer: the host
// path).  Every value and digest must equal the oracle's, and both paths must
// have run.
void kept_epoch(int n, int f, int T, int R, size_t ring, bool require_kept) {
    const int k = n - 2 * f, d = rbcref_tree_depth(n);
    rbc_ctx ctx;
    ctx.n = n;
    ctx.f = f;
    ctx.k = k;
    ctx.d = d;
    rbc_batcher *bt = nullptr;
    if (rbc_batcher_create(&ctx, 4, 200, &bt) != RBC_OK || rbc_batcher_set_validate(bt, 9, 1 << 14) != RBC_OK ||
        rbc_batcher_set_keep(bt, ring) != RBC_OK)
        abort();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            std::mt19937_64 rng(4242 + t);
            for (int r = 0; r < R; ++r) {
                std::vector<uint8_t> v(1 + rng() % 2500);
                for (auto &c : v) c = (uint8_t)rng();
                const Commit cm = commit(n, f, v);
                std::vector<std::vector<uint8_t>> rows(n), brs(n);
                std::vector<int> ok(n, -1);
                std::vector<uint64_t> tk(n, 0);
                const int bad = (int)(rng() % (2 * n)) - n;  // < 0: none tampered
                for (int j = 0; j < n; ++j) {
                    rows[j].assign(cm.shards.begin() + (size_t)j * cm.S, cm.shards.begin() + (size_t)(j + 1) * cm.S);
                    if (j == bad) rows[j][rng() % cm.S] ^= 0x10;
                    brs[j] = flat_branch(n, d, cm, (uint32_t)j);
                    EXPECT(rbc_batcher_validate(bt, cm.root, brs[j].data(), brs[j].size(), rows[j].data(),
                                                rows[j].size(), (uint32_t)j, &ok[j], &tk[j]) == RBC_OK, "kv");
                }
                std::vector<const uint8_t *> ptrs(n, nullptr);
                std::vector<size_t> lens(n, 0);
                std::vector<std::vector<uint8_t>> copies(n);
                const bool copy = r % 4 == 3;
                for (int j = 0; j < n; ++j) {
                    EXPECT(rbc_batcher_wait(bt, tk[j]) == RBC_OK, "kv wait");
                    EXPECT(ok[j] == (j != bad), "kept epoch verdict %d at %d", ok[j], j);
                    if (ok[j] == 1) {
                        copies[j] = rows[j];
                        ptrs[j] = copy ? copies[j].data() : rows[j].data();
                        lens[j] = cm.S;
                    }
                }
                std::vector<uint8_t> value((size_t)k * cm.S), digest(32), want_v((size_t)k * cm.S), want_d(32);
                std::vector<uint8_t> flat((size_t)n * cm.S, 0), valid(n, 0);
                for (int j = 0; j < n; ++j)
                    if (lens[j]) {
                        memcpy(flat.data() + (size_t)j * cm.S, rows[j].data(), cm.S);
                        valid[j] = 1;
                    }
                const int want = rbcref_interpolate(n, f, flat.data(), cm.S, cm.S, valid.data(), cm.root,
                                                    want_v.data(), want_d.data());
                size_t vlen = 0;
                uint64_t ti = 0;
                EXPECT(rbc_batcher_interpolate(bt, cm.root, ptrs.data(), lens.data(), value.data(), value.size(),
                                               &vlen, digest.data(), &ti) == RBC_OK, "ki");
                const int rc = rbc_batcher_wait(bt, ti);
                EXPECT(rc == want, "kept interpolate status %d want %d", rc, want);
                if (rc == RBC_OK)
                    EXPECT(value == want_v && digest == want_d && !memcmp(value.data(), v.data(), v.size()),
                           "kept interpolate result differs from the oracle");
            }
        });
    for (auto &x : th) x.join();
    uint64_t kept = 0, host = 0, kl = 0, ul = 0;
    rbc_batcher_keep_stats(bt, &kept, &host, &kl, &ul);
    rbc_batcher_destroy(bt);
    // the copies always take the host path; with a ring that holds many arenas the others find
    // their rows (a ring of a few arenas may recycle every region first under a slow sanitizer)
    EXPECT(host > 0 && (!require_kept || (kept > 0 && kl > 0)),
           "keep paths: %llu kept, %llu host interpolates, %llu kept launches", (unsigned long long)kept,
           (unsigned long long)host, (unsigned long long)kl);
    printf("n=%d f=%d keep ring %zu B: %llu interpolates from kept rows, %llu from host memory; %llu launches kept, "
           "%llu not\n", n, f, ring, (unsigned long long)kept, (unsigned long long)host, (unsigned long long)kl,
           (unsigned long long)ul);
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
        failed_launches(n, f, pool, std::min(T, 6), R);
        destroy_outstanding(n, f, pool, std::min(T, 6), std::max(R / 2, 8));
        kept_epoch(n, f, std::min(T, 8), std::max(R / 4, 8), (size_t)1 << 20, true);
        kept_epoch(n, f, std::min(T, 8), std::max(R / 4, 8), (size_t)6 << 10, false);  // arenas larger than the ring too
    }
    if (failures) {
        printf("FAILED %d\n", failures.load());
        return 1;
    }
    printf("ok\n");
    return 0;
}
