// rbc_test.cpp -- C++ tests of the C ABI, named after the reference's own
// (empty) Go tests so parity reads like them:
//   rbc/rbc_internal_test.go:21-31  Test_interpolate, Test_validateMessage, Test_shard
//   klauspost/reedsolomon v1.9.1 reedsolomon_test.go TestOneEncode / reconstruct tests
// Built by __graft_entry__.build() (tests/cpp/Makefile), run on the GPU by
// tests/test_cpp_abi.py.  Pure C-ABI client: no Python, no torch.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rbc_gpu.h"

static int failures = 0;
#define CHECK(cond)                                                               \
    do {                                                                          \
        if (!(cond)) {                                                            \
            fprintf(stderr, "  FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);     \
            ++failures;                                                           \
            return;                                                               \
        }                                                                         \
    } while (0)

static std::vector<uint8_t> random_bytes(size_t n, unsigned seed) {
    std::mt19937 g(seed);
    std::vector<uint8_t> v(n);
    for (auto &b : v) b = (uint8_t)g();
    return v;
}

// klauspost reedsolomon_test.go TestOneEncode: 5 data + 5 parity shards.
static void TestOneEncode() {
    rbc_rs *rs = nullptr;
    CHECK(rbc_rs_new(5, 5, 0, &rs) == RBC_OK);
    uint8_t buf[10][2] = {{0, 1}, {4, 5}, {2, 3}, {6, 7}, {8, 9}};
    uint8_t *sh[10];
    size_t lens[10];
    for (int i = 0; i < 10; ++i) { sh[i] = buf[i]; lens[i] = 2; }
    CHECK(rbc_rs_encode(rs, sh, lens, 10) == RBC_OK);
    const uint8_t want[5][2] = {{12, 13}, {10, 11}, {14, 15}, {90, 91}, {94, 95}};
    for (int i = 0; i < 5; ++i) CHECK(memcmp(buf[5 + i], want[i], 2) == 0);
    int ok = 0;
    CHECK(rbc_rs_verify(rs, sh, lens, 10, &ok) == RBC_OK && ok == 1);
    buf[8][0] ^= 1;
    CHECK(rbc_rs_verify(rs, sh, lens, 10, &ok) == RBC_OK && ok == 0);
    rbc_rs_free(rs);
}

// klauspost v1.9.1 Update: parity of the changed data equals a fresh Encode
// of the new data; the old data shard is left holding old ^ new (Go).
static void TestUpdate() {
    const int k = 10, p = 4, n = k + p;
    const size_t S = 513;
    rbc_rs *rs = nullptr;
    CHECK(rbc_rs_new(k, p, 0, &rs) == RBC_OK);
    std::vector<std::vector<uint8_t>> sh(n), fresh(n);
    for (int i = 0; i < n; ++i) sh[i] = i < k ? random_bytes(S, 100 + i) : std::vector<uint8_t>(S, 0);
    std::vector<uint8_t *> ptr(n);
    std::vector<size_t> lens(n, S);
    for (int i = 0; i < n; ++i) ptr[i] = sh[i].data();
    CHECK(rbc_rs_encode(rs, ptr.data(), lens.data(), n) == RBC_OK);
    std::vector<std::vector<uint8_t>> nd(k);
    std::vector<const uint8_t *> nptr(k, nullptr);
    std::vector<size_t> nlens(k, 0);
    for (int c : {2, 7}) {
        nd[c] = random_bytes(S, 900 + c);
        nptr[c] = nd[c].data();
        nlens[c] = S;
    }
    const auto old2 = sh[2];
    CHECK(rbc_rs_update(rs, ptr.data(), lens.data(), n, nptr.data(), nlens.data(), k) == RBC_OK);
    for (size_t x = 0; x < S; ++x) CHECK(sh[2][x] == (uint8_t)(old2[x] ^ nd[2][x]));
    std::vector<uint8_t *> fptr(n);
    for (int i = 0; i < n; ++i) {
        fresh[i] = i < k ? (nlens[i] ? nd[i] : sh[i]) : std::vector<uint8_t>(S, 0);
        fptr[i] = fresh[i].data();
    }
    CHECK(rbc_rs_encode(rs, fptr.data(), lens.data(), n) == RBC_OK);
    for (int r = k; r < n; ++r) CHECK(fresh[r] == sh[r]);
    lens[k] = 0;  // a nil parity shard
    CHECK(rbc_rs_update(rs, ptr.data(), lens.data(), n, nptr.data(), nlens.data(), k) == RBC_ERR_INVALID_INPUT);
    rbc_rs_free(rs);
}

// Reconstruct / ReconstructData restore exactly what Encode produced and never
// touch present shards; too few shards is ErrTooFewShards.
static void TestReconstruct() {
    const int k = 44, p = 84, n = k + p;
    const size_t S = 1001;
    rbc_rs *rs = nullptr;
    CHECK(rbc_rs_new(k, p, 0, &rs) == RBC_OK);
    std::vector<std::vector<uint8_t>> full(n, std::vector<uint8_t>(S));
    for (int i = 0; i < k; ++i) full[i] = random_bytes(S, 100 + i);
    std::vector<uint8_t *> sh(n);
    std::vector<size_t> lens(n, S);
    for (int i = 0; i < n; ++i) sh[i] = full[i].data();
    CHECK(rbc_rs_encode(rs, sh.data(), lens.data(), n) == RBC_OK);
    std::mt19937 g(7);
    std::vector<std::vector<uint8_t>> part = full;
    std::vector<int> idx(n);
    for (int i = 0; i < n; ++i) idx[i] = i;
    std::shuffle(idx.begin(), idx.end(), g);
    for (int t = 0; t < n - k; ++t) {  // erase n-k shards (data and parity)
        lens[idx[t]] = 0;
        memset(part[idx[t]].data(), 0xee, S);
    }
    for (int i = 0; i < n; ++i) sh[i] = part[i].data();
    CHECK(rbc_rs_reconstruct(rs, sh.data(), lens.data(), n) == RBC_OK);
    for (int i = 0; i < n; ++i) CHECK(lens[i] == S && part[i] == full[i]);
    lens.assign(n, S);
    lens[0] = lens[1] = 0;
    for (int t = 2; t < n - k + 1; ++t) lens[idx[t]] = 0;  // at most k-1 present
    int present = 0;
    for (size_t l : lens) present += l != 0;
    if (present < k) CHECK(rbc_rs_reconstruct(rs, sh.data(), lens.data(), n) == RBC_ERR_TOO_FEW_SHARDS);
    rbc_rs_free(rs);
}

struct Commit {
    std::vector<uint8_t> shards;  // n * S
    size_t S = 0;
    uint8_t root[32];
    std::vector<uint8_t> branches;  // n * d * 32 (device form)
};

static bool do_shard(rbc_ctx *ctx, int n, int d, const std::vector<uint8_t> &value, Commit &c) {
    int k = 0;
    rbc_ctx_params(ctx, &k, nullptr, nullptr);
    c.S = (value.size() + k - 1) / k;
    c.shards.assign((size_t)n * c.S, 0);
    c.branches.assign((size_t)n * (d ? d : 1) * 32, 0);
    size_t S = 0;
    const int rc = rbc_shard(ctx, value.data(), value.size(), c.shards.data(), c.shards.size(), &S, c.root,
                             c.branches.data());
    return rc == RBC_OK && S == c.S;
}

static std::string go_branch(const Commit &c, int n, int d, int j) {  // flat Go `Branch []byte`
    std::string b;
    for (int l = 0; l < d; ++l) {
        if (l == 0 && (j ^ 1) >= n) continue;
        b.append((const char *)c.branches.data() + ((size_t)j * d + l) * 32, 32);
    }
    return b;
}

// rbc/rbc_internal_test.go Test_shard: value -> N shards, systematic data
// shards, zero pad, Split/Join round trip, ErrShortData on empty input.
static void Test_shard() {
    const int n = 128, f = 42, k = n - 2 * f;
    rbc_ctx *ctx = nullptr;
    CHECK(rbc_ctx_create(n, f, 0, &ctx) == RBC_OK);
    int kk = 0, p = 0, d = 0;
    rbc_ctx_params(ctx, &kk, &p, &d);
    CHECK(kk == k && p == 2 * f && d == 7);
    const std::vector<uint8_t> value = random_bytes(1 << 20, 1);
    Commit c;
    CHECK(do_shard(ctx, n, d, value, c));
    CHECK(c.S == 23832);
    for (int j = 0; j < k; ++j) {  // systematic: shard j = value[j*S ..] (zero padded)
        const size_t off = (size_t)j * c.S;
        const size_t have = off < value.size() ? std::min(c.S, value.size() - off) : 0;
        CHECK(memcmp(c.shards.data() + off, value.data() + off, have) == 0);
        for (size_t b = have; b < c.S; ++b) CHECK(c.shards[off + b] == 0);
    }
    size_t S = 0;
    uint8_t root[32];
    std::vector<uint8_t> tmp(16);
    CHECK(rbc_shard(ctx, value.data(), 0, tmp.data(), tmp.size(), &S, root, nullptr) == RBC_ERR_SHORT_DATA);
    rbc_ctx_destroy(ctx);
}

// rbc/rbc_internal_test.go Test_validateMessage: every honest ECHO verifies;
// a flipped shard byte, a flipped branch byte, a wrong index and a truncated
// branch do not.  N = 7 covers the empty level-0 sibling.
static void Test_validateMessage() {
    for (int n : {7, 16, 128}) {
        const int f = (n - 1) / 3;
        rbc_ctx *ctx = nullptr;
        CHECK(rbc_ctx_create(n, f, 0, &ctx) == RBC_OK);
        int d = 0;
        rbc_ctx_params(ctx, nullptr, nullptr, &d);
        Commit c;
        CHECK(do_shard(ctx, n, d, random_bytes(5000 + n, n), c));
        for (int j = 0; j < n; ++j) {
            const std::string br = go_branch(c, n, d, j);
            int ok = 0;
            CHECK(rbc_validate_message(ctx, c.root, (const uint8_t *)br.data(), br.size(),
                                       c.shards.data() + (size_t)j * c.S, c.S, j, &ok) == RBC_OK && ok == 1);
        }
        std::vector<uint8_t> bad(c.shards.begin() + c.S * 2, c.shards.begin() + c.S * 3);
        bad[3] ^= 1;
        std::string br = go_branch(c, n, d, 2);
        int ok = 1;
        CHECK(rbc_validate_message(ctx, c.root, (const uint8_t *)br.data(), br.size(), bad.data(), c.S, 2, &ok) ==
                  RBC_OK && ok == 0);
        br[br.size() - 1] ^= 0x40;
        CHECK(rbc_validate_message(ctx, c.root, (const uint8_t *)br.data(), br.size(), c.shards.data() + 2 * c.S,
                                   c.S, 2, &ok) == RBC_OK && ok == 0);
        br = go_branch(c, n, d, 3);
        CHECK(rbc_validate_message(ctx, c.root, (const uint8_t *)br.data(), br.size(), c.shards.data() + 3 * c.S,
                                   c.S, 4, &ok) == RBC_OK && ok == 0);
        CHECK(rbc_validate_message(ctx, c.root, (const uint8_t *)br.data(), br.size() - 32,
                                   c.shards.data() + 3 * c.S, c.S, 3, &ok) == RBC_OK && ok == 0);
        rbc_ctx_destroy(ctx);
    }
}

// rbc/rbc_internal_test.go Test_interpolate: any N-2f shards give the value
// back; fewer is ErrTooFewShards (rbc/rbc.go:87); a wrong root or a tampered
// used shard is ROOT_MISMATCH.
static void Test_interpolate() {
    const int n = 64, f = 21, k = n - 2 * f;
    rbc_ctx *ctx = nullptr;
    CHECK(rbc_ctx_create(n, f, 0, &ctx) == RBC_OK);
    int d = 0;
    rbc_ctx_params(ctx, nullptr, nullptr, &d);
    const std::vector<uint8_t> value = random_bytes(100003, 9);
    Commit c;
    CHECK(do_shard(ctx, n, d, value, c));
    std::mt19937 g(3);
    for (int trial = 0; trial < 6; ++trial) {
        std::vector<int> idx(n);
        for (int i = 0; i < n; ++i) idx[i] = i;
        std::shuffle(idx.begin(), idx.end(), g);
        std::vector<const uint8_t *> sh(n, nullptr);
        std::vector<size_t> lens(n, 0);
        for (int t = 0; t < k; ++t) {
            sh[idx[t]] = c.shards.data() + (size_t)idx[t] * c.S;
            lens[idx[t]] = c.S;
        }
        std::vector<uint8_t> out((size_t)k * c.S), dig(32);
        size_t vlen = 0;
        CHECK(rbc_interpolate(ctx, c.root, sh.data(), lens.data(), out.data(), out.size(), &vlen, dig.data()) ==
              RBC_OK);
        CHECK(vlen == (size_t)k * c.S && memcmp(out.data(), value.data(), value.size()) == 0);
        for (size_t b = value.size(); b < vlen; ++b) CHECK(out[b] == 0);
        uint8_t wrong[32];
        memcpy(wrong, c.root, 32);
        wrong[0] ^= 1;
        CHECK(rbc_interpolate(ctx, wrong, sh.data(), lens.data(), out.data(), out.size(), &vlen, nullptr) ==
              RBC_ERR_ROOT_MISMATCH);
        std::vector<uint8_t> tampered(c.shards.begin() + (size_t)idx[0] * c.S,
                                      c.shards.begin() + (size_t)(idx[0] + 1) * c.S);
        tampered[0] ^= 0x5a;
        sh[idx[0]] = tampered.data();
        CHECK(rbc_interpolate(ctx, c.root, sh.data(), lens.data(), out.data(), out.size(), &vlen, nullptr) ==
              RBC_ERR_ROOT_MISMATCH);
        lens[idx[0]] = 0;
        sh[idx[0]] = nullptr;
        CHECK(rbc_interpolate(ctx, c.root, sh.data(), lens.data(), out.data(), out.size(), &vlen, nullptr) ==
              RBC_ERR_TOO_FEW_SHARDS);
    }
    rbc_ctx_destroy(ctx);
}

// The batcher from many threads: every request completes with its own
// result, and requests are coalesced.
static void TestBatcherConcurrent() {
    const int n = 16, f = 5;
    rbc_ctx *ctx = nullptr;
    CHECK(rbc_ctx_create(n, f, 0, &ctx) == RBC_OK);
    rbc_batcher *b = nullptr;
    CHECK(rbc_batcher_create(ctx, 32, 3000, &b) == RBC_OK);
    const int T = 64;
    std::vector<int> bad(T, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            const std::vector<uint8_t> v = random_bytes(1000 + 37 * t, 500 + t);
            const size_t S = (v.size() + 5) / 6;
            std::vector<uint8_t> sh(n * S), root(32), br(n * 4 * 32);
            size_t slen = 0;
            uint64_t tk = 0;
            if (rbc_batcher_shard(b, v.data(), v.size(), sh.data(), sh.size(), &slen, root.data(), br.data(), &tk) ||
                rbc_batcher_wait(b, tk) != RBC_OK || slen != S) { bad[t] = 1; return; }
            std::vector<const uint8_t *> p(n, nullptr);
            std::vector<size_t> l(n, 0);
            for (int j = n - 6; j < n; ++j) { p[j] = sh.data() + j * S; l[j] = S; }  // parity only
            std::vector<uint8_t> out(6 * S);
            size_t vl = 0;
            if (rbc_batcher_interpolate(b, root.data(), p.data(), l.data(), out.data(), out.size(), &vl, nullptr,
                                        &tk) ||
                rbc_batcher_wait(b, tk) != RBC_OK || memcmp(out.data(), v.data(), v.size()) != 0)
                bad[t] = 2;
        });
    for (auto &x : th) x.join();
    for (int t = 0; t < T; ++t) CHECK(bad[t] == 0);
    uint64_t batches = 0, reqs = 0;
    rbc_batcher_stats(b, &batches, &reqs);
    CHECK(reqs == 2 * (uint64_t)T && batches < reqs);
    rbc_batcher_destroy(b);
    rbc_ctx_destroy(ctx);
}

// rbc_dev_receive_step from a pure C-ABI client: three batches through the
// pipelined receiver (verify(t) + regen hashing of t-1 in one launch) give
// the same valid masks, statuses, values and digests as rbc_dev_verify +
// rbc_dev_interpolate on identical inputs; a wrong `prev` is rejected.
static void TestReceiveStep() {
    const int n = 16, f = 5, I = 20, nb = 3;
    const uint32_t B = 3001;
    rbc_ctx *ctx = nullptr;
    CHECK(rbc_ctx_create(n, f, 0, &ctx) == RBC_OK);
    int k = 0, p = 0, d = 0;
    CHECK(rbc_ctx_params(ctx, &k, &p, &d) == RBC_OK);
    const uint32_t S = (B + k - 1) / k, spitch = (S + 63) / 64 * 64;
    const uint64_t vpitch = ((uint64_t)k * S + 32 + 63) / 64 * 64;
    const uint32_t opitch = (k * S + 15) / 16 * 16;
    std::vector<uint8_t> present((size_t)I * n, 0);
    std::vector<int32_t> corrupt(I, -1);
    std::mt19937 g(77);
    for (int i = 0; i < I; ++i) {
        std::vector<int> idx(n);
        for (int j = 0; j < n; ++j) idx[j] = j;
        std::shuffle(idx.begin(), idx.end(), g);
        for (int j = 0; j < n - f; ++j) present[(size_t)i * n + idx[j]] = 1;
        if (i % 3 == 0) corrupt[i] = idx[0];
    }
    auto dmalloc = [](size_t bytes) {
        void *q = nullptr;
        return rbc_dev_malloc(0, bytes, &q) == RBC_OK ? (uint8_t *)q : nullptr;
    };
    uint8_t *d_present = dmalloc(present.size());
    int32_t *d_corrupt = (int32_t *)dmalloc(I * 4);
    CHECK(d_present && d_corrupt);
    CHECK(rbc_memcpy_h2d(d_present, present.data(), present.size()) == RBC_OK);
    CHECK(rbc_memcpy_h2d(d_corrupt, corrupt.data(), I * 4) == RBC_OK);
    struct Bufs {
        uint8_t *values, *shards, *leaves, *roots, *branches, *valid, *leaves_r, *out, *digests;
        int32_t *status;
    };
    // [mode][batch]: mode 0 = verify + interpolate, mode 1 = receive step
    Bufs b[2][nb];
    for (int m = 0; m < 2; ++m)
        for (int t = 0; t < nb; ++t) {
            Bufs &x = b[m][t];
            x.values = dmalloc(I * vpitch);
            x.shards = dmalloc((size_t)I * n * spitch);
            x.leaves = dmalloc((size_t)I * n * 32);
            x.roots = dmalloc(I * 32);
            x.branches = dmalloc((size_t)I * n * d * 32);
            x.valid = dmalloc((size_t)I * n);
            x.leaves_r = dmalloc((size_t)I * n * 32);
            x.out = dmalloc((size_t)I * opitch);
            x.digests = dmalloc(I * 32);
            x.status = (int32_t *)dmalloc(I * 4);
            CHECK(x.values && x.shards && x.leaves && x.roots && x.branches && x.valid && x.leaves_r && x.out &&
                  x.digests && x.status);
            const std::vector<uint8_t> v = random_bytes(I * vpitch, 900 + t);
            CHECK(rbc_memcpy_h2d(x.values, v.data(), v.size()) == RBC_OK);
            CHECK(rbc_dev_encode(ctx, nullptr, I, x.values, vpitch, nullptr, B, x.shards, spitch) == RBC_OK);
            CHECK(rbc_dev_leaves(ctx, nullptr, I, x.shards, spitch, nullptr, S, x.leaves) == RBC_OK);
            CHECK(rbc_dev_merkle_build(ctx, nullptr, I, x.leaves, x.roots, x.branches) == RBC_OK);
            CHECK(rbc_dev_inject_faults(ctx, nullptr, I, x.shards, spitch, d_corrupt) == RBC_OK);
        }
    for (int t = 0; t < nb; ++t) {
        Bufs &x = b[0][t];
        CHECK(rbc_dev_verify(ctx, nullptr, I, x.shards, spitch, nullptr, S, x.branches, x.roots, d_present, x.valid,
                             x.leaves_r) == RBC_OK);
        CHECK(rbc_dev_interpolate(ctx, nullptr, I, x.shards, spitch, nullptr, S, x.valid, x.leaves_r, 1, x.roots,
                                  x.out, opitch, x.digests, x.status) == RBC_OK);
    }
    rbc_rx_batch rb[nb];
    for (int t = 0; t < nb; ++t) {
        Bufs &x = b[1][t];
        rb[t] = rbc_rx_batch{I, x.shards, spitch, nullptr, S, x.branches, x.roots, d_present, x.valid, x.leaves_r,
                             x.out, opitch, x.digests, x.status};
    }
    CHECK(rbc_dev_receive_step(ctx, nullptr, &rb[0], nullptr, nullptr) == RBC_OK);
    CHECK(rbc_dev_receive_step(ctx, nullptr, &rb[1], &rb[2], nullptr) == RBC_ERR_INVALID_ARG);  // not the last cur
    for (int t = 1; t < nb; ++t) CHECK(rbc_dev_receive_step(ctx, nullptr, &rb[t], &rb[t - 1], nullptr) == RBC_OK);
    CHECK(rbc_dev_receive_step(ctx, nullptr, nullptr, &rb[nb - 1], nullptr) == RBC_OK);
    CHECK(rbc_device_sync(0) == RBC_OK);
    for (int t = 0; t < nb; ++t) {
        std::vector<int32_t> s0(I), s1(I);
        std::vector<uint8_t> v0((size_t)I * n), v1((size_t)I * n), o0((size_t)I * opitch), o1((size_t)I * opitch),
            g0(I * 32), g1(I * 32);
        CHECK(rbc_memcpy_d2h(s0.data(), b[0][t].status, I * 4) == RBC_OK);
        CHECK(rbc_memcpy_d2h(s1.data(), b[1][t].status, I * 4) == RBC_OK);
        CHECK(rbc_memcpy_d2h(v0.data(), b[0][t].valid, v0.size()) == RBC_OK);
        CHECK(rbc_memcpy_d2h(v1.data(), b[1][t].valid, v1.size()) == RBC_OK);
        CHECK(rbc_memcpy_d2h(o0.data(), b[0][t].out, o0.size()) == RBC_OK);
        CHECK(rbc_memcpy_d2h(o1.data(), b[1][t].out, o1.size()) == RBC_OK);
        CHECK(rbc_memcpy_d2h(g0.data(), b[0][t].digests, g0.size()) == RBC_OK);
        CHECK(rbc_memcpy_d2h(g1.data(), b[1][t].digests, g1.size()) == RBC_OK);
        const std::vector<uint8_t> v = random_bytes(I * vpitch, 900 + t);
        for (int i = 0; i < I; ++i) {
            CHECK(s0[i] == RBC_OK && s1[i] == RBC_OK);
            for (int j = 0; j < n; ++j)
                CHECK(v0[(size_t)i * n + j] == v1[(size_t)i * n + j]);
            CHECK(memcmp(o0.data() + (size_t)i * opitch, o1.data() + (size_t)i * opitch, k * S) == 0);
            CHECK(memcmp(o1.data() + (size_t)i * opitch, v.data() + (size_t)i * vpitch, B) == 0);
            CHECK(memcmp(g0.data() + i * 32, g1.data() + i * 32, 32) == 0);
        }
    }
    for (int m = 0; m < 2; ++m)
        for (int t = 0; t < nb; ++t) {
            Bufs &x = b[m][t];
            for (void *q : {(void *)x.values, (void *)x.shards, (void *)x.leaves, (void *)x.roots, (void *)x.branches,
                            (void *)x.valid, (void *)x.leaves_r, (void *)x.out, (void *)x.digests, (void *)x.status})
                rbc_dev_free(q);
        }
    rbc_dev_free(d_present);
    rbc_dev_free(d_corrupt);
    rbc_ctx_destroy(ctx);
}

int main() {
    int ndev = 0;
    rbc_device_count(&ndev);
    if (ndev < 1) {
        fprintf(stderr, "no GPU visible\n");
        return 2;
    }
    struct { const char *name; void (*fn)(); } tests[] = {
        {"TestOneEncode", TestOneEncode},   {"TestReconstruct", TestReconstruct},
        {"Test_shard", Test_shard},         {"Test_validateMessage", Test_validateMessage},
        {"Test_interpolate", Test_interpolate}, {"TestBatcherConcurrent", TestBatcherConcurrent},
        {"TestUpdate", TestUpdate},         {"TestReceiveStep", TestReceiveStep},
    };
    for (auto &t : tests) {
        const int before = failures;
        t.fn();
        printf("--- %s: %s\n", failures == before ? "PASS" : "FAIL", t.name);
    }
    printf(failures ? "FAIL\n" : "ok\n");
    return failures ? 1 : 0;
}
