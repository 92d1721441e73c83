// batcher_bench.cpp -- throughput of the request coalescer (rbc_batcher) that
// a Go host drives one RBC message at a time over cgo: T client threads
// submit shard / validateMessage / interpolate requests at the C2 geometry
// (N=128, f=42, 1 MiB values) and wait for them; one JSON line per phase.
//   build: make -C tools batcher_bench
//   run:   tools/batcher_bench [values] [threads] [window] [max_batch] [validate_max_batch] [max_wait_us]
//          tools/batcher_bench validate-sweep [values] [threads] [max_wait_us] [outstanding ...]
// Each phase runs twice on one batcher; the second (warm: pinned pools and
// device buffers already grown) is reported.
// validate-sweep: validateMessage alone at several levels of requests
// outstanding (a sliding window per client thread: a client waits for its
// oldest request once `outstanding / threads` are in flight, as the per-
// instance goroutines of a node each wait on their own ECHO), e.g. 88,064 =
// one C2 epoch (1,024 instances x 86 received ECHOs).  1 % of the messages
// carry a wrong root; every verdict is checked.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <deque>
#include <chrono>
#include <thread>
#include <vector>

#include "../include/rbc_gpu.h"

#define CK(x)                                                             \
    do {                                                                  \
        int rc_ = (x);                                                    \
        if (rc_) {                                                        \
            fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, rc_); \
            exit(1);                                                      \
        }                                                                 \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int validate_sweep(int argc, char **argv);
int epoch(int argc, char **argv);

int main(int argc, char **argv) {
    if (argc > 1 && !strcmp(argv[1], "validate-sweep")) return validate_sweep(argc - 1, argv + 1);
    if (argc > 1 && !strcmp(argv[1], "epoch")) return epoch(argc - 1, argv + 1);
    const int n = 128, f = 42, k = n - 2 * f, d = 7;
    const size_t B = 1 << 20, S = (B + k - 1) / k;
    const int I = argc > 1 ? atoi(argv[1]) : 256;        // values
    const int T = argc > 2 ? atoi(argv[2]) : 16;         // client threads
    const int WIN = argc > 3 ? atoi(argv[3]) : 64;       // requests a client keeps outstanding
    const int MB = argc > 4 ? atoi(argv[4]) : 64;        // max_batch for shard / interpolate
    const int VB = argc > 5 ? atoi(argv[5]) : 2048;      // max_batch for validate
    const int WAIT = argc > 6 ? atoi(argv[6]) : 200;     // max_wait_us
    rbc_ctx *ctx;
    CK(rbc_ctx_create(n, f, 0, &ctx));
    std::vector<uint8_t> values((size_t)I * B);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto &v : values) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        v = (uint8_t)x;
    }
    std::vector<uint8_t> shards((size_t)I * n * S), roots((size_t)I * 32), br((size_t)I * n * d * 32);
    std::vector<size_t> slen(I);

    auto run = [&](const char *name, int max_batch, int total, auto &&submit, double bytes) {
        rbc_batcher *b;
        CK(rbc_batcher_create(ctx, max_batch, WAIT, &b));
        std::atomic<int> next{0}, bad{0};
        double t0 = 0;
        for (int pass = 0; pass < 2; ++pass) {
        next = 0;
        bad = 0;
        t0 = now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&] {
                std::vector<uint64_t> tickets;
                std::vector<int> idx;
                for (int i; (i = next.fetch_add(1)) < total;) {
                    tickets.push_back(submit(b, i));
                    idx.push_back(i);
                    if ((int)tickets.size() >= WIN) {  // a client keeps a window of requests outstanding
                        for (uint64_t tk : tickets) bad += rbc_batcher_wait(b, tk) != RBC_OK;
                        tickets.clear();
                    }
                }
                for (uint64_t tk : tickets) bad += rbc_batcher_wait(b, tk) != RBC_OK;
            });
        for (auto &t : th) t.join();
        }
        const double dt = now() - t0;
        uint64_t nb = 0, nr = 0;
        rbc_batcher_stats(b, &nb, &nr);
        rbc_batcher_destroy(b);
        printf("{\"phase\": \"%s\", \"requests\": %d, \"threads\": %d, \"window\": %d, \"max_batch\": %d, "
               "\"max_wait_us\": %d, \"seconds\": %.4f, \"req_per_s\": %.0f, \"GBps\": %.2f, "
               "\"requests_per_launch\": %.1f, \"failed\": %d}\n",
               name, total, T, WIN, max_batch, WAIT, dt, total / dt, bytes / dt / 1e9, nb ? (double)nr / nb : 0.0,
               bad.load());
        fflush(stdout);
        return bad.load();
    };

    // shard + commit: one request per 1 MiB value (output N*S bytes)
    int fails = run("shard", MB, I, [&](rbc_batcher *b, int i) {
        uint64_t t;
        CK(rbc_batcher_shard(b, values.data() + (size_t)i * B, B, shards.data() + (size_t)i * n * S, n * S, &slen[i],
                             roots.data() + (size_t)i * 32, br.data() + (size_t)i * n * d * 32, &t));
        return t;
    }, (double)I * n * S);
    // validateMessage: one request per (value, received shard) -- N = 128 is a
    // power of two, so the device branch form [d][32] is also the Go flat form
    const int V = I * (n - f);
    std::vector<int> ok(V);
    fails += run("validate", VB, V, [&](rbc_batcher *b, int e) {
        const int i = e / (n - f), j = e % (n - f);
        uint64_t t;
        CK(rbc_batcher_validate(b, roots.data() + (size_t)i * 32, br.data() + ((size_t)i * n + j) * d * 32, d * 32,
                                shards.data() + ((size_t)i * n + j) * S, S, (uint32_t)j, &ok[e], &t));
        return t;
    }, (double)V * S);
    for (int e = 0; e < V; ++e) fails += ok[e] != 1;
    // interpolate from the first N-f shards of each value
    std::vector<const uint8_t *> ptrs((size_t)I * n);
    std::vector<size_t> lens((size_t)I * n);
    std::vector<uint8_t> out((size_t)I * k * S);
    std::vector<size_t> olen(I);
    for (int i = 0; i < I; ++i)
        for (int j = 0; j < n; ++j) {
            ptrs[(size_t)i * n + j] = j < n - f ? shards.data() + ((size_t)i * n + j) * S : nullptr;
            lens[(size_t)i * n + j] = j < n - f ? S : 0;
        }
    fails += run("interpolate", MB, I, [&](rbc_batcher *b, int i) {
        uint64_t t;
        CK(rbc_batcher_interpolate(b, roots.data() + (size_t)i * 32, ptrs.data() + (size_t)i * n,
                                   lens.data() + (size_t)i * n, out.data() + (size_t)i * k * S, k * S, &olen[i],
                                   nullptr, &t));
        return t;
    }, (double)I * n * S);
    for (int i = 0; i < I; ++i) fails += memcmp(out.data() + (size_t)i * k * S, values.data() + (size_t)i * B, B) != 0;
    rbc_ctx_destroy(ctx);
    printf("{\"phase\": \"check\", \"failures\": %d}\n", fails);
    return fails ? 1 : 0;
}

int validate_sweep(int argc, char **argv) {
    const int n = 128, f = 42, d = 7, k = n - 2 * f;
    const size_t B = 1 << 20, S = (B + k - 1) / k;
    const int I = argc > 1 ? atoi(argv[1]) : 256;    // committed values the messages come from
    const int T = argc > 2 ? atoi(argv[2]) : 16;     // client threads
    const int WAIT = argc > 3 ? atoi(argv[3]) : 200;  // max_wait_us
    std::vector<int> levels;
    for (int a = 4; a < argc; ++a) levels.push_back(atoi(argv[a]));
    if (levels.empty()) levels = {1024, 8192, 32768, 88064};
    rbc_ctx *ctx;
    CK(rbc_ctx_create(n, f, 0, &ctx));
    std::vector<uint8_t> values((size_t)I * B);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto &v : values) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        v = (uint8_t)x;
    }
    // the committed set: shards (host memory, like the Go handlers' message buffers), branches, roots
    std::vector<uint8_t> shards((size_t)I * n * S), roots((size_t)I * 32), br((size_t)I * n * d * 32);
    std::vector<uint32_t> slens(I);
    std::vector<const uint8_t *> vp(I);
    std::vector<size_t> vl(I, B);
    for (int i = 0; i < I; ++i) vp[i] = values.data() + (size_t)i * B;
    for (int i0 = 0; i0 < I; i0 += 64) {
        const int c = std::min(64, I - i0);
        CK(rbc_shard_commit(ctx, c, vp.data() + i0, vl.data() + i0, shards.data() + (size_t)i0 * n * S, S,
                            slens.data() + i0, roots.data() + (size_t)i0 * 32, br.data() + (size_t)i0 * n * d * 32,
                            nullptr));
    }
    std::vector<uint8_t> bad_roots = roots;
    for (int i = 0; i < I; ++i) bad_roots[(size_t)i * 32 + 5] ^= 0x40;
    const char *amb = getenv("RBC_BB_ARENA_MB");  // validate-lane arena size (A/B of the tool only)
    const size_t arena_bytes = amb ? (size_t)atoi(amb) << 20 : (size_t)256 << 20;
    {  // the host-side ceiling: T threads copying the same messages into pinned memory, no batcher
        void *pin = nullptr;
        CK(rbc_host_alloc(arena_bytes, &pin));
        const int M = 262144;
        for (int pass = 0; pass < 2; ++pass) {
            std::atomic<int> next{0};
            const double t0 = now();
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t)
                th.emplace_back([&] {
                    for (int e; (e = next.fetch_add(1)) < M;) {
                        const int i = (e / (n - f)) % I, j = e % (n - f);
                        const size_t off = ((size_t)e * 23872) % (arena_bytes - 2 * S) / 64 * 64;
                        memcpy((uint8_t *)pin + off, shards.data() + ((size_t)i * n + j) * S, S);
                    }
                });
            for (auto &t : th) t.join();
            const double dt = now() - t0;
            if (pass)
                printf("{\"phase\": \"copy_ceiling\", \"threads\": %d, \"messages\": %d, \"GBps\": %.3f}\n", T, M,
                       (double)M * S / dt / 1e9);
        }
        rbc_host_free(pin);
    }
    int fails = 0;
    for (const int L : levels) {
        const int W = std::max(1, L / T);
        // messages per pass: six windows' worth, so the fill and the final drain of the window
        // (the first L submissions see no completion) are a small part of the timed pass
        const int M = std::max(6 * L, 262144);
        std::vector<int> ok(M);
        rbc_batcher *b;
        CK(rbc_batcher_create(ctx, 256, WAIT, &b));
        CK(rbc_batcher_set_validate(b, 65536, arena_bytes));
        double dt = 0;
        uint64_t nb0 = 0, nr0 = 0, nb = 0, nr = 0;
        std::atomic<int> bad{0};
        std::atomic<long> ns_submit{0}, ns_wait{0};  // client time inside validate / wait (second pass)
        for (int pass = 0; pass < 2; ++pass) {  // the second pass (arenas allocated, device buffers grown) counts
            ns_submit = 0;
            ns_wait = 0;
            std::atomic<int> next{0};
            bad = 0;
            rbc_batcher_stats(b, &nb0, &nr0);
            const double t0 = now();
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t)
                th.emplace_back([&] {
                    std::vector<std::pair<uint64_t, int>> win;  // (ticket, message) oldest first
                    size_t head = 0;
                    long my_sub = 0, my_wait = 0;
                    auto drain_one = [&] {
                        const auto [tk, e] = win[head++];
                        const auto w0 = std::chrono::steady_clock::now();
                        if (rbc_batcher_wait(b, tk) != RBC_OK) ++bad;
                        my_wait += std::chrono::duration_cast<std::chrono::nanoseconds>(
                                       std::chrono::steady_clock::now() - w0).count();
                        const int want = (e % 97) != 13;
                        if (ok[e] != want) ++bad;
                    };
                    for (int e; (e = next.fetch_add(1)) < M;) {
                        // message e: received shard j < n - f of value i
                        const int i = (e / (n - f)) % I, j = e % (n - f);
                        const uint8_t *rt = ((e % 97) == 13 ? bad_roots.data() : roots.data()) + (size_t)i * 32;
                        uint64_t tk;
                        const auto s0 = std::chrono::steady_clock::now();
                        CK(rbc_batcher_validate(b, rt, br.data() + ((size_t)i * n + j) * d * 32, d * 32,
                                                shards.data() + ((size_t)i * n + j) * S, S, (uint32_t)j, &ok[e], &tk));
                        my_sub += std::chrono::duration_cast<std::chrono::nanoseconds>(
                                      std::chrono::steady_clock::now() - s0).count();
                        win.emplace_back(tk, e);
                        if ((int)(win.size() - head) >= W) drain_one();
                    }
                    while (head < win.size()) drain_one();
                    ns_submit += my_sub;
                    ns_wait += my_wait;
                });
            for (auto &t : th) t.join();
            dt = now() - t0;
            rbc_batcher_stats(b, &nb, &nr);
        }
        rbc_batcher_destroy(b);
        const double launches = (double)(nb - nb0);
        printf("{\"phase\": \"validate\", \"outstanding\": %d, \"threads\": %d, \"window\": %d, \"messages\": %d, "
               "\"shard_bytes\": %zu, \"max_wait_us\": %d, \"seconds\": %.4f, \"msg_per_s\": %.0f, \"GBps\": %.3f, "
               "\"launches\": %.0f, \"msgs_per_launch\": %.1f, \"failed\": %d, \"client_us_per_msg\": "
               "{\"submit\": %.2f, \"wait\": %.2f}}\n",
               L, T, W, M, S, WAIT, dt, M / dt, (double)M * S / dt / 1e9, launches,
               launches ? (double)(nr - nr0) / launches : 0.0, bad.load(), ns_submit.load() / 1e3 / M,
               ns_wait.load() / 1e3 / M);
        fflush(stdout);
        fails += bad.load();
    }
    rbc_ctx_destroy(ctx);
    printf("{\"phase\": \"check\", \"failures\": %d}\n", fails);
    return fails ? 1 : 0;
}

// epoch: one node's whole C2 epoch through the batcher, the way the unchanged
// Go handlers drive the drop-in (rbc/rbc.go:78, one goroutine per RBC
// instance): per instance, shard() of the node's own proposal, validateMessage
// of the N-f ECHOs it receives (10 % of the instances carry one corrupted
// ECHO), then interpolate() of the ECHOs that validated.  T client threads,
// each with W instances in flight, so thousands of requests of all three kinds
// are outstanding together.  Passes: a warm-up, then the epoch timed with the
// leaves reused (rbc_batcher_validate_leaf + rbc_batcher_interpolate_verified:
// interpolate hashes only the regenerated rows), then timed again with the
// plain calls (interpolate rehashes all N rows).  Every verdict, value, shard
// row and root is checked; the two timed passes must agree bit for bit
// (values, digests); `dump` receives sampled (value, root, digest) records for
// the oracle check in tests/test_gpu_batcher.py.
// `kinds` (default svi) drops request kinds for a breakdown: s = shard, v =
// validate, i = interpolate (with v: of the ECHOs that validated).
// With keep_mib > 0 (default 8 GiB) a fourth timed pass (after its own warm-up)
// runs the same plain calls through a batcher with rbc_batcher_set_keep: the
// validated rows stay on the device and interpolate reads them there.
//   tools/batcher_bench epoch [instances] [threads] [window] [max_wait_us] [dump|-] [kinds] [keep_mib]
int epoch(int argc, char **argv) {
    const int n = 128, f = 42, k = n - 2 * f, d = 7, R = n - f;
    const size_t B = 1 << 20, S = (B + k - 1) / k;
    const int I = argc > 1 ? atoi(argv[1]) : 1024;
    const int T = argc > 2 ? atoi(argv[2]) : 16;
    const int W = argc > 3 ? atoi(argv[3]) : 8;
    const int WAIT = argc > 4 ? atoi(argv[4]) : 200;
    const char *dump = argc > 5 && strcmp(argv[5], "-") ? argv[5] : nullptr;
    const char *kinds = argc > 6 ? argv[6] : "svi";
    const size_t keep_mib = argc > 7 ? (size_t)atol(argv[7]) : 8192;  // the kept passes' device ring (0: none): three epochs
    const bool ks = strchr(kinds, 's') != nullptr, kv = strchr(kinds, 'v') != nullptr,
               ki = strchr(kinds, 'i') != nullptr;
    rbc_ctx *ctx;
    CK(rbc_ctx_create(n, f, 0, &ctx));
    std::vector<uint8_t> values((size_t)I * B);
    uint64_t x = 0x2545F4914F6CDD1Dull;
    for (size_t w = 0; w < values.size() / 8; ++w) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        memcpy(values.data() + 8 * w, &x, 8);
    }
    // the ECHOs this node receives: every instance's committed rows (committed here, before timing)
    std::vector<uint8_t> shards_c((size_t)I * n * S), roots_c((size_t)I * 32), br_c((size_t)I * n * d * 32);
    {
        std::vector<uint32_t> sl(I);
        std::vector<const uint8_t *> vp(I);
        std::vector<size_t> vl(I, B);
        for (int i = 0; i < I; ++i) vp[i] = values.data() + (size_t)i * B;
        for (int i0 = 0; i0 < I; i0 += 64) {
            const int c = std::min(64, I - i0);
            CK(rbc_shard_commit(ctx, c, vp.data() + i0, vl.data() + i0, shards_c.data() + (size_t)i0 * n * S, S,
                                sl.data() + i0, roots_c.data() + (size_t)i0 * 32, br_c.data() + (size_t)i0 * n * d * 32,
                                nullptr));
        }
    }
    // received positions (N-f of N) and the corrupted ECHO of 10 % of the instances
    std::vector<int> recv((size_t)I * R), bad(I, -1);
    std::vector<std::vector<uint8_t>> badrow(I);
    uint64_t y = 0x9E3779B97F4A7C15ull;
    auto rnd = [&](uint64_t m) { y ^= y << 13; y ^= y >> 7; y ^= y << 17; return y % m; };
    for (int i = 0; i < I; ++i) {
        std::vector<int> perm(n);
        for (int j = 0; j < n; ++j) perm[j] = j;
        for (int j = n - 1; j > 0; --j) std::swap(perm[j], perm[rnd(j + 1)]);
        std::copy(perm.begin(), perm.begin() + R, recv.begin() + (size_t)i * R);
        if (rnd(10) == 0) {
            bad[i] = perm[rnd(R)];
            badrow[i].assign(shards_c.begin() + ((size_t)i * n + bad[i]) * S,
                             shards_c.begin() + ((size_t)i * n + bad[i] + 1) * S);
            badrow[i][S / 2] ^= 0x5A;
        }
    }
    auto echo = [&](int i, int j) -> const uint8_t * {
        return j == bad[i] ? badrow[i].data() : shards_c.data() + ((size_t)i * n + j) * S;
    };
    std::vector<uint8_t> sh_out((size_t)I * n * S), root_out((size_t)I * 32), br_out((size_t)I * n * d * 32);
    std::vector<size_t> slen(I);
    std::vector<int> ok((size_t)I * R);
    std::vector<uint8_t> leaf((size_t)I * n * 32);
    const bool kept = ki && kv && keep_mib > 0;
    const bool only_kept = kept && strchr(kinds, 'K') != nullptr;  // kinds "sviK": the kept passes alone
    std::vector<uint8_t> vout[3], dig[3];
    for (int o = 0; o < 3; ++o) {
        vout[o].resize(o < 2 || kept ? (size_t)I * k * S : 0);
        dig[o].resize((size_t)I * 32);
    }
    std::vector<size_t> vlen(I);
    int fails = 0;
    double secs[3] = {0, 0, 0};
    uint64_t launches[3] = {0, 0, 0}, reqs[3] = {0, 0, 0};
    // One pass of the epoch through batcher b; pass 0 is a warm-up (not reported: the batcher's pinned
    // arenas and launch buffers are allocated there), `o` the output set
    auto run_pass = [&](rbc_batcher *b, int pass, bool verified, int o, const char *label) {
        uint64_t nb0 = 0, nr0 = 0;
        rbc_batcher_stats(b, &nb0, &nr0);
        std::atomic<int> next{0}, bad_count{0};
        std::fill(ok.begin(), ok.end(), -1);
        const double t0 = now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&] {
                struct Inst { int i; uint64_t ts, ti; std::vector<uint64_t> tv; };
                std::deque<Inst> va, ip;  // validates pending / interpolate pending
                auto finish_validate = [&](Inst &s) {
                    std::vector<const uint8_t *> ptr(n, nullptr);
                    std::vector<size_t> len(n, 0);
                    for (int m = 0; m < R; ++m) {
                        const int j = recv[(size_t)s.i * R + m];
                        int v = j != bad[s.i];  // without validates: the rows a validate would pass
                        if (kv) {
                            if (rbc_batcher_wait(b, s.tv[m]) != RBC_OK) ++bad_count;
                            if (ok[(size_t)s.i * R + m] != v) ++bad_count;
                            v = ok[(size_t)s.i * R + m];
                        }
                        if (v == 1) { ptr[j] = echo(s.i, j); len[j] = S; }
                    }
                    const size_t i = s.i;
                    if (!ki) return;
                    if (verified)
                        CK(rbc_batcher_interpolate_verified(b, roots_c.data() + i * 32, ptr.data(), len.data(),
                                                            leaf.data() + i * n * 32, vout[o].data() + i * k * S,
                                                            k * S, &vlen[i], dig[o].data() + i * 32, &s.ti));
                    else
                        CK(rbc_batcher_interpolate(b, roots_c.data() + i * 32, ptr.data(), len.data(),
                                                   vout[o].data() + i * k * S, k * S, &vlen[i], dig[o].data() + i * 32,
                                                   &s.ti));
                };
                auto finish_interp = [&](Inst &s) {
                    if (ki && rbc_batcher_wait(b, s.ti) != RBC_OK) ++bad_count;
                    if (ks && rbc_batcher_wait(b, s.ts) != RBC_OK) ++bad_count;
                };
                for (;;) {
                    int i = -1;
                    if ((int)va.size() < W && (i = next.fetch_add(1)) < I) {
                        Inst s{i, 0, 0, std::vector<uint64_t>(R)};
                        if (ks)
                            CK(rbc_batcher_shard(b, values.data() + (size_t)i * B, B,
                                                 sh_out.data() + (size_t)i * n * S, n * S, &slen[i],
                                                 root_out.data() + (size_t)i * 32,
                                                 br_out.data() + (size_t)i * n * d * 32, &s.ts));
                        for (int m = 0; m < R && kv; ++m) {
                            const int j = recv[(size_t)i * R + m];
                            CK(rbc_batcher_validate_leaf(b, roots_c.data() + (size_t)i * 32,
                                                         br_c.data() + ((size_t)i * n + j) * d * 32, d * 32, echo(i, j),
                                                         S, (uint32_t)j, &ok[(size_t)i * R + m],
                                                         verified ? leaf.data() + ((size_t)i * n + j) * 32 : nullptr,
                                                         &s.tv[m]));
                        }
                        va.push_back(std::move(s));
                        continue;
                    }
                    if (!va.empty()) {  // the oldest instance's ECHOs are all validated: interpolate it
                        finish_validate(va.front());
                        ip.push_back(std::move(va.front()));
                        va.pop_front();
                        if ((int)ip.size() >= W) { finish_interp(ip.front()); ip.pop_front(); }
                        continue;
                    }
                    while (!ip.empty()) { finish_interp(ip.front()); ip.pop_front(); }
                    break;
                }
            });
        for (auto &t : th) t.join();
        const double dt = now() - t0;
        rbc_batcher_stats(b, &launches[o], &reqs[o]);
        launches[o] -= nb0;
        reqs[o] -= nr0;
        fails += bad_count.load();
        if (pass == 0) return;
        secs[o] = dt;
        // checks: every value, every proposer shard row / root (the verdicts were checked by the clients)
        int vbad = 0, sbad = 0;
        for (int i = 0; i < I; ++i) {
            if (ki)
                vbad += vlen[i] != k * S ||
                        memcmp(vout[o].data() + (size_t)i * k * S, values.data() + (size_t)i * B, B) != 0;
            if (ks)
                sbad += slen[i] != S || memcmp(root_out.data() + (size_t)i * 32, roots_c.data() + (size_t)i * 32, 32) != 0 ||
                        memcmp(sh_out.data() + (size_t)i * n * S, shards_c.data() + (size_t)i * n * S, n * S) != 0;
        }
        fails += vbad + sbad;
        printf("{\"phase\": \"epoch\", \"kinds\": \"%s\", \"interpolate\": \"%s\", \"instances\": %d, \"threads\": %d, \"window\": %d, "
               "\"echo_messages\": %d, \"max_wait_us\": %d, \"seconds\": %.4f, \"GBps\": %.3f, \"requests\": %llu, "
               "\"launches\": %llu, \"value_failures\": %d, \"shard_failures\": %d, \"client_failures\": %d}\n",
               kinds, label, I, T, W, I * R, WAIT, dt,
               (double)I * n * S / dt / 1e9, (unsigned long long)reqs[o], (unsigned long long)launches[o], vbad, sbad,
               bad_count.load());
        fflush(stdout);
    };
    // warm-up (verified, twice: the first timed pass after one warm-up ran slowest, profiles/r06aj/),
    // then timed with the leaves reused and with the full rehash: one batcher
    rbc_batcher *b;
    CK(rbc_batcher_create(ctx, 64, WAIT, &b));
    if (!only_kept) run_pass(b, 0, kv, 0, "warm-up");
    for (int pass = 0; pass < (only_kept ? 0 : ki && kv ? 3 : 2); ++pass)
        run_pass(b, pass, pass < 2 && kv, pass == 2 ? 1 : 0,
                 pass < 2 && kv ? "verified (leaves reused)" : "full rehash");
    if (getenv("RBC_EPOCH_ORDER_CHECK") && ki && kv && !only_kept)  // the two forms again, the other way round
        for (int pass = 1; pass <= 2; ++pass)
            run_pass(b, pass, pass == 2, pass == 2 ? 0 : 1, pass == 2 ? "verified (leaves reused), second" : "full rehash, second");
    rbc_batcher_destroy(b);
    if (kept) {  // ABI 7: the same handler calls with the shards kept on the device (rbc_batcher_set_keep)
        CK(rbc_batcher_create(ctx, 64, WAIT, &b));
        CK(rbc_batcher_set_keep(b, keep_mib << 20));
        run_pass(b, 0, false, 2, "kept");
        run_pass(b, 0, false, 2, "kept");
        run_pass(b, 1, false, 2, "kept (validated rows stay on the device)");
        uint64_t kint = 0, hint = 0, kl = 0, ul = 0;
        rbc_batcher_keep_stats(b, &kint, &hint, &kl, &ul);
        printf("{\"phase\": \"keep\", \"ring_bytes\": %zu, \"kept_interps\": %llu, \"host_interps\": %llu, "
               "\"kept_launches\": %llu, \"unkept_launches\": %llu}\n", keep_mib << 20, (unsigned long long)kint,
               (unsigned long long)hint, (unsigned long long)kl, (unsigned long long)ul);
        rbc_batcher_destroy(b);
    }
    // the leaf-reusing, the full-rehash and the kept interpolate agree bit for bit
    const int same = !(ki && kv) || only_kept ||
                     (vout[0] == vout[1] && dig[0] == dig[1] && (!kept || (vout[2] == vout[0] && dig[2] == dig[0])));
    fails += !same;
    if (dump) {  // sampled records for the oracle (tests only read this)
        FILE *fp = fopen(dump, "wb");
        if (!fp) { fprintf(stderr, "cannot write %s\n", dump); return 1; }
        for (int i = 0; i < I; i += std::max(1, I / 8)) {
            const uint32_t ii = (uint32_t)i;
            fwrite(&ii, 4, 1, fp);
            fwrite(values.data() + (size_t)i * B, 1, B, fp);
            fwrite(roots_c.data() + (size_t)i * 32, 1, 32, fp);
            fwrite(dig[0].data() + (size_t)i * 32, 1, 32, fp);
        }
        fclose(fp);
    }
    rbc_ctx_destroy(ctx);
    printf("{\"phase\": \"check\", \"failures\": %d, \"verified_equals_full\": %s, \"speedup\": %.3f, "
           "\"kept_speedup\": %.3f}\n", fails, same ? "true" : "false", secs[0] > 0 ? secs[1] / secs[0] : 0.0,
           secs[2] > 0 ? secs[0] / secs[2] : 0.0);
    return fails ? 1 : 0;
}
