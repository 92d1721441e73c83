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

#include <atomic>
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

int main(int argc, char **argv) {
    if (argc > 1 && !strcmp(argv[1], "validate-sweep")) return validate_sweep(argc - 1, argv + 1);
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
