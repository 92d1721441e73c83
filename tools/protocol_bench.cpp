// protocol_bench.cpp -- one ACS round of reliable broadcasts in process, end to
// end through the RBC state machine (include/rbc_protocol.h): N proposers x N
// nodes = N^2 rbc_node instances share one batcher; event loops route every
// marshaled pb.Message (VAL / ECHO / READY) to its recipients until every
// node has delivered every proposal, then each delivered value is checked
// byte for byte.  The broadcasts of different proposers never exchange
// messages, so T threads each run the loop for the proposers p = t mod T
// (what a Go node does with a goroutine per instance).  One JSON line.
//   build: make -C tools protocol_bench
//   run:   tools/protocol_bench [n] [f] [value_bytes] [max_wait_us] [threads]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "../include/rbc_protocol.h"

#define CK(x)                                                                 \
    do {                                                                      \
        int rc_ = (x);                                                        \
        if (rc_) {                                                            \
            fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, rc_);  \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 16;
    const int f = argc > 2 ? atoi(argv[2]) : (n - 1) / 3;
    const size_t B = argc > 3 ? (size_t)atoll(argv[3]) : (256u << 10);
    const int WAIT = argc > 4 ? atoi(argv[4]) : 200;
    const int T = argc > 5 ? atoi(argv[5]) : 1;
    rbc_ctx *ctx;
    CK(rbc_ctx_create(n, f, 0, &ctx));
    rbc_batcher *bt;
    CK(rbc_batcher_create(ctx, 4096, WAIT, &bt));
    std::vector<std::vector<uint8_t>> values(n, std::vector<uint8_t>(B));
    uint64_t x = 0x2545F4914F6CDD1Dull;
    for (auto &v : values)
        for (auto &c : v) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            c = (uint8_t)x;
        }
    std::vector<rbc_node *> nodes((size_t)n * n);  // [proposer][node]
    for (int p = 0; p < n; ++p)
        for (int i = 0; i < n; ++i) CK(rbc_node_create(bt, n, f, i, p, &nodes[(size_t)p * n + i]));
    std::atomic<uint64_t> msgs{0}, deliveries{0}, msg_bytes{0};
    std::atomic<int> rounds{0};
    std::atomic<uint64_t> ns_progress{0}, ns_next{0}, ns_handle{0}, ns_block{0};  // thread-summed
    auto loop = [&](int t) {
    std::vector<uint8_t> buf(1 << 20);
    for (int p = t; p < n; p += T) CK(rbc_node_propose(nodes[(size_t)p * n + p], values[p].data(), B));
    int my_rounds = 0;
    while (true) {
        ++my_rounds;
        bool moved = false;
        int pending_total = 0;
        for (int p = t; p < n; p += T)
            for (int i = 0; i < n; ++i) {
                rbc_node *nd = nodes[(size_t)p * n + i];
                int pend = 0;
                const double a0 = now();
                CK(rbc_node_progress(nd, 0, &pend));
                ns_progress += (uint64_t)((now() - a0) * 1e9);
                pending_total += pend;
                while (true) {
                    int to;
                    size_t len;
                    const double b0 = now();
                    int rc = rbc_node_next_message(nd, &to, buf.data(), buf.size(), &len);
                    ns_next += (uint64_t)((now() - b0) * 1e9);
                    if (rc == RBC_ERR_INVALID_ARG && len > buf.size()) {
                        buf.resize(len);
                        continue;
                    }
                    CK(rc);
                    if (len == 0) break;
                    moved = true;
                    ++msgs;
                    msg_bytes += len;
                    const double c0 = now();
                    for (int dst = 0; dst < n; ++dst) {
                        if (dst == i || (to >= 0 && dst != to)) continue;
                        ++deliveries;
                        (void)rbc_node_handle_message(nodes[(size_t)p * n + dst], i, buf.data(), len);
                    }
                    ns_handle += (uint64_t)((now() - c0) * 1e9);
                }
            }
        if (!moved && pending_total == 0) break;
        if (!moved) {  // nothing to route: block on the outstanding GPU work
            const double d0 = now();
            for (int p = t; p < n; p += T)
                for (int i = 0; i < n; ++i) CK(rbc_node_progress(nodes[(size_t)p * n + i], 1, nullptr));
            ns_block += (uint64_t)((now() - d0) * 1e9);
        }
    }
    rounds = std::max(rounds.load(), my_rounds);
    };
    const double t0 = now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(loop, t);
    for (auto &x : th) x.join();
    const double dt = now() - t0;
    uint64_t nb = 0, nr = 0;
    rbc_batcher_stats(bt, &nb, &nr);
    int bad = 0, delivered = 0;
    std::vector<uint8_t> out(B + 16);
    for (int p = 0; p < n; ++p)
        for (int i = 0; i < n; ++i) {
            size_t len = 0;
            int dl = 0;
            CK(rbc_node_value(nodes[(size_t)p * n + i], out.data(), out.size(), &len, &dl));
            delivered += dl;
            bad += !dl || len != B || memcmp(out.data(), values[p].data(), B) != 0;
        }
    printf("{\"tool\": \"protocol_bench\", \"n\": %d, \"f\": %d, \"value_bytes\": %zu, \"max_wait_us\": %d, "
           "\"threads\": %d, \"instances\": %d, "
           "\"seconds\": %.4f, \"delivered\": %d, \"bad\": %d, \"messages\": %llu, \"deliveries\": %llu, "
           "\"message_MB\": %.1f, \"delivered_value_GBps\": %.3f, \"gpu_requests\": %llu, \"gpu_launches\": %llu, "
           "\"event_loop_rounds\": %d, \"thread_seconds\": {\"progress\": %.3f, \"next_message\": %.3f, "
           "\"handle_message\": %.3f, \"blocking_progress\": %.3f}}\n",
           n, f, B, WAIT, T, n * n, dt, delivered, bad, (unsigned long long)msgs.load(),
           (unsigned long long)deliveries.load(), msg_bytes.load() / 1e6, (double)n * n * B / dt / 1e9,
           (unsigned long long)nr, (unsigned long long)nb, rounds.load(), ns_progress.load() / 1e9,
           ns_next.load() / 1e9, ns_handle.load() / 1e9, ns_block.load() / 1e9);
    for (auto *nd : nodes) rbc_node_destroy(nd);
    rbc_batcher_destroy(bt);
    rbc_ctx_destroy(ctx);
    return bad ? 1 : 0;
}
