// protocol_bench.cpp -- one ACS round of reliable broadcasts in process, end to
// end through the RBC state machine (include/rbc_protocol.h): N proposers x N
// nodes = N^2 rbc_node instances share one batcher; a single-threaded event
// loop routes every marshaled pb.Message (VAL / ECHO / READY) to its
// recipients until every node has delivered every proposal, then checks each
// delivered value byte for byte.  Prints one JSON line.
//   build: make -C tools protocol_bench     run: tools/protocol_bench [n] [f] [value_bytes] [max_wait_us]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
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
    const double t0 = now();
    for (int p = 0; p < n; ++p) CK(rbc_node_propose(nodes[(size_t)p * n + p], values[p].data(), B));
    std::vector<uint8_t> buf(1 << 20);
    uint64_t msgs = 0, deliveries = 0, msg_bytes = 0;
    int rounds = 0;
    while (true) {
        ++rounds;
        bool moved = false;
        int pending_total = 0;
        for (int p = 0; p < n; ++p)
            for (int i = 0; i < n; ++i) {
                rbc_node *nd = nodes[(size_t)p * n + i];
                int pend = 0;
                CK(rbc_node_progress(nd, 0, &pend));
                pending_total += pend;
                while (true) {
                    int to;
                    size_t len;
                    int rc = rbc_node_next_message(nd, &to, buf.data(), buf.size(), &len);
                    if (rc == RBC_ERR_INVALID_ARG && len > buf.size()) {
                        buf.resize(len);
                        continue;
                    }
                    CK(rc);
                    if (len == 0) break;
                    moved = true;
                    ++msgs;
                    msg_bytes += len;
                    for (int dst = 0; dst < n; ++dst) {
                        if (dst == i || (to >= 0 && dst != to)) continue;
                        ++deliveries;
                        (void)rbc_node_handle_message(nodes[(size_t)p * n + dst], i, buf.data(), len);
                    }
                }
            }
        if (!moved && pending_total == 0) break;
        if (!moved)  // nothing to route: block on the outstanding GPU work
            for (auto *nd : nodes) CK(rbc_node_progress(nd, 1, nullptr));
    }
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
           "\"instances\": %d, "
           "\"seconds\": %.4f, \"delivered\": %d, \"bad\": %d, \"messages\": %llu, \"deliveries\": %llu, "
           "\"message_MB\": %.1f, \"delivered_value_GBps\": %.3f, \"gpu_requests\": %llu, \"gpu_launches\": %llu, "
           "\"event_loop_rounds\": %d}\n",
           n, f, B, WAIT, n * n, dt, delivered, bad, (unsigned long long)msgs, (unsigned long long)deliveries,
           msg_bytes / 1e6, (double)n * n * B / dt / 1e9, (unsigned long long)nr, (unsigned long long)nb, rounds);
    for (auto *nd : nodes) rbc_node_destroy(nd);
    rbc_batcher_destroy(bt);
    rbc_ctx_destroy(ctx);
    return bad ? 1 : 0;
}
