// codec_fuzz.cpp -- ASan/UBSan harness for the host code that parses
// untrusted network input (csrc/rbc_node.cpp: the pb.Message / Go-JSON codec
// of include/rbc_protocol.h and the RBC state machine's message handling).
// Built with -fsanitize=address,undefined by tests/test_sanitizers.py and run
// on the CPU: the GPU batcher is replaced by the deterministic stubs below,
// so every parse path, threshold transition and the value unframing run
// without a device.  A libFuzzer-style loop feeds random bytes and mutations
// of valid messages (bit flips, truncations, insertions, splices).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "../../include/rbc_protocol.h"

// ---- batcher stubs: every validation succeeds, interpolation returns a
// framed value whose bytes come from the shards, so delivery and unframing run
extern "C" {
struct rbc_batcher {
    int dummy;
};
static uint64_t g_ticket = 1;
int rbc_batcher_shard(rbc_batcher *, const uint8_t *data, size_t len, uint8_t *shards_out, size_t shards_cap,
                      size_t *shard_len_out, uint8_t *root_out, uint8_t *branches_out, uint64_t *ticket) {
    const size_t n = 4, k = 2, S = (len + k - 1) / k;
    if (shards_cap < n * S) return RBC_ERR_INVALID_ARG;
    memset(shards_out, 0, n * S);
    memcpy(shards_out, data, len);
    *shard_len_out = S;
    memset(root_out, 0x11, 32);
    if (branches_out) memset(branches_out, 0x22, n * 2 * 32);
    *ticket = g_ticket++;
    return RBC_OK;
}
int rbc_batcher_validate(rbc_batcher *, const uint8_t *root, const uint8_t *branch, size_t branch_len,
                         const uint8_t *shard, size_t shard_len, uint32_t index, int *ok_out, uint64_t *ticket) {
    // touch every byte the caller handed over (ASan checks the bounds)
    unsigned acc = index;
    for (size_t i = 0; i < 32; ++i) acc += root[i];
    for (size_t i = 0; i < branch_len; ++i) acc += branch[i];
    for (size_t i = 0; i < shard_len; ++i) acc += shard[i];
    *ok_out = (acc & 7) != 0;  // mostly valid, sometimes not
    *ticket = g_ticket++;
    return RBC_OK;
}
int rbc_batcher_interpolate(rbc_batcher *, const uint8_t *root, const uint8_t *const *shards, const size_t *lens,
                            uint8_t *value_out, size_t value_cap, size_t *value_len, uint8_t *digest_out,
                            uint64_t *ticket) {
    size_t S = 0;
    for (int j = 0; j < 4; ++j)
        if (lens[j]) S = lens[j];
    const size_t k = 2;
    if (value_cap < k * S) return RBC_ERR_INVALID_ARG;
    size_t o = 0;
    for (int j = 0; j < (int)k; ++j) {
        if (lens[j]) memcpy(value_out + o, shards[j], S);
        else memset(value_out + o, root[j], S);
        o += S;
    }
    *value_len = k * S;
    if (digest_out) memset(digest_out, 0, 32);
    *ticket = g_ticket++;
    return RBC_OK;
}
int rbc_batcher_wait(rbc_batcher *, uint64_t) { return RBC_OK; }
int rbc_batcher_poll(rbc_batcher *, uint64_t, int *done) {
    *done = 1;
    return RBC_OK;
}
}

static int failures = 0;
#define EXPECT(c)                                                                  \
    do {                                                                           \
        if (!(c)) {                                                                \
            fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c);            \
            if (++failures > 20) exit(1);                                          \
        }                                                                          \
    } while (0)

static std::string pb(int type, const std::string &payload) {
    size_t need = rbc_pb_encode_rbc(type, (const uint8_t *)payload.data(), payload.size(), nullptr, 0);
    std::string out(need, '\0');
    EXPECT(rbc_pb_encode_rbc(type, (const uint8_t *)payload.data(), payload.size(), (uint8_t *)&out[0], need) ==
           need);
    return out;
}

static std::string json_val(const std::string &root, const std::string &br, const std::string &blk) {
    size_t need = rbc_json_encode_val((const uint8_t *)root.data(), root.size(), (const uint8_t *)br.data(),
                                      br.size(), (const uint8_t *)blk.data(), blk.size(), nullptr, 0);
    std::string out(need, '\0');
    rbc_json_encode_val((const uint8_t *)root.data(), root.size(), (const uint8_t *)br.data(), br.size(),
                        (const uint8_t *)blk.data(), blk.size(), (uint8_t *)&out[0], need);
    return out;
}

static std::string json_ready(const std::string &root) {
    size_t need = rbc_json_encode_ready((const uint8_t *)root.data(), root.size(), nullptr, 0);
    std::string out(need, '\0');
    rbc_json_encode_ready((const uint8_t *)root.data(), root.size(), (uint8_t *)&out[0], need);
    return out;
}

static std::string rnd(std::mt19937 &g, size_t n) {
    std::string s(n, '\0');
    for (auto &c : s) c = (char)g();
    return s;
}

// decode whatever it is, with heap copies sized exactly (so ASan sees overreads)
static void decode_all(const std::string &in) {
    std::vector<uint8_t> buf(in.begin(), in.end());
    const uint8_t *p = buf.empty() ? nullptr : buf.data();
    int type = 0;
    const uint8_t *pl = nullptr;
    size_t pll = 0;
    if (rbc_pb_decode_rbc(p, buf.size(), &type, &pl, &pll) == RBC_OK) {
        EXPECT(type >= 0 && type <= 2);
        EXPECT(pll == 0 || (pl >= p && pl + pll <= p + buf.size()));
    }
    uint8_t root[32];
    size_t bl = 0, kl = 0;
    int rc = rbc_json_decode_val(p, buf.size(), root, nullptr, 0, &bl, nullptr, 0, &kl);
    if (rc == RBC_ERR_INVALID_ARG || rc == RBC_OK) {
        std::vector<uint8_t> b(bl + 1), k(kl + 1);
        EXPECT(rbc_json_decode_val(p, buf.size(), root, b.data(), bl, &bl, k.data(), kl, &kl) == RBC_OK);
    }
    (void)rbc_json_decode_ready(p, buf.size(), root);
}

static std::string mutate(std::mt19937 &g, std::string s) {
    const int ops = 1 + g() % 4;
    for (int o = 0; o < ops; ++o) {
        switch (g() % 6) {
            case 0: if (!s.empty()) s[g() % s.size()] ^= (char)(1u << (g() % 8)); break;
            case 1: if (!s.empty()) s.resize(g() % s.size()); break;
            case 2: s.insert(s.empty() ? 0 : g() % s.size(), rnd(g, 1 + g() % 8)); break;
            case 3: if (s.size() > 2) { size_t a = g() % s.size(); s.erase(a, 1 + g() % (s.size() - a)); } break;
            case 4: if (!s.empty()) s[g() % s.size()] = "{}[]\",:=\\/nul0A+"[g() % 16]; break;
            case 5: if (!s.empty()) { size_t a = g() % s.size(); s += s.substr(a, g() % (s.size() - a + 1)); } break;
        }
    }
    return s;
}

int main(int argc, char **argv) {
    const long iters = argc > 1 ? atol(argv[1]) : 20000;
    std::mt19937 g(20261016);
    // 1. round trips
    for (int t = 0; t < 500; ++t) {
        std::string root = rnd(g, 32), br = rnd(g, 32 * (g() % 9)), blk = rnd(g, 1 + g() % 300);
        std::string js = json_val(root, br, blk);
        uint8_t r2[32];
        std::vector<uint8_t> b2(br.size() + 1), k2(blk.size() + 1);
        size_t bl = 0, kl = 0;
        EXPECT(rbc_json_decode_val((const uint8_t *)js.data(), js.size(), r2, b2.data(), b2.size(), &bl, k2.data(),
                                   k2.size(), &kl) == RBC_OK);
        EXPECT(memcmp(r2, root.data(), 32) == 0 && bl == br.size() && kl == blk.size());
        EXPECT(memcmp(b2.data(), br.data(), bl) == 0 && memcmp(k2.data(), blk.data(), kl) == 0);
        std::string m = pb(t % 3, js);
        int type;
        const uint8_t *pl;
        size_t pll;
        EXPECT(rbc_pb_decode_rbc((const uint8_t *)m.data(), m.size(), &type, &pl, &pll) == RBC_OK && type == t % 3);
    }
    // 2. malformed inputs (tests/test_protocol_codec.py cases) must be rejected
    const char *bad[] = {"", "[]", "{\"RootHash\":\"AAAA\"}", "{\"RootHash\":\"X\",\"Block\":[\"AA=\"]}",
                         "{\"RootHash\":", "{\"RootHash\":\"\\u12", "{\"a\":[[[[[[[[[[[[[["};
    for (const char *b : bad) {
        uint8_t root[32];
        size_t bl, kl;
        EXPECT(rbc_json_decode_val((const uint8_t *)b, strlen(b), root, nullptr, 0, &bl, nullptr, 0, &kl) ==
               RBC_ERR_PROTOCOL);
    }
    // 3. random bytes and mutated valid messages through the decoders
    std::vector<std::string> seeds;
    for (int t = 0; t < 16; ++t) {
        std::string root = rnd(g, 32);
        seeds.push_back(pb(RBC_MSG_VAL, json_val(root, rnd(g, 64), rnd(g, 40 + t))));
        seeds.push_back(pb(RBC_MSG_ECHO, json_val(root, rnd(g, 32), rnd(g, 7))));
        seeds.push_back(pb(RBC_MSG_READY, json_ready(root)));
        seeds.push_back(json_val(root, "", rnd(g, 3)));
    }
    for (long it = 0; it < iters; ++it) {
        if (it % 4 == 0) decode_all(rnd(g, g() % 200));
        else decode_all(mutate(g, seeds[g() % seeds.size()]));
    }
    // 4. the state machine over mutated traffic (n = 4, f = 1, stub batcher)
    rbc_batcher stub{};
    long delivered_ok = 0, delivered_bad = 0, rejected = 0;
    for (int round = 0; round < 200; ++round) {
        rbc_node *nodes[4];
        for (int i = 0; i < 4; ++i) EXPECT(rbc_node_create(&stub, 4, 1, i, 0, &nodes[i]) == RBC_OK);
        std::string value = rnd(g, g() % 100);
        if (round % 5 == 0) {  // a proposer whose payload frame lies about its length
            std::string lie(8, '\0');
            for (int b = 0; b < 8; ++b) lie[b] = (char)g();
            value = lie + value;
        }
        EXPECT(rbc_node_propose(nodes[0], (const uint8_t *)value.data(), value.size()) == RBC_OK);
        for (int step = 0; step < 40; ++step) {
            for (int i = 0; i < 4; ++i) {
                rbc_node_progress(nodes[i], 1, nullptr);
                for (;;) {
                    int to = 0;
                    size_t len = 0;
                    std::vector<uint8_t> buf(4096);
                    int rc = rbc_node_next_message(nodes[i], &to, buf.data(), buf.size(), &len);
                    if (rc == RBC_ERR_INVALID_ARG) {
                        buf.resize(len);
                        rc = rbc_node_next_message(nodes[i], &to, buf.data(), buf.size(), &len);
                    }
                    if (rc != RBC_OK || len == 0) break;
                    std::string msg((const char *)buf.data(), len);
                    for (int j = 0; j < 4; ++j) {
                        if (j == i || (to >= 0 && to != j)) continue;
                        std::string m = (g() % 3 == 0) ? mutate(g, msg) : msg;
                        std::vector<uint8_t> heap(m.begin(), m.end());
                        rbc_node_handle_message(nodes[j], i, heap.empty() ? nullptr : heap.data(), heap.size());
                    }
                }
            }
        }
        for (int i = 0; i < 4; ++i) {
            size_t len = 0;
            int delivered = 0;
            int rc = rbc_node_value(nodes[i], nullptr, 0, &len, &delivered);
            if (delivered && rc == RBC_OK) {
                std::vector<uint8_t> v(len + 1);
                EXPECT(rbc_node_value(nodes[i], v.data(), v.size(), &len, &delivered) == RBC_OK);
                ++delivered_ok;
            } else if (delivered) {
                EXPECT(rc == RBC_ERR_PROTOCOL && len == 0);
                ++delivered_bad;
            }
            int e, r, s, x;
            rbc_node_stats(nodes[i], &e, &r, &s, &x);
            rejected += x;
            rbc_node_destroy(nodes[i]);
        }
    }
    if (!failures)
        printf("ok %ld iterations; nodes: %ld delivered, %ld delivered-but-misframed, %ld messages rejected\n",
               iters, delivered_ok, delivered_bad, rejected);
    else
        printf("FAIL\n");
    return failures ? 1 : 0;
}
