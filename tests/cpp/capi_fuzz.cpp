// capi_fuzz.cpp -- random-argument driver for the host runtime behind
// include/rbc_gpu.h (csrc/capi.cpp), built with ASan + UBSan against the
// host-memory HIP stand-in of tests/cpp/hip_stub.cpp (tests/test_sanitizers.py).
//
// Every call gets caller buffers of exactly the size its contract in
// rbc_gpu.h asks for, built from the same random arguments, so any read or
// write past them -- or past a device / staging / workspace buffer the
// runtime sized itself -- is an ASan report, and any signed overflow or bad
// shift in the argument arithmetic a UBSan one.  Return codes are checked
// where the contract fixes them (klauspost's error values, invalid
// arguments).  Usage: capi_fuzz <iterations> [seed]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "../../include/rbc_gpu.h"

static std::mt19937_64 rng;
static int fails = 0;
#define EXPECT(cond)                                                          \
    do {                                                                      \
        if (!(cond)) {                                                        \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++fails;                                                          \
        }                                                                     \
    } while (0)

static uint64_t rnd(uint64_t n) { return n ? rng() % n : 0; }
static bool coin(int pct) { return (int)rnd(100) < pct; }
// a length that is usually sensible and sometimes extreme
static size_t rlen(size_t typical) {
    switch (rnd(10)) {
        case 0: return 0;
        case 1: return 1;
        case 2: return typical + rnd(typical + 1);
        default: return 1 + rnd(typical);
    }
}
static std::vector<uint8_t> bytes(size_t n) {
    std::vector<uint8_t> v(n);
    for (auto &b : v) b = (uint8_t)rng();
    return v;
}
static int depth_of(int n) {
    int d = 0;
    while ((1 << d) < n) ++d;
    return d;
}

struct Geo {
    int n, f, k, d;
    rbc_ctx *ctx;
};

static void fuzz_validate_batch(Geo &g) {
    const int count = (int)rnd(12);
    std::vector<std::vector<uint8_t>> sh(count), br(count), rt(count);
    std::vector<const uint8_t *> sp(count), bp(count), rp(count);
    std::vector<size_t> sl(count), bl(count);
    std::vector<uint32_t> idx(count);
    for (int i = 0; i < count; ++i) {
        sl[i] = rlen(300);
        sh[i] = bytes(sl[i]);
        sp[i] = coin(5) ? nullptr : (sl[i] ? sh[i].data() : nullptr);
        idx[i] = coin(10) ? (uint32_t)rng() : (uint32_t)rnd(g.n);
        const bool empty0 = g.d > 0 && (idx[i] ^ 1u) >= (uint32_t)g.n;
        bl[i] = coin(70) ? 32u * (g.d - (empty0 ? 1 : 0)) : rlen(200);
        br[i] = bytes(bl[i]);
        bp[i] = coin(5) ? nullptr : (bl[i] ? br[i].data() : nullptr);
        rt[i] = bytes(32);
        rp[i] = coin(5) ? nullptr : rt[i].data();
    }
    std::vector<uint8_t> ok(count + 1);
    uint64_t t = 0;
    const bool async = coin(50);
    const int rc = rbc_validate_batch(g.ctx, count, sp.data(), sl.data(), idx.data(), bp.data(), bl.data(), rp.data(),
                                      ok.data(), async ? &t : nullptr);
    EXPECT(rc == RBC_OK);
    if (async && t) EXPECT(rbc_wait(g.ctx, t) == RBC_OK);
    for (int i = 0; i < count; ++i)
        if (!sp[i] || !rp[i] || idx[i] >= (uint32_t)g.n || sl[i] == 0) EXPECT(ok[i] == 0);
}

static void fuzz_shard_commit(Geo &g) {
    const int count = (int)rnd(6);
    std::vector<std::vector<uint8_t>> val(count);
    std::vector<const uint8_t *> vp(count);
    std::vector<size_t> vl(count);
    size_t Smax = 0;
    bool empty = false;
    for (int i = 0; i < count; ++i) {
        vl[i] = rlen(4000);
        empty |= vl[i] == 0;
        val[i] = bytes(vl[i]);
        vp[i] = vl[i] ? val[i].data() : (coin(50) ? nullptr : val[i].data());
        Smax = std::max(Smax, (vl[i] + g.k - 1) / g.k);
    }
    const size_t pitch = coin(80) ? Smax + rnd(70) : rnd(Smax + 1);
    std::vector<uint8_t> shards((size_t)count * g.n * pitch + 1), roots((size_t)count * 32 + 1);
    std::vector<uint8_t> br((size_t)count * g.n * std::max(g.d, 1) * 32 + 1);
    std::vector<uint32_t> slens(count + 1);
    uint64_t t = 0;
    const bool async = coin(50);
    const int rc = rbc_shard_commit(g.ctx, count, vp.data(), vl.data(), shards.data(), pitch, slens.data(),
                                    roots.data(), coin(30) ? nullptr : br.data(), async ? &t : nullptr);
    if (count > 0 && empty) EXPECT(rc == RBC_ERR_SHORT_DATA || rc == RBC_ERR_INVALID_ARG);
    if (rc == RBC_OK && async && t) EXPECT(rbc_wait(g.ctx, t) == RBC_OK);
}

static void fuzz_interpolate_batch(Geo &g) {
    const int count = (int)rnd(5);
    const size_t pitch = 1 + rnd(600);
    std::vector<uint8_t> shards = bytes((size_t)count * g.n * pitch + 1);
    std::vector<size_t> sl(count + 1);
    for (int i = 0; i < count; ++i) sl[i] = coin(90) ? 1 + rnd(pitch) : pitch + 1 + rnd(10);
    std::vector<uint8_t> present((size_t)count * g.n + 1);
    for (auto &p : present) p = coin(70);
    std::vector<uint8_t> roots = bytes((size_t)count * 32 + 1);
    size_t Smax = 1;
    for (int i = 0; i < count; ++i) Smax = std::max(Smax, sl[i]);
    const size_t vpitch = coin(80) ? (size_t)g.k * Smax + rnd(40) : rnd((size_t)g.k * Smax);
    std::vector<uint8_t> values((size_t)count * vpitch + 1), digests((size_t)count * 32 + 1);
    std::vector<int32_t> status(count + 1);
    uint64_t t = 0;
    const bool async = coin(50);
    // ABI 6: half the calls hand in the present rows' leaves [count][n][32]
    std::vector<uint8_t> leaves = bytes((size_t)count * g.n * 32 + 1);
    const int rc = rbc_interpolate_batch_verified(g.ctx, count, shards.data(), pitch, sl.data(), present.data(),
                                                  coin(50) ? leaves.data() : nullptr, roots.data(), values.data(),
                                                  vpitch, coin(30) ? nullptr : digests.data(), status.data(),
                                                  async ? &t : nullptr);
    bool bad = vpitch < (size_t)g.k * Smax;
    for (int i = 0; i < count; ++i) bad |= sl[i] > pitch;
    if (count > 0 && bad) EXPECT(rc == RBC_ERR_INVALID_ARG);
    if (rc == RBC_OK && async && t) {
        int done = 0;
        EXPECT(rbc_poll(g.ctx, t, &done) == RBC_OK);
        EXPECT(rbc_wait(g.ctx, t) == RBC_OK);
    }
}

// rbc_validate_packed_leaves: offsets / lengths / indices in and out of
// range, dense and sparse arenas, pageable and pinned (the sparse pinned
// case takes the gather path); leaves_out sized for exactly `count` messages.
static void fuzz_validate_packed(Geo &g) {
    const int count = (int)rnd(6);
    const size_t arena_bytes = 64 * (1 + rnd(64));
    const bool pinned = coin(50);
    uint8_t *arena = nullptr;
    std::vector<uint8_t> pageable;
    if (pinned) {
        void *q = nullptr;
        EXPECT(rbc_host_alloc(arena_bytes, &q) == RBC_OK);
        arena = (uint8_t *)q;
    } else {
        pageable = bytes(arena_bytes);
        arena = pageable.data();
    }
    std::vector<uint64_t> offs(count + 1);
    std::vector<uint32_t> lens(count + 1);
    std::vector<uint8_t> idx(count + 1);
    bool bad = false;
    for (int i = 0; i < count; ++i) {
        offs[i] = coin(90) ? 64 * rnd(arena_bytes / 64) : rnd(arena_bytes + 128);
        lens[i] = coin(90) ? (uint32_t)(1 + rnd(std::min<size_t>(arena_bytes - std::min<size_t>(offs[i], arena_bytes), 200) + 1))
                           : (uint32_t)rnd(2);
        idx[i] = coin(95) ? (uint8_t)rnd(g.n) : (uint8_t)rng();
        bad |= offs[i] % 64 || lens[i] == 0 || offs[i] > arena_bytes ||
               (lens[i] + 63) / 64 * 64 > arena_bytes - offs[i] || idx[i] >= g.n;
    }
    const size_t bslot = (size_t)std::max(g.d, 1) * 32;
    std::vector<uint8_t> br = bytes((size_t)count * bslot + 1), roots = bytes((size_t)count * 32 + 1);
    std::vector<uint8_t> ok(count + 1), leaves((size_t)count * 32 + 1);
    uint64_t t = 0;
    const bool async = coin(50);
    // ABI 7: a third of the calls move the arena into a device buffer of the caller's (sometimes too small)
    void *keep = nullptr;
    const size_t keep_bytes = coin(85) ? arena_bytes + rnd(3) * 64 : rnd(arena_bytes);
    if (coin(33)) EXPECT(rbc_dev_malloc(0, keep_bytes + 1, &keep) == RBC_OK);
    const int rc = keep ? rbc_validate_packed_keep(g.ctx, count, arena, arena_bytes, offs.data(), lens.data(),
                                                   idx.data(), br.data(), roots.data(), ok.data(),
                                                   coin(50) ? leaves.data() : nullptr, (uint8_t *)keep, keep_bytes,
                                                   async ? &t : nullptr)
                        : rbc_validate_packed_leaves(g.ctx, count, arena, arena_bytes, offs.data(), lens.data(),
                                                     idx.data(), br.data(), roots.data(), ok.data(),
                                                     coin(50) ? leaves.data() : nullptr, async ? &t : nullptr);
    if (count > 0 && (bad || (keep && keep_bytes < arena_bytes))) EXPECT(rc == RBC_ERR_INVALID_ARG);
    else EXPECT(rc == RBC_OK);
    if (rc == RBC_OK && async && t) EXPECT(rbc_wait(g.ctx, t) == RBC_OK);
    if (keep) rbc_dev_free(keep);
    if (pinned) rbc_host_free(arena);
}

// ABI 7, rbc_interpolate_batch_kept: rows by device address (NULL = absent)
// inside one device buffer, ragged lengths, value pitches too small now and
// then, with and without leaves.
static void fuzz_interpolate_kept(Geo &g) {
    const int count = (int)rnd(5);
    std::vector<size_t> sl(count + 1);
    size_t Smax = 1;
    for (int i = 0; i < count; ++i) Smax = std::max(Smax, sl[i] = 1 + rnd(300));
    const size_t dev_bytes = 64 + (size_t)g.n * Smax;
    void *dev = nullptr;
    EXPECT(rbc_dev_malloc(0, dev_bytes, &dev) == RBC_OK);
    std::vector<uint8_t> fill = bytes(dev_bytes);
    EXPECT(rbc_memcpy_h2d(dev, fill.data(), dev_bytes) == RBC_OK);
    std::vector<const uint8_t *> rows((size_t)count * g.n + 1, nullptr);
    for (int i = 0; i < count; ++i)
        for (int j = 0; j < g.n; ++j)
            if (coin(70)) rows[(size_t)i * g.n + j] = (const uint8_t *)dev + rnd(dev_bytes - sl[i] + 1);
    std::vector<uint8_t> roots = bytes((size_t)count * 32 + 1), leaves = bytes((size_t)count * g.n * 32 + 1);
    const size_t vpitch = coin(85) ? (size_t)g.k * Smax + rnd(40) : rnd((size_t)g.k * Smax);
    std::vector<uint8_t> values((size_t)count * vpitch + 1), digests((size_t)count * 32 + 1);
    std::vector<int32_t> status(count + 1);
    uint64_t t = 0;
    const bool async = coin(50);
    // now and then one row in pageable host memory: refused before anything is launched
    std::vector<uint8_t> pageable_row = bytes(320);
    bool stray = false;
    if (count > 0 && coin(15)) {
        const int i = (int)rnd(count);
        int j = 0;
        while (j < g.n && !rows[(size_t)i * g.n + j]) ++j;
        if (j < g.n) {
            rows[(size_t)i * g.n + j] = pageable_row.data();
            stray = true;
        }
    }
    const int rc = rbc_interpolate_batch_kept(g.ctx, count, rows.data(), sl.data(), coin(50) ? leaves.data() : nullptr,
                                              roots.data(), values.data(), vpitch, coin(30) ? nullptr : digests.data(),
                                              status.data(), async ? &t : nullptr);
    if (count > 0 && (vpitch < (size_t)g.k * Smax || stray)) EXPECT(rc == RBC_ERR_INVALID_ARG);
    else EXPECT(rc == RBC_OK);
    if (rc == RBC_OK && async && t) EXPECT(rbc_wait(g.ctx, t) == RBC_OK);
    rbc_dev_free(dev);
}

static void fuzz_single_calls(Geo &g) {
    // shard
    size_t len = rlen(3000);
    std::vector<uint8_t> data = bytes(len);
    const size_t S = len ? (len + g.k - 1) / g.k : 0;
    const size_t cap = coin(80) ? (size_t)g.n * S : rnd((size_t)g.n * S + 1);
    std::vector<uint8_t> out(cap + 1), root(32), br((size_t)g.n * std::max(g.d, 1) * 32);
    size_t slen = 0;
    int rc = rbc_shard(g.ctx, len ? data.data() : nullptr, len, out.data(), cap, &slen, root.data(), br.data());
    if (len == 0) EXPECT(rc == RBC_ERR_SHORT_DATA);
    if (len && cap < (size_t)g.n * S) EXPECT(rc == RBC_ERR_INVALID_ARG);
    // validateMessage
    const uint32_t j = (uint32_t)rnd(g.n + 2);
    std::vector<uint8_t> shard = bytes(rlen(200)), branch = bytes(rlen(32 * 9));
    int ok = 7;
    rc = rbc_validate_message(g.ctx, root.data(), branch.empty() ? nullptr : branch.data(), branch.size(),
                              shard.empty() ? nullptr : shard.data(), shard.size(), j, &ok);
    EXPECT(rc == RBC_OK && (ok == 0 || ok == 1));
    // interpolate
    const size_t Si = 1 + rnd(300);
    std::vector<std::vector<uint8_t>> rows(g.n);
    std::vector<const uint8_t *> rp(g.n);
    std::vector<size_t> rl(g.n);
    for (int i = 0; i < g.n; ++i) {
        rl[i] = coin(70) ? Si : (coin(80) ? 0 : 1 + rnd(2 * Si));
        rows[i] = bytes(rl[i]);
        rp[i] = rl[i] ? rows[i].data() : nullptr;
    }
    const size_t vcap = coin(80) ? (size_t)g.k * 2 * Si + 2 : rnd((size_t)g.k * Si);
    std::vector<uint8_t> value(vcap + 1), dig(32);
    size_t vlen = 0;
    rc = rbc_interpolate(g.ctx, root.data(), rp.data(), rl.data(), value.data(), vcap, &vlen, dig.data());
    EXPECT(rc <= 0);
}

static void fuzz_rs(rbc_rs *rs, int k, int p) {
    const int n = k + p;
    // Split
    size_t len = rlen(2000);
    std::vector<uint8_t> data = bytes(len);
    const size_t per = len ? (len + k - 1) / k : 0;
    const size_t cap = coin(80) ? (size_t)n * per : rnd((size_t)n * per + 1);
    std::vector<uint8_t> out(cap + 1);
    size_t got = 0;
    int rc = rbc_rs_split(rs, len ? data.data() : nullptr, len, out.data(), cap, &got);
    if (len == 0) EXPECT(rc == RBC_ERR_SHORT_DATA);
    else if (cap < (size_t)n * per) EXPECT(rc == RBC_ERR_INVALID_ARG);
    else EXPECT(rc == RBC_OK && got == per);
    // shard sets with random lengths / nils for Encode / Verify / Reconstruct / Update / Join
    const size_t S = 1 + rnd(700);
    const int ns = coin(80) ? n : (int)rnd(n + 3);
    std::vector<std::vector<uint8_t>> sh(ns);
    std::vector<uint8_t *> sp(ns);
    std::vector<size_t> sl(ns);
    for (int i = 0; i < ns; ++i) {
        sl[i] = coin(80) ? S : (coin(70) ? 0 : 1 + rnd(2 * S));
        sh[i] = bytes(std::max(sl[i], S * 2));  // reconstruct writes up to the shard size into missing slots
        sp[i] = coin(3) ? nullptr : sh[i].data();
    }
    int ok = 0;
    const int op = (int)rnd(5);
    switch (op) {
        case 0: rc = rbc_rs_encode(rs, sp.data(), sl.data(), ns); break;
        case 1: rc = rbc_rs_verify(rs, sp.data(), sl.data(), ns, &ok); break;
        case 2: rc = rbc_rs_reconstruct(rs, sp.data(), sl.data(), ns); break;
        case 3: rc = rbc_rs_reconstruct_data(rs, sp.data(), sl.data(), ns); break;
        default: {
            const int nn = coin(80) ? k : (int)rnd(k + 3);
            std::vector<std::vector<uint8_t>> nd(nn);
            std::vector<const uint8_t *> np(nn);
            std::vector<size_t> nl(nn);
            for (int i = 0; i < nn; ++i) {
                nl[i] = coin(40) ? S : (coin(80) ? 0 : 1 + rnd(2 * S));
                nd[i] = bytes(nl[i]);
                np[i] = nl[i] ? nd[i].data() : nullptr;
            }
            rc = rbc_rs_update(rs, sp.data(), sl.data(), ns, np.data(), nl.data(), nn);
            // (an empty list is a NULL array here: rejected as an invalid argument first)
            if (ns != n || nn != k)
                EXPECT(rc == RBC_ERR_TOO_FEW_SHARDS || (rc == RBC_ERR_INVALID_ARG && (nn == 0 || ns == 0)));
        }
    }
    if (ns != n && !(rc == RBC_ERR_TOO_FEW_SHARDS || rc == RBC_ERR_INVALID_ARG)) {
        fprintf(stderr, "FAIL rs op %d with %d of %d shards: %d\n", op, ns, n, rc);
        ++fails;
    }
    // Join
    const size_t outsz = rnd((size_t)k * S + 5);
    std::vector<uint8_t> dst(outsz + 1);
    std::vector<const uint8_t *> cp(sp.begin(), sp.end());
    rc = rbc_rs_join(rs, cp.data(), sl.data(), ns, outsz, dst.data());
    EXPECT(rc <= 0);
}

static void fuzz_acs() {
    const int total = (int)rnd(300), nranks = 1 + (int)rnd(9);
    int slots = 0;
    EXPECT(rbc_acs_max_share(total, nranks, &slots) == RBC_OK);
    int sum = 0;
    for (int r = 0; r < nranks; ++r) {
        int first = -1, cnt = -1;
        EXPECT(rbc_acs_partition(total, nranks, r, &first, &cnt) == RBC_OK);
        EXPECT(first == sum && cnt >= 0 && cnt <= slots);
        sum += cnt;
    }
    EXPECT(sum == total);
    int first = 0, cnt = 0;
    EXPECT(rbc_acs_partition(total, nranks, nranks, &first, &cnt) == RBC_ERR_INVALID_ARG);
    EXPECT(rbc_acs_partition(-1, nranks, 0, &first, &cnt) == RBC_ERR_INVALID_ARG);
    const int s2 = coin(80) ? slots : (int)rnd(slots + 1);
    std::vector<uint8_t> g = bytes((size_t)nranks * s2 * 64 + 1);
    std::vector<int32_t> ids(total + 1);
    std::vector<uint8_t> recs((size_t)(total + 1) * 64);
    int m = -1;
    const int rc = rbc_acs_assemble(g.data(), nranks, s2, total, ids.data(), coin(50) ? recs.data() : nullptr, &m);
    if (s2 < slots && total > 0) EXPECT(rc == RBC_ERR_INVALID_ARG);
    else EXPECT(rc == RBC_OK && m >= 0 && m <= total);
}

// Device API: argument checks with buffers sized per the contract for the
// (bounded) random scalars; the stub kernels touch what the real ones write.
static void fuzz_receive_step(Geo &g) {
    const int count = 1 + (int)rnd(4);
    const uint32_t pitch = 64 * (1 + (uint32_t)rnd(8));
    const uint32_t S = coin(85) ? 1 + (uint32_t)rnd(pitch) : pitch + 64;
    const bool view = coin(50);
    const uint32_t vpitch = view ? 0 : 16 * ((g.k * S + 15) / 16 + (uint32_t)rnd(3));
    auto dev = [](size_t b) {
        void *p = nullptr;
        rbc_dev_malloc(0, b, &p);
        return (uint8_t *)p;
    };
    std::vector<void *> owned;
    auto mk = [&](size_t b) {
        uint8_t *p = dev(b);
        owned.push_back(p);
        return p;
    };
    auto batch = [&]() {
        rbc_rx_batch b{};
        b.count = count;
        b.shards = mk((size_t)count * g.n * pitch);
        b.shard_pitch = pitch;
        b.uniform_shard_len = S;
        b.branches = mk((size_t)count * g.n * std::max(g.d, 1) * 32);
        b.roots = mk((size_t)count * 32);
        b.present = coin(70) ? mk((size_t)count * g.n) : nullptr;
        b.valid = mk((size_t)count * g.n);
        b.leaves = mk((size_t)count * g.n * 32);
        b.values_out = view ? nullptr : mk((size_t)count * vpitch);
        b.value_pitch = vpitch;
        b.digests = coin(80) ? mk((size_t)count * 32) : nullptr;
        b.status = (int32_t *)mk((size_t)count * 4);
        return b;
    };
    rbc_rx_batch a = batch(), b = batch();
    const bool alias = coin(20);
    if (alias) b.leaves = a.leaves;
    const bool bad = S > pitch;
    EXPECT(rbc_dev_receive_step(g.ctx, nullptr, &a, nullptr, nullptr) == (bad ? RBC_ERR_INVALID_ARG : RBC_OK));
    if (!bad) {
        EXPECT(rbc_dev_interpolate(g.ctx, nullptr, count, a.shards, pitch, nullptr, S, a.valid, a.leaves, 1, a.roots,
                                   nullptr, 0, nullptr, a.status) == RBC_ERR_INVALID_ARG);  // a batch is pending
        EXPECT(rbc_dev_receive_step(g.ctx, nullptr, &b, &a, nullptr) == (alias ? RBC_ERR_INVALID_ARG : RBC_OK));
        EXPECT(rbc_dev_receive_step(g.ctx, nullptr, nullptr, alias ? &a : &b, nullptr) == RBC_OK);
    }
    EXPECT(rbc_dev_interpolate(g.ctx, nullptr, count, a.shards, pitch, nullptr, S, a.valid, a.leaves, 1, a.roots,
                               a.values_out, vpitch, a.digests, a.status) == (bad ? RBC_ERR_INVALID_ARG : RBC_OK));
    for (void *p : owned) rbc_dev_free(p);
}

int main(int argc, char **argv) {
    const long iters = argc > 1 ? atol(argv[1]) : 2000;
    rng.seed(argc > 2 ? strtoull(argv[2], nullptr, 10) : 20261017);
    // invalid geometries
    rbc_ctx *bad = nullptr;
    EXPECT(rbc_ctx_create(4, 2, 0, &bad) == RBC_ERR_INV_SHARD_NUM && !bad);
    EXPECT(rbc_ctx_create(300, 10, 0, &bad) == RBC_ERR_MAX_SHARD_NUM && !bad);
    EXPECT(rbc_ctx_create(16, 5, 3, &bad) == RBC_ERR_DEVICE && !bad);
    std::vector<Geo> geos;
    for (int n : {4, 7, 16, 64, 128, 256}) {
        Geo g{n, (n - 1) / 3, 0, depth_of(n), nullptr};
        g.k = n - 2 * g.f;
        EXPECT(rbc_ctx_create(n, g.f, 0, &g.ctx) == RBC_OK);
        geos.push_back(g);
    }
    std::vector<rbc_rs *> encs;
    std::vector<std::pair<int, int>> kp = {{1, 0}, {2, 2}, {5, 5}, {17, 4}, {44, 84}};
    for (auto [k, p] : kp) {
        rbc_rs *rs = nullptr;
        EXPECT(rbc_rs_new(k, p, 0, &rs) == RBC_OK);
        encs.push_back(rs);
    }
    for (long it = 0; it < iters; ++it) {
        Geo &g = geos[rnd(geos.size())];
        switch (rnd(7)) {
            case 0: fuzz_validate_batch(g); break;
            case 1: fuzz_shard_commit(g); break;
            case 2: fuzz_interpolate_batch(g); break;
            case 3: fuzz_single_calls(g); break;
            case 4: {
                const size_t e = rnd(encs.size());
                fuzz_rs(encs[e], kp[e].first, kp[e].second);
                break;
            }
            case 5: coin(50) ? fuzz_acs() : coin(50) ? fuzz_validate_packed(g) : fuzz_interpolate_kept(g); break;
            default: fuzz_receive_step(g); break;
        }
        EXPECT(rbc_strerror((int)rnd(40) - 30) != nullptr);
        {  // issue levels: 0..3, and -1 (the commit level) for the decode transforms
            const int a = (int)rnd(7) - 2, b = (int)rnd(7) - 2;
            const bool ok_w = a >= 0 && a <= 3 && b >= 0 && b <= 3, ok_d = a >= -1 && a <= 3 && b >= -1 && b <= 3;
            EXPECT(rbc_ctx_set_wave_priority(g.ctx, a, b) == (ok_w ? RBC_OK : RBC_ERR_INVALID_ARG));
            EXPECT(rbc_ctx_set_decode_priority(g.ctx, b, a) == (ok_d ? RBC_OK : RBC_ERR_INVALID_ARG));
            EXPECT(rbc_ctx_set_decode_priority(nullptr, 0, 0) == RBC_ERR_INVALID_ARG);
        }
        EXPECT(rbc_wait(g.ctx, 0) == RBC_ERR_INVALID_ARG);
        EXPECT(rbc_wait(g.ctx, (uint64_t)1 << 60) == RBC_ERR_INVALID_ARG);
    }
    for (auto &g : geos) rbc_ctx_destroy(g.ctx);
    for (auto *rs : encs) rbc_rs_free(rs);
    if (fails) {
        printf("FAIL %d\n", fails);
        return 1;
    }
    printf("ok %ld\n", iters);
    return 0;
}
