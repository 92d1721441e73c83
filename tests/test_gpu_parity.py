"""GPU parity tests: librbc_gpu.so on an MI355X vs the CPU oracle.

* golden fixtures (tests/golden/rbc_golden.json) through the single-call
  drop-ins (shard / validateMessage / interpolate) and the Encoder mirror;
* seeded batches at BASELINE.json's full shapes (C1..C4 geometry, 1 MiB /
  4 MiB / 64 KiB values) through the device-resident batch stages, compared
  with the C restatement (oracle/librbc_ref.so) on sampled instances and with
  size-independent properties on all of them (encode -> erase -> decode
  round trip, every valid ECHO verifies, corrupted ECHOs never do, roots
  recheck);
* edge cases the reference's domain has: ragged value lengths in one batch,
  S < 16, S % 64 == 0 and SHA-256 padding boundaries, N = 1, f = 0,
  non-power-of-two N, too few shards, Byzantine non-codeword commitments.
All comparisons are bit-exact (integer/byte work)."""
import os
import zlib

import numpy as np
import pytest

import rbc_oracle as orc

pytestmark = pytest.mark.gpu


def rup(x, a):
    return (x + a - 1) // a * a


# ------------------------------------------------------------------ golden


def test_golden_shard_commit(gpu, golden):
    for c in golden["cases"]:
        if c["kind"] != "commit" or c.get("byzantine_noncodeword"):
            continue
        ctx = gpu.Context(c["n"], c["f"])
        out = ctx.shard(bytes.fromhex(c["value"]))
        assert [bytes(s).hex() for s in out["shards"]] == c["shards"], (c["n"], c["f"])
        assert out["root"].hex() == c["root"]
        if c["branches"] is not None:
            assert [b.hex() for b in out["branches"]] == c["branches"]


def test_golden_validate_message(gpu, golden):
    ctxs = {}
    shards, idx, brs, roots, want = [], [], [], [], []
    for v in golden["validate"]:
        key = (v["n"], v["f"])
        if key not in ctxs:
            ctxs[key] = gpu.Context(*key)
        ok = ctxs[key].validate_message(bytes.fromhex(v["root"]), bytes.fromhex(v["branch"]),
                                        bytes.fromhex(v["shard"]), v["index"])
        assert ok == v["ok"], v
        if key == (16, 5):
            shards.append(bytes.fromhex(v["shard"]))
            idx.append(v["index"])
            brs.append(bytes.fromhex(v["branch"]))
            roots.append(bytes.fromhex(v["root"]))
            want.append(v["ok"])
    got = ctxs[(16, 5)].validate_batch(shards, idx, brs, roots)
    assert got.tolist() == want


def _interp_groups(golden):
    last = None
    for c in golden["cases"]:
        if c["kind"] == "commit":
            last = c
        else:
            yield last, c


def test_golden_interpolate(gpu, golden):
    ctxs = {}
    for com, case in _interp_groups(golden):
        key = (case["n"], case["f"])
        if key not in ctxs:
            ctxs[key] = gpu.Context(*key)
        n = case["n"]
        shards = [bytes.fromhex(s) for s in com["shards"]]
        given = [None] * n
        for j in case["present"]:
            s = bytearray(shards[j])
            if str(j) in case["tamper"]:
                s[0] ^= case["tamper"][str(j)]
            given[j] = bytes(s)
        try:
            out = ctxs[key].interpolate(bytes.fromhex(case["root"]), given)
            status = 0
        except gpu.RBCError as e:
            status = e.code
        assert status == case["status"], (case["name"], key)
        if status == 0:
            assert out["value"].hex() == case["value"], (case["name"], key)
            assert out["digest"].hex() == case["digest"], (case["name"], key)


# ------------------------------------------------------- Encoder mirror


def test_encoder_mirror_matches_klauspost_semantics(gpu):
    # TestOneEncode known answer through the GPU encoder
    e = gpu.Encoder(5, 5)
    sh = [np.array(x, np.uint8) for x in ([0, 1], [4, 5], [2, 3], [6, 7], [8, 9])] + [np.zeros(2, np.uint8)] * 5
    e.encode(sh)
    assert [list(map(int, s)) for s in sh[5:]] == [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]
    assert e.verify(sh)
    bad = [s.copy() for s in sh]
    bad[9][1] ^= 4
    assert not e.verify(bad)
    rng = np.random.default_rng(3)
    for k, p, S in [(10, 4, 1000), (22, 42, 4097), (44, 84, 333), (86, 170, 63), (3, 0, 17), (1, 5, 129)]:
        enc = gpu.Encoder(k, p)
        ref = orc.Encoder(k, p)
        data = rng.integers(0, 256, k * S, dtype=np.uint8)
        shards = enc.split(data)
        want = ref.split(data)
        assert all(np.array_equal(a, b) for a, b in zip(shards, want))
        enc.encode(shards)
        ref.encode(want)
        assert all(np.array_equal(a, b) for a, b in zip(shards, want))
        if p == 0:
            continue
        # erase data and parity; Reconstruct restores exactly, present untouched
        keep = set(rng.permutation(k + p)[:k].tolist())
        part = [s.copy() if j in keep else None for j, s in enumerate(shards)]
        enc.reconstruct(part)
        assert all(np.array_equal(a, b) for a, b in zip(part, want))
        part = [s.copy() if j in keep else None for j, s in enumerate(shards)]
        enc.reconstruct_data(part)
        for j in range(k + p):
            if j < k:
                assert np.array_equal(part[j], want[j])
            elif j not in keep:
                assert part[j] is None
        assert enc.join(part, k * S - 5) == data.tobytes()[: k * S - 5]
    e = gpu.Encoder(4, 2)
    with pytest.raises(gpu.RBCError) as ei:
        e.reconstruct([np.zeros(3, np.uint8), None, None, None, np.zeros(3, np.uint8), None])
    assert ei.value.code == -3
    with pytest.raises(gpu.RBCError) as ei:
        e.encode([np.zeros(3, np.uint8)] * 5 + [np.zeros(2, np.uint8)])
    assert ei.value.code == -5
    with pytest.raises(gpu.RBCError) as ei:
        e.split(b"")
    assert ei.value.code == -6
    with pytest.raises(gpu.RBCError) as ei:
        e.join([np.zeros(3, np.uint8), None, np.zeros(3, np.uint8), np.zeros(3, np.uint8)], 9)
    assert ei.value.code == -7


# ---------------------------------------------------- host batch API


def test_host_batch_ragged_lengths(gpu, ref):
    n, f = 64, 21
    ctx = gpu.Context(n, f)
    rng = np.random.default_rng(9)
    lens = [1, 21, 22, 23, 1000, 4096 * 3 + 5, 47663 * 22, 64 * 22, 64 * 22 + 1, 55 * 22]
    values = [rng.integers(0, 256, L, dtype=np.uint8) for L in lens]
    out = ctx.shard_commit_batch(values)
    for i, v in enumerate(values):
        shards, root, br, leaves = ref.encode_commit(n, f, v)
        S = shards.shape[1]
        assert out["shard_lens"][i] == S
        assert np.array_equal(out["shards"][i, :, :S], shards), i
        assert bytes(out["roots"][i]) == root, i
        assert np.array_equal(out["branches"][i], br), i
    # interpolate the batch back, dropping a random N-k+... subset per instance
    count = len(values)
    Smax = out["shards"].shape[2]
    present = np.zeros((count, n), np.uint8)
    for i in range(count):
        present[i, rng.permutation(n)[: n - 2 * f]] = 1
    res = ctx.interpolate_batch(out["shards"] * present[:, :, None], out["shard_lens"], present, out["roots"])
    assert (res["status"] == 0).all()
    for i, v in enumerate(values):
        S = int(out["shard_lens"][i])
        assert res["values"][i, : len(v)].tobytes() == v.tobytes()
        assert not res["values"][i, len(v): ctx.k * S].any()


# -------------------------------------------- device pipeline at full size


class Pipeline:
    """Device buffers + the bench's step for `I` instances of (n, f, B)."""

    def __init__(self, gpu, n, f, B, I, seed, corrupt_frac=0.1, present_n=None, codec="auto"):
        self.ca = gpu
        self.ctx = gpu.Context(n, f)
        self.ctx.set_codec(codec)
        self.n, self.f, self.B, self.I = n, f, B, I
        k = self.ctx.k
        self.k = k
        self.S = S = (B + k - 1) // k
        self.d = self.ctx.depth
        self.spitch = rup(S, 64)
        self.vpitch = rup(k * S + 32, 64)
        self.opitch = rup(k * S, 16)
        rng = np.random.default_rng(seed)
        self.values = rng.integers(0, 256, size=(I, self.vpitch), dtype=np.uint8)
        self.present = np.zeros((I, n), np.uint8)
        self.corrupt = np.full(I, -1, np.int32)
        pn = n - f if present_n is None else present_n
        for i in range(I):
            pres = rng.permutation(n)[:pn]
            self.present[i, pres] = 1
            if rng.random() < corrupt_frac:
                self.corrupt[i] = int(rng.choice(pres))
        mb = gpu.DeviceBuffer
        self.b = dict(values=mb(I * self.vpitch), shards=mb(I * n * self.spitch), leaves=mb(I * n * 32),
                      roots=mb(I * 32), branches=mb(I * n * max(self.d, 1) * 32), present=mb(I * n),
                      corrupt=mb(I * 4), valid=mb(I * n), leaves_r=mb(I * n * 32), out=mb(I * self.opitch),
                      digests=mb(I * 32), status=mb(I * 4))
        self.b["values"].upload(self.values)
        self.b["present"].upload(self.present)
        self.b["corrupt"].upload(self.corrupt)

    def commit(self):
        b, c = self.b, self.ctx
        c.dev_encode(None, self.I, b["values"], self.vpitch, None, self.B, b["shards"], self.spitch)
        c.dev_leaves(None, self.I, b["shards"], self.spitch, None, self.S, b["leaves"])
        c.dev_merkle_build(None, self.I, b["leaves"], b["roots"], b["branches"])

    def poison(self, seed=99, present=True):
        """Overwrite every row the receiver must regenerate -- absent, or the
        instance's corrupted ECHO -- with seeded garbage over the whole pitch
        (rbc_dev_poison_rows), so only interpolate's regeneration can restore
        it (with the proposer's intact rows left in those slots a
        regeneration that wrote nothing would pass)."""
        b = self.b
        self.ca.rbc.poison_rows(0, None, b["shards"], self.n * self.spitch, self.spitch, self.n,
                                b["present"] if present else None, b["corrupt"], self.I, seed)

    def receive(self, poison=True):
        """Fault injection, ECHO verify, interpolate (one-shot calls); every row
        the receiver must regenerate is poisoned first unless the caller did."""
        b, c = self.b, self.ctx
        if poison:
            self.poison()
        c.dev_inject_faults(None, self.I, b["shards"], self.spitch, b["corrupt"])
        c.dev_verify(None, self.I, b["shards"], self.spitch, None, self.S, b["branches"], b["roots"],
                     b["present"], b["valid"], b["leaves_r"])
        c.dev_interpolate(None, self.I, b["shards"], self.spitch, None, self.S, b["valid"], b["leaves_r"], 1,
                          b["roots"], b["out"], self.opitch, b["digests"], b["status"])

    def receive_step(self, poison=True):
        """The timed receiver: rbc_dev_receive_step(cur) then the flush that
        completes it (verify + decode, then rehash + recheck + digest)."""
        b, c = self.b, self.ctx
        if poison:
            self.poison()
        c.dev_inject_faults(None, self.I, b["shards"], self.spitch, b["corrupt"])
        cur = c.rx_batch(self.I, b["shards"], self.spitch, None, self.S, b["branches"], b["roots"], b["present"],
                         b["valid"], b["leaves_r"], b["out"], self.opitch, b["digests"], b["status"])
        c.dev_receive_step(None, cur, None)
        c.dev_receive_step(None, None, cur)
        self.ca.rbc.lib.rbc_device_sync(0)

    def shards(self):
        return self.b["shards"].download().reshape(self.I, self.n, self.spitch)

    def assert_poisoned(self, before, sample=4):
        """The poison reached the absent / corrupted rows of a few instances
        and left the received ones alone."""
        now = self.shards()
        for i in np.linspace(0, self.I - 1, min(sample, self.I)).astype(int):
            gone = ~self.present[i].astype(bool)
            if self.corrupt[i] >= 0:
                gone[self.corrupt[i]] = True
            assert np.array_equal(now[i][~gone], before[i][~gone])
            for j in np.flatnonzero(gone):
                assert (now[i, j] != before[i, j]).mean() > 0.9, (i, j)

    def arr(self, name, dtype=np.uint8, shape=None):
        a = np.frombuffer(self.b[name].download().tobytes(), dtype=dtype)
        return a.reshape(shape) if shape else a


FULL = [
    ("c1", 64, 21, 1 << 20, 6),
    ("c2", 128, 42, 1 << 20, 6),
    ("c3", 128, 42, 4 << 20, 2),
    ("c4", 256, 85, 64 << 10, 24),
]


@pytest.mark.parametrize("name,n,f,B,I", FULL, ids=[x[0] for x in FULL])
def test_device_pipeline_full_size_vs_c_oracle(gpu, ref, name, n, f, B, I):
    pl = Pipeline(gpu, n, f, B, I, seed=zlib.crc32(name.encode()))
    pl.commit()
    sh = pl.shards()
    roots = pl.arr("roots", shape=(I, 32))
    brs = pl.arr("branches", shape=(I, n, max(pl.d, 1), 32))
    leaves = pl.arr("leaves", shape=(I, n, 32))
    S = pl.S
    for i in range(I):
        want_sh, want_root, want_br, want_leaves = ref.encode_commit(n, f, pl.values[i, :B])
        assert np.array_equal(sh[i, :, :S], want_sh), (name, i)
        assert not sh[i, :, S:].any(), "pad bytes past S must be zero"
        assert bytes(roots[i]) == want_root
        assert np.array_equal(brs[i], want_br)
        assert np.array_equal(leaves[i], want_leaves)
    pl.poison()
    pl.assert_poisoned(sh)
    pl.receive(poison=False)
    valid = pl.arr("valid", shape=(I, n))
    status = pl.arr("status", np.int32)
    out = pl.arr("out", shape=(I, pl.opitch))
    digests = pl.arr("digests", shape=(I, 32))
    for i in range(I):
        exp_valid = pl.present[i].copy()
        if pl.corrupt[i] >= 0:
            exp_valid[pl.corrupt[i]] = 0
        assert np.array_equal(valid[i], exp_valid), (name, i)
        # C oracle interpolate from the received (corrupted) shards
        rx = sh[i, :, :S].copy()
        if pl.corrupt[i] >= 0:
            rx[pl.corrupt[i], 0] ^= 0x5A
        rc, value, dig = ref.interpolate(n, f, rx, exp_valid, bytes(roots[i]))
        assert status[i] == rc == 0, (name, i)
        assert np.array_equal(out[i, : pl.k * S], value)
        assert bytes(digests[i]) == dig
        # round-trip property: the decoded value is the proposer's input
        assert out[i, :B].tobytes() == pl.values[i, :B].tobytes()
        assert not out[i, B: pl.k * S].any()


BATCH = [
    ("c1", 64, 21, 1 << 20, 1024),
    ("c2", 128, 42, 1 << 20, 1024),
    ("c3", 128, 42, 4 << 20, 256),
    ("c4", 256, 85, 64 << 10, 4096),
]


@pytest.mark.parametrize("name,n,f,B,I", BATCH, ids=[x[0] for x in BATCH])
def test_device_pipeline_every_instance_of_a_bench_batch_vs_c_oracle(gpu, ref, name, n, f, B, I):
    """Every instance of a bench-sized batch against the C restatement: root,
    leaves and the branch of a rotating leaf after commit; valid mask, status,
    value (k*S bytes) and digest after the timed receive path
    (rbc_dev_receive_step; one corrupted ECHO shard in 10% of instances), with
    every absent and corrupted row poisoned first, and the whole shard set
    regenerated back to the commit.  The oracle runs on a thread pool (ctypes
    releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    pl = Pipeline(gpu, n, f, B, I, seed=zlib.crc32(name.encode()))
    pl.commit()
    sh = pl.shards()
    roots = pl.arr("roots", shape=(I, 32))
    leaves = pl.arr("leaves", shape=(I, n, 32))
    brs = pl.arr("branches", shape=(I, n, max(pl.d, 1), 32))
    pl.poison()
    pl.assert_poisoned(sh)
    pl.receive_step(poison=False)
    valid = pl.arr("valid", shape=(I, n))
    status = pl.arr("status", np.int32)
    out = pl.arr("out", shape=(I, pl.opitch))
    digests = pl.arr("digests", shape=(I, 32))
    S, k = pl.S, pl.k
    after = pl.shards()  # interpolate regenerated every poisoned row in place: the committed shard set again
    assert np.array_equal(after, sh), name

    def check(i):
        _, want_root, want_br, want_leaves = ref.encode_commit(n, f, pl.values[i, :B])
        j = i % n
        ok = (bytes(roots[i]) == want_root and np.array_equal(leaves[i], want_leaves) and
              np.array_equal(brs[i, j, :pl.d], want_br[j]))
        exp_valid = pl.present[i].copy()
        rx = sh[i, :, :S].copy()
        if pl.corrupt[i] >= 0:
            exp_valid[pl.corrupt[i]] = 0
            rx[pl.corrupt[i], 0] ^= 0x5A
        rc, value, dig = ref.interpolate(n, f, rx, exp_valid, want_root)
        ok = ok and np.array_equal(valid[i], exp_valid) and status[i] == rc == 0
        ok = ok and np.array_equal(out[i, :k * S], value) and bytes(digests[i]) == dig
        return ok

    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        bad = [i for i, ok in enumerate(ex.map(check, range(I))) if not ok]
    assert not bad, (name, bad[:10])
    assert np.array_equal(out[:, :B], pl.values[:, :B])


def test_device_pipeline_many_instances_properties(gpu, ref):
    """Bench-shaped batch (N=128 f=42, 1 MiB, 256 instances): every
    instance round-trips; 16 sampled instances bit-exact vs the C port."""
    n, f, B, I = 128, 42, 1 << 20, 256
    pl = Pipeline(gpu, n, f, B, I, seed=77)
    pl.commit()
    roots = pl.arr("roots", shape=(I, 32))
    sample = np.random.default_rng(0).permutation(I)[:16]
    sh = pl.shards()
    for i in sample:
        _, want_root, _, _ = ref.encode_commit(n, f, pl.values[i, :B])
        assert bytes(roots[i]) == want_root
    del sh
    pl.receive()
    status = pl.arr("status", np.int32)
    assert (status == 0).all()
    out = pl.arr("out", shape=(I, pl.opitch))
    assert np.array_equal(out[:, :B], pl.values[:, :B])
    # a second round over the regenerated codeword is idempotent
    pl.corrupt[:] = -1
    pl.b["corrupt"].upload(pl.corrupt)
    pl.commit()
    roots2 = pl.arr("roots", shape=(I, 32))
    assert np.array_equal(roots, roots2)


@pytest.mark.parametrize("n,f,B", [(128, 42, 5000), (256, 85, 3000), (16, 5, 700)])
def test_device_verify_present_masks_extremes(gpu, ref, n, f, B):
    """ECHO verify with the present-row compaction: an instance with no
    received shard, one with every shard, one with a single shard, and random
    ones (C2 takes the compacted per-leaf walk, C4 the compacted leaves + shared
    paths): valid = present and proved, exactly."""
    I = 6
    pl = Pipeline(gpu, n, f, B, I, seed=n + B, corrupt_frac=0.0)
    pl.commit()
    rng = np.random.default_rng(n)
    present = np.zeros((I, n), np.uint8)
    present[1] = 1
    present[2, rng.integers(n)] = 1
    for i in range(3, I):
        present[i, rng.permutation(n)[: rng.integers(1, n)]] = 1
    pl.b["present"].upload(present)
    sh = pl.shards().copy()
    sh[4, np.flatnonzero(present[4])[0], 0] ^= 1  # one received shard that does not verify
    pl.b["shards"].upload(sh)
    c, b = pl.ctx, pl.b
    b["valid"].upload(np.full(I * n, 7, np.uint8))
    c.dev_verify(None, I, b["shards"], pl.spitch, None, pl.S, b["branches"], b["roots"], b["present"], b["valid"],
                 b["leaves_r"])
    got = pl.arr("valid", shape=(I, n))
    want = present.copy()
    want[4, np.flatnonzero(present[4])[0]] = 0
    assert np.array_equal(got, want)


@pytest.mark.parametrize("n,f,B", [(128, 42, 44 * 600 + 7), (256, 85, 86 * 500), (64, 21, 22 * 901)])
def test_device_interpolate_present_set_extremes(gpu, ref, n, f, B):
    """Interpolate on the FFT codec's geometries with the decode's extreme
    shapes: exactly k shards all parity (every data row regenerated, m = k),
    exactly k all data (nothing to solve, every parity row re-encoded), every
    shard present, and a random k: value, digest and status equal the C
    oracle's."""
    k = n - 2 * f
    I = 4
    pl = Pipeline(gpu, n, f, B, I, seed=B, corrupt_frac=0.0)
    pl.commit()
    present = np.zeros((I, n), np.uint8)
    present[0, k:2 * k] = 1                       # k parity rows only
    present[1, :k] = 1                            # the k data rows
    present[2, :] = 1                             # everything
    present[3, np.random.default_rng(B).permutation(n)[:k]] = 1
    pl.b["present"].upload(present)
    pl.receive()
    status = pl.arr("status", np.int32)
    out = pl.arr("out", shape=(I, pl.opitch))
    digests = pl.arr("digests", shape=(I, 32))
    sh = pl.shards()
    roots = pl.arr("roots", shape=(I, 32))
    for i in range(I):
        rc, value, dig = ref.interpolate(n, f, sh[i, :, :pl.S] * present[i, :, None], present[i], bytes(roots[i]))
        assert status[i] == rc == 0, i
        assert np.array_equal(out[i, :k * pl.S], value) and bytes(digests[i]) == dig, i
        assert out[i, :B].tobytes() == pl.values[i, :B].tobytes()


@pytest.mark.parametrize("n,f,B", [(16, 5, 6 * (32 << 20) + 5), (256, 85, 86 * (1 << 20)), (128, 42, 44 * (4 << 20))],
                         ids=["S=32MiB", "N=256,S=1MiB", "N=128,S=4MiB"])
def test_device_pipeline_large_instances(gpu, ref, n, f, B):
    """Maximum-size shapes: one instance of 0.5-1.2 GiB of shards (row
    offsets past 2^24 / 2^31 bits of a single row stay exact), through commit,
    verify and interpolate against the C oracle."""
    I = 1
    pl = Pipeline(gpu, n, f, B, I, seed=n, corrupt_frac=1.0)
    pl.commit()
    sh = pl.shards()
    root = bytes(pl.arr("roots", shape=(I, 32))[0])
    want_sh, want_root, _, _ = ref.encode_commit(n, f, pl.values[0, :B])
    assert root == want_root
    assert np.array_equal(sh[0, :, :pl.S], want_sh)
    pl.receive()
    assert pl.arr("status", np.int32)[0] == 0
    out = pl.arr("out", shape=(I, pl.opitch))
    assert out[0, :B].tobytes() == pl.values[0, :B].tobytes()
    exp_valid = pl.present[0].copy()
    exp_valid[pl.corrupt[0]] = 0
    rx = want_sh.copy()
    rx[pl.corrupt[0], 0] ^= 0x5A
    rc, value, dig = ref.interpolate(n, f, rx, exp_valid, want_root)
    assert rc == 0 and bytes(pl.arr("digests", shape=(I, 32))[0]) == dig


def test_device_too_few_and_root_mismatch(gpu):
    """present = k-1 -> TOO_FEW_SHARDS; wrong expected root -> ROOT_MISMATCH;
    a corrupted used shard that passes verify (present mask forged) ->
    ROOT_MISMATCH, never a wrong value."""
    n, f, B, I = 16, 5, 5000, 6
    pl = Pipeline(gpu, n, f, B, I, seed=5, corrupt_frac=0.0, present_n=n - 2 * f - 1)
    pl.commit()
    pl.receive()
    assert (pl.arr("status", np.int32) == -3).all()
    pl = Pipeline(gpu, n, f, B, I, seed=6, corrupt_frac=0.0)
    pl.commit()
    roots = pl.arr("roots", shape=(I, 32)).copy()
    bad = roots.copy()
    bad[::2, 0] ^= 1
    pl.b["roots"].upload(bad)
    c, b = pl.ctx, pl.b
    c.dev_verify(None, I, b["shards"], pl.spitch, None, pl.S, b["branches"], b["roots"], b["present"], b["valid"],
                 b["leaves_r"])
    assert not pl.arr("valid", shape=(I, n))[::2].any()
    # forge: mark all present as valid against the wrong root, decode
    b["valid"].upload(pl.present)
    c.dev_interpolate(None, I, b["shards"], pl.spitch, None, pl.S, b["valid"], b["leaves"], 0, b["roots"],
                      b["out"], pl.opitch, b["digests"], b["status"])
    st = pl.arr("status", np.int32)
    assert (st[::2] == -8).all() and (st[1::2] == 0).all()


@pytest.mark.parametrize("n,f,B", [
    (4, 1, 1024), (4, 1, 1), (5, 0, 77), (1, 0, 10), (7, 2, 333), (13, 4, 5 * 64), (13, 4, 5 * 55),
    (13, 4, 5 * 56), (13, 4, 5 * 63), (64, 21, 22 * 16), (64, 21, 22 * 15), (256, 85, 86 * 4096 + 3),
    # the FFT codec's geometries at tiny and odd shard lengths (S = 1, 3, 17, 2, 7, 4097)
    (128, 42, 1), (128, 42, 44 * 3), (128, 42, 44 * 17 - 5), (64, 21, 22 * 2 - 1), (256, 85, 86 * 7),
    (128, 42, 44 * 4097),
])
def test_device_pipeline_edge_geometries(gpu, ref, n, f, B):
    I = 5
    pl = Pipeline(gpu, n, f, B, I, seed=n * 1000 + B, corrupt_frac=0.5)
    pl.commit()
    sh = pl.shards()
    roots = pl.arr("roots", shape=(I, 32))
    for i in range(I):
        want_sh, want_root, _, _ = ref.encode_commit(n, f, pl.values[i, :B])
        assert np.array_equal(sh[i, :, : pl.S], want_sh)
        assert bytes(roots[i]) == want_root
    pl.receive()
    status = pl.arr("status", np.int32)
    out = pl.arr("out", shape=(I, pl.opitch))
    valid = pl.arr("valid", shape=(I, n))
    for i in range(I):
        ok = valid[i].sum() >= pl.k
        assert status[i] == (0 if ok else -3)
        if ok:
            assert out[i, :B].tobytes() == pl.values[i, :B].tobytes()


def test_byzantine_noncodeword_rejected_by_every_subset(gpu, golden):
    com = [c for c in golden["cases"] if c.get("byzantine_noncodeword")][0]
    n, f = com["n"], com["f"]
    ctx = gpu.Context(n, f)
    shards = [bytes.fromhex(s) for s in com["shards"]]
    root = bytes.fromhex(com["root"])
    rng = np.random.default_rng(0)
    for _ in range(8):
        keep = set(rng.permutation(n)[: n - 2 * f].tolist())
        with pytest.raises(gpu.RBCError) as ei:
            ctx.interpolate(root, [s if j in keep else None for j, s in enumerate(shards)])
        assert ei.value.code == -8


def test_batcher_coalesces_concurrent_requests(gpu, ref):
    """Many threads (the Go goroutines) submit single-instance shard /
    validate / interpolate requests; the batcher merges them into few
    launches and every result is bit-exact."""
    import threading

    n, f = 16, 5
    ctx = gpu.Context(n, f)
    bt = gpu.Batcher(ctx, max_batch=64, max_wait_us=2000)
    rng = np.random.default_rng(42)
    values = [rng.integers(0, 256, int(rng.integers(1, 5000)), dtype=np.uint8) for _ in range(96)]
    results = [None] * len(values)
    errors = []

    def worker(idx):
        try:
            h = bt.submit_shard(values[idx])
            out = bt.wait(h)
            shards, root, br, _ = ref.encode_commit(n, f, values[idx])
            assert out["root"] == root
            assert all(np.array_equal(out["shards"][j], shards[j]) for j in range(n))
            # validate every shard, then interpolate from a random k subset
            hs = []
            com = orc.rbc_commit(shards)
            for j in range(n):
                hs.append(bt.submit_validate(root, orc.flat_branch(com["branches"][j]), shards[j], j))
            assert all(bt.wait(hh) for hh in hs)
            keep = set(np.random.default_rng(idx).permutation(n)[: ctx.k].tolist())
            hi = bt.submit_interpolate(root, [shards[j] if j in keep else b"" for j in range(n)])
            res = bt.wait(hi)
            assert res["value"][: len(values[idx])] == values[idx].tobytes()
            results[idx] = True
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(len(values))]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not errors, errors[:3]
    assert all(results)
    batches, requests = bt.stats()
    assert requests == len(values) * (2 + n)
    assert batches < requests / 4, (batches, requests)  # actually coalesced
    bt.close()


# ------------------------------------------- FFT codec vs matrix codec


FFT_GEOMS = [(4, 1, 1000, 8), (16, 5, 4099, 8), (64, 21, 1 << 20, 4), (128, 42, 1 << 20, 6),
             (256, 85, 64 << 10, 16)]


@pytest.mark.parametrize("n,f,B,I", FFT_GEOMS, ids=[f"n{g[0]}" for g in FFT_GEOMS])
def test_fft_codec_matches_matrix_codec(gpu, n, f, B, I):
    """The additive-FFT codec (rs_fft.hip) and the klauspost encode-matrix
    kernel produce identical shards, statuses, values, digests and re-hash
    lists on the same inputs, across erasure classes: random N-f present,
    parity only, data only, exactly k, plus corrupted ECHO shards."""
    outs = {}
    for codec in ("matrix", "fft"):
        pl = Pipeline(gpu, n, f, B, I, seed=n * 7 + B, corrupt_frac=0.3, codec=codec)
        assert pl.ctx.codec == codec
        k = pl.k
        for i in range(I):  # erasure classes on the first instances
            if i % 4 == 1:
                pl.present[i] = 0
                pl.present[i, k:] = 1            # parity only (n-k >= k here)
                if n - k < k:
                    pl.present[i, :k - (n - k)] = 1
            elif i % 4 == 2:
                pl.present[i] = 0
                pl.present[i, :k] = 1            # data only
                pl.corrupt[i] = -1
            elif i % 4 == 3:
                pl.present[i] = 0
                pl.present[i, np.random.default_rng(i).permutation(n)[:k]] = 1
                pl.corrupt[i] = -1
        pl.b["present"].upload(pl.present)
        pl.b["corrupt"].upload(pl.corrupt)
        pl.commit()
        enc_shards = pl.shards().copy()
        pl.receive()
        outs[codec] = dict(enc=enc_shards, dec=pl.shards(), status=pl.arr("status", np.int32).copy(),
                           out=pl.arr("out", shape=(I, pl.opitch)).copy(),
                           digests=pl.arr("digests", shape=(I, 32)).copy(), values=pl.values, B=B)
    a, b = outs["matrix"], outs["fft"]
    assert np.array_equal(a["enc"], b["enc"])
    assert np.array_equal(a["status"], b["status"])
    ok = a["status"] == 0
    S = (B + (n - 2 * f) - 1) // (n - 2 * f)
    kS = (n - 2 * f) * S  # the value is k*S bytes; bytes past it are unspecified
    assert np.array_equal(a["out"][ok][:, :kS], b["out"][ok][:, :kS])
    assert np.array_equal(a["digests"][ok], b["digests"][ok])
    for i in np.nonzero(ok)[0]:
        assert b["out"][i, :B].tobytes() == b["values"][i, :B].tobytes()
    # the full regenerated codeword is the encoding (both codecs, in place)
    assert np.array_equal(a["dec"][ok], a["enc"][ok])
    assert np.array_equal(b["dec"][ok], b["enc"][ok])


def test_fft_codec_rejects_noncodeword(gpu):
    """Byzantine proposer commits to a non-codeword: the FFT codec's compare
    path must catch it (ROOT_MISMATCH) whatever subset is decoded."""
    n, f, B, I = 128, 42, 44 * 640, 8
    pl = Pipeline(gpu, n, f, B, I, seed=11, corrupt_frac=0.0, codec="fft")
    c, b = pl.ctx, pl.b
    c.dev_encode(None, I, b["values"], pl.vpitch, None, B, b["shards"], pl.spitch)
    sh = pl.shards().copy()
    sh[:, 100, 5] ^= 0x21                       # parity row no longer a codeword row
    b["shards"].upload(sh)
    c.dev_leaves(None, I, b["shards"], pl.spitch, None, pl.S, b["leaves"])
    c.dev_merkle_build(None, I, b["leaves"], b["roots"], b["branches"])
    rng = np.random.default_rng(1)
    for i in range(I):
        pl.present[i] = 0
        pl.present[i, rng.permutation(n)[: n - f]] = 1
        pl.present[i, 100] = 1 if i % 2 else 0   # tampered row present (valid) or absent
    b["present"].upload(pl.present)
    c.dev_verify(None, I, b["shards"], pl.spitch, None, pl.S, b["branches"], b["roots"], b["present"],
                 b["valid"], b["leaves_r"])
    c.dev_interpolate(None, I, b["shards"], pl.spitch, None, pl.S, b["valid"], b["leaves_r"], 1, b["roots"],
                      b["out"], pl.opitch, b["digests"], b["status"])
    assert (pl.arr("status", np.int32) == -8).all()


def test_host_api_pipelined_submissions(gpu, ref):
    """Host batch API tickets are asynchronous: several submissions are in
    flight at once (more than the context's slots, so slot reuse retires the
    oldest), completion order is the caller's, and every result is bit-exact."""
    n, f = 16, 5
    ctx = gpu.Context(n, f)
    rng = np.random.default_rng(123)
    batches = [[rng.integers(0, 256, int(rng.integers(1, 9000)), dtype=np.uint8) for _ in range(7)]
               for _ in range(5)]
    tickets = [ctx.shard_commit_submit(b) for b in batches]
    polled = [t.done() for t in tickets]  # any mix of done / not yet
    assert len(polled) == 5
    for t, b in zip(reversed(tickets), reversed(batches)):
        out = t.wait()
        for i, v in enumerate(b):
            shards, root, br, _ = ref.encode_commit(n, f, v)
            S = shards.shape[1]
            assert out["shard_lens"][i] == S
            assert np.array_equal(out["shards"][i, :, :S], shards)
            assert bytes(out["roots"][i]) == root
            assert np.array_equal(out["branches"][i], br)
    assert tickets[0].wait() is tickets[0].result  # waiting twice is harmless


@pytest.mark.parametrize("pinned", [False, True])
def test_host_api_mixed_submissions_deferred_copies(gpu, ref, pinned):
    """The three host batch entry points interleaved with more tickets in
    flight than slots: each submission's device-to-host copies are deferred
    until the next submission (or a poll / wait), so polls, waits in reverse
    order and slot reuse must all still land bit-exact outputs, pinned or
    pageable caller memory alike."""
    n, f = 16, 5
    k = n - 2 * f
    ctx = gpu.Context(n, f)
    rng = np.random.default_rng(7 + pinned)
    B, count = 6000, 5
    S = (B + k - 1) // k
    alloc = (lambda shape: gpu.pinned_empty(shape)) if pinned else (lambda shape: np.zeros(shape, np.uint8))
    vals = []
    for _ in range(3):
        vv = []
        for _ in range(count):
            a = alloc(B)
            a[:] = rng.integers(0, 256, B, dtype=np.uint8)
            vv.append(a)
        vals.append(vv)
    want = [[ref.encode_commit(n, f, v) for v in vv] for vv in vals]
    # receiver inputs from the oracle's codewords: N-f present, one absent-by-zero row each
    rx = alloc((count, n, S))
    present = np.zeros((count, n), np.uint8)
    roots = np.zeros((count, 32), np.uint8)
    for i in range(count):
        sh, root, _, _ = want[2][i]
        pres = rng.permutation(n)[: n - f]
        present[i, pres] = 1
        rx[i] = sh * present[i, :, None]
        roots[i] = np.frombuffer(root, np.uint8)
    outs = {"shards": alloc((count, n, S)), "roots": alloc((count, 32)),
            "branches": alloc((count, n, max(ctx.depth, 1), 32))} if pinned else None
    t1 = ctx.shard_commit_submit(vals[0], out=outs)
    t2 = ctx.interpolate_submit(rx, [S] * count, present, roots, values_out=alloc((count, k * S)))
    t3 = ctx.shard_commit_val_submit(vals[1])
    t4 = ctx.shard_commit_submit(vals[2])
    assert isinstance(t3.done(), bool)  # a poll enqueues t3's deferred copies
    r4, r3, r2, r1 = t4.wait(), t3.wait(), t2.wait(), t1.wait()
    for r, w in ((r1, want[0]), (r4, want[2])):
        for i in range(count):
            sh, root, br, _ = w[i]
            assert np.array_equal(r["shards"][i, :, :S], sh) and bytes(r["roots"][i]) == root
            assert np.array_equal(r["branches"][i], br)
    assert (r2["status"] == 0).all()
    for i in range(count):
        rc, value, dig = ref.interpolate(n, f, rx[i], present[i], bytes(roots[i]))
        assert rc == 0 and np.array_equal(r2["values"][i], value) and bytes(r2["digests"][i]) == dig
        assert bytes(r3["roots"][i]) == want[1][i][1]
    # the VAL messages equal the host codec's bytes for (root, branch j, shard j)
    from cleisthenes_amd import protocol
    for i in (0, count - 1):
        sh, root, br, _ = want[1][i]
        for j in (0, n - 1):
            flat = b"".join(bytes(br[j, lvl]) for lvl in range(ctx.depth) if not (lvl == 0 and (j ^ 1) >= n))
            assert r3["message"](i, j) == protocol.pb_encode(protocol.VAL, protocol.json_encode_val(root, flat,
                                                                                                   bytes(sh[j])))


@pytest.mark.parametrize("n,f,S", [(64, 21, 187), (64, 21, 192), (128, 42, 200)])
def test_two_rows_per_lane_sha_path(gpu, ref, n, f, S):
    """ECHO verify grids of >= 262,144 rows take sha_rows2_kernel (two rows
    per lane, interleaved compressions): every leaf equals hashlib, every valid bit the
    expectation, sampled instances bit-exact vs the C port; tails of
    len % 64 > 55 (two padding blocks), == 0 and short."""
    import hashlib
    k = n - 2 * f
    I = (4 * 64 * 1024) // n
    B = S * k
    pl = Pipeline(gpu, n, f, B, I, seed=S)
    pl.commit()
    sh = pl.shards()
    leaves = pl.arr("leaves", shape=(I, n, 32))
    for i in range(I):
        for j in range(n):
            assert leaves[i, j].tobytes() == hashlib.sha256(sh[i, j, :S].tobytes()).digest(), (i, j)
    roots = pl.arr("roots", shape=(I, 32))
    for i in np.random.default_rng(1).permutation(I)[:8]:
        _, want_root, _, _ = ref.encode_commit(n, f, pl.values[i, :B])
        assert bytes(roots[i]) == want_root
    pl.receive()
    valid = pl.arr("valid", shape=(I, n))
    exp = pl.present.copy()
    for i in range(I):
        if pl.corrupt[i] >= 0:
            exp[i, pl.corrupt[i]] = 0
    assert np.array_equal(valid, exp)
    leaves_r = pl.arr("leaves_r", shape=(I, n, 32))
    assert np.array_equal(leaves_r[exp == 1], leaves[exp == 1])  # verify's own leaf hashes
    assert (pl.arr("status", np.int32) == 0).all()
    # with a present mask verify hashes the compacted received rows; without
    # one every row is hashed, by the two-rows-per-lane kernel at this size
    c, b = pl.ctx, pl.b
    c.dev_verify(None, I, b["shards"], pl.spitch, None, S, b["branches"], b["roots"], None, b["valid"], b["leaves_r"])
    exp_all = np.ones((I, n), np.uint8)  # interpolate rewrote every row with the re-encoding
    assert np.array_equal(pl.arr("valid", shape=(I, n)), exp_all)
    assert np.array_equal(pl.arr("leaves_r", shape=(I, n, 32)), leaves)  # = the committed leaves
    out = pl.arr("out", shape=(I, pl.opitch))
    assert np.array_equal(out[:, :B], pl.values[:, :B])


@pytest.mark.parametrize("n,f,B,I", [(4, 1, 1024, 8), (7, 2, 333, 8), (13, 4, 5 * 55, 8), (16, 5, 600, 8),
                                     (128, 42, 44 * 70, 8), (256, 85, 86 * 9, 8)])
def test_device_verify_shared_paths_adversarial(gpu, ref, n, f, B, I):
    """rbc_dev_verify (shared-path kernel: one hash per distinct walk input)
    against the per-leaf oracle walk on adversarial ECHO sets: corrupted
    shards, corrupted branch slots at every level, branches spliced from a
    different tree, a wrong root, garbage in the empty level-0 slot, sparse
    present masks.  valid[i][j] must equal present && oracle verify."""
    pl = Pipeline(gpu, n, f, B, I, seed=1000 + n, corrupt_frac=0.0, present_n=n)
    pl.commit()
    c, b, d, S = pl.ctx, pl.b, pl.d, pl.S
    sh = pl.shards().copy()
    roots = pl.arr("roots", shape=(I, 32)).copy()
    brs = pl.arr("branches", shape=(I, n, d, 32)).copy()
    rng = np.random.default_rng(77 + n)
    present = np.ones((I, n), np.uint8)
    # 1: one corrupted shard; 2: one corrupted branch slot per level;
    # 3: leaves 0..n/2 carry instance 0's shards + branches (another tree);
    # 4: wrong root; 5: 30% of branch slots corrupted; 6: sparse present;
    # 7: garbage in every (empty or not) level-0 slot of odd-N last leaf + a
    #    shard corrupted so that its sibling's walk diverges
    sh[1, rng.integers(n), rng.integers(S)] ^= 0x5A
    for l in range(d):
        brs[2, rng.integers(n), l, rng.integers(32)] ^= 1
    h = max(1, n // 2)
    sh[3, :h] = sh[0, :h]
    brs[3, :h] = brs[0, :h]
    roots[4, 0] ^= 0x80
    m = rng.random((n, d)) < 0.3
    brs[5][m] ^= 0xFF
    present[6] = (rng.random(n) < 0.5).astype(np.uint8)
    brs[7, n - 1, 0] = 0xEE
    sh[7, 0, 0] ^= 1
    b["shards"].upload(sh)
    b["branches"].upload(brs)
    b["roots"].upload(roots)
    b["present"].upload(present)
    b["valid"].upload(np.full((I, n), 7, np.uint8))
    c.dev_verify(None, I, b["shards"], pl.spitch, None, S, b["branches"], b["roots"], b["present"], b["valid"],
                 b["leaves_r"])
    got = pl.arr("valid", shape=(I, n))
    leaves = pl.arr("leaves_r", shape=(I, n, 32))
    for i in range(I):
        for j in range(n):
            slots = brs[i, j].copy()
            if (j ^ 1) >= n:
                slots[0] = 0  # device form: an empty level-0 sibling is a zero slot
            want = bool(present[i, j]) and ref.verify(n, sh[i, j, :S], j, slots, bytes(roots[i]))
            assert got[i, j] == int(want), (n, i, j)
            if present[i, j]:  # only received shards are hashed (leaves of absent rows: unspecified)
                assert leaves[i, j].tobytes() == ref.sha256(sh[i, j, :S].tobytes()), (n, i, j)
    assert got[0].all() and not got[4].any()


@pytest.mark.parametrize("n,f", [(256, 85), (200, 66)])
def test_device_verify_speculative_top_levels(gpu, ref, n, f):
    """merkle_path_kernel's speculative top levels (W = 256: every node above
    level 2 hashed at once from the children the branches claim, proven or
    re-run exactly) against the per-leaf oracle walk, one instance per case:
    honest; whole 8/16/32/128-leaf blocks absent (claims missing, a chain of
    dependent node hashes up to six deep); a single participant; one leaf's
    slot corrupted at each level 2..7; a level-3 subtree whose leaves agree on
    a wrong level-3 sibling; two leaves of a level-2 node reaching different
    level-2 values; a level-2 sibling claim that disagrees with the exact
    value; a wrong root; nothing present; random sparse sets with random slot
    corruption.  valid[i][j] must equal present && oracle verify."""
    B, I = 9 * (n - 2 * f), 40
    pl = Pipeline(gpu, n, f, B, I, seed=500 + n, corrupt_frac=0.0, present_n=n)
    pl.commit()
    c, b, d, S = pl.ctx, pl.b, pl.d, pl.S
    assert d == 8
    sh = pl.shards().copy()
    roots = pl.arr("roots", shape=(I, 32)).copy()
    brs = pl.arr("branches", shape=(I, n, d, 32)).copy()
    rng = np.random.default_rng(3 + n)
    present = np.ones((I, n), np.uint8)
    i = 1
    for blk in (8, 16, 32, 128):  # 1-4: whole blocks absent
        present[i, blk:2 * blk] = 0
        present[i, 0:min(n, 4)] = 0
        i += 1
    present[5] = 0  # 5: one participant
    present[5, 37] = 1
    for l in range(2, 8):  # 6-11: one leaf's level-l slot corrupted
        brs[6 + l - 2, int(rng.integers(n)), l, int(rng.integers(32))] ^= 0x40
    brs[12, 8:16, 3, 0] ^= 0x01  # 12: a level-3 subtree agrees on a wrong level-3 sibling
    sh[13, 41, 0] ^= 0x01  # 13: leaf 41's level-2 value differs from leaves 40, 42, 43
    brs[14, 4:8, 2, 7] ^= 0x80  # 14: leaves 4..7 claim a wrong value for node (2, 0)
    roots[15, 31] ^= 0x01  # 15: wrong root
    present[16] = 0  # 16: nothing present
    brs[17, 0:64, 6, 3] ^= 0x02  # 17: the left quarter agrees on a wrong level-6 sibling
    present[18] = 0  # 18: only the right half
    present[18, 128:] = 1
    for i in range(19, I):  # random sparse sets, some with a corrupted slot or shard
        present[i] = (rng.random(n) < rng.uniform(0.05, 0.9)).astype(np.uint8)
        if i % 3 == 0:
            brs[i, int(rng.integers(n)), int(rng.integers(d)), int(rng.integers(32))] ^= 0x10
        if i % 5 == 0:
            sh[i, int(rng.integers(n)), int(rng.integers(S))] ^= 0x10
    b["shards"].upload(sh)
    b["branches"].upload(brs)
    b["roots"].upload(roots)
    b["present"].upload(present)
    b["valid"].upload(np.full((I, n), 7, np.uint8))
    c.dev_verify(None, I, b["shards"], pl.spitch, None, S, b["branches"], b["roots"], b["present"], b["valid"],
                 b["leaves_r"])
    got = pl.arr("valid", shape=(I, n))
    for i in range(I):
        for j in range(n):
            slots = brs[i, j].copy()
            if (j ^ 1) >= n:
                slots[0] = 0
            want = bool(present[i, j]) and ref.verify(n, sh[i, j, :S], j, slots, bytes(roots[i]))
            assert got[i, j] == int(want), (n, i, j)
    assert got[0].all() and got[1:5][present[1:5] == 1].all() and got[5, 37] and got[18, 128:].all()
    assert not got[15].any() and not got[16].any() and not got[12, 8:16].any() and not got[17, 0:64].any()


def test_device_verify_shared_paths_large_grid(gpu, ref):
    """The shared-path kernel over a large grid: 4096 instances at N = 256, 64 of them adversarial (corrupted shards and
    branch slots at random levels, a wrong root, a spliced subtree), checked
    against the per-leaf oracle walk; the honest rest must be all-valid."""
    n, f, B, I = 256, 85, 86 * 9, 4096
    pl = Pipeline(gpu, n, f, B, I, seed=4242, corrupt_frac=0.0, present_n=n)
    pl.commit()
    c, b, d, S = pl.ctx, pl.b, pl.d, pl.S
    sh = pl.shards().copy()
    roots = pl.arr("roots", shape=(I, 32)).copy()
    brs = pl.arr("branches", shape=(I, n, d, 32)).copy()
    rng = np.random.default_rng(99)
    bad = sorted(rng.choice(I, 64, replace=False).tolist())
    for q, i in enumerate(bad):
        kind = q % 4
        if kind == 0:
            sh[i, rng.integers(n), rng.integers(S)] ^= 0x11
        elif kind == 1:
            for _ in range(3):
                brs[i, rng.integers(n), rng.integers(d), rng.integers(32)] ^= 4
        elif kind == 2:
            roots[i, 5] ^= 1
        else:
            o = (i + 1) % I
            lo = 32 * rng.integers(8)
            sh[i, lo:lo + 32] = sh[o, lo:lo + 32]
            brs[i, lo:lo + 32] = brs[o, lo:lo + 32]
    b["shards"].upload(sh)
    b["branches"].upload(brs)
    b["roots"].upload(roots)
    c.dev_verify(None, I, b["shards"], pl.spitch, None, S, b["branches"], b["roots"], None, b["valid"],
                 b["leaves_r"])
    got = pl.arr("valid", shape=(I, n))
    honest = np.ones(I, bool)
    honest[bad] = False
    assert got[honest].all()
    for i in bad:
        for j in range(n):
            want = ref.verify(n, sh[i, j, :S], j, brs[i, j], bytes(roots[i]))
            assert got[i, j] == int(want), (i, j)
        assert not got[i].all()


@pytest.mark.parametrize("lens", [[5000] * 6, [1, 21, 22, 23, 1000, 4096 * 3 + 5]], ids=["uniform", "ragged"])
def test_host_batch_pinned_direct_copies(gpu, ref, lens):
    """Pinned (rbc_host_alloc) caller buffers take the direct H2D/D2H path of
    rbc_shard_commit / rbc_interpolate_batch: results byte-identical to the
    staged path and to the oracle, including the rows' bytes past S_i."""
    n, f = 16, 5
    ctx = gpu.Context(n, f)
    rng = np.random.default_rng(31)
    values = [rng.integers(0, 256, L, dtype=np.uint8) for L in lens]
    staged = ctx.shard_commit_batch(values)
    pv = []
    for v in values:
        p = gpu.pinned_empty(len(v))
        p[:] = v
        pv.append(p)
    count, Smax, d = len(values), staged["shards"].shape[2], ctx.depth
    out = {"shards": gpu.pinned_empty((count, n, Smax)), "roots": gpu.pinned_empty((count, 32)),
           "branches": gpu.pinned_empty((count, n, d, 32))}
    out["shards"][:] = 0xAB  # every byte of a row up to Smax must be written (zeros past S_i)
    direct = ctx.shard_commit_submit(pv, out=out).wait()
    for key in ("shards", "roots", "branches", "shard_lens"):
        assert np.array_equal(np.asarray(direct[key]), np.asarray(staged[key])), key
    for i, v in enumerate(values):
        shards, root, br, _ = ref.encode_commit(n, f, v)
        assert bytes(direct["roots"][i]) == root
    present = np.zeros((count, n), np.uint8)
    for i in range(count):
        present[i, rng.permutation(n)[: n - f]] = 1
    rx = gpu.pinned_empty((count, n, Smax))
    rx[:] = direct["shards"] * present[:, :, None]
    vout = gpu.pinned_empty((count, ctx.k * Smax))
    vout[:] = 0xCD
    res = ctx.interpolate_batch(rx, direct["shard_lens"], present, direct["roots"], values_out=vout)
    ref_res = ctx.interpolate_batch(np.array(rx), direct["shard_lens"], present, direct["roots"])
    assert (res["status"] == 0).all()
    assert np.array_equal(res["values"], ref_res["values"]) and np.array_equal(res["digests"], ref_res["digests"])
    for i, v in enumerate(values):
        assert res["values"][i, : len(v)].tobytes() == v.tobytes()


def test_host_api_errors_do_not_disturb_tickets_in_flight(gpu, ref):
    """Argument errors are returned at submit without touching the tickets in
    flight; per-instance failures (too few shards, wrong root, ragged lengths)
    come back as per-instance status of an otherwise good batch; every other
    ticket still lands bit-exact."""
    n, f = 16, 5
    k = n - 2 * f
    ctx = gpu.Context(n, f)
    rng = np.random.default_rng(55)
    B, count = 3000, 4
    S = (B + k - 1) // k
    vals = [rng.integers(0, 256, B, dtype=np.uint8) for _ in range(count)]
    want = [ref.encode_commit(n, f, v) for v in vals]
    t_ok = ctx.shard_commit_submit(vals)
    # an argument error at submit: a zero-length value (Split's ErrShortData)
    with pytest.raises(Exception) as ei:
        ctx.shard_commit_submit([vals[0], np.zeros(0, np.uint8)])
    assert getattr(ei.value, "code", None) == -6  # RBC_ERR_SHORT_DATA
    rx = np.zeros((count, n, S), np.uint8)
    present = np.zeros((count, n), np.uint8)
    roots = np.zeros((count, 32), np.uint8)
    for i in range(count):
        sh, root, _, _ = want[i]
        pres = rng.permutation(n)[: n - f]
        present[i, pres] = 1
        rx[i] = sh * present[i, :, None]
        roots[i] = np.frombuffer(root, np.uint8)
    present[1] = 0
    present[1, :k - 1] = 1           # instance 1: k-1 shards -> too few
    roots[2, 0] ^= 1                 # instance 2: wrong root -> root mismatch
    t_rx = ctx.interpolate_submit(rx, [S] * count, present, roots)
    t_ok2 = ctx.shard_commit_submit(vals[::-1])
    r_rx = t_rx.wait()
    st = r_rx["status"]
    assert st[0] == 0 and st[3] == 0
    assert st[1] == -3 and st[2] == -8, st  # RBC_ERR_TOO_FEW_SHARDS, RBC_ERR_ROOT_MISMATCH
    for i in (0, 3):
        assert r_rx["values"][i, :B].tobytes() == vals[i].tobytes()
    for t, vv in ((t_ok, vals), (t_ok2, vals[::-1])):
        r = t.wait()
        for i, v in enumerate(vv):
            assert bytes(r["roots"][i]) == ref.encode_commit(n, f, v)[1]


def test_host_api_randomized_interleaving(gpu, ref):
    """A seeded random mix of the host batch entry points (shard_commit,
    interpolate, shard_commit_val, validate_batch), pinned or pageable, with
    more tickets outstanding than slots and waits / polls in random order:
    every result equals the C oracle.  Exercises slot reuse and the deferred
    device-to-host copies under arbitrary orderings."""
    import random
    from cleisthenes_amd import protocol
    n, f = 16, 5
    k = n - 2 * f
    ctx = gpu.Context(n, f)
    rnd = random.Random(4242)
    rng = np.random.default_rng(4242)
    live = []  # (ticket, check)

    def alloc(shape, pinned):
        return gpu.pinned_empty(shape) if pinned else np.zeros(shape, np.uint8)

    for step in range(40):
        kind = rnd.choice(["commit", "interp", "val", "validate"])
        pinned = rnd.random() < 0.5
        count = rnd.randint(1, 5)
        B = rnd.choice([1, 7, 600, 4096, 6 * 1000 + 3])
        vals = []
        for _ in range(count):
            a = alloc(B, pinned)
            a[:] = rng.integers(0, 256, B, dtype=np.uint8)
            vals.append(a)
        want = [ref.encode_commit(n, f, v) for v in vals]
        if kind == "commit":
            t = ctx.shard_commit_submit(vals)

            def check(r, want=want):
                for i, (sh, root, br, _) in enumerate(want):
                    S = sh.shape[1]
                    assert np.array_equal(r["shards"][i, :, :S], sh) and bytes(r["roots"][i]) == root
        elif kind == "val":
            t = ctx.shard_commit_val_submit(vals)

            def check(r, want=want):
                for i, (sh, root, br, _) in enumerate(want):
                    j = rnd.randrange(n)
                    flat = b"".join(bytes(br[j, lvl]) for lvl in range(ctx.depth) if not (lvl == 0 and (j ^ 1) >= n))
                    assert r["message"](i, j) == protocol.pb_encode(protocol.VAL, protocol.json_encode_val(
                        root, flat, bytes(sh[j])))
        elif kind == "interp":
            S = want[0][0].shape[1]
            rx = alloc((count, n, S), pinned)
            present = np.zeros((count, n), np.uint8)
            roots = np.zeros((count, 32), np.uint8)
            for i, (sh, root, _, _) in enumerate(want):
                present[i, rng.permutation(n)[: rnd.randint(k, n)]] = 1
                rx[i] = sh * present[i, :, None]
                roots[i] = np.frombuffer(root, np.uint8)
            t = ctx.interpolate_submit(rx, [S] * count, present, roots,
                                       values_out=alloc((count, k * S), pinned) if pinned else None)

            def check(r, vals=vals, B=B):
                assert (r["status"] == 0).all()
                for i, v in enumerate(vals):
                    assert r["values"][i, :B].tobytes() == v.tobytes()
        else:
            sh, root, br, _ = want[0]
            js = [rnd.randrange(n) for _ in range(6)]
            shards = [bytes(sh[j]) for j in js]
            bad = rnd.randrange(6)
            shards[bad] = bytes([shards[bad][0] ^ 1]) + shards[bad][1:]
            flats = [b"".join(bytes(br[j, lvl]) for lvl in range(ctx.depth) if not (lvl == 0 and (j ^ 1) >= n))
                     for j in js]
            ok = ctx.validate_batch(shards, js, flats, [root] * 6)  # synchronous
            assert list(ok) == [i != bad for i in range(6)]
            continue
        live.append((t, check))
        # randomly complete some outstanding tickets, in random order
        while live and rnd.random() < 0.4:
            i = rnd.randrange(len(live))
            t, chk = live.pop(i)
            if rnd.random() < 0.5:
                t.done()
            chk(t.wait())
    rnd.shuffle(live)
    for t, chk in live:
        chk(t.wait())


@pytest.mark.parametrize("n,f,B,pad", [(16, 5, 6000, 0), (16, 5, 5999, 13), (128, 42, 1 << 20, 0),
                                        (256, 85, 64 << 10, 5), (4, 1, 1, 3)])
def test_host_interpolate_zero_copy_reads_present_rows_only(gpu, ref, n, f, B, pad):
    """A pinned, uniform-length receive batch is gathered on the device
    straight from host memory, present rows only: absent rows and the bytes
    of a row past S (a host pitch > S) hold garbage here and must not change
    status, value or digest -- equal to the C oracle on the zeroed input."""
    k = n - 2 * f
    S = (B + k - 1) // k
    count = 3
    ctx = gpu.Context(n, f)
    rng = np.random.default_rng(n + pad)
    rx = gpu.pinned_empty((count, n, S + pad))
    rx[:] = rng.integers(0, 256, rx.shape, dtype=np.uint8)  # garbage everywhere first
    present = np.zeros((count, n), np.uint8)
    roots = np.zeros((count, 32), np.uint8)
    clean = np.zeros((count, n, S), np.uint8)
    for i in range(count):
        v = rng.integers(0, 256, B, dtype=np.uint8)
        sh, root, _, _ = ref.encode_commit(n, f, v)
        roots[i] = np.frombuffer(root, np.uint8)
        pres = rng.permutation(n)[: n - f]
        present[i, pres] = 1
        rx[i, pres, :S] = sh[pres]
        clean[i] = sh * present[i, :, None]
    vout = gpu.pinned_empty((count, k * S))
    # the host row stride is S + pad; the lengths give S
    res = ctx.interpolate_submit(rx, [S] * count, present, roots, values_out=vout).wait()
    assert (res["status"] == 0).all()
    for i in range(count):
        rc, value, dig = ref.interpolate(n, f, clean[i], present[i], bytes(roots[i]))
        assert rc == 0 and np.array_equal(res["values"][i], value) and bytes(res["digests"][i]) == dig, i


REGEN_COUNTS = [
    # (n, f, S, missing data rows per instance, parity rows absent too):
    # gf_regen_kernel gives each 256-B (S <= 2048) or 512-B column tile to one
    # wave, which accumulates every missing row in passes of at most 40 / 24
    # rows (one body per exact row count), its block's 3 / 4 waves sharing the
    # LDS tables; the counts straddle every pass boundary of both forms, and a
    # last tile group with idle waves.  With parity rows absent as well, the
    # first-k set takes the first m present parity rows, not parity 0..m-1
    (256, 85, 763, [1, 3, 4, 5, 16, 17, 29, 39, 40, 41, 48, 64, 79, 80, 81, 86], False),
    (128, 42, 23832, [1, 4, 5, 11, 12, 13, 23, 24, 25, 44], False),
    (128, 42, 700, [1, 4, 16, 17, 32, 39, 40, 41, 44], False),
    (256, 85, 763, [1, 12, 13, 29, 40, 41, 86], True),
    (128, 42, 23832, [1, 12, 13, 24, 25, 44], True),
    (128, 42, 95326, [1, 12, 13, 24, 25, 44], True),  # C3's shard (4 MiB values)
    (64, 21, 47663, [1, 11, 12, 13, 22], True),       # C1's geometry and shard (1 MiB values)
]


@pytest.mark.parametrize("n,f,S,ms,parity_gone", REGEN_COUNTS,
                         ids=["n256-short", "n128-long", "n128-short", "n256-short-pgone", "c2-pgone", "c3-pgone",
                              "c1-pgone"])
def test_device_regen_missing_data_row_counts(gpu, n, f, S, ms, parity_gone):
    """Interpolate with exactly m missing data rows per instance (and, with
    parity_gone, a random set of absent parity rows that still leaves >= m):
    every absent row holds garbage (poisoned), so only the regeneration can
    restore it; each regenerated row -- data and parity -- equals the committed
    one, zero past S, and the value is the input.  One-shot interpolate and
    the receive step, on the same inputs."""
    k = n - 2 * f
    p = n - k
    I = len(ms)
    for mode in ("oneshot", "step"):
        pl = Pipeline(gpu, n, f, k * S, I, seed=n + S, corrupt_frac=0.0)
        rng = np.random.default_rng(S + parity_gone)
        pl.present[:] = 1
        for i, m in enumerate(ms):
            pl.present[i, rng.permutation(k)[:m]] = 0
            if parity_gone:
                gone = int(rng.integers(1, p - m + 1))
                pl.present[i, k + rng.permutation(p)[:gone]] = 0
        pl.b["present"].upload(pl.present)
        pl.commit()
        committed = pl.shards().copy()
        pl.poison(seed=S)
        pl.assert_poisoned(committed, sample=I)
        pl.receive(poison=False) if mode == "oneshot" else pl.receive_step(poison=False)
        assert (pl.arr("status", np.int32) == 0).all(), mode
        out = pl.arr("out", shape=(I, pl.opitch))
        assert np.array_equal(out[:, : pl.B], pl.values[:, : pl.B]), mode
        after = pl.shards()
        for i, m in enumerate(ms):
            miss = np.flatnonzero(pl.present[i, :k] == 0)
            assert len(miss) == m
            assert np.array_equal(after[i], committed[i]), (mode, i, m)  # every row, data and parity
            assert not after[i][:, S:].any(), (mode, i, m)


@pytest.mark.parametrize("S", [763, 100, 1400, 1500, 2000, 2049, 3000])
def test_device_interpolate_short_rows(gpu, S):
    """Missing-data GF rows for short shards (256-B column tiles up to S =
    2048, C4's S = 763 in 3; 512-B above), including last tile groups whose
    waves have no tile (S = 2000: 8 tiles in blocks of 3; S = 2049: 5 in
    blocks of 4) and lanes past the row pitch: interpolate returns the value
    and rewrites every regenerated row exactly as committed, zero past S."""
    n, f, I = 256, 85, 6
    k = n - 2 * f
    pl = Pipeline(gpu, n, f, k * S, I, seed=S, corrupt_frac=0.3)
    pl.commit()
    committed = pl.shards().copy()
    pl.receive()
    assert (pl.arr("status", np.int32) == 0).all()
    out = pl.arr("out", shape=(I, pl.opitch))
    assert np.array_equal(out[:, : pl.B], pl.values[:, : pl.B])
    after = pl.shards()
    for i in range(I):
        ok = pl.present[i].astype(bool)
        if pl.corrupt[i] >= 0:
            ok[pl.corrupt[i]] = False  # verify rejected it, interpolate regenerated it
        regen = ~ok
        assert np.array_equal(after[i][regen], committed[i][regen]), i


@pytest.mark.parametrize("n,f", [(16, 5), (256, 85)])
def test_device_verify_ragged_lengths(gpu, ref, n, f):
    """rbc_dev_verify with per-instance shard lengths (the shared-path kernel
    runs whenever lengths are ragged): a ragged batch committed through the
    host API, a few shards / branch slots corrupted, valid[] and the leaves
    against the oracle walk."""
    ctx = gpu.Context(n, f)
    k, d = ctx.k, ctx.depth
    rng = np.random.default_rng(n + 17)
    lens = [1, k, 3 * k + 1, 50 * k, 7, 200 * k + 5]
    values = [rng.integers(0, 256, L, dtype=np.uint8) for L in lens]
    out = ctx.shard_commit_batch(values)
    I, Smax = len(values), out["shards"].shape[2]
    pitch = rup(Smax, 64)
    sh = np.zeros((I, n, pitch), np.uint8)
    sh[:, :, :Smax] = out["shards"]
    brs = np.ascontiguousarray(out["branches"])
    roots = out["roots"].copy()
    for i in range(I):
        sh[i, rng.integers(n), rng.integers(int(out["shard_lens"][i]))] ^= 0x40
        brs[i, rng.integers(n), rng.integers(d), rng.integers(32)] ^= 2
    mb = gpu.DeviceBuffer
    b = dict(sh=mb(sh.nbytes), br=mb(brs.nbytes), rt=mb(roots.nbytes), ln=mb(4 * I), va=mb(I * n),
             lv=mb(I * n * 32))
    b["sh"].upload(sh)
    b["br"].upload(brs)
    b["rt"].upload(roots)
    b["ln"].upload(out["shard_lens"].astype(np.uint32))
    ctx.dev_verify(None, I, b["sh"], pitch, b["ln"], 0, b["br"], b["rt"], None, b["va"], b["lv"])
    got = np.frombuffer(b["va"].download().tobytes(), np.uint8).reshape(I, n)
    leaves = np.frombuffer(b["lv"].download().tobytes(), np.uint8).reshape(I, n, 32)
    for i in range(I):
        S = int(out["shard_lens"][i])
        for j in range(n):
            want = ref.verify(n, sh[i, j, :S], j, brs[i, j], bytes(roots[i]))
            assert got[i, j] == int(want), (i, j)
            assert leaves[i, j].tobytes() == ref.sha256(sh[i, j, :S].tobytes())
        assert 1 <= (got[i] == 0).sum() <= 2


# every tree depth 1..8 (W = 2..256), non-power-of-two N, and an odd instance
# count so the last merkle block holds fewer trees than trees_per_block: the
# branch-write loop steps (j, l) by (32 / d, 32 % d) with a carry, so each
# depth exercises a different stepping
@pytest.mark.gpu
@pytest.mark.parametrize("n,f", [(2, 0), (3, 1), (6, 1), (11, 3), (17, 5), (32, 10), (33, 10), (100, 33),
                                 (129, 42), (256, 85)])
def test_merkle_build_branches_every_depth(gpu, ref, n, f):
    k = n - 2 * f
    B = 37 * k + 5
    I = 5
    pl = Pipeline(gpu, n, f, B, I, seed=4242 + n)
    pl.commit()
    roots = pl.arr("roots", shape=(I, 32))
    brs = pl.arr("branches", shape=(I, n, max(pl.d, 1), 32))
    for i in range(I):
        _, want_root, want_br, _ = ref.encode_commit(n, f, pl.values[i, :B])
        assert bytes(roots[i]) == want_root, (n, i)
        assert np.array_equal(brs[i], want_br), (n, i)


@pytest.mark.parametrize("n,f,B,I,all_present", [(128, 42, 1 << 16, 96, False), (16, 5, 3001, 64, False),
                                                  (256, 85, 86 * 40, 48, False), (64, 21, 22 * 700, 40, True),
                                                  (7, 2, 1000, 33, False)])
@pytest.mark.parametrize("clobber", [False, True], ids=["", "released-set-clobbered"])
def test_receive_step_pipeline_equals_verify_then_interpolate(gpu, ref, n, f, B, I, all_present, clobber):
    """rbc_dev_receive_step over three batches (verify(t) + rehash(t-1) in
    one SHA launch, recheck(t-1), decode(t), join on the aux stream, a final
    flush) yields exactly rbc_dev_verify + rbc_dev_interpolate(leaves_verified
    = 1) per batch: valid masks, statuses, values, digests and leaves, with
    corrupted ECHO shards, wrong committed roots and (all_present) no present
    mask; the C4 shape takes the shared-path verify inside the step.  With
    clobber, a second stream waits for each call's prev_released mark and
    then overwrites prev's shards, branches and roots with garbage while the
    call's decode of cur runs: nothing of prev may be read after the mark.
    Sampled instances are also checked against the C oracle."""
    nb = 3
    want, got = [], []
    for mode in ("oneshot", "step"):
        pls = []
        for bi in range(nb):
            pl = Pipeline(gpu, n, f, B, I, seed=1000 * n + 17 * bi + B, corrupt_frac=0.3)
            b, c = pl.b, pl.ctx
            c.dev_encode(None, I, b["values"], pl.vpitch, None, B, b["shards"], pl.spitch)
            # a Byzantine proposer commits to a non-codeword every 7th instance
            # (last row altered before the Merkle build: every branch verifies,
            # interpolate's full re-encode must reject it)
            byz = np.full(I, -1, np.int32)
            byz[bi::7] = n - 1
            d_byz = gpu.DeviceBuffer(I * 4)
            d_byz.upload(byz)
            c.dev_inject_faults(None, I, b["shards"], pl.spitch, d_byz)
            c.dev_leaves(None, I, b["shards"], pl.spitch, None, pl.S, b["leaves"])
            c.dev_merkle_build(None, I, b["leaves"], b["roots"], b["branches"])
            pl.poison(seed=bi, present=not all_present)  # absent + corrupted rows: garbage
            c.dev_inject_faults(None, I, b["shards"], pl.spitch, b["corrupt"])
            pls.append(pl)
        present = (lambda pl: None) if all_present else (lambda pl: pl.b["present"])
        if mode == "oneshot":
            for pl in pls:
                b, c = pl.b, pl.ctx
                c.dev_verify(None, I, b["shards"], pl.spitch, None, pl.S, b["branches"], b["roots"], present(pl),
                             b["valid"], b["leaves_r"])
                c.dev_interpolate(None, I, b["shards"], pl.spitch, None, pl.S, b["valid"], b["leaves_r"], 1,
                                  b["roots"], b["out"], pl.opitch, b["digests"], b["status"])
        else:
            rx = gpu.Context(n, f)
            st = gpu.Stream(0)
            bs = [rx.rx_batch(I, pl.b["shards"], pl.spitch, None, pl.S, pl.b["branches"], pl.b["roots"],
                              present(pl), pl.b["valid"], pl.b["leaves_r"], pl.b["out"], pl.opitch,
                              pl.b["digests"], pl.b["status"]) for pl in pls]
            prev = None
            cl = gpu.Stream(0)
            for cur in bs + [None]:
                if clobber and prev is not None:
                    rel = gpu.Event()
                    rx.dev_receive_step(st.ptr, cur, prev, prev_released=rel)
                    cl.wait(rel)  # prev's set is the producer's again: refill it with garbage
                    pp = pls[[id(b_) for b_ in bs].index(id(prev))]
                    gpu.rbc.fill_random(0, cl.ptr, pp.b["shards"], 0, I, n * pp.spitch, 99)
                    gpu.rbc.fill_random(0, cl.ptr, pp.b["branches"], 0, I, n * max(pp.d, 1) * 32, 98)
                    gpu.rbc.fill_random(0, cl.ptr, pp.b["roots"], 0, I, 32, 97)
                else:
                    rx.dev_receive_step(st.ptr, cur, prev)
                if cur is not None and prev is None:  # a batch is pending: interpolate must refuse
                    pl = pls[0]
                    with pytest.raises(gpu.RBCError):
                        rx.dev_interpolate(st.ptr, I, pl.b["shards"], pl.spitch, None, pl.S, pl.b["valid"],
                                           pl.b["leaves_r"], 1, pl.b["roots"], pl.b["out"], pl.opitch,
                                           pl.b["digests"], pl.b["status"])
                prev = cur
            with pytest.raises(gpu.RBCError):  # prev must be the last call's cur
                rx.dev_receive_step(st.ptr, None, bs[0])
            st.sync()
            cl.sync()
        gpu.rbc.lib.rbc_device_sync(0)
        res = []
        for pl in pls:
            stt = pl.arr("status", np.int32)
            ok = stt == 0
            res.append((stt, pl.arr("valid", shape=(I, n)), pl.arr("out", shape=(I, pl.opitch))[:, : pl.k * pl.S][ok],
                        pl.arr("digests", shape=(I, 32))[ok], pl.arr("leaves_r", shape=(I, n, 32))[ok], pl))
        (want if mode == "oneshot" else got).append(res)
    for bi in range(nb):
        (s0, v0, o0, d0, l0, _), (s1, v1, o1, d1, l1, pl) = want[0][bi], got[0][bi]
        assert np.array_equal(s0, s1), bi
        assert set(s1[bi::7]) == {-8} and (s1[np.arange(I) % 7 != bi] == 0).all(), bi
        pr = np.ones((I, n), bool) if all_present else pl.present.astype(bool)
        assert np.array_equal(v0[pr], v1[pr]) and not v1[~pr].any(), bi
        assert np.array_equal(o0, o1) and np.array_equal(d0, d1) and np.array_equal(l0, l1), bi
        ok = np.flatnonzero(s1 == 0)
        for i in (ok[0], ok[-1]):
            assert bytes(pl.values[i, :B]) == bytes(o1[np.searchsorted(ok, i)][:B])


@pytest.mark.parametrize("n,f,B,I", [(128, 42, 1 << 16, 96), (16, 5, 3001, 64), (256, 85, 86 * 40, 48)])
def test_row_view_interpolate_equals_joined_value(gpu, ref, n, f, B, I):
    """interpolate with values_out = NULL (the row view: no join) leaves the
    same statuses, digests and leaves as the joined form, and its k data rows
    ARE the joined value (rbc_dev_count_mismatch_rows finds no difference;
    the host compares them too); wrong committed roots and corrupted ECHOs
    included.  The receive step's row view gives the same."""
    outs = []
    for mode in ("joined", "view", "step_view"):
        pl = Pipeline(gpu, n, f, B, I, seed=n + B, corrupt_frac=0.3)
        pl.commit()
        pl.poison()
        b, c = pl.b, pl.ctx
        c.dev_inject_faults(None, I, b["shards"], pl.spitch, b["corrupt"])
        roots = pl.arr("roots", shape=(I, 32)).copy()
        roots[::7, 0] ^= 0x80  # after the verify: the recheck against a wrong root every 7th instance
        if mode == "step_view":
            rb = c.rx_batch(I, b["shards"], pl.spitch, None, pl.S, b["branches"], b["roots"], b["present"],
                            b["valid"], b["leaves_r"], None, 0, b["digests"], b["status"])
            c.dev_receive_step(None, rb, None)  # verify + decode
            gpu.rbc.lib.rbc_device_sync(0)
            b["roots"].upload(roots)
            c.dev_receive_step(None, None, rb)  # rehash + recheck
        else:
            c.dev_verify(None, I, b["shards"], pl.spitch, None, pl.S, b["branches"], b["roots"], b["present"],
                         b["valid"], b["leaves_r"])
            gpu.rbc.lib.rbc_device_sync(0)
            b["roots"].upload(roots)
            c.dev_interpolate(None, I, b["shards"], pl.spitch, None, pl.S, b["valid"], b["leaves_r"], 1, b["roots"],
                              b["out"] if mode == "joined" else None, pl.opitch if mode == "joined" else 0,
                              b["digests"], b["status"])
        cnt = gpu.DeviceBuffer(16)
        gpu.rbc.count_mismatch_rows(0, None, b["shards"], pl.n * pl.spitch, pl.spitch, pl.k, pl.S, b["values"],
                                    pl.vpitch, B, I, cnt)
        gpu.rbc.lib.rbc_device_sync(0)
        st = pl.arr("status", np.int32)
        ok = st == 0
        rows = pl.shards()[:, : pl.k, : pl.S].reshape(I, pl.k * pl.S)
        outs.append((st, rows[ok], pl.arr("digests", shape=(I, 32))[ok], pl.arr("leaves_r", shape=(I, n, 32))[ok],
                     pl.arr("out", shape=(I, pl.opitch))[:, : pl.k * pl.S][ok], pl, int(cnt.download(4).view(np.uint32)[0])))
    (s0, r0, d0, l0, v0, _, mism0), = outs[:1]
    assert set(s0[::7]) == {-8} and (s0[np.arange(I) % 7 != 0] == 0).all()
    assert np.array_equal(r0, v0)  # the joined value is the data rows
    for (s1, r1, d1, l1, _, pl1, mism) in outs:
        assert np.array_equal(s0, s1) and np.array_equal(r0, r1) and np.array_equal(d0, d1)
        assert np.array_equal(l0, l1)
        ok = np.flatnonzero(s1 == 0)
        assert all(bytes(pl1.values[i, :B]) == bytes(r1[t, :B]) for t, i in enumerate(ok))
        # the decode ran on every instance (the wrong roots fail only the recheck afterwards),
        # so every instance's data rows are its input with the Split pad
        assert mism == 0


def test_count_mismatch_rows_finds_single_byte_differences(gpu):
    """The bench guard's row-view check: a value split into k rows (zero pad
    past B) compares equal to its rows, and one flipped byte in a data row,
    in the pad or at the last valid byte is one mismatching chunk."""
    n, f, B, I = 16, 5, 1001, 6
    k = n - 2 * f
    S = (B + k - 1) // k
    spitch, vpitch = rup(S, 64), rup(k * S + 32, 64)
    rng = np.random.default_rng(3)
    values = rng.integers(0, 256, (I, vpitch), dtype=np.uint8)
    rows = np.zeros((I, n, spitch), np.uint8)
    for i in range(I):
        v = np.zeros(k * S, np.uint8)
        v[:B] = values[i, :B]
        rows[i, :k, :S] = v.reshape(k, S)
    for i, (j, x) in {1: (0, 0), 2: (k - 1, S - 1), 3: (3, 17), 5: ((B - 1) // S, (B - 1) % S)}.items():
        rows[i, j, x] ^= 0x40
    d_rows, d_vals, cnt = gpu.DeviceBuffer(rows.nbytes), gpu.DeviceBuffer(values.nbytes), gpu.DeviceBuffer(16)
    d_rows.upload(rows)
    d_vals.upload(values)
    gpu.rbc.count_mismatch_rows(0, None, d_rows, n * spitch, spitch, k, S, d_vals, vpitch, B, I, cnt)
    gpu.rbc.lib.rbc_device_sync(0)
    assert int(cnt.download(4).view(np.uint32)[0]) == 4


def test_receive_step_rejects_aliased_batches(gpu, ref):
    """cur and prev sharing an output buffer (leaves, status, valid, values,
    digests) is rejected before any work, as is a cur that fails its argument
    checks; prev then stays pending and a later call completes it with the
    statuses, values and digests of verify + interpolate."""
    n, f, B, I = 16, 5, 2000, 24
    pls = []
    for bi in range(2):
        pl = Pipeline(gpu, n, f, B, I, seed=77 + bi, corrupt_frac=0.3)
        pl.commit()
        pl.poison()
        pl.ctx.dev_inject_faults(None, I, pl.b["shards"], pl.spitch, pl.b["corrupt"])
        pls.append(pl)
    rx = gpu.Context(n, f)

    def rb(pl, **over):
        b = dict(pl.b, **over)
        return rx.rx_batch(I, b["shards"], pl.spitch, None, pl.S, b["branches"], b["roots"], b["present"], b["valid"],
                           b["leaves_r"], b["out"], pl.opitch, b["digests"], b["status"])
    p0 = rb(pls[0])
    rx.dev_receive_step(None, p0, None)
    for key in ("leaves_r", "status", "valid", "out", "digests"):
        with pytest.raises(gpu.RBCError):
            rx.dev_receive_step(None, rb(pls[1], **{key: pls[0].b[key]}), p0)
    bad = rb(pls[1])
    bad.uniform_shard_len = pls[1].spitch + 64  # > shard_pitch: rejected by cur's checks before any launch
    with pytest.raises(gpu.RBCError):
        rx.dev_receive_step(None, bad, p0)
    rx.dev_receive_step(None, None, p0)  # prev still pending: complete it
    gpu.rbc.lib.rbc_device_sync(0)
    want = Pipeline(gpu, n, f, B, I, seed=77, corrupt_frac=0.3)
    want.commit()
    want.receive()
    gpu.rbc.lib.rbc_device_sync(0)
    for name in ("status", "digests", "valid"):
        assert np.array_equal(want.arr(name), pls[0].arr(name)), name
    ok = want.arr("status", np.int32) == 0
    assert np.array_equal(want.arr("out", shape=(I, want.opitch))[ok], pls[0].arr("out", shape=(I, want.opitch))[ok])


def test_wave_priority_changes_no_result(gpu, ref):
    """rbc_ctx_set_wave_priority / rbc_ctx_set_decode_priority only reorder
    issue on the SIMDs: commit and receive at 0/0 and 3/3, the bench's 0/2 with
    the GEMV at the receive level, and mixed levels give identical shards,
    roots, branches, valid masks, values, digests and statuses; a level outside
    0..3 (-1 allowed for the decode levels) is rejected."""
    n, f, B, I = 128, 42, 1 << 16, 64
    outs = []
    for tx, rx, gv, rv in ((0, 0, -1, -1), (3, 3, -1, -1), (0, 2, 2, -1), (1, 0, 3, 2)):
        pl = Pipeline(gpu, n, f, B, I, seed=4242, corrupt_frac=0.3)
        pl.ctx.set_wave_priority(tx, rx)
        pl.ctx.set_decode_priority(gv, rv)
        pl.commit()
        pl.receive()
        gpu.rbc.lib.rbc_device_sync(0)
        outs.append([pl.arr(k) for k in ("shards", "roots", "branches", "valid", "out", "digests", "status",
                                          "leaves_r")])
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert np.array_equal(a, b)
    for bad in ((4, 0), (0, -1)):
        with pytest.raises(gpu.RBCError):
            pl.ctx.set_wave_priority(*bad)
    for bad in ((4, 0), (0, -2)):
        with pytest.raises(gpu.RBCError):
            pl.ctx.set_decode_priority(*bad)


@pytest.mark.parametrize("n,f", [(16, 5), (256, 85)])
def test_receive_step_ragged_lengths_and_too_few_shards(gpu, ref, n, f):
    """rbc_dev_receive_step with per-instance shard lengths (ragged batch from
    the host shard+commit API), instances with only k-1 received shards
    (TOO_FEW_SHARDS) and corrupted ECHOs: two batches through the receive step
    equal rbc_dev_verify + rbc_dev_interpolate on copies of the same inputs;
    every decoded value equals its input."""
    ctx = gpu.Context(n, f)
    k = ctx.k
    rng = np.random.default_rng(n + 99)
    lens = [1, k, 3 * k + 1, 50 * k, 7, 200 * k + 5, 64 * k, 5 * k + 3, 1000]
    I = len(lens)
    mb = gpu.DeviceBuffer
    batches = []
    for bi in range(2):
        values = [rng.integers(0, 256, L, dtype=np.uint8) for L in lens]
        out = ctx.shard_commit_batch(values)
        Smax = out["shards"].shape[2]
        pitch = rup(Smax, 64)
        opitch = rup(k * Smax, 16)
        sh = np.zeros((I, n, pitch), np.uint8)
        sh[:, :, :Smax] = out["shards"]
        present = np.zeros((I, n), np.uint8)
        for i in range(I):
            cnt = k - 1 if i % 4 == bi + 1 else n - f
            pres = rng.permutation(n)[:cnt]
            present[i, pres] = 1
            if i % 3 == 0:
                sh[i, pres[0], rng.integers(int(out["shard_lens"][i]))] ^= 0x21
            # every absent row holds garbage across the whole pitch: only the decode can restore it
            gone = np.flatnonzero(present[i] == 0)
            sh[i, gone] = rng.integers(0, 256, (len(gone), pitch), dtype=np.uint8)
        batches.append(dict(values=values, out=out, sh=sh, present=present, pitch=pitch, opitch=opitch))
    res = {}
    for mode in ("oneshot", "step"):
        c = gpu.Context(n, f)
        bufs = []
        for bt in batches:
            d = dict(sh=mb(bt["sh"].nbytes), br=mb(bt["out"]["branches"].nbytes), rt=mb(I * 32), ln=mb(4 * I),
                     pr=mb(I * n), va=mb(I * n), lv=mb(I * n * 32), vo=mb(I * bt["opitch"]), dg=mb(I * 32),
                     st=mb(4 * I))
            d["sh"].upload(bt["sh"])
            d["br"].upload(np.ascontiguousarray(bt["out"]["branches"]))
            d["rt"].upload(bt["out"]["roots"])
            d["ln"].upload(bt["out"]["shard_lens"].astype(np.uint32))
            d["pr"].upload(bt["present"])
            bufs.append(d)
        if mode == "oneshot":
            for bt, d in zip(batches, bufs):
                c.dev_verify(None, I, d["sh"], bt["pitch"], d["ln"], 0, d["br"], d["rt"], d["pr"], d["va"], d["lv"])
                c.dev_interpolate(None, I, d["sh"], bt["pitch"], d["ln"], 0, d["va"], d["lv"], 1, d["rt"], d["vo"],
                                  bt["opitch"], d["dg"], d["st"])
        else:
            rbs = [c.rx_batch(I, d["sh"], bt["pitch"], d["ln"], 0, d["br"], d["rt"], d["pr"], d["va"], d["lv"],
                              d["vo"], bt["opitch"], d["dg"], d["st"]) for bt, d in zip(batches, bufs)]
            c.dev_receive_step(None, rbs[0], None)
            c.dev_receive_step(None, rbs[1], rbs[0])
            c.dev_receive_step(None, None, rbs[1])
        gpu.rbc.lib.rbc_device_sync(0)
        res[mode] = [(np.frombuffer(d["st"].download().tobytes(), np.int32).copy(),
                      np.frombuffer(d["va"].download().tobytes(), np.uint8).reshape(I, n).copy(),
                      np.frombuffer(d["vo"].download().tobytes(), np.uint8).reshape(I, bt["opitch"]).copy(),
                      np.frombuffer(d["dg"].download().tobytes(), np.uint8).reshape(I, 32).copy())
                     for bt, d in zip(batches, bufs)]
    for bi, bt in enumerate(batches):
        (s0, v0, o0, g0), (s1, v1, o1, g1) = res["oneshot"][bi], res["step"][bi]
        assert np.array_equal(s0, s1) and np.array_equal(v0, v1), bi
        for i in range(I):
            if i % 4 == bi + 1:
                assert s1[i] == -3, (bi, i)  # TOO_FEW_SHARDS
                continue
            assert s1[i] == 0, (bi, i)
            L = lens[i]
            assert bytes(o1[i, :L]) == bytes(bt["values"][i]) and np.array_equal(o0[i, :L], o1[i, :L])
            assert np.array_equal(g0[i], g1[i])


def test_receive_step_batches_of_different_sizes(gpu, ref):
    """Consecutive receive steps on batches of 40, 17 and 33 instances (the
    hashing launch covers cur's and prev's counts separately) give the same
    statuses, values and digests as verify + interpolate."""
    n, f, B = 16, 5, 2000
    sizes = [40, 17, 33]
    res = {}
    for mode in ("oneshot", "step"):
        pls = []
        for bi, I in enumerate(sizes):
            pl = Pipeline(gpu, n, f, B, I, seed=555 + bi, corrupt_frac=0.3)
            pl.commit()
            pl.poison(seed=bi)
            pl.ctx.dev_inject_faults(None, I, pl.b["shards"], pl.spitch, pl.b["corrupt"])
            pls.append(pl)
        if mode == "oneshot":
            for pl in pls:
                b, c, I = pl.b, pl.ctx, pl.I
                c.dev_verify(None, I, b["shards"], pl.spitch, None, pl.S, b["branches"], b["roots"], b["present"],
                             b["valid"], b["leaves_r"])
                c.dev_interpolate(None, I, b["shards"], pl.spitch, None, pl.S, b["valid"], b["leaves_r"], 1,
                                  b["roots"], b["out"], pl.opitch, b["digests"], b["status"])
        else:
            rx = gpu.Context(n, f)
            bs = [rx.rx_batch(pl.I, pl.b["shards"], pl.spitch, None, pl.S, pl.b["branches"], pl.b["roots"],
                              pl.b["present"], pl.b["valid"], pl.b["leaves_r"], pl.b["out"], pl.opitch,
                              pl.b["digests"], pl.b["status"]) for pl in pls]
            prev = None
            for cur in bs + [None]:
                rx.dev_receive_step(None, cur, prev)
                prev = cur
        gpu.rbc.lib.rbc_device_sync(0)
        res[mode] = [(pl.arr("status", np.int32).copy(), pl.arr("out", shape=(pl.I, pl.opitch)).copy(),
                      pl.arr("digests", shape=(pl.I, 32)).copy(), pl) for pl in pls]
    for (s0, o0, d0, _), (s1, o1, d1, pl) in zip(res["oneshot"], res["step"]):
        assert (s0 == 0).all() and np.array_equal(s0, s1)
        assert np.array_equal(o0[:, : pl.k * pl.S], o1[:, : pl.k * pl.S]) and np.array_equal(d0, d1)
        assert all(bytes(pl.values[i, :B]) == bytes(o1[i, :B]) for i in range(pl.I))


RECHECK_GEOMS = [(7, 2, 1000, 40), (16, 5, 3001, 48), (33, 10, 13 * 50 + 3, 40), (64, 21, 22 * 300, 40),
                 (128, 42, 44 * 200, 48), (256, 85, 86 * 40, 48)]


@pytest.mark.parametrize("n,f,B,I", RECHECK_GEOMS, ids=[f"n{g[0]}" for g in RECHECK_GEOMS])
def test_receive_step_node_reuse_recheck_equals_full_recheck(gpu, ref, n, f, B, I):
    """rbc_dev_receive_step's root recheck over the nodes ECHO verify
    established (RBC_RECHECK_REUSE: hash only the subtrees that hold no valid
    leaf, compare their roots with a valid leaf's branch) against the whole-
    tree recheck (RBC_RECHECK_FULL) and one-shot verify + interpolate, on the
    same three batches: statuses, valid masks, digests, leaves, values and the
    regenerated shard sets are identical.  Inputs per instance: honest with
    random, data-only, parity-heavy and all-present ECHO sets; corrupted
    shards; a corrupted branch slot at every level (the leaf is invalid, its
    siblings' anchors are not); a Byzantine non-codeword commitment (a valid
    unused row the re-encoding changes: the full-recheck fallback, or a
    regenerated row that misses its anchor); wrong roots written after the
    verify (the copy of the verified roots must disagree)."""
    k = n - 2 * f
    d = max(1, (n - 1).bit_length())
    nb = 3

    def make_batches():
        pls, plan = [], []
        for bi in range(nb):
            rng = np.random.default_rng(7000 + 31 * n + bi)
            pl = Pipeline(gpu, n, f, B, I, seed=900 * n + bi, corrupt_frac=0.0)
            kind = [rng.integers(0, 7) for _ in range(I)]
            byz = np.full(I, -1, np.int32)
            for i, kd in enumerate(kind):
                if kd == 3:
                    pl.present[i] = 0
                    pl.present[i, :k] = 1                    # data rows only
                elif kd == 4:
                    pl.present[i] = 0
                    pl.present[i, rng.permutation(n)[:k]] = 1  # exactly k
                elif kd == 5:
                    pl.present[i] = 1                        # everything received
                if kd == 6 and n > k:
                    byz[i] = int(rng.integers(k, n))          # non-codeword: a parity row altered before the tree
            pl.b["present"].upload(pl.present)
            b, c = pl.b, pl.ctx
            c.dev_encode(None, I, b["values"], pl.vpitch, None, B, b["shards"], pl.spitch)
            d_byz = gpu.DeviceBuffer(I * 4)
            d_byz.upload(byz)
            c.dev_inject_faults(None, I, b["shards"], pl.spitch, d_byz)
            c.dev_leaves(None, I, b["shards"], pl.spitch, None, pl.S, b["leaves"])
            c.dev_merkle_build(None, I, b["leaves"], b["roots"], b["branches"])
            gpu.rbc.lib.rbc_device_sync(0)
            sh = pl.shards().copy()
            brs = pl.arr("branches", shape=(I, n, d, 32)).copy()
            for i, kd in enumerate(kind):
                pres = np.flatnonzero(pl.present[i])
                if kd == 1:   # a corrupted received shard
                    sh[i, pres[rng.integers(len(pres))], rng.integers(pl.S)] ^= 0x10
                elif kd == 2:  # a corrupted branch slot of a received leaf, at every level in turn
                    j = pres[rng.integers(len(pres))]
                    lvl = i % d
                    if not (lvl == 0 and (j ^ 1) >= n):
                        brs[i, j, lvl, rng.integers(32)] ^= 0x04
            # absent rows hold garbage
            for i in range(I):
                gone = np.flatnonzero(pl.present[i] == 0)
                sh[i, gone] = rng.integers(0, 256, (len(gone), pl.spitch), dtype=np.uint8)
            b["shards"].upload(sh)
            b["branches"].upload(brs)
            pls.append(pl)
            plan.append(kind)
        return pls, plan

    def run(mode):
        pls, plan = make_batches()
        if mode == "oneshot":
            for pl in pls:
                b, c = pl.b, pl.ctx
                c.dev_verify(None, I, b["shards"], pl.spitch, None, pl.S, b["branches"], b["roots"], b["present"],
                             b["valid"], b["leaves_r"])
                gpu.rbc.lib.rbc_device_sync(0)
                wrong = pl.arr("roots", shape=(I, 32)).copy()
                wrong[5::11, 3] ^= 0x01
                b["roots"].upload(wrong)
                c.dev_interpolate(None, I, b["shards"], pl.spitch, None, pl.S, b["valid"], b["leaves_r"], 1,
                                  b["roots"], b["out"], pl.opitch, b["digests"], b["status"])
        else:
            rx = gpu.Context(n, f)
            rx.set_recheck(mode)
            bs = [rx.rx_batch(I, pl.b["shards"], pl.spitch, None, pl.S, pl.b["branches"], pl.b["roots"],
                              pl.b["present"], pl.b["valid"], pl.b["leaves_r"], pl.b["out"], pl.opitch,
                              pl.b["digests"], pl.b["status"]) for pl in pls]
            prev = None
            for bi, cur in enumerate(bs + [None]):
                rx.dev_receive_step(None, cur, prev)
                gpu.rbc.lib.rbc_device_sync(0)
                if cur is not None:  # after cur's verify, before its recheck in the next call
                    pl = pls[bi]
                    wrong = pl.arr("roots", shape=(I, 32)).copy()
                    wrong[5::11, 3] ^= 0x01
                    pl.b["roots"].upload(wrong)
                prev = cur
        gpu.rbc.lib.rbc_device_sync(0)
        out = []
        for pl in pls:
            st = pl.arr("status", np.int32).copy()
            ok = st == 0
            out.append(dict(status=st, valid=pl.arr("valid", shape=(I, n)).copy(),
                            digests=pl.arr("digests", shape=(I, 32))[ok].copy(),
                            leaves=pl.arr("leaves_r", shape=(I, n, 32))[ok].copy(),
                            out=pl.arr("out", shape=(I, pl.opitch))[ok, : pl.k * pl.S].copy(),
                            shards=pl.shards()[ok].copy(), present=pl.present.copy(), values=pl.values))
        return out, plan

    res = {m: run(m) for m in ("oneshot", "full", "reuse")}
    plan = res["reuse"][1]
    for bi in range(nb):
        a, b_, c_ = res["oneshot"][0][bi], res["full"][0][bi], res["reuse"][0][bi]
        pr = c_["present"].astype(bool)
        for key in ("status", "digests", "leaves", "out", "shards"):
            assert np.array_equal(a[key], c_[key]) and np.array_equal(b_[key], c_[key]), (bi, key)
        assert np.array_equal(a["valid"][pr], c_["valid"][pr]) and np.array_equal(b_["valid"], c_["valid"]), bi
        st, kind = c_["status"], np.array(plan[bi])
        assert (st[5::11] == -8).all(), bi  # the roots changed after the verify
        assert (st[kind == 6][(np.arange(I)[kind == 6] % 11) != 5] == -8).all() or n == k, bi  # non-codeword
        honest = (kind != 6) & (np.arange(I) % 11 != 5)
        assert (st[honest] == 0).all(), (bi, st[honest])
        for t, i in enumerate(np.flatnonzero(st == 0)):
            assert bytes(c_["out"][t][:B]) == bytes(c_["values"][i, :B])


def _padding_nodes_with_real_sibling(n):
    """(heap index, level, first and end leaf under its sibling) of every
    all-padding node at levels 1 .. d-1 whose sibling holds a real leaf."""
    W, d = orc.tree_width(n), orc.tree_depth(n)
    out = []
    for lvl in range(1, d):
        m = W >> lvl
        for i in range(m, 2 * m):
            lo = ((i ^ 1) << lvl) - W
            if ((i - m) << lvl) >= n and lo < n:
                out.append((i, lvl, lo, min(n, lo + (1 << lvl))))
    return out


@pytest.mark.parametrize("n,f,B,I", [(33, 10, 13 * 40 + 1, 48), (100, 33, 34 * 60 + 7, 48)], ids=["n33", "n100"])
def test_receive_step_rejects_a_byzantine_padding_node(gpu, n, f, B, I):
    """a Byzantine proposer commits to a tree whose padding
    node at level >= 1 is a value of its choosing.  Every ECHO verifies (the
    walk takes that node from the branch), the full recheck rebuilds standard
    padding and rejects the root.  The node-reuse recheck must reject it too,
    both when a valid leaf sits under the padding node's parent and when none
    does; honest instances of the same batches still deliver.  One-shot, FULL
    and REUSE give identical statuses."""
    k = n - 2 * f
    W, d = orc.tree_width(n), orc.tree_depth(n)
    pads = _padding_nodes_with_real_sibling(n)
    assert pads

    def make():
        rng = np.random.default_rng(4242 + n)
        pl = Pipeline(gpu, n, f, B, I, seed=31 * n, corrupt_frac=0.0)
        pl.commit()
        gpu.rbc.lib.rbc_device_sync(0)
        leaves = pl.arr("leaves", shape=(I, n, 32))
        roots = pl.arr("roots", shape=(I, 32)).copy()
        brs = pl.arr("branches", shape=(I, n, d, 32)).copy()
        byz = np.zeros(I, bool)
        for i in range(I):
            if i % 3 == 2:
                continue  # honest
            ip, lvl, lo, hi = pads[(i // 3) % len(pads)]
            mt = [b""] * (2 * W)
            for j in range(n):
                mt[W + j] = bytes(leaves[i, j])
            x = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
            for h in range(W - 1, 0, -1):
                mt[h] = x if h == ip else orc.sha256(mt[2 * h] + mt[2 * h + 1])
            roots[i] = np.frombuffer(mt[1], np.uint8)
            for j in range(n):
                for l_, sib in enumerate(orc.merkle_branch(mt, j)):
                    brs[i, j, l_] = np.frombuffer(sib, np.uint8) if sib else 0
            pres = np.zeros(n, np.uint8)
            pres[rng.permutation(n)[: n - f]] = 1
            pres[lo:hi] = 0
            if i % 3 == 0:
                pres[lo] = 1  # a valid leaf under the padding node's parent
            assert pres.sum() >= k
            pl.present[i] = pres
            byz[i] = True
        pl.b["roots"].upload(roots)
        pl.b["branches"].upload(brs)
        pl.b["present"].upload(pl.present)
        pl.poison()
        return pl, byz

    st = {}
    for mode in ("oneshot", "full", "reuse"):
        pl, byz = make()
        b, c = pl.b, pl.ctx
        if mode == "oneshot":
            c.dev_verify(None, I, b["shards"], pl.spitch, None, pl.S, b["branches"], b["roots"], b["present"],
                         b["valid"], b["leaves_r"])
            c.dev_interpolate(None, I, b["shards"], pl.spitch, None, pl.S, b["valid"], b["leaves_r"], 1,
                              b["roots"], b["out"], pl.opitch, b["digests"], b["status"])
        else:
            c.set_recheck(mode)
            cur = c.rx_batch(I, b["shards"], pl.spitch, None, pl.S, b["branches"], b["roots"], b["present"],
                             b["valid"], b["leaves_r"], b["out"], pl.opitch, b["digests"], b["status"])
            c.dev_receive_step(None, cur, None)
            c.dev_receive_step(None, None, cur)
        gpu.rbc.lib.rbc_device_sync(0)
        valid = pl.arr("valid", shape=(I, n))
        assert np.array_equal(valid.astype(bool), pl.present.astype(bool)), mode  # every ECHO verifies
        st[mode] = pl.arr("status", np.int32).copy()
        assert (st[mode][byz] == -8).all(), (mode, np.flatnonzero(st[mode][byz] != -8))
        assert (st[mode][~byz] == 0).all(), mode
    assert np.array_equal(st["oneshot"], st["reuse"]) and np.array_equal(st["full"], st["reuse"])


def test_verify_form_matches_the_profiling_tools_rule(gpu):
    """rbc_ctx_verify_form (the library's choice of ECHO-verify form) is the
    rule tools/trace_summary.py names kernel roles by, at every bench config:
    the per-leaf walk at C1-C3, leaves + merkle_path_kernel at C4."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import trace_summary as ts
    for cfg, (n, f) in ts.CONFIGS.items():
        k = n - 2 * f
        S = (ts.VALUE_BYTES[cfg] + k - 1) // k
        form = gpu.Context(n, f).verify_form(S)
        assert (form == "shared_path") == ts.shared_path(cfg), (cfg, form)
        assert form == ("shared_path" if cfg == "c4" else "walk")


@pytest.mark.parametrize("n,f,B,tail", [
    (128, 42, 44 * 40 - 3, 48), (128, 42, 44 * 40 - 3, 176), (128, 42, 44 * 300, 240),
    # rows that start off a 4-byte boundary (S mod 4 != 0): S = 41, 5, 3, 763, 257
    (128, 42, 44 * 41 - 7, 0), (128, 42, 44 * 41 - 7, 32), (128, 42, 44 * 5 - 1, 16), (128, 42, 44 * 3, 16),
    (128, 42, 44 * 763, 0), (128, 42, 44 * 257 - 43, 240),
    (256, 85, 86 * 763 - 5, 0), (256, 85, 86 * 7, 64), (64, 21, 22 * 47663 - 9, 0)])
def test_fused_join_zeroes_the_whole_padded_value_tail(gpu, n, f, B, tail):
    """the FFT re-encode's fused join zeroes a value's tail from
    tile 0, whose lanes past the shard row pitch have already returned.  With
    a short row (S = 40, pitch 64) and a value pitch padded past k*S by more
    than the pitch, the tail beyond the pitch would stay unwritten; the fused
    join is then not used and the separate join zero-fills it.  Every byte of
    every value row (data, then zero tail) is checked, the buffer having been
    filled with garbage first.  Rows of S bytes with S mod 4 != 0 start off a
    dword boundary in the value, so neighbouring rows share a dword.  Rows
    shorter than kFusedJoinMinS (capi.cpp) take join_kernel instead: both
    forms are checked here."""
    I = 32
    pl = Pipeline(gpu, n, f, B, I, seed=B + tail, corrupt_frac=0.2)
    k, S = pl.k, pl.S
    vp = rup(k * S, 16) + rup(tail, 16)
    out = gpu.DeviceBuffer(I * vp)
    out.upload(np.full(I * vp, 0xA5, np.uint8))
    pl.commit()
    pl.poison()
    b, c = pl.b, pl.ctx
    c.dev_inject_faults(None, I, b["shards"], pl.spitch, b["corrupt"])
    c.dev_verify(None, I, b["shards"], pl.spitch, None, S, b["branches"], b["roots"], b["present"], b["valid"],
                 b["leaves_r"])
    c.dev_interpolate(None, I, b["shards"], pl.spitch, None, S, b["valid"], b["leaves_r"], 1, b["roots"], out, vp,
                      b["digests"], b["status"])
    gpu.rbc.lib.rbc_device_sync(0)
    assert (pl.arr("status", np.int32) == 0).all()
    got = out.download(I * vp).reshape(I, vp)
    for i in range(I):
        want = np.zeros(vp, np.uint8)
        want[:B] = pl.values[i, :B]
        assert np.array_equal(got[i], want), (i, np.flatnonzero(got[i] != want)[:8])
