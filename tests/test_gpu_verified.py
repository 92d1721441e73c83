"""The host-fed receive path with the validate lane's leaves reused (ABI 6,
VERDICT r05 item 2): validateMessage (rbc/rbc.go:92-95) establishes the
SHA-256 leaf of every received ECHO, so interpolate (rbc/rbc.go:86-90) needs
to hash only the rows it regenerates -- as the device pipeline
(rbc_dev_receive_step) already does.

* rbc_validate_packed_leaves over a receiver's [count][N][pitch] pinned ECHO
  buffer that names only the received rows (the sparse zero-copy gather) and
  over the same messages in pageable memory (one DMA): verdicts equal the C
  oracle's, leaves equal oracle SHA-256 of every message's bytes;
* rbc_interpolate_batch_verified with those leaves: values, digests and
  statuses bit-identical to rbc_interpolate_batch (full rehash) and to the
  oracle, with tampered ECHOs dropped by validate, and a Byzantine
  non-codeword proposer (every row valid under its root) rejected in both
  forms;
* the batcher: rbc_batcher_validate_leaf + rbc_batcher_interpolate_verified
  from many threads, against the oracle."""
import threading

import numpy as np
import pytest

import rbc_oracle as orc
import rbc_ref

pytestmark = pytest.mark.gpu


def _epoch(n, f, count, B, seed, tamper=0.1):
    """count committed values (oracle), each instance's n-f received ECHO
    rows and, for `tamper` of them, one received row with a flipped byte."""
    rng = np.random.default_rng(seed)
    k = n - 2 * f
    S = (B + k - 1) // k
    vals, shards, roots, brs = [], [], [], []
    for i in range(count):
        v = rng.integers(0, 256, B, dtype=np.uint8)
        sh, root, br, _ = rbc_ref.encode_commit(n, f, v)
        vals.append(v)
        shards.append(sh)
        roots.append(np.frombuffer(root, np.uint8))
        brs.append(br)
    present = np.zeros((count, n), np.uint8)
    bad = np.full(count, -1)
    for i in range(count):
        rec = rng.permutation(n)[: n - f]
        present[i, rec] = 1
        if rng.random() < tamper:
            bad[i] = int(rng.choice(rec))
    return dict(vals=vals, shards=np.stack(shards), roots=np.stack(roots), br=np.stack(brs), present=present,
                bad=bad, S=S, k=k)


def _receive_buffer(gpu, e, n, pinned):
    """The receiver's ECHO buffer [count][n][pitch]: received rows at their
    leaf positions (the tampered one flipped), every other row garbage."""
    count, S = e["shards"].shape[0], e["S"]
    pitch = (S + 63) // 64 * 64
    shape = (count, n, pitch)
    buf = gpu.pinned_empty(shape) if pinned else np.empty(shape, np.uint8)
    buf[:] = np.random.default_rng(5).integers(0, 256, shape, dtype=np.uint8)
    buf[:, :, :S] = np.where(e["present"][:, :, None] == 1, e["shards"], buf[:, :, :S])
    for i in np.flatnonzero(e["bad"] >= 0):
        buf[i, e["bad"][i], S // 2] ^= 0x40
    return buf, pitch


def _messages(e, n, pitch):
    inst, pos = np.nonzero(e["present"])
    offs = ((inst * n + pos) * pitch).astype(np.uint64)
    lens = np.full(len(inst), e["S"], np.uint32)
    br = e["br"][inst, pos].reshape(len(inst), -1)
    roots = e["roots"][inst]
    return inst, pos, offs, lens, pos.astype(np.uint8), br, roots


@pytest.mark.parametrize("n,f,B", [(128, 42, 44 * 600 + 7), (37, 12, 13 * 70)])
def test_validate_packed_leaves_sparse_and_dense(gpu, n, f, B):
    e = _epoch(n, f, 48, B, seed=n)
    ctx = gpu.Context(n, f)
    for pinned in (True, False):  # sparse zero-copy gather / whole-arena DMA
        buf, pitch = _receive_buffer(gpu, e, n, pinned)
        inst, pos, offs, lens, idx, br, roots = _messages(e, n, pitch)
        ok, leaves = ctx.validate_packed(buf, offs, lens, idx, br, roots, leaves=True)
        want = e["bad"][inst] != pos
        assert np.array_equal(ok, want), np.flatnonzero(ok != want)[:8]
        flat = buf.reshape(-1)
        for m in range(0, len(inst), 7):  # every 7th message's leaf vs the oracle's SHA-256
            o = int(offs[m])
            assert bytes(leaves[m]) == rbc_ref.sha256(flat[o:o + e["S"]]), m
        # the same verdicts without leaves (rbc_validate_packed)
        assert np.array_equal(ctx.validate_packed(buf, offs, lens, idx, br, roots), want)
    assert (e["bad"] >= 0).any()


@pytest.mark.parametrize("n,f,B", [(128, 42, 44 * 600 + 7), (128, 42, 1 << 20), (37, 12, 13 * 70)])
def test_interpolate_verified_equals_full_and_oracle(gpu, n, f, B):
    count = 40 if B < (1 << 20) else 12
    e = _epoch(n, f, count, B, seed=3 * n + B % 7)
    ctx = gpu.Context(n, f)
    k, S = e["k"], e["S"]
    buf, pitch = _receive_buffer(gpu, e, n, pinned=True)
    inst, pos, offs, lens, idx, br, roots = _messages(e, n, pitch)
    ok, lv = ctx.validate_packed(buf, offs, lens, idx, br, roots, leaves=True)
    # what a node passes to interpolate: the ECHOs that validated, with their leaves
    valid = np.zeros((count, n), np.uint8)
    valid[inst[ok], pos[ok]] = 1
    leaves = gpu.pinned_empty((count, n, 32))
    leaves[:] = 0
    leaves[inst[ok], pos[ok]] = lv[ok]
    shards_in = gpu.pinned_empty((count, n, pitch))
    shards_in[:] = buf
    v_out = gpu.pinned_empty((count, k * S))
    got = ctx.interpolate_submit(shards_in, [S] * count, valid, e["roots"], values_out=v_out, leaves=leaves).wait()
    full = ctx.interpolate_batch(np.array(buf), [S] * count, valid, e["roots"])
    assert np.array_equal(got["status"], full["status"]) and (got["status"] == 0).all()
    assert np.array_equal(got["values"], full["values"])
    assert np.array_equal(got["digests"], full["digests"])
    for i in range(count):
        assert got["values"][i, :B].tobytes() == e["vals"][i].tobytes(), i
    for i in range(0, count, 5):  # digests vs the C restatement (reusing its own verified leaves)
        sh = np.where(valid[i][:, None] == 1, buf[i, :, :S], 0)
        st, val, dig = rbc_ref.interpolate(n, f, sh, valid[i], e["roots"][i].tobytes())
        assert st == 0 and dig == bytes(got["digests"][i]) and val.tobytes() == got["values"][i].tobytes()


def test_interpolate_verified_rejects_noncodeword(gpu):
    """A Byzantine proposer commits rows that are no codeword: every ECHO
    validates under its root, and interpolate must still fail the root
    recheck (valid-but-unused rows that disagree with the re-encoding are
    rehashed) -- with reused leaves exactly as with the full rehash."""
    n, f, S, count = 128, 42, 333, 16
    rng = np.random.default_rng(9)
    rows = rng.integers(0, 256, (count, n, S), dtype=np.uint8)
    roots, leaves_all = [], []
    for i in range(count):
        com = orc.rbc_commit([rows[i, j].tobytes() for j in range(n)])
        roots.append(np.frombuffer(com["root"], np.uint8))
        leaves_all.append(np.stack([np.frombuffer(x, np.uint8) for x in com["leaves"]]))
    roots, leaves_all = np.stack(roots), np.stack(leaves_all)
    ctx = gpu.Context(n, f)
    valid = np.zeros((count, n), np.uint8)
    for i in range(count):
        valid[i, rng.permutation(n)[: n - f]] = 1
    lv = np.ascontiguousarray(leaves_all * valid[:, :, None])
    got = ctx.interpolate_batch(rows, [S] * count, valid, roots, leaves=lv)
    full = ctx.interpolate_batch(rows, [S] * count, valid, roots)
    assert (got["status"] == -8).all() and (full["status"] == -8).all()


def test_batcher_validate_leaf_then_interpolate_verified(gpu):
    n, f, B, count = 128, 42, 44 * 900 + 3, 24
    e = _epoch(n, f, count, B, seed=21)
    k, S = e["k"], e["S"]
    ctx = gpu.Context(n, f)
    bt = gpu.Batcher(ctx, max_batch=8, max_wait_us=500)
    results, errors = [None] * count, []

    def node(i):  # one RBC instance's goroutine: validate every ECHO, then interpolate the valid ones
        try:
            hs = []
            for j in np.flatnonzero(e["present"][i]):
                sh = e["shards"][i, j].copy()
                if e["bad"][i] == j:
                    sh[S // 2] ^= 0x40
                hs.append((j, sh, bt.submit_validate(e["roots"][i].tobytes(), e["br"][i, j].tobytes(), sh, int(j),
                                                     leaf=True)))
            shards, leaves = [b""] * n, np.zeros((n, 32), np.uint8)
            for j, sh, h in hs:
                ok, leaf = bt.wait(h)
                assert ok == (e["bad"][i] != j)
                if ok:
                    assert leaf == rbc_ref.sha256(sh)
                    shards[j], leaves[j] = sh.tobytes(), np.frombuffer(leaf, np.uint8)
            r = bt.wait(bt.submit_interpolate(e["roots"][i].tobytes(), shards, leaves=leaves))
            r0 = bt.wait(bt.submit_interpolate(e["roots"][i].tobytes(), shards))
            results[i] = (r, r0, shards)
        except Exception as x:  # noqa: BLE001
            errors.append(repr(x))

    th = [threading.Thread(target=node, args=(i,)) for i in range(count)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    bt.close()
    assert not errors, errors[:3]
    for i, (r, r0, shards) in enumerate(results):
        assert r == r0
        assert r["value"][:B] == e["vals"][i].tobytes()
        if i % 6 == 0:  # vs the C restatement
            valid = np.array([1 if s else 0 for s in shards], np.uint8)
            rows = np.stack([np.frombuffer(s, np.uint8) if s else np.zeros(S, np.uint8) for s in shards])
            st, val, dig = rbc_ref.interpolate(n, f, rows, valid, e["roots"][i].tobytes())
            assert st == 0 and val.tobytes() == r["value"] and dig == r["digest"]


@pytest.mark.parametrize("n,f,B,pinned", [(128, 42, 44 * 600 + 7, True), (128, 42, 44 * 600 + 7, False),
                                          (256, 85, 86 * 380, True), (37, 12, 13 * 70, True)])
def test_receive_batch_fused_equals_validate_then_interpolate(gpu, n, f, B, pinned):
    """rbc_receive_batch: the present rows cross PCIe once, are verified on
    the device (the walk at N <= 128, leaves + merkle_path_kernel at N = 256)
    and interpolate reuses the verify's leaves.  Its verdicts equal the
    oracle's validateMessage of every present row (tampered ECHOs rejected),
    and values / digests / statuses equal the full-rehash interpolate over the
    rows that validated, and the input values."""
    count = 24
    e = _epoch(n, f, count, B, seed=7 * n + B % 11)
    ctx = gpu.Context(n, f)
    S = e["S"]
    buf, pitch = _receive_buffer(gpu, e, n, pinned)
    d = e["br"].shape[2]
    br = gpu.pinned_empty((count, n, max(d, 1), 32)) if pinned else np.zeros((count, n, max(d, 1), 32), np.uint8)
    br[:] = e["br"].reshape(count, n, max(d, 1), 32)
    got = ctx.receive_batch(buf, [S] * count, e["present"], br, e["roots"])
    want_valid = e["present"].copy()
    for i in np.flatnonzero(e["bad"] >= 0):
        want_valid[i, e["bad"][i]] = 0
    assert np.array_equal(got["valid"], want_valid)
    for i in range(0, count, 6):  # the verdicts vs the oracle's validateMessage
        for j in np.flatnonzero(e["present"][i])[::9]:
            assert bool(got["valid"][i, j]) == rbc_ref.verify(n, buf[i, j, :S], int(j), e["br"][i, j], e["roots"][i].tobytes())
    full = ctx.interpolate_batch(np.array(buf), [S] * count, want_valid, e["roots"])
    assert (got["status"] == 0).all() and np.array_equal(got["status"], full["status"])
    assert np.array_equal(got["values"], full["values"]) and np.array_equal(got["digests"], full["digests"])
    for i in range(count):
        assert got["values"][i, :B].tobytes() == e["vals"][i].tobytes(), i


@pytest.mark.parametrize("n,f", [(256, 85), (37, 12)])
def test_shard_commit_many_short_pinned_values_gathered(gpu, n, f):
    """rbc_shard_commit over >= 64 short pinned values reads them with one
    gather launch over their host addresses (not one DMA per value), and a
    pinned output at a 64-B pitch comes back in one flat copy (bytes past
    S_i zero): shards, roots and branches equal the oracle's for ragged
    lengths (1 byte up to 64 KiB) -- and equal the pageable-memory path."""
    ctx = gpu.Context(n, f)
    rng = np.random.default_rng(n)
    lens = [1, 2, 63, 64, 65, 1000] + [int(x) for x in rng.integers(1, 1 << 16, 94)]
    count = len(lens)
    block = gpu.pinned_empty((count, 1 << 16))
    block[:] = rng.integers(0, 256, block.shape, dtype=np.uint8)
    vals = [block[i, :lens[i]] for i in range(count)]
    k = ctx.k
    Smax = max((L + k - 1) // k for L in lens)
    pitch = (Smax + 63) // 64 * 64
    d = max(ctx.depth, 1)
    out = {"shards": gpu.pinned_empty((count, n, pitch)), "roots": gpu.pinned_empty((count, 32)),
           "branches": gpu.pinned_empty((count, n, d, 32))}
    out["shards"][:] = 0xEE
    got = ctx.shard_commit_submit(vals, out=out).wait()
    ref = ctx.shard_commit_submit([np.array(v) for v in vals]).wait()  # pageable values and outputs
    for i in range(count):
        S = (lens[i] + k - 1) // k
        shards, root, br, _ = rbc_ref.encode_commit(n, f, np.array(vals[i]))
        assert got["shard_lens"][i] == S
        assert np.array_equal(out["shards"][i, :, :S], shards), i
        assert not out["shards"][i, :, S:].any(), i  # the flat copy returns the zero pad
        assert bytes(got["roots"][i]) == root and np.array_equal(got["branches"][i], br), i
        assert np.array_equal(ref["shards"][i, :, :S], shards) and bytes(ref["roots"][i]) == root, i


@pytest.mark.parametrize("n,f,B,pinned", [(128, 42, 44 * 600 + 7, True), (128, 42, 44 * 600 + 7, False),
                                          (256, 85, 86 * 380, True), (37, 12, 13 * 70, True)])
def test_validate_keep_then_interpolate_kept(gpu, n, f, B, pinned):
    """ABI 7: rbc_validate_packed_keep leaves the ECHO rows in a device buffer
    and rbc_interpolate_batch_kept interpolates from there (the rows cross
    PCIe once on the drop-in's validate -> interpolate path).  Verdicts and
    leaves equal rbc_validate_packed_leaves'; values / digests / statuses
    equal the host-memory interpolate over the rows that validated (leaves
    reused, and with leaves=None the full rehash), and the input values."""
    count = 24
    e = _epoch(n, f, count, B, seed=11 * n + B % 13)
    ctx = gpu.Context(n, f)
    k, S = e["k"], e["S"]
    buf, pitch = _receive_buffer(gpu, e, n, pinned)
    inst, pos, offs, lens, idx, br, roots = _messages(e, n, pitch)
    keep = gpu.DeviceBuffer(buf.nbytes)
    ok, lv = ctx.validate_packed_submit(buf, offs, lens, idx, br, roots, leaves=True, keep=keep).wait()
    ok0, lv0 = ctx.validate_packed(buf, offs, lens, idx, br, roots, leaves=True)
    assert np.array_equal(ok, ok0) and np.array_equal(lv[ok], lv0[ok])
    valid = np.zeros((count, n), np.uint8)
    valid[inst[ok], pos[ok]] = 1
    rows = np.zeros((count, n), np.uint64)
    rows[inst[ok], pos[ok]] = keep.value + offs[ok]
    leaves = np.zeros((count, n, 32), np.uint8)
    leaves[inst[ok], pos[ok]] = lv[ok]
    got = ctx.interpolate_kept_submit(rows, [S] * count, e["roots"], leaves=leaves).wait()
    rehash = ctx.interpolate_kept_submit(rows, [S] * count, e["roots"]).wait()
    full = ctx.interpolate_batch(np.array(buf), [S] * count, valid, e["roots"])
    assert (full["status"] == 0).all()
    for r in (got, rehash):
        assert np.array_equal(r["status"], full["status"])
        assert np.array_equal(r["values"], full["values"]) and np.array_equal(r["digests"], full["digests"])
    for i in range(count):
        assert got["values"][i, :B].tobytes() == e["vals"][i].tobytes(), i


def test_interpolate_kept_ragged_from_two_keep_buffers(gpu):
    """Instances of two shard lengths, their rows kept by two validate
    launches in two device buffers, interpolated in ONE kept batch: each
    instance's value is k*S_i bytes, zero past it in the value row."""
    n, f = 128, 42
    ea = _epoch(n, f, 10, 44 * 500 + 9, seed=31)
    eb = _epoch(n, f, 10, 44 * 333 + 1, seed=32)
    ctx = gpu.Context(n, f)
    k = ea["k"]
    rows, lens, roots, leaves, want = [], [], [], [], []
    keeps = []
    for e in (ea, eb):
        buf, pitch = _receive_buffer(gpu, e, n, pinned=True)
        inst, pos, offs, ln, idx, br, rt = _messages(e, n, pitch)
        keep = gpu.DeviceBuffer(buf.nbytes)
        keeps.append(keep)
        ok, lv = ctx.validate_packed_submit(buf, offs, ln, idx, br, rt, leaves=True, keep=keep).wait()
        r = np.zeros((10, n), np.uint64)
        r[inst[ok], pos[ok]] = keep.value + offs[ok]
        l = np.zeros((10, n, 32), np.uint8)
        l[inst[ok], pos[ok]] = lv[ok]
        rows.append(r)
        leaves.append(l)
        lens += [e["S"]] * 10
        roots.append(e["roots"])
        want += [v.tobytes() for v in e["vals"]]
    got = ctx.interpolate_kept_submit(np.concatenate(rows), lens, np.concatenate(roots),
                                      leaves=np.concatenate(leaves)).wait()
    assert (got["status"] == 0).all()
    for i in range(20):
        v = got["values"][i]
        assert v[:len(want[i])].tobytes() == want[i], i
        assert not v[k * lens[i]:].any(), i


@pytest.mark.parametrize("ring_mib", [512, 3])
def test_batcher_keep_validate_then_interpolate(gpu, ring_mib):
    """ABI 7, rbc_batcher_set_keep: the unchanged handler sequence (validate
    every ECHO, then interpolate the ones that validated, through the batcher
    from many threads) with the shards kept on the device.  With a ring that
    holds the epoch every interpolate reads kept rows; with a ring of a few
    arenas launches go unkept and regions are recycled, and those interpolates
    take the host path.  Every value and digest equals the oracle's, and an
    interpolate handed copies of the shards (other pointers) takes the host
    path with the same result."""
    n, f, B, count = 128, 42, 44 * 900 + 3, 32
    e = _epoch(n, f, count, B, seed=41 + ring_mib)
    S = e["S"]
    ctx = gpu.Context(n, f)
    bt = gpu.Batcher(ctx, max_batch=8, max_wait_us=500)
    bt.set_validate(4096, 1 << 20)  # 1 MiB arenas: a 3 MiB ring holds three
    bt.set_keep(ring_mib << 20)
    results, errors = [None] * count, []

    def node(i):
        try:
            rows, hs = {}, []
            for j in np.flatnonzero(e["present"][i]):
                sh = e["shards"][i, j].copy()
                if e["bad"][i] == j:
                    sh[S // 2] ^= 0x40
                rows[j] = sh
                hs.append((j, bt.submit_validate(e["roots"][i].tobytes(), e["br"][i, j].tobytes(), sh, int(j))))
            shards = [np.zeros(0, np.uint8)] * n
            for j, h in hs:
                ok = bt.wait(h)
                assert ok == (e["bad"][i] != j)
                if ok:
                    shards[j] = rows[j]
            r = bt.wait(bt.submit_interpolate(e["roots"][i].tobytes(), shards))
            r2 = bt.wait(bt.submit_interpolate(e["roots"][i].tobytes(), [s.copy() for s in shards]))
            results[i] = (r, r2, shards)
        except Exception as x:  # noqa: BLE001
            errors.append(repr(x))

    th = [threading.Thread(target=node, args=(i,)) for i in range(count)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    st = bt.keep_stats()
    bt.close()
    assert not errors, errors[:3]
    for i, (r, r2, shards) in enumerate(results):
        assert r == r2 and r["value"][:B] == e["vals"][i].tobytes(), i
        if i % 8 == 0:
            valid = np.array([1 if len(s) else 0 for s in shards], np.uint8)
            rows = np.stack([s if len(s) else np.zeros(S, np.uint8) for s in shards])
            stc, val, dig = rbc_ref.interpolate(n, f, rows, valid, e["roots"][i].tobytes())
            assert stc == 0 and val.tobytes() == r["value"] and dig == r["digest"]
    assert st["host_interps"] >= count  # the copies
    if ring_mib >= 512:
        assert st["kept_interps"] == count and st["unkept_launches"] == 0, st
    else:
        assert st["kept_launches"] > 0, st


def test_interpolate_pinned_values_at_an_odd_pitch(gpu):
    """Pinned values_out at a pitch the device rows do not use (k*Smax + 5,
    not a multiple of 16): the rows are repacked on the device and come back
    in one copy.  Ragged instances (two shard lengths): every row holds its
    value then zeros up to the pitch (the last row up to k*S_i), equal to the
    pageable (staged) result."""
    n, f = 128, 42
    ea = _epoch(n, f, 9, 44 * 400 + 3, seed=51)
    eb = _epoch(n, f, 9, 44 * 257 + 11, seed=52)
    ctx = gpu.Context(n, f)
    k = ea["k"]
    Sa, Sb = ea["S"], eb["S"]
    Smax = max(Sa, Sb)
    pitch = (Smax + 63) // 64 * 64
    count = 18
    shards = np.zeros((count, n, pitch), np.uint8)
    shards[:9, :, :Sa] = ea["shards"]
    shards[9:, :, :Sb] = eb["shards"]
    present = np.concatenate([ea["present"], eb["present"]])
    roots = np.concatenate([ea["roots"], eb["roots"]])
    lens = [Sa] * 9 + [Sb] * 9
    vp = k * Smax + 5
    v_pin = gpu.pinned_empty((count, vp))
    v_pin[:] = 0xA5
    got = ctx.interpolate_submit(shards, lens, present, roots, values_out=v_pin).wait()
    ref = ctx.interpolate_batch(shards, lens, present, roots)
    assert (got["status"] == 0).all() and np.array_equal(got["digests"], ref["digests"])
    vals = [v.tobytes() for v in ea["vals"]] + [v.tobytes() for v in eb["vals"]]
    for i in range(count):
        kS = k * lens[i]
        assert v_pin[i, :len(vals[i])].tobytes() == vals[i], i
        assert np.array_equal(v_pin[i, :kS], ref["values"][i, :kS]), i
        end = vp if i < count - 1 else k * Smax
        assert not v_pin[i, kS:end].any(), i
