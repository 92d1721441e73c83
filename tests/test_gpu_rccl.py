"""The multi-GPU exchange on the device (BASELINE north_star (5)):
a 1-rank RCCL communicator through librbc_gpu.so, the ragged-share record
all-gather (rbc_dev_allgather_records) of HIP-computed roots and digests
compared byte-for-byte with the C oracle's, the ACS assembly of the gathered
buffer, and the bench's synthetic-input / result-check kernels.  (N > 1 ranks
are covered on CPU by tests/test_distributed.py and tests/test_acs_host.py;
RCCL needs one device per rank.)"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def rup(x, a):
    return (x + a - 1) // a * a


def test_fill_random_matches_host_restatement(gpu):
    ca = gpu
    from cleisthenes_amd import synth
    rows, pitch, first, seed = 7, 4160, 1234, 99
    buf = ca.DeviceBuffer(rows * pitch)
    ca.rbc.fill_random(0, None, buf, first, rows, pitch, seed)
    ca.rbc.lib.rbc_device_sync(0)
    got = buf.download().reshape(rows, pitch)
    for r in range(rows):
        assert np.array_equal(got[r], synth.row(seed, first + r, pitch, pitch)), r


def test_count_mismatch_counts_differing_chunks(gpu):
    ca = gpu
    rows, pa, pb, length = 9, 4096, 4160, 4001  # length not a multiple of 16: the tail is masked
    rng = np.random.default_rng(5)
    a = rng.integers(0, 256, (rows, pa), dtype=np.uint8)
    b = np.zeros((rows, pb), dtype=np.uint8)
    b[:, :pa] = a
    b[:, length:] ^= 0xFF  # past `length`: ignored
    da, db, dc = ca.DeviceBuffer(a.nbytes), ca.DeviceBuffer(b.nbytes), ca.DeviceBuffer(16)
    da.upload(a)
    db.upload(b)
    ca.rbc.count_mismatch(0, None, da, pa, db, pb, rows, length, dc)
    ca.rbc.lib.rbc_device_sync(0)
    assert dc.download(4).view(np.uint32)[0] == 0
    b[2, 0] ^= 1          # chunk 0 of row 2
    b[5, 4000] ^= 1       # last (partial) chunk of row 5
    b[5, 17] ^= 1         # chunk 1 of row 5
    db.upload(b)
    ca.rbc.count_mismatch(0, None, da, pa, db, pb, rows, length, dc)
    ca.rbc.lib.rbc_device_sync(0)
    assert dc.download(4).view(np.uint32)[0] == 3


def _device_round(ca, ctx, values, bad_root):
    """shard+commit -> verify -> interpolate on the device for `count`
    instances; instances in bad_root get a wrong expected root (status -8)."""
    n, k, d = ctx.n, ctx.k, ctx.depth
    count, B = values.shape
    S = (B + k - 1) // k
    sp, vp, op = rup(S, 64), rup(k * S + 32, 64), rup(k * S, 16)
    vals = np.zeros((count, vp), np.uint8)
    vals[:, :B] = values
    dv, dsh = ca.DeviceBuffer(vals.nbytes), ca.DeviceBuffer(count * n * sp)
    dv.upload(vals)
    dlv, drt, dbr = ca.DeviceBuffer(count * n * 32), ca.DeviceBuffer(count * 32), ca.DeviceBuffer(count * n * d * 32)
    ctx.dev_shard_commit(None, count, dv, vp, None, B, dsh, sp, None, dlv, drt, dbr)
    dval, dlr = ca.DeviceBuffer(count * n), ca.DeviceBuffer(count * n * 32)
    ctx.dev_verify(None, count, dsh, sp, None, S, dbr, drt, None, dval, dlr)
    roots = drt.download().reshape(count, 32).copy()
    exp = roots.copy()
    for i in bad_root:
        exp[i] ^= 0xA5
    dexp = ca.DeviceBuffer(exp.nbytes)
    dexp.upload(exp)
    dout, ddig, dst = ca.DeviceBuffer(count * op), ca.DeviceBuffer(count * 32), ca.DeviceBuffer(count * 4)
    ddig.zero()
    ctx.dev_interpolate(None, count, dsh, sp, None, S, dval, dlr, 1, dexp, dout, op, ddig, dst)
    ca.rbc.lib.rbc_device_sync(0)
    return drt, ddig, dst, roots


def test_rccl_one_rank_allgather_records_vs_oracle(gpu, ref):
    ca = gpu
    from cleisthenes_amd import acs
    n, f, B, count = 16, 5, 3001, 10
    ctx = ca.Context(n, f)
    ctx.comm_init(1, 0, ca.Context.comm_unique_id())
    info = ctx.comm_info()
    assert info["nranks"] == 1 and info["rank"] == 0
    assert info["version"] > 0 and os.path.basename(info["lib"]).startswith("librccl")
    assert "torch" not in info["lib"] and "torch" not in info["hip_lib"], info
    rng = np.random.default_rng(77)
    values = rng.integers(0, 256, (count, B), dtype=np.uint8)
    bad = {3, 7}
    drt, ddig, dst, roots = _device_round(ca, ctx, values, bad)
    status = dst.download().view(np.int32)
    assert [i for i in range(count) if status[i] != 0] == sorted(bad)
    assert set(status[list(bad)]) == {-8}
    slots = count + 3  # ragged padding: every rank sends max_share slots
    dg = ca.DeviceBuffer(slots * 64)
    dg.upload(np.full(slots * 64, 0xEE, np.uint8))  # stale bytes must be overwritten
    ctx.dev_allgather_records(None, count, slots, drt, ddig, dst, dg)
    ca.rbc.lib.rbc_device_sync(0)
    g = dg.download().reshape(1, slots, 64)
    k = ctx.k
    for i in range(count):
        _, root, _, leaves = ref.encode_commit(n, f, values[i])
        assert bytes(g[0, i, :32]) == root, i
        want_dig = bytes(32) if i in bad else ref.sha256(np.ascontiguousarray(leaves[:k]).tobytes())
        assert bytes(g[0, i, 32:]) == want_dig, i
        assert bytes(roots[i]) == root
    assert not g[0, count:].any()
    out = acs.assemble_output_set(g[:, :count], count, 1)
    assert [o["instance"] for o in out] == [i for i in range(count) if i not in bad]
    # the square form: every rank sends exactly `count`
    dg2 = ca.DeviceBuffer(count * 64)
    ctx.dev_allgather_roots(None, count, drt, ddig, dg2)
    ca.rbc.lib.rbc_device_sync(0)
    g2 = dg2.download().reshape(count, 64)
    assert np.array_equal(g2[:, :32], roots)
    ctx.close()


def test_allgather_before_comm_init_is_an_error(gpu):
    ca = gpu
    ctx = ca.Context(4, 1)
    buf = ca.DeviceBuffer(64 * 4)
    with pytest.raises(ca.RBCError) as e:
        ctx.dev_allgather_records(None, 2, 4, buf, buf, None, buf)
    assert e.value.code == -12
    ctx.close()
