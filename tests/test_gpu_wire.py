"""Device-side VAL / ECHO marshaling (rbc_dev_marshal_val, csrc/wire.hip)
against the host codec (rbc_pb_encode_rbc over rbc_json_encode_val, itself
pinned to the protobuf runtime and Go-JSON rules in test_protocol_codec.py):
byte-identical messages for every (instance, recipient), including ragged
shard lengths, every S mod 3 phase, odd N (the empty level-0 sibling),
and a full-size C2 instance."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def rup(x, a):
    return (x + a - 1) // a * a


def marshal_and_check(ca, n, f, lens, msg_type, seed=0):
    from cleisthenes_amd import protocol
    ctx = ca.Context(n, f)
    try:
        rng = np.random.default_rng(seed)
        values = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in lens]
        c = ctx.shard_commit_batch(values)
        count = len(values)
        slens = c["shard_lens"].astype(np.uint32)
        Smax = int(slens.max())
        pitch = rup(Smax, 64)
        sh = np.zeros((count, n, pitch), np.uint8)
        sh[:, :, : c["shards"].shape[2]] = c["shards"]
        d = ctx.depth
        br = np.ascontiguousarray(c["branches"]).reshape(count, n, d, 32) if d else np.zeros(1, np.uint8)
        out_pitch = rup(max(ctx.val_message_size(int(S), 0, msg_type) for S in slens), 16)
        dsh, dbr, drt = ca.DeviceBuffer(sh.nbytes), ca.DeviceBuffer(max(br.nbytes, 1)), ca.DeviceBuffer(count * 32)
        dln, dout = ca.DeviceBuffer(count * 4), ca.DeviceBuffer(count * n * out_pitch)
        dol = ca.DeviceBuffer(count * n * 4)
        dsh.upload(sh)
        dbr.upload(br.reshape(-1))
        drt.upload(np.ascontiguousarray(c["roots"]).reshape(-1))
        dln.upload(slens)
        dout.upload(np.full(count * n * out_pitch, 0xEE, np.uint8))  # poison
        ragged = len(set(slens.tolist())) > 1
        ctx.dev_marshal_val(None, count, msg_type, dsh, pitch, dln if ragged else None, 0 if ragged else int(Smax),
                            dbr, drt, dout, out_pitch, dol)
        ca.rbc.lib.rbc_device_sync(0)
        out = dout.download().reshape(count, n, out_pitch)
        ol = dol.download().view(np.uint32).reshape(count, n)
        for i in range(count):
            S = int(slens[i])
            for j in range(n):
                flat = b"".join(bytes(br[i, j, lvl]) for lvl in range(d) if not (lvl == 0 and (j ^ 1) >= n))
                want = protocol.pb_encode(msg_type, protocol.json_encode_val(bytes(c["roots"][i]), flat,
                                                                             bytes(c["shards"][i, j, :S])))
                assert ol[i, j] == len(want) == ctx.val_message_size(S, j, msg_type), (i, j)
                got = bytes(out[i, j, : len(want)])
                assert got == want, (i, j, next(x for x in range(len(want)) if got[x] != want[x]))
                assert not out[i, j, len(want): rup(len(want), 16)].any()  # chunk tail zeroed
        return out
    finally:
        ctx.close()


@pytest.mark.parametrize("n,f", [(4, 1), (7, 2), (16, 5), (64, 21)])
@pytest.mark.parametrize("msg_type", [0, 1])
def test_marshal_matches_host_codec_ragged(gpu, n, f, msg_type):
    k = n - 2 * f
    # every S mod 3 phase, tiny to a few KB (slow-path heavy), ragged within one launch
    lens = [1, k, 2 * k + 1, 3 * k * 7 + 5, 1000, 4096 + 13, 20000, 3 * k * 100]
    marshal_and_check(gpu, n, f, lens, msg_type, seed=n + msg_type)


def test_marshal_full_size_c2_instance(gpu):
    marshal_and_check(gpu, 128, 42, [1 << 20, (1 << 20) - 1], 0, seed=5)


def test_marshal_round_trips_through_the_state_machine(gpu):
    """A device-marshaled VAL is accepted by an rbc_node as its proposer's VAL."""
    from cleisthenes_amd import protocol
    ca = gpu
    n, f = 4, 1
    out = None
    ctx = ca.Context(n, f)
    bt = ca.Batcher(ctx, max_batch=64, max_wait_us=500)
    try:
        v = np.random.default_rng(3).integers(0, 256, 777, dtype=np.uint8).tobytes()
        c = ctx.shard_commit_batch([v])
        S = int(c["shard_lens"][0])
        pitch = rup(S, 64)
        sh = np.zeros((1, n, pitch), np.uint8)
        sh[:, :, : c["shards"].shape[2]] = c["shards"]
        out_pitch = rup(ctx.val_message_size(S, 0, 0), 16)
        dsh, dbr, drt = ca.DeviceBuffer(sh.nbytes), ca.DeviceBuffer(n * ctx.depth * 32), ca.DeviceBuffer(32)
        dout, dol = ca.DeviceBuffer(n * out_pitch), ca.DeviceBuffer(n * 4)
        dsh.upload(sh)
        dbr.upload(np.ascontiguousarray(c["branches"]).reshape(-1))
        drt.upload(np.ascontiguousarray(c["roots"]).reshape(-1))
        ctx.dev_marshal_val(None, 1, 0, dsh, pitch, None, S, dbr, drt, dout, out_pitch, dol)
        ca.rbc.lib.rbc_device_sync(0)
        out = dout.download().reshape(n, out_pitch)
        ol = dol.download().view(np.uint32)
        node = protocol.Node(bt, n, f, 2, 0)
        assert node.handle_message(0, bytes(out[2, : ol[2]])) == 0
        node.progress(wait=True)
        msgs = node.messages()
        assert len(msgs) == 1 and msgs[0][0] == -1  # its ECHO, to everyone
        t, payload = protocol.pb_decode(msgs[0][1])
        assert t == protocol.ECHO and protocol.json_decode_val(payload)["Block"] == [bytes(c["shards"][0, 2, :S])]
        node.close()
    finally:
        bt.close()
        ctx.close()


@pytest.mark.parametrize("n,f,lens,pinned", [(16, 5, [1001, 777, 5000], False), (7, 2, [333, 1, 2000], True),
                                             (128, 42, [1 << 20, (1 << 20) - 3], True)])
def test_shard_commit_val_hands_over_every_recipients_message(gpu, n, f, lens, pinned):
    """rbc_shard_commit_val: every per-recipient VAL is
    byte-identical to the host codec over the oracle's commitment, handed
    over in one D2H into a pinned (or pageable) ring."""
    import rbc_oracle as orc
    from cleisthenes_amd import protocol
    ca = gpu
    ctx = ca.Context(n, f)
    rng = np.random.default_rng(sum(lens))
    vals = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in lens]
    k = n - 2 * f
    Smax = max((L + k - 1) // k for L in lens)
    pitch = rup(max(ctx.val_message_size(Smax, 0, 0), ctx.val_message_size(Smax, n - 1, 0)), 16)
    ring = ca.pinned_empty((len(vals), n, pitch)) if pinned else None
    out = ctx.shard_commit_val(vals, ring=ring)
    enc = orc.Encoder(k, 2 * f)
    for i, v in enumerate(vals):
        shards = orc.rbc_shard(enc, np.frombuffer(v, np.uint8))
        com = orc.rbc_commit(shards)
        assert bytes(out["roots"][i]) == com["root"]
        for j in range(n):
            br = orc.flat_branch(com["branches"][j])
            want = protocol.pb_encode(protocol.VAL, protocol.json_encode_val(com["root"], br, bytes(shards[j])))
            assert out["message"](i, j) == want, (i, j)
    ctx.close()
