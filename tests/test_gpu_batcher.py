"""The batcher's validate lane on the GPU at epoch scale:
validateMessage (rbc/rbc.go:92-95) arrives once per ECHO from every
instance's goroutine, so tens of thousands are outstanding per node.  Here
16,384 are submitted from 8 threads before any is waited on; every verdict
must equal the C oracle's (oracle/rbc_ref.verify) on the same message, and
the lane must coalesce them into few launches.  Messages come from proposals
committed by the oracle, with mixed shard lengths in one arena (ragged
values), honest and tampered: a flipped shard byte, a flipped branch byte, a
wrong root, a wrong index, a truncated branch, an empty shard."""
import threading

import numpy as np
import pytest

import rbc_ref

pytestmark = pytest.mark.gpu


def _unflatten(flat, j, n, d):
    """Go flat branch -> device slots [d][32] (zero level-0 slot when j ^ 1 >= n), or None on a bad length."""
    empty0 = d > 0 and (j ^ 1) >= n
    if j >= n or len(flat) != 32 * (d - empty0):
        return None
    slots = np.zeros((max(d, 1), 32), np.uint8)
    body = np.frombuffer(flat, np.uint8).reshape(-1, 32) if flat else np.zeros((0, 32), np.uint8)
    slots[int(empty0):d] = body
    return slots[:d]


def _messages(n, f, count, seed):
    rng = np.random.default_rng(seed)
    d = max(1, (n - 1).bit_length()) if n > 1 else 0
    commits = []
    for _ in range(24):
        v = rng.integers(0, 256, int(rng.integers(1, 180_000)), dtype=np.uint8)
        shards, root, br, _ = rbc_ref.encode_commit(n, f, v)
        commits.append((shards, root, br))
    msgs = []
    for m in range(count):
        shards, root, br = commits[int(rng.integers(len(commits)))]
        j = int(rng.integers(n))
        flat = b"".join(bytes(br[j, l]) for l in range(d) if not (l == 0 and (j ^ 1) >= n))
        shard = shards[j].tobytes()
        idx = j
        kind = int(rng.integers(10))
        if kind == 1:
            b = bytearray(shard)
            b[int(rng.integers(len(b)))] ^= 0x10
            shard = bytes(b)
        elif kind == 2 and flat:
            b = bytearray(flat)
            b[int(rng.integers(len(b)))] ^= 0x02
            flat = bytes(b)
        elif kind == 3:
            root = bytes([root[0] ^ 1]) + root[1:]
        elif kind == 4:
            idx = (j + 1 + int(rng.integers(n - 1))) % n if n > 1 else j
        elif kind == 5 and flat:
            flat = flat[:-32]
        elif kind == 6:
            shard = b""
        slots = _unflatten(flat, idx, n, d)
        want = bool(shard) and slots is not None and rbc_ref.verify(n, np.frombuffer(shard, np.uint8), idx, slots,
                                                                    root)
        msgs.append((root, flat, shard, idx, want))
    return msgs


@pytest.mark.parametrize("n,f", [(128, 42), (37, 12)])
def test_validate_lane_16k_outstanding_matches_oracle(gpu, n, f):
    msgs = _messages(n, f, 16384, seed=n)
    ctx = gpu.Context(n, f)
    for arena_msgs, max_wait in ((65536, 3_000_000), (1000, 200)):
        bt = gpu.Batcher(ctx, max_batch=256, max_wait_us=max_wait)
        bt.set_validate(arena_msgs, 256 << 20)
        handles = [None] * len(msgs)

        def submit(t):
            for m in range(t, len(msgs), 8):
                root, flat, shard, idx, _ = msgs[m]
                handles[m] = bt.submit_validate(root, flat, shard, idx)

        th = [threading.Thread(target=submit, args=(t,)) for t in range(8)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        got = [bt.wait(h) for h in handles]  # all 16,384 were outstanding before the first wait
        want = [m[4] for m in msgs]
        assert got == want, [i for i, (a, b) in enumerate(zip(got, want)) if a != b][:10]
        launches, requests = bt.stats()
        assert requests == len(msgs)
        if arena_msgs == 65536:  # one arena holds every outstanding message: one launch, at most a few
            assert launches <= 2, launches
        else:  # 1,000-message arenas rotate through the lane's six, four in flight
            assert launches >= len(msgs) // 1000, launches
        bt.close()
    assert 0.3 < np.mean(want) < 0.9  # honest and tampered messages both present


@pytest.mark.parametrize("n,f", [(128, 42), (37, 12), (256, 85)])
def test_validate_packed_matches_oracle_and_checks_its_layout(gpu, n, f):
    """rbc_validate_packed, the launch the lane (and a Go batcher with its own
    pinned rings) calls: messages packed at 64-B aligned offsets with gaps, in
    pageable and in pinned memory, ragged lengths, device-form branches (zero
    level-0 slot where j ^ 1 >= n), honest and tampered -- every verdict equals
    the C oracle's.  A misaligned offset, a message past the arena's end, a
    zero length and a leaf index >= n are refused before any work; count 0 is
    a no-op."""
    rng = np.random.default_rng(7 * n)
    d = max(1, (n - 1).bit_length())
    msgs = [m for m in _messages(n, f, 3000, seed=11 * n) if m[2] and _unflatten(m[1], m[3], n, d) is not None]
    count = len(msgs)
    offs, pos = np.zeros(count, np.uint64), 0
    for i, m in enumerate(msgs):
        offs[i] = pos
        pos += (len(m[2]) + 63) // 64 * 64 + 64 * int(rng.integers(0, 3))  # gaps of 0-2 blocks
    lens = np.array([len(m[2]) for m in msgs], np.uint32)
    idx = np.array([m[3] for m in msgs], np.uint8)
    br = np.stack([_unflatten(m[1], m[3], n, d).reshape(-1) for m in msgs])
    roots = np.stack([np.frombuffer(m[0], np.uint8) for m in msgs])
    want = np.array([m[4] for m in msgs])
    ctx = gpu.Context(n, f)
    for pinned in (False, True):
        arena = gpu.pinned_empty((pos,)) if pinned else np.zeros(pos, np.uint8)
        arena[:] = rng.integers(0, 256, pos, dtype=np.uint8)  # the gaps hold garbage
        for i, m in enumerate(msgs):
            arena[int(offs[i]): int(offs[i]) + len(m[2])] = np.frombuffer(m[2], np.uint8)
        got = ctx.validate_packed(arena, offs, lens, idx, br, roots)
        assert np.array_equal(got, want), np.flatnonzero(got != want)[:10]
    assert 0.3 < want.mean() < 0.95
    small = np.zeros(4096, np.uint8)
    one = dict(branches=br[:1], roots=roots[:1])
    bad = [(8, 100, 0), (4096 - 64, 100, 0), (0, 0, 0), (2 ** 64 - 64, 100, 0)]  # the last wraps past 2^64
    bad += [(0, 100, n)] if n < 256 else []  # idx is a byte
    for o, ln, ix in bad:
        with pytest.raises(gpu.RBCError):
            ctx.validate_packed(small, [o], [ln], [ix], **one)
    assert ctx.validate_packed(small, [], [], [], br[:0], roots[:0]).size == 0


def test_batcher_epoch_all_three_kinds_with_reused_leaves(tmp_path):
    """one node's C2 epoch through the batcher as the Go
    handlers drive it -- 1,024 shard, 88,064 validateMessage and 1,024
    interpolate requests from 16 client threads at once, 10 % of the
    instances with a corrupted ECHO.  tools/batcher_bench checks every
    verdict, value, shard row and root itself, and that interpolate with the
    validate lane's leaves (only regenerated rows hashed) equals the full
    rehash bit for bit, and so does the pass with the validated rows kept on
    the device (ABI 7, rbc_batcher_set_keep); the sampled digests and roots are checked here against
    the C oracle."""
    import json
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tools", "batcher_bench")
    assert os.path.exists(exe), "build() makes tools/batcher_bench"
    dump = tmp_path / "epoch.bin"
    r = subprocess.run([exe, "epoch", "1024", "16", "64", "200", str(dump)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    rows = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    ep = [x for x in rows if x["phase"] == "epoch"]
    assert [x["interpolate"].split()[0] for x in ep] == ["verified", "full", "kept"]
    for x in ep:
        assert x["instances"] == 1024 and x["echo_messages"] == 1024 * 86 and x["requests"] == 1024 * 88
        assert x["value_failures"] == 0 and x["shard_failures"] == 0 and x["client_failures"] == 0 and x["GBps"] > 0
    chk = rows[-1]
    assert chk["phase"] == "check" and chk["failures"] == 0 and chk["verified_equals_full"]
    # ABI 7: with rbc_batcher_set_keep every interpolate of the kept pass read its rows on the device
    keep = next(x for x in rows if x["phase"] == "keep")
    assert keep["kept_interps"] >= 1024 and keep["kept_launches"] > 0, keep
    n, f, B = 128, 42, 1 << 20
    k = n - 2 * f
    raw = dump.read_bytes()
    rec = 4 + B + 64
    assert len(raw) == 8 * rec
    for q in range(8):
        o = q * rec
        value = np.frombuffer(raw[o + 4:o + 4 + B], np.uint8)
        _, root, _, leaves = rbc_ref.encode_commit(n, f, value)
        assert raw[o + 4 + B:o + 4 + B + 32] == root
        assert raw[o + 4 + B + 32:o + rec] == rbc_ref.sha256(np.ascontiguousarray(leaves[:k]).tobytes())
