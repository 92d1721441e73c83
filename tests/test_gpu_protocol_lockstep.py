"""The C++ RBC state machine on the GPU data path, in lock step with the
state-machine oracle (oracle/rbc_protocol_oracle.py).

Every node of an instance exists twice -- a ``protocol.Node`` (rbc_node.cpp,
shard / validateMessage / interpolate on the GPU through one shared batcher)
and an ``OracleNode`` (pure Python over the RS / Merkle oracle).  A seeded
scheduler delivers the in-flight messages in random order and random batch
sizes; Byzantine senders rewrite them; both twins receive the same bytes.
After every batch each touched node runs ``progress`` and the test asserts:

* the same handle_message status for every message;
* the same outgoing messages, in the same order, byte for byte (VAL, ECHO,
  READY pb.Message bytes, recipients included);
* the same stats (valid ECHOs / READYs for the leading root, READY sent,
  rejected) and the same delivered value or protocol error.

Faults covered: silent nodes, corrupted ECHO shards, forged READY roots,
replayed (duplicate) messages, garbage and truncated pb bytes, wrong-sender
VALs, an equivocating proposer, a non-codeword proposal, a badly framed
payload, a proposal whose committed shards have ragged lengths.
"""
import random
import zlib

import numpy as np
import pytest

import rbc_oracle as orc
import rbc_protocol_oracle as po

pytestmark = pytest.mark.gpu


def rand(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


class Twins:
    def __init__(self, ca, n, f, proposer, seed, byz=(), mode=None, max_batch=64):
        from cleisthenes_amd import protocol
        self.pr = protocol
        self.ctx = ca.Context(n, f)
        self.bt = ca.Batcher(self.ctx, max_batch=max_batch, max_wait_us=200)
        self.n, self.f, self.proposer = n, f, proposer
        self.gpu = [protocol.Node(self.bt, n, f, i, proposer) for i in range(n)]
        self.orc = [po.OracleNode(n, f, i, proposer) for i in range(n)]
        self.rng = random.Random(seed)
        self.byz, self.mode = set(byz), mode
        self.flight = []
        self.sent = []     # every message ever sent (for replays)
        self.compared = 0

    def close(self):
        for nd in self.gpu:
            nd.close()
        self.bt.close()
        self.ctx.close()

    # -- both twins ----------------------------------------------------------
    def sync(self, i):
        self.gpu[i].progress(wait=True)
        self.orc[i].progress()
        a, b = self.gpu[i].messages(), self.orc[i].messages()
        assert a == b, (i, [(t, m[:40]) for t, m in a], [(t, m[:40]) for t, m in b])
        self.compared += len(a)
        assert self.gpu[i].stats() == self.orc[i].stats(), i
        self.check_value(i)
        for to, m in a:
            for dst in (range(self.n) if to < 0 else [to]):
                if dst != i:
                    self.flight.append((i, dst, m))
                    self.sent.append((i, dst, m))

    def check_value(self, i):
        ov = self.orc[i].value()
        if ov == po.ERR_PROTOCOL:
            with pytest.raises(Exception) as ei:
                self.gpu[i].value()
            assert getattr(ei.value, "code", None) == -20
        else:
            assert self.gpu[i].value() == ov, i

    def handle(self, src, dst, m):
        rg = self.gpu[dst].handle_message(src, m)
        ro = self.orc[dst].handle_message(src, m)
        assert rg == ro, (src, dst, rg, ro, m[:60])

    def propose(self, value):
        p = self.proposer
        self.gpu[p].propose(value)
        assert self.orc[p].propose(value) == 0
        self.sync(p)

    # -- Byzantine rewriting --------------------------------------------------
    def tamper(self, src, dst, m):
        if src not in self.byz:
            return [m]
        mode, rng = self.mode, self.rng
        if mode == "silent":
            return []
        t, pl = po.pb_decode(m)
        if mode == "bad_echo" and t == po.ECHO:
            r = po.json_decode(pl)
            blk = bytearray(r["block"][0])
            blk[rng.randrange(len(blk))] ^= 1 << rng.randrange(8)
            return [po.pb_encode(t, po.json_encode_val(r["root"], r["branch"], bytes(blk)))]
        if mode == "bad_ready" and t in (po.ECHO, po.READY):
            return [po.pb_encode(po.READY, po.json_encode_ready(rand(32, src)))]
        if mode == "chaos":
            roll = rng.random()
            if roll < 0.15:
                return []
            if roll < 0.3:
                return [m, m]                                  # duplicate
            if roll < 0.4:
                return [m[:rng.randrange(len(m))]]             # truncated pb
            if roll < 0.5:
                return [bytes(rng.randrange(256) for _ in range(rng.randrange(1, 40)))]
            if roll < 0.6 and self.sent:
                return [m, rng.choice(self.sent)[2]]           # replay another message
            if roll < 0.7:
                b = bytearray(m)
                b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
                return [bytes(b)]
        return [m]

    # -- scheduler ------------------------------------------------------------
    def run(self, max_rounds=10000):
        for _ in range(max_rounds):
            if not self.flight:
                return
            self.rng.shuffle(self.flight)
            take = self.rng.randint(1, min(len(self.flight), 3 * self.n))
            batch, self.flight = self.flight[:take], self.flight[take:]
            touched = []
            for src, dst, m in batch:
                for mm in self.tamper(src, dst, m):
                    # a Byzantine sender may also pose as the proposer (VAL from a
                    # non-proposer is dropped by handleValueRequest)
                    self.handle(src, dst, mm)
                    if dst not in touched:
                        touched.append(dst)
            for i in touched:
                self.sync(i)
        raise AssertionError("did not quiesce")


@pytest.fixture(scope="module")
def ca(gpu):
    return gpu


@pytest.mark.parametrize("n,f,B,seed", [(4, 1, 1000, 0), (7, 2, 333, 1), (10, 3, 4096, 2), (4, 1, 0, 3),
                                        (16, 5, 20000, 4)])
def test_lockstep_honest(ca, n, f, B, seed):
    tw = Twins(ca, n, f, proposer=seed % n, seed=seed)
    try:
        v = rand(B, seed)
        tw.propose(v)
        tw.run()
        for i in range(n):
            assert tw.gpu[i].value() == v
        # proposer: N-1 VALs; every node: one ECHO and one READY, all compared
        assert tw.compared == (n - 1) + 2 * n
    finally:
        tw.close()


@pytest.mark.parametrize("mode", ["silent", "bad_echo", "bad_ready", "chaos"])
@pytest.mark.parametrize("seed", [10, 11])
def test_lockstep_byzantine_nodes(ca, mode, seed):
    n, f = 7, 2
    tw = Twins(ca, n, f, proposer=0, seed=seed, byz={5, 6}, mode=mode)
    try:
        v = rand(2500, seed)
        tw.propose(v)
        tw.run()
        for i in range(5):
            assert tw.gpu[i].value() == v, (mode, i)
    finally:
        tw.close()


def _vals(n, f, payload, corrupt=False, ragged=False):
    enc = orc.Encoder(n - 2 * f, 2 * f)
    sh = [bytes(x) for x in orc.rbc_shard(enc, payload)]
    if corrupt:
        sh[n - 1] = bytes([sh[n - 1][0] ^ 1]) + sh[n - 1][1:]
    if ragged:  # committed, so it validates; interpolate must refuse it
        sh[0] = sh[0] + b"\x00"
    mt = orc.merkle_tree(sh)
    return [po.pb_encode(po.VAL, po.json_encode_val(mt[1], orc.flat_branch(
        [b for b in orc.merkle_branch(mt, j) if b]), sh[j])) for j in range(n)]


@pytest.mark.parametrize("case", ["equivocate", "noncodeword", "bad_frame", "ragged", "wrong_sender"])
def test_lockstep_byzantine_proposer(ca, case):
    n, f = 7, 2
    P = n - 1
    tw = Twins(ca, n, f, proposer=P, seed=zlib.crc32(case.encode()))
    try:
        fr = lambda x: len(x).to_bytes(8, "little") + x  # noqa: E731
        if case == "equivocate":
            va, vb = _vals(n, f, fr(rand(900, 1))), _vals(n, f, fr(rand(900, 2)))
            msgs = [va[j] if j < n - f else vb[j] for j in range(n - 1)]
        elif case == "noncodeword":
            msgs = _vals(n, f, fr(rand(700, 3)), corrupt=True)[:n - 1]
        elif case == "bad_frame":
            msgs = _vals(n, f, (10 ** 9).to_bytes(8, "little") + rand(500, 4))[:n - 1]
        elif case == "ragged":
            msgs = _vals(n, f, fr(rand(700, 5)), ragged=True)[:n - 1]
        else:
            msgs = _vals(n, f, fr(rand(700, 6)))[:n - 1]
        for j in range(n - 1):
            src = 0 if case == "wrong_sender" and j % 2 else P
            tw.handle(src, j, msgs[j])
            tw.sync(j)
        tw.run()
        vals = set()
        for j in range(n - 1):
            ov = tw.orc[j].value()
            vals.add(ov if ov is None or ov == po.ERR_PROTOCOL else bytes(ov))
        if case == "equivocate":
            assert vals <= {None, rand(900, 1)}
        elif case in ("noncodeword", "ragged"):
            assert vals == {None}
        elif case == "bad_frame":
            assert vals == {po.ERR_PROTOCOL}
    finally:
        tw.close()
