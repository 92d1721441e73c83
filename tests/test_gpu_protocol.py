"""The RBC state machine (include/rbc_protocol.h) over the GPU data path.

An in-process network of N nodes per proposer exchanges marshaled
pb.Message bytes; every shard / validateMessage / interpolate goes through
one shared rbc_batcher, so concurrent instances share launches.  Cases follow
the HBBFT reliable-broadcast properties (docs/RBC-EN.md): every honest node
delivers the proposer's value with f silent or lying nodes; nothing is
delivered for a proposal that is not a codeword; an equivocating proposer
cannot make honest nodes deliver different values.  Delivered values are
checked byte-for-byte against the proposer's input: the node frames the
value with its length before Split (interpolate alone returns k*S bytes with
the zero pad, rbc/rbc.go:86-90).
"""
import numpy as np
import pytest

import rbc_oracle as orc

pytestmark = pytest.mark.gpu


class Net:
    """Nodes[(proposer, i)] for the given proposers; `tamper(p, src, dst, msg)`
    may rewrite or drop (None) any message in flight."""

    def __init__(self, ca, n, f, proposers, tamper=None, max_batch=1024, max_wait_us=5000, keep=0):
        from cleisthenes_amd import protocol
        self.protocol = protocol
        self.ctx = ca.Context(n, f)
        self.bt = ca.Batcher(self.ctx, max_batch=max_batch, max_wait_us=max_wait_us)
        if keep:  # ABI 7: validated ECHO rows stay on the device for the interpolates
            self.bt.set_keep(keep)
        self.n, self.f = n, f
        self.nodes = {(p, i): protocol.Node(self.bt, n, f, i, p) for p in proposers for i in range(n)}
        self.tamper = tamper
        self.rejected_at_handle = 0

    def post(self, p, src, dst, msg):
        if self.tamper is not None:
            msg = self.tamper(p, src, dst, msg)
            if msg is None:
                return
        rc = self.nodes[(p, dst)].handle_message(src, msg)
        self.rejected_at_handle += rc != 0

    def deliver(self):
        moved = False
        for (p, i), node in self.nodes.items():
            for to, msg in node.messages():
                moved = True
                for dst in (range(self.n) if to < 0 else [to]):
                    if dst != i:
                        self.post(p, i, dst, msg)
        return moved

    def run(self, max_rounds=500):
        """Deliver until quiet: no message in flight and no GPU work pending."""
        for _ in range(max_rounds):
            moved = self.deliver()
            pending = sum(nd.progress(wait=not moved) for nd in self.nodes.values())
            if not moved and pending == 0 and not self.deliver():
                return
        raise AssertionError("network did not quiesce")

    def close(self):
        for nd in self.nodes.values():
            nd.close()
        self.bt.close()
        self.ctx.close()


@pytest.fixture(scope="module")
def ca(gpu):
    return gpu


def rand(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


@pytest.mark.parametrize("n,f,B", [(4, 1, 1024), (4, 1, 1000), (7, 2, 333), (16, 5, 65536), (4, 1, 0), (4, 1, 1)])
def test_honest_network_delivers(ca, n, f, B):
    net = Net(ca, n, f, proposers=[0])
    try:
        v = rand(B, n)
        net.nodes[(0, 0)].propose(v)
        net.run()
        k = n - 2 * f
        for i in range(n):
            nd = net.nodes[(0, i)]
            assert nd.value() == v, i
            st = nd.stats()
            assert st["ready_sent"] and st["echoes"] == n and st["readies"] == n and st["rejected"] == 0
        assert net.rejected_at_handle == 0
    finally:
        net.close()


@pytest.mark.parametrize("keep", [0, 64 << 20])
def test_all_proposers_concurrently_share_launches(ca, keep):
    """An ACS round: N proposers x N nodes = 256 instances, one batcher; with
    keep, the batcher keeps validated ECHO rows on the device (ABI 7) and the
    round must deliver the same values."""
    n, f = 16, 5
    net = Net(ca, n, f, proposers=list(range(n)), keep=keep)
    try:
        vals = {p: rand(4096 + 17 * p, 100 + p) for p in range(n)}
        for p in range(n):
            net.nodes[(p, p)].propose(vals[p])
        net.run()
        for (p, i), nd in net.nodes.items():
            assert nd.value() == vals[p], (p, i)
        batches, requests = net.bt.stats()
        # 16 shards + 16*15 VAL + 16*16*15 ECHO validations + >= 256 interpolations
        assert requests >= 16 + 240 + 3840 + 256
        assert requests / batches >= 8, (batches, requests)
    finally:
        net.close()


@pytest.mark.parametrize("mode", ["silent", "bad_echo", "bad_ready"])
def test_f_byzantine_nodes_cannot_block_or_forge(ca, mode):
    n, f = 7, 2
    byz = {5, 6}
    ready_forged = {}

    def tamper(p, src, dst, msg):
        if src not in byz:
            return msg
        if mode == "silent":
            return None
        t, payload = net.protocol.pb_decode(msg)
        if mode == "bad_echo" and t == net.protocol.ECHO:
            d = net.protocol.json_decode_val(payload)
            blk = bytearray(d["Block"][0])
            blk[dst % len(blk)] ^= 0x5A
            return net.protocol.pb_encode(t, net.protocol.json_encode_val(d["RootHash"], d["Branch"], bytes(blk)))
        if mode == "bad_ready" and t == net.protocol.ECHO:
            # lie: READY for a root nobody proposed, and no ECHO at all
            fake = bytes(32 * [src])
            ready_forged[src] = fake
            return net.protocol.pb_encode(net.protocol.READY, net.protocol.json_encode_ready(fake))
        return msg

    net = Net(ca, n, f, proposers=[0], tamper=tamper)
    try:
        v = rand(5000, 3)
        net.nodes[(0, 0)].propose(v)
        net.run()
        for i in range(n):
            if i in byz:
                continue
            nd = net.nodes[(0, i)]
            assert nd.value() == v, (mode, i)
            st = nd.stats()
            if mode == "bad_echo":
                assert st["rejected"] == len(byz)  # each lying ECHO failed validateMessage
                assert st["echoes"] == n - len(byz)
    finally:
        net.close()


def _vals_for(ctx, value):
    c = ctx.shard(value)
    return c["root"], c["branches"], c["shards"]


def test_equivocating_proposer_cannot_split_honest_nodes(ca):
    """Proposer n-1 sends root A to nodes 0..n-f-1 and root B to the rest."""
    n, f = 7, 2
    P = n - 1
    net = Net(ca, n, f, proposers=[P])
    try:
        pr = net.protocol
        va, vb = rand(3000, 11), rand(3000, 12)
        ra, ba, sa = _vals_for(net.ctx, pr.frame(va))
        rb, bb, sb = _vals_for(net.ctx, pr.frame(vb))
        for j in range(n - 1):
            root, br, sh = (ra, ba, sa) if j < n - f else (rb, bb, sb)
            rc = net.nodes[(P, j)].handle_message(P, pr.pb_encode(pr.VAL, pr.json_encode_val(root, br[j],
                                                                                          bytes(sh[j]))))
            assert rc == 0
        net.run()
        got = {net.nodes[(P, j)].value() for j in range(n - 1)}
        assert got == {va}
    finally:
        net.close()


def test_noncodeword_proposal_is_never_delivered(ca):
    """Consistent Merkle proofs over shards that are not a codeword: every
    node validates its shard, reaches N-f ECHOs, fails the interpolate root
    recheck, and never sends READY (HBBFT's abort)."""
    n, f = 7, 2
    P = 0
    net = Net(ca, n, f, proposers=[P])
    try:
        pr = net.protocol
        shards = [bytearray(s) for s in _vals_for(net.ctx, rand(2000, 21))[2]]
        shards[n - 1][0] ^= 1  # one parity byte: no longer a codeword
        mt = orc.merkle_tree([bytes(s) for s in shards])
        root = mt[1]
        for j in range(1, n):
            br = orc.flat_branch([b for b in orc.merkle_branch(mt, j) if b])
            net.nodes[(P, j)].handle_message(P, pr.pb_encode(pr.VAL, pr.json_encode_val(root, br, bytes(shards[j]))))
        net.run()
        for j in range(1, n):
            nd = net.nodes[(P, j)]
            st = nd.stats()
            assert nd.value() is None and not st["ready_sent"], j
            assert st["echoes"] == n - 1 and st["rejected"] == 0
    finally:
        net.close()


def test_out_of_protocol_messages_are_dropped(ca):
    n, f = 4, 1
    net = Net(ca, n, f, proposers=[0])
    try:
        pr = net.protocol
        r, br, sh = _vals_for(net.ctx, rand(999, 5))
        nd = net.nodes[(0, 1)]
        val = pr.pb_encode(pr.VAL, pr.json_encode_val(r, br[1], bytes(sh[1])))
        assert nd.handle_message(2, val) != 0           # VAL from a non-proposer
        assert nd.handle_message(0, val) == 0
        assert nd.handle_message(0, val) != 0           # second VAL
        echo = pr.pb_encode(pr.ECHO, pr.json_encode_val(r, br[2], bytes(sh[2])))
        assert nd.handle_message(2, echo) == 0
        assert nd.handle_message(2, echo) != 0          # duplicate ECHO
        assert nd.handle_message(3, b"\x1a\x01") != 0   # malformed pb
        assert nd.handle_message(3, pr.pb_encode(pr.READY, b"{}")) != 0  # READY without a root
        nd.progress(wait=True)
        st = nd.stats()
        assert st["echoes"] == 2 and st["rejected"] == 5  # own ECHO + node 2's
        with pytest.raises(Exception):
            net.nodes[(0, 2)].propose(b"x")             # only the proposer proposes
    finally:
        net.close()


def test_badly_framed_proposal_is_agreed_but_unusable(ca):
    """A Byzantine proposer commits (consistently) to a payload whose length
    frame exceeds the decoded bytes: every honest node still delivers (RBC
    agreement holds) and every one reports the same protocol error."""
    n, f = 4, 1
    P = 0
    net = Net(ca, n, f, proposers=[P])
    try:
        pr = net.protocol
        bad = (10 ** 9).to_bytes(8, "little") + rand(500, 31)  # claims 1e9 bytes
        r, br, sh = _vals_for(net.ctx, bad)
        for j in range(1, n):
            net.nodes[(P, j)].handle_message(P, pr.pb_encode(pr.VAL, pr.json_encode_val(r, br[j], bytes(sh[j]))))
        net.run()
        for j in range(1, n):
            with pytest.raises(Exception) as ei:
                net.nodes[(P, j)].value()
            assert getattr(ei.value, "code", None) == -20
            assert net.nodes[(P, j)].stats()["ready_sent"]
    finally:
        net.close()
