"""CPU model of the receive step's node-reuse root recheck
(cleisthenes_amd/csrc/kernels.hip merkle_recheck_kernel, DESIGN.md section
5.4b), checked against the full recheck of the frozen interpolate spec
(oracle/rbc_oracle.py rbc_interpolate: interpolate, rbc/rbc.go:86-90).

The model restates the kernel's rule on the oracle's Merkle functions:
hash only the nodes of the maximal subtrees that hold no valid ECHO leaf,
compare each such subtree's root with the branch entry of the first valid
leaf under its sibling, require the root the branches were verified against
to equal the expected root, and fall back to the whole tree when the decode
changed a valid row.  Random honest and adversarial receptions (absent rows,
corrupted shards, corrupted branch slots, non-codeword commitments, a root
changed after the verify, non-power-of-two N) must give the same status as
the full recheck.  The GPU test of the kernel itself is
tests/test_gpu_parity.py::test_receive_step_node_reuse_recheck_equals_full_recheck.
"""
import numpy as np
import pytest

import rbc_oracle as orc


def _reception(rng, n, f, B):
    k = n - 2 * f
    enc = orc.Encoder(k, n - k)
    value = rng.integers(0, 256, B, dtype=np.uint8)
    shards = orc.rbc_shard(enc, value)
    noncodeword = rng.random() < 0.25
    if noncodeword:  # a Byzantine proposer commits to a vector that is not a codeword
        shards[int(rng.integers(n))][int(rng.integers(len(shards[0])))] ^= 0x21
    com = orc.rbc_commit(shards)
    root = com["root"]
    present = np.zeros(n, bool)
    present[rng.permutation(n)[: int(rng.integers(k, n + 1))]] = True
    rx = [s.copy() for s in shards]
    branches = [list(b) for b in com["branches"]]
    for j in np.flatnonzero(present):
        u = rng.random()
        if u < 0.05:
            rx[j][int(rng.integers(len(rx[j])))] ^= 0x40  # corrupted ECHO shard
        elif u < 0.10 and branches[j]:
            lvl = int(rng.integers(len(branches[j])))
            if branches[j][lvl]:
                b = bytearray(branches[j][lvl])
                b[int(rng.integers(32))] ^= 0x08  # corrupted branch slot
                branches[j][lvl] = bytes(b)
    expect = root if rng.random() < 0.85 else bytes([root[0] ^ 1]) + root[1:]  # changed after the verify
    return enc, rx, branches, present, root, expect, noncodeword


def _decode(enc, rx, valid):
    n, k = enc.shards, enc.data_shards
    work = [rx[j].copy() if valid[j] else None for j in range(n)]
    enc.reconstruct_data(work)  # klauspost: the first k valid rows by index
    data = [work[i] for i in range(k)]
    full = data + orc.gf_rows(enc.parity, data)
    used = np.flatnonzero(valid)[:k]
    flagged = [j for j in np.flatnonzero(valid) if j not in used and not np.array_equal(full[j], rx[j])]
    return full, flagged


def reuse_recheck(n, full, rx, valid, branches, verified_root, expect_root, flagged):
    """The kernel's rule.  Returns (ok, node hashes done)."""
    if flagged:  # the decode changed a valid row: the full recheck
        return orc.merkle_tree(full)[1] == expect_root, None
    W, d = orc.tree_width(n), orc.tree_depth(n)
    hv = [False] * (2 * W)  # has a valid leaf, heap order (leaves at W + j)
    for j in range(n):
        hv[W + j] = bool(valid[j])
    for i in range(W - 1, 0, -1):
        hv[i] = hv[2 * i] or hv[2 * i + 1]
    E, hashed = {}, 0

    def e(i):  # the re-encoding's node i, only inside valid-free subtrees
        nonlocal hashed
        if i >= W:
            return orc.sha256(full[i - W]) if i - W < n else b""
        if i not in E:
            E[i] = orc.sha256(e(2 * i) + e(2 * i + 1))
            hashed += 1
        return E[i]

    ok = True
    for lvl in range(d):
        m = W >> lvl
        for i in range(m, 2 * m):
            if hv[i] or not hv[i >> 1] or (lvl == 0 and i - m >= n):
                continue  # only an empty leaf is forced by the walk; padding nodes above are compared
            s = i ^ 1
            while s < W:  # the first valid leaf under the sibling
                s = 2 * s if hv[2 * s] else 2 * s + 1
            ok = ok and e(i) == branches[s - W][lvl]
    return ok and verified_root == expect_root, hashed


@pytest.mark.parametrize("n,f", [(4, 1), (7, 2), (16, 5), (33, 10), (64, 21), (100, 33), (128, 42)])
def test_node_reuse_recheck_equals_full_recheck(n, f):
    rng = np.random.default_rng(1000 + n)
    k = n - 2 * f
    trials = {4: 300, 7: 300, 16: 200, 33: 120, 64: 60, 100: 40, 128: 30}[n]
    seen = {"ok": 0, "mismatch": 0, "fallback": 0}
    for _ in range(trials):
        B = int(rng.integers(1, 40 * k))
        enc, rx, branches, present, root, expect, noncw = _reception(rng, n, f, B)
        valid = np.array([present[j] and orc.merkle_verify(n, rx[j], root, branches[j], j) for j in range(n)])
        if valid.sum() < k:
            continue  # TOO_FEW_SHARDS before any recheck
        full, flagged = _decode(enc, rx, valid)
        want = orc.merkle_tree(full)[1] == expect
        got, hashed = reuse_recheck(n, full, rx, valid, branches, root, expect, flagged)
        assert got == want, (n, f, B, noncw, list(np.flatnonzero(~valid)), flagged)
        seen["fallback" if hashed is None else ("ok" if got else "mismatch")] += 1
        if hashed is not None:  # never more node hashes than the valid-free subtrees hold
            assert hashed <= orc.tree_width(n) - 1
    # every branch of the rule was exercised
    assert seen["ok"] and seen["mismatch"] and seen["fallback"], seen


def byzantine_padding_commit(leaf_hashes, n, overrides):
    """A proposer's tree whose padding node(s) at level >= 1 hold chosen
    values (heap index -> 32 bytes) instead of the standard empty-subtree
    hash; every ECHO walk still verifies, because the walk takes those nodes
    from the branches.  Returns (root, branches)."""
    W = orc.tree_width(n)
    mt = [b""] * (2 * W)
    for j in range(n):
        mt[W + j] = bytes(leaf_hashes[j])
    for i in range(W - 1, 0, -1):
        mt[i] = overrides.get(i, orc.sha256(mt[2 * i] + mt[2 * i + 1]))
    return mt[1], [orc.merkle_branch(mt, j) for j in range(n)]


def padding_nodes(n):
    """Heap indices of the all-padding nodes at levels 1 .. d-1."""
    W, d = orc.tree_width(n), orc.tree_depth(n)
    out = []
    for lvl in range(1, d):
        m = W >> lvl
        out += [(i, lvl) for i in range(m, 2 * m) if ((i - m) << lvl) >= n]
    return out


@pytest.mark.parametrize("n,f", [(33, 10), (100, 33), (13, 4), (200, 66)])
def test_node_reuse_rejects_a_byzantine_padding_node(n, f):
    """a proposer that commits to a non-standard padding
    node at level >= 1 passes every ECHO verify; the full recheck rebuilds the
    tree with standard padding and rejects it.  The reuse rule must reject it
    too whether or not a valid leaf sits under the padding node's parent --
    otherwise two honest receivers disagree on delivery."""
    rng = np.random.default_rng(77 + n)
    k = n - 2 * f
    W = orc.tree_width(n)
    enc = orc.Encoder(k, n - k)
    cases = 0
    for i_pad, lvl in padding_nodes(n):
        shards = orc.rbc_shard(enc, rng.integers(0, 256, 3 * k + 5, dtype=np.uint8))
        leaves = [orc.sha256(s) for s in shards]
        root, branches = byzantine_padding_commit(leaves, n, {i_pad: bytes(rng.integers(0, 256, 32, dtype=np.uint8))})
        assert all(orc.merkle_verify(n, shards[j], root, branches[j], j) for j in range(n))
        sib = i_pad ^ 1  # the real leaves under the padding node's sibling
        lo, hi = (sib << lvl) - W, min(n, ((sib + 1) << lvl) - W)
        if lo >= n:
            continue  # the parent is padding too: the case of a higher node
        for under_parent in (True, False):
            valid = np.zeros(n, bool)
            valid[rng.permutation(n)[: n - f]] = True
            valid[lo:hi] = False
            if under_parent:
                valid[lo] = True
            if valid.sum() < k:
                continue
            full, flagged = _decode(enc, shards, valid)
            want = orc.merkle_tree(full)[1] == root
            assert not want  # the full recheck rebuilds standard padding
            got, _ = reuse_recheck(n, full, shards, valid, branches, root, root, flagged)
            assert got == want, (n, i_pad, lvl, under_parent)
            cases += 1
    assert cases >= 2


def test_node_reuse_hashes_few_nodes_at_the_bench_shapes():
    """At C2 / C4's reception (N - f of N received, all honest) the rule hashes
    a small fraction of the W - 1 internal nodes the full recheck hashes."""
    rng = np.random.default_rng(7)
    for n, f, bound in ((128, 42, 0.35), (256, 85, 0.2)):
        k = n - 2 * f
        enc = orc.Encoder(k, n - k)
        counts = []
        for _ in range(3):
            shards = orc.rbc_shard(enc, rng.integers(0, 256, 4 * k, dtype=np.uint8))
            com = orc.rbc_commit(shards)
            valid = np.zeros(n, bool)
            valid[rng.permutation(n)[: n - f]] = True
            full, flagged = _decode(enc, shards, valid)
            ok, hashed = reuse_recheck(n, full, shards, valid, com["branches"], com["root"], com["root"], flagged)
            assert ok and not flagged
            counts.append(hashed)
        assert max(counts) <= bound * (orc.tree_width(n) - 1), (n, counts)
