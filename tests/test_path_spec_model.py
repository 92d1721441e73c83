"""CPU model of merkle_path_kernel's speculative top levels
(cleisthenes_amd/csrc/kernels.hip), checked against
the per-leaf branch walk of validateMessage (oracle/rbc_oracle.py
merkle_verify, rbc/rbc.go:92-95).

At W = 256 the kernel runs levels 0 and 1 of every walk exactly, then hashes
every node above level 2 at once from the values the branches claim for its
children, and declares the instance proven (every participating leaf valid)
only if (i) the participants under each level-l node (l >= 2) hold the same
level-l entry, (ii) they reached the same exact level-2 value, equal to the
claim for that node where one exists, and (iii) every node hash equals its
claim, the root at the top.  Otherwise it re-runs levels 2..7 exactly.  The
model restates that rule and requires: proven => every participant's own
walk reaches the root (soundness, so valid[] stays bit-identical to the walk);
every honest reception is proven (the fast path is the common path); and the
chain of node hashes that wait on another one is never deeper than the six
passes the kernel allows.  The GPU test of the kernel itself is
tests/test_gpu_parity.py::test_device_verify_speculative_top_levels.
"""
import numpy as np
import pytest

import rbc_oracle as orc

W, D, L0 = 256, 8, 2


def _walk(leaf, br, j, upto):
    h = leaf
    for lvl in range(upto):
        h = orc.sha256(br[lvl] + h) if (j >> lvl) & 1 else orc.sha256(h + br[lvl])
    return h


def spec_rule(n, leaves, brs, part, root):
    """The kernel's rule.  Returns (proven, passes of node hashes)."""
    def has(lvl, v):
        return any(part[j] for j in range(v << lvl, min((v + 1) << lvl, n)))

    def rep(lvl, v):
        return next(j for j in range(v << lvl, min((v + 1) << lvl, n)) if part[j])

    ok = True
    for lvl in range(L0, D):  # (i)
        for j in range(n):
            if part[j] and brs[j][lvl] != brs[rep(lvl, j >> lvl)][lvl]:
                ok = False
    x2 = {j: _walk(leaves[j], brs[j], j, L0) for j in range(n) if part[j]}
    X = {}
    for v in range(W >> L0):  # (ii), first half
        if has(L0, v):
            X[v] = x2[rep(L0, v)]
            ok = ok and all(x2[j] == X[v] for j in x2 if j >> L0 == v)

    def claim(lvl, v):
        return brs[rep(lvl, v ^ 1)][lvl]

    inputs, deps = {}, {}
    for m in range(L0 + 1, D + 1):
        for P in range(W >> m):
            lvl = m - 1
            h = [has(lvl, 2 * P), has(lvl, 2 * P + 1)]
            if not any(h):
                continue
            inp = [None, None]
            for k in range(2):
                c = 2 * P + k
                if lvl == L0 and h[k]:
                    inp[k] = X[c]
                    if h[1 - k]:
                        ok = ok and claim(lvl, c) == X[c]  # (ii), second half
                elif h[1 - k]:
                    inp[k] = claim(lvl, c)
                else:
                    deps[(m, P, k)] = (lvl, c)
            inputs[(m, P)] = inp
    out, passes = {}, 0
    while len(out) < len(inputs):  # one pass hashes every task whose inputs are known
        ready = [t for t in inputs if t not in out and all(
            inputs[t][k] is not None or out.get(deps[(t[0], t[1], k)]) is not None for k in range(2))]
        assert ready, "a dependency cycle cannot happen"
        for (m, P) in ready:
            inp = [inputs[(m, P)][k] if inputs[(m, P)][k] is not None else out[deps[(m, P, k)]] for k in range(2)]
            out[(m, P)] = orc.sha256(inp[0] + inp[1])
        passes += 1
    for (m, P), hval in out.items():  # (iii)
        if m == D:
            ok = ok and hval == root
        elif has(m, P ^ 1):
            ok = ok and hval == claim(m, P)
    return ok, passes


def _instance(rng, n):
    data = [rng.integers(0, 256, 12, dtype=np.uint8).tobytes() for _ in range(n)]
    mt = orc.merkle_tree(data)
    leaves = [mt[W + j] for j in range(n)]
    brs = [orc.merkle_branch(mt, j) for j in range(n)]
    return leaves, brs, mt[1]


def _tamper(rng, n, leaves, brs, root, part):
    brs = [list(b) for b in brs]
    leaves = list(leaves)
    kind = int(rng.integers(9))
    if kind == 0:  # one slot at a random level
        j, lvl = int(rng.integers(n)), int(rng.integers(D))
        if brs[j][lvl]:
            brs[j][lvl] = bytes([brs[j][lvl][0] ^ 1]) + brs[j][lvl][1:]
    elif kind == 1:  # a whole subtree agrees on a wrong sibling at its level
        lvl = int(rng.integers(L0, D))
        v = int(rng.integers(W >> lvl))
        bad = orc.sha256(b"x" + bytes([lvl, v & 255]))
        for j in range(v << lvl, min((v + 1) << lvl, n)):
            brs[j][lvl] = bad
    elif kind == 2:  # a wrong leaf (corrupted shard)
        j = int(rng.integers(n))
        leaves[j] = orc.sha256(leaves[j])
    elif kind == 3:  # wrong root
        root = bytes([root[0] ^ 1]) + root[1:]
    elif kind == 4:  # a spliced subtree from another tree, consistent inside
        l2, b2, _ = _instance(rng, n)
        lvl = int(rng.integers(1, D))
        v = int(rng.integers(W >> lvl))
        for j in range(v << lvl, min((v + 1) << lvl, n)):
            leaves[j], brs[j] = l2[j], list(b2[j])
    return leaves, brs, root


@pytest.mark.parametrize("n", [256, 200, 129])
def test_spec_rule_is_sound_and_proves_honest_receptions(n):
    rng = np.random.default_rng(4000 + n)
    trials = {256: 40, 200: 30, 129: 30}[n]
    seen = {"honest": 0, "tampered_proven": 0, "fallback": 0, "deep": 0}
    for t in range(trials):
        leaves, brs, root = _instance(rng, n)
        part = np.zeros(n, bool)
        mode = t % 4
        if mode == 0:
            part[:] = True
        elif mode == 1:  # N - f present, random
            part[rng.permutation(n)[: n - (n - 1) // 3]] = True
        elif mode == 2:  # whole blocks absent (claims missing: dependent hashes)
            part[:] = True
            blk = 1 << int(rng.integers(3, 8))
            v = int(rng.integers(max(1, n // blk)))
            part[v * blk:(v + 1) * blk] = False
        else:  # sparse
            part[rng.random(n) < rng.uniform(0.01, 0.5)] = True
        honest = t % 2 == 0
        if not honest:
            leaves, brs, root = _tamper(rng, n, leaves, brs, root, part)
        proven, passes = spec_rule(n, leaves, brs, part, root)
        assert passes <= D - L0
        walk = [bool(part[j]) and _walk(leaves[j], brs[j], j, D) == root for j in range(n)]
        if proven:  # soundness: the fast path only ever claims what the walks give
            assert all(walk[j] for j in range(n) if part[j]), (n, t)
        if honest:
            assert proven, (n, t, mode)
            seen["honest"] += 1
        else:
            seen["tampered_proven" if proven else "fallback"] += 1
        seen["deep"] += passes > 1
    assert seen["honest"] and seen["fallback"] and seen["deep"], seen


def test_spec_rule_single_participant_chain():
    """One participant: every node above level 2 waits on the one below it --
    six passes, the kernel's bound -- and the leaf is still proven."""
    rng = np.random.default_rng(9)
    leaves, brs, root = _instance(rng, 256)
    part = np.zeros(256, bool)
    part[137] = True
    proven, passes = spec_rule(256, leaves, brs, part, root)
    assert proven and passes == D - L0
