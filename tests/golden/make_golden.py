"""Generate the committed golden fixtures for the RBC data path.

Run:  python tests/golden/make_golden.py   (writes tests/golden/rbc_golden.json)

The vectors come from oracle/rbc_oracle.py, the CPU restatement of
klauspost/reedsolomon v1.9.1 + crypto/sha256 + the frozen HBBFT Merkle spec.
The reference's own tests for this path are empty (rbc/rbc_internal_test.go:
21-31) and its RS dependency is not vendored, so the only reference-held
answers are klauspost's unit-test vectors, which are checked separately in
tests/test_oracle.py (KNOWN_ANSWERS).  These fixtures freeze the oracle's
outputs so any later change to oracle or product shows up as a diff.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import rbc_oracle as orc  # noqa: E402

SEED = 20261015


def hx(b) -> str:
    return bytes(b).hex()


def case_commit(n, f, value_len, seed):
    rng = np.random.default_rng(seed)
    value = rng.integers(0, 256, value_len, dtype=np.uint8)
    k, p = orc.parity_k(n, f)
    enc = orc.Encoder(k, p)
    shards = orc.rbc_shard(enc, value)
    com = orc.rbc_commit(shards)
    return {
        "kind": "commit",
        "n": n, "f": f, "value": hx(value),
        "shard_len": len(shards[0]),
        "shards": [hx(s) for s in shards],
        "leaves": [hx(x) for x in com["leaves"]],
        "root": hx(com["root"]),
        # N=256 branches are 256 B each: keep them for one geometry only
        "branches": ([hx(orc.flat_branch(b)) for b in com["branches"]]
                     if (n < 256 or value_len == 300) else None),
    }, enc, value, shards, com


def interp_case(name, n, f, enc, shards, com, present, root=None, tamper=None):
    """present: list of indices given to interpolate; tamper: {idx: xor byte0}."""
    given = [None] * n
    for j in present:
        s = shards[j].copy()
        if tamper and j in tamper:
            s[0] ^= tamper[j]
        given[j] = s
    rt = com["root"] if root is None else root
    out = {"kind": "interpolate", "name": name, "n": n, "f": f,
           "present": sorted(int(j) for j in present),
           "tamper": {str(k): v for k, v in (tamper or {}).items()},
           "root": hx(rt)}
    try:
        r = orc.rbc_interpolate(enc, rt, given)
        out.update(status=0, value=hx(r["value"]), digest=hx(r["digest"]))
    except orc.RSError as e:
        out.update(status=e.code)
    return out


def main():
    cases = []
    rng = np.random.default_rng(SEED)
    geoms = [
        (4, 1, 1024),      # C0: the reference's Go-test plumbing shape
        (4, 1, 1),
        (7, 2, 333),       # non power of two N: empty padding leaves
        (16, 5, 1001),     # odd B
        (13, 4, 129),
        (64, 21, 2000),
        (128, 42, 3000),
        (256, 85, 1),      # Split edge: S = 1
        (256, 85, 85),
        (256, 85, 86),
        (256, 85, 87),
        (256, 85, 300),
        (5, 0, 77),        # f = 0: no parity
        (1, 0, 10),        # N = 1: depth 0
    ]
    for gi, (n, f, B) in enumerate(geoms):
        c, enc, value, shards, com = case_commit(n, f, B, SEED + gi)
        cases.append(c)
        k = n - 2 * f
        perm = rng.permutation(n)
        if k < n:
            cases.append(interp_case("random_k", n, f, enc, shards, com, perm[:k]))
            cases.append(interp_case("parity_only", n, f, enc, shards, com, list(range(n - k, n))
                                     if n - k >= k else list(range(k, n)) + list(range(n - k))[: 2 * k - n]))
            cases.append(interp_case("data_only", n, f, enc, shards, com, list(range(k))))
            cases.append(interp_case("k_minus_1", n, f, enc, shards, com, perm[: k - 1]))
            cases.append(interp_case("mixed_k_plus_f", n, f, enc, shards, com, perm[: min(n, k + f)]))
            cases.append(interp_case("wrong_root", n, f, enc, shards, com, perm[:k], root=b"\x11" * 32))
            # Byzantine: a corrupted shard among the first k present -> decoded
            # value differs -> root mismatch (full re-encode recheck)
            first = sorted(perm[:k])
            cases.append(interp_case("tampered_used", n, f, enc, shards, com, perm[:k], tamper={int(first[0]): 0x5a}))
            # a corrupted present shard that is NOT among the first k: ignored
            # by klauspost's rule, overwritten by the re-encoding -> ok
            extra = sorted(perm[: min(n, k + 1)])
            if len(extra) > k:
                cases.append(interp_case("tampered_unused", n, f, enc, shards, com, extra,
                                         tamper={int(extra[-1]): 0x5a}))
        else:
            cases.append(interp_case("all_present", n, f, enc, shards, com, list(range(n))))

    # Byzantine proposer: commits to a vector that is not a codeword.  Every
    # honest receiver must reject it whatever subset it decodes from.
    n, f = 16, 5
    k = n - 2 * f
    value = rng.integers(0, 256, 600, dtype=np.uint8)
    enc = orc.Encoder(k, 2 * f)
    shards = orc.rbc_shard(enc, value)
    shards[n - 1] = shards[n - 1].copy()
    shards[n - 1][7] ^= 0xFF
    com = orc.rbc_commit(shards)
    cases.append({"kind": "commit", "n": n, "f": f, "value": hx(value), "shard_len": len(shards[0]),
                  "shards": [hx(s) for s in shards], "leaves": [hx(x) for x in com["leaves"]],
                  "root": hx(com["root"]), "branches": [hx(orc.flat_branch(b)) for b in com["branches"]],
                  "byzantine_noncodeword": True})
    for sub in (list(range(k)), list(range(n - k, n)), sorted(rng.permutation(n)[:k].tolist())):
        cases.append(interp_case("noncodeword", n, f, enc, shards, com, sub))

    # validateMessage vectors: valid, flipped shard byte, flipped branch byte,
    # wrong index, truncated branch
    c = [x for x in cases if x["kind"] == "commit" and x["n"] == 16 and not x.get("byzantine_noncodeword")][0]
    n = c["n"]
    vm = []
    for j in range(n):
        vm.append({"index": j, "shard": c["shards"][j], "branch": c["branches"][j], "root": c["root"], "ok": True})
    s = bytearray(bytes.fromhex(c["shards"][2])); s[5] ^= 1
    vm.append({"index": 2, "shard": s.hex(), "branch": c["branches"][2], "root": c["root"], "ok": False})
    b = bytearray(bytes.fromhex(c["branches"][9])); b[40] ^= 0x80
    vm.append({"index": 9, "shard": c["shards"][9], "branch": b.hex(), "root": c["root"], "ok": False})
    vm.append({"index": 4, "shard": c["shards"][5], "branch": c["branches"][5], "root": c["root"], "ok": False})
    vm.append({"index": 1, "shard": c["shards"][1], "branch": c["branches"][1][:-64], "root": c["root"], "ok": False})
    c7 = cases[[i for i, x in enumerate(cases) if x["kind"] == "commit" and x["n"] == 7][0]]
    for j in range(7):  # N=7: leaf 6's level-0 sibling is empty (omitted from the flat branch)
        vm.append({"index": j, "shard": c7["shards"][j], "branch": c7["branches"][j], "root": c7["root"], "ok": True,
                   "n": 7, "f": 2})
    for v in vm:
        v.setdefault("n", 16)
        v.setdefault("f", 5)
    # sanity: the oracle agrees with every expectation
    for v in vm:
        br = orc.unflatten_branch(bytes.fromhex(v["branch"]), v["index"], v["n"])
        ok = br is not None and orc.merkle_verify(v["n"], bytes.fromhex(v["shard"]), bytes.fromhex(v["root"]), br,
                                                   v["index"])
        assert ok == v["ok"], v
    out = {"seed": SEED, "generator": "tests/golden/make_golden.py (oracle/rbc_oracle.py)",
           "cases": cases, "validate": vm}
    path = os.path.join(HERE, "rbc_golden.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=0, sort_keys=True)
    print(f"wrote {path}: {len(cases)} cases, {len(vm)} validate vectors, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
