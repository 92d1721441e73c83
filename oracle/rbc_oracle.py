"""CPU oracle for the Cleisthenes RBC data path -- TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The shipped path (``cleisthenes_amd`` -> ``librbc_gpu.so``) never routes
through here and fails loudly when the HIP library is missing.

What it restates
----------------
* ``rbc/rbc.go:97-100`` ``shard(enc, data)``  = ``enc.Split`` + ``enc.Encode``
* ``rbc/rbc.go:92-95`` ``validateMessage(echo)`` = Merkle branch verify
* ``rbc/rbc.go:86-90`` ``interpolate(rootHash, shards)`` = reconstruct,
  re-encode, re-commit, compare the root
* ``rbc/rbc.go:20`` ``enc reedsolomon.Encoder``: the third-party
  ``github.com/klauspost/reedsolomon v1.9.1`` (``go.mod:10``, ``go.sum:17-18``),
  which is NOT vendored in /root/reference.  Its published algorithm (the
  Backblaze JavaReedSolomon construction) is restated below: GF(2^8) with
  generating polynomial 0x11D (``generatingPolynomial = 29``), generator 2,
  encode matrix ``vandermonde(N, k) * inverse(top k x k)``, Split/Encode/
  Verify/Reconstruct/ReconstructData/Join with v1.9.1 argument checks.
* SHA-256 is Go ``crypto/sha256`` == FIPS 180-4 == ``hashlib.sha256``.

Parity pinning (see DESIGN.md "Oracle")
---------------------------------------
* GF(2^8) and matrix inversion: pinned by klauspost's own unit-test vectors
  (galois_test.go / matrix_test.go) and by the v1.9.1 ``TestOneEncode``
  codeword (5+5 shards); all are asserted in ``tests/test_oracle.py``.
* SHA-256: FIPS 180-4 known answers.
* Merkle tree / branch / interpolate root recheck: the reference has NO code
  for it (``rbc/rbc.go`` is all ``panic`` stubs, tests empty).  The convention
  is frozen here (HBBFT, as cited by ``docs/RBC-EN.md:31-38``) and is
  "parity unpinned" beyond SHA-256 itself.

Frozen Merkle / RBC spec (DESIGN.md section 3 repeats it)
--------------------------------------------------------
* leaf_j = SHA-256(s_j), exactly S bytes of shard j (zero pad included).
* bottom width W = 2**ceil(log2 N) (W = 1 for N = 1), depth d = log2 W.
  Slots j >= N are EMPTY byte strings (not hashed).
* node = SHA-256(left || right), byte concatenation, an empty child adds
  nothing (so SHA-256 of 64, 32 or 0 bytes).
* branch_j = d siblings, leaf -> root; only the level-0 sibling can be empty
  (exactly when j ^ 1 >= N).  Flat ``Branch []byte`` (``rbc/request.go:11``)
  = concatenation of the non-empty siblings.
* verify: h = SHA-256(s); for level l: h = SHA-256(br || h) if bit l of j is 1
  else SHA-256(h || br); valid iff h == root.
* interpolate: klauspost rule (first k present shards by index) to recover
  the k data shards, then a FULL re-encode of all N shards, Merkle root over
  the re-encoding must equal rootHash (else ROOT_MISMATCH); value = the k
  data shards concatenated (k*S bytes, pad kept -- the length is not carried).
* batch digest = SHA-256(leaf_0 || ... || leaf_{k-1}) over the data-shard
  leaves of the re-encoding (commits to the value; parallel-hashable).
"""
from __future__ import annotations

import hashlib
from typing import List, Optional, Sequence

import numpy as np

# ----------------------------------------------------------------------------
# Errors: klauspost/reedsolomon v1.9.1 error values (reedsolomon.go) plus the
# two the RBC layer adds.  Names match the Go identifiers.
# ----------------------------------------------------------------------------


class RSError(Exception):
    code = -100


class ErrInvShardNum(RSError):
    code = -1


class ErrMaxShardNum(RSError):
    code = -2


class ErrTooFewShards(RSError):
    code = -3


class ErrShardNoData(RSError):
    code = -4


class ErrShardSize(RSError):
    code = -5


class ErrShortData(RSError):
    code = -6


class ErrReconstructRequired(RSError):
    code = -7


class ErrRootMismatch(RSError):
    code = -8


class ErrSingular(RSError):
    code = -11


class ErrInvalidInput(RSError):
    code = -13


# ----------------------------------------------------------------------------
# GF(2^8), generating polynomial x^8+x^4+x^3+x^2+1 (0x11D), generator 2.
# klauspost galois.go: logTable/expTable, galMultiply, galDivide, galExp.
# ----------------------------------------------------------------------------

POLY = 0x11D


def _build_tables():
    exp = np.zeros(512, dtype=np.int32)
    log = np.zeros(256, dtype=np.int32)
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= POLY
    for i in range(255, 512):
        exp[i] = exp[i - 255]
    return exp, log


EXP, LOG = _build_tables()


def gal_mul(a: int, b: int) -> int:
    """galMultiply (galois.go)."""
    if a == 0 or b == 0:
        return 0
    return int(EXP[(LOG[a] + LOG[b]) % 255])


def gal_div(a: int, b: int) -> int:
    """galDivide (galois.go): a==0 -> 0, b==0 -> panic."""
    if a == 0:
        return 0
    if b == 0:
        raise ZeroDivisionError("Argument 'divisor' is 0")
    r = LOG[a] - LOG[b]
    if r < 0:
        r += 255
    return int(EXP[r])


def gal_exp(a: int, n: int) -> int:
    """galExp (galois.go): exp(., 0) = 1, exp(0, n>0) = 0."""
    if n == 0:
        return 1
    if a == 0:
        return 0
    return int(EXP[(LOG[a] * n) % 255])


# Full 256x256 product table (mulTable in galois.go).
MUL = np.zeros((256, 256), dtype=np.uint8)
for _a in range(1, 256):
    for _b in range(1, 256):
        MUL[_a, _b] = EXP[(LOG[_a] + LOG[_b]) % 255]
del _a, _b


# ----------------------------------------------------------------------------
# Matrices (klauspost matrix.go)
# ----------------------------------------------------------------------------


def mat_identity(n: int) -> np.ndarray:
    return np.eye(n, dtype=np.uint8)


def mat_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """matrix.Multiply: GF(2^8) product."""
    rows, inner = a.shape
    inner2, cols = b.shape
    assert inner == inner2
    out = np.zeros((rows, cols), dtype=np.uint8)
    for r in range(rows):
        acc = np.zeros(cols, dtype=np.uint8)
        for i in range(inner):
            if a[r, i]:
                acc ^= MUL[a[r, i], b[i]]
        out[r] = acc
    return out


def mat_invert(m: np.ndarray) -> np.ndarray:
    """matrix.Invert: Gauss-Jordan on [m | I] (gaussianElimination)."""
    n = m.shape[0]
    assert m.shape == (n, n)
    work = np.concatenate([m.astype(np.uint8), mat_identity(n)], axis=1)
    for r in range(n):
        if work[r, r] == 0:
            for below in range(r + 1, n):
                if work[below, r] != 0:
                    work[[r, below]] = work[[below, r]]
                    break
        if work[r, r] == 0:
            raise ErrSingular("matrix is singular")
        if work[r, r] != 1:
            scale = gal_div(1, int(work[r, r]))
            work[r] = MUL[scale, work[r]]
        for below in range(r + 1, n):
            if work[below, r] != 0:
                work[below] ^= MUL[work[below, r], work[r]]
    for d in range(n):
        for above in range(d):
            if work[above, d] != 0:
                work[above] ^= MUL[work[above, d], work[d]]
    return work[:, n:].copy()


def vandermonde(rows: int, cols: int) -> np.ndarray:
    """matrix.go vandermonde: v[r][c] = galExp(r, c)."""
    v = np.zeros((rows, cols), dtype=np.uint8)
    for r in range(rows):
        for c in range(cols):
            v[r, c] = gal_exp(r, c)
    return v


def build_matrix(data_shards: int, total_shards: int) -> np.ndarray:
    """reedsolomon.go buildMatrix: vandermonde(total, data) * top^-1."""
    vm = vandermonde(total_shards, data_shards)
    top_inv = mat_invert(vm[:data_shards, :data_shards])
    return mat_mul(vm, top_inv)


def gf_rows(coef: np.ndarray, inputs: Sequence[np.ndarray]) -> List[np.ndarray]:
    """out[r] = XOR_j coef[r][j] * inputs[j]  (codeSomeShards)."""
    outs = []
    for r in range(coef.shape[0]):
        acc = np.zeros(len(inputs[0]), dtype=np.uint8)
        for j, x in enumerate(inputs):
            c = int(coef[r, j])
            if c:
                acc ^= MUL[c, x]
        outs.append(acc)
    return outs


# ----------------------------------------------------------------------------
# Encoder: reedsolomon.Encoder (v1.9.1) restated.
# ----------------------------------------------------------------------------

_MATRIX_CACHE = {}


def encode_matrix(k: int, n: int) -> np.ndarray:
    key = (k, n)
    if key not in _MATRIX_CACHE:
        _MATRIX_CACHE[key] = build_matrix(k, n)
    return _MATRIX_CACHE[key]


def _as_u8(s) -> np.ndarray:
    if s is None:
        return np.zeros(0, dtype=np.uint8)
    if isinstance(s, np.ndarray):
        return s.astype(np.uint8, copy=False)
    return np.frombuffer(bytes(s), dtype=np.uint8)


def _shard_size(shards) -> int:
    for s in shards:
        if s is not None and len(s) != 0:
            return len(s)
    return 0


def _check_shards(shards, nilok: bool) -> None:
    size = _shard_size(shards)
    if size == 0:
        raise ErrShardNoData("no shard data")
    for s in shards:
        ln = 0 if s is None else len(s)
        if ln != size:
            if ln != 0 or not nilok:
                raise ErrShardSize("shard sizes do not match")


class Encoder:
    """reedsolomon.New(dataShards, parityShards) (reedsolomon.go New)."""

    def __init__(self, data_shards: int, parity_shards: int):
        if data_shards <= 0 or parity_shards < 0:
            raise ErrInvShardNum("cannot create Encoder with zero or less data/parity shards")
        if data_shards + parity_shards > 256:
            raise ErrMaxShardNum("cannot create Encoder with more than 256 data+parity shards")
        self.data_shards = data_shards
        self.parity_shards = parity_shards
        self.shards = data_shards + parity_shards
        self.m = encode_matrix(data_shards, self.shards)
        self.parity = self.m[data_shards:]

    # Split (reedsolomon.go Split); callers pass cap == len so the pad is zero.
    def split(self, data) -> List[np.ndarray]:
        d = _as_u8(data)
        if len(d) == 0:
            raise ErrShortData("not enough data to fill the number of requested shards")
        per = (len(d) + self.data_shards - 1) // self.data_shards
        buf = np.zeros(self.shards * per, dtype=np.uint8)
        buf[: len(d)] = d
        return [buf[i * per:(i + 1) * per].copy() for i in range(self.shards)]

    def encode(self, shards: List[np.ndarray]) -> None:
        if len(shards) != self.shards:
            raise ErrTooFewShards("too few shards given")
        _check_shards(shards, False)
        data = [_as_u8(s) for s in shards[: self.data_shards]]
        outs = gf_rows(self.parity, data)
        for i, o in enumerate(outs):
            shards[self.data_shards + i] = o

    def verify(self, shards) -> bool:
        if len(shards) != self.shards:
            raise ErrTooFewShards("too few shards given")
        _check_shards(shards, False)
        data = [_as_u8(s) for s in shards[: self.data_shards]]
        outs = gf_rows(self.parity, data)
        return all(np.array_equal(o, _as_u8(shards[self.data_shards + i])) for i, o in enumerate(outs))

    def _reconstruct(self, shards, data_only: bool) -> None:
        if len(shards) != self.shards:
            raise ErrTooFewShards("too few shards given")
        _check_shards(shards, True)
        size = _shard_size(shards)
        present = [s is not None and len(s) != 0 for s in shards]
        if sum(present) == self.shards:
            return
        if sum(present) < self.data_shards:
            raise ErrTooFewShards("too few shards given")
        valid = [i for i in range(self.shards) if present[i]][: self.data_shards]
        sub = self.m[valid, :]
        dec = mat_invert(sub)
        sub_shards = [_as_u8(shards[i]) for i in valid]
        missing_data = [i for i in range(self.data_shards) if not present[i]]
        if missing_data:
            outs = gf_rows(dec[missing_data, :], sub_shards)
            for i, o in zip(missing_data, outs):
                shards[i] = o
        if data_only:
            return
        missing_par = [i for i in range(self.data_shards, self.shards) if not present[i]]
        if missing_par:
            data = [_as_u8(shards[i]) for i in range(self.data_shards)]
            outs = gf_rows(self.m[missing_par, :], data)
            for i, o in zip(missing_par, outs):
                shards[i] = o
        assert all(len(s) == size for s in shards)

    # Update (reedsolomon.go Update / updateParityShards, v1.9.1): parity +=
    # M[k+r][c] * (old_c ^ new_c) for every changed data shard c (new_c non-nil).
    # As in Go, the old data shard in `shards` is left holding old ^ new
    # (sliceXor(in, oldin) writes into oldin).
    def update(self, shards, new_data) -> None:
        # v1.9.1 reedsolomon.go Update: len(shards) != r.Shards and
        # len(newDatashards) != r.DataShards are both ErrTooFewShards
        if len(shards) != self.shards:
            raise ErrTooFewShards("too few shards given")
        if len(new_data) != self.data_shards:
            raise ErrTooFewShards("too few shards given")
        _check_shards(shards, True)
        _check_shards(new_data, True)
        for i in range(len(new_data)):
            if new_data[i] is not None and len(new_data[i]) and (shards[i] is None or len(shards[i]) == 0):
                raise ErrInvalidInput("invalid input")
        for pi in range(self.data_shards, self.shards):
            if shards[pi] is None or len(shards[pi]) == 0:
                raise ErrInvalidInput("invalid input")
        size = _shard_size(shards)
        for c in range(self.data_shards):
            nd = new_data[c]
            if nd is None or len(nd) == 0:
                continue
            nd = _as_u8(nd)
            if len(nd) != size:  # Go would index past a shorter shard; reported as a size mismatch
                raise ErrShardSize("shard sizes do not match")
            delta = _as_u8(shards[c]) ^ nd
            shards[c] = delta
            for r in range(self.parity_shards):
                (outs,) = gf_rows(self.parity[r:r + 1, c:c + 1], [delta])
                shards[self.data_shards + r] = _as_u8(shards[self.data_shards + r]) ^ outs

    def reconstruct(self, shards) -> None:
        self._reconstruct(shards, False)

    def reconstruct_data(self, shards) -> None:
        self._reconstruct(shards, True)

    def join(self, shards, out_size: int) -> bytes:
        if len(shards) < self.data_shards:
            raise ErrTooFewShards("too few shards given")
        shards = shards[: self.data_shards]
        size = 0
        for s in shards:
            if s is None:
                raise ErrReconstructRequired(
                    "reconstruction required as one or more required data shards are nil")
            size += len(s)
            if size >= out_size:
                break
        if size < out_size:
            raise ErrShortData("not enough data to fill the number of requested shards")
        out = bytearray()
        write = out_size
        for s in shards:
            b = bytes(_as_u8(s))
            if write < len(b):
                out += b[:write]
                return bytes(out)
            out += b
            write -= len(b)
        return bytes(out)


# ----------------------------------------------------------------------------
# Merkle (frozen HBBFT convention, see module docstring)
# ----------------------------------------------------------------------------


def sha256(b) -> bytes:
    return hashlib.sha256(bytes(b)).digest()


def tree_width(n: int) -> int:
    w = 1
    while w < n:
        w <<= 1
    return w


def tree_depth(n: int) -> int:
    return tree_width(n).bit_length() - 1


def merkle_tree(leaves_data: Sequence) -> List[bytes]:
    """mt[1] = root, mt[W + j] = leaf j (b'' beyond N)."""
    n = len(leaves_data)
    w = tree_width(n)
    mt = [b""] * (2 * w)
    for j in range(n):
        mt[w + j] = sha256(leaves_data[j])
    for i in range(w - 1, 0, -1):
        mt[i] = sha256(mt[2 * i] + mt[2 * i + 1])
    return mt


def merkle_tree_from_leaves(leaves: Sequence[bytes]) -> List[bytes]:
    n = len(leaves)
    w = tree_width(n)
    mt = [b""] * (2 * w)
    for j in range(n):
        mt[w + j] = bytes(leaves[j])
    for i in range(w - 1, 0, -1):
        mt[i] = sha256(mt[2 * i] + mt[2 * i + 1])
    return mt


def merkle_branch(mt: List[bytes], index: int) -> List[bytes]:
    res = []
    t = index + (len(mt) >> 1)
    while t > 1:
        res.append(mt[t ^ 1])
        t >>= 1
    return res


def flat_branch(branch: List[bytes]) -> bytes:
    return b"".join(branch)


def unflatten_branch(flat: bytes, index: int, n: int) -> Optional[List[bytes]]:
    """Inverse of flat_branch given (index, N); None if the length is wrong."""
    d = tree_depth(n)
    empty0 = d > 0 and (index ^ 1) >= n
    want = 32 * (d - (1 if empty0 else 0))
    if len(flat) != want:
        return None
    out = []
    off = 0
    for lvl in range(d):
        if lvl == 0 and empty0:
            out.append(b"")
        else:
            out.append(bytes(flat[off:off + 32]))
            off += 32
    return out


def merkle_verify(n: int, val, root: bytes, branch: List[bytes], index: int) -> bool:
    """validateMessage (rbc/rbc.go:92-95) restated, HBBFT merkleVerify."""
    if index < 0 or index >= n or len(branch) != tree_depth(n):
        return False
    tmp = sha256(val)
    t = index
    for br in branch:
        tmp = sha256(br + tmp) if (t & 1) else sha256(tmp + br)
        t >>= 1
    return tmp == bytes(root)


# ----------------------------------------------------------------------------
# RBC data path (rbc/rbc.go stubs, restated)
# ----------------------------------------------------------------------------


def rbc_shard(enc: Encoder, data) -> List[np.ndarray]:
    """shard(enc, data) (rbc/rbc.go:97-100): Split then Encode."""
    shards = enc.split(data)
    enc.encode(shards)
    return shards


def rbc_commit(shards) -> dict:
    """Merkle build for VAL construction (rbc/rbc.go:42 broadcast)."""
    mt = merkle_tree(shards)
    n = len(shards)
    return {
        "root": mt[1],
        "branches": [merkle_branch(mt, j) for j in range(n)],
        "leaves": mt[tree_width(n):tree_width(n) + n],
    }


def batch_digest(data_leaves: Sequence[bytes]) -> bytes:
    return sha256(b"".join(bytes(x) for x in data_leaves))


def rbc_interpolate(enc: Encoder, root: bytes, shards) -> dict:
    """interpolate(rootHash, shards) (rbc/rbc.go:86-90), frozen spec.

    Returns {"value": bytes (k*S), "digest": bytes, "root": recomputed root}.
    Raises ErrTooFewShards / ErrShardSize / ErrShardNoData / ErrRootMismatch.
    """
    k = enc.data_shards
    if len(shards) != enc.shards:
        raise ErrTooFewShards("too few shards given")
    work = [None if (s is None or len(s) == 0) else _as_u8(s).copy() for s in shards]
    present = sum(1 for s in work if s is not None)
    if present < k:
        raise ErrTooFewShards("too few shards given")
    enc.reconstruct_data(work)          # first k present by index
    data = [work[i] for i in range(k)]
    full = data + gf_rows(enc.parity, data)   # FULL re-encode
    mt = merkle_tree(full)
    leaves = mt[tree_width(enc.shards):tree_width(enc.shards) + enc.shards]
    if mt[1] != bytes(root):
        raise ErrRootMismatch("interpolated merkle root mismatch")
    return {
        "value": b"".join(bytes(d) for d in data),
        "digest": batch_digest(leaves[:k]),
        "root": mt[1],
    }


def parity_k(n: int, f: int):
    """(k, p) for an RBC instance: k = N - 2f data shards, p = 2f parity."""
    return n - 2 * f, 2 * f


def shard_len(value_len: int, k: int) -> int:
    return (value_len + k - 1) // k
