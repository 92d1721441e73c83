"""ctypes wrapper of oracle/librbc_ref.so (the C restatement) -- TEST
INFRASTRUCTURE ONLY: used by tests/ as a fast checker at full sizes and by
bench.py's cpu_baseline leg.  Never imported by the product package."""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_int, c_int32, c_size_t, c_uint8, c_uint32, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "librbc_ref.so")


def load():
    if not os.path.exists(LIB):
        import subprocess
        subprocess.run(["make", "-C", HERE], check=True, capture_output=True)
    lib = ctypes.CDLL(LIB)
    lib.rbcref_encode_matrix.argtypes = [c_int, c_int, c_void_p]
    lib.rbcref_invert.argtypes = [c_int, c_void_p, c_void_p]
    lib.rbcref_gf_rows.argtypes = [c_int, c_int, c_void_p, c_void_p, c_void_p, c_size_t]
    lib.rbcref_gf_rows.restype = None
    lib.rbcref_sha256.argtypes = [c_void_p, c_size_t, c_void_p]
    lib.rbcref_sha256.restype = None
    lib.rbcref_merkle_from_leaves.argtypes = [c_int, c_void_p, c_void_p, c_void_p]
    lib.rbcref_merkle_from_leaves.restype = None
    lib.rbcref_merkle_verify.argtypes = [c_int, c_void_p, c_size_t, c_uint32, c_void_p, c_void_p]
    lib.rbcref_encode_commit.argtypes = [c_int, c_int, c_void_p, c_size_t, c_void_p, c_size_t, c_void_p, c_void_p,
                                         c_void_p]
    lib.rbcref_interpolate.argtypes = [c_int, c_int, c_void_p, c_size_t, c_size_t, c_void_p, c_void_p, c_void_p,
                                       c_void_p]
    lib.rbcref_pipeline.argtypes = [c_int, c_int, c_int, c_size_t, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                    POINTER(c_int)]
    lib.rbcref_pipeline.restype = c_double
    lib.rbcref_pipeline2.argtypes = [c_int, c_int, c_int, c_size_t, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                     POINTER(c_int), POINTER(c_double), POINTER(c_double)]
    lib.rbcref_pipeline2.restype = c_double
    lib.rbcref_interpolate_leaves.argtypes = [c_int, c_int, c_void_p, c_size_t, c_size_t, c_void_p, c_void_p,
                                              c_void_p, c_void_p, c_void_p]
    lib.rbcref_tree_depth.argtypes = [c_int]
    lib.rbcref_cpu_features.restype = c_int
    lib.rbcref_force_scalar.argtypes = [c_int]
    lib.rbcref_force_scalar.restype = None
    lib.rbcref_verify_many.argtypes = [c_int, c_size_t, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int,
                                       c_void_p]
    lib.rbcref_verify_many.restype = c_double
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = load()
    return _lib


def p(a: np.ndarray) -> c_void_p:
    return c_void_p(a.ctypes.data)


def sha256(b) -> bytes:
    a = np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else np.ascontiguousarray(b)
    out = np.zeros(32, dtype=np.uint8)
    lib().rbcref_sha256(p(a) if a.size else None, a.size, p(out))
    return bytes(out)


def encode_matrix(k: int, n: int) -> np.ndarray:
    out = np.zeros(n * k, dtype=np.uint8)
    rc = lib().rbcref_encode_matrix(k, n, p(out))
    assert rc == 0
    return out.reshape(n, k)


def encode_commit(n: int, f: int, value: np.ndarray):
    """-> shards [n][S], root, branches [n][d][32], leaves [n][32]"""
    k = n - 2 * f
    B = len(value)
    S = (B + k - 1) // k
    d = lib().rbcref_tree_depth(n)
    shards = np.zeros((n, S), dtype=np.uint8)
    root = np.zeros(32, dtype=np.uint8)
    br = np.zeros((n, max(d, 1), 32), dtype=np.uint8)
    leaves = np.zeros((n, 32), dtype=np.uint8)
    value = np.ascontiguousarray(value, dtype=np.uint8)
    rc = lib().rbcref_encode_commit(n, f, p(value), B, p(shards), S, p(root), p(br), p(leaves))
    assert rc == 0, rc
    return shards, bytes(root), br[:, :d], leaves


def verify(n: int, shard: np.ndarray, index: int, branch_slots: np.ndarray, root: bytes) -> bool:
    shard = np.ascontiguousarray(shard, dtype=np.uint8)
    b = np.ascontiguousarray(branch_slots, dtype=np.uint8)
    r = np.frombuffer(root, dtype=np.uint8).copy()
    return bool(lib().rbcref_merkle_verify(n, p(shard), shard.size, index, p(b) if b.size else None, p(r)))


def interpolate(n: int, f: int, shards: np.ndarray, valid: np.ndarray, root: bytes):
    """shards [n][S]; valid [n] -> (status, value k*S, digest)"""
    k = n - 2 * f
    shards = np.ascontiguousarray(shards, dtype=np.uint8)
    S = shards.shape[1]
    v = np.ascontiguousarray(valid, dtype=np.uint8)
    r = np.frombuffer(root, dtype=np.uint8).copy()
    value = np.zeros(k * S, dtype=np.uint8)
    dig = np.zeros(32, dtype=np.uint8)
    rc = lib().rbcref_interpolate(n, f, p(shards), S, S, p(v), p(r), p(value), p(dig))
    return rc, value, bytes(dig)


def interpolate_leaves(n: int, f: int, shards: np.ndarray, valid: np.ndarray, leaves: np.ndarray, root: bytes):
    """interpolate reusing the verified leaves of valid shards -> (status, value, digest)"""
    k = n - 2 * f
    shards = np.ascontiguousarray(shards, dtype=np.uint8)
    S = shards.shape[1]
    v = np.ascontiguousarray(valid, dtype=np.uint8)
    lv = np.ascontiguousarray(leaves, dtype=np.uint8)
    r = np.frombuffer(root, dtype=np.uint8).copy()
    value = np.zeros(k * S, dtype=np.uint8)
    dig = np.zeros(32, dtype=np.uint8)
    rc = lib().rbcref_interpolate_leaves(n, f, p(shards), S, S, p(v), p(lv), p(r), p(value), p(dig))
    return rc, value, bytes(dig)


def pipeline(n, f, count, B, threads, values, present, corrupt, phases=False):
    """values: [nvals][B]; instance i encodes values[i % nvals].  -> (wall
    seconds, status sum[, encode+commit thread-seconds, verify+decode
    thread-seconds])"""
    st = c_int(0)
    es, ds = c_double(0), c_double(0)
    values = np.ascontiguousarray(values, dtype=np.uint8)
    secs = lib().rbcref_pipeline2(n, f, count, B, threads, p(values), values.shape[0], p(present), p(corrupt),
                                  ctypes.byref(st), ctypes.byref(es), ctypes.byref(ds))
    if phases:
        return secs, st.value, es.value, ds.value
    return secs, st.value


def verify_many(n, shards, branches, roots, inst, j, threads):
    """validateMessage of messages (inst[m], j[m]) over a committed set
    (shards [I][n][S], branches [I][n][d][32], roots [I][32]) on `threads`
    host threads -> (wall seconds, ok [count])."""
    shards = np.ascontiguousarray(shards, dtype=np.uint8)
    branches = np.ascontiguousarray(branches, dtype=np.uint8)
    roots = np.ascontiguousarray(roots, dtype=np.uint8)
    inst = np.ascontiguousarray(inst, dtype=np.int32)
    j = np.ascontiguousarray(j, dtype=np.int32)
    ok = np.zeros(len(inst), dtype=np.uint8)
    secs = lib().rbcref_verify_many(n, shards.shape[2], p(shards), p(branches), p(roots), len(inst), p(inst), p(j),
                                    threads, p(ok))
    return secs, ok
