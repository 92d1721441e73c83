"""Host binding of the RBC state machine and wire codec (include/rbc_protocol.h).

* ``pb_encode`` / ``pb_decode``      -> pb.Message{rbc: pb.RBC{payload, type}} (pb/message.proto:11-35)
* ``json_encode_val`` / ``..._ready`` -> Go encoding/json of ValRequest / EchoRequest / ReadyRequest
                                       (rbc/request.go:9-21)
* ``Node``                          -> one RBC instance at one node (rbc/rbc.go:9-100: NewRBC,
                                       HandleMessage, Value, Messages)

The codec is host-only; a ``Node`` does its shard / validateMessage /
interpolate work on the GPU through a shared ``Batcher``.
"""
from __future__ import annotations

import struct
from ctypes import byref, c_int, c_size_t, c_void_p
from typing import List, Optional, Tuple

import numpy as np

from ._lib import RBC_ERR_INVALID_ARG, RBC_ERR_PROTOCOL, RBCError, check, lib
from .rbc import Batcher, _bytes_array, _ptr

VAL, ECHO, READY = 0, 1, 2


def frame(value: bytes) -> bytes:
    """The payload a Node broadcasts for `value`: [u64 little-endian len][value]
    (rbc_node_propose), so delivery can return exactly the proposed bytes."""
    return struct.pack("<Q", len(value)) + bytes(value)


def _buf(x) -> Tuple[np.ndarray, Optional[c_void_p]]:
    a = _bytes_array(x)
    return a, (_ptr(a) if len(a) else None)


def _emit(fn, *args) -> bytes:
    need = fn(*args, None, 0)
    out = np.zeros(max(need, 1), np.uint8)
    got = fn(*args, _ptr(out), need)
    assert got == need
    return bytes(out[:need])


def pb_encode(msg_type: int, payload: bytes) -> bytes:
    p, pp = _buf(payload)
    return _emit(lib.rbc_pb_encode_rbc, msg_type, pp, len(p))


def pb_decode(msg: bytes) -> Tuple[int, bytes]:
    m, mp = _buf(msg)
    t, pl, n = c_int(0), c_void_p(), c_size_t(0)
    check(lib.rbc_pb_decode_rbc(mp, len(m), byref(t), byref(pl), byref(n)), "rbc_pb_decode_rbc")
    if not n.value:
        return t.value, b""
    off = pl.value - m.ctypes.data
    return t.value, bytes(m[off:off + n.value])


def json_encode_val(root: bytes, branch: bytes, block: bytes) -> bytes:
    r, rp = _buf(root)
    b, bp = _buf(branch)
    k, kp = _buf(block)
    return _emit(lib.rbc_json_encode_val, rp, len(r), bp, len(b), kp, len(k))


def json_encode_ready(root: bytes) -> bytes:
    r, rp = _buf(root)
    return _emit(lib.rbc_json_encode_ready, rp, len(r))


def json_decode_val(js: bytes) -> dict:
    j, jp = _buf(js)
    root = np.zeros(32, np.uint8)
    bl, kl = c_size_t(0), c_size_t(0)
    rc = lib.rbc_json_decode_val(jp, len(j), _ptr(root), None, 0, byref(bl), None, 0, byref(kl))
    if rc not in (0, RBC_ERR_INVALID_ARG):  # INVALID_ARG here: the size query
        raise RBCError(rc, "rbc_json_decode_val")
    br, blk = np.zeros(max(bl.value, 1), np.uint8), np.zeros(max(kl.value, 1), np.uint8)
    check(lib.rbc_json_decode_val(jp, len(j), _ptr(root), _ptr(br), bl.value, byref(bl), _ptr(blk), kl.value,
                                  byref(kl)), "rbc_json_decode_val")
    return {"RootHash": bytes(root), "Branch": bytes(br[:bl.value]), "Block": [bytes(blk[:kl.value])]}


def json_decode_ready(js: bytes) -> bytes:
    j, jp = _buf(js)
    root = np.zeros(32, np.uint8)
    check(lib.rbc_json_decode_ready(jp, len(j), _ptr(root)), "rbc_json_decode_ready")
    return bytes(root)


class Node:
    """One RBC instance (proposer ``proposer``'s broadcast) at node ``self_id``."""

    def __init__(self, batcher: Batcher, n: int, f: int, self_id: int, proposer: int):
        p = c_void_p()
        check(lib.rbc_node_create(batcher._p, n, f, self_id, proposer, byref(p)), "rbc_node_create")
        self._p = p
        self.batcher = batcher  # keeps the batcher alive while the node is
        self.n, self.f, self.self_id, self.proposer = n, f, self_id, proposer

    def close(self) -> None:
        if getattr(self, "_p", None):
            lib.rbc_node_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def propose(self, value: bytes) -> None:
        v, vp = _buf(value)
        check(lib.rbc_node_propose(self._p, vp, len(v)), "rbc_node_propose")

    def handle_message(self, sender: int, msg: bytes) -> int:
        """Returns the status (RBC_OK, or RBC_ERR_PROTOCOL for a dropped message)."""
        m, mp = _buf(msg)
        rc = lib.rbc_node_handle_message(self._p, sender, mp, len(m))
        if rc not in (0, RBC_ERR_PROTOCOL):
            raise RBCError(rc, "rbc_node_handle_message")
        return rc

    def progress(self, wait: bool = False) -> int:
        pending = c_int(0)
        check(lib.rbc_node_progress(self._p, 1 if wait else 0, byref(pending)), "rbc_node_progress")
        return pending.value

    def messages(self) -> List[Tuple[int, bytes]]:
        """Drains the outgoing queue: [(to, pb bytes)], to = -1 for everyone else."""
        out = []
        buf = np.zeros(1 << 16, np.uint8)
        while True:
            to, n = c_int(0), c_size_t(0)
            rc = lib.rbc_node_next_message(self._p, byref(to), _ptr(buf), buf.nbytes, byref(n))
            if rc == RBC_ERR_INVALID_ARG and n.value > buf.nbytes:
                buf = np.zeros(n.value, np.uint8)
                continue
            check(rc, "rbc_node_next_message")
            if n.value == 0:
                return out
            out.append((to.value, bytes(buf[:n.value])))

    def value(self) -> Optional[bytes]:
        """The delivered value (exactly the proposer's bytes), None before
        delivery; RBCError(RBC_ERR_PROTOCOL) if the agreed payload is badly
        framed (a Byzantine proposer)."""
        n, d = c_size_t(0), c_int(0)
        check(lib.rbc_node_value(self._p, None, 0, byref(n), byref(d)), "rbc_node_value")
        if not d.value:
            return None
        buf = np.zeros(max(n.value, 1), np.uint8)
        check(lib.rbc_node_value(self._p, _ptr(buf), buf.nbytes, byref(n), byref(d)), "rbc_node_value")
        return bytes(buf[:n.value])

    def stats(self) -> dict:
        e, r, s, x = c_int(0), c_int(0), c_int(0), c_int(0)
        check(lib.rbc_node_stats(self._p, byref(e), byref(r), byref(s), byref(x)), "rbc_node_stats")
        return {"echoes": e.value, "readies": r.value, "ready_sent": bool(s.value), "rejected": x.value}
