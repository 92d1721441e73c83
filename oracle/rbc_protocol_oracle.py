"""CPU oracle for the RBC state machine above the data path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module; the product state machine is
``cleisthenes_amd/csrc/rbc_node.cpp`` behind ``include/rbc_protocol.h``.

What it restates, independently of that C++ (pure Python over
``rbc_oracle``'s RS codec and Merkle functions, no GPU):

* the wire codec: ``pb.Message{rbc: pb.RBC{payload, type}}`` in protobuf
  wire format (pb/message.proto:11-35; the generated code carries RBC.type
  as field 2, pb/message.pb.go:182-183) and the Go ``encoding/json`` form of
  ValRequest / EchoRequest / ReadyRequest (rbc/request.go:9-21): fields in
  struct order, ``[]byte`` as padded standard base64, nil as ``null``, keys
  matched case-insensitively on decode, unknown keys skipped;
* the HBBFT reliable broadcast at one node (docs/RBC-EN.md:31-44), in the
  shape rbc/rbc.go:9-100 declares (NewRBC, HandleMessage with
  handleValueRequest / handleEchoRequest / handleReadyRequest, Value,
  Messages):
    - VAL(h, b_i, s_i) from the proposer: validateMessage at our own index,
      then ECHO(h, b_i, s_i) to every other node, the proposer included,
      and our own ECHO counted locally.  This is the HBBFT paper's rule
      (Miller et al. 2016, Algorithm RBC: "multicast ECHO(h, b_i, s_i)",
      i.e. to all parties) and deliberately NOT docs/RBC-EN.md:34, which
      sends ECHO "to the node except the sender and itself": a proposer that
      receives no ECHO can never reach step 5 (RBC-EN.md:42, "wait for N-2f
      ECHO messages and decode"), so it would not deliver its own broadcast
      and totality fails; and a node that does not count its own shard needs
      N-f ECHOs from only N-1 peers.  The product does the same
      (csrc/rbc_node.cpp on_val); DESIGN.md section 5.7 records the deviation;
    - ECHO from node j counts iff validateMessage proves s_j at leaf j
      under h (RBC-EN.md:35); one VAL / ECHO / READY per sender;
    - N-f valid ECHOs for h: interpolate, and on a root match READY(h)
      (RBC-EN.md:36-39); f+1 READY(h): READY(h) (RBC-EN.md:41);
    - 2f+1 READY(h) with N-2f valid ECHOs: interpolate and deliver
      (RBC-EN.md:42);
* the decisions the reference leaves open (its handlers are stubs), as
  DESIGN.md section 5.7 fixes them: the broadcast payload is framed
  ``[u64 LE len][value]`` before Split; an interpolate that fails (root
  mismatch, ragged shards) marks the root failed for good; a badly framed
  delivered payload is delivered but unusable (RBC_ERR_PROTOCOL).

GPU work in the product is asynchronous (submitted to a batcher, applied in
submission order by ``progress``).  The oracle models exactly that with a
FIFO of deferred operations, so a test can drive both in lock step and
compare every outgoing message byte for byte.

Parity: the reference has no RBC implementation or tests
(rbc/rbc_internal_test.go:21-31), so this oracle is "parity unpinned" beyond
the codec rules pinned by the protobuf runtime in tests/test_protocol_codec.py.
"""
from __future__ import annotations

import base64
import json
from collections import deque
from typing import Dict, List, Optional, Tuple

import numpy as np

import rbc_oracle as orc

VAL, ECHO, READY = 0, 1, 2
ERR_PROTOCOL = -20
FRAME = 8

# ----------------------------------------------------------------------------
# protobuf wire format
# ----------------------------------------------------------------------------


def _varint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def pb_encode(msg_type: int, payload: bytes) -> bytes:
    """Message{rbc (field 3): RBC{payload (1, bytes), type (2, enum)}}; proto3
    omits empty / zero scalars, the oneof member is always written."""
    body = b""
    if payload:
        body += b"\x0a" + _varint(len(payload)) + bytes(payload)
    if msg_type:
        body += b"\x10" + _varint(msg_type)
    return b"\x1a" + _varint(len(body)) + body


class _Bad(Exception):
    pass


def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    v = 0
    for sh in range(0, 64, 7):
        if i >= len(b):
            raise _Bad()
        c = b[i]
        i += 1
        v |= (c & 0x7F) << sh
        if not c & 0x80:
            return v & ((1 << 64) - 1), i
    raise _Bad()


def _skip(b: bytes, i: int, wire: int) -> int:
    if wire == 0:
        return _read_varint(b, i)[1]
    if wire == 1:
        if len(b) - i < 8:
            raise _Bad()
        return i + 8
    if wire == 2:
        n, i = _read_varint(b, i)
        if n > len(b) - i:
            raise _Bad()
        return i + n
    if wire == 5:
        if len(b) - i < 4:
            raise _Bad()
        return i + 4
    raise _Bad()


def pb_decode(msg: bytes) -> Optional[Tuple[int, bytes]]:
    """(type, payload) of a Message carrying an RBC, None if malformed or not
    an RBC.  Protobuf merge rules: a repeated RBC field merges (later scalars
    win), a BBA field (4) switches the oneof away, unknown fields skipped."""
    b = bytes(msg)
    try:
        i, is_rbc, t, pl = 0, False, 0, b""
        while i < len(b):
            key, i = _read_varint(b, i)
            field, wire = key >> 3, key & 7
            if field == 0:
                raise _Bad()
            if field in (3, 4) and wire == 2:
                n, i = _read_varint(b, i)
                if n > len(b) - i:
                    raise _Bad()
                body, i = b[i:i + n], i + n
                if field == 4:
                    is_rbc, t, pl = False, 0, b""
                    continue
                is_rbc = True
                j = 0
                while j < len(body):
                    k2, j = _read_varint(body, j)
                    f2, w2 = k2 >> 3, k2 & 7
                    if f2 == 0:
                        raise _Bad()
                    if f2 == 1 and w2 == 2:
                        m, j = _read_varint(body, j)
                        if m > len(body) - j:
                            raise _Bad()
                        pl, j = body[j:j + m], j + m
                    elif f2 == 2 and w2 == 0:
                        t, j = _read_varint(body, j)
                    else:
                        j = _skip(body, j, w2)
            else:
                i = _skip(b, i, wire)
        if not is_rbc or t > READY:
            return None
        return t, pl
    except _Bad:
        return None


# ----------------------------------------------------------------------------
# Go encoding/json of the request structs
# ----------------------------------------------------------------------------

_B64 = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"


def _jbytes(x: bytes) -> str:
    return "null" if not x else '"' + base64.b64encode(bytes(x)).decode() + '"'


def json_encode_val(root: bytes, branch: bytes, block: bytes) -> bytes:
    blk = "null" if not block else '["' + base64.b64encode(bytes(block)).decode() + '"]'
    return ('{"RootHash":' + _jbytes(root) + ',"Branch":' + _jbytes(branch) + ',"Block":' + blk + "}").encode()


def json_encode_ready(root: bytes) -> bytes:
    return ('{"RootHash":' + _jbytes(root) + "}").encode()


def _b64_decode(s: str) -> bytes:
    """base64.StdEncoding.DecodeString as encoding/json uses it: padding
    required, CR/LF ignored, non-zero trailing bits tolerated."""
    s = s.replace("\r", "").replace("\n", "")
    if len(s) % 4:
        raise _Bad()
    out = bytearray()
    for i in range(0, len(s), 4):
        q = s[i:i + 4]
        pad = 0
        if i + 4 == len(s) and q[3] == "=":
            pad = 2 if q[2] == "=" else 1
        v = 0
        for j in range(4):
            if j < 4 - pad:
                c = _B64.find(q[j])
                if c < 0:
                    raise _Bad()
            else:
                c = 0
            v = (v << 6) | c
        out += bytes([v >> 16, (v >> 8) & 255, v & 255])[:3 - pad]
    return bytes(out)


def _field_bytes(v) -> bytes:
    if v is None:
        return b""
    if not isinstance(v, str):
        raise _Bad()
    return _b64_decode(v)


def _no_constant(_):
    raise _Bad()


def json_decode(payload: bytes) -> Optional[dict]:
    """json.Unmarshal into the request shape: {"root", "branch", "block": [..]}
    (later duplicate keys win), None if malformed."""
    try:
        # invalid UTF-8 is kept (encoding/json substitutes U+FFFD): it can
        # only make a key unknown or a base64 string undecodable
        pairs = json.loads(bytes(payload).decode("utf-8", "surrogateescape"), object_pairs_hook=lambda kv: kv,
                           parse_constant=_no_constant)
    except (ValueError, _Bad, RecursionError):
        return None
    if not isinstance(pairs, list):
        return None
    r = {"root": b"", "branch": b"", "block": []}
    try:
        for key, v in pairs:
            kl = key.lower()
            if kl == "roothash":
                r["root"] = _field_bytes(v)
            elif kl == "branch":
                r["branch"] = _field_bytes(v)
            elif kl == "block":
                if v is None:
                    r["block"] = []
                elif isinstance(v, list):
                    r["block"] = [_field_bytes(x) for x in v]
                else:
                    raise _Bad()
    except _Bad:
        return None
    return r


# ----------------------------------------------------------------------------
# the node
# ----------------------------------------------------------------------------


class _RootState:
    def __init__(self, n: int):
        self.echo: List[bytes] = [b""] * n
        self.echoes = 0
        self.ready = [False] * n
        self.readies = 0
        self.inflight = self.failed = self.have_value = False
        self.value = b""


class OracleNode:
    """One RBC instance (proposer ``proposer``'s broadcast) seen at node ``self_id``."""

    def __init__(self, n: int, f: int, self_id: int, proposer: int):
        if n < 1 or f < 0 or n < 3 * f + 1 or not (0 <= self_id < n) or not (0 <= proposer < n):
            raise ValueError("n >= 3f + 1 and indices in range")
        self.n, self.f, self.k = n, f, n - 2 * f
        self.self_id, self.proposer = self_id, proposer
        self.enc = orc.Encoder(self.k, 2 * f)
        self.proposed = self.val_seen = self.ready_sent = self.delivered = self.value_ok = False
        self.echo_from = [False] * n
        self.ready_from = [False] * n
        self.roots: Dict[bytes, _RootState] = {}
        self.delivered_root = b""
        self.out_value = b""
        self.ops: deque = deque()   # deferred "GPU" work, applied in order by progress()
        self.outq: deque = deque()
        self.rejected = 0

    # -- helpers --------------------------------------------------------------
    def _state(self, root: bytes) -> _RootState:
        if root not in self.roots:
            self.roots[root] = _RootState(self.n)
        return self.roots[root]

    def _send(self, to: int, t: int, payload: bytes) -> None:
        self.outq.append((to, pb_encode(t, payload)))

    def _validate(self, req: dict, index: int) -> bool:
        branch = orc.unflatten_branch(req["branch"], index, self.n)
        return branch is not None and orc.merkle_verify(self.n, req["block"][0], req["root"], branch, index)

    # -- API (rbc_protocol.h) -------------------------------------------------
    def propose(self, value: bytes) -> int:
        if self.self_id != self.proposer or self.proposed:
            return ERR_PROTOCOL
        self.proposed = True
        self.ops.append(("shard", len(value).to_bytes(FRAME, "little") + bytes(value)))
        return 0

    def handle_message(self, sender: int, msg: bytes) -> int:
        if not 0 <= sender < self.n:
            raise ValueError("sender out of range")
        dec = pb_decode(msg)
        req = json_decode(dec[1]) if dec is not None else None
        if req is None or len(req["root"]) != 32:
            self.rejected += 1
            return ERR_PROTOCOL
        t = dec[0]
        if t == READY:
            if self.ready_from[sender] or sender == self.self_id:
                self.rejected += 1
                return ERR_PROTOCOL
            self.ready_from[sender] = True
            self._on_ready(sender, req["root"])
            return 0
        if t == VAL:
            dup = sender != self.proposer or self.val_seen
        else:
            dup = self.echo_from[sender] or sender == self.self_id
        if dup or len(req["block"]) != 1 or not req["block"][0]:
            self.rejected += 1
            return ERR_PROTOCOL
        if t == VAL:
            self.val_seen = True
            self.ops.append(("val", req, sender))
        else:
            self.echo_from[sender] = True
            self.ops.append(("echo", req, sender))
        return 0

    def progress(self) -> int:
        """Applies every deferred operation in order (those it queues too)."""
        while self.ops:
            self._complete(self.ops.popleft())
        return 0

    def messages(self) -> List[Tuple[int, bytes]]:
        out = list(self.outq)
        self.outq.clear()
        return out

    def value(self):
        """None before delivery, the proposer's bytes after; ERR_PROTOCOL
        (returned, not raised) for a delivered, badly framed payload."""
        if not self.delivered:
            return None
        return self.out_value if self.value_ok else ERR_PROTOCOL

    def stats(self) -> dict:
        lead = None
        if self.delivered:
            lead = self.roots[self.delivered_root]
        else:
            for root in sorted(self.roots):   # std::map order, first strict maximum
                s = self.roots[root]
                if lead is None or s.echoes + s.readies > lead.echoes + lead.readies:
                    lead = s
        return {"echoes": lead.echoes if lead else 0, "readies": lead.readies if lead else 0,
                "ready_sent": self.ready_sent, "rejected": self.rejected}

    # -- protocol -------------------------------------------------------------
    def _complete(self, op) -> None:
        kind = op[0]
        if kind == "shard":
            shards = orc.rbc_shard(self.enc, op[1])
            mt = orc.merkle_tree(shards)
            root = mt[1]
            own = None
            for j in range(self.n):
                req = {"root": root, "branch": orc.flat_branch([b for b in orc.merkle_branch(mt, j) if b]),
                       "block": [bytes(shards[j])]}
                if j == self.self_id:
                    own = req
                else:
                    self._send(j, VAL, json_encode_val(req["root"], req["branch"], req["block"][0]))
            self._on_val(own)
        elif kind == "val":
            if not self._validate(op[1], self.self_id):
                self.rejected += 1
                return
            self._on_val(op[1])
        elif kind == "echo":
            req, sender = op[1], op[2]
            if not self._validate(req, sender):
                self.rejected += 1   # the sender's one ECHO slot stays used
                return
            self._on_echo(sender, req["root"], req["block"][0])
        else:  # interp
            root, shards = op[1], op[2]
            s = self._state(root)
            s.inflight = False
            try:
                res = orc.rbc_interpolate(self.enc, root, [np.frombuffer(x, np.uint8) if x else None
                                                           for x in shards])
            except orc.RSError:
                s.failed = True   # not a codeword under this root: never READY for it
                return
            s.have_value = True
            s.value = res["value"]
            self._send_ready(root)
            self._advance(root)

    def _on_val(self, req: dict) -> None:
        self._send(-1, ECHO, json_encode_val(req["root"], req["branch"], req["block"][0]))
        self._on_echo(self.self_id, req["root"], req["block"][0])

    def _on_echo(self, frm: int, root: bytes, shard: bytes) -> None:
        s = self._state(root)
        if not s.echo[frm]:
            s.echo[frm] = bytes(shard)
            s.echoes += 1
        self._advance(root)

    def _on_ready(self, frm: int, root: bytes) -> None:
        s = self._state(root)
        if not s.ready[frm]:
            s.ready[frm] = True
            s.readies += 1
        self._advance(root)

    def _send_ready(self, root: bytes) -> None:
        if self.ready_sent:
            return
        self.ready_sent = True
        self._send(-1, READY, json_encode_ready(root))
        self._on_ready(self.self_id, root)

    def _advance(self, root: bytes) -> None:
        n, f = self.n, self.f
        s = self._state(root)
        if (not s.have_value and not s.inflight and not s.failed and
                ((s.echoes >= n - f and not self.ready_sent) or (s.readies >= 2 * f + 1 and s.echoes >= n - 2 * f))):
            s.inflight = True
            self.ops.append(("interp", root, list(s.echo)))   # snapshot of the ECHOs so far
        if s.readies >= f + 1:
            self._send_ready(root)
        if not self.delivered and s.have_value and s.readies >= 2 * f + 1 and s.echoes >= n - 2 * f:
            self.delivered = True
            self.delivered_root = root
            v = s.value
            if len(v) >= FRAME:
                L = int.from_bytes(v[:FRAME], "little")
                self.value_ok = L <= len(v) - FRAME
                if self.value_ok:
                    self.out_value = bytes(v[FRAME:FRAME + L])
