"""Wire codec of the RBC state machine (include/rbc_protocol.h), no GPU.

pb side: pinned against the protobuf runtime (google.protobuf 7.x, here) with
a schema built from pb/message.proto:11-35 plus the generated code's RBC.type
field 2 (pb/message.pb.go:182-183).  JSON side: Go encoding/json output for
rbc/request.go:9-21 is restated with Python json + base64 (compact
separators, struct field order, nil -> null), which for base64 strings is
byte-identical to Go's encoder (no characters Go would escape occur).
Parity of the payload format with a Go build is unpinned: the reference's
handlers are stubs, so no Go-produced message exists to compare against.
"""
import base64
import json
import os

import numpy as np
import pytest

from cleisthenes_amd import _lib, protocol


def _schema():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    fd = descriptor_pb2.FileDescriptorProto(name="rbc_test_message.proto", package="pbtest", syntax="proto3")
    rbc = fd.message_type.add(name="RBC")
    rbc.field.add(name="payload", number=1, type=descriptor_pb2.FieldDescriptorProto.TYPE_BYTES,
                  label=descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL)
    rbc.field.add(name="type", number=2, type=descriptor_pb2.FieldDescriptorProto.TYPE_INT32,
                  label=descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL)
    bba = fd.message_type.add(name="BBA")
    bba.field.add(name="payload", number=1, type=descriptor_pb2.FieldDescriptorProto.TYPE_BYTES,
                  label=descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL)
    msg = fd.message_type.add(name="Message")
    msg.field.add(name="signature", number=1, type=descriptor_pb2.FieldDescriptorProto.TYPE_BYTES,
                  label=descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL)
    msg.oneof_decl.add(name="payload")
    msg.field.add(name="rbc", number=3, type=descriptor_pb2.FieldDescriptorProto.TYPE_MESSAGE,
                  type_name=".pbtest.RBC", label=descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL, oneof_index=0)
    msg.field.add(name="bba", number=4, type=descriptor_pb2.FieldDescriptorProto.TYPE_MESSAGE,
                  type_name=".pbtest.BBA", label=descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL, oneof_index=0)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = message_factory.GetMessageClass
    return get(pool.FindMessageTypeByName("pbtest.Message")), get(pool.FindMessageTypeByName("pbtest.RBC"))


@pytest.fixture(scope="module")
def pbm():
    pytest.importorskip("google.protobuf")
    return _schema()


def go_json_val(root, branch, block):
    enc = lambda b: None if not b else base64.b64encode(b).decode()  # noqa: E731
    d = {"RootHash": enc(root), "Branch": enc(branch), "Block": None if not block else [base64.b64encode(block).decode()]}
    return json.dumps(d, separators=(",", ":")).encode()


def go_json_ready(root):
    return json.dumps({"RootHash": base64.b64encode(root).decode() if root else None},
                      separators=(",", ":")).encode()


@pytest.mark.parametrize("plen", [0, 1, 127, 128, 300, 70000])
@pytest.mark.parametrize("mtype", [0, 1, 2])
def test_pb_encode_matches_protobuf_runtime(pbm, mtype, plen):
    Message, RBC = pbm
    payload = np.random.default_rng(plen + mtype).integers(0, 256, plen, dtype=np.uint8).tobytes()
    ours = protocol.pb_encode(mtype, payload)
    m = Message()
    m.rbc.CopyFrom(RBC(payload=payload, type=mtype))
    assert ours == m.SerializeToString(deterministic=True)
    t, p = protocol.pb_decode(ours)
    assert (t, p) == (mtype, payload)


def test_pb_decode_accepts_runtime_messages_with_extra_fields(pbm):
    Message, RBC = pbm
    m = Message(signature=b"sig" * 30)
    m.rbc.CopyFrom(RBC(payload=b'{"RootHash":null}', type=2))
    raw = m.SerializeToString()
    assert protocol.pb_decode(raw) == (2, b'{"RootHash":null}')
    # unknown field 9 (varint) and field 2 timestamp (length-delimited) are skipped
    extra = bytes([0x48, 0x05, 0x12, 0x02, 0x08, 0x01]) + raw
    assert protocol.pb_decode(extra) == (2, b'{"RootHash":null}')
    # a later RBC field merges into the earlier one (later scalars win)
    merged = raw + bytes([0x1a, 0x02, 0x10, 0x01])
    assert protocol.pb_decode(merged) == (1, b'{"RootHash":null}')


@pytest.mark.parametrize("raw", [
    b"",                                  # no oneof set
    bytes([0x22, 0x00]),                  # BBA, not RBC
    bytes([0x1a, 0x02, 0x10, 0x03]),      # unknown RBC type 3
    bytes([0x1a, 0x05, 0x0a, 0x09, 0x41]),  # payload longer than its message
    bytes([0x1a]),                        # truncated length
    bytes([0x1a, 0x02, 0x10]),            # truncated varint
    bytes([0x03]),                        # field 0
    bytes([0x1a, 0x01, 0x0b]),            # group wire type inside RBC
])
def test_pb_decode_rejects_malformed(raw):
    with pytest.raises(_lib.RBCError) as e:
        protocol.pb_decode(raw)
    assert e.value.code == _lib.RBC_ERR_PROTOCOL


def test_pb_oneof_switch_to_bba_rejected(pbm):
    Message, RBC = pbm
    m = Message()
    m.rbc.CopyFrom(RBC(payload=b"x", type=1))
    raw = m.SerializeToString() + bytes([0x22, 0x00])
    with pytest.raises(_lib.RBCError):
        protocol.pb_decode(raw)


@pytest.mark.parametrize("blen", [1, 2, 3, 4, 5, 64, 1000, 4097])
def test_json_val_matches_go_encoding(blen):
    rng = np.random.default_rng(blen)
    root = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    branch = rng.integers(0, 256, 32 * 7, dtype=np.uint8).tobytes()
    block = rng.integers(0, 256, blen, dtype=np.uint8).tobytes()
    js = protocol.json_encode_val(root, branch, block)
    assert js == go_json_val(root, branch, block)
    d = protocol.json_decode_val(js)
    assert d == {"RootHash": root, "Branch": branch, "Block": [block]}


def test_json_nil_fields_and_ready():
    root = bytes(range(32))
    assert protocol.json_encode_val(root, b"", b"") == b'{"RootHash":"' + base64.b64encode(root) + \
        b'","Branch":null,"Block":null}'
    assert protocol.json_encode_ready(root) == go_json_ready(root)
    assert protocol.json_encode_ready(b"") == b'{"RootHash":null}'
    assert protocol.json_decode_ready(go_json_ready(root)) == root
    # a depth-0 (N=1) branch is nil
    d = protocol.json_decode_val(go_json_val(root, b"", b"\x07"))
    assert d["Branch"] == b"" and d["Block"] == [b"\x07"]


def test_json_decode_follows_encoding_json_rules():
    root = bytes(range(32))
    r64 = base64.b64encode(root).decode()
    blk = base64.b64encode(b"shard").decode()
    # whitespace, case-insensitive keys, unknown keys of every kind, escaped '/'
    js = ('{ "roothash" : "%s",\n "x": {"a":[1,2.5e3,true,null,{"b":"c"}]}, "BRANCH": null, '
          '"block": [ "%s" ] , "z":-1}' % (r64.replace("/", "\\/"), blk)).encode()
    d = protocol.json_decode_val(js)
    assert d == {"RootHash": root, "Branch": b"", "Block": [b"shard"]}
    # a later duplicate key wins, as in encoding/json
    js2 = ('{"RootHash":"%s","Block":["AA=="],"Block":["%s"]}' % (r64, blk)).encode()
    assert protocol.json_decode_val(js2)["Block"] == [b"shard"]
    # base64.StdEncoding is not Strict(): non-zero trailing bits of the last
    # quantum are ignored ("AB==" -> 0x00, "AAB=" -> 0x00 0x00), as Go decodes them
    for b64, want in (("AB==", b"\x00"), ("AAB=", b"\x00\x00"), ("/w==", b"\xff"), ("//8=", b"\xff\xff")):
        js3 = ('{"RootHash":"%s","Block":["%s"]}' % (r64, b64)).encode()
        assert protocol.json_decode_val(js3)["Block"] == [want], b64


@pytest.mark.parametrize("js", [
    b'',
    b'[]',
    b'{"RootHash":"AAAA"}',                                  # root not 32 bytes
    b'{"RootHash":"%s","Block":["AA="]}',                    # bad padding
    b'{"RootHash":"%s","Block":["A-=="]}',                   # URL alphabet
    b'{"RootHash":"%s","Block":[]}',                         # no shard
    b'{"RootHash":"%s","Block":["AA==","AA=="]}',            # two shards
    b'{"RootHash":"%s","Block":["AA=="]',                    # unterminated
    b'{"RootHash":"%s","Block":["AA=="]} x',                 # trailing garbage
    b'{"RootHash":"%s","Block":["AA=="],}',                  # trailing comma
    b'{"RootHash":"%s","Block":"AA=="}',                     # not an array
])
def test_json_decode_rejects_malformed(js):
    r64 = base64.b64encode(bytes(range(32)))
    js = js.replace(b"%s", r64)
    with pytest.raises(_lib.RBCError) as e:
        protocol.json_decode_val(js)
    assert e.value.code == _lib.RBC_ERR_PROTOCOL


def test_json_fuzz_roundtrip_against_python():
    rng = np.random.default_rng(7)
    for _ in range(200):
        root = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        branch = rng.integers(0, 256, 32 * int(rng.integers(0, 9)), dtype=np.uint8).tobytes()
        block = rng.integers(0, 256, int(rng.integers(1, 200)), dtype=np.uint8).tobytes()
        js = protocol.json_encode_val(root, branch, block)
        assert json.loads(js) == json.loads(go_json_val(root, branch, block))
        assert protocol.json_decode_val(js) == {"RootHash": root, "Branch": branch, "Block": [block]}
        # truncations never crash and never decode
        cut = int(rng.integers(0, len(js)))
        with pytest.raises(_lib.RBCError):
            protocol.json_decode_val(js[:cut])


def test_node_create_rejects_bad_arguments_without_gpu():
    import ctypes
    p = ctypes.c_void_p()
    assert _lib.lib.rbc_node_create(None, 4, 1, 0, 0, ctypes.byref(p)) == _lib.RBC_ERR_INVALID_ARG
    # n < 3f + 1 breaks HBBFT quorum intersection: rejected before the batcher
    # is touched (a dummy non-NULL handle is never dereferenced on this path)
    dummy = ctypes.c_void_p(1)
    for n, f in ((5, 2), (3, 1), (6, 2), (8, 3), (255, 85)):
        assert _lib.lib.rbc_node_create(dummy, n, f, 0, 0, ctypes.byref(p)) == _lib.RBC_ERR_INVALID_ARG, (n, f)
    assert _lib.lib.rbc_strerror(_lib.RBC_ERR_PROTOCOL).startswith(b"malformed")
