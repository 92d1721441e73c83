#!/usr/bin/env python3
"""Extract the reference-held protobuf layout of the RBC wire message into
committed fixtures (run in the build container, where /root/reference
exists; the tests read only the fixtures).

* pb_message_descriptor.bin: the FileDescriptorProto that protoc-gen-go
  embedded in pb/message.pb.go:272-293 (`fileDescriptor_33c57e4bae7b9afd`,
  "290 bytes of a gzipped FileDescriptorProto"), gunzipped -- the serialized
  descriptor itself, i.e. data, not the Go source.
* pb_struct_tags.json: the wire facts of the generated Go structs'
  `protobuf:"..."` tags (pb/message.pb.go:84-86,140-144,182-183,223-224),
  which golang/protobuf v1.3.1 marshals from -- notably RBC.Type, field 2
  varint, present in the struct tags but absent from the descriptor.

usage: python tests/golden/extract_pb_descriptor.py [/root/reference]
"""
import gzip
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main(ref="/root/reference"):
    src = open(os.path.join(ref, "pb", "message.pb.go")).read()
    body = src[src.index("var fileDescriptor_33c57e4bae7b9afd = []byte{"):]
    body = body[: body.index("}")]
    raw = bytes(int(x, 16) for x in re.findall(r"0x([0-9a-f]{2})", body))
    assert len(raw) == 290, len(raw)
    desc = gzip.decompress(raw)
    with open(os.path.join(HERE, "pb_message_descriptor.bin"), "wb") as f:
        f.write(desc)
    tags = {}
    struct = None
    for line in src.splitlines():
        m = re.match(r"^type (\w+) struct \{", line)
        if m:
            struct = m.group(1)
        m = re.search(r"^\s+(\w+)\s+\S+\s+`protobuf:\"([^\"]+)\"", line)
        if struct and m:
            wire, num, *rest = m.group(2).split(",")
            tags[f"{struct}.{m.group(1)}"] = {"wire": wire, "number": int(num),
                                              "options": [x for x in rest if x]}
    with open(os.path.join(HERE, "pb_struct_tags.json"), "w") as f:
        json.dump({"source": "pb/message.pb.go struct tags (golang/protobuf v1.3.1, go.mod:7)", "fields": tags},
                  f, indent=1, sort_keys=True)
    print(f"descriptor {len(raw)} B gzipped -> {len(desc)} B; {len(tags)} tagged fields")


if __name__ == "__main__":
    main(*sys.argv[1:])
