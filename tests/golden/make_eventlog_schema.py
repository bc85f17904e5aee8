"""Extract the event-log schema facts the hash path depends on.

Run from the repo root, in a container that has /root/reference:
    python tests/golden/make_eventlog_schema.py

The reference's generated Go code (``pkg/pb/{recording,state,msgs}/*.pb.go``)
embeds each .proto file as a serialized ``FileDescriptorProto`` (the
``file_*_proto_rawDesc`` byte literal, written by protoc-gen-go). This script
parses those bytes with the protobuf runtime and keeps, for the messages a
recorded HashResult (or hash Action) passes through, only the field table:
name, number, type, label, message type and oneof membership. That table is
data -- the schema as the reference's own Go binary sees it -- and it pins
``mirbft_amd/eventlog.py``'s hand-written decoder (tests/test_eventlog.py):

* every field number the decoder uses is checked against it, and
* the official protobuf runtime, driven by a descriptor pool rebuilt from it,
  encodes events that the decoder must read back field for field (and our
  own encoder must reproduce byte for byte).

Nothing here is read at test time; the JSON is the committed fixture.
"""
from __future__ import annotations

import json
import os
import re
import sys

from google.protobuf import descriptor_pb2

REF = "/root/reference/pkg/pb"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "eventlog_schema.json")

FILES = {  # package -> generated Go file holding its raw descriptor
    "msgs": "msgs/msgs.pb.go",
    "state": "state/state.pb.go",
    "recording": "recording/recording.pb.go",
}
KEEP = [  # the hash path: recording.Event -> state.Event.hash_result -> origin -> acks / epoch change
    "recording.Event",
    "state.Event", "state.EventTickElapsed", "state.EventHashResult",
    "state.HashOrigin", "state.HashOrigin.Batch", "state.HashOrigin.EpochChange", "state.HashOrigin.VerifyBatch",
    "state.Action", "state.ActionHashRequest",
    "msgs.RequestAck", "msgs.Checkpoint", "msgs.EpochChange", "msgs.EpochChange.SetEntry",
]


def raw_descriptor(path: str) -> bytes:
    src = open(path).read()
    m = re.search(r"_rawDesc = \[\]byte\{(.*?)\n\}", src, re.S)
    if not m:
        raise SystemExit(f"no raw descriptor literal in {path}")
    return bytes(int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]{2})", m.group(1)))


def messages(fd: descriptor_pb2.FileDescriptorProto):
    def walk(ms, prefix):
        for mt in ms:
            name = f"{prefix}.{mt.name}"
            yield name, mt
            yield from walk(mt.nested_type, name)
    yield from walk(fd.message_type, fd.package)


def main() -> int:
    table = {}
    for pkg, rel in FILES.items():
        path = os.path.join(REF, rel)
        fd = descriptor_pb2.FileDescriptorProto.FromString(raw_descriptor(path))
        assert fd.package == pkg, (fd.package, pkg)
        for name, mt in messages(fd):
            if name not in KEEP:
                continue
            table[name] = {
                "source": f"pkg/pb/{rel} (file_{fd.name.replace('/', '_').replace('.', '_')}_rawDesc)",
                "oneofs": [o.name for o in mt.oneof_decl],
                "fields": [{
                    "name": f.name, "number": f.number,
                    "type": descriptor_pb2.FieldDescriptorProto.Type.Name(f.type),
                    "label": descriptor_pb2.FieldDescriptorProto.Label.Name(f.label),
                    "type_name": f.type_name.lstrip("."),
                    "oneof": mt.oneof_decl[f.oneof_index].name if f.HasField("oneof_index") else None,
                } for f in mt.field],
            }
    missing = [k for k in KEEP if k not in table]
    if missing:
        raise SystemExit(f"messages not found: {missing}")
    doc = {
        "_comment": "Field tables extracted from the reference's generated descriptors by "
                    "tests/golden/make_eventlog_schema.py (data only; see its docstring).",
        "messages": {k: table[k] for k in KEEP},
    }
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print(f"wrote {OUT}: {len(KEEP)} messages")
    return 0


if __name__ == "__main__":
    sys.exit(main())
