"""Event-log golden traces: the reference's log framing and
HashResult reconstruction, checked on CPU with the oracle as the hasher and on
the GPU with the engine."""
import hashlib
import json
import os
import random
import struct
import zlib

import pytest

from mirbft_amd import eventlog as EL
from mirbft_amd.encoding import Checkpoint, EpochChange, RequestAck, SetEntry, epoch_change_hash_data
from mirbft_amd.processor import HashOrigin, HashOriginBatch, HashOriginEpochChange, HashOriginVerifyBatch
from oracle import oracle


class OracleHasher:  # test-only stand-in for GPUHasher.hash_batch
    def hash_batch(self, actions):
        return oracle.process_hash_actions(actions)


def _acks(n, salt=0):
    return [RequestAck(i % 4, i // 4, hashlib.sha256(bytes([i, salt])).digest()) for i in range(n)]


def _synthetic_log(corrupt_index=None):
    origins = [
        HashOrigin(HashOriginBatch(source=0, epoch=1, seq_no=5, request_acks=_acks(20))),
        HashOrigin(HashOriginBatch(source=1, epoch=1, seq_no=6, request_acks=_acks(1, 7))),
        HashOrigin(HashOriginVerifyBatch(source=2, seq_no=9, request_acks=_acks(3, 9), expected_digest=b"x" * 32)),
        HashOrigin(HashOriginVerifyBatch(source=2, seq_no=10, request_acks=[])),
        HashOrigin(HashOriginEpochChange(source=3, origin=1, epoch_change=EpochChange(
            new_epoch=4, checkpoints=[Checkpoint(20, b"\x11" * 40), Checkpoint(40, b"\x22" * 332)],
            p_set=[SetEntry(3, 21, b"\x33" * 32), SetEntry(3, 22, b"")],
            q_set=[SetEntry(2, 21, b"\x44" * 32)]))),
        HashOrigin(HashOriginEpochChange(source=0, origin=2, epoch_change=EpochChange(new_epoch=7))),
    ]
    recs = [EL.encode_event(1, 2, tick=True)]
    for k, o in enumerate(origins):
        t = o.type
        if isinstance(t, HashOriginEpochChange):
            data = epoch_change_hash_data(t.epoch_change)
        else:
            data = [a.digest for a in t.request_acks]
        d = hashlib.sha256(b"".join(data)).digest()
        if k == corrupt_index:
            d = bytes([d[0] ^ 1]) + d[1:]
        recs.append(EL.encode_event(k % 4, 1000 + k, hash_result=(d, o)))
    recs.append(EL.encode_event(1, 2, tick=True))
    return EL.write_log(recs), origins


def test_reference_reader_spec_two_tick_events():
    # pkg/eventlog/interceptor_test.go:55-94: two TickElapsed events from node 1 at time 2
    log = EL.write_log([EL.encode_event(1, 2, tick=True), EL.encode_event(1, 2, tick=True)])
    evs = list(EL.read_events(log))
    assert [(e.node_id, e.time, e.kind) for e in evs] == [(1, 2, 10), (1, 2, 10)]


def test_reference_recorder_byte_count():
    # interceptor_test.go:38-50: the reference's Recorder wrote exactly 46 bytes for two
    # TickElapsed events from node 1 at time 2 (gzip.BestSpeed, interceptor.go:59).
    # Go's BestSpeed deflate hands a window under 128 bytes to writeBlockHuff, which
    # stores it (a Huffman table alone outweighs it), and Close appends an empty final
    # stored block: 10 (gzip header) + 5 + len(body) + 5 + 8 (trailer). 46 bytes
    # therefore means the size-prefixed records are 18 bytes, 9 per event.
    recs = [EL.encode_event(1, 2, tick=True)] * 2
    body = b"".join(EL._put_varint_signed(len(r)) + r for r in recs)
    assert len(body) == 18
    # that same stream, byte for byte as Go lays it out, must read back as two ticks
    go = (b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x04\xff"            # header, XFL 4 = BestSpeed, OS unknown
          + b"\x00" + struct.pack("<HH", len(body), len(body) ^ 0xFFFF) + body   # stored, not final
          + b"\x01\x00\x00\xff\xff"                                  # empty final stored block
          + struct.pack("<II", zlib.crc32(body), len(body)))
    assert len(go) == 46
    evs = list(EL.read_events(go))
    assert [(e.node_id, e.time, e.kind_name) for e in evs] == [(1, 2, "tick_elapsed")] * 2


def test_truncated_log_is_an_error():
    # interceptor_test.go:96-106: output.Truncate(2) -> "could not read source as a gzip stream"
    log = EL.write_log([EL.encode_event(1, 2, tick=True)])
    with pytest.raises(EL.EventLogError, match="could not read source as a gzip stream"):
        list(EL.read_events(log[:2]))


def test_hash_results_round_trip_and_reconstruct():
    log, origins = _synthetic_log()
    evs = [e.hash_result for e in EL.read_events(log) if e.hash_result]
    assert len(evs) == len(origins)
    for e, o in zip(evs, origins):
        assert type(e.origin.type) is type(o.type)
        exp = (epoch_change_hash_data(o.type.epoch_change) if isinstance(o.type, HashOriginEpochChange)
               else [a.digest for a in o.type.request_acks])
        assert e.hash_data() == exp
    assert evs[2].origin.type.expected_digest == b"x" * 32
    assert evs[4].origin.type.epoch_change.p_set[1].digest == b""


def test_verify_trace_with_oracle_detects_corruption():
    log, _ = _synthetic_log()
    rep = EL.verify_trace(OracleHasher(), log)
    assert rep.ok and rep.hash_results == 6
    assert rep.by_kind == {"HashOriginBatch": 2, "HashOriginVerifyBatch": 2, "HashOriginEpochChange": 2}
    bad, _ = _synthetic_log(corrupt_index=4)
    rep = EL.verify_trace(OracleHasher(), bad)
    assert not rep.ok and [m[0] for m in rep.mismatches] == [4]


@pytest.mark.gpu
def test_verify_trace_on_gpu(engine):
    from mirbft_amd import GPUHasher
    log, _ = _synthetic_log()
    assert EL.verify_trace(GPUHasher(engine), log).ok
    bad, _ = _synthetic_log(corrupt_index=0)
    rep = EL.verify_trace(GPUHasher(engine), bad)
    assert [m[0] for m in rep.mismatches] == [0]


# ---------------------------------------------------------------------------
# The decoder against the reference's own schema (tests/golden/eventlog_schema.json,
# extracted from pkg/pb/*/*.pb.go by tests/golden/make_eventlog_schema.py).
# ---------------------------------------------------------------------------
_SCHEMA_JSON = os.path.join(os.path.dirname(__file__), "golden", "eventlog_schema.json")
_KIND = {"TYPE_UINT64": "uint64", "TYPE_INT64": "int64", "TYPE_BYTES": "bytes"}


def _ref_schema():
    with open(_SCHEMA_JSON) as f:
        return json.load(f)["messages"]


def test_schema_matches_reference_descriptors():
    ref = _ref_schema()
    for name, spec in EL.SCHEMA.items():
        assert name in ref, name
        by_num = {f["number"]: f for f in ref[name]["fields"]}
        for num, (fname, kind, rep) in spec.items():
            f = by_num[num]
            assert f["name"] == fname, (name, num)
            assert _KIND.get(f["type"], f["type_name"]) == kind, (name, fname)
            assert (f["label"] == "LABEL_REPEATED") == rep, (name, fname)
        if name != "state.Event":           # every field of a hash-path message is interpreted
            assert set(by_num) == set(spec), name
    kinds = {f["number"]: f["name"] for f in ref["state.Event"]["fields"] if f["oneof"] == "type"}
    assert kinds == EL.EVENT_KINDS


def _official_classes():
    """Message classes of the official protobuf runtime, built from the reference's field tables."""
    descriptor_pb2 = pytest.importorskip("google.protobuf.descriptor_pb2")
    from google.protobuf import descriptor_pool, message_factory
    ref = _ref_schema()
    files = {}
    for name in ref:
        pkg, *path = name.split(".")
        fd = files.setdefault(pkg, descriptor_pb2.FileDescriptorProto(name=f"{pkg}/{pkg}.proto", package=pkg,
                                                                       syntax="proto3"))
        parent = fd.message_type
        for part in path[:-1]:
            parent = next(m for m in parent if m.name == part).nested_type
        mt = parent.add(name=path[-1])
        for o in ref[name]["oneofs"]:
            mt.oneof_decl.add(name=o)
        for f in ref[name]["fields"]:
            if f["type_name"] and f["type_name"] not in ref:
                continue                     # a member off the hash path (e.g. state.Event.step)
            fp = mt.field.add(name=f["name"], number=f["number"],
                              type=descriptor_pb2.FieldDescriptorProto.Type.Value(f["type"]),
                              label=descriptor_pb2.FieldDescriptorProto.Label.Value(f["label"]))
            if f["type_name"]:
                fp.type_name = "." + f["type_name"]
            if f["oneof"] is not None:
                fp.oneof_index = ref[name]["oneofs"].index(f["oneof"])
    files["state"].dependency.append("msgs/msgs.proto")
    files["recording"].dependency.append("state/state.proto")
    pool = descriptor_pool.DescriptorPool()
    for pkg in ("msgs", "state", "recording"):
        pool.Add(files[pkg])
    return lambda n: message_factory.GetMessageClass(pool.FindMessageTypeByName(n))


def _random_origin(rng):
    acks = lambda k: [RequestAck(rng.randrange(1 << 64), rng.choice([0, 1, rng.randrange(1 << 40)]),
                                 rng.randbytes(rng.choice([0, 11, 32]))) for _ in range(k)]
    t = rng.randrange(3)
    if t == 0:
        return HashOrigin(HashOriginBatch(rng.randrange(8), rng.randrange(1 << 33), rng.randrange(300),
                                          acks(rng.randrange(0, 6))))
    if t == 1:
        return HashOrigin(HashOriginVerifyBatch(rng.randrange(8), rng.randrange(300), acks(rng.randrange(0, 6)),
                                                rng.randbytes(rng.choice([0, 32]))))
    ec = None if rng.random() < 0.2 else EpochChange(
        new_epoch=rng.randrange(50),
        checkpoints=[Checkpoint(rng.randrange(1000), rng.randbytes(rng.randrange(0, 300))) for _ in range(rng.randrange(3))],
        p_set=[SetEntry(rng.randrange(9), rng.randrange(99), rng.randbytes(rng.choice([0, 32]))) for _ in range(rng.randrange(4))],
        q_set=[SetEntry(rng.randrange(9), rng.randrange(99), rng.randbytes(32)) for _ in range(rng.randrange(4))])
    return HashOrigin(HashOriginEpochChange(rng.randrange(8), rng.randrange(8), ec))


def _fill_official(cls, o: HashOrigin, digest, node, t):
    ev = cls("recording.Event")(node_id=node, time=t)
    hr = ev.state_event.hash_result
    hr.digest = digest
    ty = o.type

    def ack(dst, a):
        dst.add(client_id=a.client_id, req_no=a.req_no, digest=a.digest)
    if isinstance(ty, HashOriginBatch):
        b = hr.origin.batch
        b.source, b.epoch, b.seq_no = ty.source, ty.epoch, ty.seq_no
        b.SetInParent()
        for a in ty.request_acks:
            ack(b.request_acks, a)
    elif isinstance(ty, HashOriginVerifyBatch):
        v = hr.origin.verify_batch
        v.source, v.seq_no, v.expected_digest = ty.source, ty.seq_no, ty.expected_digest
        v.SetInParent()
        for a in ty.request_acks:
            ack(v.request_acks, a)
    else:
        e = hr.origin.epoch_change
        e.source, e.origin = ty.source, ty.origin
        e.SetInParent()
        if ty.epoch_change is not None:
            ec = e.epoch_change
            ec.SetInParent()
            ec.new_epoch = ty.epoch_change.new_epoch
            for c in ty.epoch_change.checkpoints:
                ec.checkpoints.add(seq_no=c.seq_no, value=c.value)
            for dst, src in ((ec.p_set, ty.epoch_change.p_set), (ec.q_set, ty.epoch_change.q_set)):
                for s in src:
                    dst.add(epoch=s.epoch, seq_no=s.seq_no, digest=s.digest)
    return ev


def test_official_protobuf_encoding_reads_back():
    """Events encoded by the official protobuf runtime from the reference's schema decode
    field for field, and our encoder writes the same bytes (field-number order, zero
    scalars omitted: what Go's proto.Marshal emits for these proto3 messages)."""
    cls = _official_classes()
    rng = random.Random(0x4D495242)
    recs, exp = [], []
    for i in range(300):
        o = _random_origin(rng)
        digest = rng.randbytes(32)
        node, t = rng.randrange(4), rng.choice([0, 5, -3, 1 << 62, -(1 << 63)])
        b = _fill_official(cls, o, digest, node, t).SerializeToString(deterministic=True)
        assert EL.encode_event(node, t, hash_result=(digest, o)) == b, i
        recs.append(b)
        exp.append((node, t, digest, o))
    tick = cls("recording.Event")(node_id=3, time=7)
    tick.state_event.tick_elapsed.SetInParent()
    recs.append(tick.SerializeToString(deterministic=True))
    assert recs[-1] == EL.encode_event(3, 7, tick=True)
    evs = list(EL.read_events(EL.write_log(recs)))
    assert len(evs) == len(recs) and evs[-1].kind_name == "tick_elapsed" and evs[-1].hash_result is None
    for e, (node, t, digest, o) in zip(evs, exp):
        assert (e.node_id, e.time, e.kind_name) == (node, t, "hash_result")
        hr = e.hash_result
        assert hr.digest == digest and hr.origin == o


def test_unknown_fields_are_skipped():
    # a state.Event member off the hash path (step = 9) and an unknown field inside an
    # origin are skipped the way the protobuf runtime skips them
    o = HashOrigin(HashOriginBatch(1, 2, 3, _acks(2)))
    b = EL.encode_event(0, 1, hash_result=(b"d" * 32, o))
    extra = EL._put_uvarint(99 << 3) + EL._put_uvarint(5)
    step = EL.encode_event(2, 4, tick=True).replace(EL._put_uvarint(10 << 3 | 2) + b"\x00",
                                                    EL._put_uvarint(9 << 3 | 2) + b"\x00")
    evs = list(EL.read_events(EL.write_log([b + extra, step])))
    assert evs[0].hash_result.origin == o
    assert evs[1].kind_name == "step" and evs[1].hash_result is None
