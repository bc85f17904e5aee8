"""MirBFT event-log traces as golden (input, digest) pairs for the hash path.

The reference records every state event a node applies -- HashResult events
included -- as a gzip stream of size-prefixed ``recording.Event`` protobufs
(``pkg/eventlog/interceptor.go:212-233``; the size prefix is Go's signed
``binary.PutVarint``, i.e. a zig-zag varint). A HashResult carries the digest
Go ``crypto/sha256`` produced and its ``HashOrigin``, from which the hashed
bytes are fully reconstructible:

* Batch / VerifyBatch: the concatenated ``RequestAck.digest``s
  (``sequence.go:155-158``, ``batch_tracker.go:175-178``);
* EpochChange: ``epochChangeHashData(origin.epoch_change)``
  (``stateless.go:323-352``).

So a log recorded by the reference on a Go-equipped box is a set of golden
pairs from the real protocol: ``verify_trace`` re-hashes every reconstructed
input on the GPU (one batch) and compares with the recorded digests.

Protobuf wire format is decoded by hand (no protoc in this image) against
``SCHEMA``, the field tables of the messages on the hash path; every other field
is skipped. ``SCHEMA`` is pinned to the reference's own generated descriptors
(``pkg/pb/*/*.pb.go`` raw descriptors -> tests/golden/eventlog_schema.json), and
the official protobuf runtime, driven by those descriptors, encodes the events
the tests decode.
"""
from __future__ import annotations

import gzip
import io
from dataclasses import dataclass, field
from typing import Dict, Iterator, List, Optional, Tuple, Union

from .encoding import (Checkpoint, EpochChange, RequestAck, SetEntry, batch_hash_data,
                       epoch_change_hash_data, verify_batch_hash_data)
from .processor import (HashOrigin, HashOriginBatch, HashOriginEpochChange, HashOriginVerifyBatch)


class EventLogError(ValueError):
    pass


# ---------------------------------------------------------------------------
# protobuf wire format
# ---------------------------------------------------------------------------
def _uvarint(buf: bytes, i: int) -> Tuple[int, int]:
    x = s = 0
    while True:
        if i >= len(buf):
            raise EventLogError("truncated varint")
        b = buf[i]
        i += 1
        x |= (b & 0x7F) << s
        if b < 0x80:
            return x, i
        s += 7
        if s > 63:
            raise EventLogError("varint overflow")


def _fields(buf: bytes) -> Iterator[Tuple[int, int, Union[int, bytes]]]:
    """Yield (field_number, wire_type, value) for one message."""
    i = 0
    while i < len(buf):
        key, i = _uvarint(buf, i)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _uvarint(buf, i)
        elif wt == 1:
            v, i = int.from_bytes(buf[i:i + 8], "little"), i + 8
        elif wt == 2:
            n, i = _uvarint(buf, i)
            if i + n > len(buf):
                raise EventLogError("truncated length-delimited field")
            v, i = bytes(buf[i:i + n]), i + n
        elif wt == 5:
            v, i = int.from_bytes(buf[i:i + 4], "little"), i + 4
        else:
            raise EventLogError(f"unsupported wire type {wt}")
        yield fn, wt, v


def _put_uvarint(x: int) -> bytes:
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


def _put_varint_signed(x: int) -> bytes:
    """Go binary.PutVarint: zig-zag then unsigned varint."""
    return _put_uvarint((x << 1) ^ (x >> 63) if x < 0 else x << 1)


def _read_varint_signed(stream: io.BufferedReader) -> Optional[int]:
    x = s = 0
    while True:
        b = stream.read(1)
        if not b:
            if s == 0:
                return None  # clean EOF between records
            raise EventLogError("truncated size prefix")
        x |= (b[0] & 0x7F) << s
        if b[0] < 0x80:
            break
        s += 7
    return (x >> 1) ^ -(x & 1)


# ---------------------------------------------------------------------------
# the schema of the hash path
# ---------------------------------------------------------------------------
# message -> {field number: (field name, kind, repeated)}; kind is "uint64",
# "int64", "bytes" or a message name. Restates the field tables of
# protos/recording/recording.proto:14-18, protos/state/state.proto:16-31,78-109
# and protos/msgs/msgs.proto:231-235,255-289 for the messages a HashResult passes
# through. tests/test_eventlog.py checks every entry against the reference's
# generated descriptors (tests/golden/eventlog_schema.json).
SCHEMA: Dict[str, Dict[int, Tuple[str, str, bool]]] = {
    "recording.Event": {1: ("node_id", "uint64", False), 2: ("time", "int64", False),
                        3: ("state_event", "state.Event", False)},
    "state.Event": {4: ("hash_result", "state.EventHashResult", False),
                    10: ("tick_elapsed", "state.EventTickElapsed", False)},
    "state.EventTickElapsed": {},
    "state.EventHashResult": {1: ("digest", "bytes", False), 2: ("origin", "state.HashOrigin", False)},
    "state.HashOrigin": {1: ("batch", "state.HashOrigin.Batch", False),
                         2: ("epoch_change", "state.HashOrigin.EpochChange", False),
                         3: ("verify_batch", "state.HashOrigin.VerifyBatch", False)},
    "state.HashOrigin.Batch": {1: ("source", "uint64", False), 2: ("epoch", "uint64", False),
                               3: ("seq_no", "uint64", False), 5: ("request_acks", "msgs.RequestAck", True)},
    "state.HashOrigin.EpochChange": {1: ("source", "uint64", False), 2: ("origin", "uint64", False),
                                     3: ("epoch_change", "msgs.EpochChange", False)},
    "state.HashOrigin.VerifyBatch": {1: ("source", "uint64", False), 2: ("seq_no", "uint64", False),
                                     3: ("request_acks", "msgs.RequestAck", True),
                                     4: ("expected_digest", "bytes", False)},
    "msgs.RequestAck": {1: ("client_id", "uint64", False), 2: ("req_no", "uint64", False),
                        3: ("digest", "bytes", False)},
    "msgs.Checkpoint": {1: ("seq_no", "uint64", False), 2: ("value", "bytes", False)},
    "msgs.EpochChange": {1: ("new_epoch", "uint64", False), 2: ("checkpoints", "msgs.Checkpoint", True),
                         3: ("p_set", "msgs.EpochChange.SetEntry", True),
                         4: ("q_set", "msgs.EpochChange.SetEntry", True)},
    "msgs.EpochChange.SetEntry": {1: ("epoch", "uint64", False), 2: ("seq_no", "uint64", False),
                                  3: ("digest", "bytes", False)},
}

# state.Event's oneof members by field number (state.proto:16-31): RecordedEvent.kind.
EVENT_KINDS = {1: "initialize", 2: "load_persisted_entry", 3: "complete_initialization", 4: "hash_result",
               5: "checkpoint_result", 6: "request_persisted", 7: "state_transfer_complete",
               8: "state_transfer_failed", 9: "step", 10: "tick_elapsed", 11: "actions_received"}

_SCALAR_WIRE = {"uint64": 0, "int64": 0, "bytes": 2}


def _decode(buf: bytes, name: str) -> dict:
    """One message as {field name: value}; unknown fields are skipped (proto3)."""
    spec = SCHEMA[name]
    out: dict = {}
    for fn, wt, v in _fields(buf):
        if fn not in spec:
            continue
        fname, kind, rep = spec[fn]
        if wt != _SCALAR_WIRE.get(kind, 2):
            raise EventLogError(f"{name}.{fname}: wire type {wt}")
        if kind == "int64":
            v = v - (1 << 64) if v >= 1 << 63 else v
        elif kind in SCHEMA:
            v = _decode(v, kind)
        if rep:
            out.setdefault(fname, []).append(v)
        else:
            out[fname] = v      # last one wins, as in proto3
    return out


def _encode(name: str, msg: dict) -> bytes:
    """Inverse of _decode: fields in number order, zero scalars omitted (what
    Go's proto.Marshal writes for these proto3 messages)."""
    out = bytearray()
    for fn, (fname, kind, rep) in sorted(SCHEMA[name].items()):
        v = msg.get(fname)
        for x in (v or []) if rep else ([] if v is None else [v]):
            if kind in ("uint64", "int64"):
                if x:
                    out += _put_uvarint(fn << 3) + _put_uvarint(x & 0xFFFFFFFFFFFFFFFF)
            elif kind == "bytes":
                if x:
                    out += _put_uvarint(fn << 3 | 2) + _put_uvarint(len(x)) + x
            else:
                body = _encode(kind, x)
                out += _put_uvarint(fn << 3 | 2) + _put_uvarint(len(body)) + body
    return bytes(out)


# ---------------------------------------------------------------------------
# decoded events
# ---------------------------------------------------------------------------
@dataclass
class HashResultEvent:
    node_id: int
    time: int
    digest: bytes
    origin: HashOrigin

    def hash_data(self) -> List[bytes]:
        """The parts whose SHA-256 the reference recorded (see module docstring)."""
        t = self.origin.type
        if isinstance(t, HashOriginBatch):
            return batch_hash_data(t.request_acks)
        if isinstance(t, HashOriginVerifyBatch):
            return verify_batch_hash_data(t.request_acks)
        if isinstance(t, HashOriginEpochChange):
            return epoch_change_hash_data(t.epoch_change or EpochChange(new_epoch=0))
        raise EventLogError("HashResult without an origin")


@dataclass
class RecordedEvent:
    node_id: int
    time: int
    kind: int                       # state.Event oneof field number (EVENT_KINDS: 4 = hash_result, 10 = tick_elapsed)
    hash_result: Optional[HashResultEvent] = None

    @property
    def kind_name(self) -> str:
        return EVENT_KINDS.get(self.kind, f"unknown({self.kind})")


def _acks(ms: List[dict]) -> List[RequestAck]:
    return [RequestAck(a.get("client_id", 0), a.get("req_no", 0), a.get("digest", b"")) for a in ms]


def _epoch_change(m: dict) -> EpochChange:
    sets = lambda k: [SetEntry(e.get("epoch", 0), e.get("seq_no", 0), e.get("digest", b"")) for e in m.get(k, [])]
    return EpochChange(new_epoch=m.get("new_epoch", 0),
                       checkpoints=[Checkpoint(c.get("seq_no", 0), c.get("value", b""))
                                    for c in m.get("checkpoints", [])],
                       p_set=sets("p_set"), q_set=sets("q_set"))


def _hash_origin(m: dict) -> HashOrigin:
    if "batch" in m:
        b = m["batch"]
        return HashOrigin(HashOriginBatch(b.get("source", 0), b.get("epoch", 0), b.get("seq_no", 0),
                                          _acks(b.get("request_acks", []))))
    if "epoch_change" in m:
        e = m["epoch_change"]
        ec = e.get("epoch_change")
        return HashOrigin(HashOriginEpochChange(e.get("source", 0), e.get("origin", 0),
                                                None if ec is None else _epoch_change(ec)))
    if "verify_batch" in m:
        v = m["verify_batch"]
        return HashOrigin(HashOriginVerifyBatch(v.get("source", 0), v.get("seq_no", 0),
                                                _acks(v.get("request_acks", [])), v.get("expected_digest", b"")))
    return HashOrigin(None)


def decode_event(b: bytes) -> RecordedEvent:
    """One recording.Event (recording.proto:14-18)."""
    m = _decode(b, "recording.Event")
    kind = 0
    for fn, _, v in _fields(b):          # which state.Event oneof member is set (any, known or not)
        if fn == 3:
            for f2, _, _ in _fields(v):
                kind = f2
    ev = RecordedEvent(m.get("node_id", 0), m.get("time", 0), kind)
    hr = m.get("state_event", {}).get("hash_result")
    if hr is not None:
        ev.hash_result = HashResultEvent(ev.node_id, ev.time, hr.get("digest", b""),
                                         _hash_origin(hr.get("origin", {})))
    return ev


def read_events(source: Union[str, bytes, io.IOBase]) -> Iterator[RecordedEvent]:
    """eventlog.Reader.ReadEvent over a whole log (interceptor.go:235-289)."""
    if isinstance(source, (bytes, bytearray)):
        raw = io.BytesIO(source)
    elif isinstance(source, str):
        raw = open(source, "rb")
    else:
        raw = source
    try:
        gz = gzip.GzipFile(fileobj=raw)
        stream = io.BufferedReader(gz)
        stream.peek(1)  # surfaces a broken gzip header here, like gzip.NewReader
    except (OSError, EOFError) as e:
        raise EventLogError(f"could not read source as a gzip stream: {e}") from e
    while True:
        try:
            n = _read_varint_signed(stream)
        except (OSError, EOFError) as e:
            raise EventLogError(f"could not read size prefix: {e}") from e
        if n is None:
            return
        body = stream.read(n)
        if len(body) != n:
            raise EventLogError("could not read message")
        yield decode_event(body)


# ---------------------------------------------------------------------------
# encoder (fixtures, round-trip tests)
# ---------------------------------------------------------------------------
def _ack_msg(a: RequestAck) -> dict:
    return {"client_id": a.client_id, "req_no": a.req_no, "digest": a.digest}


def _origin_msg(o: HashOrigin) -> dict:
    t = o.type
    if isinstance(t, HashOriginBatch):
        return {"batch": {"source": t.source, "epoch": t.epoch, "seq_no": t.seq_no,
                          "request_acks": [_ack_msg(a) for a in t.request_acks]}}
    if isinstance(t, HashOriginEpochChange):
        m = {"source": t.source, "origin": t.origin}
        ec = t.epoch_change
        if ec is not None:
            m["epoch_change"] = {
                "new_epoch": ec.new_epoch,
                "checkpoints": [{"seq_no": c.seq_no, "value": c.value} for c in ec.checkpoints],
                "p_set": [{"epoch": e.epoch, "seq_no": e.seq_no, "digest": e.digest} for e in ec.p_set],
                "q_set": [{"epoch": e.epoch, "seq_no": e.seq_no, "digest": e.digest} for e in ec.q_set]}
        return {"epoch_change": m}
    if isinstance(t, HashOriginVerifyBatch):
        return {"verify_batch": {"source": t.source, "seq_no": t.seq_no,
                                 "request_acks": [_ack_msg(a) for a in t.request_acks],
                                 "expected_digest": t.expected_digest}}
    return {}


def encode_event(node_id: int, time: int, hash_result: Optional[Tuple[bytes, HashOrigin]] = None,
                 tick: bool = False) -> bytes:
    """recording.Event{node_id, time, state_event} with a HashResult or a TickElapsed."""
    if hash_result is not None:
        se = {"hash_result": {"digest": hash_result[0], "origin": _origin_msg(hash_result[1])}}
    elif tick:
        se = {"tick_elapsed": {}}
    else:
        raise ValueError("nothing to encode")
    return _encode("recording.Event", {"node_id": node_id, "time": time, "state_event": se})


def write_log(records: List[bytes]) -> bytes:
    """Size-prefixed records (signed varint, writeSizePrefixedProto) in a gzip stream."""
    body = b"".join(_put_varint_signed(len(r)) + r for r in records)
    return gzip.compress(body, mtime=0)


# ---------------------------------------------------------------------------
# the golden-pair check
# ---------------------------------------------------------------------------
@dataclass
class TraceReport:
    hash_results: int = 0
    by_kind: Dict[str, int] = field(default_factory=dict)
    mismatches: List[Tuple[int, HashResultEvent, bytes]] = field(default_factory=list)

    @property
    def ok(self) -> bool:
        return self.hash_results > 0 and not self.mismatches


def verify_trace(hasher, source) -> TraceReport:
    """Re-hash every HashResult's reconstructed input on the GPU (one batch via
    hasher.hash_batch, e.g. mirbft_amd.GPUHasher) and compare with the digest the
    reference recorded."""
    evs = [e.hash_result for e in read_events(source) if e.hash_result is not None]
    rep = TraceReport(hash_results=len(evs))
    for e in evs:
        k = type(e.origin.type).__name__
        rep.by_kind[k] = rep.by_kind.get(k, 0) + 1
    got = hasher.hash_batch([e.hash_data() for e in evs]) if evs else []
    for i, (e, g) in enumerate(zip(evs, got)):
        if g != e.digest:
            rep.mismatches.append((i, e, g))
    return rep


def main(argv=None) -> int:
    """python -m mirbft_amd.eventlog LOG.gz [...]: check recorded HashResults on the GPU."""
    import argparse
    import json
    from .processor import GPUHasher
    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("logs", nargs="+")
    ap.add_argument("--device-mask", type=int, default=1)
    args = ap.parse_args(argv)
    hasher = GPUHasher(device_mask=args.device_mask)
    rc = 0
    for path in args.logs:
        rep = verify_trace(hasher, path)
        print(json.dumps({"log": path, "hash_results": rep.hash_results, "by_kind": rep.by_kind,
                          "mismatches": len(rep.mismatches), "ok": rep.ok}))
        rc |= 0 if rep.ok else 1
    return rc


if __name__ == "__main__":
    raise SystemExit(main())
