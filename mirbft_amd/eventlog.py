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

Protobuf wire format is decoded by hand (no protoc in this image); only the
fields on the hash path are interpreted, every other field is skipped.
Field numbers: protos/recording/recording.proto:14-18,
protos/state/state.proto:16-31,78-109, protos/msgs/msgs.proto:231-235,255-289.
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


def _msg(fn: int, payload: bytes) -> bytes:
    return _put_uvarint(fn << 3 | 2) + _put_uvarint(len(payload)) + payload


def _u64(fn: int, v: int) -> bytes:
    return b"" if v == 0 else _put_uvarint(fn << 3) + _put_uvarint(v & 0xFFFFFFFFFFFFFFFF)


def _bytes(fn: int, v: bytes) -> bytes:
    return b"" if not v else _msg(fn, v)


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
    kind: int                       # state.Event oneof field number (4 = hash_result, 10 = tick_elapsed, ...)
    hash_result: Optional[HashResultEvent] = None


def _request_ack(b: bytes) -> RequestAck:
    c = r = 0
    d = b""
    for fn, _, v in _fields(b):
        if fn == 1: c = v
        elif fn == 2: r = v
        elif fn == 3: d = v
    return RequestAck(c, r, d)


def _epoch_change(b: bytes) -> EpochChange:
    ec = EpochChange(new_epoch=0)
    for fn, _, v in _fields(b):
        if fn == 1:
            ec.new_epoch = v
        elif fn == 2:
            sq, val = 0, b""
            for f2, _, v2 in _fields(v):
                if f2 == 1: sq = v2
                elif f2 == 2: val = v2
            ec.checkpoints.append(Checkpoint(sq, val))
        elif fn in (3, 4):
            ep = sq = 0
            dg = b""
            for f2, _, v2 in _fields(v):
                if f2 == 1: ep = v2
                elif f2 == 2: sq = v2
                elif f2 == 3: dg = v2
            (ec.p_set if fn == 3 else ec.q_set).append(SetEntry(ep, sq, dg))
    return ec


def _hash_origin(b: bytes) -> HashOrigin:
    for fn, _, v in _fields(b):
        if fn == 1:     # Batch{source=1, epoch=2, seq_no=3, request_acks=5}
            o = HashOriginBatch(0, 0, 0)
            for f2, _, v2 in _fields(v):
                if f2 == 1: o.source = v2
                elif f2 == 2: o.epoch = v2
                elif f2 == 3: o.seq_no = v2
                elif f2 == 5: o.request_acks.append(_request_ack(v2))
            return HashOrigin(o)
        if fn == 2:     # EpochChange{source=1, origin=2, epoch_change=3}
            o = HashOriginEpochChange(0, 0, None)
            for f2, _, v2 in _fields(v):
                if f2 == 1: o.source = v2
                elif f2 == 2: o.origin = v2
                elif f2 == 3: o.epoch_change = _epoch_change(v2)
            return HashOrigin(o)
        if fn == 3:     # VerifyBatch{source=1, seq_no=2, request_acks=3, expected_digest=4}
            o = HashOriginVerifyBatch(0, 0)
            for f2, _, v2 in _fields(v):
                if f2 == 1: o.source = v2
                elif f2 == 2: o.seq_no = v2
                elif f2 == 3: o.request_acks.append(_request_ack(v2))
                elif f2 == 4: o.expected_digest = v2
            return HashOrigin(o)
    return HashOrigin(None)


def decode_event(b: bytes) -> RecordedEvent:
    node_id = time = 0
    kind = 0
    hr = None
    for fn, _, v in _fields(b):
        if fn == 1:
            node_id = v
        elif fn == 2:
            time = v - (1 << 64) if v >= 1 << 63 else v  # int64
        elif fn == 3:
            for f2, _, v2 in _fields(v):
                kind = f2
                if f2 == 4:  # EventHashResult{digest=1, origin=2}
                    dg, org = b"", HashOrigin(None)
                    for f3, _, v3 in _fields(v2):
                        if f3 == 1: dg = v3
                        elif f3 == 2: org = _hash_origin(v3)
                    hr = (dg, org)
    ev = RecordedEvent(node_id, time, kind)
    if hr is not None:
        ev.hash_result = HashResultEvent(node_id, time, hr[0], hr[1])
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
def _enc_ack(a: RequestAck) -> bytes:
    return _u64(1, a.client_id) + _u64(2, a.req_no) + _bytes(3, a.digest)


def _enc_epoch_change(ec: EpochChange) -> bytes:
    out = _u64(1, ec.new_epoch)
    for cp in ec.checkpoints:
        out += _msg(2, _u64(1, cp.seq_no) + _bytes(2, cp.value))
    for fn, s in ((3, ec.p_set), (4, ec.q_set)):
        for e in s:
            out += _msg(fn, _u64(1, e.epoch) + _u64(2, e.seq_no) + _bytes(3, e.digest))
    return out


def _enc_origin(o: HashOrigin) -> bytes:
    t = o.type
    if isinstance(t, HashOriginBatch):
        body = _u64(1, t.source) + _u64(2, t.epoch) + _u64(3, t.seq_no)
        for a in t.request_acks:
            body += _msg(5, _enc_ack(a))
        return _msg(1, body)
    if isinstance(t, HashOriginEpochChange):
        body = _u64(1, t.source) + _u64(2, t.origin)
        if t.epoch_change is not None:
            body += _msg(3, _enc_epoch_change(t.epoch_change))
        return _msg(2, body)
    if isinstance(t, HashOriginVerifyBatch):
        body = _u64(1, t.source) + _u64(2, t.seq_no)
        for a in t.request_acks:
            body += _msg(3, _enc_ack(a))
        return _msg(3, body + _bytes(4, t.expected_digest))
    return b""


def encode_event(node_id: int, time: int, hash_result: Optional[Tuple[bytes, HashOrigin]] = None,
                 tick: bool = False) -> bytes:
    """recording.Event{node_id, time, state_event} with a HashResult or a TickElapsed."""
    if hash_result is not None:
        se = _msg(4, _bytes(1, hash_result[0]) + _msg(2, _enc_origin(hash_result[1])))
    elif tick:
        se = _msg(10, b"")
    else:
        raise ValueError("nothing to encode")
    return _u64(1, node_id) + _u64(2, time & 0xFFFFFFFFFFFFFFFF) + _msg(3, se)


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
