"""Host-side mirror of the reference's hash plugin surface, backed by the GPU.

Reference interface (Go, /root/reference/pkg/processor/serial.go):

    type Hasher interface { New() hash.Hash }                              // :21-23
    func ProcessHashActions(hasher Hasher, actions *statemachine.ActionList)
            (*statemachine.EventList, error)                               // :180-198

with the action/event constructors of pkg/statemachine/actions.go:173-187 and
events.go:96-110 and the schema of protos/state/state.proto:78-109,168-171.

Names, argument meaning and error behaviour follow the reference:
``ProcessHashActions`` returns one ``HashResult`` per action, in list order,
whose ``origin`` is the *same object* as the action's; a non-hash action makes
it fail with "unexpected type for Hash action: <type>" (serial.go:192-194),
raised here as ``ProcessorError``. The whole list is hashed by ONE
``msha_hash_actions`` call (one H2D, one launch per GPU, one D2H).

An EpochChange payload the list already carries is packed once (as the Go
drop-in does, go/pkg/processor/gpuhash.go epochChangeAliases): actions whose
origin holds the same EpochChange object, or an equal payload from the same
origin node, share the first one's (off, len), so it crosses PCIe once.

``GPUHasher.new()`` keeps the per-message ``hash.Hash`` surface that
``Client.Propose`` (clients.go:189-192) and the testengine app chain
(recorder.go:288-359) use: writes are buffered and ``sum()`` submits a
one-message batch to the GPU. Nothing in this module hashes on the CPU.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Iterator, List, Optional, Sequence, Union

import numpy as np

from .encoding import EpochChange, RequestAck, checkpoint_hash_data
from .engine import Engine


class ProcessorError(RuntimeError):
    pass


# ---------------------------------------------------------------------------
# state.HashOrigin and friends (protos/state/state.proto:78-104)
# ---------------------------------------------------------------------------
@dataclass
class HashOriginBatch:
    source: int
    epoch: int
    seq_no: int
    request_acks: List[RequestAck] = field(default_factory=list)


@dataclass
class HashOriginVerifyBatch:
    source: int
    seq_no: int
    request_acks: List[RequestAck] = field(default_factory=list)
    expected_digest: bytes = b""


@dataclass
class HashOriginEpochChange:
    source: int
    origin: int
    epoch_change: Optional[EpochChange] = None


@dataclass
class HashOrigin:
    type: Union[HashOriginBatch, HashOriginVerifyBatch, HashOriginEpochChange, None] = None


@dataclass
class ActionHashRequest:
    """state.ActionHashRequest{repeated bytes data; HashOrigin origin} (state.proto:168-171)."""
    data: List[bytes]
    origin: Optional[HashOrigin]


@dataclass
class ActionHash:
    hash: ActionHashRequest


@dataclass
class Action:
    """state.Action: a oneof; only ActionHash is valid on the hash path."""
    type: Any


@dataclass
class EventHashResult:
    """state.EventHashResult{bytes digest; HashOrigin origin} (state.proto:106-109)."""
    digest: bytes
    origin: Optional[HashOrigin]


@dataclass
class EventHashResultType:
    hash_result: EventHashResult


@dataclass
class Event:
    type: Any


class ActionList:
    """statemachine.ActionList (a linked list in Go; order is what matters)."""

    def __init__(self, actions: Optional[Sequence[Action]] = None):
        self._l: List[Action] = list(actions or [])

    def push_back(self, a: Action) -> "ActionList":
        self._l.append(a)
        return self

    def hash(self, data: List[bytes], origin: Optional[HashOrigin]) -> "ActionList":
        """ActionList.Hash (actions.go:173-176)."""
        return self.push_back(action_hash(data, origin))

    def __iter__(self) -> Iterator[Action]:
        return iter(self._l)

    def __len__(self) -> int:
        return len(self._l)


class EventList:
    def __init__(self):
        self._l: List[Event] = []

    def push_back(self, e: Event) -> "EventList":
        self._l.append(e)
        return self

    def hash_result(self, digest: bytes, origin: Optional[HashOrigin]) -> "EventList":
        """EventList.HashResult (events.go:96-99)."""
        return self.push_back(Event(EventHashResultType(EventHashResult(digest, origin))))

    def __iter__(self) -> Iterator[Event]:
        return iter(self._l)

    def __len__(self) -> int:
        return len(self._l)


def action_hash(data: List[bytes], origin: Optional[HashOrigin]) -> Action:
    """statemachine.ActionHash (actions.go:178-187)."""
    return Action(ActionHash(ActionHashRequest(data=list(data), origin=origin)))


# ---------------------------------------------------------------------------
# Hasher
# ---------------------------------------------------------------------------
class _GPUHash:
    """hash.Hash over the GPU engine: Write appends, Sum(b) appends the digest
    of everything written so far without resetting (Go hash.Hash semantics)."""

    size = 32
    block_size = 64

    def __init__(self, engine: Engine):
        self._engine = engine
        self._buf = bytearray()

    def write(self, p: bytes) -> int:
        self._buf += p
        return len(p)

    def sum(self, b: bytes = b"") -> bytes:
        return bytes(b) + self._engine.hash_actions([[bytes(self._buf)]])[0]

    def reset(self) -> None:
        self._buf.clear()


class GPUHasher:
    """processor.Hasher backed by libmirsha; also exposes the batched surface
    ProcessHashActions uses."""

    def __init__(self, engine: Optional[Engine] = None, device_mask: int = 1):
        self.engine = engine if engine is not None else Engine(device_mask)

    def new(self) -> _GPUHash:
        return _GPUHash(self.engine)

    def hash_batch(self, actions: Sequence[Sequence[bytes]]) -> List[bytes]:
        return self.engine.hash_actions(actions)

    def close(self) -> None:
        """Release the packing buffers (the engine stays open)."""
        for name in ("_arena", "_off", "_len", "_out"):
            buf = self.__dict__.pop(name, None)
            if buf is not None and getattr(self.engine, "_ctx", None):
                self.engine.pinned_free(buf)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _pinned(self, name: str, nbytes: int) -> np.ndarray:
        """A page-locked buffer of at least nbytes, grown on demand (the Go
        adapter's pinnedBuf)."""
        buf = getattr(self, name, None)
        if buf is None or buf.size < nbytes:
            if buf is not None:
                self.engine.pinned_free(buf)
            buf = self.engine.pinned_empty(max(nbytes + nbytes // 4, 4096))
            setattr(self, name, buf)
        return buf[:nbytes]

    def hash_requests(self, reqs: Sequence["ActionHashRequest"]) -> List[bytes]:
        """One digest per hash request, packed the way the Go drop-in packs an
        ActionList (gpuhash.go digests): each request's parts back to back,
        16-byte aligned, in a pinned arena; off/len and the digests pinned
        too; ONE msha_digest_batch. EpochChange payloads are packed once
        (_epoch_change_aliases). last_pack holds what was packed."""
        n = len(reqs)
        alias = _epoch_change_aliases(reqs)
        off = self._pinned("_off", 8 * n).view(np.uint64)
        ln = self._pinned("_len", 8 * n).view(np.uint64)
        chunks, pos = [], 0
        for i, r in enumerate(reqs):
            j = alias[i]
            if j >= 0:
                off[i], ln[i] = off[j], ln[j]
                continue
            data = b"".join(r.data)
            off[i], ln[i] = pos, len(data)
            chunks.append((pos, data))
            pos = (pos + len(data) + 15) & ~15
        arena = self._pinned("_arena", pos + 64)
        for p, data in chunks:
            arena[p:p + len(data)] = np.frombuffer(data, dtype=np.uint8)
        out = self._pinned("_out", 32 * n).reshape(n, 32)
        self.engine.digest_batch(arena, off, ln, out=out)
        self.last_pack = {"actions": n, "payloads": len(chunks), "packed_bytes": pos,
                          "payload_bytes": sum(len(d) for _, d in chunks),
                          "aliased": int(sum(1 for a in alias if a >= 0))}
        return [bytes(r) for r in out]

    def request_digests(self, requests: Sequence[bytes]) -> List[bytes]:
        """Batched request intake: the digest that
        Client.Propose computes per call (clients.go:189-192, ``h.Write(data);
        h.Sum(nil)``) for a whole batch of proposals, in one GPU call
        (msha_digest_batch over a packed arena)."""
        if not requests:
            return []
        lens = np.fromiter((len(r) for r in requests), dtype=np.uint64, count=len(requests))
        offs = np.zeros(len(requests), dtype=np.uint64)
        if len(requests) > 1:
            offs[1:] = np.cumsum(lens)[:-1]
        arena = np.frombuffer(b"".join(bytes(r) for r in requests), dtype=np.uint8)
        out = self.engine.digest_batch(arena, offs, lens)
        return [bytes(r) for r in out]


def checkpoint_hashes(hasher: GPUHasher, intervals: Sequence[tuple]) -> List[bytes]:
    """the testengine's app-level checkpoint value
    (NodeState.Snap, recorder.go:288-300) for many (node, interval) pairs in one
    GPU call. intervals[i] = (prev_checkpoint_hash or None, [committed request
    digests]); result[i] = ActiveHash.Sum(nil) at Snap = SHA-256 of
    checkpoint_hash_data(prev, digests). Every part is a 32-byte digest, so this
    is the digest-of-digests kernel over one table of all parts. A node's
    successive intervals form a chain (each starts from the previous result), so
    the batch dimension is across nodes / ready intervals."""
    if not intervals:
        return []
    parts: List[bytes] = []
    begin = [0]
    for prev, digests in intervals:
        for d in checkpoint_hash_data(prev, list(digests)):
            if len(d) != 32:
                raise ProcessorError("checkpoint_hashes: every part must be a 32-byte digest")
            parts.append(bytes(d))
        begin.append(len(parts))
    table = np.frombuffer(b"".join(parts), dtype=np.uint8).reshape(-1, 32) if parts \
        else np.zeros((0, 32), dtype=np.uint8)
    idx = np.arange(len(parts), dtype=np.uint32)
    out = hasher.engine.digest_of_digests(table, idx, np.array(begin, dtype=np.uint64))
    return [bytes(r) for r in out]


def _epoch_change_aliases(reqs: Sequence[ActionHashRequest]) -> List[int]:
    """alias[i] = an earlier request carrying request i's EpochChange payload,
    else -1 (the Go drop-in's epochChangeAliases, gpuhash.go). Each origin's
    EpochChange is hashed once per ack (epoch_target.go:486-528,
    epoch_tracker.go:349-350). The testengine's acks hold the originator's
    message itself (recorder.go:39-47): the same object is the same payload.
    Acks off the wire hold equal copies: payloads from the same origin node
    with the same length are compared byte for byte (an altered copy is packed
    and hashed on its own), and so is a request whose object was seen before
    but whose Data differs in length."""
    alias = [-1] * len(reqs)
    by_obj: dict = {}       # id(EpochChange) -> request index (objects live as long as reqs)
    by_content: dict = {}   # (origin node, length) -> [(index, payload)]
    for i, r in enumerate(reqs):
        t = r.origin.type if r.origin is not None else None
        if not isinstance(t, HashOriginEpochChange):
            continue
        ec = t.epoch_change
        # the same object names the same payload only if the Data built from it is
        # the same (the contract is SHA-256(Data)): part for part the same object
        # or equal bytes (list == compares identity first), else the joined bytes
        data = None
        if ec is not None and id(ec) in by_obj:
            j = by_obj[id(ec)]
            if reqs[j].data == r.data or b"".join(reqs[j].data) == (data := b"".join(r.data)):
                alias[i] = j
                continue
        if data is None:
            data = b"".join(r.data)
        key = (t.origin, len(data))
        match = next((j for j, d in by_content.get(key, ()) if d == data), -1)
        if ec is not None:
            by_obj[id(ec)] = match if match >= 0 else i
        if match >= 0:
            alias[i] = match
        else:
            by_content.setdefault(key, []).append((i, data))
    return alias


def ProcessHashActions(hasher: GPUHasher, actions: ActionList) -> EventList:
    """processor.ProcessHashActions (serial.go:180-198), one GPU batch per list."""
    if not hasattr(hasher, "hash_requests"):
        raise TypeError("ProcessHashActions needs a GPU-backed hasher (GPUHasher); "
                        "this engine has no CPU hashing path")
    reqs: List[ActionHashRequest] = []
    for action in actions:
        t = action.type
        if not isinstance(t, ActionHash):
            raise ProcessorError(f"unexpected type for Hash action: {type(t).__name__}")
        reqs.append(t.hash)
    digests = hasher.hash_requests(reqs) if reqs else []
    events = EventList()
    for r, d in zip(reqs, digests):
        events.hash_result(d, r.origin)
    return events
