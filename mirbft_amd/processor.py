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


def ProcessHashActions(hasher: GPUHasher, actions: ActionList) -> EventList:
    """processor.ProcessHashActions (serial.go:180-198), one GPU batch per list."""
    if not hasattr(hasher, "hash_batch"):
        raise TypeError("ProcessHashActions needs a GPU-backed hasher (GPUHasher); "
                        "this engine has no CPU hashing path")
    reqs: List[ActionHashRequest] = []
    for action in actions:
        t = action.type
        if not isinstance(t, ActionHash):
            raise ProcessorError(f"unexpected type for Hash action: {type(t).__name__}")
        reqs.append(t.hash)
    digests = hasher.hash_batch([r.data for r in reqs]) if reqs else []
    events = EventList()
    for r, d in zip(reqs, digests):
        events.hash_result(d, r.origin)
    return events
