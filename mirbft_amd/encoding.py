"""Hash-input formats of MirBFT's three hash-action producers (host logic).

These restate how the reference state machine builds ``ActionHashRequest.Data``
so that tests and synthetic workloads feed the engine exactly the byte strings
the reference would. They are inputs to the hash path, not part of the GPU
kernels.

* Batch          sequence.allocate         /root/reference/pkg/statemachine/sequence.go:155-172
* VerifyBatch    applyForwardBatchMsg      /root/reference/pkg/statemachine/batch_tracker.go:175-188
* EpochChange    epochChangeHashData       /root/reference/pkg/statemachine/stateless.go:323-352
                 uint64ToBytes (BIG-endian) /root/reference/pkg/statemachine/proposer.go:16-20
* checkpoint value (app-level running hash)  NodeState.Snap/Apply/TransferTo
                 /root/reference/pkg/testengine/recorder.go:288-353 (New at :420)
* testengine request payload  RequestByReqNo  /root/reference/pkg/testengine/recorder.go:258-270
                 uint64ToBytes (LITTLE-endian) /root/reference/pkg/testengine/recorder.go:33-37
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional


@dataclass(frozen=True)
class RequestAck:
    """msgs.RequestAck{client_id, req_no, digest} (protos/msgs/msgs.proto:231-235)."""
    client_id: int
    req_no: int
    digest: bytes


@dataclass(frozen=True)
class Checkpoint:
    """msgs.Checkpoint{seq_no, value} as carried by EpochChange.checkpoints."""
    seq_no: int
    value: bytes


@dataclass(frozen=True)
class SetEntry:
    """msgs.EpochChange_SetEntry{epoch, seq_no, digest} (P and Q sets)."""
    epoch: int
    seq_no: int
    digest: bytes


@dataclass
class EpochChange:
    """msgs.EpochChange{new_epoch, checkpoints, p_set, q_set} (protos/msgs/msgs.proto:269-289)."""
    new_epoch: int
    checkpoints: List[Checkpoint] = field(default_factory=list)
    p_set: List[SetEntry] = field(default_factory=list)
    q_set: List[SetEntry] = field(default_factory=list)


def uint64_to_bytes_be(v: int) -> bytes:
    """statemachine.uint64ToBytes: binary.BigEndian.PutUint64 (proposer.go:16-20)."""
    return struct.pack(">Q", v & 0xFFFFFFFFFFFFFFFF)


def uint64_to_bytes_le(v: int) -> bytes:
    """testengine.uint64ToBytes: binary.LittleEndian.PutUint64 (recorder.go:33-37)."""
    return struct.pack("<Q", v & 0xFFFFFFFFFFFFFFFF)


def batch_hash_data(request_acks: List[RequestAck]) -> List[bytes]:
    """Data of a Batch hash action: the acks' digests, in order (sequence.go:155-158).

    (An empty batch never reaches the hasher: sequence.go:149-153 uses a nil digest.)"""
    return [ack.digest for ack in request_acks]


def verify_batch_hash_data(request_acks: List[RequestAck]) -> List[bytes]:
    """Data of a VerifyBatch hash action (batch_tracker.go:175-178); may be empty."""
    return [ack.digest for ack in request_acks]


def epoch_change_hash_data(ec: EpochChange) -> List[bytes]:
    """epochChangeHashData (stateless.go:323-352):
    [BE64(new_epoch)] ++ [BE64(cp.seq_no), cp.value]* ++ [BE64(e.epoch), BE64(e.seq_no), e.digest]* (P) ++ (Q)."""
    data: List[bytes] = [uint64_to_bytes_be(ec.new_epoch)]
    for cp in ec.checkpoints:
        data += [uint64_to_bytes_be(cp.seq_no), cp.value]
    for e in ec.p_set:
        data += [uint64_to_bytes_be(e.epoch), uint64_to_bytes_be(e.seq_no), e.digest]
    for e in ec.q_set:
        data += [uint64_to_bytes_be(e.epoch), uint64_to_bytes_be(e.seq_no), e.digest]
    assert len(data) == 1 + 2 * len(ec.checkpoints) + 3 * len(ec.p_set) + 3 * len(ec.q_set)
    return data


def recorder_request_bytes(client_id: int, req_no: int) -> Optional[bytes]:
    """RecorderClient.RequestByReqNo payload: LE64(client) ++ '-' ++ LE64(reqNo) (17 bytes)."""
    return uint64_to_bytes_le(client_id) + b"-" + uint64_to_bytes_le(req_no)


def checkpoint_hash_data(prev_checkpoint_hash: Optional[bytes], committed_digests: List[bytes]) -> List[bytes]:
    """Everything NodeState.ActiveHash has been written with when Snap takes its
    Sum (recorder.go:288-300): the previous CheckpointHash (written right after
    the previous Snap, :299-300, or by TransferTo, :326-328; absent for the
    first interval, whose ActiveHash is a fresh Hasher.New(), :420), then the
    digest of every request Apply committed since, in commit order (:348)."""
    head = [] if prev_checkpoint_hash is None else [prev_checkpoint_hash]
    return head + list(committed_digests)
