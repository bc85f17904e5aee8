"""Event-log golden traces: the reference's log framing and
HashResult reconstruction, checked on CPU with the oracle as the hasher and on
the GPU with the engine."""
import hashlib

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
