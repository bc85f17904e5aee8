"""Generate the committed golden fixtures for the hash path.

Run from the repo root:  python tests/golden/make_golden.py

Expected digests come from Python ``hashlib.sha256`` (OpenSSL 3.0.2 here), an
implementation independent of both oracle/ and the GPU engine. The reference
(Go crypto/sha256 via processor.ProcessHashActions) cannot run in this image
(no Go toolchain) and ships no digest fixtures of its own, so:

* kat.json       FIPS 180-4 / NIST published known answers (values copied from
                 the standard's examples, NOT computed here; make_golden only
                 checks hashlib agrees with them).
* lengths.json   one message per length 0..300 plus every padding boundary
                 (55/56/63/64/119/120 ...) and larger sizes; inputs as hex.
* actions.json   multi-part hash actions as processor.ProcessHashActions sees
                 them: empty parts, zero parts, the Batch / VerifyBatch /
                 EpochChange encodings (mirbft_amd/encoding.py), the 11-byte
                 fake ack digests of the reference's own (disabled) test
                 pkg/statemachine/sequence_test.go:40-107, and testengine
                 request payloads (recorder.go:258-270).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from mirbft_amd.encoding import (Checkpoint, EpochChange, RequestAck, SetEntry,  # noqa: E402
                                 batch_hash_data, epoch_change_hash_data, recorder_request_bytes,
                                 verify_batch_hash_data)
from mirbft_amd.workloads import SEED, random_bytes  # noqa: E402

# FIPS 180-4 / NIST CSRC "SHA-256 examples" known answers.
KAT = [
    ("", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
    ("abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
    ("abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
     "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
    ("abcdefghbcdefghicdefghijdefghijkefghijklfghijklmghijklmnhijklmnoijklmnopjklmnopqklmnopqrlmnopqrsmnopqrstnopqrstu",
     "cf5b16a778af8380036ce59e7b0492370b249b11e8f07a51afac45037afee9d1"),
]
KAT_MILLION_A = "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"

BOUNDARY_LENGTHS = [447, 448, 503, 504, 511, 512, 513, 567, 568, 575, 576, 577, 639, 640, 1000,
                    1023, 1024, 1025, 4095, 4096, 4097, 65535, 65536]


def H(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def msg_for_length(L: int) -> bytes:
    # message of length L = bytes [L*2^20, L*2^20 + L) of the fixture stream
    return random_bytes(SEED ^ 0x60, L << 20, L).tobytes()


def make_kat():
    for m, d in KAT:
        assert H(m.encode()) == d, m
    assert H(b"a" * 1_000_000) == KAT_MILLION_A
    return {
        "source": "FIPS 180-4 / NIST CSRC SHA-256 examples (published values)",
        "vectors": [{"msg_ascii": m, "sha256": d} for m, d in KAT],
        "million_a": {"msg": "'a' * 1000000", "sha256": KAT_MILLION_A},
    }


def make_lengths():
    out = []
    for L in list(range(0, 301)) + BOUNDARY_LENGTHS:
        m = msg_for_length(L)
        e = {"len": L, "sha256": H(m)}
        if L <= 1025:
            e["msg_hex"] = m.hex()
        else:
            e["msg_gen"] = "random_bytes(SEED ^ 0x60, len << 20, len)"
        out.append(e)
    return {"generator": "mirbft_amd.workloads.random_bytes", "messages": out}


def ack(c, r, d):
    return RequestAck(client_id=c, req_no=r, digest=d)


def make_actions():
    actions = []

    def add(name, parts, kind="generic"):
        actions.append({"name": name, "kind": kind, "parts_hex": [p.hex() for p in parts],
                        "sha256": H(b"".join(parts))})

    add("zero parts", [])
    add("one empty part", [b""])
    add("three empty parts", [b"", b"", b""])
    add("empty parts around data", [b"", b"abc", b"", b""])
    add("abc split", [b"a", b"b", b"c"])
    add("block-straddling parts", [bytes(range(60)), bytes(range(10)), bytes(200)])
    for L in (55, 56, 63, 64, 119, 120):
        m = msg_for_length(L)
        add(f"len {L} split 3 ways", [m[: L // 3], m[L // 3: 2 * L // 3], m[2 * L // 3:]])
    # Reference's own (disabled) sequence test uses 11-byte fake digests:
    # pkg/statemachine/sequence_test.go:40-107 -> Hash([]{"msg1-digest","msg2-digest"}, Batch{...})
    add("sequence_test fake acks", batch_hash_data([ack(1, 1, b"msg1-digest"), ack(2, 1, b"msg2-digest")]),
        kind="batch")
    # Batch of 20 real request digests (config c1/c3 shape).
    reqs = [recorder_request_bytes(c, r) for c in range(4) for r in range(5)]
    acks = [ack(c, r, hashlib.sha256(recorder_request_bytes(c, r)).digest()) for c in range(4) for r in range(5)]
    add("batch 20 request digests", batch_hash_data(acks), kind="batch")
    add("batch 1 request digest", batch_hash_data(acks[:1]), kind="batch")
    add("verify batch empty (zero parts)", verify_batch_hash_data([]), kind="verify_batch")
    add("verify batch 7", verify_batch_hash_data(acks[:7]), kind="verify_batch")
    for r in reqs[:6]:
        add(f"testengine request {r.hex()}", [r], kind="request")
    ec0 = EpochChange(new_epoch=1)
    add("epoch change, no sets", epoch_change_hash_data(ec0), kind="epoch_change")
    ec1 = EpochChange(new_epoch=4,
                      checkpoints=[Checkpoint(20, b"\x11" * 40), Checkpoint(40, b"\x22" * 332)],
                      p_set=[SetEntry(3, 21, b"\x33" * 32), SetEntry(3, 22, b"")],   # null batch: empty digest
                      q_set=[SetEntry(2, 21, b"\x44" * 32), SetEntry(3, 21, b"\x33" * 32)])
    add("epoch change, checkpoints + P/Q with empty digest", epoch_change_hash_data(ec1), kind="epoch_change")
    big = EpochChange(new_epoch=7,
                      checkpoints=[Checkpoint(500 * (j + 1), random_bytes(SEED ^ 0x61, 512 * j, 332).tobytes())
                                   for j in range(2)],
                      p_set=[SetEntry(6, s, random_bytes(SEED ^ 0x62, 32 * s, 32).tobytes()) for s in range(300)],
                      q_set=[SetEntry(5, s, random_bytes(SEED ^ 0x63, 32 * s, 32).tobytes()) for s in range(200)])
    add("epoch change, 300 P + 200 Q entries", epoch_change_hash_data(big), kind="epoch_change")
    return {"actions": actions}


def main():
    for name, fn in (("kat.json", make_kat), ("lengths.json", make_lengths), ("actions.json", make_actions)):
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(fn(), f, indent=1)
            f.write("\n")
        print("wrote", name)


if __name__ == "__main__":
    main()
