"""The oracle pinned against FIPS 180-4 known answers and an independent
implementation (hashlib/OpenSSL) on every golden fixture. CPU only."""
import hashlib

import numpy as np
import pytest

from oracle import oracle


def test_kat_vectors(kat):
    for v in kat["vectors"]:
        m = v["msg_ascii"].encode()
        assert oracle.sha256(m).hex() == v["sha256"]
        assert oracle.py_sha256(m).hex() == v["sha256"]


def test_kat_million_a(kat):
    assert oracle.sha256(b"a" * 1_000_000).hex() == kat["million_a"]["sha256"]


def test_lengths_fixture(lengths_golden):
    msgs = [m for m, _ in lengths_golden]
    exp = [d for _, d in lengths_golden]
    arena = np.frombuffer(b"".join(msgs), dtype=np.uint8)
    lens = np.array([len(m) for m in msgs], dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    got = oracle.digest_batch(arena, offs, lens)
    for i, (m, d) in enumerate(lengths_golden):
        assert got[i].tobytes() == d, len(m)
        assert hashlib.sha256(m).digest() == d
        if len(m) <= 300:
            assert oracle.py_sha256(m) == d


def test_actions_fixture(actions_golden):
    got = oracle.process_hash_actions([parts for _, _, parts, _ in actions_golden])
    for (name, _, parts, d), g in zip(actions_golden, got):
        assert g == d, name
        assert hashlib.sha256(b"".join(parts)).digest() == d


def test_streaming_write_boundaries():
    # h.Write in arbitrary chunkings == one-shot (Go digest.Write buffering)
    rng = np.random.default_rng(7)
    for L in (0, 1, 55, 56, 63, 64, 65, 127, 128, 129, 1000):
        m = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        cuts = sorted(rng.integers(0, L + 1, 5).tolist()) if L else []
        parts, prev = [], 0
        for c in cuts + [L]:
            parts.append(m[prev:c])
            prev = c
        assert oracle.process_hash_actions([parts])[0] == hashlib.sha256(m).digest()


def test_digest_of_digests_oracle():
    rng = np.random.default_rng(3)
    table = rng.integers(0, 256, (50, 32), dtype=np.uint8)
    counts = [0, 1, 2, 3, 20, 7]
    idx = rng.integers(0, 50, sum(counts)).astype(np.uint32)
    begin = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    got = oracle.digest_of_digests(table, idx, begin)
    for i in range(len(counts)):
        data = b"".join(table[j].tobytes() for j in idx[begin[i]:begin[i + 1]])
        assert got[i].tobytes() == hashlib.sha256(data).digest()


@pytest.mark.parametrize("L", [0, 17, 512, 640, 65536])
def test_random_lengths_vs_hashlib(L):
    m = np.random.default_rng(L).integers(0, 256, L, dtype=np.uint8).tobytes()
    assert oracle.sha256(m) == hashlib.sha256(m).digest()


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_openssl_oracle_matches_c_oracle(lengths_golden, threads):
    """Third restatement (OpenSSL libcrypto, threaded ranges) == scalar C oracle == fixtures."""
    msgs = [m for m, _ in lengths_golden]
    lens = np.array([len(m) for m in msgs], dtype=np.uint64)
    off = np.zeros(len(msgs), dtype=np.uint64)
    off[1:] = np.cumsum(lens)[:-1]
    arena = np.frombuffer(b"".join(msgs) + b"\0", dtype=np.uint8)
    got = oracle.openssl_digest_batch(arena, off, lens, threads=threads)
    assert np.array_equal(got, oracle.digest_batch(arena, off, lens))
    assert [g.tobytes() for g in got] == [d for _, d in lengths_golden]
