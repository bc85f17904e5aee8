"""Seeded random layouts through the host entry points, bit-exact against the oracle.

Each case draws a batch shape -- message count, a length distribution (empty, tiny,
padding boundaries, multi-block, occasional large), an offset layout (packed 16-byte
aligned, unaligned, overlapping, aliased back into a pool, reversed) and an arena kind
(pageable numpy or msha_pinned_alloc) -- and runs it through msha_digest_batch under a
path setting (the small-call path, the pipelined path forced with MSHA_SMALL_BYTES=0,
or the pipelined path over MSHA_VIRTUAL_SHARDS=3). hash_actions and digest_of_digests
get random part structures the same way. The expected digests come from the oracle's
OpenSSL leg (distinct payloads hashed once) or, for parts, hashlib.
"""
import hashlib

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

BOUNDARY = [0, 1, 55, 56, 63, 64, 65, 119, 120, 127, 128]


def _lengths(rng, n):
    kind = rng.integers(0, 4)
    if kind == 0:
        return rng.choice(BOUNDARY, n).astype(np.uint64)
    if kind == 1:
        return rng.integers(0, 700, n).astype(np.uint64)
    if kind == 2:                                   # one size for the whole batch
        return np.full(n, int(rng.choice([0, 17, 512, 640, 4096])), dtype=np.uint64)
    ln = rng.integers(0, 3000, n).astype(np.uint64)   # mostly small, a few large
    big = rng.random(n) < 0.01
    ln[big] = rng.integers(10_000, 200_000, int(big.sum())).astype(np.uint64)
    return ln


def _layout(rng, ln, kind=None):
    """Offsets for lengths ln in an arena; returns (arena_size, off)."""
    n = ln.size
    kind = rng.integers(0, 5) if kind is None else kind
    align = 16 if kind in (0, 3, 4) else 1
    steps = (ln + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    if kind == 1:                                   # unaligned gaps
        steps = steps + rng.integers(0, 9, n).astype(np.uint64)
    off = np.concatenate([[0], np.cumsum(steps)[:-1]]).astype(np.uint64) if n else np.zeros(0, np.uint64)
    size = int(off[-1] + ln[-1]) if n else 0
    if kind == 2:                                   # overlapping windows into one buffer
        size = int(ln.max()) + 5000 if n else 0
        off = rng.integers(0, 5000, n).astype(np.uint64)
    if kind == 3 and n > 1:                         # 10 % alias an earlier message
        src = rng.integers(0, n, n)
        al = (rng.random(n) < 0.1) & (src < np.arange(n))
        off[al], ln[al] = off[src[al]], ln[src[al]]
    if kind == 4:                                   # reversed order in the arena
        off = off[::-1].copy()
        ln[:] = ln[::-1].copy()
    return size, off


def _expect(arena, off, ln):
    if off.size == 0:
        return np.zeros((0, 32), np.uint8)
    key = np.stack([off, ln], axis=1)
    uniq, first, inv = np.unique(key, axis=0, return_index=True, return_inverse=True)
    d = oracle.openssl_digest_batch(arena, off[first], ln[first], 8)
    return d[inv.reshape(-1)]


PATHS = ["small", "pipeline", "sharded"]


@pytest.mark.parametrize("seed", range(36))
def test_random_digest_batch(seed, monkeypatch):
    from mirbft_amd import Engine
    rng = np.random.default_rng(1000 + seed)
    path = PATHS[seed % 3]
    if path != "small":
        monkeypatch.setenv("MSHA_SMALL_BYTES", "0")
    if path == "sharded":
        monkeypatch.setenv("MSHA_VIRTUAL_SHARDS", "3")
    n = int(rng.choice([1, 2, 63, 64, 65, 1000, 5000, 20000]))
    ln = _lengths(rng, n)
    size, off = _layout(rng, ln)
    data = rng.integers(0, 256, size + 64, dtype=np.uint8)
    exp = _expect(data, off, ln)
    with Engine(1) as e:
        pinned = bool(rng.integers(0, 2))
        arena = data
        if pinned:
            arena = e.pinned_empty(data.size)
            arena[:] = data
        st0 = e.stats()
        got = e.digest_batch(arena, off, ln)
        st1 = e.stats()
    assert np.array_equal(got, exp), (path, n, pinned)
    small = st1["small_calls"] - st0["small_calls"]
    if path != "small":
        assert small == 0
    elif int(((ln + np.uint64(15)) // np.uint64(16) * np.uint64(16)).sum()) <= 4 << 20:
        assert small == 1          # within the packed limit: always the latency path


@pytest.mark.parametrize("seed", range(12))
def test_random_hash_actions_and_batches(engine, seed, monkeypatch):
    rng = np.random.default_rng(2000 + seed)
    if seed % 2:
        monkeypatch.setenv("MSHA_SMALL_BYTES", "0")
    n = int(rng.choice([1, 7, 300, 3000]))
    actions = []
    for _ in range(n):
        k = int(rng.integers(0, 6))
        actions.append([rng.integers(0, 256, int(rng.choice(BOUNDARY + [32, 300])), dtype=np.uint8).tobytes()
                        for _ in range(k)])
    assert engine.hash_actions(actions) == [hashlib.sha256(b"".join(p)).digest() for p in actions]
    table = rng.integers(0, 256, size=(int(rng.integers(1, 500)), 32), dtype=np.uint8)
    counts = rng.integers(0, 45, n)
    begin = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    idx = rng.integers(0, table.shape[0], int(begin[-1]), dtype=np.uint32)
    got = engine.digest_of_digests(table, idx, begin)
    assert np.array_equal(got, oracle.digest_of_digests(table, idx, begin))


@pytest.mark.parametrize("seed", range(24))
def test_random_direct_gpu_planned(seed, monkeypatch):
    """The pinned (direct) path, whose lanes the GPU plans (plan.hip): random
    16-byte aligned layouts -- packed, aliased back into the batch, reversed, with
    empty messages and a few large ones -- over 1 to 8 virtual shards, with the
    off/len arrays pageable or pinned (uploaded as they are), every digest
    against the oracle and the call counted as direct."""
    from mirbft_amd import Engine
    rng = np.random.default_rng(3000 + seed)
    monkeypatch.setenv("MSHA_SMALL_BYTES", "0")                 # never the latency path
    monkeypatch.setenv("MSHA_VIRTUAL_SHARDS", str(1 + seed % 8))
    n = int(rng.choice([70_000, 130_000, 200_000]))
    ln = _lengths(rng, n)
    size, off = _layout(rng, ln, kind=int(rng.choice([0, 3, 4])))  # the 16-byte aligned layouts
    data = rng.integers(0, 256, size + 64, dtype=np.uint8)
    exp = _expect(data, off, ln)
    with Engine(1) as e:
        arena = e.pinned_empty(data.size)
        arena[:] = data
        if seed % 2:
            po = e.pinned_empty(off.nbytes).view(np.uint64)
            pl = e.pinned_empty(ln.nbytes).view(np.uint64)
            po[:], pl[:] = off, ln
            off_in, ln_in = po, pl
        else:
            off_in, ln_in = off, ln
        got = e.digest_batch(arena, off_in, ln_in)
        direct = e.stats()["direct_calls"]
    assert np.array_equal(got, exp), (seed, n)
    lo, hi, total = int(off.min()), int((off + ln).max()), int(ln.sum())
    dense = hi > lo and hi - lo <= min(total, hi - lo) + 16 * n + (1 << 20)    # msha_digest_batch's rule
    assert direct == int(dense), (direct, dense)
