"""Seeded synthetic hash-action workloads for BASELINE.json's configs.

PRNG: counter-based splitmix64, seed 0x4D49524246540000
("MIRBFT"); byte k of a stream is byte (k % 8) of splitmix64(seed, k // 8), so
any slice of a workload is reproducible on its own (per-rank shards, test
samples). SHA-256 timing does not depend on the data.

Configs (BASELINE.json "configs"):
  c1  testengine plumbing, 4 nodes / 4 clients, BatchSize 20: correctness only
      (request payloads LE64(client)-LE64(reqNo), 17 B; Batch = 20 x 32 B digests)
  c2  2^20 client requests x 512 B (request digests)               <- headline
  c3  200,000 Batch actions, each 20 x 32-byte request-ack digests (640 B)
  c4  65,536 requests x 64 KiB
  c5  2^23 mixed actions: 70% 512-B requests, 25% Batch (k~U[1,20] x 32 B),
      5% EpochChange drawn from a pool of 100 distinct N=100/CI=500 encodings
      (|P|,|Q| ~ U[0,1000], 2 checkpoints with 332-B values), aliased.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

SEED = 0x4D49524246540000
_G = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, start: int, count: int) -> np.ndarray:
    """splitmix64 outputs start..start+count-1 of the stream `seed` (uint64)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (np.arange(start + 1, start + count + 1, dtype=np.uint64) * _G)
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def random_bytes(seed: int, offset: int, nbytes: int, chunk: int = 1 << 22) -> np.ndarray:
    """Bytes [offset, offset+nbytes) of the splitmix64 byte stream (offset % 8 == 0).
    Chunks are generated on a few threads (numpy releases the GIL): the full-size
    configs need GBs of payload (c4: 4.3 GB)."""
    assert offset % 8 == 0
    out = np.empty(nbytes, dtype=np.uint8)
    w0 = offset // 8
    nwords = (nbytes + 7) // 8

    def fill(s: int) -> None:
        c = min(chunk, nwords - s)
        b = splitmix64(seed, w0 + s, c).view(np.uint8)
        pos = 8 * s
        take = min(8 * c, nbytes - pos)
        out[pos:pos + take] = b[:take]

    starts = range(0, nwords, chunk)
    if nwords <= chunk:
        for s in starts:
            fill(s)
        return out
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        list(ex.map(fill, starts))
    return out


@dataclass
class Workload:
    """Messages arena[off[i] : off[i]+len[i]] (16-byte aligned starts)."""
    name: str
    arena: np.ndarray          # uint8, with >= 64 B slack at the end
    off: np.ndarray            # uint64
    len: np.ndarray            # uint64
    # digest-of-digests form (c3): out[i] = SHA256(table[idx[begin[i]:begin[i+1]]])
    table: Optional[np.ndarray] = None
    idx: Optional[np.ndarray] = None
    begin: Optional[np.ndarray] = None
    uniform_stride: Optional[int] = None   # set when message i starts at i*stride
    shared: Optional[np.ndarray] = None    # c5: True where the message names a shared (aliased) payload

    @property
    def n(self) -> int:
        return int(self.off.size)

    @property
    def message_bytes(self) -> int:
        return int(self.len.sum())

    @property
    def blocks(self) -> int:
        L = self.len.astype(np.uint64)
        return int(((L >> np.uint64(6)) + np.where((L & np.uint64(63)) < 56, 1, 2).astype(np.uint64)).sum())


def _round16(x):
    return (x + 15) & ~15


def uniform_requests(n: int, size: int, seed: int = SEED, first: int = 0, name: str = "uniform") -> Workload:
    """n requests of `size` bytes, message i = requests first+i of the global stream."""
    stride = _round16(size)
    arena = np.zeros(n * stride + 64, dtype=np.uint8)
    if stride == size and size % 8 == 0:
        arena[: n * size] = random_bytes(seed, first * size, n * size)
    else:
        for i in range(n):
            arena[i * stride: i * stride + size] = random_bytes(seed, (first + i) * _round16(size + 7), size)
    off = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    length = np.full(n, size, dtype=np.uint64)
    return Workload(name, arena, off, length, uniform_stride=stride)


def c2_requests(n: int = 1 << 20, size: int = 512, first: int = 0) -> Workload:
    return uniform_requests(n, size, SEED, first, name=f"c2: {n} requests x {size} B")


def c4_large(n: int = 65536, size: int = 65536, first: int = 0) -> Workload:
    return uniform_requests(n, size, SEED ^ 0x4, first, name=f"c4: {n} requests x {size} B")


def c3_batches(n: int = 200_000, k: int = 20, first: int = 0) -> Workload:
    """n Batch actions of k request-ack digests each (32 B): both as a packed
    640-byte arena and as a digest table + index lists (digest-of-digests)."""
    table = random_bytes(SEED ^ 0x3, first * k * 32, n * k * 32).reshape(n * k, 32)
    idx = np.arange(n * k, dtype=np.uint32)
    begin = np.arange(n + 1, dtype=np.uint64) * np.uint64(k)
    size = 32 * k
    stride = _round16(size)
    arena = np.zeros(n * stride + 64, dtype=np.uint8)
    arena[: n * stride].reshape(n, stride)[:, :size] = table.reshape(n, size)
    off = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    length = np.full(n, size, dtype=np.uint64)
    return Workload(f"c3: {n} batches x {k} x 32 B", arena, off, length, table=table, idx=idx,
                    begin=begin, uniform_stride=stride)


def epoch_change_pool(count: int = 100, seed: int = SEED ^ 0x5, n_nodes: int = 100, ci: int = 500,
                      max_set: int = 1000) -> list[bytes]:
    """`count` distinct EpochChange hash payloads (epochChangeHashData concatenated)."""
    from .encoding import Checkpoint, EpochChange, SetEntry, epoch_change_hash_data
    rng = np.random.Generator(np.random.PCG64(seed))
    pool = []
    for c in range(count):
        cps = [Checkpoint(seq_no=ci * (j + 1), value=rng.bytes(332)) for j in range(2)]
        npq = rng.integers(0, max_set + 1, size=2)
        p = [SetEntry(epoch=int(rng.integers(0, 8)), seq_no=int(s), digest=rng.bytes(32))
             for s in range(int(npq[0]))]
        q = [SetEntry(epoch=int(rng.integers(0, 8)), seq_no=int(s), digest=rng.bytes(32))
             for s in range(int(npq[1]))]
        ec = EpochChange(new_epoch=c + 1, checkpoints=cps, p_set=p, q_set=q)
        pool.append(b"".join(epoch_change_hash_data(ec)))
    return pool


def c5_storm(n: int = 1 << 23, first: int = 0, pool: Optional[list] = None) -> Workload:
    """Mixed actions (see module docstring). Action kinds are drawn per index
    from the global stream, so ranks can build disjoint slices independently."""
    u = splitmix64(SEED ^ 0xC5, first, n)
    kind_r = (u >> np.uint64(32)).astype(np.float64) / 2.0 ** 32
    kind = np.where(kind_r < 0.70, 0, np.where(kind_r < 0.95, 1, 2))
    k = ((u & np.uint64(0xFFFF)) % np.uint64(20) + np.uint64(1)).astype(np.uint64)
    ec_pick = ((u >> np.uint64(16)) & np.uint64(0xFFFF)) % np.uint64(100)
    if pool is None:
        pool = epoch_change_pool()
    pool_len = np.array([len(p) for p in pool], dtype=np.uint64)
    pool_off = np.zeros(len(pool), dtype=np.uint64)
    pool_off[1:] = np.cumsum(np.array([_round16(len(p)) for p in pool], dtype=np.uint64))[:-1]
    pool_bytes = int(pool_off[-1] + _round16(int(pool_len[-1])))

    length = np.where(kind == 0, np.uint64(512), np.where(kind == 1, k * np.uint64(32), pool_len[ec_pick]))
    length = length.astype(np.uint64)
    own = kind != 2                          # requests and batches own their payload
    own_sz = np.where(own, (length + np.uint64(15)) & ~np.uint64(15), np.uint64(0))
    own_off = np.zeros(n, dtype=np.uint64)
    own_off[1:] = np.cumsum(own_sz)[:-1]
    own_total = int(own_sz.sum())
    arena = np.zeros(pool_bytes + own_total + 64, dtype=np.uint8)
    for p, o in zip(pool, pool_off):
        arena[int(o): int(o) + len(p)] = np.frombuffer(p, dtype=np.uint8)
    arena[pool_bytes: pool_bytes + own_total] = random_bytes(SEED ^ 0x55, 0, own_total)
    off = np.where(own, own_off + np.uint64(pool_bytes), pool_off[ec_pick]).astype(np.uint64)
    return Workload(f"c5: {n} mixed actions (70/25/5)", arena, off, length, shared=~own)


def unaliased_layout(w: Workload):
    """w's messages packed the way a caller without payload sharing packs an
    ActionList (every action its own copy, in action order, 16-byte aligned:
    go/pkg/processor/gpuhash.go before round 4's epochChangeAliases): (offsets,
    arena bytes)."""
    steps = (w.len + np.uint64(15)) // np.uint64(16) * np.uint64(16)
    off = np.zeros(w.n, dtype=np.uint64)
    if w.n > 1:
        off[1:] = np.cumsum(steps)[:-1]
    return off, int(steps.sum())


def fill_unaliased(w: Workload, new_off: np.ndarray, dst: np.ndarray, threads: int = 16) -> None:
    """Copy w's payloads into dst at new_off (unaliased_layout). Messages that own
    their payload are contiguous runs in both layouts (copied run by run); every
    shared-payload message gets its own copy."""
    assert w.shared is not None
    sh = np.flatnonzero(w.shared)
    # runs of own messages between shared ones: [a, b)
    starts = np.concatenate([[0], sh + 1])
    ends = np.concatenate([sh, [w.n]])
    keep = ends > starts
    runs = list(zip(starts[keep].tolist(), ends[keep].tolist()))

    def copy_part(part):
        lo, hi = part
        for a, b in runs[lo:hi]:
            src0 = int(w.off[a])
            nb = int(w.off[b - 1]) + int(w.len[b - 1]) - src0
            d0 = int(new_off[a])
            dst[d0:d0 + nb] = w.arena[src0:src0 + nb]

    def copy_shared(part):
        lo, hi = part
        for i in sh[lo:hi].tolist():
            o, l, d0 = int(w.off[i]), int(w.len[i]), int(new_off[i])
            dst[d0:d0 + l] = w.arena[o:o + l]

    from concurrent.futures import ThreadPoolExecutor
    T = max(1, threads)
    with ThreadPoolExecutor(max_workers=T) as ex:
        list(ex.map(copy_part, [(len(runs) * t // T, len(runs) * (t + 1) // T) for t in range(T)]))
        list(ex.map(copy_shared, [(len(sh) * t // T, len(sh) * (t + 1) // T) for t in range(T)]))
