"""GPU parity past 32-bit addressing: payloads at offsets >= 4 GiB in an HBM arena
(one straddling the 4 GiB boundary), under each batch-kernel policy and through
split chaining, and digest-of-digests over a digest table larger than 4 GiB.

The reference places no limit on message sizes or batch sizes (SURVEY.md §8b:
"There is no length limit beyond memory"); with 288 GB of HBM per MI355X a batch
arena beyond 4 GiB is a normal shape (c4 alone is 4 GiB), so every offset, digest
slot and table index in the kernels is 64-bit. Expected digests come from
hashlib / the oracle over host copies of just the written bytes.
"""
import hashlib

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

G4 = 1 << 32
MiB = 1 << 20


@pytest.fixture(scope="module")
def big_arena(engine):
    """(device arena, [(off, payload bytes)]): 4 GiB + 4 MiB of zeros with random payloads written
    below, across and above the 4 GiB boundary."""
    import torch
    rng = np.random.default_rng(0x4B)
    d = torch.zeros(G4 + 4 * MiB + 64, dtype=torch.uint8, device="cuda:0")
    specs = [(0, 119), (G4 - 4096, 8192), (G4, 55), (G4 + 16, 64), (G4 + 1 * MiB, MiB + 7),
             (G4 + 3 * MiB, 0), (G4 + 3 * MiB + 4096, 56)]
    for off, n in specs:
        if n:
            d[off:off + n] = torch.from_numpy(rng.integers(0, 256, n, dtype=np.uint8)).to("cuda:0")
    # payloads may overlap (the straddling one spans the next two: overlapping / aliased
    # payloads are legal in the device API), so read each back after all writes
    payloads = [(off, d[off:off + n].cpu().numpy().tobytes()) for off, n in specs]
    yield d, payloads
    del d
    torch.cuda.empty_cache()


def _run(engine, d_arena, offs, lens, order=None):
    import torch
    off = torch.from_numpy(np.asarray(offs, dtype=np.uint64).view(np.int64)).to("cuda:0")
    ln = torch.from_numpy(np.asarray(lens, dtype=np.uint64).view(np.int64)).to("cuda:0")
    out = torch.empty((len(offs), 32), dtype=torch.uint8, device="cuda:0")
    engine.digest_batch_device(d_arena, off, ln, out, order=order)
    engine.device_status()
    return out.cpu().numpy()


@pytest.mark.parametrize("policy", ["auto", "lane", "coop"])
def test_payloads_beyond_4gib(engine, big_arena, policy):
    d, payloads = big_arena
    # every payload, plus aliases of the straddling and the 1 MiB payloads
    sel = list(range(len(payloads))) + [1, 4, 1]
    offs = [payloads[i][0] for i in sel]
    lens = [len(payloads[i][1]) for i in sel]
    exp = np.array([np.frombuffer(hashlib.sha256(payloads[i][1]).digest(), np.uint8) for i in sel])
    engine.set_kernel_policy(policy)
    try:
        got = _run(engine, d, offs, lens)
    finally:
        engine.set_kernel_policy("auto")
    assert np.array_equal(got, exp)


def test_split_chain_surplus_beyond_4gib(engine, big_arena):
    """q = 2 full rounds of waves + 1 surplus wave: the surplus (the last 64 messages,
    run as a split chain of segment waves) reads payloads above 4 GiB."""
    import torch
    d, payloads = big_arena
    simds = torch.cuda.get_device_properties(0).multi_processor_count * 4
    n = 2 * simds * 64 + 64
    idx = np.zeros(n, dtype=np.int64)                       # main waves: the 119-B payload at offset 0
    idx[-64:] = np.arange(64) % (len(payloads) - 1) + 1     # surplus: the payloads at/above the boundary
    offs = [payloads[i][0] for i in idx]
    lens = [len(payloads[i][1]) for i in idx]
    ref = [np.frombuffer(hashlib.sha256(p).digest(), np.uint8) for _, p in payloads]
    exp = np.array([ref[i] for i in idx])
    assert np.array_equal(_run(engine, d, offs, lens), exp)


def test_digest_of_digests_table_beyond_4gib(engine):
    """Batch digests over a 32-B digest table of 2^27 + 4096 rows (> 4 GiB): the parts
    are rows on both sides of row 2^27 (byte offset 4 GiB)."""
    import torch
    rows = (1 << 27) + 4096
    table = torch.zeros((rows, 32), dtype=torch.uint8, device="cuda:0")
    rng = np.random.default_rng(0x4C)
    used = np.unique(np.concatenate([np.arange(0, 8), np.arange((1 << 27) - 8, (1 << 27) + 8),
                                     np.arange(rows - 8, rows)])).astype(np.int64)
    vals = rng.integers(0, 256, (len(used), 32), dtype=np.uint8)
    table[torch.from_numpy(used).to("cuda:0")] = torch.from_numpy(vals).to("cuda:0")
    counts = [0, 1, 2, 3, 20, 40, 7]
    begin = np.zeros(len(counts) + 1, dtype=np.uint64)
    begin[1:] = np.cumsum(counts)
    pos = rng.integers(0, len(used), int(begin[-1]))         # positions into `used`
    idx = used[pos].astype(np.uint32)
    exp = oracle.digest_of_digests(vals, pos.astype(np.uint32), begin)
    out = torch.empty((len(counts), 32), dtype=torch.uint8, device="cuda:0")
    engine.digest_of_digests_device(table, torch.from_numpy(idx.view(np.int32)).to("cuda:0"),
                                    torch.from_numpy(begin.view(np.int64)).to("cuda:0"), out)
    engine.device_status()
    assert np.array_equal(out.cpu().numpy(), exp)
    del table
    torch.cuda.empty_cache()


def test_message_bit_length_above_32_bits(engine):
    """FIPS 180-4 appends the message length in bits as a 64-bit big-endian word;
    at 2^29 bytes (512 MiB) the bit length passes 2^32 and its high 32-bit word
    becomes nonzero. One wave of messages over one shared 512 MiB payload, with
    lengths just under, at and past 2^29 bytes across every padding case (tail
    r = 0, 1, 55, 56, 63, 64 + ..., one-block and two-block padding), hashed
    through the host entry point with the cooperative and the lane kernels.
    Expected digests: hashlib over the common prefix once, then each tail."""
    base = 1 << 29
    lens = [base - 1, base, base + 1, base + 55, base + 56, base + 63, base + 64, base + 119, base + 120]
    rng = np.random.default_rng(29)
    arena = rng.integers(0, 256, base + 256, dtype=np.uint8)
    pre = hashlib.sha256(memoryview(arena[:base - 1]))
    exp = []
    for n in lens:
        h = pre.copy()
        h.update(memoryview(arena[base - 1:n]))
        exp.append(np.frombuffer(h.digest(), dtype=np.uint8))
    exp = np.stack(exp)
    off = np.zeros(len(lens), dtype=np.uint64)
    ln = np.array(lens, dtype=np.uint64)
    for policy in ("coop", "lane"):
        engine.set_kernel_policy(policy)
        try:
            got = engine.digest_batch(arena, off, ln)
        finally:
            engine.set_kernel_policy("auto")
        assert np.array_equal(got, exp), policy
