"""GPU parity: libmirsha (HIP, gfx950) vs the CPU oracle and the golden fixtures.

Every check is bit-exact. Run on the GPU box:  python -m pytest tests -m gpu -x -q
"""
import hashlib

import numpy as np
import pytest

from mirbft_amd import _lib as L
from mirbft_amd import (ActionList, GPUHasher, HashOrigin, HashOriginBatch, HashOriginEpochChange,
                        HashOriginVerifyBatch, MshaError, ProcessHashActions, ProcessorError,
                        pack_parts)
from mirbft_amd.encoding import EpochChange, RequestAck
from mirbft_amd import workloads as W
from oracle import oracle

pytestmark = pytest.mark.gpu


def _arena_from(msgs, align=16):
    offs, pos = [], 0
    for m in msgs:
        offs.append(pos)
        pos += (len(m) + align - 1) // align * align if align else len(m)
    arena = np.zeros(pos + 64, dtype=np.uint8)
    for o, m in zip(offs, msgs):
        arena[o:o + len(m)] = np.frombuffer(m, dtype=np.uint8)
    return arena, np.array(offs, dtype=np.uint64), np.array([len(m) for m in msgs], dtype=np.uint64)


@pytest.fixture(params=["small", "small_copy", "pipeline"])
def host_path(request, engine, monkeypatch):
    """Run a host-API test through the small-call path (calls of a few actions
    zero-copy: the kernel reads the packed list and writes the digests in coherent
    pinned memory; larger ones one H2D, one launch, one D2H), through the small path
    with zero-copy off (MSHA_SMALL_ZC_BYTES=0) and through the pipelined path
    (forced by MSHA_SMALL_BYTES=0), and check which one ran (msha_stats.small_calls,
    small_zc_calls)."""
    monkeypatch.delenv("MSHA_SMALL_ZC_BYTES", raising=False)
    if request.param == "pipeline":
        monkeypatch.setenv("MSHA_SMALL_BYTES", "0")
    else:
        monkeypatch.delenv("MSHA_SMALL_BYTES", raising=False)
        monkeypatch.delenv("MSHA_SMALL_MSGS", raising=False)
        if request.param == "small_copy":
            monkeypatch.setenv("MSHA_SMALL_ZC_BYTES", "0")
    before = engine.stats()
    yield request.param
    after = engine.stats()
    ran = after["small_calls"] - before["small_calls"]
    zc = after["small_zc_calls"] - before["small_zc_calls"]
    assert ran > 0 if request.param != "pipeline" else ran == 0
    if request.param != "small":
        assert zc == 0


# ---------------------------------------------------------------- fixtures --
def test_kat(engine, kat, host_path):
    msgs = [v["msg_ascii"].encode() for v in kat["vectors"]] + [b"a" * 1_000_000]
    exp = [v["sha256"] for v in kat["vectors"]] + [kat["million_a"]["sha256"]]
    got = engine.hash_actions([[m] for m in msgs])
    assert [g.hex() for g in got] == exp


def test_lengths_golden_one_batch(engine, lengths_golden, host_path):
    msgs = [m for m, _ in lengths_golden]
    arena, off, ln = _arena_from(msgs)
    got = engine.digest_batch(arena, off, ln)
    for i, (m, d) in enumerate(lengths_golden):
        assert got[i].tobytes() == d, f"len {len(m)}"


def test_lengths_golden_unaligned_host_arena(engine, lengths_golden, host_path):
    # caller arena with arbitrary (unaligned) offsets: the library repacks
    msgs = [m for m, _ in lengths_golden]
    arena, off, ln = _arena_from(msgs, align=0)
    got = engine.digest_batch(arena, off, ln)
    assert [g.tobytes() for g in got] == [d for _, d in lengths_golden]


def test_actions_golden(engine, actions_golden, host_path):
    got = engine.hash_actions([parts for _, _, parts, _ in actions_golden])
    for (name, _, _, d), g in zip(actions_golden, got):
        assert g == d, name


def test_each_length_alone(engine, lengths_golden, host_path):
    # one-message batches: exercises the launch path at n=1 for every padding case
    for m, d in lengths_golden[:130]:
        assert engine.hash_actions([[m]])[0] == d, len(m)


# ------------------------------------------------- reference-shaped surface --
def test_process_hash_actions_mirror(engine, actions_golden):
    """serial.go:180-198: one HashResult per action, in order, same Origin object."""
    hasher = GPUHasher(engine)
    al = ActionList()
    origins = []
    for i, (name, kind, parts, _) in enumerate(actions_golden):
        if kind == "epoch_change":
            o = HashOrigin(HashOriginEpochChange(source=i, origin=i, epoch_change=EpochChange(new_epoch=i)))
        elif kind == "verify_batch":
            o = HashOrigin(HashOriginVerifyBatch(source=i, seq_no=i, expected_digest=b""))
        else:
            o = HashOrigin(HashOriginBatch(source=i, epoch=0, seq_no=i))
        origins.append(o)
        al.hash(parts, o)
    events = ProcessHashActions(hasher, al)
    assert len(events) == len(actions_golden)
    for ev, o, (name, _, _, d) in zip(events, origins, actions_golden):
        assert ev.type.hash_result.origin is o
        assert ev.type.hash_result.digest == d, name
        assert len(ev.type.hash_result.digest) == 32


def test_process_hash_actions_empty_list(engine):
    assert len(ProcessHashActions(GPUHasher(engine), ActionList())) == 0


def test_process_hash_actions_error(engine):
    from mirbft_amd.processor import Action
    al = ActionList().hash([b"x"], None)
    al.push_back(Action(type="not a hash"))
    with pytest.raises(ProcessorError, match="unexpected type for Hash action"):
        ProcessHashActions(GPUHasher(engine), al)


def test_gpu_hash_object_semantics(engine):
    """hash.Hash: Write appends; Sum(b) appends the digest and does NOT reset."""
    h = GPUHasher(engine).new()
    h.write(b"ab")
    h.write(b"")
    h.write(b"c")
    assert h.sum() == hashlib.sha256(b"abc").digest()
    assert h.sum(b"prefix") == b"prefix" + hashlib.sha256(b"abc").digest()
    h.write(b"d")
    assert h.sum() == hashlib.sha256(b"abcd").digest()


# ------------------------------------------------------------ randomized --
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_multipart_vs_oracle(engine, seed):
    rng = np.random.default_rng(seed)
    actions = []
    for _ in range(3000):
        nparts = int(rng.integers(0, 6))
        actions.append([rng.integers(0, 256, int(rng.integers(0, 400)), dtype=np.uint8).tobytes()
                        for _ in range(nparts)])
    assert engine.hash_actions(actions) == oracle.process_hash_actions(actions)


def test_aliased_payloads(engine):
    """EpochChange re-hashing: many actions alias one payload (off/len repeated)."""
    pool = [bytes(np.random.default_rng(i).integers(0, 256, 1000 * (i + 1), dtype=np.uint8)) for i in range(5)]
    arena, off, ln = _arena_from(pool)
    pick = np.random.default_rng(9).integers(0, 5, 2000)
    got = engine.digest_batch(arena, off[pick], ln[pick])
    exp = [hashlib.sha256(p).digest() for p in pool]
    for g, k in zip(got, pick):
        assert g.tobytes() == exp[k]


def test_alias_dedup_keys_on_offset_and_length(engine):
    """Hash dedup is per (off, len): a shared start with different lengths, or
    equal bytes at different offsets, are distinct lanes; repeats copy digests."""
    base = bytes(np.random.default_rng(3).integers(0, 256, 5000, dtype=np.uint8))
    arena = np.zeros(2 * 5008 + 64, dtype=np.uint8)
    arena[:5000] = np.frombuffer(base, dtype=np.uint8)
    arena[5008:10008] = np.frombuffer(base, dtype=np.uint8)
    off = np.array([0, 0, 0, 5008, 0, 16, 0], dtype=np.uint64)
    ln = np.array([5000, 4999, 5000, 5000, 0, 100, 5000], dtype=np.uint64)
    got = engine.digest_batch(arena, off, ln)
    for g, o, n_ in zip(got, off, ln):
        assert g.tobytes() == hashlib.sha256(arena[int(o):int(o + n_)].tobytes()).digest()


def test_mixed_sizes_many_lanes(engine):
    """> 3 waves/SIMD of mixed sizes: non-prefetch kernel + size-class ordering."""
    n = 250_000
    rng = np.random.default_rng(11)
    lens = rng.choice([0, 17, 55, 56, 64, 120, 512, 640, 1500], n).astype(np.uint64)
    stride = (lens + 15) // 16 * 16
    off = np.concatenate([[0], np.cumsum(stride)[:-1]]).astype(np.uint64)
    arena = W.random_bytes(W.SEED ^ 0x70, 0, int(stride.sum()) + 64)
    got = engine.digest_batch(arena, off, lens)
    exp = oracle.digest_batch(arena, off, lens)
    assert np.array_equal(got, exp)


def test_out_of_range_rejected(engine):
    arena = np.zeros(100, dtype=np.uint8)
    with pytest.raises(MshaError) as ei:
        engine.digest_batch(arena, np.array([90], dtype=np.uint64), np.array([20], dtype=np.uint64))
    assert ei.value.code == L.MSHA_ERR_INVALID_ARG


@pytest.mark.parametrize("n_actions", [1000, 300_000])
def test_hash_actions_rejects_first_bad_part(engine, n_actions):
    """msha_hash_actions validates on several threads from 2^18 parts on: the
    error still names the FIRST part outside the arena, a non-monotone
    action_part_begin is rejected, and a valid batch of that size is bit-exact."""
    rng = np.random.default_rng(n_actions)
    per = rng.integers(0, 5, n_actions)
    begin = np.concatenate([[0], np.cumsum(per)]).astype(np.uint64)
    n_parts = int(begin[-1])
    arena = W.random_bytes(W.SEED ^ 0x72, 0, 4096)
    plen = rng.integers(0, 64, n_parts).astype(np.uint64)
    poff = rng.integers(0, 4096 - 64, n_parts).astype(np.uint64)
    got = engine.hash_actions_packed(arena, poff, plen, begin)
    for a in rng.integers(0, n_actions, 64).tolist() + [0, n_actions - 1]:
        msg = b"".join(arena[int(poff[j]):int(poff[j] + plen[j])].tobytes()
                       for j in range(int(begin[a]), int(begin[a + 1])))
        assert got[a].tobytes() == hashlib.sha256(msg).digest()
    bad = poff.copy()
    first, later = n_parts // 3, n_parts - 2
    bad[later] = 4090
    bad[first] = 4095
    plen2 = plen.copy()
    plen2[[first, later]] = 10
    with pytest.raises(MshaError) as ei:
        engine.hash_actions_packed(arena, bad, plen2, begin)
    assert ei.value.code == L.MSHA_ERR_INVALID_ARG and f"part {first} outside arena" in str(ei.value)
    b2 = begin.copy()
    b2[n_actions // 2] = b2[n_actions // 2 + 1] + 1
    with pytest.raises(MshaError) as ei:
        engine.hash_actions_packed(arena, poff, plen, b2)
    assert "non-decreasing" in str(ei.value)


def test_digest_of_digests_rejects_index_past_table(engine):
    """The index check of msha_digest_of_digests (threaded from 2^18 indices)."""
    n = 20_000
    table = W.random_bytes(W.SEED ^ 0x73, 0, 32 * 4096).reshape(4096, 32)
    idx = np.random.default_rng(5).integers(0, 4096, 20 * n).astype(np.uint32)
    begin = (np.arange(n + 1) * 20).astype(np.uint64)
    idx[-1] = 4096
    with pytest.raises(MshaError) as ei:
        engine.digest_of_digests(table, idx, begin)
    assert ei.value.code == L.MSHA_ERR_INVALID_ARG and "idx out of table range" in str(ei.value)
    idx[-1] = 4095
    out = engine.digest_of_digests(table, idx, begin)
    assert out[-1].tobytes() == hashlib.sha256(table[idx[-20:]].tobytes()).digest()


def test_empty_batch(engine):
    out = engine.digest_batch(np.zeros(0, dtype=np.uint8), np.zeros(0, dtype=np.uint64),
                              np.zeros(0, dtype=np.uint64))
    assert out.shape == (0, 32)
    assert engine.hash_actions([]) == []


def test_large_single_message(engine):
    m = W.random_bytes(W.SEED ^ 0x71, 0, (64 << 20) + 13).tobytes()
    assert engine.hash_actions([[m], [b"x"], [m[:1000]]]) == [hashlib.sha256(m).digest(),
                                                              hashlib.sha256(b"x").digest(),
                                                              hashlib.sha256(m[:1000]).digest()]


# ------------------------------------------------ digest-of-digests path --
def test_digest_of_digests_host(engine):
    rng = np.random.default_rng(5)
    table = rng.integers(0, 256, (500, 32), dtype=np.uint8)
    counts = rng.integers(0, 21, 3000)
    counts[:4] = [0, 1, 2, 20]
    idx = rng.integers(0, 500, int(counts.sum())).astype(np.uint32)
    begin = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    got = engine.digest_of_digests(table, idx, begin)
    assert np.array_equal(got, oracle.digest_of_digests(table, idx, begin))


def test_request_then_batch_chain_on_device(engine):
    """c1/c3 shape end to end on the GPU: request digests -> Batch digests over them."""
    import torch
    from mirbft_amd.encoding import recorder_request_bytes
    reqs = [recorder_request_bytes(c, r) for c in range(4) for r in range(50)]
    arena, off, ln = _arena_from(reqs)
    dev = torch.device("cuda:0")
    d_arena = torch.from_numpy(arena).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_len = torch.from_numpy(ln.view(np.int64)).to(dev)
    d_req = torch.empty((len(reqs), 32), dtype=torch.uint8, device=dev)
    engine.digest_batch_device(d_arena, d_off, d_len, d_req)
    # 10 batches of 20 acks each
    idx = torch.arange(len(reqs), dtype=torch.int32, device=dev)
    begin = torch.arange(0, len(reqs) + 1, 20, dtype=torch.int64, device=dev)
    d_batch = torch.empty((10, 32), dtype=torch.uint8, device=dev)
    engine.digest_of_digests_device(d_req, idx, begin, d_batch)
    engine.device_status()
    req_d = [hashlib.sha256(r).digest() for r in reqs]
    assert [bytes(x) for x in d_req.cpu().numpy()] == req_d
    exp = [hashlib.sha256(b"".join(req_d[20 * i:20 * i + 20])).digest() for i in range(10)]
    assert [bytes(x) for x in d_batch.cpu().numpy()] == exp


# ------------------------------------------------ device-resident paths --
def _to_dev(w: W.Workload):
    import torch
    dev = torch.device("cuda:0")
    return (torch.from_numpy(w.arena).to(dev), torch.from_numpy(w.off.view(np.int64)).to(dev),
            torch.from_numpy(w.len.view(np.int64)).to(dev))


def test_c2_full_size_bit_exact(engine):
    """BASELINE config c2 at full size (2^20 x 512 B): every digest vs the oracle."""
    import torch
    w = W.c2_requests()
    d_arena, d_off, d_len = _to_dev(w)
    out = torch.empty((w.n, 32), dtype=torch.uint8, device="cuda:0")
    before = engine.stats()
    engine.digest_batch_device(d_arena, d_off, d_len, out)
    engine.device_status()
    # the kernel bench.py times for c2: one lane per message, nothing else
    st = engine.stats()
    assert st["launches_lane"] == before["launches_lane"] + 1
    assert all(st[k] == before[k] for k in ("launches_pipe", "launches_coop", "launches_split"))
    out2 = torch.empty_like(out)
    engine.digest_uniform_device(d_arena, w.uniform_stride, 512, w.n, out2)
    engine.device_status()
    exp = oracle.digest_batch(w.arena, w.off, w.len)
    assert np.array_equal(out.cpu().numpy(), exp)
    assert np.array_equal(out2.cpu().numpy(), exp)


def test_c3_full_size_bit_exact(engine):
    """BASELINE config c3 (200K Batch actions x 20 x 32 B): both kernel forms."""
    import torch
    w = W.c3_batches()
    dev = torch.device("cuda:0")
    table = torch.from_numpy(np.ascontiguousarray(w.table)).to(dev)
    idx = torch.from_numpy(w.idx.view(np.int32)).to(dev)
    begin = torch.from_numpy(w.begin.view(np.int64)).to(dev)
    out = torch.empty((w.n, 32), dtype=torch.uint8, device=dev)
    before = engine.stats()
    engine.digest_of_digests_device(table, idx, begin, out)
    engine.device_status()
    # bench.py's c3dd and c3 legs time split chaining (3 full waves per SIMD + a
    # surplus): a planner change that moved either form off it would fail here
    mid = engine.stats()
    assert mid["launches_split"] == before["launches_split"] + 1 and mid["launches_dod"] == before["launches_dod"]
    d_arena, d_off, d_len = _to_dev(w)
    out2 = torch.empty_like(out)
    engine.digest_batch_device(d_arena, d_off, d_len, out2)
    engine.device_status()
    st = engine.stats()
    assert st["launches_split"] == mid["launches_split"] + 1
    assert all(st[k] == mid[k] for k in ("launches_lane", "launches_pipe", "launches_coop"))
    exp = oracle.digest_batch(w.arena, w.off, w.len)
    assert np.array_equal(out.cpu().numpy(), exp)
    assert np.array_equal(out2.cpu().numpy(), exp)


def _oracle_threaded(w, threads: int = 16):
    """Every digest of a full-size workload: the OpenSSL leg of the oracle over
    `threads` threads, each distinct (off, len) payload hashed once."""
    key = (w.off << np.uint64(24)) | w.len          # off < 2^40, len < 2^24 in these configs
    assert int(w.off.max()) < (1 << 40) and int(w.len.max()) < (1 << 24)
    uniq, first, inv = np.unique(key, return_index=True, return_inverse=True)
    d = oracle.openssl_digest_batch(w.arena, w.off[first], w.len[first], threads)
    return d[inv.reshape(-1)]


def test_c4_full_size_bit_exact(engine):
    """BASELINE config c4 (65,536 x 64 KiB) at full size, every digest vs the oracle,
    through BOTH kernels that run it: the off/len pipelined lane kernel
    (k_digest_batch_pipe, the one bench.py times) and the uniform-layout one."""
    import torch
    w = W.c4_large()
    exp = _oracle_threaded(w)
    d_arena, d_off, d_len = _to_dev(w)
    out = torch.empty((w.n, 32), dtype=torch.uint8, device="cuda:0")
    before = engine.stats()
    engine.digest_batch_device(d_arena, d_off, d_len, out)
    engine.device_status()
    assert engine.stats()["launches_pipe"] == before["launches_pipe"] + 1   # the timed kernel ran
    assert np.array_equal(out.cpu().numpy(), exp)
    out.zero_()
    engine.digest_uniform_device(d_arena, w.uniform_stride, 65536, w.n, out)
    engine.device_status()
    assert np.array_equal(out.cpu().numpy(), exp)
    del d_arena, d_off, d_len, out
    torch.cuda.empty_cache()


def test_c5_full_size_ordered_device(engine):
    """BASELINE config c5 at its full 2^23 actions on one GPU, through the ordered
    device path bench.py times (size-class order, aliased EpochChange payloads):
    every digest vs the oracle."""
    import torch
    from mirbft_amd.engine import order_by_blocks
    w = W.c5_storm()
    exp = _oracle_threaded(w)
    d_arena, d_off, d_len = _to_dev(w)
    d_order = torch.from_numpy(order_by_blocks(w.len).view(np.int32)).to("cuda:0")
    out = torch.empty((w.n, 32), dtype=torch.uint8, device="cuda:0")
    engine.digest_batch_device(d_arena, d_off, d_len, out, order=d_order)
    engine.device_status()
    assert np.array_equal(out.cpu().numpy(), exp)
    del d_arena, d_off, d_len, d_order, out
    torch.cuda.empty_cache()


def test_misaligned_device_message_flagged(engine):
    import torch
    arena = torch.zeros(4096, dtype=torch.uint8, device="cuda:0")
    off = torch.tensor([0, 8], dtype=torch.int64, device="cuda:0")
    ln = torch.tensor([10, 10], dtype=torch.int64, device="cuda:0")
    out = torch.full((2, 32), 0xAB, dtype=torch.uint8, device="cuda:0")
    engine.digest_batch_device(arena, off, ln, out)
    with pytest.raises(MshaError) as ei:
        engine.device_status()
    assert ei.value.code == L.MSHA_ERR_ALIGNMENT
    o = out.cpu().numpy()
    assert o[0].tobytes() == hashlib.sha256(b"\0" * 10).digest()
    assert not o[1].any()
    engine.device_status()  # flag was cleared


def test_c5_sample_mixed(engine):
    """BASELINE config c5 mix (requests / batches / aliased EpochChange pool) at 2^17 actions."""
    w = W.c5_storm(1 << 17)
    got = engine.digest_batch(w.arena, w.off, w.len)
    exp = oracle.digest_batch(w.arena, w.off, w.len)
    assert np.array_equal(got, exp)


def test_pack_parts_layout():
    arena, po, pl, b = pack_parts([[b"ab", b""], [], [b"c"]])
    assert arena.tobytes() == b"abc" and list(pl) == [2, 0, 1] and list(b) == [0, 2, 2, 3]


def test_c5_device_ordered(engine):
    """Mixed sizes through the device path with the size-class order (bench c5 form)."""
    import torch
    from mirbft_amd.engine import order_by_blocks
    w = W.c5_storm(1 << 16)
    d_arena, d_off, d_len = _to_dev(w)
    d_order = torch.from_numpy(order_by_blocks(w.len).view(np.int32)).to("cuda:0")
    out = torch.empty((w.n, 32), dtype=torch.uint8, device="cuda:0")
    engine.digest_batch_device(d_arena, d_off, d_len, out, order=d_order)
    engine.device_status()
    assert np.array_equal(out.cpu().numpy(), oracle.digest_batch(w.arena, w.off, w.len))


@pytest.mark.parametrize("staged", ["1", "0"])
@pytest.mark.parametrize("shards", [2, 3])
def test_host_path_sharded(shards, staged, monkeypatch):
    """The multi-GPU host path (partition by blocks, per-shard placement, alias
    dedup reset per shard, per-shard order) on virtual shards of one GPU: the
    staged direct path, and the gather pipeline (MSHA_STAGED_DIRECT=0)."""
    from mirbft_amd import Engine
    monkeypatch.setenv("MSHA_VIRTUAL_SHARDS", str(shards))
    monkeypatch.setenv("MSHA_STAGED_DIRECT", staged)
    with Engine(1) as e:
        w = W.c5_storm(1 << 15)                      # aliased EpochChange pool + mixed sizes
        assert np.array_equal(e.digest_batch(w.arena, w.off, w.len),
                              oracle.digest_batch(w.arena, w.off, w.len))
        rng = np.random.default_rng(shards)
        actions = [[rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
                    for _ in range(int(rng.integers(0, 4)))] for _ in range(5000)]
        assert e.hash_actions(actions) == oracle.process_hash_actions(actions)
        st = e.stats()
        assert st["calls"] == 2 and st["messages"] == w.n + len(actions)


def test_host_path_chunked_large_batch(engine):
    """A batch spanning many 32 MiB staging chunks (c2 at full size) through the host API."""
    w = W.c2_requests()
    got = engine.digest_batch(w.arena, w.off, w.len)
    assert np.array_equal(got, oracle.digest_batch(w.arena, w.off, w.len))


def test_request_digests_batched_intake(engine):
    """8f-1: Client.Propose's digest (clients.go:189-192) for a batch of proposals in one call."""
    from mirbft_amd.encoding import recorder_request_bytes
    reqs = [recorder_request_bytes(c, r) for c in range(4) for r in range(200)] + [b"", b"x" * 512]
    got = GPUHasher(engine).request_digests(reqs)
    assert got == [hashlib.sha256(r).digest() for r in reqs]
    assert GPUHasher(engine).request_digests([]) == []


def test_missing_device_in_mask_is_an_error():
    from mirbft_amd import Engine, device_count
    n = device_count()
    with pytest.raises(MshaError) as ei:
        Engine(1 << n)          # one past the last visible device
    assert ei.value.code == L.MSHA_ERR_NO_DEVICE


def test_pinned_arena_direct_upload(engine):
    """A batch packed in msha_pinned_alloc memory with 16-B aligned starts is DMA'd
    as is (stats.direct_calls); misaligned or gappy layouts take the gather path.
    Digests identical either way, with aliases and mixed sizes."""
    w = W.c5_storm(1 << 14)
    pinned = engine.pinned_empty(w.arena.size)
    pinned[:] = w.arena
    exp = oracle.digest_batch(w.arena, w.off, w.len)
    before = engine.stats()["direct_calls"]
    assert np.array_equal(engine.digest_batch(pinned, w.off, w.len), exp)
    assert engine.stats()["direct_calls"] == before + 1
    # an unaligned start: gather path, same digests
    off2 = w.off.copy()
    pinned2 = engine.pinned_empty(w.arena.size + 16)
    pinned2[8:8 + w.arena.size] = w.arena
    off2 += 8
    assert np.array_equal(engine.digest_batch(pinned2, off2, w.len), exp)
    assert engine.stats()["direct_calls"] == before + 1
    # pageable memory of the same shape: the same GPU-planned path, staged
    staged = engine.stats()["staged_calls"]
    assert np.array_equal(engine.digest_batch(w.arena, w.off, w.len), exp)
    assert engine.stats()["direct_calls"] == before + 1
    assert engine.stats()["staged_calls"] == staged + 1


def _mismatch(w, got, exp, e, what):
    """What a failed comparison tells: how many digests differ, their messages'
    block counts, and the call's figures (heads, lanes, split retries)."""
    bad = np.nonzero(np.any(got != exp, axis=1))[0]
    blocks = (w.len[bad].astype(np.int64) + 8) // 64 + 1
    st = e.stats()
    return {"what": what, "bad": int(bad.size), "first": bad[:8].tolist(),
            "blocks": sorted(set(blocks.tolist()))[:16],
            "split_retries": st.get("split_retries"),
            "shards": [{k: s[k] for k in ("lanes", "head_lanes", "messages")} for s in e.shard_stats()]}


def _oracle_dedup(w):
    """Oracle digests of a batch with many aliases: hash each distinct (off, len) once."""
    key = np.stack([w.off, w.len], axis=1)
    uniq, inv = np.unique(key, axis=0, return_inverse=True)
    return oracle.digest_batch(w.arena, uniq[:, 0].copy(), uniq[:, 1].copy())[inv.reshape(-1)]


def test_alias_table_regions_large_batch(engine):
    """>= 2^20 messages with aliases: the alias table is built over 16 hash regions
    (bucketed keys, prefetched probes); pageable (gather) and pinned (direct) paths."""
    w = W.c5_storm((1 << 20) + 4099)
    exp = _oracle_dedup(w)
    assert np.array_equal(engine.digest_batch(w.arena, w.off, w.len), exp)
    pinned = engine.pinned_empty(w.arena.size)
    pinned[:] = w.arena
    before = engine.stats()["direct_calls"]
    assert np.array_equal(engine.digest_batch(pinned, w.off, w.len), exp)
    assert engine.stats()["direct_calls"] == before + 1


@pytest.mark.parametrize("layout", ["ascending", "reversed", "mixed_aliased"])
@pytest.mark.parametrize("pinned_out", [False, True])
def test_pinned_direct_chunked_span(engine, layout, pinned_out):
    """Direct uploads larger than one 64 MiB span chunk: kernels start per landed
    chunk (lanes grouped by the chunk completing their payload) and identity-order
    digests come back per launch, into the caller's buffer when it is pinned."""
    if layout == "mixed_aliased":
        w = W.c5_storm(1 << 18)
        exp = _oracle_dedup(w)
    else:
        w = W.c2_requests(3 << 16)                   # 96 MiB of 512-B requests
        if layout == "reversed":                     # lane order descends through the span
            w.off = w.off[::-1].copy()
            w.len = w.len[::-1].copy()
        exp = oracle.digest_batch(w.arena, w.off, w.len)
    pinned = engine.pinned_empty(w.arena.size)
    pinned[:] = w.arena
    out = engine.pinned_empty(w.n * 32).reshape(w.n, 32) if pinned_out else None
    before = engine.stats()["direct_calls"]
    got = engine.digest_batch(pinned, w.off, w.len, out=out)
    assert engine.stats()["direct_calls"] == before + 1
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("pinned_out", [False, True])
def test_pinned_direct_streamed_digests_shuffled(engine, pinned_out):
    """Ordered direct lanes stream their digests back after each launch (the
    slots below the lowest slot any later lane group writes). A c5 batch whose
    messages are shuffled within index windows -- slot order and arena order
    agree only roughly, so each launch finalises a different, ragged prefix --
    plus aliases, over several 64 MiB upload pieces: every digest bit-exact."""
    w = W.c5_storm(1 << 19)
    rng = np.random.default_rng(5)
    perm = np.arange(w.n)
    for a in range(0, w.n, 4096):          # shuffle inside 4,096-message windows
        rng.shuffle(perm[a:a + 4096])
    w.off = w.off[perm].copy()
    w.len = w.len[perm].copy()
    exp = _oracle_dedup(w)
    pinned = engine.pinned_empty(w.arena.size)
    pinned[:] = w.arena
    out = engine.pinned_empty(w.n * 32).reshape(w.n, 32) if pinned_out else None
    before = engine.stats()["direct_calls"]
    got = engine.digest_batch(pinned, w.off, w.len, out=out)
    assert engine.stats()["direct_calls"] == before + 1
    assert np.array_equal(got, exp)
    assert w.arena.size > 3 * (64 << 20)   # several upload pieces, several lane groups


def test_pinned_direct_chunked_sharded(monkeypatch):
    """The chunked direct path over 2 virtual shards of one GPU (each shard its own span)."""
    from mirbft_amd import Engine
    monkeypatch.setenv("MSHA_VIRTUAL_SHARDS", "2")
    with Engine(1) as e:
        w = W.c5_storm(3 << 17)
        pinned = e.pinned_empty(w.arena.size)
        pinned[:] = w.arena
        out = e.pinned_empty(w.n * 32).reshape(w.n, 32)
        assert np.array_equal(e.digest_batch(pinned, w.off, w.len, out=out), _oracle_dedup(w))
        w2 = W.c2_requests(3 << 16)
        p2 = e.pinned_empty(w2.arena.size)
        p2[:] = w2.arena
        assert np.array_equal(e.digest_batch(p2, w2.off, w2.len),
                              oracle.digest_batch(w2.arena, w2.off, w2.len))
        assert e.stats()["direct_calls"] == 2


def _pinned_copy(e, a: np.ndarray) -> np.ndarray:
    """a copied into msha_pinned_alloc memory (same dtype and shape)."""
    p = e.pinned_empty(a.nbytes).view(a.dtype).reshape(a.shape)
    p[...] = a
    return p


@pytest.mark.parametrize("shards", [1, 3, 8])
def test_pinned_direct_gpu_planned(shards, monkeypatch):
    """The direct path is planned on the GPU (plan.hip): aliases folded by the
    device hash table, lanes bucketed by (upload piece, descending blocks),
    digest slots streamed back per group. c5 batches over 1, 3 and 8 virtual
    shards, with pageable and pinned off/len (the latter uploaded as they are):
    every digest bit-exact, every shard's first kernel queued and its planner
    timed."""
    from mirbft_amd import Engine
    monkeypatch.setenv("MSHA_VIRTUAL_SHARDS", str(shards))
    w = W.c5_storm(3 << 17)
    exp = _oracle_dedup(w)
    with Engine(1) as e:
        arena = _pinned_copy(e, w.arena)
        out = e.pinned_empty(w.n * 32).reshape(w.n, 32)
        for meta in ("pageable", "pinned"):
            off, ln = (w.off, w.len) if meta == "pageable" else (_pinned_copy(e, w.off), _pinned_copy(e, w.len))
            out[...] = 0
            got = e.digest_batch(arena, off, ln, out=out)
            assert np.array_equal(got, exp), meta
            sh = e.shard_stats()
            assert len(sh) == shards and sum(s["messages"] for s in sh) == w.n
            assert all(s["first_launch_ms"] > 0 and s["plan_kernel_ms"] > 0 for s in sh), sh
            assert sum(s["lanes"] for s in sh) < w.n                      # aliases folded on the GPU
            # upload and kernel spans lie inside the shard's device window
            assert all(0 < s["upload_ms"] <= s["device_ms"] + 1e-3 and 0 < s["kernel_ms"] <= s["device_ms"] + 1e-3
                       for s in sh), sh
        assert e.stats()["direct_calls"] == 2


def test_pinned_alloc_striped_over_numa_nodes(monkeypatch):
    """msha_pinned_alloc on a context whose GPUs sit on several NUMA nodes cuts the
    allocation into one region per shard, each bound to its GPU's node, and
    page-locks it with hipHostRegister. MSHA_PINNED_STRIPE=1 forces that path on
    this one-node box: the memory must still count as pinned (the direct path
    runs), give bit-exact digests over 3 virtual shards, and free cleanly."""
    from mirbft_amd import Engine
    monkeypatch.setenv("MSHA_PINNED_STRIPE", "1")
    monkeypatch.setenv("MSHA_VIRTUAL_SHARDS", "3")
    w = W.c5_storm(1 << 17)
    exp = _oracle_dedup(w)
    with Engine(1) as e:
        arena = _pinned_copy(e, w.arena)
        out = e.pinned_empty(w.n * 32).reshape(w.n, 32)
        got = e.digest_batch(arena, _pinned_copy(e, w.off), _pinned_copy(e, w.len), out=out)
        assert np.array_equal(got, exp)
        assert e.stats()["direct_calls"] == 1
        small = e.pinned_empty(100)                     # smaller than one 2 MiB region
        small[:] = 7
        assert e._lib.msha_pinned_free(e._ctx, small.ctypes.data) == 0
        e._pinned.remove(small.ctypes.data)


def test_early_metadata_upload_on_every_path():
    """Pinned off/len of a one-shard call go up before validation (EarlyMeta);
    only the direct path consumes that upload. With a pageable arena (the
    pipeline path), an unaligned pinned arena, and a batch that fails validation,
    the call must still be bit-exact or fail cleanly, and the next direct call
    correct."""
    from mirbft_amd import Engine
    w = W.c2_requests(n=100_000)
    exp = oracle.digest_batch(w.arena, w.off, w.len)
    with Engine(1) as e:
        off, ln = _pinned_copy(e, w.off), _pinned_copy(e, w.len)
        assert np.array_equal(e.digest_batch(w.arena, off, ln), exp)          # pageable arena
        parena = _pinned_copy(e, w.arena)
        shifted = e.pinned_empty(w.arena.size + 1)
        shifted[1:] = w.arena
        off1 = _pinned_copy(e, w.off + np.uint64(1))
        assert np.array_equal(e.digest_batch(shifted, off1, ln), exp)         # unaligned: not direct
        bad = _pinned_copy(e, w.off)
        bad[-1] = w.arena.size                                               # outside the arena
        with pytest.raises(MshaError):
            e.digest_batch(parena, bad, ln)
        before = e.stats()["direct_calls"]
        assert np.array_equal(e.digest_batch(parena, off, ln), exp)          # direct, early metadata
        assert e.stats()["direct_calls"] == before + 1


@pytest.mark.parametrize("shards", [1, 3])
def test_staged_direct_pageable(shards, monkeypatch):
    """A pageable arena of the direct path's shape (16-B aligned, dense) is planned
    on the GPU like a pinned one, its touched runs copied through two pinned
    staging slots while earlier ones upload and their lane groups hash: c5
    batches (aliases folded on the GPU) with pageable or pinned off/len and
    pageable or pinned digests, bit-exact, staged_calls counted, the copy timed;
    with MSHA_STAGED_DIRECT=0 the same batch takes the gather pipeline."""
    from mirbft_amd import Engine
    monkeypatch.setenv("MSHA_VIRTUAL_SHARDS", str(shards))
    w = W.c5_storm(3 << 17)
    exp = _oracle_dedup(w)
    with Engine(1) as e:
        for meta, outk in (("pageable", "pageable"), ("pinned", "pinned")):
            off, ln = (w.off, w.len) if meta == "pageable" else (_pinned_copy(e, w.off), _pinned_copy(e, w.len))
            out = None if outk == "pageable" else e.pinned_empty(w.n * 32).reshape(w.n, 32)
            st0 = e.stats()
            got = e.digest_batch(w.arena, off, ln, out=out)
            assert np.array_equal(got, exp), _mismatch(w, got, exp, e, (meta, outk))
            st1 = e.stats()
            assert st1["staged_calls"] == st0["staged_calls"] + 1 and st1["direct_calls"] == st0["direct_calls"]
            sh = e.shard_stats()
            assert sum(s["lanes"] for s in sh) < w.n
            assert all(s["gather_ms"] > 0 and s["first_launch_ms"] > 0 for s in sh), sh
        monkeypatch.setenv("MSHA_STAGED_DIRECT", "0")
        st0 = e.stats()
        assert np.array_equal(e.digest_batch(w.arena, w.off, w.len), exp)
        assert e.stats()["staged_calls"] == st0["staged_calls"]


@pytest.mark.parametrize("shards", [1, 3])
def test_staged_direct_interleaved(shards, monkeypatch):
    """The staged (pageable) direct path with its interleavings forced: 256 KiB
    upload pieces, 128 KiB staging slots and a 40 us pause before each refill, so
    the plan is read, the long payloads' heads start on the side stream and lane
    groups launch between slot refills while later pieces still upload -- the
    orderings a wrong digest there would come from (slot refill after its
    slot_free event, a piece's event after all its bytes are queued, heads behind
    their piece, the head D2H behind the last head; DESIGN.md (d) "The staged
    path's orderings"). c5 batches with pageable and pinned off/len and digests:
    every digest exact, the heads ran, and launches were issued before the last
    staging copy (the interleaving happened)."""
    from mirbft_amd import Engine
    monkeypatch.setenv("MSHA_VIRTUAL_SHARDS", str(shards))
    monkeypatch.setenv("MSHA_DIRECT_PIECE_SHIFT", "18")
    monkeypatch.setenv("MSHA_STAGED_SLOT_BYTES", str(128 << 10))
    monkeypatch.setenv("MSHA_STAGED_DELAY_US", "40")
    w = W.c5_storm(1 << 17)
    exp = _oracle_dedup(w)
    with Engine(1) as e:
        for meta, outk in (("pageable", "pageable"), ("pinned", "pinned"), ("pageable", "pinned")):
            off, ln = (w.off, w.len) if meta == "pageable" else (_pinned_copy(e, w.off), _pinned_copy(e, w.len))
            out = None if outk == "pageable" else e.pinned_empty(w.n * 32).reshape(w.n, 32)
            st0 = e.stats()
            got = e.digest_batch(w.arena, off, ln, out=out)
            assert np.array_equal(got, exp), _mismatch(w, got, exp, e, (meta, outk))
            assert e.stats()["staged_calls"] == st0["staged_calls"] + 1
            sh = e.shard_stats()
            assert all(s["head_lanes"] > 0 for s in sh), sh
            # a kernel was queued before the shard's last staging copy ended
            assert all(0 < s["first_launch_ms"] < s["gather_end_ms"] for s in sh), sh


def _pinned_batch(e, lens, offs=None, seed=21):
    """A pinned arena holding messages of the given lengths (16-byte aligned starts
    unless offs is given) and the oracle's digests."""
    lens = np.asarray(lens, dtype=np.uint64)
    if offs is None:
        offs = np.zeros(lens.size, dtype=np.uint64)
        offs[1:] = np.cumsum((lens + np.uint64(15)) & ~np.uint64(15))[:-1]
    offs = np.asarray(offs, dtype=np.uint64)
    size = int((offs + lens).max()) + 64
    host = W.random_bytes(seed, 0, size)
    arena = e.pinned_empty(size)
    arena[:] = host
    w = W.Workload("planner-edge", host, offs, lens)
    return arena, w, _oracle_dedup(w)


def test_gpu_planner_edge_cases(engine):
    """The GPU lane planner (plan.hip) on the shapes its fast paths do not cover:
    (a) every message one payload (one lane, all others aliases);
    (b) 4,096 distinct block counts in one 4,096-message tile, so the LDS key table
        (1,024 slots) overflows and lanes fall back to the global counters;
    (c) a 64 MiB message among 70,000 requests: pieces x (bmax + 1) > 2^20
        counters, so lanes are bucketed by upload piece only;
    (d) zero-length messages everywhere (and a shard of nothing else, below)."""
    # (a) 100,000 actions on one 300-byte payload (+ one other)
    lens = np.full(100_001, 300, dtype=np.uint64)
    offs = np.zeros(100_001, dtype=np.uint64)
    offs[-1] = 320
    arena, w, exp = _pinned_batch(engine, lens, offs)
    before = engine.stats()["direct_calls"]
    assert np.array_equal(engine.digest_batch(arena, w.off, w.len), exp)
    assert engine.shard_stats()[0]["lanes"] == 2
    # (b) lengths i * 64 + 5: block counts 1 .. 4,096, all distinct, in one tile
    i = np.arange(4096, dtype=np.uint64)
    arena, w, exp = _pinned_batch(engine, i * np.uint64(64) + np.uint64(5), seed=22)
    assert np.array_equal(engine.digest_batch(arena, w.off, w.len), exp)
    # (c) two 64 MiB messages among 70,000 x 512 B
    lens = np.full(70_002, 512, dtype=np.uint64)
    lens[7] = lens[50_000] = 64 << 20
    arena, w, exp = _pinned_batch(engine, lens, seed=23)
    assert np.array_equal(engine.digest_batch(arena, w.off, w.len), exp)
    # (d) every third message empty
    lens = np.full(90_000, 700, dtype=np.uint64)
    lens[::3] = 0
    arena, w, exp = _pinned_batch(engine, lens, seed=24)
    assert np.array_equal(engine.digest_batch(arena, w.off, w.len), exp)
    assert engine.stats()["direct_calls"] == before + 4


def test_gpu_planner_shard_of_empty_messages(monkeypatch):
    """Over 3 virtual shards, a batch whose middle third is zero-length messages
    only: that shard uploads nothing and hashes SHA-256("") for every one."""
    from mirbft_amd import Engine
    monkeypatch.setenv("MSHA_VIRTUAL_SHARDS", "3")
    lens = np.full(300_000, 50, dtype=np.uint64)      # 1 block each, like an empty message:
    lens[100_000:200_000] = 0                         # the partition cuts at 100,000 and 200,000
    with Engine(1) as e:
        arena, w, exp = _pinned_batch(e, lens, seed=25)
        got = e.digest_batch(arena, w.off, w.len)
        assert np.array_equal(got, exp)
        assert bytes(got[150_000]) == hashlib.sha256(b"").digest()
        sh = e.shard_stats()
        assert len(sh) == 3 and e.stats()["direct_calls"] == 1
        assert [s["messages"] for s in sh] == [100_000] * 3, sh
        assert sh[1]["h2d_payload_bytes"] == 0 and sh[0]["h2d_payload_bytes"] > 0, sh


def test_pinned_direct_empty_message_at_arena_end(engine):
    """A zero-length message whose offset is the arena's length, in an exact-size
    pinned arena ending on a page boundary, through the pipelined direct path
    (> 64 K messages): it needs no bytes, so no upload reads past the arena
    (ADVICE r2), and its digest is SHA-256("")."""
    w = W.c2_requests(3 << 16)
    n = w.n + 1
    size = (w.arena.size + 4095) // 4096 * 4096
    arena = engine.pinned_empty(size)
    arena[: w.arena.size] = w.arena
    off = np.append(w.off, np.uint64(size))
    ln = np.append(w.len, np.uint64(0))
    before = engine.stats()["direct_calls"]
    got = engine.digest_batch(arena, off, ln)
    assert engine.stats()["direct_calls"] == before + 1
    assert np.array_equal(got[:-1], oracle.digest_batch(w.arena, w.off, w.len))
    assert bytes(got[-1]) == hashlib.sha256(b"").digest()
    assert engine.shard_stats()[0]["h2d_payload_bytes"] <= size


def _cus():
    import torch
    return torch.cuda.get_device_properties(0).multi_processor_count


@pytest.mark.parametrize("rounds", [1, 2])
@pytest.mark.parametrize("surplus_waves,tail", [(1, 0), (6, 17), (53, 0), (None, 5)])
def test_split_chaining_tail(engine, rounds, surplus_waves, tail):
    """Launches of q >= 1 full rounds of waves plus a surplus of 1..SIMDs/2 waves
    run the surplus as split chains (a message's state handed between segment
    waves); every digest bit-exact vs the oracle, with and without a lane order,
    mixed lengths (segments of 0 blocks included), and through the host API."""
    import torch
    simds = _cus() * 4
    r = surplus_waves if surplus_waves is not None else simds // 2    # max surplus
    n = rounds * simds * 64 + r * 64 - (64 - tail if tail else 0)
    rng = np.random.default_rng(r)
    lens = rng.choice(np.array([0, 55, 56, 64, 119, 640, 1000], dtype=np.uint64), size=n)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum((lens + np.uint64(15)) & ~np.uint64(15))[:-1]
    arena = W.random_bytes(7, 0, int(offs[-1] + lens[-1]) + 128)
    w = W.Workload("split", arena, offs, lens)
    exp = oracle.digest_batch(w.arena, w.off, w.len)
    d_arena, d_off, d_len = _to_dev(w)
    out = torch.empty((n, 32), dtype=torch.uint8, device="cuda:0")
    split0 = engine.stats()["launches_split"]
    engine.digest_batch_device(d_arena, d_off, d_len, out)
    engine.device_status()
    assert np.array_equal(out.cpu().numpy(), exp)
    from mirbft_amd.engine import order_by_blocks
    d_order = torch.from_numpy(order_by_blocks(w.len).view(np.int32)).to("cuda:0")
    out.zero_()
    engine.digest_batch_device(d_arena, d_off, d_len, out, order=d_order)
    engine.device_status()
    assert np.array_equal(out.cpu().numpy(), exp)
    assert engine.stats()["launches_split"] == split0 + 2     # both launches were split chains
    # host API (lane-indexed metadata + out_idx through the pipeline)
    assert np.array_equal(engine.digest_batch(w.arena, w.off, w.len), exp)


@pytest.mark.parametrize("rounds", [1, 2])
@pytest.mark.parametrize("surplus_waves,tail", [(1, 0), (7, 33), (None, 0)])
def test_split_chaining_digest_of_digests(engine, rounds, surplus_waves, tail):
    """Digest-of-digests launches with a surplus of waves run the surplus as split
    chains; ragged digest counts (0, 1, odd, even, up to 40) so segments start on
    pair blocks, the odd-digest final block and the length-only final block."""
    import torch
    simds = _cus() * 4
    r = surplus_waves if surplus_waves is not None else simds // 2
    n = rounds * simds * 64 + r * 64 - (64 - tail if tail else 0)
    rng = np.random.default_rng(100 + r)
    table = rng.integers(0, 256, size=(4096, 32), dtype=np.uint8)
    cnt = rng.choice(np.array([0, 1, 2, 3, 19, 20, 40], dtype=np.uint64), size=n)
    begin = np.zeros(n + 1, dtype=np.uint64)
    begin[1:] = np.cumsum(cnt)
    idx = rng.integers(0, table.shape[0], size=int(begin[-1]), dtype=np.uint32)
    exp = oracle.digest_of_digests(table, idx, begin)
    out = torch.empty((n, 32), dtype=torch.uint8, device="cuda:0")
    split0 = engine.stats()["launches_split"]
    engine.digest_of_digests_device(torch.from_numpy(table).to("cuda:0"),
                                    torch.from_numpy(idx.view(np.int32)).to("cuda:0"),
                                    torch.from_numpy(begin.view(np.int64)).to("cuda:0"), out)
    engine.device_status()
    assert engine.stats()["launches_split"] == split0 + 1
    assert np.array_equal(out.cpu().numpy(), exp)
    assert np.array_equal(engine.digest_of_digests(table, idx, begin), exp)


@pytest.mark.parametrize("split,count", [(False, c) for c in (0, 1, 2, 3, 20, 21, 40, 1000)]
                         + [(True, c) for c in (0, 1, 2, 3, 20, 21, 40, 121)])
def test_digest_of_digests_uniform_counts(engine, count, split):
    """Whole waves of Batch digests with one digest count: an even count takes the
    wave-uniform final block (length-only, schedule on the SALU), an odd one the VALU
    final block; 0 parts is SHA256(""). split: a launch with surplus waves (split chains),
    >= 131 K Batches, so its longest case is 121 digests (a 1000-digest one would be 4 GB
    of oracle input)."""
    import torch
    n = 2 * _cus() * 4 * 64 + 3 * 64 + 5 if split else 64 * 6 + 5
    rng = np.random.default_rng(200 + count)
    table = rng.integers(0, 256, size=(2048, 32), dtype=np.uint8)
    begin = np.arange(n + 1, dtype=np.uint64) * np.uint64(count)
    idx = rng.integers(0, table.shape[0], size=int(begin[-1]), dtype=np.uint32)
    exp = oracle.digest_of_digests(table, idx, begin)
    if count == 0:
        idx = np.zeros(1, dtype=np.uint32)   # no part is read, but the device API takes no null pointer
        assert bytes(exp[0]) == hashlib.sha256(b"").digest()
    out = torch.empty((n, 32), dtype=torch.uint8, device="cuda:0")
    engine.digest_of_digests_device(torch.from_numpy(table).to("cuda:0"),
                                    torch.from_numpy(idx.view(np.int32)).to("cuda:0"),
                                    torch.from_numpy(begin.view(np.int64)).to("cuda:0"), out)
    engine.device_status()
    assert np.array_equal(out.cpu().numpy(), exp)


def test_split_chaining_long_surplus_message(engine):
    """A 32 MiB message among the surplus waves of an unordered launch: its chain's
    segments run ~0.2 s each, far past the handoff timeout, but the running segment's
    per-block progress beat keeps the waiting segments from timing out."""
    import torch
    simds = _cus() * 4
    n = 2 * simds * 64 + 64
    lens = np.full(n, 64, dtype=np.uint64)
    lens[-3] = 32 << 20
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum((lens + np.uint64(15)) & ~np.uint64(15))[:-1]
    arena = W.random_bytes(11, 0, int(offs[-1] + lens[-1]) + 128)
    w = W.Workload("split-long", arena, offs, lens)
    exp = oracle.digest_batch(w.arena, w.off, w.len)
    d_arena, d_off, d_len = _to_dev(w)
    out = torch.empty((n, 32), dtype=torch.uint8, device="cuda:0")
    engine.digest_batch_device(d_arena, d_off, d_len, out)
    engine.device_status()
    assert np.array_equal(out.cpu().numpy(), exp)


def test_direct_upload_compacted_ranges_sharded(monkeypatch):
    """Direct (pinned) uploads over 4 virtual shards of a c5 batch whose aliased
    EpochChange pool sits at the arena's start: each shard uploads its own slice
    plus only the pool granules its aliases touch (before: every shard's span
    started at offset 0, ~2.5x the arena in total at 4 shards)."""
    from mirbft_amd import Engine
    monkeypatch.setenv("MSHA_VIRTUAL_SHARDS", "4")
    w = W.c5_storm(1 << 18)
    own = w.len != 0
    pool_bytes = int((w.off + w.len)[w.len > 4096].max())          # EpochChange payloads: the pool
    with Engine(1) as e:
        pinned = e.pinned_empty(w.arena.size)
        pinned[:] = w.arena
        got = e.digest_batch(pinned, w.off, w.len)
        assert np.array_equal(got, _oracle_dedup(w))
        sh = e.shard_stats()
        assert len(sh) == 4 and e.stats()["direct_calls"] == 1
        payload = sum(s["h2d_payload_bytes"] for s in sh)
        granule_slack = 4 * 2 * 65536
        assert payload <= w.arena.size + 3 * pool_bytes + granule_slack, (payload, w.arena.size, pool_bytes)
        assert e.stats()["h2d_bytes"] == sum(s["h2d_bytes"] for s in sh)
        assert sum(s["messages"] for s in sh) == w.n and own.any()


@pytest.mark.parametrize("staged", ["1", "0"])
def test_pageable_gather_runs_per_shard_in_parallel(monkeypatch, staged):
    """Pageable arenas over 2 shards: one gather/issue thread per GPU, so the
    host copies for the two shards overlap in time instead of alternating on
    one thread (msha_shard_stats gather windows) -- on the staged direct path
    and on the gather pipeline (MSHA_STAGED_DIRECT=0)."""
    from mirbft_amd import Engine
    monkeypatch.setenv("MSHA_VIRTUAL_SHARDS", "2")
    monkeypatch.setenv("MSHA_STAGED_DIRECT", staged)
    w = W.c2_requests(1 << 20)                  # 512 MiB: 8 staging chunks per shard
    with Engine(1) as e:
        # the first call also allocates each shard's pinned staging (hipHostMalloc
        # calls the runtime may serialise across threads): time the second
        e.digest_batch(w.arena, w.off, w.len)
        got = e.digest_batch(w.arena, w.off, w.len)
        assert np.array_equal(got, oracle.digest_batch(w.arena, w.off, w.len))
        sh = e.shard_stats()
        assert all(s["gather_ms"] > 0 for s in sh)
        assert max(s["gather_begin_ms"] for s in sh) < min(s["gather_end_ms"] for s in sh), sh
        assert sum(s["h2d_payload_bytes"] for s in sh) == int(w.len.sum())
        assert sum(s["launches"] for s in sh) >= 2


@pytest.mark.parametrize("shards", [1, 2])
def test_concurrent_contexts_on_threads(monkeypatch, shards):
    """mirsha.h: distinct contexts may be used concurrently. Two Python threads
    (ctypes drops the GIL in the call), each with its own context, hash different
    batches at the same time through the host API -- with aliases and mixed sizes,
    pinned and pageable arenas, one and two shards per context -- every digest right."""
    import threading
    from mirbft_amd import Engine
    monkeypatch.setenv("MSHA_VIRTUAL_SHARDS", str(shards))
    wa = W.c5_storm(1 << 16)
    wb = W.c2_requests(1 << 17)
    exp = {"a": _oracle_dedup(wa), "b": oracle.digest_batch(wb.arena, wb.off, wb.len)}
    got, errs = {}, []

    def run(tag, w, pinned):
        try:
            with Engine(1) as e:
                arena = w.arena
                if pinned:
                    arena = e.pinned_empty(w.arena.size)
                    arena[:] = w.arena
                for _ in range(3):
                    got[tag] = e.digest_batch(arena, w.off, w.len)
                    if not np.array_equal(got[tag], exp[tag]):
                        errs.append(tag)
        except Exception as ex:  # surfaced below
            errs.append(repr(ex))

    th = [threading.Thread(target=run, args=("a", wa, True)), threading.Thread(target=run, args=("b", wb, False))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs, errs
    assert set(got) == {"a", "b"}


def test_shared_context_on_threads(engine):
    """mirsha.h: calls on one context are serialised inside the library, so four
    threads may share it: small and pipelined calls of all three host entry points
    interleave on one context, every digest right (before the context mutex, the
    planning buffers of two concurrent calls would have been shared)."""
    import threading
    rng = np.random.default_rng(5)
    wa = W.c5_storm(1 << 15)
    wb = W.c2_requests(3000)
    table = rng.integers(0, 256, size=(256, 32), dtype=np.uint8)
    begin = np.arange(0, 20 * 501, 20, dtype=np.uint64)
    idx = rng.integers(0, 256, int(begin[-1]), dtype=np.uint32)
    actions = [[rng.integers(0, 256, int(k), dtype=np.uint8).tobytes() for k in rng.integers(0, 200, 3)]
               for _ in range(400)]
    exp = {"a": _oracle_dedup(wa), "b": oracle.digest_batch(wb.arena, wb.off, wb.len),
           "d": oracle.digest_of_digests(table, idx, begin),
           "h": [hashlib.sha256(b"".join(p)).digest() for p in actions]}
    calls = {"a": lambda: engine.digest_batch(wa.arena, wa.off, wa.len),      # pipelined (aliases)
             "b": lambda: engine.digest_batch(wb.arena, wb.off, wb.len),      # small
             "d": lambda: engine.digest_of_digests(table, idx, begin),        # small, packed Batches
             "h": lambda: engine.hash_actions(actions)}                       # small, parts
    errs = []

    def run(tag):
        try:
            for _ in range(8):
                g = calls[tag]()
                ok = g == exp[tag] if tag == "h" else np.array_equal(g, exp[tag])
                if not ok:
                    errs.append(tag)
        except Exception as ex:  # surfaced below
            errs.append(repr(ex))

    th = [threading.Thread(target=run, args=(t,)) for t in calls]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs, errs


# ------------------------------------------------------- small-call path --
def test_small_path_pinned_span_aliases_and_edges(engine):
    """The latency path on a pinned, 16-B aligned arena whose span is over 512 KiB
    (metadata H2D + the caller's span as is): aliases, empty messages, a message
    ending at the arena's last byte."""
    rng = np.random.default_rng(7)
    lens = [0, 1, 55, 56, 63, 64, 119, 120, 512, 600_000, 0]
    msgs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    arena, off, ln = _arena_from(msgs)
    arena = arena[:int(off[-2] + ln[-2])]           # the 600,000-B message ends the arena
    off = np.concatenate([off[:-1], off[[3, 3, 8]]]).astype(np.uint64)   # aliases of 56 and 512 B
    ln = np.concatenate([ln[:-1], ln[[3, 3, 8]]]).astype(np.uint64)
    pinned = engine.pinned_empty(arena.size)
    pinned[:] = arena
    st0 = engine.stats()
    got = engine.digest_batch(pinned, off, ln)
    st1 = engine.stats()
    assert st1["small_calls"] == st0["small_calls"] + 1 and st1["direct_calls"] == st0["direct_calls"] + 1
    exp = [hashlib.sha256(arena[int(o):int(o) + int(n)].tobytes()).digest() for o, n in zip(off, ln)]
    assert [g.tobytes() for g in got] == exp
    assert engine.shard_stats()[0]["messages"] == off.size
    # a small pinned span is packed instead (one H2D): not a direct call
    st0 = engine.stats()
    got = engine.digest_batch(pinned, off[:9], ln[:9])
    st1 = engine.stats()
    assert st1["small_calls"] == st0["small_calls"] + 1 and st1["direct_calls"] == st0["direct_calls"]
    assert [g.tobytes() for g in got] == exp[:9]


def test_small_path_digest_of_digests_and_actions(engine):
    """digest-of-digests and hash_actions calls of a few Batches through the latency
    path: zero-part Batches (SHA256("")), repeated indices, odd and even counts."""
    rng = np.random.default_rng(11)
    table = rng.integers(0, 256, size=(64, 32), dtype=np.uint8)
    counts = [0, 1, 2, 3, 20, 21, 0, 40]
    begin = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    idx = rng.integers(0, 64, size=int(begin[-1]), dtype=np.uint32)
    st0 = engine.stats()
    got = engine.digest_of_digests(table, idx, begin)
    assert engine.stats()["small_calls"] == st0["small_calls"] + 1
    assert np.array_equal(got, oracle.digest_of_digests(table, idx, begin))
    actions = [[table[k].tobytes() for k in idx[begin[i]:begin[i + 1]]] for i in range(len(counts))]
    assert engine.hash_actions(actions) == [bytes(g) for g in got]
    assert engine.stats()["small_calls"] == st0["small_calls"] + 2


@pytest.mark.parametrize("zc", ["default", "0"])
def test_small_path_zero_copy(engine, actions_golden, monkeypatch, zc):
    """Calls of a few actions (MirBFT's hash worker at low load, mirbft.go:282-302)
    run zero-copy: one launch of the eight-lane chain reading the packed list in
    coherent pinned memory over PCIe and writing the digests there (no H2D, no
    D2H). Every golden action alone and in small groups, request digests of one to
    100 (under both limits' defaults), an aliased payload, empty messages; the same calls
    with zero-copy off (MSHA_SMALL_ZC_BYTES=0) take the copying small path. Each
    call's digests exact, each call counted by its path and kernel."""
    if zc == "0":
        monkeypatch.setenv("MSHA_SMALL_ZC_BYTES", "0")
    else:
        monkeypatch.delenv("MSHA_SMALL_ZC_BYTES", raising=False)
    monkeypatch.delenv("MSHA_SMALL_BYTES", raising=False)
    calls = [[parts] for _, _, parts, _ in actions_golden]
    exp_calls = [[d] for _, _, _, d in actions_golden]
    calls.append([parts for _, _, parts, _ in actions_golden[:7]])
    exp_calls.append([d for _, _, _, d in actions_golden[:7]])
    w = W.c2_requests(100)
    reqs = [w.arena[int(o):int(o) + int(n)].tobytes() for o, n in zip(w.off, w.len)]
    for k in (1, 2, 16, 17, 64, 100):
        calls.append([[r] for r in reqs[:k]])
        exp_calls.append([hashlib.sha256(r).digest() for r in reqs[:k]])
    calls.append([[reqs[0]], [b""], [reqs[0]], [], [reqs[1][:55]], [reqs[0]]])
    exp_calls.append([hashlib.sha256(b"".join(p)).digest() for p in calls[-1]])
    for c, e in zip(calls, exp_calls):
        st0 = engine.stats()
        assert engine.hash_actions(c) == e
        st1 = engine.stats()
        assert st1["small_calls"] == st0["small_calls"] + 1
        want_zc = int(zc != "0")
        assert st1["small_zc_calls"] - st0["small_zc_calls"] == want_zc, len(c)
        if want_zc:  # the eight-lane chain, nothing copied
            assert st1["launches_chain8"] == st0["launches_chain8"] + 1
            assert st1["h2d_bytes"] == 0 and st1["d2h_bytes"] == 0
    # at and over the limits (MSHA_SMALL_ZC_MSGS; MSHA_SMALL_ZC_BYTES over the packed
    # [off | len | payload], metadata rounded to 64 B): zero-copy, then the copying path
    if zc == "0":
        return
    packed16 = (16 * 16 + 63) // 64 * 64 + 16 * 512
    for env, val, k, fits in (("MSHA_SMALL_ZC_MSGS", "16", 16, True), ("MSHA_SMALL_ZC_MSGS", "16", 17, False),
                              ("MSHA_SMALL_ZC_BYTES", str(packed16), 16, True),
                              ("MSHA_SMALL_ZC_BYTES", str(packed16 - 1), 16, False)):
        monkeypatch.setenv(env, val)
        st0 = engine.stats()
        got = engine.digest_batch(w.arena, w.off[:k], w.len[:k])
        assert np.array_equal(got, oracle.digest_batch(w.arena, w.off[:k], w.len[:k]))
        ran = engine.stats()["small_zc_calls"] - st0["small_zc_calls"]
        assert ran == int(fits), (env, val, k)
        monkeypatch.delenv(env)


def test_small_path_limits(engine, monkeypatch):
    """A call above MSHA_SMALL_MSGS messages or MSHA_SMALL_BYTES of payload takes the
    pipelined path; at the limit it takes the small one."""
    monkeypatch.setenv("MSHA_SMALL_MSGS", "100")
    monkeypatch.setenv("MSHA_SMALL_BYTES", str(100 * 512))
    w = W.c2_requests(101)
    exp = oracle.digest_batch(w.arena, w.off, w.len)
    for n, small in ((100, True), (101, False)):
        st0 = engine.stats()["small_calls"]
        assert np.array_equal(engine.digest_batch(w.arena, w.off[:n], w.len[:n]), exp[:n])
        assert engine.stats()["small_calls"] == st0 + int(small), n
    monkeypatch.setenv("MSHA_SMALL_BYTES", str(100 * 512 - 16))
    st0 = engine.stats()["small_calls"]
    assert np.array_equal(engine.digest_batch(w.arena, w.off[:100], w.len[:100]), exp[:100])
    assert engine.stats()["small_calls"] == st0


@pytest.mark.parametrize("nodes", [24, 100])
def test_epoch_change_storm_packed_once(engine, nodes):
    """An epoch-change storm through the Python mirror (epoch_target.go:486-528:
    every origin's EpochChange hashed once per ack): acks sharing the
    originator's object (the testengine), equal copies (off the wire) and one
    altered copy per origin. Each distinct payload is packed and uploaded once
    (h2d_payload_bytes = the packed span), every digest equals the oracle's.
    24 nodes take the latency path (a pinned span), 100 the direct path."""
    from mirbft_amd.encoding import Checkpoint, SetEntry, epoch_change_hash_data
    rng = np.random.default_rng(nodes)
    hasher = GPUHasher(engine)
    al, want, total = ActionList(), [], 0
    for o in range(nodes):
        ec = EpochChange(new_epoch=9, checkpoints=[Checkpoint(seq_no=500 * (j + 1), value=rng.bytes(332))
                                                   for j in range(2)],
                         p_set=[SetEntry(epoch=8, seq_no=s, digest=rng.bytes(32))
                                for s in range(int(rng.integers(0, 1000)))],
                         q_set=[SetEntry(epoch=7, seq_no=s, digest=rng.bytes(32))
                                for s in range(int(rng.integers(0, 300)))])
        parts = epoch_change_hash_data(ec)
        payload = b"".join(parts)
        for src in range(nodes):
            m = ec
            if src % 3 == 1:   # an equal copy: another object, the same fields
                m = EpochChange(new_epoch=ec.new_epoch, checkpoints=list(ec.checkpoints), p_set=list(ec.p_set),
                                q_set=list(ec.q_set))
            al.hash(parts if m is ec else epoch_change_hash_data(m),
                    HashOrigin(HashOriginEpochChange(source=src, origin=o, epoch_change=m)))
            want.append(hashlib.sha256(payload).digest() if src == 0 else want[-1])
            total += len(payload)
        bad = EpochChange(new_epoch=ec.new_epoch, checkpoints=[Checkpoint(seq_no=500, value=bytes(332)),
                                                               ec.checkpoints[1]],
                          p_set=list(ec.p_set), q_set=list(ec.q_set))
        bad_parts = epoch_change_hash_data(bad)
        al.hash(bad_parts, HashOrigin(HashOriginEpochChange(source=999, origin=o, epoch_change=bad)))
        want.append(hashlib.sha256(b"".join(bad_parts)).digest())
        total += len(payload)
    events = ProcessHashActions(hasher, al)
    assert [e.type.hash_result.digest for e in events] == want
    pk = hasher.last_pack
    assert pk["payloads"] == 2 * nodes and pk["aliased"] == nodes * nodes - nodes
    up = sum(s["h2d_payload_bytes"] for s in engine.shard_stats())
    assert pk["packed_bytes"] - 16 <= up <= pk["packed_bytes"], (up, pk)
    assert up * (nodes // 2) < total      # vs packing every ack
    st = engine.stats()
    assert (st["small_calls"] > 0) if nodes == 24 else (st["direct_calls"] > 0)
    hasher.close()
