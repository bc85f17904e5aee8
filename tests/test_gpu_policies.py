"""Both batch kernels, forced: one lane per message (MSHA_KERNEL_LANE) and
cooperative chaining (MSHA_KERNEL_COOP: producer wave expands the schedule
into LDS, consumer wave runs the rounds). Bit-exact vs the oracle and the
golden fixtures under each policy; AUTO is covered by test_gpu_parity.py,
plus the pipelined lane kernels' edge cases at the end of this file.
"""
import hashlib

import numpy as np
import pytest

from mirbft_amd import _lib as L
from mirbft_amd import MshaError
from mirbft_amd import workloads as W
from oracle import oracle

pytestmark = pytest.mark.gpu

POLICIES = ["lane", "coop"]


@pytest.fixture(params=POLICIES)
def eng(request, engine):
    engine.set_kernel_policy(request.param)
    engine._policy = request.param
    yield engine
    engine.set_kernel_policy("auto")
    engine._policy = "auto"


def _dev(a, dtype=None):
    import torch
    t = torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a)
    return t.to("cuda:0")


def test_lengths_golden(eng, lengths_golden):
    msgs = [m for m, _ in lengths_golden]
    got = eng.hash_actions([[m] for m in msgs])
    assert got == [d for _, d in lengths_golden]


def test_each_length_alone(eng, lengths_golden):
    for m, d in lengths_golden[:130:3]:
        assert eng.hash_actions([[m]])[0] == d, len(m)


def test_actions_golden(eng, actions_golden):
    got = eng.hash_actions([parts for _, _, parts, _ in actions_golden])
    assert got == [d for _, _, _, d in actions_golden]


@pytest.mark.parametrize("seed", [4, 5])
def test_random_multipart(eng, seed):
    rng = np.random.default_rng(seed)
    actions = [[rng.integers(0, 256, int(rng.integers(0, 2000)), dtype=np.uint8).tobytes()
                for _ in range(int(rng.integers(0, 5)))] for _ in range(2500)]
    assert eng.hash_actions(actions) == oracle.process_hash_actions(actions)


def test_device_unordered_mixed_blocks(eng):
    """Device path, no order: every 64-message group mixes block counts 1..40
    (coop: the group runs to its longest message, shorter ones store early)."""
    import torch
    rng = np.random.default_rng(21)
    n = 5000
    lens = rng.integers(0, 2500, n).astype(np.uint64)
    stride = (lens + 15) // 16 * 16
    off = np.concatenate([[0], np.cumsum(stride)[:-1]]).astype(np.uint64)
    arena = W.random_bytes(W.SEED ^ 0x72, 0, int(stride.sum()) + 64)
    out = torch.empty((n, 32), dtype=torch.uint8, device="cuda:0")
    st0 = eng.stats()
    eng.digest_batch_device(_dev(arena), _dev(off), _dev(lens), out)
    eng.device_status()
    assert np.array_equal(out.cpu().numpy(), oracle.digest_batch(arena, off, lens))
    _assert_policy_kernel(eng, st0)


def _assert_policy_kernel(eng, st0):
    """The forced policy's kernel is the one that ran (msha_stats launch counters)."""
    st1 = eng.stats()
    ran = {k: st1[k] - st0[k] for k in ("launches_lane", "launches_pipe", "launches_coop", "launches_split")}
    if eng._policy == "coop":
        assert ran == {"launches_lane": 0, "launches_pipe": 0, "launches_coop": 1, "launches_split": 0}, ran
    else:   # one lane per message: the plain or the pipelined lane kernel
        assert ran["launches_coop"] == 0 and ran["launches_lane"] + ran["launches_pipe"] + ran["launches_split"] == 1, ran


@pytest.mark.parametrize("n", [1 << 14, 40_000])   # coop: latency form (G=2) / balanced form (G=4)
def test_device_ordered_c5(eng, n):
    import torch
    from mirbft_amd.engine import order_by_blocks
    w = W.c5_storm(n)
    out = torch.empty((w.n, 32), dtype=torch.uint8, device="cuda:0")
    order = _dev(order_by_blocks(w.len).view(np.int32))
    st0 = eng.stats()
    eng.digest_batch_device(_dev(w.arena), _dev(w.off), _dev(w.len), out, order=order)
    eng.device_status()
    assert np.array_equal(out.cpu().numpy(), oracle.digest_batch(w.arena, w.off, w.len))
    _assert_policy_kernel(eng, st0)


def test_partial_last_group(eng):
    """n not a multiple of 64 (coop: idle lanes in the last workgroup)."""
    for n in (1, 63, 65, 130):
        msgs = [bytes([i % 251]) * (i * 37 % 700) for i in range(n)]
        assert eng.hash_actions([[m] for m in msgs]) == [hashlib.sha256(m).digest() for m in msgs]


def test_misaligned_flagged(eng):
    import torch
    arena = torch.zeros(4096, dtype=torch.uint8, device="cuda:0")
    off = torch.tensor([0, 8, 32], dtype=torch.int64, device="cuda:0")
    ln = torch.tensor([10, 10, 100], dtype=torch.int64, device="cuda:0")
    out = torch.full((3, 32), 0xAB, dtype=torch.uint8, device="cuda:0")
    eng.digest_batch_device(arena, off, ln, out)
    with pytest.raises(MshaError) as ei:
        eng.device_status()
    assert ei.value.code == L.MSHA_ERR_ALIGNMENT
    o = out.cpu().numpy()
    assert o[0].tobytes() == hashlib.sha256(b"\0" * 10).digest()
    assert not o[1].any()
    assert o[2].tobytes() == hashlib.sha256(b"\0" * 100).digest()
    eng.device_status()


def test_large_messages(eng):
    """Few long messages (the cooperative regime): 8 x 1 MiB + ragged tails."""
    msgs = [W.random_bytes(W.SEED ^ 0x73, i << 24, (1 << 20) + 13 * i).tobytes() for i in range(8)]
    assert eng.hash_actions([[m] for m in msgs]) == [hashlib.sha256(m).digest() for m in msgs]


def _device_digests(engine, lens, salt, kernel="launches_pipe"):
    import torch
    lens = np.asarray(lens, dtype=np.uint64)
    stride = (lens + 15) // 16 * 16
    off = np.concatenate([[0], np.cumsum(stride)[:-1]]).astype(np.uint64)
    arena = W.random_bytes(W.SEED ^ salt, 0, int(stride.sum()) + 64)
    out = torch.empty((len(lens), 32), dtype=torch.uint8, device="cuda:0")
    before = engine.stats()[kernel]
    engine.digest_batch_device(_dev(arena), _dev(off), _dev(lens), out)
    engine.device_status()
    assert engine.stats()[kernel] == before + 1, f"{kernel} did not run"
    return out.cpu().numpy(), oracle.digest_batch(arena, off, lens)


# The pipelined lane kernel (auto policy, n in (CUs*128, CUs*256]: one wave per
# SIMD) exits its ping-pong loop after an odd or an even number of full blocks,
# and hands wave-uniform padding-only final blocks to the SALU schedule.
@pytest.mark.parametrize("size", [0, 55, 56, 63, 64, 119, 128, 183, 192, 200, 256, 1000])
def test_pipe_uniform_lengths(engine, size):
    got, want = _device_digests(engine, [size] * 40_000, 0x90 + size)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("size,stride", [(0, 16), (56, 64), (128, 128), (183, 192), (1000, 1024)])
def test_pipe_uniform_kernel(engine, size, stride):
    """k_digest_uniform_pipe (uniform layout, n in the one-wave-per-SIMD range)."""
    import torch
    n = 40_000
    arena = W.random_bytes(W.SEED ^ 0x92, 8 * size, n * stride + 64)
    out = torch.empty((n, 32), dtype=torch.uint8, device="cuda:0")
    before = engine.stats()["launches_pipe"]
    engine.digest_uniform_device(_dev(arena), stride, size, n, out)
    engine.device_status()
    assert engine.stats()["launches_pipe"] == before + 1      # the uniform pipelined kernel ran
    off = (np.arange(n, dtype=np.uint64) * stride).astype(np.uint64)
    want = oracle.digest_batch(arena, off, np.full(n, size, dtype=np.uint64))
    assert np.array_equal(out.cpu().numpy(), want)


def test_pipe_ragged_lengths(engine):
    rng = np.random.default_rng(31)
    lens = rng.integers(0, 1500, 50_000)
    lens[::7] = rng.integers(0, 5, len(lens[::7])) * 64   # exact block multiples
    lens[3::7] = rng.integers(0, 5, len(lens[3::7])) * 64 + 56
    got, want = _device_digests(engine, lens, 0x91)
    assert np.array_equal(got, want)


def test_unknown_policy_rejected(engine):
    rc = engine._lib.msha_set_kernel_policy(engine._ctx, 7)
    assert rc == L.MSHA_ERR_INVALID_ARG
