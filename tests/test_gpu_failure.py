"""Failure paths of split chaining (kernels.hip k_digest_split) on the GPU.

MSHA_SPLIT_STALL=1 (test-only, read per launch) makes chain 0's first segment
skip its handoff, so the segments waiting on it hit the 100 ms timeout: they set
error bit 2 and release the chain, so the kernel still drains (no hang). What
must then happen (reference contract: a wrong digest is a safety bug,
batch_tracker.go:192-195; errors surface through doHashWork, mirbft.go:290-293):
  * device entry points: msha_device_status() returns MSHA_ERR_HIP;
  * host entry points: the shard is re-hashed unsplit in the same call, every
    digest is correct, and msha_stats.split_retries counts it.
"""
import os
import time

import numpy as np
import pytest

from mirbft_amd import MshaError
from mirbft_amd import _lib as L
from mirbft_amd import workloads as W
from oracle import oracle

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(os.environ.get("MSHA_SPLIT") == "0",
                                 reason="split chaining disabled (MSHA_SPLIT=0 A/B run): nothing to stall")]


def _cus():
    import torch
    return torch.cuda.get_device_properties(0).multi_processor_count


def _split_workload():
    """One full round of waves plus one surplus wave of 640-B messages: a split
    launch with one chain of 8 segments (plan_split)."""
    n = _cus() * 4 * 64 + 64
    return W.uniform_requests(n, 640, W.SEED ^ 0xF1, name="split-stall")


def test_split_stall_device_api_reports_hip_error(engine, monkeypatch):
    import torch
    w = _split_workload()
    dev = torch.device("cuda:0")
    d_arena = torch.from_numpy(w.arena).to(dev)
    d_off = torch.from_numpy(w.off.view(np.int64)).to(dev)
    d_len = torch.from_numpy(w.len.view(np.int64)).to(dev)
    out = torch.empty((w.n, 32), dtype=torch.uint8, device=dev)
    monkeypatch.setenv("MSHA_SPLIT_STALL", "1")
    before = engine.stats()["launches_split"]
    t0 = time.perf_counter()
    engine.digest_batch_device(d_arena, d_off, d_len, out)
    with pytest.raises(MshaError) as ei:
        engine.device_status()
    elapsed = time.perf_counter() - t0
    assert ei.value.code == L.MSHA_ERR_HIP
    assert "split-chain" in str(ei.value)
    assert engine.stats()["launches_split"] == before + 1
    assert elapsed < 10.0, elapsed          # the 100 ms release drained the kernel
    # the main (unsplit) lanes are still right; the flag is cleared afterwards
    exp = oracle.digest_batch(w.arena, w.off, w.len)
    got = out.cpu().numpy()
    main = _cus() * 4 * 64
    assert np.array_equal(got[:main], exp[:main])
    monkeypatch.delenv("MSHA_SPLIT_STALL")
    engine.digest_batch_device(d_arena, d_off, d_len, out)
    engine.device_status()
    assert np.array_equal(out.cpu().numpy(), exp)


@pytest.mark.parametrize("pinned", [False, True])
def test_split_stall_host_api_reruns_unsplit(engine, monkeypatch, pinned):
    w = _split_workload()
    exp = oracle.digest_batch(w.arena, w.off, w.len)
    arena = w.arena
    if pinned:
        arena = engine.pinned_empty(w.arena.size)
        arena[:] = w.arena
    monkeypatch.setenv("MSHA_SPLIT_STALL", "1")
    monkeypatch.setenv("MSHA_SMALL_BYTES", "0")      # the pipelined path (the one that splits)
    st0 = engine.stats()
    t0 = time.perf_counter()
    got = engine.digest_batch(arena, w.off, w.len)
    assert time.perf_counter() - t0 < 10.0
    st1 = engine.stats()
    assert np.array_equal(got, exp)
    assert st1["split_retries"] == st0["split_retries"] + 1
    assert st1["launches_split"] == st0["launches_split"] + 1
    assert st1["direct_calls"] == st0["direct_calls"] + int(pinned)


def test_split_stall_digest_of_digests_host_reruns(engine, monkeypatch):
    n = _cus() * 4 * 64 + 64
    rng = np.random.default_rng(77)
    table = rng.integers(0, 256, (4096, 32), dtype=np.uint8)
    begin = np.arange(n + 1, dtype=np.uint64) * np.uint64(20)
    idx = rng.integers(0, 4096, int(begin[-1]), dtype=np.uint32)
    exp = oracle.digest_of_digests(table, idx, begin)
    monkeypatch.setenv("MSHA_SPLIT_STALL", "1")
    monkeypatch.setenv("MSHA_SMALL_BYTES", "0")
    st0 = engine.stats()
    assert np.array_equal(engine.digest_of_digests(table, idx, begin), exp)
    st1 = engine.stats()
    assert st1["split_retries"] == st0["split_retries"] + 1
    assert st1["launches_split"] == st0["launches_split"] + 1
    assert st1["launches_dod"] == st0["launches_dod"] + 1      # the unsplit re-run
