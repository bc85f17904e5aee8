"""GPU parity and timing of the host path's long-chain heads (msha_digest_batch on
a pinned arena, what the Go adapter calls): payloads of >= 256 blocks are
uploaded first, whatever their place in the caller's arena, and run as heads on
the two-lane chain kernel with CUs of their own, so a long EpochChange payload
the caller packed last (gpuhash.go packs in action order) no longer ends the
call as a lone chain on the lane kernel. Checked bit-exact against the oracle;
the per-shard figures say that the heads ran (head_lanes) and how far each
shard's last kernel ends after its last upload. Writes the measured tails to
gpurun_out/host_head_tails.jsonl (the A/B with MSHA_HOST_HEAD=0)."""
import json
import os

import numpy as np
import pytest

from mirbft_amd import workloads as W
from oracle import oracle

pytestmark = pytest.mark.gpu

N_REQ = 1 << 20
N_LONG = 64
LONG_LEN = 1400 * 64 - 20          # 1,400 blocks
PER_LONG = 40                      # actions naming each long payload (the N^2 re-hash)


def _layout():
    """2^20 requests of 512 B packed first, the 64 long payloads packed LAST
    (the last upload piece); their 2,560 actions scattered over the batch, so
    every shard of a sharded call names some of them."""
    rng = np.random.default_rng(1400)
    req_off = np.arange(N_REQ, dtype=np.uint64) * np.uint64(512)
    long_base = N_REQ * 512
    long_off = np.uint64(long_base) + np.arange(N_LONG, dtype=np.uint64) * np.uint64((LONG_LEN + 15) // 16 * 16)
    size = int(long_off[-1]) + LONG_LEN
    n = N_REQ + N_LONG * PER_LONG
    off = np.empty(n, np.uint64)
    ln = np.empty(n, np.uint64)
    is_long = np.zeros(n, bool)
    is_long[rng.choice(n, N_LONG * PER_LONG, replace=False)] = True
    off[~is_long], ln[~is_long] = req_off, 512
    pick = np.repeat(np.arange(N_LONG), PER_LONG)
    rng.shuffle(pick)
    off[is_long], ln[is_long] = long_off[pick], LONG_LEN
    arena = W.random_bytes(W.SEED ^ 0x1400, 0, size + 64)
    return arena, off, ln


@pytest.fixture(scope="module")
def layout():
    arena, off, ln = _layout()
    key = np.stack([off, ln], axis=1)
    _, first, inv = np.unique(key, axis=0, return_index=True, return_inverse=True)
    exp = oracle.openssl_digest_batch(arena, off[first], ln[first], 16)[inv.reshape(-1)]
    return arena, off, ln, exp


def _run(layout, shards, head, monkeypatch):
    from mirbft_amd import Engine
    arena, off, ln, exp = layout
    monkeypatch.setenv("MSHA_VIRTUAL_SHARDS", str(shards))
    monkeypatch.setenv("MSHA_HOST_HEAD", "1" if head else "0")
    eng = Engine(1)
    try:
        def pinned(a):
            p = eng.pinned_empty(a.nbytes).view(a.dtype).reshape(a.shape)
            p[...] = a
            return p
        pa, po, pl = pinned(arena), pinned(off), pinned(ln)
        out = eng.pinned_empty(32 * off.size).reshape(-1, 32)
        st0 = eng.stats()
        tails = []
        for _ in range(3):   # the first call allocates; keep the last's figures
            eng.digest_batch(pa, po, pl, out=out)
            assert np.array_equal(out, exp)
            sh = eng.shard_stats()
            tails = [s["device_ms"] - s["upload_ms"] for s in sh]
        return eng.stats(), st0, sh, tails
    finally:
        eng.close()


@pytest.mark.parametrize("shards", [1, 8])
def test_long_chains_packed_last_run_as_heads(layout, shards, monkeypatch):
    """One GPU: every digest exact, the 64 long payloads hashed once each as
    heads, and the call's last kernel ends within 1 ms of its last upload (the
    A/B without heads is recorded). 8 virtual shards of one GPU: every shard
    folds its aliases (each names the long payloads from a region of the arena
    far from its own requests) and runs them as heads; their tails are recorded,
    not asserted: 8 shards share one GPU's CUs and one PCIe link, so a shard's
    kernels also wait for the other shards' (DESIGN.md (d))."""
    st, st0, sh, tails = _run(layout, shards, True, monkeypatch)
    assert st["direct_calls"] - st0["direct_calls"] == 3
    assert all(0 < s["head_lanes"] <= N_LONG for s in sh), [s["head_lanes"] for s in sh]
    assert st["launches_coop"] - st0["launches_coop"] >= 3 * shards
    _, _, sh_off, tails_off = _run(layout, shards, False, monkeypatch)
    assert all(s["head_lanes"] == 0 for s in sh_off)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/host_head_tails.jsonl", "a") as f:
        f.write(json.dumps({"shards": shards, "tail_ms_heads": tails, "tail_ms_no_heads": tails_off,
                            "upload_ms": [s["upload_ms"] for s in sh], "device_ms": [s["device_ms"] for s in sh],
                            "upload_ms_no_heads": [s["upload_ms"] for s in sh_off],
                            "device_ms_no_heads": [s["device_ms"] for s in sh_off],
                            "head_lanes": [s["head_lanes"] for s in sh]}) + "\n")
    # the long chains no longer end the call: its last kernel ends within 1 ms
    # of its last upload (without heads: a 1,400-block chain on the lane kernel
    # after the last piece, ~2 ms more)
    if shards == 1:
        assert max(tails) <= 1.0, (tails, tails_off)


def test_lane_policy_runs_no_heads(layout):
    """A context held to the lane kernel (MSHA_KERNEL_LANE) runs its long payloads as
    ordinary lanes, as the device-planned path does: no head lanes, no cooperative or
    two-lane launch, every digest exact."""
    from mirbft_amd import Engine
    arena, off, ln, exp = layout
    eng = Engine(1)
    try:
        eng.set_kernel_policy("lane")
        def pinned(a):
            p = eng.pinned_empty(a.nbytes).view(a.dtype).reshape(a.shape)
            p[...] = a
            return p
        out = eng.pinned_empty(32 * off.size).reshape(-1, 32)
        st0 = eng.stats()
        eng.digest_batch(pinned(arena), pinned(off), pinned(ln), out=out)
        assert np.array_equal(out, exp)
        st = eng.stats()
        assert all(s["head_lanes"] == 0 for s in eng.shard_stats())
        assert st["launches_coop"] == st0["launches_coop"]
    finally:
        eng.close()
