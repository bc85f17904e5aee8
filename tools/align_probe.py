#!/usr/bin/env python3
"""Round 5 probe: does the folded c5 lane kernel's HBM traffic (~1.5x its
algorithmic bytes, profiles/r05_pmc.json) come from the arena's 16-byte packing?
Times msha_digest_batch_device_planned(FOLD) on c5's 8.4 M actions as packed
(16-byte aligned, what the drop-in packs) and re-packed with every owned payload
128-byte aligned (same messages, same digests). One JSON line per layout; run under
rocprofv3 --pmc for traffic."""
import json
import os
import sys
import types

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mirbft_amd import workloads as W  # noqa: E402


def repack(w, align):
    own = ~w.shared
    sz = np.where(own, (w.len + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align), np.uint64(0))
    pool_end = int(w.off[w.shared].max() + w.len[w.shared].max()) if w.shared.any() else 0
    base = (pool_end + align - 1) // align * align
    new_off = np.zeros(w.n, np.uint64)
    new_off[1:] = np.cumsum(sz)[:-1]
    new_off = new_off + np.uint64(base)
    arena = np.zeros(base + int(sz.sum()) + 64, np.uint8)
    arena[:pool_end] = w.arena[:pool_end]
    idx = np.flatnonzero(own)
    for i0 in range(0, idx.size, 1 << 16):  # vectorised byte copy, 65,536 messages at a time
        ii = idx[i0:i0 + (1 << 16)]
        ln = w.len[ii].astype(np.int64)
        tot = int(ln.sum())
        within = np.arange(tot, dtype=np.int64) - np.repeat(np.cumsum(ln) - ln, ln)
        arena[np.repeat(new_off[ii].astype(np.int64), ln) + within] = \
            w.arena[np.repeat(w.off[ii].astype(np.int64), ln) + within]
    off = np.where(own, new_off, w.off)
    return W.Workload(f"{w.name} (owned payloads {align}-B aligned)", arena, off, w.len.copy(), shared=w.shared)


def main():
    import torch
    from mirbft_amd import Engine
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = Engine(1)
    stream = torch.cuda.Stream(dev)
    args = types.SimpleNamespace(warmup=3, steps=int(os.environ.get("TIMED_STEPS", "20")), min_warmup_ms=300,
                                 events="span")
    w16 = W.c5_storm(n=1 << int(os.environ.get("LOG_N", "23")))
    layouts = [int(x) for x in os.environ.get("LAYOUTS", "16 128").split()]
    for w in [w16 if a == 16 else repack(w16, a) for a in layouts]:
        step, d_out = bench.kernel_step(eng, w, "c5_folded", dev, stream)
        elapsed, kern_ms, warm, _ = bench.time_steps(step, args, dev, stream)
        eng.device_status()
        bench.verify_sample(w, d_out)
        clk = bench.clock_reading(eng)
        print(json.dumps({"layout": w.name, "arena_bytes": int(w.arena.size), "kernel_ms": kern_ms,
                          "clock_after": clk.get("effective_clock_ghz")}), flush=True)
        del step, d_out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
