#!/usr/bin/env python3
"""c5 per-rank slices on one GPU: where does strong scaling of BASELINE config 5
stop? Times, kernel-resident like bench.py, the slice rank 0 of an N-GPU job
hashes (N = 1, 2, 4, 8) -- in bench.py's c5 forms (FORMS: c5, c5_planned, c5_folded)
-- and, with EC_ONLY=1, the slice's EpochChange actions alone (the long serial
chains: up to ~1,500 blocks per message, the same payloads re-hashed).
One JSON line per measurement on stdout."""
import json
import os
import sys
import types

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mirbft_amd import workloads as W  # noqa: E402


def main():
    import torch
    from mirbft_amd import Engine
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = Engine(1)
    stream = torch.cuda.Stream(dev)
    args = types.SimpleNamespace(warmup=3, steps=int(os.environ.get("TIMED_STEPS", "10")), min_warmup_ms=300,
                                 events="span")
    pool = W.epoch_change_pool()
    for world in [int(x) for x in os.environ.get("WORLDS", "1 2 4 8").split()]:
        per = (1 << 23) // world
        full = W.c5_storm(n=per, first=0, pool=pool)
        ec = full.len > 4096
        subsets = [(form, full) for form in os.environ.get("FORMS", "c5").split()]
        if os.environ.get("EC_ONLY", "0") == "1":
            sub = W.Workload(f"c5 slice 0/{world}: EpochChange actions only", full.arena,
                             np.ascontiguousarray(full.off[ec]), np.ascontiguousarray(full.len[ec]))
            subsets.append(("c5", sub))
        for tag, w in subsets:
            step, d_out = bench.kernel_step(eng, w, tag, dev, stream)
            st0 = eng.stats()
            elapsed, kern_ms, warm, _ = bench.time_steps(step, args, dev, stream)
            eng.device_status()
            kind = bench.kind_of(st0, eng.stats())
            bench.verify_sample(w, d_out)
            lmax = int(w.len.max())
            blocks_max = (lmax >> 6) + (1 if (lmax & 63) < 56 else 2)
            print(json.dumps({"world": world, "form": tag, "workload": w.name, "n": int(w.n),
                              "blocks": int(w.blocks), "hashed_blocks": bench.hashed_blocks(w, tag),
                              "max_blocks": blocks_max, "kernel_ms": kern_ms, "kernel": kind,
                              "g_blocks_per_s": w.blocks / kern_ms / 1e6}), flush=True)
            del step, d_out
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
