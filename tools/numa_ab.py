#!/usr/bin/env python3
"""Which buffer makes a striped (mmap + mbind + hipHostRegister) pinned
allocation slower on the direct host path: c5 through msha_digest_batch with
each of arena / off+len / out allocated striped (MSHA_PINNED_STRIPE is read per
msha_pinned_alloc call) or by hipHostMalloc. One JSON line per combination."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402  (torch's HIP runtime first, as bench.py does)
import numpy as np  # noqa: E402
from mirbft_amd import Engine  # noqa: E402
from mirbft_amd import workloads as W  # noqa: E402

w = W.c5_storm(1 << 23)
steps = int(os.environ.get("STEPS", "6"))
with Engine(1) as e:
    def alloc(a, striped):
        os.environ["MSHA_PINNED_STRIPE"] = "1" if striped else "0"
        p = e.pinned_empty(a.nbytes).view(a.dtype).reshape(a.shape)
        p[...] = a
        return p
    bufs = {}
    for striped in (0, 1):
        bufs[striped] = (alloc(w.arena, striped), alloc(w.off, striped), alloc(w.len, striped),
                         alloc(np.zeros((w.n, 32), dtype=np.uint8), striped))
    ref = None
    for combo in ("000", "100", "010", "001", "111", "000"):
        a, m, o = (int(c) for c in combo)
        arena, off, ln, out = bufs[a][0], bufs[m][1], bufs[m][2], bufs[o][3]
        e.digest_batch(arena, off, ln, out=out)
        t0 = time.perf_counter()
        for _ in range(steps):
            e.digest_batch(arena, off, ln, out=out)
        el = (time.perf_counter() - t0) / steps
        if ref is None:
            ref = out.copy()
        assert np.array_equal(out, ref)
        s = e.shard_stats()[0]
        print(json.dumps({"arena_striped": a, "meta_striped": m, "out_striped": o, "ms_per_call": round(el * 1e3, 2),
                          **{k: round(s[k], 2) for k in ("first_launch_ms", "upload_ms", "kernel_ms", "device_ms")}}),
              flush=True)
