#!/usr/bin/env python3
"""A/B: host-call digest D2H on its own stream (MSHA_D2H_STREAM=1, default) or
on the kernel stream (=0), alternating call by call in one process, c5 and c2
through msha_digest_batch from pinned memory. One JSON line per setting."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
import numpy as np  # noqa: E402
from mirbft_amd import Engine  # noqa: E402
from mirbft_amd import workloads as W  # noqa: E402

reps = int(os.environ.get("REPS", "8"))
for name, w in (("c5", W.c5_storm(1 << 23)), ("c2", W.c2_requests())):
    with Engine(1) as e:
        def pin(a):
            p = e.pinned_empty(a.nbytes).view(a.dtype).reshape(a.shape)
            p[...] = a
            return p
        arena, off, ln = pin(w.arena), pin(w.off), pin(w.len)
        out = e.pinned_empty(w.n * 32).reshape(w.n, 32)
        times = {"0": [], "1": []}
        ref = None
        for r in range(reps + 1):
            for mode in ("1", "0") if r % 2 else ("0", "1"):
                os.environ["MSHA_D2H_STREAM"] = mode
                t = time.perf_counter()
                e.digest_batch(arena, off, ln, out=out)
                dt = (time.perf_counter() - t) * 1e3
                if ref is None:
                    ref = out.copy()
                assert np.array_equal(out, ref)
                if r:
                    times[mode].append(round(dt, 2))
        for mode, t in times.items():
            print(json.dumps({"config": name, "d2h_stream": int(mode), "median_ms": float(np.median(t)),
                              "min_ms": min(t), "calls_ms": t}), flush=True)
