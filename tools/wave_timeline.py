#!/usr/bin/env python3
"""Summarise tools/wave_timeline records: where a lane-kernel launch spends
its time beyond the steady compression rate.

    python3 tools/wave_timeline.py gpurun_out/timeline/*.bin

Per file (one launch): span (first wave start .. last wave end), how late the
waves start (ramp), how early SIMDs fall idle before the end (drain), waves per
SIMD and how many run concurrently, in microseconds (s_memrealtime: 100 MHz).
"""
import json
import sys

import numpy as np

TICK_US = 0.01


def decode(rec):
    hw = rec[:, 2].astype(np.int64)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    xcc = rec[:, 3].astype(np.int64) & 15
    return ((xcc * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd


def summarise(path):
    rec = np.fromfile(path, dtype=np.uint64).reshape(-1, 4)
    t0 = rec[:, 0].astype(np.int64)
    t1 = rec[:, 1].astype(np.int64)
    base = t0.min()
    s = (t0 - base) * TICK_US
    e = (t1 - base) * TICK_US
    span = e.max()
    key = decode(rec)
    simds, inv = np.unique(key, return_inverse=True)
    n_simd = simds.size
    per = np.bincount(inv)
    last_end = np.full(n_simd, -1.0)
    first_start = np.full(n_simd, np.inf)
    busy = np.zeros(n_simd)
    np.maximum.at(last_end, inv, e)
    np.minimum.at(first_start, inv, s)
    # time a SIMD has >= 1 wave resident: union of its waves' intervals
    order = np.lexsort((s, inv))
    cur_simd, cur_a, cur_b = -1, 0.0, 0.0
    for j in order:
        g = inv[j]
        if g != cur_simd:
            if cur_simd >= 0:
                busy[cur_simd] += cur_b - cur_a
            cur_simd, cur_a, cur_b = g, s[j], e[j]
        elif s[j] > cur_b:
            busy[g] += cur_b - cur_a
            cur_a, cur_b = s[j], e[j]
        else:
            cur_b = max(cur_b, e[j])
    if cur_simd >= 0:
        busy[cur_simd] += cur_b - cur_a
    # concurrency: active waves per SIMD sampled over the span
    grid = np.linspace(0, span, 200)
    active = ((s[None, :] <= grid[:, None]) & (e[None, :] > grid[:, None])).sum(1) / n_simd
    dur = e - s
    return {
        "file": path, "waves": int(rec.shape[0]), "simds_seen": int(n_simd),
        "waves_per_simd": {"min": int(per.min()), "max": int(per.max()), "mean": float(per.mean())},
        "span_us": float(span),
        "start_us": {"p50": float(np.percentile(s, 50)), "p99": float(np.percentile(s, 99)), "max": float(s.max())},
        "end_us": {"min": float(e.min()), "p10": float(np.percentile(e, 10)), "p50": float(np.percentile(e, 50)),
                   "p90": float(np.percentile(e, 90)), "max": float(e.max())},
        "wave_us": {"min": float(dur.min()), "p50": float(np.percentile(dur, 50)), "max": float(dur.max())},
        "simd_idle_before_end_us": {"mean": float((span - last_end).mean()),
                                    "p90": float(np.percentile(span - last_end, 90))},
        "simd_idle_at_start_us": {"mean": float(first_start.mean()), "max": float(first_start.max())},
        "simd_busy_frac": float(busy.sum() / (n_simd * span)),
        "active_waves_per_simd_over_time": [round(float(x), 2) for x in active[::10]],
    }


if __name__ == "__main__":
    out = [summarise(p) for p in sys.argv[1:]]
    print(json.dumps(out, indent=1))
