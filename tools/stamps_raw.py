#!/usr/bin/env python3
"""Deeper look at one raw wave-stamp dump (tools/lane_stamps.py RAW_DIR=...):
per time slice of the lane kernel, how many SIMDs hold 0 / 1 / 2-3 / 4-7 / 8 lane
waves; the head kernels' long-running waves (which CUs, how long) and the lane
waves on those CUs; and the lane waves' block counts over time.

    python3 tools/stamps_raw.py gpurun_out/.../raw/stamps_c5_folded.npz [slices]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lane_stamps import KINDS, decode  # noqa: E402


def main(path, slices=20):
    d = decode(np.load(path)["recs"])
    lane = d["kind"] == 1
    r0, r1, simd, nb = d["r0"][lane], d["r1"][lane], d["simd"][lane], d["nb"][lane]
    lo, hi = int(r0.min()), int(r1.max())
    edges = np.linspace(lo, hi, slices + 1)
    simds = np.unique(d["simd"])
    print("lane kernel: %d waves, span %.1f us; SIMDs by resident lane waves (time-averaged) per slice" %
          (lane.sum(), (hi - lo) / 100))
    print("slice   t_us   0      1     2-3    4-7     8   | mean nb of waves starting")
    sidx = {s: k for k, s in enumerate(simds)}
    si = np.array([sidx[s] for s in simd])
    for b in range(slices):
        a, z = edges[b], edges[b + 1]
        ov = np.clip(np.minimum(r1, z) - np.maximum(r0, a), 0, None) / (z - a)
        occ = np.bincount(si, weights=ov, minlength=len(simds))
        # SIMDs never touched by the lane kernel count as 0
        h = [np.sum(occ < 0.5), np.sum((occ >= 0.5) & (occ < 1.5)), np.sum((occ >= 1.5) & (occ < 3.5)),
             np.sum((occ >= 3.5) & (occ < 7.5)), np.sum(occ >= 7.5)]
        h[0] += 1024 - len(simds)
        st = (r0 >= a) & (r0 < z)
        print("%4d %8.1f %5d %5d %5d %6d %6d   | %.2f (%d waves)" % (b, (a - lo) / 100, *h,
                                                                   nb[st].mean() if st.any() else 0, st.sum()))
    for k in sorted(set(d["kind"].tolist()) - {1}):
        m = d["kind"] == k
        dur = (d["r1"][m] - d["r0"][m]) / 100
        longw = dur > 100
        cus = np.unique(d["cu"][m][longw])
        print("%s: %d waves, %d longer than 100 us on %d CUs (%s us)" %
              (KINDS.get(k, k), m.sum(), longw.sum(), cus.size,
               ", ".join("%.0f" % x for x in sorted(dur[longw])[-6:])))
        if cus.size:
            on = np.isin(d["cu"][lane], cus)
            tot = (r1[on] - r0[on]).sum() / max(1, hi - lo) / (4 * cus.size)
            print("   lane waves per SIMD on those CUs over the lane span: %.2f (all CUs: %.2f)" %
                  (tot, (r1 - r0).sum() / (hi - lo) / 1024))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
