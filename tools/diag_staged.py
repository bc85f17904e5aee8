#!/usr/bin/env python3
"""Diagnostic: the staged (pageable) direct path on a c5 storm, as
tests/test_gpu_parity.py::test_staged_direct_pageable runs it, printing which
digests differ from the oracle (count, their lengths in blocks, whether they are
head-length payloads) and the shard figures. One JSON line per call.
    MSHA_VIRTUAL_SHARDS=1 python tools/diag_staged.py [n]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mirbft_amd import Engine  # noqa: E402
from mirbft_amd import workloads as W  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3 << 17
    w = W.c5_storm(n)
    key = np.stack([w.off, w.len], axis=1)
    uniq, inv = np.unique(key, axis=0, return_inverse=True)
    exp = oracle.digest_batch(w.arena, uniq[:, 0].copy(), uniq[:, 1].copy())[inv.reshape(-1)]
    blocks = (w.len.astype(np.int64) + 8) // 64 + 1
    with Engine(1) as e:
        def pinned_copy(a):
            p = e.pinned_empty(a.nbytes).view(a.dtype)
            p[...] = a
            return p
        for rep in range(int(os.environ.get("REPS", "2"))):
            for meta in ("pageable", "pinned"):
                off, ln = (w.off, w.len) if meta == "pageable" else (pinned_copy(w.off), pinned_copy(w.len))
                got = e.digest_batch(w.arena, off, ln)
                bad = np.nonzero(np.any(got != exp, axis=1))[0]
                sh = e.shard_stats()
                print(json.dumps({"rep": rep, "meta": meta, "bad": int(bad.size),
                                  "bad_blocks": sorted(set(int(b) for b in blocks[bad]))[:20],
                                  "bad_first": [int(i) for i in bad[:8]],
                                  "bad_distinct": int(np.unique(inv.reshape(-1)[bad]).size),
                                  "long_msgs": int((blocks >= 256).sum()),
                                  "head_lanes": [s["head_lanes"] for s in sh], "lanes": [s["lanes"] for s in sh]}),
                      flush=True)


if __name__ == "__main__":
    main()
