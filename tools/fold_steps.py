#!/usr/bin/env python3
"""Per-step kernel times of planned device calls (folded or not) in a rocprofv3
database (tools/c5_slice.py under rocprofv3 --kernel-trace): a step starts at the
planner's first kernel (k_fold_tilemax, or k_fold_keys unfolded) and ends at the
last kernel that ends before the next step starts. Steps are grouped by their lane
kernel's length (one group per slice size); for each kernel of a group the mean
start (from the step's start), the mean duration and its range are printed, with
the step's span."""
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = [(n.split("(")[0].replace("void ", "").replace("msha::", ""), s, e)
            for n, s, e in c.execute(f"select {name}, start, end from kernels order by start")]
    steps, cur = [], None
    for n, s, e in rows:
        if n.startswith("k_fold_tilemax") or n.startswith("k_fold_keys"):
            cur = {"t0": s, "t1": s, "k": {}, "form": "folded" if n.startswith("k_fold_tilemax") else "unfolded"}
            steps.append(cur)
        if cur is None:
            continue
        cur["k"].setdefault(n, []).append((s, e))
        cur["t1"] = max(cur["t1"], e)
    groups = {}
    for st in steps:
        lane = st["k"].get("k_digest_batch<2>")
        if not lane:
            continue
        key = (st["form"], round(max(e - s for s, e in lane) / 1e5))  # 0.1 ms classes
        groups.setdefault(key, []).append(st)
    for key, sts in sorted(groups.items(), reverse=True):
        print(f"{key[0]}, lane kernel ~{key[1] / 10:.1f} ms: {len(sts)} steps, span mean "
              f"{sum(st['t1'] - st['t0'] for st in sts) / len(sts) / 1e3:.1f} us (planner start .. last end)")
        names = sorted({n for st in sts for n in st["k"]},
                       key=lambda n: sum(min(s for s, _ in st["k"][n]) - st["t0"] for st in sts if n in st["k"]))
        for n in names:
            d = [sum(e - s for s, e in st["k"][n]) / 1e3 for st in sts if n in st["k"]]
            t = [(min(s for s, _ in st["k"][n]) - st["t0"]) / 1e3 for st in sts if n in st["k"]]
            print(f"   {n:28s} start {sum(t) / len(t):8.1f} us  dur {sum(d) / len(d):9.1f} us"
                  f"  (min {min(d):8.1f}, max {max(d):8.1f})")


if __name__ == "__main__":
    main(sys.argv[1])
