#!/usr/bin/env python3
"""Per-kernel duration summary from a rocprofv3 SQLite database (run_results.db):
name, calls, mean / min / max microseconds; plus the last call's kernels in time order."""
import sqlite3
import sys


def main(db, last=40):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, start, end, stream_id, queue_id from kernels order by start").fetchall()
    stats = {}
    for n, s, e, *_ in rows:
        stats.setdefault(n, []).append((e - s) / 1e3)
    print(f"{'kernel':70s} {'calls':>6s} {'mean_us':>10s} {'min_us':>10s} {'max_us':>10s}")
    for n, v in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
        print(f"{n[:70]:70s} {len(v):6d} {sum(v)/len(v):10.1f} {min(v):10.1f} {max(v):10.1f}")
    if last <= 0:
        return
    t0 = rows[-last][1] if len(rows) >= last else rows[0][1]
    print("\nlast kernels (start_us end_us stream queue name):")
    for n, s, e, st, q in rows[-last:]:
        print(f"{(s - t0)/1e3:10.1f} {(e - t0)/1e3:10.1f} {st:4d} {q:4d} {n[:60]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
