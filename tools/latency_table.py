#!/usr/bin/env python3
"""Print tools/latency.cpp's JSON lines as a table: api, arena, n, p50/p99 us, digests/s."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        d = json.loads(line)
        print(f"{d['api']:24s} {d['arena']:8s} {d['n']:6d} {d['p50_us']:8.1f} {d['p99_us']:8.1f} "
              f"{d['digests_per_s_at_p50'] / 1e6:8.2f} M/s")
