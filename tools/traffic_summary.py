#!/usr/bin/env python3
"""Summarise tools/pmc_traffic.sh output into profiles/<round>_traffic.json.

traffic_bytes_per_launch = FETCH_SIZE x calib_factor + WRITE_SIZE (both KB x 1024),
averaged over the timed launches of our kernel; calib_factor = known bytes read
by tools/traffic_calib / its FETCH_SIZE (the gfx950 half-count correction,
measured on the engine's own access pattern). bench.py copies the matching
entry into its JSON line as roofline.traffic.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SRC = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/traffic"
DST = sys.argv[2] if len(sys.argv) > 2 else "profiles/r01_traffic.json"


def per_dispatch(name, counter, kernel_substr):
    f = os.path.join(SRC, name, "run_counter_collection.csv")
    vals = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if kernel_substr in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    calib_read = 1 << 29          # tools/traffic_calib: 2^20 lanes x 512 B
    calib_write = (1 << 20) * 4
    cf = per_dispatch("calib_fetch", "FETCH_SIZE", "k_read_like_c2")
    cw = per_dispatch("calib_write", "WRITE_SIZE", "k_read_like_c2")
    factor = calib_read / (1024.0 * (sum(cf[1:]) / len(cf[1:])))
    out = {"method": "rocprofv3 --kernel-trace --pmc, FETCH_SIZE and WRITE_SIZE in separate passes; "
                     "FETCH_SIZE x calib_factor (tools/traffic_calib.hip, same per-lane pattern)",
           "calib": {"bytes_read": calib_read, "fetch_size_kb": cf, "calib_factor": factor,
                     "bytes_written": calib_write, "write_size_kb": cw},
           "configs": {}}
    for d in sorted(glob.glob(os.path.join(SRC, "*_fetch"))):
        cfg = os.path.basename(d)[: -len("_fetch")]
        if cfg == "calib":
            continue
        f = per_dispatch(f"{cfg}_fetch", "FETCH_SIZE", "msha::")
        w = per_dispatch(f"{cfg}_write", "WRITE_SIZE", "msha::")
        f_t, w_t = f[1:] or f, w[1:] or w          # skip the first (cold) dispatch
        fetch_b = sum(f_t) / len(f_t) * 1024 * factor
        write_b = sum(w_t) / len(w_t) * 1024
        out["configs"][cfg] = {"fetch_size_kb": f, "write_size_kb": w,
                               "read_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
                               "traffic_bytes_per_launch": fetch_b + write_b}
    with open(DST, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: v["traffic_bytes_per_launch"] for k, v in out["configs"].items()}), "factor", factor)


if __name__ == "__main__":
    main()
