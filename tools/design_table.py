#!/usr/bin/env python3
"""DESIGN.md's roofline table, generated from one default bench line, the
rocprofv3 kernel summaries of the same configs and the PMC summary:

    python3 tools/design_table.py profiles/r05_final/bench_default.json \\
        profiles/r05_final profiles/r05_pmc.json > profiles/r05_final/design_table.md

One markdown row per config: digests/s, GB/s hashed, the mean launch from the
line's HIP events beside rocprofv3's average for the dominant kernel, roofline
frac (at 78.64 T), the PMC pass's VALU busy, SIMD cycles per VALU instruction
and HBM bytes over the algorithmic ones. No fraction "at a clock" is printed: the
only clocks are the PMC-counted one and a probe kernel's after the timed steps
(round 6: the in-kernel stamps of tools/lane_stamps.py are the clock evidence)."""
import csv
import json
import os
import sys

PMC_NAME = {"c2": "c2_auto", "c3": "c3_auto", "c3dd": "c3dd_auto", "c4": "c4_auto", "c5": "c5_auto",
            "c5_planned": "c5_planned_auto", "c5_folded": "c5_folded_auto"}


def rocprof_avg_us(prof_dir, cfg, kernel):
    path = os.path.join(prof_dir, f"rocprof_{cfg}_kernel_stats.csv")
    if not os.path.exists(path):
        return None
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        if r["Name"].startswith(kernel) or kernel in r["Name"]:
            return float(r["AverageNs"]) / 1e3
    return None


def main():
    bench, prof_dir, pmc_path = sys.argv[1:4]
    line = json.load(open(bench))
    pmc = json.load(open(pmc_path))["configs"]
    legs = {"c2": dict(line, frac=line["roofline"]["frac"], traffic=line["roofline"]["traffic"])}
    legs.update(line.get("extra_configs", {}))
    print("| config | dominant kernel (launches in the line) | digests/s | GB/s hashed | mean launch (default line) | "
          "rocprof command: events / rocprof avg | roofline.frac | VALU busy | SIMD cycles / VALU instr | "
          "HBM ÷ algorithmic |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for cfg, leg in legs.items():
        p = pmc.get(PMC_NAME.get(cfg, ""), {})
        kern = p.get("kernel", "")
        short = kern.replace("msha::", "")
        rp = rocprof_avg_us(prof_dir, cfg, kern) if kern else None
        ev_us = leg["kernel_ms_mean"] * 1e3
        rp_s = f"{rp:,.1f}" if rp is not None else "—"
        own = os.path.join(prof_dir, f"rocprof_{cfg}_bench_line.json")  # the rocprof command's own line
        own_us = json.load(open(own))["kernel_ms_mean"] * 1e3 if os.path.exists(own) else None
        own_s = f"{own_us:,.1f}" if own_us is not None else "—"
        hbm = p.get("hbm_over_algorithmic")

        def f(v, fmt, suffix=""):  # a figure the PMC summary left null (unresolved clock) prints as a dash
            return format(v, fmt) + suffix if isinstance(v, (int, float)) else "—"
        print(f"| {cfg} | `{short}` ({leg.get('kernel', '')}) | {leg['value'] / 1e9:.3g} G | {leg['gbps_hashed']:,.0f} | "
              f"{ev_us:,.1f} µs | {own_s} / {rp_s} µs | {leg['frac']:.3f} | "
              f"{f(p.get('valu_busy_pct'), '.1f', ' %')} | "
              f"{f(p.get('simd_cycles_per_valu_instr'), '.2f')} | {f(hbm, '.2f', '×')} |")

if __name__ == "__main__":
    main()
