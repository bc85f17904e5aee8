#!/usr/bin/env python3
"""DESIGN.md's roofline table, generated from one default bench line, the
rocprofv3 kernel summaries of the same configs and the PMC summary:

    python3 tools/design_table.py profiles/r04_final/bench_default.json \\
        profiles/r04_final profiles/r04_pmc.json

One markdown row per config: digests/s, GB/s hashed, the mean launch from the
line's HIP events beside rocprofv3's average for the dominant kernel, roofline
frac (at 78.64 T and at the line's own effective clock), the PMC pass's VALU
busy, SIMD cycles per VALU instruction and HBM bytes over the algorithmic ones."""
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
    legs = {"c2": dict(line, frac=line["roofline"]["frac"], frac_at_clock=line["roofline"]["frac_at_clock"],
                       traffic=line["roofline"]["traffic"])}
    legs.update(line.get("extra_configs", {}))
    print("| config | kernel | digests/s | GB/s hashed | mean launch, events / rocprof avg | roofline.frac "
          "(at the line's clock) | clock GHz | VALU busy | SIMD cycles / VALU instr | HBM ÷ algorithmic |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for cfg, leg in legs.items():
        p = pmc.get(PMC_NAME.get(cfg, ""), {})
        kern = p.get("kernel", "")
        short = kern.replace("msha::", "")
        rp = rocprof_avg_us(prof_dir, cfg, kern) if kern else None
        ev_us = leg["kernel_ms_mean"] * 1e3
        rp_s = f"{rp:,.1f}" if rp is not None else "—"
        hbm = p.get("hbm_over_algorithmic")
        print(f"| {cfg} | `{short}` | {leg['value'] / 1e9:.3g} G | {leg['gbps_hashed']:,.0f} | "
              f"{ev_us:,.1f} / {rp_s} µs | {leg['frac']:.3f} ({leg.get('frac_at_clock', 0):.3f}) | "
              f"{leg.get('effective_clock_ghz', 0):.2f} | {p.get('valu_busy_pct', 0):.1f} % | "
              f"{p.get('simd_cycles_per_valu_instr', 0):.2f} | {hbm:.2f}× |" if hbm is not None else
              f"| {cfg} | `{short}` | {leg['value'] / 1e9:.3g} G | {leg['gbps_hashed']:,.0f} | "
              f"{ev_us:,.1f} / {rp_s} µs | {leg['frac']:.3f} | — | — | — | — |")


if __name__ == "__main__":
    main()
