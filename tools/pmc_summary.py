#!/usr/bin/env python3
"""Summarise tools/pmc_valu.sh output (rocprofv3 --kernel-trace --pmc passes per
config) into profiles/<round>_pmc.json: the counters that justify the kernel
choices -- VALU issue (instructions per block, SIMD cycles per instruction,
VALUBusy, VALUUtilization), integer-op throughput against the int32 VALU peak,
clock under load, and HBM bytes/GB/s (FETCH_SIZE x the gfx950 calibration +
WRITE_SIZE).

    python3 tools/pmc_summary.py gpurun_out/pmc profiles/r05_pmc.json [calib.json] [bench_line.json]

A bench step may run several kernels (the GPU-planned c5 forms: the k_fold_*
planner, the head on k_digest_chain2 / k_digest_coop, the lane kernel, the alias
fill). Every kernel whose name starts with msha:: is summarised on its own from
its last 3 dispatches (bench.py --steps 3: the timed steps; everything before is
warmup, >= 300 ms so clocks settle), and the step's HBM bytes are the sum over
its kernels. Under --pmc rocprofv3 serialises dispatches, so the head and the
lane kernel, concurrent in the bench, run one after the other here: per-kernel
figures are exact, the step's kernel time is the serial sum.

Top-level fields of a config describe its dominant hash kernel (the longest
k_digest_*), as in earlier rounds' files, plus "kernels" (each kernel) and
"step" (whole-step sums).

Only valid derived figures are published (round 5):
- clock_ghz (and the per-cycle figures built on it: SIMD cycles per VALU
  instruction, VALUBusy) is null for a kernel shorter than MIN_CLOCK_US, when
  it would exceed MAX_CLOCK_GHZ, or when VALUBusy would exceed 100 %:
  GRBM_GUI_ACTIVE also counts the dispatch's ramp and drain, which a 5-15 us
  kernel does not amortise (round 4 printed 6.01 GHz for k_fold_tilescan), and
  round 5's c5 read 103.7 % busy, so its counted cycles were short; the entry
  says why in clock_note.
- No fraction "at the clock" is derived: the only clocks are this counted one
  and msha_clock_probe's, read by a separate kernel after the timed steps.
- A step of several kernels runs them one after another under --pmc, so its
  frac over the serial sum is "serialized_frac"; "roofline_frac" is the
  overlapped step's, taken from a bench line (4th argument: a JSON line with
  extra_configs, e.g. the round's default bench output), else null.
"""
import csv
import json
import os
import sys
from collections import defaultdict

SRC = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
DST = sys.argv[2] if len(sys.argv) > 2 else "profiles/r04_pmc.json"
CALIB = sys.argv[3] if len(sys.argv) > 3 else None
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPS_PER_BLOCK = 1400
PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
SIMDS, CUS, XCDS = 1024, 256, 8
HBM_PEAK_GBS = 8000.0
TIMED = 3  # bench.py --steps 3 in tools/pmc_valu.sh
MIN_CLOCK_US = 50.0   # below this, GRBM_GUI_ACTIVE / ns does not resolve the clock
MAX_CLOCK_GHZ = 2.45  # MI355X tops at 2.4 GHz (+2 %): more is the counter window outlasting the kernel
MAX_BUSY_PCT = 100.0  # VALU busy above 100 %: the cycle count under the figures is wrong
BENCH = sys.argv[4] if len(sys.argv) > 4 else None
# waves per workgroup of the kernels that hold a CU each (heads): the CUs they occupy
WAVES_PER_WG = {"k_digest_chain2": 3, "k_digest_chain8": 4, "k_digest_coop": 4}


def calib_factor():
    """FETCH_SIZE -> bytes on gfx950: this run's calibration pass (calib_fetch:
    tools/traffic_calib reads 2^29 bytes with the engine's per-lane pattern; its
    first dispatch is cold and skipped) if present, else a given JSON, else
    round 1's (profiles/r01_traffic.json)."""
    f = os.path.join(SRC, "calib_fetch", "run_counter_collection.csv")
    if os.path.exists(f):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if "k_read_like_c2" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
                per[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        kb = [per[d] for d in sorted(per)][1:]
        if kb:
            return (1 << 29) / (1024.0 * sum(kb) / len(kb)), "this run's calib_fetch pass (tools/traffic_calib)"
    if CALIB and os.path.exists(CALIB):
        with open(CALIB) as f:
            return json.load(f)["calib_factor"], CALIB
    with open(os.path.join(ROOT, "profiles", "r01_traffic.json")) as f:
        return json.load(f)["calib"]["calib_factor"], "profiles/r01_traffic.json"


def short(name):
    return name.split("(")[0].replace("void ", "")


def counters(run):
    """{kernel: [(counters, ns) for its last TIMED dispatches]} for msha:: kernels."""
    f = os.path.join(SRC, run, "run_counter_collection.csv")
    if not os.path.exists(f):
        return None
    vals = defaultdict(lambda: defaultdict(float))
    kname = {}
    for r in csv.DictReader(open(f)):
        if "msha::k_" in r["Kernel_Name"]:
            d = int(r["Dispatch_Id"])
            vals[d][r["Counter_Name"]] += float(r["Counter_Value"])
            kname[d] = short(r["Kernel_Name"])
    dur = {}
    for r in csv.DictReader(open(os.path.join(SRC, run, "run_kernel_trace.csv"))):
        d = int(r["Dispatch_Id"])
        if d in kname:
            dur[d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    by = defaultdict(list)
    for d in sorted(kname):
        by[kname[d]].append((vals[d], dur.get(d, 0)))
    out = {}
    for k, v in by.items():
        if k.split("<")[0].split("::")[-1] in WAVES_PER_WG:
            # a folded step launches the head twice (the early head and the scan's
            # cut, one of them empty): keep the TIMED longest of the last 2 x TIMED
            out[k] = sorted(v[-2 * TIMED:], key=lambda r: -r[1])[:TIMED]
        else:
            out[k] = v[-TIMED:]
    return out


def mean(rows, name):
    return sum(c.get(name, 0.0) for c, _ in rows) / len(rows)


def mean_ns(rows):
    return sum(ns for _, ns in rows) / len(rows)


def bench_line(run):
    with open(os.path.join(SRC, run + ".log")) as f:
        lines = [l for l in f if l.startswith("{")]
    return json.loads(lines[-1])


def kernel_entry(k, sq, sq2, fe, wr, cf, max_blocks=0):
    rows = sq[k]
    ns = mean_ns(rows)
    grbm = mean(rows, "GRBM_GUI_ACTIVE")
    cyc = grbm / XCDS
    insts = mean(rows, "SQ_INSTS_VALU")
    active = mean(rows, "SQ_ACTIVE_INST_VALU")
    waves = mean(rows, "SQ_WAVES")
    wave_cyc = mean(rows, "SQ_WAVE_CYCLES")
    clk = cyc / ns if ns else None
    note = None
    if ns < MIN_CLOCK_US * 1e3:
        note = ("kernel shorter than %g us: GRBM_GUI_ACTIVE spans the dispatch's ramp and drain, so the clock "
                "and the per-cycle figures are not resolved" % MIN_CLOCK_US)
    elif clk and clk > MAX_CLOCK_GHZ:
        note = "counted clock %.2f GHz is above the part's %.1f GHz: not published" % (clk, 2.4)
    elif cyc and 100 * active / CUS / cyc > MAX_BUSY_PCT:
        # round 5 published 103.7 % for c5: SQ_ACTIVE_INST_VALU counted more VALU-busy
        # cycles than GRBM_GUI_ACTIVE / 8 counted cycles, so that cycle count (and the
        # clock and cycles per instruction built on it) is short for this kernel
        note = ("VALU busy %.1f %% > 100 %%: GRBM_GUI_ACTIVE under-counts this kernel's cycles, so its clock, "
                "busy and cycles per instruction are not published" % (100 * active / CUS / cyc))
    ok = note is None
    e = {"us": ns / 1e3, "clock_ghz": clk if ok else None,
         "valu_lane_instr": insts * 64, "salu_instr": mean(rows, "SQ_INSTS_SALU"), "waves": waves,
         "simd_cycles_per_valu_instr": cyc * SIMDS / insts if insts and ok else None,
         "valu_busy_pct": 100 * active / CUS / cyc if cyc and ok else None,
         "wait_any_share": mean(rows, "SQ_WAIT_ANY") / wave_cyc if wave_cyc else None}
    if note:
        e["clock_note"] = note
    base = k.split("<")[0].split("::")[-1]
    if base in WAVES_PER_WG and max_blocks and ok:
        # a head: its time is its longest chain's (max_blocks blocks, serial);
        # every workgroup of the launch is dispatched, those past the head's
        # lanes exit at once, so per-CU occupancy figures would mislead
        e["chain_blocks"] = max_blocks
        e["us_per_chain_block"] = ns / 1e3 / max_blocks
        e["cycles_per_chain_block"] = cyc / max_blocks
        e["wave_valu_instr_per_chain_block"] = insts / max_blocks
    if sq2 and k in sq2:
        r2 = sq2[k]
        thr, act2 = mean(r2, "SQ_THREAD_CYCLES_VALU"), mean(r2, "SQ_ACTIVE_INST_VALU")
        e.update({"int32_share": mean(r2, "SQ_INSTS_VALU_INT32") / insts if insts else None,
                  "valu_utilization_pct": 100 * thr / (act2 * 64) if act2 else None,
                  "lds_instr": mean(r2, "SQ_INSTS_LDS") * 64})
    if fe and wr and k in fe and k in wr:
        e["hbm_bytes"] = mean(fe[k], "FETCH_SIZE") * 1024 * cf + mean(wr[k], "WRITE_SIZE") * 1024
        e["hbm_gbs"] = e["hbm_bytes"] / ns if ns else None
    return e


def overlapped_fracs():
    """{config: roofline.frac} of the bench line's extra_configs (and its headline),
    measured with the step's kernels overlapped as they run in the bench."""
    if not BENCH or not os.path.exists(BENCH):
        return {}
    with open(BENCH) as f:
        lines = [l for l in f if l.lstrip().startswith("{")]
    if not lines:
        return {}
    line = json.loads(lines[-1])
    line = line.get("parsed", line) if "extra_configs" not in line else line
    out = {}
    for cfg, e in (line.get("extra_configs") or {}).items():
        if not isinstance(e, dict):
            continue
        if isinstance(e.get("roofline"), dict):
            out[cfg] = e["roofline"].get("frac")
        elif "frac" in e:  # bench.py's extra_configs legs carry frac at top level
            out[cfg] = e["frac"]
    return out


def main():
    cf, cf_src = calib_factor()
    over = overlapped_fracs()
    names = sorted({d.rsplit("_", 1)[0] for d in os.listdir(SRC)
                    if os.path.isdir(os.path.join(SRC, d)) and d.endswith("_sq")})
    out = {"source": "tools/pmc_valu.sh (rocprofv3 --kernel-trace --pmc, one pass per counter group); "
                     "tools/pmc_summary.py",
           "calib_factor": cf, "calib_source": cf_src,
           "definitions": {
               "clock_ghz": "GRBM_GUI_ACTIVE / 8 XCDs / kernel ns",
               "valu_instr_per_block": "SQ_INSTS_VALU x 64 lanes / 64-byte blocks hashed (lane-instructions "
                                       "per block; the step's hash kernels)",
               "simd_cycles_per_valu_instr": "clock cycles x 1024 SIMDs / SQ_INSTS_VALU",
               "valu_busy_pct": "VALUBusy = 100 x SQ_ACTIVE_INST_VALU / 256 CUs / (GRBM_GUI_ACTIVE / 8)",
               "cycles_per_chain_block": "heads: GRBM clock cycles of the launch / its longest chain's blocks "
                                         "(the head's time is that chain's)",
               "valu_utilization_pct": "VALUUtilization = 100 x SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64)",
               "int32_share": "SQ_INSTS_VALU_INT32 / SQ_INSTS_VALU",
               "algorithmic_tops": "1400 x hashed blocks / the step's serial kernel ns; serialized_frac vs 78.64 T",
               "roofline_frac": "one-kernel steps: serialized_frac; several kernels: the bench line's overlapped frac",
               "hbm_bytes": "FETCH_SIZE x calib_factor (gfx950 half-count) + WRITE_SIZE, per kernel; the step's "
                            "is the sum over its kernels"},
           "configs": {}}
    for nm in names:
        sq = counters(nm + "_sq")
        if not sq:
            continue
        sq2 = counters(nm + "_sq2")
        fe = counters(nm + "_fetch")
        wr = counters(nm + "_write")
        b = bench_line(nm + "_sq")
        cfg = b["config"]
        blocks, msgs = cfg["blocks_per_gpu"], cfg["messages_per_gpu"]
        hashed = cfg.get("hashed_blocks_per_gpu", blocks)
        kernels = {k: kernel_entry(k, sq, sq2, fe, wr, cf, cfg.get("max_blocks_per_message", 0)) for k in sq}
        # msha_clock_probe runs after the timed steps (bench.py effective_clock_ghz): not part of a step
        probe = {k: kernels.pop(k) for k in list(kernels) if "k_clock_probe" in k}
        hash_k = [k for k in kernels if "k_digest" in k]
        dom = max(hash_k, key=lambda k: kernels[k]["us"]) if hash_k else max(kernels, key=lambda k: kernels[k]["us"])
        step_us = sum(e["us"] for e in kernels.values())
        hash_instr = sum(kernels[k]["valu_lane_instr"] for k in hash_k)
        d = kernels[dom]
        e = {"kernel": dom, "workload": cfg["workload"], "messages": msgs, "blocks": blocks,
             "hashed_blocks": hashed, "kernel_us": d["us"], "clock_ghz": d["clock_ghz"],
             "valu_instr_per_block": hash_instr / hashed,
             "simd_cycles_per_valu_instr": d["simd_cycles_per_valu_instr"],
             "valu_busy_pct": d["valu_busy_pct"], "wait_any_share": d["wait_any_share"],
             "int32_share": d.get("int32_share"), "valu_utilization_pct": d.get("valu_utilization_pct"),
             "algorithmic_tops": OPS_PER_BLOCK * hashed / step_us / 1e6,
             "serialized_frac": OPS_PER_BLOCK * hashed / step_us / 1e6 / PEAK_TOPS,
             "step": {"us_serialized": step_us, "kernels": sorted(kernels, key=lambda k: -kernels[k]["us"])},
             "kernels": kernels}
        cfg_name = nm.rsplit("_", 1)[0]
        if len(kernels) == 1:
            e["roofline_frac"] = e["serialized_frac"]  # one kernel: nothing to overlap
        else:
            e["roofline_frac"] = over.get(cfg_name)
            e["roofline_frac_note"] = ("the step's kernels overlap in the bench but run one after another under "
                                       "--pmc: serialized_frac is over their serial sum; roofline_frac is the "
                                       "bench line's (%s)" % (BENCH or "none given: null"))
        if probe:
            e["clock_probe_after_steps"] = next(iter(probe.values()))
        if all("hbm_bytes" in k for k in kernels.values()):
            hbm = sum(k["hbm_bytes"] for k in kernels.values())
            alg = b["roofline"]["algorithmic_bytes_per_launch"]
            e.update({"hbm_bytes": hbm, "algorithmic_bytes": alg, "hbm_over_algorithmic": hbm / alg,
                      "hbm_gbs": hbm / (step_us * 1e3), "hbm_frac_of_8TBs": hbm / (step_us * 1e3) / HBM_PEAK_GBS})
        out["configs"][nm] = e
    with open(DST, "w") as f:
        json.dump(out, f, indent=1)
    for nm, e in out["configs"].items():
        print(f"{nm:20s} {e['kernel'][:34]:34s} {e['kernel_us']:9.1f} us step {e['step']['us_serialized']:9.1f}"
              f"  clk {e['clock_ghz'] or 0:.2f}  valu/blk {e['valu_instr_per_block']:7.0f}"
              f"  cyc/instr {e['simd_cycles_per_valu_instr'] or 0:.2f}  busy {e['valu_busy_pct'] or 0:5.1f}%"
              f"  frac {e['roofline_frac'] if e['roofline_frac'] is not None else float('nan'):.3f}"
              f" (serialized {e['serialized_frac']:.3f})  hbm x{e.get('hbm_over_algorithmic', 0):.2f}")
        for k, v in e["kernels"].items():
            if k != e["kernel"]:
                ch = v.get("cycles_per_chain_block")
                print(f"    {k[:44]:44s} {v['us']:8.1f} us  busy {v['valu_busy_pct'] or 0:5.1f}%"
                      + (f" (chain: {v['us_per_chain_block']:.3f} us, {ch:.0f} cycles per block)" if ch else "")
                      + f"  hbm {v.get('hbm_bytes', 0) / 1e6:8.1f} MB")


if __name__ == "__main__":
    main()
