#!/usr/bin/env python3
"""Summarise tools/pmc_valu.sh output (rocprofv3 --kernel-trace --pmc passes per
config) into profiles/<round>_pmc.json: the counters that justify the kernel
choices -- VALU issue (instructions per block, SIMD cycles per instruction,
VALUBusy, VALUUtilization), integer-op throughput against the int32 VALU peak,
clock under load, and HBM bytes/GB/s (FETCH_SIZE x the gfx950 calibration of
profiles/r01_traffic.json + WRITE_SIZE).

    python3 tools/pmc_summary.py gpurun_out/pmc profiles/r01_pmc.json

Only the last 3 dispatches of each run (bench.py's timed steps) are used; the
earlier ones are warmup (the bench warms up for >= 300 ms so clocks settle).
"""
import csv
import json
import os
import sys
from collections import defaultdict

SRC = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
DST = sys.argv[2] if len(sys.argv) > 2 else "profiles/r01_pmc.json"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPS_PER_BLOCK = 1400
PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
SIMDS, CUS, XCDS = 1024, 256, 8
HBM_PEAK_GBS = 8000.0


def calib_factor():
    with open(os.path.join(ROOT, "profiles", "r01_traffic.json")) as f:
        return json.load(f)["calib"]["calib_factor"]


def counters(run):
    """{dispatch: {counter: value}} and {dispatch: duration_ns} for our kernels."""
    vals = defaultdict(lambda: defaultdict(float))
    f = os.path.join(SRC, run, "run_counter_collection.csv")
    if not os.path.exists(f):
        return None, None
    for r in csv.DictReader(open(f)):
        if "msha::k_digest" in r["Kernel_Name"]:
            vals[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = {}
    for r in csv.DictReader(open(os.path.join(SRC, run, "run_kernel_trace.csv"))):
        if "msha::k_digest" in r["Kernel_Name"]:
            dur[int(r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return vals, dur


TIMED = 3  # bench.py --steps 3 in tools/pmc_valu.sh: the last 3 dispatches are the timed ones


def mean_timed(vals, dur, name):
    ds = sorted(vals)[-TIMED:]   # everything before them is warmup (clocks settling)
    return sum(vals[d].get(name, 0.0) for d in ds) / len(ds), sum(dur[d] for d in ds) / len(ds)


def bench_line(run):
    with open(os.path.join(SRC, run + ".log")) as f:
        lines = [l for l in f if l.startswith("{")]
    return json.loads(lines[-1])


def kernel_name(run):
    for r in csv.DictReader(open(os.path.join(SRC, run, "run_kernel_trace.csv"))):
        if "msha::k_digest" in r["Kernel_Name"]:
            return r["Kernel_Name"].split("(")[0].replace("void ", "")
    return None


def main():
    cf = calib_factor()
    names = sorted({d.rsplit("_", 1)[0] for d in os.listdir(SRC)
                    if os.path.isdir(os.path.join(SRC, d)) and d.endswith("_sq")})
    out = {"source": "tools/pmc_valu.sh (rocprofv3 --kernel-trace --pmc, one pass per counter group); "
                     "tools/pmc_summary.py",
           "definitions": {
               "clock_ghz": "GRBM_GUI_ACTIVE / 8 XCDs / kernel ns",
               "valu_instr_per_block": "SQ_INSTS_VALU x 64 lanes / 64-byte blocks (lane-instructions per block)",
               "simd_cycles_per_valu_instr": "clock cycles x 1024 SIMDs / SQ_INSTS_VALU",
               "valu_busy_pct": "VALUBusy = 100 x SQ_ACTIVE_INST_VALU / 256 CUs / (GRBM_GUI_ACTIVE / 8)",
               "valu_utilization_pct": "VALUUtilization = 100 x SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64)",
               "int32_share": "SQ_INSTS_VALU_INT32 / SQ_INSTS_VALU",
               "algorithmic_tops": "1400 x blocks / kernel ns (bench roofline.achieved); frac vs 78.64 T",
               "hbm_bytes": "FETCH_SIZE x calib (gfx950 half-count, profiles/r01_traffic.json) + WRITE_SIZE"},
           "configs": {}}
    for nm in names:
        sq, dsq = counters(nm + "_sq")
        sq2, dsq2 = counters(nm + "_sq2")
        fe, dfe = counters(nm + "_fetch")
        wr, dwr = counters(nm + "_write")
        b = bench_line(nm + "_sq")
        blocks, msgs = b["config"]["blocks_per_gpu"], b["config"]["messages_per_gpu"]
        grbm, ns = mean_timed(sq, dsq, "GRBM_GUI_ACTIVE")
        insts, _ = mean_timed(sq, dsq, "SQ_INSTS_VALU")
        active, _ = mean_timed(sq, dsq, "SQ_ACTIVE_INST_VALU")
        salu, _ = mean_timed(sq, dsq, "SQ_INSTS_SALU")
        wave_cyc, _ = mean_timed(sq, dsq, "SQ_WAVE_CYCLES")
        wait_any, _ = mean_timed(sq, dsq, "SQ_WAIT_ANY")
        cyc = grbm / XCDS
        e = {"kernel": kernel_name(nm + "_sq"), "workload": b["config"]["workload"],
             "messages": msgs, "blocks": blocks, "kernel_us": ns / 1e3,
             "clock_ghz": cyc / ns,
             "valu_instr_per_block": insts * 64 / blocks,
             "salu_instr_per_block": salu * 64 / blocks,
             "simd_cycles_per_valu_instr": cyc * SIMDS / insts,
             "valu_busy_pct": 100 * active / CUS / cyc,
             "wait_any_share": wait_any / wave_cyc if wave_cyc else None,
             "algorithmic_tops": OPS_PER_BLOCK * blocks / ns / 1e3,
             "roofline_frac": OPS_PER_BLOCK * blocks / ns / 1e3 / PEAK_TOPS}
        if sq2:
            i32, _ = mean_timed(sq2, dsq2, "SQ_INSTS_VALU_INT32")
            iops, ns2 = mean_timed(sq2, dsq2, "SQ_INSTS_VALU_IOPS")
            thr, _ = mean_timed(sq2, dsq2, "SQ_THREAD_CYCLES_VALU")
            act2, _ = mean_timed(sq2, dsq2, "SQ_ACTIVE_INST_VALU")
            lds, _ = mean_timed(sq2, dsq2, "SQ_INSTS_LDS")
            e.update({"int32_share": i32 / insts if insts else None,
                      "valu_iops_counter_T_per_s": iops / ns2 / 1e3,
                      "valu_utilization_pct": 100 * thr / (act2 * 64) if act2 else None,
                      "lds_instr_per_block": lds * 64 / blocks})
        if fe and wr:
            fetch_kb, _ = mean_timed(fe, dfe, "FETCH_SIZE")
            write_kb, _ = mean_timed(wr, dwr, "WRITE_SIZE")
            hbm = fetch_kb * 1024 * cf + write_kb * 1024
            alg = b["roofline"]["algorithmic_bytes_per_launch"]
            e.update({"hbm_bytes": hbm, "algorithmic_bytes": alg, "hbm_over_algorithmic": hbm / alg,
                      "hbm_gbs": hbm / ns, "hbm_frac_of_8TBs": hbm / ns / HBM_PEAK_GBS})
        out["configs"][nm] = e
    with open(DST, "w") as f:
        json.dump(out, f, indent=1)
    for nm, e in out["configs"].items():
        print(f"{nm:24s} {e['kernel_us']:9.1f} us  clk {e['clock_ghz']:.2f}  "
              f"valu/blk {e['valu_instr_per_block']:7.0f}  cyc/instr {e['simd_cycles_per_valu_instr']:.2f}  "
              f"busy {e['valu_busy_pct']:5.1f}%  util {e.get('valu_utilization_pct') or 0:5.1f}%  "
              f"int32 {e.get('int32_share') or 0:.2f}  frac {e['roofline_frac']:.3f}  "
              f"hbm {e.get('hbm_gbs', 0):6.0f} GB/s x{e.get('hbm_over_algorithmic', 0):.2f}")


if __name__ == "__main__":
    main()
