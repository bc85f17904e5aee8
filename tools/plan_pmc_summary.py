#!/usr/bin/env python3
"""Per-dispatch PMC figures of the folded planner's kernels (tools/r06_plan_pmc.sh):

    python3 tools/plan_pmc_summary.py gpurun_out/r06_plan_pmc > profiles/.../plan_pmc.json

Per kernel: dispatches; LDS instructions, LDS bank-conflict cycles (SQ_LDS_BANK_CONFLICT,
summed over the chip) and their ratio; the LDS-wait share of wave cycles; vector
memory instructions; FETCH_SIZE / WRITE_SIZE in KiB as counted (FETCH_SIZE half-counts
on gfx950: tools/pmc_summary.py's calibration is not applied here, so compare fetch
figures only with each other)."""
import csv
import glob
import json
import os
import sys


def load(path):
    fs = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    acc = {}
    if not fs:
        return acc
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"]
        if "fold" not in k:
            continue
        k = k.split("(")[0].replace("msha::", "")
        d = acc.setdefault(k, {"_dispatches": set()})
        d["_dispatches"].add(r["Dispatch_Id"])
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return acc


def main(out):
    lds, fetch, write = (load(os.path.join(out, p)) for p in ("lds", "fetch", "write"))
    res = {}
    for k, d in sorted(lds.items()):
        n = len(d["_dispatches"])
        per = {c: v / n for c, v in d.items() if not c.startswith("_")}
        e = {"dispatches": n,
             "lds_instr": round(per.get("SQ_INSTS_LDS", 0)),
             "lds_bank_conflict_cycles": round(per.get("SQ_LDS_BANK_CONFLICT", 0)),
             "conflict_cycles_per_lds_instr": round(per["SQ_LDS_BANK_CONFLICT"] / per["SQ_INSTS_LDS"], 2)
             if per.get("SQ_INSTS_LDS") else None,
             "lds_wait_share_of_wave_cycles": round(per.get("SQ_WAIT_INST_LDS", 0) / per["SQ_WAVE_CYCLES"], 4)
             if per.get("SQ_WAVE_CYCLES") else None,
             "vmem_rd_instr": round(per.get("SQ_INSTS_VMEM_RD", 0)),
             "vmem_wr_instr": round(per.get("SQ_INSTS_VMEM_WR", 0))}
        for name, src, ctr in (("fetch_kib_counted", fetch, "FETCH_SIZE"), ("write_kib", write, "WRITE_SIZE")):
            f = src.get(k)
            if f and ctr in f:
                e[name] = round(f[ctr] / len(f["_dispatches"]), 1)
        res[k] = e
    print(json.dumps({"source": out, "kernels": res}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
