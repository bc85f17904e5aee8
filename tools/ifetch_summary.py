#!/usr/bin/env python3
"""Summarise the `ifetch` PMC pass of tools/pmc_valu.sh (instruction cache hits/misses,
instruction fetches per VALU instruction, share of wave cycles waiting for issue) for the
last msha kernel dispatch in each run_counter_collection.csv given."""
import csv,sys,collections
for f in sys.argv[1:]:
    rows=list(csv.DictReader(open(f)))
    k=collections.defaultdict(lambda: collections.defaultdict(float)); names={}
    for r in rows:
        d=r["Dispatch_Id"]; names[d]=r["Kernel_Name"]; k[d][r["Counter_Name"]]+=float(r["Counter_Value"])
    ds=[d for d in k if "msha" in names[d]]
    d=ds[-1]; c=k[d]
    print(f.split('/')[-2], names[d][:45])
    print("  icache req %.4g hit %.4f miss %.4g dup %.4g | ifetch %.4g | wait_inst/wave_cycles %.4f | valu %.4g ifetch/valu %.4f" % (
        c["SQC_ICACHE_REQ"], c["SQC_ICACHE_HITS"]/max(c["SQC_ICACHE_REQ"],1), c["SQC_ICACHE_MISSES"], c["SQC_ICACHE_MISSES_DUPLICATE"],
        c["SQ_IFETCH"], c["SQ_WAIT_INST_ANY"]/c["SQ_WAVE_CYCLES"], c["SQ_INSTS_VALU"], c["SQ_IFETCH"]/c["SQ_INSTS_VALU"]))
