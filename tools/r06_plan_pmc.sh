#!/bin/bash
# Round 6: PMC passes over the folded planner's kernels (c5_folded, bench.py steps):
# LDS instructions, bank-conflict cycles and LDS waits; HBM bytes (FETCH_SIZE,
# WRITE_SIZE). Then an A/B of the early-head gate's workgroups (MSHA_GATE_WGS).
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06_plan_pmc}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
cmd="python3 bench.py --config c5_folded --steps 3 --warmup 1 --no-cpu-baseline --no-extra --no-host-api"
prof() {  # name, counters
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $2 --output-format csv -d $OUT/$1 -o run -- $cmd > $OUT/$1.log 2>&1
  local rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0
}
prof lds "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
prof fetch FETCH_SIZE
prof write WRITE_SIZE
python3 - $OUT <<'PY'
import csv, glob, os, sys
out = sys.argv[1]
for p in ("lds", "fetch", "write"):
    fs = glob.glob(os.path.join(out, p, "**", "*counter_collection.csv"), recursive=True)
    if not fs:
        print(p, "no counter file"); continue
    acc = {}
    for r in csv.DictReader(open(fs[0])):
        k = r.get("Kernel_Name", "")
        if "fold" not in k: continue
        k = k.split("(")[0].replace("msha::", "")
        d = acc.setdefault(k, {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["_n"] = d.get("_n", 0) + (1 if r["Counter_Name"] == list(d.keys())[0] else 0)
    for k, d in sorted(acc.items()):
        print(p, k, {c: round(v) for c, v in d.items()})
PY
for rep in 1 2; do
  for e in MSHA_X=1 MSHA_GATE_WGS=128 MSHA_GATE_WGS=32; do
    env $e timeout -k 10 300 python bench.py --config c5_folded --no-cpu-baseline --no-host-api --no-extra \
      > $OUT/bench_$(echo $e | tr '=' '_')_rep$rep.json 2>/dev/null || exit 1
    python3 -c "
import json; d = json.load(open('$OUT/bench_$(echo $e | tr '=' '_')_rep$rep.json'))
print('$e rep$rep', round(d['kernel_ms_mean'], 4), round(d['roofline']['frac'], 4))"
  done
done
