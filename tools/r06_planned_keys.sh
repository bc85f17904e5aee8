#!/bin/bash
# Round 6: c5_planned (unfolded) after k_fold_keys' loads were hoisted: 2 bench lines
# and a rocprofv3 summary (k_fold_keys / scan / scatter beside the lane kernel).
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06_planned_keys}
mkdir -p $OUT
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config c5_planned --no-cpu-baseline --no-host-api --no-extra \
    > $OUT/bench_c5_planned_rep$rep.json 2>/dev/null || exit 1
  python3 -c "
import json; d = json.load(open('$OUT/bench_c5_planned_rep$rep.json'))
print('c5_planned rep$rep', round(d['kernel_ms_mean'], 4), round(d['roofline']['frac'], 4))"
done
rm -rf $OUT/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --config c5_planned --no-cpu-baseline --no-host-api --no-extra > $OUT/prof.log 2>&1 \
  || { tail -5 $OUT/prof.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')):
    if 'fold' in r['Name']: print(r['Name'][:44], round(float(r['AverageNs'])/1e3, 1))"
