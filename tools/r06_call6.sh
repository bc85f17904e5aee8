#!/bin/bash
# Round 6: the planner's packed histogram (k_fold_insert at 4 workgroups a CU) --
# planned GPU tests, a rocprofv3 kernel summary of c5_folded (the insert's time) --
# and the early-head fork again with a small gate grid (MSHA_LONGS_WGS=64), one GPU
# and an 8-GPU rank slice, interleaved.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_call6
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_planned.py -m gpu -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_planned.txt 2>&1 || { tail -30 $OUT/pytest_planned.txt; exit 1; }
tail -1 $OUT/pytest_planned.txt
rm -rf $OUT/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --config c5_folded --no-cpu-baseline --no-host-api --no-extra > $OUT/prof_bench.log 2>&1 \
  || { tail -5 $OUT/prof_bench.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kernel_stats.csv')):
    print(r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1e3, 1))"
for rep in 1 2; do
  for v in "MSHA_EARLY_FORK=0" "MSHA_EARLY_FORK=1 MSHA_LONGS_WGS=64" "MSHA_LONGS_WGS=64"; do
    tag=$(echo $v | tr ' =' '__')
    env $v FORMS=c5_folded WORLDS="1 8" TIMED_STEPS=30 timeout -k 10 300 python -u tools/c5_slice.py \
      > $OUT/slices_${tag}_rep$rep.jsonl 2> $OUT/slices_${tag}_rep$rep.err || { tail $OUT/slices_${tag}_rep$rep.err; exit 1; }
    python3 -c "
import json
for l in open('$OUT/slices_${tag}_rep$rep.jsonl'):
    d = json.loads(l); print('$v rep$rep', d['world'], round(d['kernel_ms'], 4))"
  done
done
