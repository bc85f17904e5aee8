#!/bin/bash
# Round 6: the work-stealing lane kernel's claim taken one tile ahead (default) vs at
# each tile's start (-DMSHA_WS_NO_PREFETCH variant, built here, loaded by path) vs
# the static lane kernel (MSHA_LANE_WS=0): planned GPU tests on the product, then
# c5_folded bench lines interleaved, 3 reps.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_ws3
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_planned.py -m gpu -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_planned.txt 2>&1 || { tail -30 $OUT/pytest_planned.txt; exit 1; }
tail -1 $OUT/pytest_planned.txt
timeout -k 10 300 bash tools/ab_build.sh noprefetch -DMSHA_WS_NO_PREFETCH > $OUT/build.log 2>&1 || { tail $OUT/build.log; exit 1; }
for rep in 1 2 3; do
  for v in "MSHA_X=1" "MSHA_LIB_PATH=/tmp/msha_ab/noprefetch.so MSHA_ALLOW_FOREIGN_LIB=1" "MSHA_LANE_WS=0" "MSHA_FILL_WGS=256"; do
    tag=$(echo $v | cut -d' ' -f1 | tr '=/' '__')
    env $v timeout -k 10 300 python bench.py --config c5_folded --no-cpu-baseline --no-host-api --no-extra \
      > $OUT/bench_${tag}_rep$rep.json 2> $OUT/bench_${tag}_rep$rep.err || { tail $OUT/bench_${tag}_rep$rep.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/bench_${tag}_rep$rep.json'))
print('$tag rep$rep', round(d['kernel_ms_mean'], 4), round(d['roofline']['frac'], 4), d['kernel'])"
  done
done
rm -rf $OUT/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --config c5_folded --no-cpu-baseline --no-host-api --no-extra > $OUT/prof_bench.log 2>&1 \
  || { tail -5 $OUT/prof_bench.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kernel_stats.csv')):
    print(r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1e3, 1))"
