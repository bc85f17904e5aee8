#!/bin/bash
# Round 6: planner changes -- wave-aggregated scatter positions and unfolded key
# counts, sampled lengths in the tile prefix (MSHA_TILE_SAMPLE=1: every tile, A/B) --
# planned GPU tests, then c5_folded (both) and c5_planned bench lines, 3 reps, and a
# rocprofv3 summary of each planned form.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_plan2
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_planned.py -m gpu -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_planned.txt 2>&1 || { tail -30 $OUT/pytest_planned.txt; exit 1; }
tail -1 $OUT/pytest_planned.txt
for rep in 1 2 3; do
  for v in "c5_folded MSHA_X=1" "c5_folded MSHA_TILE_SAMPLE=1" "c5_planned MSHA_X=1"; do
    cfg=${v%% *}; e=${v#* }; tag=${cfg}_$(echo $e | tr '=' '_')
    env $e timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-host-api --no-extra \
      > $OUT/bench_${tag}_rep$rep.json 2> $OUT/bench_${tag}_rep$rep.err || { tail $OUT/bench_${tag}_rep$rep.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/bench_${tag}_rep$rep.json'))
print('$tag rep$rep', round(d['kernel_ms_mean'], 4), round(d['roofline']['frac'], 4), d['kernel'])"
  done
done
for cfg in c5_folded c5_planned; do
  rm -rf $OUT/prof_$cfg
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$cfg -o run -- \
    python3 bench.py --config $cfg --no-cpu-baseline --no-host-api --no-extra > $OUT/prof_$cfg.log 2>&1 \
    || { tail -5 $OUT/prof_$cfg.log; exit 1; }
  f=$(find $OUT/prof_$cfg -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats_$cfg.csv
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kernel_stats_$cfg.csv')):
    if 'fold' in r['Name'] or 'batch' in r['Name']: print('$cfg', r['Name'][:40], round(float(r['AverageNs'])/1e3, 1))"
done
