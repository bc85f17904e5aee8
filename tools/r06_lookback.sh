#!/bin/bash
# Round 6: the folded insert's tile look-back (no k_fold_tilemax / k_fold_tilescan)
# -- planned GPU tests, then c5_folded with the look-back (default) and with the
# two-kernel prefix (MSHA_FOLD_LOOKBACK=0), 3 reps interleaved, and a rocprofv3
# summary + kernel trace of the default folded step.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06_lookback}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_planned.py -m gpu -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_planned.txt 2>&1 || { tail -30 $OUT/pytest_planned.txt; exit 1; }
tail -1 $OUT/pytest_planned.txt
for rep in 1 2 3; do
  for v in "c5_folded MSHA_X=1" "c5_folded MSHA_FOLD_LOOKBACK=0"; do
    cfg=${v%% *}; e=${v#* }; tag=${cfg}_$(echo $e | tr '=' '_')
    env $e timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-host-api --no-extra \
      > $OUT/bench_${tag}_rep$rep.json 2> $OUT/bench_${tag}_rep$rep.err || { tail $OUT/bench_${tag}_rep$rep.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/bench_${tag}_rep$rep.json'))
print('$tag rep$rep', round(d['kernel_ms_mean'], 4), round(d['roofline']['frac'], 4), d['kernel'])"
  done
done
for cfg in c5_folded; do
  rm -rf $OUT/prof_$cfg
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$cfg -o run -- \
    python3 bench.py --config $cfg --no-cpu-baseline --no-host-api --no-extra > $OUT/prof_$cfg.log 2>&1 \
    || { tail -5 $OUT/prof_$cfg.log; exit 1; }
  f=$(find $OUT/prof_$cfg -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats_$cfg.csv
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kernel_stats_$cfg.csv')):
    if 'fold' in r['Name'] or 'batch' in r['Name'] or 'chain' in r['Name']: print('$cfg', r['Name'][:40], round(float(r['AverageNs'])/1e3, 1))"
done
# planner stamps (diagnostic build outside the package), look-back on and off
timeout -k 10 300 bash tools/ab_build.sh pstamps -DMSHA_PLAN_STAMPS > $OUT/build.log 2>&1 || { tail $OUT/build.log; exit 1; }
for lb in 1 0; do
  MSHA_FOLD_LOOKBACK=$lb RAW_DIR=$OUT/raw_lb$lb MSHA_LIB_PATH=/tmp/msha_ab/pstamps.so MSHA_ALLOW_FOREIGN_LIB=1 \
    timeout -k 10 300 python -u tools/plan_stamps.py > $OUT/plan_stamps_lb$lb.jsonl 2> $OUT/plan_stamps_lb$lb.err \
    || { tail -20 $OUT/plan_stamps_lb$lb.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/plan_stamps_lb$lb.jsonl').readline())
print('lb$lb step', round(d['step_ms_stamped_build'], 4))
for k, v in d['kernels'].items():
    if v.get('workgroups'): print(' ', k, 'start', v['first_start_us'], 'end', v['end_us'], 'span', v['span_us'], {p: (x['p50'], x['p90'], round(x['wgs_in_phase'], 1)) for p, x in v['phases'].items()})"
done
