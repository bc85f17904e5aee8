#!/bin/bash
# Round 6: the folded planner after the look-back -- two-pass insert, register/wave
# k_fold_scan, one aligned memset. Planned GPU tests; c5_folded default vs the
# two-kernel prefix (MSHA_FOLD_LOOKBACK=0), 3 reps interleaved; folded rank slices
# (N = 1, 2, 4, 8) both ways; planner stamps; a rocprofv3 trace of the default.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06_plan3}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_planned.py -m gpu -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_planned.txt 2>&1 || { tail -30 $OUT/pytest_planned.txt; exit 1; }
tail -1 $OUT/pytest_planned.txt
for rep in 1 2 3; do
  for e in MSHA_X=1 MSHA_FOLD_LOOKBACK=0; do
    tag=c5_folded_$(echo $e | tr '=' '_')
    env $e timeout -k 10 300 python bench.py --config c5_folded --no-cpu-baseline --no-host-api --no-extra \
      > $OUT/bench_${tag}_rep$rep.json 2> $OUT/bench_${tag}_rep$rep.err || { tail $OUT/bench_${tag}_rep$rep.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/bench_${tag}_rep$rep.json'))
print('$tag rep$rep', round(d['kernel_ms_mean'], 4), round(d['roofline']['frac'], 4), d['kernel'])"
  done
done
for e in MSHA_X=1 MSHA_FOLD_LOOKBACK=0; do
  env $e FORMS=c5_folded timeout -k 10 300 python -u tools/c5_slice.py > $OUT/slices_$(echo $e | tr '=' '_').jsonl \
    2> $OUT/slices.err || { tail $OUT/slices.err; exit 1; }
  python3 -c "
import json
for l in open('$OUT/slices_$(echo $e | tr '=' '_').jsonl'):
    d = json.loads(l); print('$e', {k: d[k] for k in d if k in ('world', 'form', 'kernel_ms_mean', 'kernel_ms')})"
done
timeout -k 10 300 bash tools/ab_build.sh pstamps -DMSHA_PLAN_STAMPS > $OUT/build.log 2>&1 || { tail $OUT/build.log; exit 1; }
MSHA_LIB_PATH=/tmp/msha_ab/pstamps.so MSHA_ALLOW_FOREIGN_LIB=1 RAW_DIR=$OUT/raw \
  timeout -k 10 300 python -u tools/plan_stamps.py > $OUT/plan_stamps.jsonl 2> $OUT/plan_stamps.err \
  || { tail -20 $OUT/plan_stamps.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$OUT/plan_stamps.jsonl').readline())
print('stamped step', round(d['step_ms_stamped_build'], 4))
for k, v in d['kernels'].items():
    if v.get('workgroups'): print(' ', k, 'start', v['first_start_us'], 'end', v['end_us'], 'span', v['span_us'], {p: (x['p50'], x['p90'], round(x['wgs_in_phase'], 1)) for p, x in v['phases'].items()})"
rm -rf $OUT/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --config c5_folded --no-cpu-baseline --no-host-api --no-extra > $OUT/prof.log 2>&1 \
  || { tail -5 $OUT/prof.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')):
    print(r['Name'][:44], round(float(r['AverageNs'])/1e3, 1))"
