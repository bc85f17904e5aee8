#!/bin/bash
# Round-6 evidence run: GPU tests, smoke, the default bench line, and a
# rocprofv3 kernel summary per config next to that command's own event timing.
# Every GPU step has its own time limit; a fault/abort/timeout ends the run.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06_final}
mkdir -p $OUT
stop() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -ne 0 ] && { echo "stopping after $name"; exit $rc; }; return 0; }
if [[ ${STEPS:-all} == all || $STEPS == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; stop $? pytest
  tail -2 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; stop $? smoke
fi
if [[ ${STEPS:-all} == all || $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err; stop $? bench
  python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print('c2', d['value'], d['roofline']['frac'], 'clock_after', d.get('clock_after', {}).get('effective_clock_ghz'), {k: (round(v['frac'],4), v.get('kernel')) for k, v in d['extra_configs'].items()}, 'host_api', d['host_api'].get('value'), 'unaliased', d.get('host_api_unaliased', {}).get('value'))"
fi
if [[ ${STEPS:-all} == all || $STEPS == *prof* ]]; then
  for cfg in ${PCFGS:-c2 c3 c3dd c4 c5 c5_planned c5_folded}; do
    rm -rf $OUT/prof_$cfg
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$cfg -o run -- \
      python3 bench.py --config $cfg --no-cpu-baseline --no-host-api --no-extra > $OUT/prof_bench_$cfg.log 2>&1; stop $? rocprof_$cfg
    f=$(find $OUT/prof_$cfg -name "*kernel_stats.csv" | head -1); cp $f $OUT/rocprof_${cfg}_kernel_stats.csv
    grep '^{' $OUT/prof_bench_$cfg.log > $OUT/rocprof_${cfg}_bench_line.json
    python3 -c "
import csv, json
d = json.load(open('$OUT/rocprof_${cfg}_bench_line.json'))
rows = list(csv.DictReader(open('$OUT/rocprof_${cfg}_kernel_stats.csv')))
top = max(rows, key=lambda r: float(r['TotalDurationNs']))
print('$cfg', top['Name'][:50], 'rocprof avg', round(float(top['AverageNs'])/1e3, 2), 'us; events', round(d['kernel_ms_mean']*1e3, 2), 'us')"
  done
fi
