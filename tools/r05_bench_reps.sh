#!/bin/bash
# Round 5: the default bench line three times on one box (run-to-run spread of the
# headline and of the extra configs), each run under its own time limit.
set -u
OUT=${OUT:-gpurun_out/r05_reps}
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --no-host-api > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail -3 $OUT/bench_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_$i.json'))
print($i, 'c2 %.4g' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'clock %.3f' % d['effective_clock_ghz'],
      ' '.join('%s %.4f' % (k, v['frac']) for k, v in d['extra_configs'].items()))"
done
