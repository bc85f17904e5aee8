#!/bin/bash
# Round 6: default bench lines (GPU legs only) on whatever box this call gets, twice,
# for the box-to-box spread beside profiles/r06_final/bench_default.json.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_reps/$(date +%s)
mkdir -p $OUT
for rep in 1 2; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --no-host-api > $OUT/bench_rep$rep.json 2> $OUT/bench_rep$rep.err \
    || { tail $OUT/bench_rep$rep.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$OUT/bench_rep$rep.json'))
print('rep$rep c2', round(d['roofline']['frac'], 4), round(d['kernel_ms_mean'], 4), 'clock_after', round(d['clock_after'].get('effective_clock_ghz', 0), 3),
      {k: round(v['frac'], 4) for k, v in d['extra_configs'].items()})"
done
