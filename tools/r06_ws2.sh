#!/bin/bash
# Round 6: the work-stealing lane kernel's cut threshold (MSHA_WS_LONG: chains of at
# least this many blocks kept off it; 4294967295 = the cost model alone) against the
# static lane kernel (MSHA_LANE_WS=0), c5_folded bench lines interleaved, 3 reps.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_ws2
mkdir -p $OUT
for rep in 1 2 3; do
  for v in "MSHA_LANE_WS=0" "MSHA_WS_LONG=4294967295" "MSHA_WS_LONG=256" "MSHA_WS_LONG=64" "MSHA_WS_LONG=600"; do
    tag=$(echo $v | tr '=' '_')
    env $v timeout -k 10 300 python bench.py --config c5_folded --no-cpu-baseline --no-host-api --no-extra \
      > $OUT/bench_${tag}_rep$rep.json 2> $OUT/bench_${tag}_rep$rep.err || { tail $OUT/bench_${tag}_rep$rep.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/bench_${tag}_rep$rep.json'))
print('$v rep$rep', round(d['kernel_ms_mean'], 4), round(d['roofline']['frac'], 4))"
  done
done
