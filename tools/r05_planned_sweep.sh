#!/bin/bash
# Round 5: the unfolded planned head's cut at 8 GPUs -- c5_planned N = 8 slices
# under cost-model knobs (KNOBS: space-separated NAME=VALUE[,NAME=VALUE] sets;
# "base" = defaults), interleaved, two reps.
set -u
OUT=${OUT:-gpurun_out/r05_psweep}
mkdir -p $OUT
KNOBS=${KNOBS:-"base MSHA_PLAN_WAVE_CYCLES=5500 MSHA_PLAN_WAVE_CYCLES=4500 MSHA_PLAN_LANE_CYCLES=7000 MSHA_PLAN_LANE_CYCLES=6000"}
for rep in 1 2; do
  for k in $KNOBS; do
    env_args=""; [ "$k" != base ] && env_args=$(echo $k | tr ',' ' ')
    env $env_args FORMS=c5_planned WORLDS="${WORLDS:-8}" timeout -k 10 300 python tools/c5_slice.py > $OUT/${k//[=,]/_}_$rep.jsonl 2> $OUT/${k//[=,]/_}_$rep.err || { echo "$k failed"; tail -3 $OUT/${k//[=,]/_}_$rep.err; exit 1; }
    python3 -c "
import json
for l in open('$OUT/${k//[=,]/_}_$rep.jsonl'):
    d = json.loads(l); print('$k', 'rep$rep', 'N=%d' % d['world'], round(d['kernel_ms'], 4))"
  done
done
