#!/bin/bash
# Interleaved A/B of environment-selected kernel variants, per config.
#   VARIANTS="MSHA_X2=0 MSHA_X2=1" CONFIGS="c2 c3" REPS=2 OUT=gpurun_out/ab_x2 bash tools/ab_env.sh
# Each variant is one env assignment (or several joined by ','), e.g. "MSHA_LOAD_MODE=1,MSHA_X2=1".
set -u
OUT=${OUT:-gpurun_out/ab_env}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${CONFIGS:-c2}; do
    for v in ${VARIANTS}; do
      tag=$(echo $v | tr ',=' '__')
      env $(echo $v | tr ',' ' ') timeout -k 10 300 python bench.py --config $cfg --steps ${BSTEPS:-20} --no-cpu-baseline > $OUT/${cfg}_${tag}_r${rep}.json 2> $OUT/${cfg}_${tag}_r${rep}.err
      rc=$?; if [ $rc -ne 0 ]; then echo "$cfg $v rc=$rc"; tail -3 $OUT/${cfg}_${tag}_r${rep}.err; [ $rc -ge 124 ] && exit $rc; continue; fi
      python3 -c "import json; d=json.load(open('$OUT/${cfg}_${tag}_r${rep}.json')); print('$cfg', '$v', 'rep $rep', round(d['value']/1e6,1), 'Mdig/s', round(d['kernel_ms_mean'],4), 'ms', 'frac', round(d['roofline']['frac'],4))"
    done
  done
done
exit 0
