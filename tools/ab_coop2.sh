#!/bin/bash
# A/B of the batch kernels around one wave per SIMD: lane vs cooperative
# latency form (G=2) vs balanced form (G=4). The G=4 form (MSHA_COOP_G) was
# removed after this A/B (profiles/r01_ab_coop2/: no gain over the lane kernel).
set -u
OUT=${OUT:-gpurun_out/ab_coop2}
mkdir -p $OUT
for rep in 1 2; do
for cfg in ${CFGS:-c4 ub:49152:65536 ub:40000:16384 ub:32768:4096 ub:65536:4096}; do
  for v in lane coop:2 coop:4; do
    pol=${v%%:*}; g=${v##*:}; [ $pol == lane ] && g=0
    tag=$(echo ${cfg}_${pol}${g} | tr ':' '_')
    MSHA_COOP_G=$g timeout -k 10 300 python bench.py --config $cfg --policy $pol --steps 10 --warmup 2 --no-cpu-baseline > $OUT/${tag}_r$rep.json 2>$OUT/err.log; rc=$?
    [ $rc -ne 0 ] && { echo "$tag rc=$rc"; tail -3 $OUT/err.log; [ $rc -ge 124 ] && exit $rc; continue; }
    python3 -c "import json; d=json.load(open('$OUT/${tag}_r$rep.json')); print('$cfg', '$v', round(d['kernel_ms_mean'],4), 'ms', 'frac', round(d['roofline']['frac'],4))"
  done
done
done
exit 0
