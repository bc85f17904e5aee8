#!/bin/bash
# A/B: nontemporal payload loads (MSHA_NT=1) vs default, interleaved.
# (The nontemporal variant was removed after this A/B: profiles/r01_ab_nt/.)
set -u
mkdir -p gpurun_out/ab_nt
for rep in 1 2 3; do
  for cfg in c2 c4 c5; do
    for nt in 0 1; do
      MSHA_NT=$nt timeout -k 10 300 python bench.py --config $cfg --steps 20 --no-cpu-baseline > gpurun_out/ab_nt/${cfg}_nt${nt}_r${rep}.json 2>/dev/null
      rc=$?; [ $rc -ge 124 ] && exit $rc
      python3 -c "import json; d=json.load(open('gpurun_out/ab_nt/${cfg}_nt${nt}_r${rep}.json')); print('$cfg nt=$nt rep $rep', round(d['value']/1e6,1), 'Mdig/s', round(d['kernel_ms_mean'],4), 'ms frac', round(d['roofline']['frac'],4))"
    done
  done
done
