#!/bin/bash
# A/B of the kernel load modes (MSHA_LOAD_MODE 0..3), interleaved, per config.
# (Mode 3, LDS-DMA prefetch, was removed after this A/B: profiles/r01_ab_modes/.)
set -u
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for rep in 1 2; do
  for cfg in ${CONFIGS:-c2 c3 c4}; do
    for m in ${MODES:-0 1 2 3}; do
      MSHA_LOAD_MODE=$m timeout -k 10 300 python bench.py --config $cfg --steps 20 --no-cpu-baseline > gpurun_out/ab/${cfg}_m${m}_r${rep}.json 2>/dev/null
      rc=$?; if [ $rc -ne 0 ]; then echo "$cfg m$m rc=$rc"; [ $rc -ge 124 ] && exit $rc; fi
      python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/${cfg}_m${m}_r${rep}.json')); print('$cfg', 'mode $m', 'rep $rep', round(d['value']/1e6,1), 'Mdig/s', round(d['kernel_ms_mean'],4), 'ms', 'frac', round(d['roofline']['frac'],4))"
    done
  done
done
exit 0
