#!/bin/bash
# A/B: issue-priority rotation between the waves of a SIMD (MSHA_PRIO_ROT=1) vs
# age-ordered arbitration, kernel-resident bench lines, interleaved runs.
set -u
mkdir -p gpurun_out/ab_prio
export TMPDIR=/tmp
for rep in 1 2; do
  for cfg in ${CONFIGS:-c2 c3 ub:196608:640 c5}; do
    for rot in 0 1; do
      tag=$(echo $cfg | tr ':' '_')_rot${rot}_rep${rep}
      MSHA_PRIO_ROT=$rot timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-extra \
        > gpurun_out/ab_prio/$tag.json 2> gpurun_out/ab_prio/$tag.err
      rc=$?; if [ $rc -ne 0 ]; then echo "$tag rc=$rc"; exit $rc; fi
      python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_prio/$tag.json')); print('$tag', round(d['kernel_ms_mean'],5), round(d['roofline']['frac'],4), d['kernel'])"
    done
  done
done
