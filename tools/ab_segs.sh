#!/bin/bash
# A/B: split chaining's segment cap (MSHA_SPLIT_SEGS 8 = the earlier cap, 16 = default), c3 and c3dd,
# alternated twice; then the split-chaining parity tests under the default.
set -u
mkdir -p gpurun_out/ab_segs
for r in 1 2; do
  for segs in ${SEGS:-8 16}; do
    for cfg in c3 c3dd; do
      MSHA_SPLIT_SEGS=$segs timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/ab_segs/${cfg}_s${segs}_r$r.json 2> gpurun_out/ab_segs/${cfg}_s${segs}_r$r.err || { echo "$cfg segs=$segs failed"; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/ab_segs/${cfg}_s${segs}_r$r.json')); print('$cfg segs=$segs r$r', round(d['kernel_ms_mean']*1000,2), 'us frac', round(d['roofline']['frac'],4))"
    done
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k split --timeout 120 > gpurun_out/ab_segs/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/ab_segs/pytest.log; exit $rc
