#!/bin/bash
set -u
mkdir -p gpurun_out/split
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "split or c3 or c5 or alias or chunked or digest_of" > gpurun_out/split/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/split/pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for sp in 0 1; do
    for cfg in c3 c3dd; do
      MSHA_SPLIT=$([ $sp == 0 ] && echo 0 || echo -1) timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/split/${cfg}_s${sp}_r${rep}.json 2> gpurun_out/split/${cfg}_s${sp}_r${rep}.err; rc=$?
      [ $rc -ne 0 ] && { echo "$cfg s$sp rc=$rc"; tail -3 gpurun_out/split/${cfg}_s${sp}_r${rep}.err; exit $rc; }
      python3 -c "import json; d=json.load(open('gpurun_out/split/${cfg}_s${sp}_r${rep}.json')); print('$cfg split=$sp rep $rep', round(d['kernel_ms_mean'],4), 'ms frac', round(d['roofline']['frac'],4))"
    done
  done
done
