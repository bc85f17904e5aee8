#!/bin/bash
# digest-of-digests GPU tests, then c3dd bench (uniform-pad final block on the SALU) x2.
set -u
mkdir -p gpurun_out/ab_dod
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "digest_of_digests or c3_full or batch_digest" --timeout 120 --timeout-method thread > gpurun_out/ab_dod/pytest.log 2>&1 || { tail -30 gpurun_out/ab_dod/pytest.log; exit 1; }
tail -2 gpurun_out/ab_dod/pytest.log
for r in 1 2; do
  for cfg in c3dd c3; do
    timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/ab_dod/${cfg}_r$r.json 2>/dev/null || { echo "$cfg failed"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_dod/${cfg}_r$r.json')); print('$cfg r$r', round(d['kernel_ms_mean']*1000,2), 'us frac', round(d['roofline']['frac'],4))"
  done
done
