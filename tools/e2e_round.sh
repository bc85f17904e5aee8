#!/bin/bash
# GPU tests + end-to-end host-path lines (pack + H2D + kernel + D2H) per config.
set -u
OUT=${OUT:-gpurun_out/e2e}
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${TESTS:-1}" == 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
  tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for cfg in ${CONFIGS:-c2 c4 c5}; do
  for mode in ${MODES:-pageable pinned}; do
    extra=""; [ $mode == pinned ] && extra="--pinned"
    timeout -k 10 400 python bench.py --config $cfg --e2e $extra --steps ${BSTEPS:-3} --warmup 1 > $OUT/e2e_${cfg}_$mode.json 2> $OUT/e2e_${cfg}_$mode.err; rc=$?
    [ $rc -ne 0 ] && { echo "$cfg $mode rc=$rc"; tail -3 $OUT/e2e_${cfg}_$mode.err; [ $rc -ge 124 ] && exit $rc; continue; }
    python3 -c "import json; d=json.load(open('$OUT/e2e_${cfg}_$mode.json')); s=d['last_call_stats']; print('$cfg', '$mode', round(d['value']/1e6,2), 'M dig/s', round(d['gbps_hashed'],1), 'GB/s', 'plan', round(s['plan_ms'],1), 'pack', round(s['pack_ms'],1), 'dev', round(s['device_ms'],1), 'total', round(s['total_ms'],1), 'direct', s['direct_calls'])"
  done
done
exit 0
