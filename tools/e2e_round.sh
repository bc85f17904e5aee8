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
  timeout -k 10 400 python bench.py --config $cfg --e2e --steps ${BSTEPS:-3} --warmup 1 > $OUT/e2e_$cfg.json 2> $OUT/e2e_$cfg.err; rc=$?
  [ $rc -ne 0 ] && { echo "$cfg rc=$rc"; tail -3 $OUT/e2e_$cfg.err; [ $rc -ge 124 ] && exit $rc; continue; }
  cat $OUT/e2e_$cfg.json
done
exit 0
