#!/bin/bash
# Round 5: the ring chain8 with double-buffered producer loads (c8g4b) against the
# committed pair form (check): one chain alone (anatomy), in situ (c5_folded N = 8
# rocprofv3 timelines), the planned and fuzz GPU tests, then c5_folded slices A/B.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05_ring2}
mkdir -p $OUT
for rep in 1 2; do
  for v in head g4b; do
    timeout -k 10 60 tools/chain8_anatomy_$v 1427 8 > $OUT/anat_${v}_$rep.json || { echo "anatomy $v failed"; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/anat_${v}_$rep.json'))
print('$v', $rep, d['kernel_ms'], d['us_per_block'])"
  done
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_planned.py tests/test_gpu_fuzz.py > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT/prof VARIANTS="check c8g4b" bash tools/r05_ring_prof.sh 2>&1 | grep -E "==|chain8|kernel_ms" || exit 1
OUT=$OUT/ab VARIANTS="check c8g4b" FORMS="c5_folded" WORLDS="1 2 8" REPS=2 bash tools/ab_slices.sh
