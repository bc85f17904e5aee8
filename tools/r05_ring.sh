#!/bin/bash
# Round 5: k_digest_chain8 with a three-group K+W ring and one barrier per
# MSHA_CHAIN8_GROUP blocks (2 / 4 / 8) against the committed pair form: one
# 1,427-block chain alone (tools/chain8_anatomy_*, two reps interleaved), the
# planned and fuzz GPU tests on the tree's build, then c5_folded slices (N = 2, 8).
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05_ring}
mkdir -p $OUT
for rep in 1 2; do
  for v in head g2 g4 g8; do
    timeout -k 10 60 tools/chain8_anatomy_$v 1427 8 > $OUT/anat_${v}_$rep.json || { echo "anatomy $v failed"; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/anat_${v}_$rep.json'))
print('$v', $rep, d['kernel_ms'], d['us_per_block'], d['consumer_compute_ticks_median'], d['consumer_wait_ticks_median'])"
  done
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_planned.py tests/test_gpu_fuzz.py > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT/ab VARIANTS="${VARIANTS:-check c8g4 c8g8}" FORMS="c5_folded" WORLDS="2 8" REPS=2 bash tools/ab_slices.sh
