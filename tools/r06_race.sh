#!/bin/bash
# The planner's defensive check (k_fold_scatter resolves the heads): a -DMSHA_FOLD_RACE_TEST build, made
# here on the box and loaded through MSHA_LIB_PATH (never the product library),
# forces an early-head list that misses long lanes; every digest must stay exact.
# A second build without the check (-DMSHA_SCAN_NO_EARLY_CHECK) must FAIL the test.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06_race}
mkdir -p $OUT
timeout -k 10 300 bash tools/ab_build.sh race -DMSHA_FOLD_RACE_TEST > $OUT/build.log 2>&1 || { tail $OUT/build.log; exit 1; }
timeout -k 10 300 bash tools/ab_build.sh race_nocheck -DMSHA_FOLD_RACE_TEST -DMSHA_SCAN_NO_EARLY_CHECK >> $OUT/build.log 2>&1 \
  || { tail $OUT/build.log; exit 1; }
MSHA_LIB_PATH=/tmp/msha_ab/race.so MSHA_ALLOW_FOREIGN_LIB=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_planned.py \
  -m gpu -q -k insert_claims_first --timeout 200 --timeout-method thread > $OUT/check.txt 2>&1
echo "with the check (expected: pass): rc=$?"; tail -1 $OUT/check.txt
MSHA_LIB_PATH=/tmp/msha_ab/race_nocheck.so MSHA_ALLOW_FOREIGN_LIB=1 timeout -k 10 300 python -u -m pytest \
  tests/test_gpu_planned.py -m gpu -q -k insert_claims_first --timeout 200 --timeout-method thread > $OUT/nocheck.txt 2>&1
echo "without the check (expected: fail): rc=$?"; tail -1 $OUT/nocheck.txt
# the tile look-back's give-up path, forced on every third tile (expected: pass)
timeout -k 10 300 bash tools/ab_build.sh giveup -DMSHA_LOOKBACK_GIVEUP_TEST >> $OUT/build.log 2>&1 || { tail $OUT/build.log; exit 1; }
MSHA_LIB_PATH=/tmp/msha_ab/giveup.so MSHA_ALLOW_FOREIGN_LIB=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_planned.py \
  -m gpu -q -k lookback_give_up --timeout 200 --timeout-method thread > $OUT/giveup.txt 2>&1
echo "look-back give-up (expected: pass): rc=$?"; tail -1 $OUT/giveup.txt
