#!/bin/bash
# Round 5: the early head's list vs the alias insert's claims. k_fold_longs lists
# the long payloads it claims while k_fold_insert runs beside it; a payload the
# insert claims first is a long lane off the list. MSHA_FOLD_LONGS_SKIP_ODD=1 forces
# that for half the payloads. 1) the build without k_fold_scan's check
# ($AB_DIR/nocheck.so, -DMSHA_SCAN_NO_EARLY_CHECK) on that test: expected to FAIL;
# 2) the tree's build: the planned and fuzz GPU suites; 3) c5_folded slices, A/B.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05_race}
mkdir -p $OUT
export MSHA_LIB_PATH=${AB_DIR:-/tmp/msha_ab}/nocheck.so MSHA_ALLOW_FOREIGN_LIB=1 || exit 1
MSHA_ALLOW_FOREIGN_LIB=1 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_planned.py -k insert_claims_first > $OUT/nocheck.log 2>&1
echo "nocheck rc=$? (1 = the forced race gives wrong digests without the check)"; tail -3 $OUT/nocheck.log
export MSHA_LIB_PATH=${AB_DIR:-/tmp/msha_ab}/check.so MSHA_ALLOW_FOREIGN_LIB=1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_planned.py tests/test_gpu_fuzz.py > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT/ab VARIANTS="${VARIANTS:-new12 check}" FORMS="c5_folded" WORLDS="1 8" REPS=2 bash tools/ab_slices.sh
