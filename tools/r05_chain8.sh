#!/bin/bash
# Round 5: the eight-lane head (k_digest_chain8). GPU tests of the planned path on
# the product build first, then same-box A/B of the two-lane head (new9) against the
# eight-lane one (new10) on c5_folded rank slices at N = 1 and 8.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05_chain8}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_planned.py tests/test_gpu_fuzz.py > $OUT/t.log 2>&1
rc=$?; tail -3 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT/ab VARIANTS="${VARIANTS:-new9 new10}" FORMS="c5_folded" WORLDS="${WORLDS:-1 2 8}" REPS=${REPS:-2} bash tools/ab_slices.sh
