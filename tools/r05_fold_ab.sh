#!/bin/bash
# Round 5: the folded planner's kernels (k_fold_insert / k_fold_tilemax
# with vector loads, the early head's list in tilemax, LDS-staged representatives, batched claims). GPU tests of the
# planned path on the new build, then same-box A/B of old vs new on c5 slices
# (tools/ab_slices.sh), then a rocprofv3 kernel summary of the new build's folded c5.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05_fold}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_planned.py > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT/ab VARIANTS="${VARIANTS:-old new}" FORMS="c5_folded" WORLDS="${WORLDS:-1 8}" REPS=${REPS:-2} bash tools/ab_slices.sh || exit 1
cd /tmp && FORMS=c5_folded WORLDS="1 8" TIMED_STEPS=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/c5_slice.py > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; find $OUT/prof -name "*kernel_stats.csv" | head -3; exit $rc
