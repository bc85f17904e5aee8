#!/bin/bash
# Round 5: the early head's list built by the tile prefix (k_fold_tilemax per-tile
# LDS lists, merged and claimed in k_fold_tilescan) instead of k_fold_longs' global
# claims beside the insert. GPU tests of the planned and fuzz paths on the new build,
# same-box A/B of c5_folded slices (VARIANTS), a rocprofv3 timeline of the new build.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05_longs}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_planned.py tests/test_gpu_fuzz.py > $OUT/t.log 2>&1
rc=$?; tail -3 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT/ab VARIANTS="${VARIANTS:-new12 new16}" FORMS="c5_folded" WORLDS="${WORLDS:-1 2 8}" REPS=${REPS:-2} \
  bash tools/ab_slices.sh || exit 1
cd /tmp && FORMS=c5_folded WORLDS="1 8" TIMED_STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace \
  -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/c5_slice.py > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; [ $rc -eq 0 ] || { tail -5 $OUT/prof.log; exit $rc; }
for db in $(find $OUT/prof -name "*.db"); do python3 tools/fold_steps.py $db; done > $OUT/steps.txt
grep -A14 "^folded" $OUT/steps.txt | head -60
