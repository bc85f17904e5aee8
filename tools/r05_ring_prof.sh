#!/bin/bash
# Round 5: the ring chain8 in situ -- rocprofv3 timelines of c5_folded N = 8 slices
# for $AB_DIR/<variant>.so, tools/ab_build.sh (VARIANTS), the early head's kernel time per variant.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05_ringprof}
mkdir -p $OUT
for v in ${VARIANTS:-check c8g4}; do
  export MSHA_LIB_PATH=${AB_DIR:-/tmp/msha_ab}/$v.so MSHA_ALLOW_FOREIGN_LIB=1 || exit 1
  (cd /tmp && FORMS=c5_folded WORLDS="8" TIMED_STEPS=20 timeout -k 10 300 rocprofv3 --kernel-trace \
    -d $GRAFT_REPO_ROOT/$OUT/prof_$v -o run -- python3 $GRAFT_REPO_ROOT/tools/c5_slice.py > $GRAFT_REPO_ROOT/$OUT/prof_$v.log 2>&1)
  rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/prof_$v.log; exit $rc; }
  for db in $(find $OUT/prof_$v -name "*.db"); do python3 tools/fold_steps.py $db; done > $OUT/steps_$v.txt
  echo "== $v"; grep '^{' $OUT/prof_$v.log | cut -c150-260; grep -A12 "lane kernel ~0.7" $OUT/steps_$v.txt
done
