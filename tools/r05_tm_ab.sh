#!/bin/bash
# Round 5: what the early head's tile listing costs in k_fold_tilemax
# ($AB_DIR/<variant>.so, tools/ab_build.sh: tm1 = no listing, tm2 = LDS listing without the global
# append, new17 = both). rocprofv3 timeline per variant of c5_folded slices (N = 1, 8).
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05_tm}
mkdir -p $OUT
for v in ${VARIANTS:-new17 tm1 tm2}; do
  export MSHA_LIB_PATH=${AB_DIR:-/tmp/msha_ab}/$v.so MSHA_ALLOW_FOREIGN_LIB=1 || exit 1
  (cd /tmp && FORMS=c5_folded WORLDS="1 8" TIMED_STEPS=5 timeout -k 10 300 rocprofv3 --kernel-trace \
    -d $GRAFT_REPO_ROOT/$OUT/prof_$v -o run -- python3 $GRAFT_REPO_ROOT/tools/c5_slice.py > $GRAFT_REPO_ROOT/$OUT/prof_$v.log 2>&1)
  rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/prof_$v.log; exit $rc; }
  for db in $(find $OUT/prof_$v -name "*.db"); do python3 tools/fold_steps.py $db; done > $OUT/steps_$v.txt
  echo "== $v"; grep '^{' $OUT/prof_$v.log | cut -c1-120
  grep -E "^folded|tilemax|tilescan|k_fold_insert|chain8" $OUT/steps_$v.txt | grep -B1 -A3 "^folded, lane kernel ~(0.7|2.5)" | head -12
done
