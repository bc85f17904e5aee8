#!/bin/bash
# Round 5: where c5_planned's 8-GPU rank slice spends its time. rocprofv3 kernel
# trace of tools/c5_slice.py (FORMS/WORLDS below), then tools/fold_steps.py's
# per-step timeline (each kernel's start and duration from the planner's start).
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05_planned}
mkdir -p $OUT
cd /tmp && FORMS="${FORMS:-c5_planned}" WORLDS="${WORLDS:-8}" TIMED_STEPS=${TIMED_STEPS:-10} \
  timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/prof -o run \
  -- python3 $GRAFT_REPO_ROOT/tools/c5_slice.py > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; [ $rc -eq 0 ] || { tail -20 $OUT/prof.log; exit $rc; }
grep '^{' $OUT/prof.log
for db in $(find $OUT/prof -name "*.db"); do python3 tools/fold_steps.py $db; done > $OUT/steps.txt
cat $OUT/steps.txt
