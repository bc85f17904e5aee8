#!/bin/bash
# Same-box A/B of the head cut's tie-break (MSHA_PLAN_TIEBREAK 0 = round 3's
# smaller head, 1 = the most lane-kernel room) on c5 rank slices, N = 1..8,
# both planned forms, interleaved per rep; then the planned-path tests.
set -u
OUT=${OUT:-gpurun_out/tiebreak}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for tb in 0 1; do
    MSHA_PLAN_TIEBREAK=$tb FORMS="c5_folded c5_planned" WORLDS="${WORLDS:-1 2 4 8}" timeout -k 10 400 \
      python tools/c5_slice.py > $OUT/tb${tb}_rep$rep.jsonl 2> $OUT/tb${tb}_rep$rep.err || exit $?
    python3 -c "
import json
for l in open('$OUT/tb${tb}_rep$rep.jsonl'):
    d = json.loads(l); print('tb$tb rep$rep N=%d' % d['world'], d['form'], round(d['kernel_ms'], 4))"
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_planned.py > $OUT/t.log 2>&1
rc=$?; tail -1 $OUT/t.log; exit $rc
