#!/bin/bash
# Same-box A/B of the folded call's early head (MSHA_EARLY_HEAD 0 = the head
# launched after the scan and scatter, 1 = the long payloads listed first and
# started right then) on c5 rank slices, both planned forms, interleaved per rep;
# the planned-path tests first.
set -u
OUT=${OUT:-gpurun_out/early_head}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_planned.py > $OUT/t.log 2>&1
rc=$?; tail -1 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/t.log | head -5; exit $rc; }
for rep in $(seq 1 ${REPS:-2}); do
  for eh in 0 1; do
    MSHA_EARLY_HEAD=$eh FORMS="c5_folded c5_planned" WORLDS="${WORLDS:-1 2 4 8}" timeout -k 10 400 \
      python tools/c5_slice.py > $OUT/eh${eh}_rep$rep.jsonl 2> $OUT/eh${eh}_rep$rep.err || exit $?
    python3 -c "
import json
for l in open('$OUT/eh${eh}_rep$rep.jsonl'):
    d = json.loads(l); print('eh$eh rep$rep N=%d' % d['world'], d['form'], round(d['kernel_ms'], 4))"
  done
done
