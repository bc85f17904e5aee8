#!/bin/bash
# Round 5: the planned and fuzz GPU tests under the A/B knobs that change which
# kernels run (the early head on the two-lane kernel; no early head; the
# cooperative head everywhere), each once.
set -u
OUT=${OUT:-gpurun_out/r05_knobs}
mkdir -p $OUT
for k in MSHA_KNOBS_NONE=1 MSHA_HEAD_CHAIN8=0 MSHA_EARLY_HEAD=0 MSHA_HEAD_CHAIN2=0; do
  env $k timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_planned.py tests/test_gpu_fuzz.py > $OUT/${k%%=*}.log 2>&1
  rc=$?; echo "$k: $(tail -1 $OUT/${k%%=*}.log)"; [ $rc -eq 0 ] || exit $rc
done
