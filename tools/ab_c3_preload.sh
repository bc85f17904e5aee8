#!/bin/bash
# A/B (round 3): split chaining's segment waves fetching their first block before
# the handoff wait (new) vs after it (old), and the segment cap with the early
# fetch, on c3 / c3dd and other split shapes. Same box, interleaved.
set -u
export TMPDIR=/tmp
VARIANTS="old new" CONFIGS="c3 c3dd" REPS=2 bash tools/ab_lib.sh || exit 1
for rep in 1 2; do
  for segs in 8 12; do
    echo "(segs=$segs)"
    MSHA_SPLIT_SEGS=$segs VARIANTS="new" CONFIGS="${SEG_CONFIGS:-c3 ub:81920:16384 ub:98304:2048 ub:200000:4096}" REPS=1 bash tools/ab_lib.sh || exit 1
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_failure.py -x -q -k "split or c3 or stall or timeout" --timeout 120 > gpurun_out/ab_lib/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/ab_lib/pytest.log; exit $rc
