#!/bin/bash
# A/B (round 3): split-chaining hand-off through write-through (sc1) state stores
# and a drained flag (new) vs plain stores + agent release fence (old); then the
# segment cap under the new hand-off; then the split / failure-path tests.
set -u
export TMPDIR=/tmp
VARIANTS="old new" CONFIGS="c3 c3dd ub:200000:4096" REPS=2 bash tools/ab_lib.sh || exit 1
for segs in ${SEGS:-12 16 24}; do
  echo "(segs=$segs)"
  MSHA_SPLIT_SEGS=$segs VARIANTS="new" CONFIGS="c3 c3dd ub:200000:4096" REPS=1 bash tools/ab_lib.sh || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_failure.py -x -q -k "split or c3 or stall or timeout or digest_of_digests" --timeout 120 > gpurun_out/ab_lib/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/ab_lib/pytest.log; exit $rc
