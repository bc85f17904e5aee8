#!/bin/bash
# A/B (round 3, experiment): the split-chaining consumer reading the parked state
# with sc1 (L1-bypassing) loads and no agent acquire (sc1ld) vs one agent acquire
# + plain loads (acq), at segment caps 12 and 16; then the split tests under sc1ld,
# three times (every digest checked).
set -u
export TMPDIR=/tmp
for segs in 12 16; do
  echo "(segs=$segs)"
  MSHA_SPLIT_SEGS=$segs VARIANTS="acq sc1ld" CONFIGS="c3 c3dd ub:200000:4096" REPS=2 bash tools/ab_lib.sh || exit 1
done
export MSHA_LIB_PATH=${AB_DIR:-/tmp/msha_ab}/sc1ld.so MSHA_ALLOW_FOREIGN_LIB=1
for r in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_failure.py -x -q -k "split or c3 or stall or timeout or digest_of_digests" --timeout 120 > gpurun_out/ab_lib/pytest_sc1ld_$r.log 2>&1; rc=$?; tail -1 gpurun_out/ab_lib/pytest_sc1ld_$r.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
