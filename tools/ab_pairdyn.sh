#!/bin/bash
# The paired barrier only for workgroups whose longest message has >= 64 blocks
# ($AB_DIR/pairdyn.so) against a barrier per block ($AB_DIR/nopair.so): the
# chain-kernel tests, AUTO small launches, c5 rank slices at N = 1 and 8.
set -u
OUT=${OUT:-gpurun_out/pairdyn}
mkdir -p $OUT
export MSHA_LIB_PATH=${AB_DIR:-/tmp/msha_ab}/pairdyn.so MSHA_ALLOW_FOREIGN_LIB=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_planned.py \
  tests/test_gpu_host_head.py tests/test_gpu_policies.py tests/test_gpu_fuzz.py > $OUT/t.log 2>&1
rc=$?; tail -1 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="nopair pairdyn" CONFIGS="ub:8000:8192 ub:256:65536 ub:1024:640" REPS=2 BENCH_ARGS="--no-host-api" bash tools/ab_lib.sh || exit 1
OUT=$OUT/ab VARIANTS="nopair pairdyn" FORMS="c5_folded" WORLDS="1 8" REPS=2 bash tools/ab_slices.sh
