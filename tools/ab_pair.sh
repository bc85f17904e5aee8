#!/bin/bash
# Same-box A/B of k_digest_chain2 with a barrier per block ($AB_DIR/nopair.so,
# MSHA_CHAIN2_PAIR=0) or per pair of blocks ($AB_DIR/pair.so): one 1,427-block
# chain (tools/chain2_anatomy_f3 / _f4: kernel time), the chain-kernel tests on
# the pair build, then c5 rank slices interleaved.
set -u
OUT=${OUT:-gpurun_out/pair}
mkdir -p $OUT
for f in f3 f4; do timeout -k 10 60 ./tools/chain2_anatomy_$f > $OUT/anat_$f.jsonl || exit 1; echo "$f $(cut -c1-120 $OUT/anat_$f.jsonl)"; done
export MSHA_LIB_PATH=${AB_DIR:-/tmp/msha_ab}/pair.so MSHA_ALLOW_FOREIGN_LIB=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_planned.py \
  tests/test_gpu_host_head.py tests/test_gpu_policies.py tests/test_gpu_fuzz.py > $OUT/t.log 2>&1
rc=$?; tail -1 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT/ab VARIANTS="nopair pair" FORMS="c5_folded c5_planned" WORLDS="1 2 8" REPS=2 bash tools/ab_slices.sh
