#!/bin/bash
# Same-box A/B of k_digest_chain2 round forms (MSHA_CHAIN2_FORM; $AB_DIR/form<N>.so
# and tools/chain2_anatomy_f<N>, built on the CPU side): round microbenchmark,
# per-block anatomy of one 1,427-block chain, the head tests on the first form
# listed, then c5 rank slices at N = 8 interleaved (tools/ab_slices.sh).
#   FORMS_AB="4 3" bash tools/ab_forms.sh
set -u
OUT=${OUT:-gpurun_out/forms}
mkdir -p $OUT
timeout -k 10 60 ./tools/round_issue_microbench > $OUT/rounds.jsonl || exit 1
for f in ${FORMS_AB:-4 3}; do
  timeout -k 10 60 ./tools/chain2_anatomy_f$f > $OUT/anat_f$f.jsonl || exit 1
  echo "form$f $(cut -c1-220 $OUT/anat_f$f.jsonl)"
done
first=${FORMS_AB%% *}
export MSHA_LIB_PATH=${AB_DIR:-/tmp/msha_ab}/form$first.so MSHA_ALLOW_FOREIGN_LIB=1
MSHA_ALLOW_FOREIGN_LIB=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_planned.py \
  tests/test_gpu_host_head.py tests/test_gpu_policies.py tests/test_gpu_fuzz.py > $OUT/t_form$first.log 2>&1
rc=$?; tail -2 $OUT/t_form$first.log; [ $rc -eq 0 ] || exit $rc
V=""; for f in ${FORMS_AB:-4 3}; do V="$V form$f"; done
OUT=$OUT/ab VARIANTS="$V" FORMS="c5_folded c5_planned" WORLDS="8" REPS=${REPS:-2} bash tools/ab_slices.sh
