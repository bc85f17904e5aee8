#!/bin/bash
# Same-box A/B of libmirsha builds ($AB_DIR/<variant>.so, tools/ab_build.sh) on c5 per-rank slices
# (tools/c5_slice.py: FORMS, WORLDS), variants interleaved per rep.
#   VARIANTS="old new" FORMS="c5_folded c5_planned" WORLDS="1 8" REPS=2 bash tools/ab_slices.sh
# The last variant listed is left installed in mirbft_amd/.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab_slices}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-old new}; do
    export MSHA_LIB_PATH=${AB_DIR:-/tmp/msha_ab}/$v.so MSHA_ALLOW_FOREIGN_LIB=1 || exit 1
    timeout -k 10 400 python tools/c5_slice.py > $OUT/${v}_rep${rep}.jsonl 2> $OUT/${v}_rep${rep}.err
    rc=$?; if [ $rc -ne 0 ]; then echo "$v rep$rep rc=$rc"; tail -3 $OUT/${v}_rep${rep}.err; exit $rc; fi
    python3 -c "
import json
for l in open('$OUT/${v}_rep${rep}.jsonl'):
    d = json.loads(l); print('$v', 'rep$rep', 'N=%d' % d['world'], d['form'], round(d['kernel_ms'], 4), d['kernel'])"
  done
done
