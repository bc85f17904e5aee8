#!/bin/bash
# Round 5: the early head's list (k_fold_longs). CFGS: "LF:DEDUP" pairs --
# LF = MSHA_LONGS_BEFORE_INSERT (1: on the planner's stream before the alias insert;
# 0: beside it on the head's stream), DEDUP = MSHA_LONGS_DEDUP (1: one claim per
# distinct payload of a tile). The planned GPU tests under each, c5_folded slices
# interleaved, then a rocprofv3 timeline of each at N = 8.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05_lf}
CFGS=${CFGS:-"0:0 0:1 1:1"}
mkdir -p $OUT
for c in $CFGS; do
  MSHA_LONGS_BEFORE_INSERT=${c%:*} MSHA_LONGS_DEDUP=${c#*:} timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread -m gpu tests/test_gpu_planned.py > $OUT/t_${c/:/_}.log 2>&1
  rc=$?; echo "tests $c: $(tail -1 $OUT/t_${c/:/_}.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for c in $CFGS; do
    t=${c/:/_}
    MSHA_LONGS_BEFORE_INSERT=${c%:*} MSHA_LONGS_DEDUP=${c#*:} FORMS=c5_folded WORLDS="1 2 8" timeout -k 10 300 \
      python tools/c5_slice.py > $OUT/s_${t}_$rep.jsonl 2> $OUT/s_${t}_$rep.err || exit 1
    python3 -c "
import json
for l in open('$OUT/s_${t}_$rep.jsonl'):
    d = json.loads(l); print('$c', 'rep$rep', 'N=%d' % d['world'], round(d['kernel_ms'], 4))"
  done
done
for c in $CFGS; do
  t=${c/:/_}
  (cd /tmp && MSHA_LONGS_BEFORE_INSERT=${c%:*} MSHA_LONGS_DEDUP=${c#*:} FORMS=c5_folded WORLDS="8" TIMED_STEPS=20 \
    timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/prof_$t -o run \
    -- python3 $GRAFT_REPO_ROOT/tools/c5_slice.py > $GRAFT_REPO_ROOT/$OUT/prof_$t.log 2>&1) || exit 1
  for db in $(find $OUT/prof_$t -name "*.db"); do python3 tools/fold_steps.py $db; done > $OUT/steps_$t.txt
  echo "== $c"; grep -A12 "lane kernel ~0.7" $OUT/steps_$t.txt | grep -E "longs|insert|chain8|tilescan|fill"
done
