#!/bin/bash
# Round 5: the insert's tile prefix by decoupled look-back (MSHA_FOLD_LOOKBACK=1,
# default) against the prefix kernels before the insert (0): planned and fuzz GPU
# tests under both, c5_folded slices interleaved, rocprofv3 timelines (N = 1, 8).
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05_lb}
mkdir -p $OUT
for lb in 1 2; do
  MSHA_FOLD_LOOKBACK=$lb timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_planned.py tests/test_gpu_fuzz.py > $OUT/t_$lb.log 2>&1
  rc=$?; echo "tests lb=$lb: $(tail -1 $OUT/t_$lb.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for lb in 0 1; do
    MSHA_FOLD_LOOKBACK=$lb FORMS=c5_folded WORLDS="1 2 8" timeout -k 10 300 python tools/c5_slice.py > $OUT/s_${lb}_$rep.jsonl 2> $OUT/s_${lb}_$rep.err || exit 1
    python3 -c "
import json
for l in open('$OUT/s_${lb}_$rep.jsonl'):
    d = json.loads(l); print('lb=$lb', 'rep$rep', 'N=%d' % d['world'], round(d['kernel_ms'], 4))"
  done
done
for lb in 0 1; do
  (cd /tmp && MSHA_FOLD_LOOKBACK=$lb FORMS=c5_folded WORLDS="1 8" TIMED_STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace \
    -d $GRAFT_REPO_ROOT/$OUT/prof_$lb -o run -- python3 $GRAFT_REPO_ROOT/tools/c5_slice.py > $GRAFT_REPO_ROOT/$OUT/prof_$lb.log 2>&1) || exit 1
  for db in $(find $OUT/prof_$lb -name "*.db"); do python3 tools/fold_steps.py $db; done > $OUT/steps_$lb.txt
  echo "== lb=$lb"; grep -A12 -E "lane kernel ~(2.5|0.7)" $OUT/steps_$lb.txt | grep -E "lane kernel|tilemax|tilescan|insert|longs|chain8|scan |digest_batch"
done
