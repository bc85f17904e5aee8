#!/bin/bash
# Round 6: the full GPU suite and smoke on the tree's build, then c5_folded bench
# lines (default: work-stealing lane kernel, early fork off) and c5 rank slices.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_call5
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.txt 2>&1 || { tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for rep in 1 2 3; do
  for v in "MSHA_X=1" "MSHA_LANE_WS=0"; do
    tag=$(echo $v | tr '=' '_')
    env $v timeout -k 10 300 python bench.py --config c5_folded --no-cpu-baseline --no-host-api --no-extra \
      > $OUT/bench_${tag}_rep$rep.json 2> $OUT/bench_${tag}_rep$rep.err || { tail $OUT/bench_${tag}_rep$rep.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/bench_${tag}_rep$rep.json'))
print('$v rep$rep', round(d['kernel_ms_mean'], 4), round(d['roofline']['frac'], 4), d['kernel'])"
  done
done
FORMS="c5_folded" WORLDS="1 2 4 8" TIMED_STEPS=20 timeout -k 10 300 python -u tools/c5_slice.py \
  > $OUT/slices.jsonl 2> $OUT/slices.err || { tail $OUT/slices.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/slices.jsonl'):
    d = json.loads(l); print('slice', d['world'], d['form'], round(d['kernel_ms'], 4), d['kernel'])"
