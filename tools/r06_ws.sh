#!/bin/bash
# Round 6: the work-stealing lane kernel (k_digest_batch_ws) on planned calls --
# the planned GPU tests, then c5_folded / c5_planned bench lines and c5 rank slices
# with MSHA_LANE_WS=1 / 0 interleaved, and wave stamps of the folded step.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_ws
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_planned.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_planned.txt 2>&1 || { tail -30 $OUT/pytest_planned.txt; exit 1; }
tail -1 $OUT/pytest_planned.txt
for rep in 1 2; do
  for ws in 1 0; do
    for cfg in c5_folded c5_planned; do
      MSHA_LANE_WS=$ws timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-host-api --no-extra \
        > $OUT/bench_${cfg}_ws${ws}_rep$rep.json 2> $OUT/bench_${cfg}_ws${ws}_rep$rep.err \
        || { tail $OUT/bench_${cfg}_ws${ws}_rep$rep.err; exit 1; }
      python3 -c "
import json; d = json.load(open('$OUT/bench_${cfg}_ws${ws}_rep$rep.json'))
print('$cfg ws=$ws rep$rep', round(d['kernel_ms_mean'], 4), round(d['roofline']['frac'], 4), d['kernel'])"
    done
  done
done
for ws in 1 0; do
  MSHA_LANE_WS=$ws FORMS="c5_folded c5_planned" WORLDS="2 8" TIMED_STEPS=20 timeout -k 10 300 python -u tools/c5_slice.py \
    > $OUT/slices_ws$ws.jsonl 2> $OUT/slices_ws$ws.err || { tail $OUT/slices_ws$ws.err; exit 1; }
  python3 -c "
import json
for l in open('$OUT/slices_ws$ws.jsonl'):
    d = json.loads(l); print('slice ws=$ws', d['world'], d['form'], round(d['kernel_ms'], 4))"
done
timeout -k 10 300 bash tools/ab_build.sh stamps -DMSHA_LANE_STAMPS > $OUT/build.log 2>&1 || { tail $OUT/build.log; exit 1; }
RAW_DIR=$OUT/raw FORMS="c5_folded c5_planned" MSHA_LIB_PATH=/tmp/msha_ab/stamps.so MSHA_ALLOW_FOREIGN_LIB=1 \
  timeout -k 10 300 python -u tools/lane_stamps.py > $OUT/stamps.jsonl 2> $OUT/stamps.err || { tail -20 $OUT/stamps.err; exit 1; }
python3 tools/stamps_raw.py $OUT/raw/stamps_c5_folded.npz 10
