#!/bin/bash
# Round 6, first GPU call: the product build's GPU suite, then the wave-stamp
# diagnostic on a variant built here on the box (never the
# product library), then the latency path with the eight-lane chain on / off
# (VERDICT r5 item 6). Every GPU step has its own time limit; the first failure
# ends the script.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_call1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.txt 2>&1 || { tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
timeout -k 10 300 bash tools/ab_build.sh stamps -DMSHA_LANE_STAMPS > $OUT/build_stamps.log 2>&1 || { tail $OUT/build_stamps.log; exit 1; }
MSHA_LIB_PATH=/tmp/msha_ab/stamps.so MSHA_ALLOW_FOREIGN_LIB=1 timeout -k 10 300 python -u tools/lane_stamps.py \
  > $OUT/stamps.jsonl 2> $OUT/stamps.err || { tail -20 $OUT/stamps.err; exit 1; }
for v in 1 0 1 0; do
  MSHA_SMALL_CHAIN8=$v timeout -k 10 240 ./tools/latency > $OUT/latency_chain8_$v.jsonl 2> $OUT/latency_chain8_$v.err \
    || { tail $OUT/latency_chain8_$v.err; exit 1; }
  cp $OUT/latency_chain8_$v.jsonl $OUT/latency_chain8_${v}_$RANDOM.jsonl
done
python3 tools/latency_table.py $OUT/latency_chain8_1.jsonl
python3 tools/latency_table.py $OUT/latency_chain8_0.jsonl
