#!/bin/bash
# Round 6: the wave-stamp diagnostic on a variant built here on
# the box (never the product library), then the latency path with the eight-lane
# chain on / off. Each GPU step has its own time limit; the
# first failure ends the script.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_call2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_multirank.txt 2>&1 || { tail -30 $OUT/pytest_multirank.txt; exit 1; }
tail -1 $OUT/pytest_multirank.txt
timeout -k 10 300 bash tools/ab_build.sh stamps -DMSHA_LANE_STAMPS > $OUT/build_stamps.log 2>&1 || { tail $OUT/build_stamps.log; exit 1; }
MSHA_LIB_PATH=/tmp/msha_ab/stamps.so MSHA_ALLOW_FOREIGN_LIB=1 timeout -k 10 300 python -u tools/lane_stamps.py \
  > $OUT/stamps.jsonl 2> $OUT/stamps.err || { tail -20 $OUT/stamps.err; exit 1; }
for rep in 1 2; do
  for v in 1 0; do
    MSHA_SMALL_CHAIN8=$v timeout -k 10 240 ./tools/latency > $OUT/latency_chain8_${v}_rep$rep.jsonl \
      2> $OUT/latency_chain8_${v}_rep$rep.err || { tail $OUT/latency_chain8_${v}_rep$rep.err; exit 1; }
  done
done
for f in $OUT/latency_chain8_*.jsonl; do echo "== $f"; python3 tools/latency_table.py $f; done
