#!/bin/bash
# Round 6: the zero-copy latency path -- its GPU tests, then
# tools/latency with zero-copy on / off and the eight-lane small kernel on / off,
# interleaved -- and the wave stamps without the contended counter (kernels.hip:
# each wave's record at a fixed slot).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_call3
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "small or kat or golden or each_length" > $OUT/pytest_small.txt 2>&1 || { tail -30 $OUT/pytest_small.txt; exit 1; }
tail -1 $OUT/pytest_small.txt
for rep in 1 2; do
  for v in "zc" "copy" "copy2"; do
    case $v in
      zc) env="" ;;
      copy) env="MSHA_SMALL_ZC_BYTES=0" ;;
      copy2) env="MSHA_SMALL_ZC_BYTES=0 MSHA_SMALL_CHAIN8=0" ;;
    esac
    env $env timeout -k 10 240 ./tools/latency > $OUT/latency_${v}_rep$rep.jsonl 2> $OUT/latency_${v}_rep$rep.err \
      || { tail $OUT/latency_${v}_rep$rep.err; exit 1; }
  done
done
for f in $OUT/latency_*_rep1.jsonl; do echo "== $f"; python3 tools/latency_table.py $f | head -12; done
timeout -k 10 300 bash tools/ab_build.sh stamps -DMSHA_LANE_STAMPS > $OUT/build_stamps.log 2>&1 || { tail $OUT/build_stamps.log; exit 1; }
RAW_DIR=$OUT/raw MSHA_LIB_PATH=/tmp/msha_ab/stamps.so MSHA_ALLOW_FOREIGN_LIB=1 timeout -k 10 300 python -u tools/lane_stamps.py \
  > $OUT/stamps.jsonl 2> $OUT/stamps.err || { tail -20 $OUT/stamps.err; exit 1; }
