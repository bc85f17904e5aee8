#!/bin/bash
# Round 6: why folded c5's lane kernel leaves two XCDs at ~3 waves per SIMD
# (tools/lane_stamps.py, r06_call4): wave stamps of the folded step under head
# variants -- the product; no late head (MSHA_PLAN_HEAD=0); the late head on the
# cooperative kernel (MSHA_HEAD_CHAIN2=0); a nearly free head (PCT=1); and a build
# whose heads share their CUs at normal priority (-DMSHA_HEAD_NO_EXCL).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_xcd
mkdir -p $OUT
timeout -k 10 300 bash tools/ab_build.sh stamps -DMSHA_LANE_STAMPS > $OUT/build.log 2>&1 || { tail $OUT/build.log; exit 1; }
timeout -k 10 300 bash tools/ab_build.sh stamps_noexcl -DMSHA_LANE_STAMPS -DMSHA_HEAD_NO_EXCL >> $OUT/build.log 2>&1 \
  || { tail $OUT/build.log; exit 1; }
run() {  # tag lib env...
  local tag=$1 lib=$2; shift 2
  env "$@" RAW_DIR=$OUT/raw_$tag FORMS=c5_folded MSHA_LIB_PATH=/tmp/msha_ab/$lib.so MSHA_ALLOW_FOREIGN_LIB=1 \
    timeout -k 10 300 python -u tools/lane_stamps.py > $OUT/stamps_$tag.jsonl 2> $OUT/stamps_$tag.err \
    || { tail -20 $OUT/stamps_$tag.err; exit 1; }
  python3 tools/stamps_raw.py $OUT/raw_$tag/stamps_c5_folded.npz 10 > $OUT/raw_$tag.txt
  python3 -c "
import json; d = json.loads(open('$OUT/stamps_$tag.jsonl').readline()); l = d['kernels']['lane']
print('$tag', 'step', round(d['step_ms_stamped_build'], 4), 'lane span', l['span_us'], 'busy', round(l['simd_busy_frac'], 3),
      'cyc/wblk', round(l['busy_simd_cycles_per_wave_block']), 'clk', round(l['clock_ghz'], 3))"
}
run base stamps MSHA_X=0
run nohead stamps MSHA_PLAN_HEAD=0
run coophead stamps MSHA_HEAD_CHAIN2=0
run freehead stamps MSHA_PLAN_HEAD_PCT=1
run noexcl stamps_noexcl MSHA_X=0
run base2 stamps MSHA_X=0
