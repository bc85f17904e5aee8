#!/bin/bash
# Round 6: wave stamps of the folded step with the insert-listed early head
# (MSHA_INSERT_LIST=1) against the default -- where does its lane kernel lose ~300 us?
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06_il_stamps}
mkdir -p $OUT
timeout -k 10 300 bash tools/ab_build.sh stamps -DMSHA_LANE_STAMPS > $OUT/build.log 2>&1 || { tail $OUT/build.log; exit 1; }
for e in MSHA_X=1 MSHA_INSERT_LIST=1; do
  tag=$(echo $e | tr '=' '_')
  env $e RAW_DIR=$OUT/raw_$tag FORMS=c5_folded MSHA_LIB_PATH=/tmp/msha_ab/stamps.so MSHA_ALLOW_FOREIGN_LIB=1 \
    timeout -k 10 300 python -u tools/lane_stamps.py > $OUT/stamps_$tag.jsonl 2> $OUT/stamps_$tag.err \
    || { tail -20 $OUT/stamps_$tag.err; exit 1; }
  python3 tools/stamps_raw.py $OUT/raw_$tag/stamps_c5_folded.npz 10 > $OUT/raw_$tag.txt
  python3 -c "
import json; d = json.loads(open('$OUT/stamps_$tag.jsonl').readline()); l = d['kernels']['lane']
print('$tag', 'step', round(d['step_ms_stamped_build'], 4), 'lane span', l['span_us'], 'busy', round(l['simd_busy_frac'], 3),
      'cyc/wblk', round(l['busy_simd_cycles_per_wave_block']), 'clk', round(l['clock_ghz'], 3), 'wave_blocks', l['wave_blocks'])"
  cat $OUT/raw_$tag.txt
done
