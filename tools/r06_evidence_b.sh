#!/bin/bash
# Round-6 evidence, part B: the PMC passes per config (tools/pmc_valu.sh: separate
# rocprofv3 --kernel-trace --pmc runs), the final wave stamps (c2, c5, c5_folded on
# the tree's code plus stamps), and the latency sweep. Each GPU step has its own
# limit; pmc_valu.sh stops at a timed-out pass.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_evb
mkdir -p $OUT
OUT=$OUT/pmc bash tools/pmc_valu.sh > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
tail -3 $OUT/pmc.log
timeout -k 10 300 bash tools/ab_build.sh stamps -DMSHA_LANE_STAMPS > $OUT/build_stamps.log 2>&1 || { tail $OUT/build_stamps.log; exit 1; }
RAW_DIR=$OUT/raw FORMS="c2 c5 c5_folded" MSHA_LIB_PATH=/tmp/msha_ab/stamps.so MSHA_ALLOW_FOREIGN_LIB=1 \
  timeout -k 10 300 python -u tools/lane_stamps.py > $OUT/stamps.jsonl 2> $OUT/stamps.err || { tail -20 $OUT/stamps.err; exit 1; }
timeout -k 10 240 ./tools/latency > $OUT/latency.jsonl 2> $OUT/latency.err || { tail $OUT/latency.err; exit 1; }
python3 tools/latency_table.py $OUT/latency.jsonl | head -30
