#!/bin/bash
# rocprofv3 kernel trace of the host path (bench --mode lib): per-kernel
# durations of the GPU lane planner (plan.hip) and the hash kernels.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=${OUT:-gpurun_out/r03_prof_lib}
mkdir -p $OUT
for spec in ${SPECS:-c5:1 c5:8}; do
  cfg=${spec%%:*}; v=${spec##*:}
  MSHA_VIRTUAL_SHARDS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${cfg}_v$v -o run -- \
    python3 bench.py --mode lib --config $cfg --steps 3 --warmup 1 > $OUT/${cfg}_v$v.json 2> $OUT/${cfg}_v$v.err || { tail -5 $OUT/${cfg}_v$v.err; exit 1; }
  echo "== $cfg v$v"; python3 tools/prof_db_summary.py $(find $OUT/${cfg}_v$v -name "*.db" | head -1) 0 | head -12
done
