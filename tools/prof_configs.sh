#!/bin/bash
# rocprofv3 kernel summaries of the bench command per config (kernel time vs the bench line's HIP events).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in ${PCFGS:-c3 c4}; do
  rm -rf gpurun_out/prof_$cfg
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$cfg -o run -- python3 bench.py --config $cfg --no-cpu-baseline --no-host-api > gpurun_out/prof_bench_$cfg.log 2>&1 || { echo "rocprof $cfg rc=$?"; exit 1; }
  f=$(find gpurun_out/prof_$cfg -name "*kernel_stats.csv" | head -1); head -3 $f | cut -c1-200
  grep '^{' gpurun_out/prof_bench_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg bench kernel_ms_mean', d['kernel_ms_mean'])"
done
