#!/bin/bash
# Kernel-only time of the launches a small call makes (n messages, one size),
# lane vs coop policy: how much of a small call's latency is the hash chain itself.
set -u
mkdir -p gpurun_out/small_kernel
for spec in ${SPECS:-ub:1:32 ub:1:512 ub:1:4096 ub:64:512 ub:1024:512}; do
  for pol in lane coop; do
    tag=$(echo $spec | tr ':' '_')_$pol
    timeout -k 10 120 python bench.py --config $spec --policy $pol --steps 200 --warmup 20 --no-cpu-baseline --no-extra \
      > gpurun_out/small_kernel/$tag.json 2> gpurun_out/small_kernel/$tag.err || { echo "$tag failed"; tail -3 gpurun_out/small_kernel/$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/small_kernel/$tag.json')); print('$tag', round(d['kernel_ms_mean']*1e3,2), 'us', d['kernel'])"
  done
done
