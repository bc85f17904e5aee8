#!/bin/bash
# Where does c2 lose vs the bare compression loop? Same total bytes at growing
# message sizes; and c2's exact instruction stream with every lane reading one
# cached message (stride 0: no HBM traffic).
set -u
mkdir -p gpurun_out/anatomy
for rep in 1 2; do
  for cfg in "u:1048576:512" "u:1048576:512:0" "u:524288:1024" "u:262144:2048" "u:131072:4096" "u:32768:16384" "c2"; do
    tag=$(echo $cfg | tr ':' '_')
    timeout -k 10 300 python bench.py --config $cfg --steps 20 --no-cpu-baseline > gpurun_out/anatomy/${tag}_r$rep.json 2>gpurun_out/anatomy/${tag}_r$rep.err
    rc=$?; [ $rc -ge 124 ] && exit $rc
    python3 -c "import json; d=json.load(open('gpurun_out/anatomy/${tag}_r$rep.json')); b=d['config']['blocks_per_gpu']; print('$cfg', 'rep $rep', round(b/d['kernel_ms_mean']/1e6,2), 'Gblocks/s', round(d['kernel_ms_mean'],4), 'ms')" || tail -3 gpurun_out/anatomy/${tag}_r$rep.err
  done
done
