#!/bin/bash
# c3 anatomy: memory vs wave-count effects at 640-B messages.
#   u:N:640:0  every lane hashes one cached message (no HBM stream)
#   u:N:640    N distinct messages, uniform kernel (no split chaining)
#   ub:N:640   N distinct messages through the batch kernel (off/len; split chaining when it applies)
# N = 196608 is exactly 3 waves per SIMD on 256 CUs; 200000 is c3's count.
set -u
mkdir -p gpurun_out/c3_anatomy
for cfg in u:196608:640:0 u:196608:640 ub:196608:640 u:200000:640:0 u:200000:640 ub:200000:640 c3; do
  name=$(echo $cfg | tr ':' '_')
  timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/c3_anatomy/$name.json 2> gpurun_out/c3_anatomy/$name.err || { echo "$cfg failed rc=$?"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c3_anatomy/$name.json')); print('$cfg', round(d['kernel_ms_mean']*1000,2), 'us', round(d['roofline']['frac'],3))"
done
