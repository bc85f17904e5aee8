#!/bin/bash
# Pageable arenas: staged direct path (default) vs the gather pipeline
# (MSHA_STAGED_DIRECT=0), bench.py --mode lib --pageable, c2 and c5, 1 GPU.
set -u
export TMPDIR=/tmp
for rep in $(seq ${REPS:-2}); do
for cfg in ${CFGS:-c2 c5}; do
  for st in 1 0; do
    o=gpurun_out/staged_${cfg}_s${st}_r${rep}
    MSHA_STAGED_DIRECT=$st timeout -k 10 200 python bench.py --mode lib --pageable --config $cfg --steps 6 --warmup 2 \
      > $o.json 2> $o.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['last_call_shards'][0]; print(sys.argv[1], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms', d['call_ms'], {k: round(s[k],2) for k in ('gather_ms','upload_ms','kernel_ms','first_launch_ms')})" $o.json
  done
done
done
