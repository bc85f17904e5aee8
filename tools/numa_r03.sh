#!/bin/bash
# Striped (mmap + mbind + hipHostRegister) vs hipHostMalloc pinned arenas on the
# direct host path: bench.py --mode lib, 1 GPU, alternating, REPS times.
set -u
export TMPDIR=/tmp
for rep in $(seq ${REPS:-1}); do
for cfg in ${CFGS:-c5 c2}; do
  for stripe in 0 1; do
    o=gpurun_out/numa_${cfg}_s${stripe}_r${rep}
    MSHA_PINNED_STRIPE=$stripe timeout -k 10 150 python bench.py --mode lib --config $cfg --steps ${STEPS:-5} --warmup 2 \
      > $o.json 2> $o.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', 'upload', [round(x['upload_ms'],1) for x in d['last_call_shards']])" $o.json
  done
done
done
