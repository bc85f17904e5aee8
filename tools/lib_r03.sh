#!/bin/bash
# Host path (GPU-planned direct path): parity tests for the host entry points,
# then bench --mode lib lines with per-shard traces at 1/2/4/8 virtual shards.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r03_lib}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -k "${K:-pinned or direct or sharded or alias or host or small or threads or request or golden or kat}" -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/pytest.log | head; exit $rc; }
for spec in ${SPECS:-c5:1 c5:2 c5:4 c5:8 c2:1 c4:1}; do
  cfg=${spec%%:*}; v=${spec##*:}
  MSHA_TRACE=1 MSHA_VIRTUAL_SHARDS=$v timeout -k 10 300 python3 bench.py --mode lib --config $cfg --steps 5 --warmup 2 \
    > $OUT/${cfg}_v$v.json 2> $OUT/${cfg}_v$v.err || { tail -3 $OUT/${cfg}_v$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/${cfg}_v$v.json').read().strip().splitlines()[-1]); s=d['last_call_stats']
print('$cfg v$v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms/call plan', round(s['plan_ms'],2),
      'first launch', [round(x['first_launch_ms'],2) for x in d['last_call_shards']],
      'upload', [round(x['upload_ms'],1) for x in d['last_call_shards']],
      'GB/s', [round(x['h2d_bytes']/x['upload_ms']/1e6,1) for x in d['last_call_shards'] if x['upload_ms']>0],
      'kernel', [round(x['kernel_ms'],1) for x in d['last_call_shards']])"
  grep "\[msha\]" $OUT/${cfg}_v$v.err | tail -40 > $OUT/${cfg}_v$v.trace
done
