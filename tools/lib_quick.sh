#!/bin/bash
# Quick host-path check: direct/pinned parity tests, then bench --mode lib lines.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/libq
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "pinned or direct or sharded or alias_table or stall" -v --timeout 240 --timeout-method thread > gpurun_out/libq/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/libq/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/libq/pytest.log | head; exit $rc; }
for spec in ${SPECS:-c5:1 c5:2 c5:4 c2:1 c4:1}; do
  cfg=${spec%%:*}; v=${spec##*:}
  MSHA_TRACE=1 MSHA_VIRTUAL_SHARDS=$v timeout -k 10 300 python3 bench.py --mode lib --config $cfg --steps 5 --warmup 2 \
    > gpurun_out/libq/${cfg}_v$v.json 2> gpurun_out/libq/${cfg}_v$v.err || { tail -3 gpurun_out/libq/${cfg}_v$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/libq/${cfg}_v$v.json').read().strip().splitlines()[-1]); print('$cfg v$v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms', [round(s['device_ms'],1) for s in d['last_call_shards']])"
  grep "\[msha\]" gpurun_out/libq/${cfg}_v$v.err | tail -14 > gpurun_out/libq/${cfg}_v$v.trace
done
