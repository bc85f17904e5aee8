#!/bin/bash
# GPU-planned device batches: parity tests, then c5's forms (caller-ordered /
# planned / planned + folded) over the per-rank slices of 1-8 GPUs, then the
# c2 headline (kernel signatures changed: check it did not move).
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/planned}
mkdir -p $OUT
stop() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -ne 0 ] && { echo "stopping after $name"; exit $rc; }; return 0; }
if [[ ${STEPS:-all} == all || $STEPS == *tests* ]]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_planned.py} -m gpu -x -v --timeout 200 --timeout-method thread \
    > $OUT/pytest.log 2>&1; stop $? pytest
  tail -2 $OUT/pytest.log
fi
if [[ ${STEPS:-all} == all || $STEPS == *slices* ]]; then
  FORMS="${FORMS:-c5 c5_planned c5_folded}" timeout -k 10 400 python tools/c5_slice.py > $OUT/slices.jsonl 2> $OUT/slices.err
  stop $? slices
  python3 -c "
import json
for l in open('$OUT/slices.jsonl'):
    d = json.loads(l); print(d['world'], d['form'].ljust(11), round(d['kernel_ms'], 3), 'ms', d['kernel'])"
fi
if [[ ${STEPS:-all} == all || $STEPS == *bench* ]]; then
  timeout -k 10 300 python bench.py --no-host-api --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err; stop $? bench
  python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('c2', round(d['kernel_ms_mean']*1e3,2), 'us frac', round(d['roofline']['frac'],4), {k: (round(v['kernel_ms_mean'],4), round(v['frac'],4)) for k, v in d['extra_configs'].items()})"
fi
