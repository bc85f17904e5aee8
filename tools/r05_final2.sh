#!/bin/bash
# Round 5, final evidence at the final code: tools/r05_final.sh (GPU tests, smoke,
# default bench line, rocprof per config), then the c5 rank slices.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05_final2}
export OUT
bash tools/r05_final.sh || exit $?
FORMS="c5 c5_planned c5_folded" WORLDS="1 2 4 8" timeout -k 10 400 python tools/c5_slice.py > $OUT/c5_slices.jsonl 2> $OUT/c5_slices.err
rc=$?; echo "slices rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json
for l in open('$OUT/c5_slices.jsonl'):
    d = json.loads(l); print(d['world'], d['form'], round(d['kernel_ms'], 3))"
