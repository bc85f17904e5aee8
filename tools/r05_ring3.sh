#!/bin/bash
# Round 5: the ring chain8 (g4b) against the pair form (head) alone, with 1, 16
# and 112 messages of 1,427 blocks (one message, one full workgroup, seven).
set -u
OUT=${OUT:-gpurun_out/r05_ring3}
mkdir -p $OUT
for rep in 1 2; do
  for m in 1 16 112; do
    for v in ${ANAT:-head g4b}; do
      timeout -k 10 60 tools/chain8_anatomy_$v 1427 8 $m > $OUT/anat_${v}_${m}_$rep.json || { echo "anatomy $v failed"; exit 1; }
      python3 -c "
import json; d = json.load(open('$OUT/anat_${v}_${m}_$rep.json'))
print('$v', 'M=$m', $rep, d['kernel_ms'])"
    done
  done
done
