set -u
OUT=gpurun_out/head_prio; mkdir -p $OUT
for rep in 1 2; do
  for v in "EH=0 PR=1" "EH=1 PR=0" "EH=1 PR=1"; do
    eval $v
    MSHA_EARLY_HEAD=$EH MSHA_HEAD_STREAM_PRIO=$PR FORMS="c5_folded" WORLDS="1 2 8" timeout -k 10 300 python tools/c5_slice.py > $OUT/eh${EH}_pr${PR}_rep$rep.jsonl 2> $OUT/e.err || exit $?
    python3 -c "
import json
print('eh$EH pr$PR rep$rep', [(json.loads(l)['world'], round(json.loads(l)['kernel_ms'], 4)) for l in open('$OUT/eh${EH}_pr${PR}_rep$rep.jsonl')])"
  done
done
