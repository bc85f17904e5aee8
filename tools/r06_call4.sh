#!/bin/bash
# Round 6: full GPU suite on the tree's build; the latency path (zero-copy with
# polled completion / with a stream synchronize / copying; larger zero-copy
# limits); the early head forked before the tile prefix (MSHA_EARLY_FORK) on c5
# folded rank slices, interleaved, and one kernel timeline; the wave stamps with
# raw records. Each GPU step has its own limit; the first failure ends the script.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_call4
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.txt 2>&1 || { tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
for rep in 1 2; do
  for v in poll sync copy big; do
    case $v in
      poll) env="MSHA_SMALL_ZC_POLL=1" ;;
      sync) env="MSHA_SMALL_ZC_POLL=0" ;;
      copy) env="MSHA_SMALL_ZC_BYTES=0" ;;
      big) env="MSHA_SMALL_ZC_BYTES=4194304 MSHA_SMALL_ZC_MSGS=4096" ;;
    esac
    env $env timeout -k 10 240 ./tools/latency > $OUT/latency_${v}_rep$rep.jsonl 2> $OUT/latency_${v}_rep$rep.err \
      || { tail $OUT/latency_${v}_rep$rep.err; exit 1; }
  done
done
for f in $OUT/latency_*_rep1.jsonl; do echo "== $f"; python3 tools/latency_table.py $f | grep -E "digest_batch +pinned"; done
for rep in 1 2; do
  for fork in 1 0; do
    MSHA_EARLY_FORK=$fork FORMS=c5_folded WORLDS="1 8" TIMED_STEPS=20 timeout -k 10 300 python -u tools/c5_slice.py \
      > $OUT/slices_fork${fork}_rep$rep.jsonl 2> $OUT/slices_fork${fork}_rep$rep.err || { tail $OUT/slices_fork${fork}_rep$rep.err; exit 1; }
    python3 -c "
import json
for l in open('$OUT/slices_fork${fork}_rep$rep.jsonl'):
    d = json.loads(l); print('fork=$fork rep$rep', d['world'], round(d['kernel_ms'], 4), d['kernel'])"
  done
done
(cd /tmp && MSHA_EARLY_FORK=1 FORMS=c5_folded WORLDS="1 8" TIMED_STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace \
  -d $GRAFT_REPO_ROOT/$OUT/prof_fork1 -o run -- python3 $GRAFT_REPO_ROOT/tools/c5_slice.py > $GRAFT_REPO_ROOT/$OUT/prof_fork1.log 2>&1) \
  || { tail -5 $OUT/prof_fork1.log; exit 1; }
for db in $(find $OUT/prof_fork1 -name "*.db"); do python3 tools/fold_steps.py $db; done > $OUT/steps_fork1.txt
timeout -k 10 300 bash tools/ab_build.sh stamps -DMSHA_LANE_STAMPS > $OUT/build_stamps.log 2>&1 || { tail $OUT/build_stamps.log; exit 1; }
RAW_DIR=$OUT/raw MSHA_LIB_PATH=/tmp/msha_ab/stamps.so MSHA_ALLOW_FOREIGN_LIB=1 timeout -k 10 300 python -u tools/lane_stamps.py \
  > $OUT/stamps.jsonl 2> $OUT/stamps.err || { tail -20 $OUT/stamps.err; exit 1; }
echo stamps done
