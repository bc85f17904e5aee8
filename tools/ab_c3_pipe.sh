#!/bin/bash
# c3's base case with the pipelined lane kernel (kPipe: the next block's schedule
# expanded inside the current block's rounds) at 3 waves per SIMD: c3 as shipped
# (split), c3 unsplit (MSHA_SPLIT=0) with kPair / kPipe, and exactly 3 waves per
# SIMD (196,608 x 640 B) with kPair / kPipe; interleaved reps, one JSON line each.
set -u
OUT=${OUT:-gpurun_out/c3_pipe}
mkdir -p $OUT
run() {  # tag, env..., -- config
  local tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --config $CFG --no-cpu-baseline --no-extra --no-host-api \
    --steps 200 --warmup 20 > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -3 $OUT/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['kernel_ms_mean']*1e3, 2), 'us', d['kernel'], round(d['roofline']['frac'], 4))"
}
for rep in 1 2; do
  CFG=c3 run c3_split_r$rep MSHA_X=0
  CFG=c3 run c3_nosplit_pair_r$rep MSHA_SPLIT=0 MSHA_LOAD_MODE=2
  CFG=c3 run c3_nosplit_pipe_r$rep MSHA_SPLIT=0 MSHA_LOAD_MODE=3
  CFG=ub:196608:640 run u3_pair_r$rep MSHA_LOAD_MODE=2
  CFG=ub:196608:640 run u3_pipe_r$rep MSHA_LOAD_MODE=3
done
