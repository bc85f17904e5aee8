#!/bin/bash
# North-star host path on one box: bench.py --mode lib (one libmirsha context,
# msha_digest_batch per step, PCIe-inclusive) over 1 GPU and over virtual shards
# of it (MSHA_VIRTUAL_SHARDS: the multi-GPU code path -- per-shard streams,
# partition by blocks, compacted direct uploads, per-shard gather threads), plus
# the --gpus N self-spawn of the kernel-resident bench (both ranks on GPU 0).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/lib
mkdir -p $OUT
run() {  # tag, env, args...
  local tag=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py "$@" > $OUT/$tag.json 2> $OUT/$tag.err
  local rc=$?; echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/$tag.err; exit $rc; }
  python3 - $OUT/$tag.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sh = d.get("last_call_shards", [])
print(f"  value {d['value']/1e6:.1f} M/s  {d.get('gbps_hashed', 0):.1f} GB/s  ms/step {d['ms_per_step']:.2f}  n_gpus {d['n_gpus']}  "
      f"h2d {[round(s['h2d_payload_bytes']/1e6, 1) for s in sh]} MB  gather {[(round(s['gather_begin_ms'],1), round(s['gather_end_ms'],1)) for s in sh]}")
PY
}
for cfg in ${CONFIGS:-c2 c5}; do
  for shards in 1 2 4; do
    run ${cfg}_pinned_v$shards MSHA_VIRTUAL_SHARDS=$shards --mode lib --config $cfg --steps 5 --warmup 2
    run ${cfg}_pageable_v$shards MSHA_VIRTUAL_SHARDS=$shards --mode lib --config $cfg --steps 5 --warmup 2 --pageable
  done
done
env timeout -k 10 300 python3 bench.py --gpus 2 --share-device --steps 20 --warmup 5 --no-cpu-baseline > $OUT/spawn2.json 2> $OUT/spawn2.err
rc=$?; echo "spawn2 rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/spawn2.err; exit $rc; }
python3 -c "import json; d=json.loads(open('$OUT/spawn2.json').read().strip().splitlines()[-1]); print('  spawn2 n_gpus', d['n_gpus'], 'value', d['value'])"
