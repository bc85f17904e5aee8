#!/bin/bash
# HBM traffic per launch from PMC counters, gfx950 recipe (MI355X_MICROARCH.md
# HBM section): FETCH_SIZE and WRITE_SIZE in SEPARATE rocprofv3 passes
# (--kernel-trace + --pmc only), FETCH_SIZE calibrated on a kernel that reads a
# known byte count with the engine's own per-lane pattern (tools/traffic_calib).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/traffic
mkdir -p $OUT
prof() {  # name, counter, cmd...
  local name=$1 ctr=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $OUT/$name -o run -- "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0
}
prof calib_fetch FETCH_SIZE ./tools/traffic_calib
prof calib_write WRITE_SIZE ./tools/traffic_calib
for cfg in ${CONFIGS:-c2 c4}; do
  prof ${cfg}_fetch FETCH_SIZE python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline
  prof ${cfg}_write WRITE_SIZE python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline
done
