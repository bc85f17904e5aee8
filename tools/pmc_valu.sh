#!/bin/bash
# PMC passes per config (separate rocprofv3 runs, --kernel-trace + --pmc only):
#   sq    : VALU/SALU instruction counts, VALU-active and wave cycles, waits, clock (GRBM)
#   sq2   : INT32 VALU instructions, integer ops, VALU thread-cycles, SALU cycles, LDS instrs
#   fetch : FETCH_SIZE        write : WRITE_SIZE   (HBM bytes, gfx950 recipe)
#   ifetch: instruction cache (SQC_ICACHE_*), instruction-issue waits, instruction fetches
# -> gpurun_out/pmc/<cfg>_<pass>/run_counter_collection.csv; summarise with
#    python3 tools/pmc_summary.py gpurun_out/pmc profiles/r04_pmc.json
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
prof() {  # name, counters, cmd...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $OUT/$name -o run -- "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0
}
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
SQ2="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_IOPS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
IF="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH SQ_INSTS_VALU GRBM_GUI_ACTIVE"
PASSES=${PASSES:-sq sq2 fetch write}
has() { [[ " $PASSES " == *" $1 "* ]]; }
# FETCH_SIZE calibration of this box (tools/traffic_calib, built on the CPU side)
if has fetch && [ -x tools/traffic_calib ] && [ -z "${NO_CALIB:-}" ]; then
  prof calib_fetch FETCH_SIZE ./tools/traffic_calib
fi
for spec in ${SPECS:-c2:auto c3:auto c3dd:auto c4:auto c5:auto c5_planned:auto c5_folded:auto}; do
  cfg=${spec%%:*}; pol=${spec##*:}; arg=$cfg
  case $cfg in ub_*|u_*) arg=$(echo $cfg | tr '_' ':') ;; esac
  name=${cfg}_${pol}
  cmd="python3 bench.py --config $arg --policy $pol --steps 3 --warmup 1 --no-cpu-baseline --no-extra --no-host-api"
  has sq && prof ${name}_sq "$SQ" $cmd
  has sq2 && prof ${name}_sq2 "$SQ2" $cmd
  has fetch && prof ${name}_fetch FETCH_SIZE $cmd
  has write && prof ${name}_write WRITE_SIZE $cmd
  has ifetch && prof ${name}_ifetch "$IF" $cmd
done
exit 0
