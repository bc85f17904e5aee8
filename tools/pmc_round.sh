#!/bin/bash
# PMC counter passes (separate rocprofv3 runs, --kernel-trace only besides --pmc).
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
CFG=${PCFG:-c2}
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
for set in "${PMC_SETS[@]:-}"; do :; done
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d gpurun_out/pmc/$name -o run -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum
