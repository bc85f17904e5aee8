#!/bin/bash
# Round-3 evidence run, part B: PMC passes for the split-chaining configs (c3, c3dd),
# then the host path (bench --mode lib) at 1/2/4/8 virtual shards with traces.
set -u
export TMPDIR=/tmp
SPECS="c3:auto c3dd:auto" PASSES="sq fetch write" bash tools/pmc_valu.sh || exit 1
OUT=gpurun_out/r03_final_lib K=kat bash tools/lib_r03.sh || exit 1
