#!/bin/bash
# Same-box A/B of two builds of libmirsha.so ($AB_DIR/<variant>.so, tools/ab_build.sh, built on the
# CPU side beforehand): kernel-resident bench lines, variants interleaved per rep.
#   VARIANTS="old new" CONFIGS="c4" REPS=3 bash tools/ab_lib.sh
# Variants load through MSHA_LIB_PATH; the product library is never touched.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/ab_lib
mkdir -p $OUT
VARIANTS=${VARIANTS:-old new}
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${CONFIGS:-c4}; do
    for v in $VARIANTS; do
      export MSHA_LIB_PATH=${AB_DIR:-/tmp/msha_ab}/$v.so MSHA_ALLOW_FOREIGN_LIB=1 || exit 1
      tag=$(echo $cfg | tr ':' '_')_${v}_rep${rep}
      timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-extra ${BENCH_ARGS:-} \
        > $OUT/$tag.json 2> $OUT/$tag.err
      rc=$?; if [ $rc -ne 0 ]; then echo "$tag rc=$rc"; tail -3 $OUT/$tag.err; exit $rc; fi
      python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['kernel_ms_mean'],5), round(d['roofline']['frac'],4), d['kernel'])"
    done
  done
done
