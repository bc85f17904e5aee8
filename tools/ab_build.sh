#!/bin/bash
# Builds an A/B or diagnostic variant of libmirsha.so OUTSIDE the package, on the
# machine that will run it (the GPU box: variants never travel with the tree and
# never overwrite mirbft_amd/libmirsha.so):
#   bash tools/ab_build.sh NAME [EXTRA_FLAGS...]   ->  $AB_DIR/NAME.so  (AB_DIR=/tmp/msha_ab)
# Load it with MSHA_LIB_PATH=$AB_DIR/NAME.so MSHA_ALLOW_FOREIGN_LIB=1 (mirbft_amd/_lib.py);
# its msha_build_id() names the extra flags, so tests and bench.py know it is foreign.
set -eu
AB_DIR=${AB_DIR:-/tmp/msha_ab}
name=$1
shift
make -s -j16 -C "$(dirname "$0")/../mirbft_amd/csrc" BUILD="$AB_DIR/$name" OUT="$AB_DIR/$name.so" \
  EXTRA_FLAGS="$*" >&2
echo "$AB_DIR/$name.so"
