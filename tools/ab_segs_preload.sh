set -u
export TMPDIR=/tmp
for rep in 1 2; do
  for segs in 10 12 14 16; do
    echo "(segs=$segs)"
    MSHA_SPLIT_SEGS=$segs VARIANTS="new" CONFIGS="c3 ub:200000:4096" REPS=1 bash tools/ab_lib.sh || exit 1
  done
done
