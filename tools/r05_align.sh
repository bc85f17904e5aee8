#!/bin/bash
# Round 5 probe: the folded c5 lane kernel's HBM traffic and clock with the arena
# as packed (16-byte aligned) and with owned payloads 128-byte aligned
# (tools/align_probe.py): timing, then PMC passes (FETCH_SIZE; clock and VALU).
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05_align}
mkdir -p $OUT
timeout -k 10 500 python tools/align_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -5 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
for a in 16 128; do
  for pass in fetch sq; do
    ctr=FETCH_SIZE; [ $pass = sq ] && ctr="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
    (cd /tmp && LAYOUTS=$a LOG_N=22 TIMED_STEPS=3 timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $ctr --output-format csv \
      -d $GRAFT_REPO_ROOT/$OUT/pmc_${a}_$pass -o run -- python3 $GRAFT_REPO_ROOT/tools/align_probe.py > $GRAFT_REPO_ROOT/$OUT/pmc_${a}_$pass.log 2>&1)
    rc=$?; echo "pmc $a $pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python3 - <<'PY'
import csv, glob, collections
for a in (16, 128):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for pas in ("fetch", "sq"):
        for f in glob.glob(f"gpurun_out/r05_align/pmc_{a}_{pas}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_digest_batch<2>" in r["Kernel_Name"]:
                    vals[r["Counter_Name"]][(pas, int(r["Dispatch_Id"]))] += float(r["Counter_Value"])
    print(a, {k: (len(v), sum(v.values()) / len(v)) for k, v in vals.items()})
PY
