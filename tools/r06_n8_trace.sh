#!/bin/bash
# Round 6: the folded N = 8 rank slice's timeline (rocprofv3 kernel trace) -- when the
# early head's chain starts and ends against the planner and the lane kernel.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06_n8_trace}
mkdir -p $OUT
rm -rf $OUT/prof
WORLDS=${WORLDS:-8} FORMS=c5_folded TIMED_STEPS=5 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
  python3 tools/c5_slice.py > $OUT/slice.jsonl 2> $OUT/slice.err || { tail $OUT/slice.err; exit 1; }
cat $OUT/slice.jsonl | cut -c1-300
python3 - $OUT/prof/run_kernel_trace.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_fold_insert' in r['Kernel_Name']]
for a, b in [(idx[-3], idx[-2])]:
    t0 = int(rows[a]['Start_Timestamp'])
    for r in rows[a - 2:b]:
        s = int(r['Start_Timestamp']) - t0; e = int(r['End_Timestamp']) - t0
        print(f"{s/1e3:9.1f} {e/1e3:9.1f} {(e-s)/1e3:8.1f} q{r['Queue_Id']} {r['Kernel_Name'][:60]}")
PY
