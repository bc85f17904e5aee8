#!/bin/bash
# Round 6 A/B: MSHA_EARLY_ONLY=1 (the early head takes every distinct long payload,
# no late head) against the default -- planned GPU tests under it, c5_folded 3 reps
# interleaved, rank slices both ways, and a kernel trace of one early-only step.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06_early_only}
mkdir -p $OUT
MSHA_EARLY_ONLY=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_planned.py -m gpu -q --timeout 300 \
  --timeout-method thread > $OUT/pytest_planned_early_only.txt 2>&1; tail -1 $OUT/pytest_planned_early_only.txt
for rep in 1 2 3; do
  for e in MSHA_X=1 MSHA_EARLY_ONLY=1; do
    env $e timeout -k 10 300 python bench.py --config c5_folded --no-cpu-baseline --no-host-api --no-extra \
      > $OUT/bench_$(echo $e | tr '=' '_')_rep$rep.json 2>/dev/null || exit 1
    python3 -c "
import json; d = json.load(open('$OUT/bench_$(echo $e | tr '=' '_')_rep$rep.json'))
print('$e rep$rep', round(d['kernel_ms_mean'], 4), round(d['roofline']['frac'], 4), d['kernel'])"
  done
done
for e in MSHA_X=1 MSHA_EARLY_ONLY=1; do
  env $e FORMS=c5_folded timeout -k 10 300 python -u tools/c5_slice.py > $OUT/slices_$(echo $e | tr '=' '_').jsonl \
    2> $OUT/slices.err || { tail $OUT/slices.err; exit 1; }
  python3 -c "
import json
for l in open('$OUT/slices_$(echo $e | tr '=' '_').jsonl'):
    d = json.loads(l); print('$e', d['world'], round(d['kernel_ms'], 4))"
done
rm -rf $OUT/prof
MSHA_EARLY_ONLY=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --config c5_folded --no-cpu-baseline --no-host-api --no-extra > $OUT/prof.log 2>&1 \
  || { tail -5 $OUT/prof.log; exit 1; }
python3 - $OUT/prof/run_kernel_trace.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_fold_insert' in r['Kernel_Name']]
a, b = idx[-3], idx[-2]
t0 = int(rows[a]['Start_Timestamp'])
for r in rows[a - 2:b]:
    s = int(r['Start_Timestamp']) - t0; e = int(r['End_Timestamp']) - t0
    print(f"{s/1e3:9.1f} {e/1e3:9.1f} {(e-s)/1e3:8.1f} q{r['Queue_Id']} {r['Kernel_Name'][:60]}")
PY
