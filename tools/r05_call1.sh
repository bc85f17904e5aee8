set -u
mkdir -p gpurun_out/r05_chain
timeout -k 10 60 ./tools/round_issue_microbench > gpurun_out/r05_chain/rounds.jsonl || exit 1
VARIANTS="old new9" CONFIGS="c4" REPS=2 BENCH_ARGS="--no-host-api" bash tools/ab_lib.sh || exit 1
VARIANTS="new7 new9" REPS=2 bash tools/r05_fold_ab.sh || exit 1
python tools/fold_steps.py gpurun_out/r05_fold/prof/run_results.db > gpurun_out/r05_fold/steps.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "c4 or staged or pinned_direct" > gpurun_out/r05_chain/t_c4.log 2>&1; rc=$?; tail -2 gpurun_out/r05_chain/t_c4.log; exit $rc
