#!/bin/bash
# One GPU-box session: parity tests, smoke, bench lines per config, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a fault/abort/timeout ends the session.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ $rc -ge 124 ]; then echo "FAULT/TIMEOUT in $name: stopping"; exit $rc; fi; }
STEPS=${STEPS:-all}
if [[ $STEPS == all || $STEPS == *tests* ]]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; stop_on_fault $? pytest
  tail -5 gpurun_out/pytest_gpu.log
fi
if [[ $STEPS == all || $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; stop_on_fault $? smoke
  tail -2 gpurun_out/smoke.log
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
  for cfg in ${CONFIGS:-c2 c3 c3dd c4 c5}; do
    extra="--no-extra"; [ $cfg == c2 ] && extra=""
    timeout -k 10 400 python bench.py --config $cfg ${BSTEPS:+--steps $BSTEPS} $extra > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err; stop_on_fault $? bench_$cfg
    cat gpurun_out/bench_$cfg.json
  done
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
  rm -rf gpurun_out/prof
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --config ${PCFG:-c2} --no-cpu-baseline --no-extra --no-host-api > gpurun_out/prof_bench.log 2>&1; stop_on_fault $? rocprof
  find gpurun_out/prof -name "*kernel_stats*" | head -3
  for f in $(find gpurun_out/prof -name "*kernel_stats.csv"); do cat $f; done
fi
if [[ $STEPS == *dist* ]]; then
  # 2-rank rehearsal of the torchrun path on a 1-GPU box (both ranks on GPU 0)
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --share-device --no-cpu-baseline > gpurun_out/bench_dist2.json 2> gpurun_out/bench_dist2.err; stop_on_fault $? dist2
  cat gpurun_out/bench_dist2.json
fi
