set -u
mkdir -p gpurun_out/ab_coop
timeout -k 10 600 python -u -m pytest tests/test_gpu_policies.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_coop/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ab_coop/pytest.log; [ $rc -ne 0 ] && exit $rc
for cfg in ${CFGS:-c4 ub:16384:65536 ub:1024:1048576 ub:4096:16384 ub:2000:512 ub:32768:4096 ub:32768:512}; do
  for pol in lane coop; do
    timeout -k 10 300 python bench.py --config $cfg --policy $pol --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_coop/$(echo $cfg | tr ':' '_')_$pol.json 2>gpurun_out/ab_coop/err.log; rc=$?
    [ $rc -ne 0 ] && { echo "$cfg $pol rc=$rc"; tail -3 gpurun_out/ab_coop/err.log; [ $rc -ge 124 ] && exit $rc; continue; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_coop/$(echo $cfg | tr ':' '_')_$pol.json')); print('$cfg', '$pol', round(d['value']/1e6,3), 'Mdig/s', round(d['kernel_ms_mean'],4), 'ms', 'frac', round(d['roofline']['frac'],4))"
  done
done
