timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "small or host_path or golden or kat or pinned or length" > gpurun_out/pytest_small.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_small.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_small.log | head -20; exit $rc; }
timeout -k 10 200 ./tools/latency > gpurun_out/latency3.jsonl 2> gpurun_out/latency3.err; rc=$?
python3 tools/latency_table.py gpurun_out/latency3.jsonl
exit $rc
