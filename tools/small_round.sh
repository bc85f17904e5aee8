#!/bin/bash
# GPU session for the host-API latency work: full -m gpu suite, then the per-call
# latency sweep (tools/latency.cpp) printed as a table.
set -u
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 200 ./tools/latency > gpurun_out/${LAT:-latency}.jsonl 2> gpurun_out/${LAT:-latency}.err; rc=$?
python3 tools/latency_table.py gpurun_out/${LAT:-latency}.jsonl
exit $rc
