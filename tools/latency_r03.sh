#!/bin/bash
# Per-call latency sweep of the host API (tools/latency.cpp) only, as a table.
set -u
export TMPDIR=/tmp
timeout -k 10 240 ./tools/latency > gpurun_out/${LAT:-latency}.jsonl 2> gpurun_out/${LAT:-latency}.err; rc=$?
python3 tools/latency_table.py gpurun_out/${LAT:-latency}.jsonl
exit $rc
