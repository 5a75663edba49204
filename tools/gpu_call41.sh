#!/bin/bash
# concurrency: two worker queues + control-plane updates; then the full GPU suite
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "concurrent" > $OUT/pytest_conc.log 2>&1
s=$?; grep -E "PASS|FAIL|Error|passed|failed|assert" $OUT/pytest_conc.log | tail -15; [ $s -eq 0 ] || exit $s
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
s=$?; tail -3 $OUT/pytest_gpu.log; exit $s
