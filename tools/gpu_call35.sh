#!/bin/bash
# host path: staged copies vs zero-copy kernel, parity then rates
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "host_memory" > $OUT/pytest_host.log 2>&1
s=$?; grep -E "PASS|FAIL|Error|passed|failed" $OUT/pytest_host.log | head -20; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python tools/host_path_ab.py > $OUT/host_ab.jsonl 2> $OUT/host_ab.err
s=$?; cat $OUT/host_ab.jsonl; tail -3 $OUT/host_ab.err; exit $s
