#!/bin/bash
# Differential fuzz tests (tests/test_fuzz.py) on the GPU.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_fuzz.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_fuzz.log 2>&1
s=$?; grep -E "PASS|FAIL|Error|passed|failed|assert" $OUT/pytest_fuzz.log | tail -30; exit $s
