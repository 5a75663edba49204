#!/bin/bash
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_oracle_kat.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_kat.log 2>&1
s=$?; grep -E "PASS|FAIL|Error|passed|failed|assert" $OUT/pytest_kat.log | tail -16; exit $s
