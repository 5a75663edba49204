#!/bin/bash
# node path tests (hand-back, registered frames, graph walks)
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_node_shim.py tests/test_graph_walk.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_node.log 2>&1
s=$?; grep -E "PASS|FAIL|Error|passed|failed|assert" $OUT/pytest_node.log | tail -12; exit $s
