#!/bin/bash
# the grout node in an rte_graph walk, on the GPU
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_graph_walk.py tests/test_node_shim.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_graph.log 2>&1
s=$?; tail -30 $OUT/pytest_graph.log; exit $s
