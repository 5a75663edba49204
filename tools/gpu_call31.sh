#!/bin/bash
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 120 python -X faulthandler tools/graph_debug.py > $OUT/graph_debug.log 2>&1
s=$?; head -60 $OUT/graph_debug.log; exit $s
