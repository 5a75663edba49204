#!/bin/bash
# Long differential fuzz sweep on the GPU (tools/fuzz_sweep.py).
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u tools/fuzz_sweep.py --seeds ${SEEDS:-300} > $OUT/fuzz_sweep.log 2>&1
s=$?; tail -20 $OUT/fuzz_sweep.log; exit $s
