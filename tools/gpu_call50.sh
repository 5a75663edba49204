#!/bin/bash
# Placement vs box state: tools/placement_probe.py, then two bench processes.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u tools/placement_probe.py --sets 8 --passes 3 --steps 50 --fib-reloads 4 > $OUT/placement.jsonl 2> $OUT/placement.err || { tail $OUT/placement.err; exit 1; }
tail -3 $OUT/placement.jsonl
