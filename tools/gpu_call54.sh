#!/bin/bash
# Tile order against the placement spread (tools/placement_probe.py --orders 0,1),
# and the corpus/fullview parity with tile_order 1.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u tools/placement_probe.py --sets 8 --passes 2 --steps 30 --orders 0,1 > $OUT/placement_order.jsonl 2> $OUT/placement.err || { tail $OUT/placement.err; exit 1; }
grep summary $OUT/placement_order.jsonl
