#!/bin/bash
# Plain stream copy over 8 separate allocations (tools/ceiling_sets.hip),
# then the ring kernel's placement probe in the same call.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 120 ./tools/ceiling_sets > $OUT/ceiling_sets.jsonl 2>&1 || { cat $OUT/ceiling_sets.jsonl; exit 1; }
cat $OUT/ceiling_sets.jsonl
timeout -k 10 300 python -u tools/placement_probe.py --sets 8 --passes 2 --steps 30 > $OUT/placement.jsonl 2> $OUT/placement.err || { tail $OUT/placement.err; exit 1; }
grep summary $OUT/placement.jsonl
