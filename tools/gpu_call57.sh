#!/bin/bash
# Placement spread: one-route FIB (gathers always in L2) against the full view.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
for w in single64 fullview64 single64; do
timeout -k 10 300 python -u tools/placement_probe.py --workload $w --sets 8 --passes 2 --steps 30 > $OUT/placement_$w.jsonl 2> $OUT/placement.err || { tail $OUT/placement.err; exit 1; }
echo $w; grep summary $OUT/placement_$w.jsonl | cut -c1-200
done
