#!/bin/bash
# frame-pointer batches: device, registered host memory (node), graph walk
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
true
true
timeout -k 10 300 python tools/host_path_ab.py > $OUT/host_ab.jsonl 2> $OUT/host_ab.err
s=$?; cat $OUT/host_ab.jsonl; tail -3 $OUT/host_ab.err; exit $s
