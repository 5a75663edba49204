#!/bin/bash
# ring geometry 1 vs 2 against batch size
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python tools/batch_sweep.py --rings 2 --rounds 4 --reps 8 --log2 10,12,14,16,18,20 > $OUT/batch_ring12.jsonl 2> $OUT/batch_ring12.err
s=$?; cat $OUT/batch_ring12.jsonl; tail -2 $OUT/batch_ring12.err; exit $s
