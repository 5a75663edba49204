#!/bin/bash
# A/B of library builds (build/ab/<name>.so, LIBS) on the hand-back's CPU
# cost (tools/apply_cost.py), alternating processes, cold (1M packets) and
# L3-hot (2 batches) mbufs.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
for r in 1 2; do
  for v in ${LIBS:-base}; do
    for cfg in "--pkts 1048576" "--pkts 30720"; do
      timeout -k 10 120 python -u tools/apply_cost.py --lib build/ab/$v.so --reps 3 $cfg >> $OUT/ab_apply.jsonl 2>> $OUT/ab_apply.err || exit 1
    done
  done
done
