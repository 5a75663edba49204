#!/bin/bash
# A/B prebuilt libgrout_hip.so builds on one box: build/ab/<name>.so for each
# name in LIBS (default "old new"), alternating processes, on one workload.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
cp grout_amd/libgrout_hip.so build/ab/cur.so
for r in 1 2 3; do
  for v in ${LIBS:-old new}; do
    cp build/ab/$v.so grout_amd/libgrout_hip.so
    GR_HIP_AB_OLD=$([ $v = old ] && echo 1 || echo 0) timeout -k 10 200 python tools/variants.py --workload ${WL:-fullview64} --fib16 2 --nt 1 --wg 0 --ring 2 --rounds 3 --reps 5 > $OUT/ab_$v$r.jsonl 2> $OUT/ab.err
    s=$?; echo "$v $r $(cat $OUT/ab_$v$r.jsonl)"; [ $s -eq 0 ] || { cp build/ab/cur.so grout_amd/libgrout_hip.so; exit $s; }
  done
done
cp build/ab/cur.so grout_amd/libgrout_hip.so
