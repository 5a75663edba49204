#!/bin/bash
# non-headline bench lines: config 2 (one route), config 4 (IMIX), IPv6 view
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
for w in single64 imix fullview6; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $OUT/bench_$w.json 2> $OUT/bench_$w.err
  s=$?; cat $OUT/bench_$w.json; tail -2 $OUT/bench_$w.err; [ $s -eq 0 ] || exit $s
done
