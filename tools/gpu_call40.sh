#!/bin/bash
# config 4 with whole frames resident in mbuf-like slots: 2240 B (grout's
# mempool object) and 2048 B (a power of two)
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
for slot in 2240 2048; do
  timeout -k 10 400 python bench.py --workload imix_frames --slot $slot --no-cpu-baseline --no-host-path > $OUT/bench_imix_frames_$slot.json 2> $OUT/bench_imix_frames.err
  s=$?; cat $OUT/bench_imix_frames_$slot.json; tail -1 $OUT/bench_imix_frames.err; [ $s -eq 0 ] || exit $s
done
