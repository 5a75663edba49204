#!/bin/bash
# Non-headline workloads with calibrated placement (bench.py defaults).
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
for w in single64 imix fullview6 imix_frames; do
  timeout -k 10 400 python bench.py --workload $w --no-host-path > $OUT/bench_$w.json 2> $OUT/bench_$w.err
  s=$?; [ $s -eq 0 ] || { tail -3 $OUT/bench_$w.err; exit $s; }
  python -c "import json; d=json.load(open('$OUT/bench_$w.json')); print('$w', d['value'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'])"
done
