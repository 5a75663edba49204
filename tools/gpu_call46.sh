#!/bin/bash
# warm-up length against the measured rate (same box, alternating processes)
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
for kw in "20 5" "200 2000" "20 5" "200 2000" "200 200" "20 5" "200 2000"; do
  set -- $kw
  timeout -k 10 300 python bench.py --steps $1 --warmup $2 --no-cpu-baseline --no-host-path > $OUT/bench_kw.json 2> $OUT/bench_kw.err
  s=$?; python -c "import json; d=json.load(open('$OUT/bench_kw.json')); print('steps $1 warmup $2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"; [ $s -eq 0 ] || exit $s
done
