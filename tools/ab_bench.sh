#!/bin/bash
# A/B prebuilt libgrout_hip.so builds (build/ab/<name>.so, LIBS="a b ...") on
# sustained bench runs (STEPS timed after WARMUP), alternating processes.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
cp grout_amd/libgrout_hip.so build/ab/cur.so
for r in ${ROUNDS:-1 2}; do
  for v in $LIBS; do
    cp build/ab/$v.so grout_amd/libgrout_hip.so
    timeout -k 10 300 python bench.py --steps ${STEPS:-500} --warmup ${WARMUP:-50} --no-cpu-baseline --no-host-path > $OUT/abb_$v$r.json 2> $OUT/abb.err
    s=$?; python -c "import json; d=json.load(open('$OUT/abb_$v$r.json')); print('$v $r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
    [ $s -eq 0 ] || { cp build/ab/cur.so grout_amd/libgrout_hip.so; tail -3 $OUT/abb.err; exit $s; }
  done
done
cp build/ab/cur.so grout_amd/libgrout_hip.so
