#!/bin/bash
# A/B prebuilt libgrout_hip.so builds (build/ab/<name>.so, LIBS="a b ...") on
# bench.py --workload WL, alternating processes, ROUNDS rounds.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
cp grout_amd/libgrout_hip.so build/ab/cur.so
for r in ${ROUNDS:-1 2}; do
  for v in $LIBS; do
    cp build/ab/$v.so grout_amd/libgrout_hip.so
    timeout -k 10 300 python bench.py --workload ${WL:-fullview64} --steps ${STEPS:-100} --warmup ${WARMUP:-10} --no-cpu-baseline --no-host-path > $OUT/abw_$v$r.json 2> $OUT/abw.err
    s=$?; [ $s -eq 0 ] || { cp build/ab/cur.so grout_amd/libgrout_hip.so; tail -3 $OUT/abw.err; exit $s; }
    python -c "import json; d=json.load(open('$OUT/abw_$v$r.json')); print(json.dumps({'lib': '$v', 'workload': '${WL:-fullview64}', 'round': $r, 'value': d['value'], 'kernel_ms_avg': d['roofline']['kernel_ms_avg']}))" | tee -a $OUT/ab_bench_wl.jsonl
  done
done
cp build/ab/cur.so grout_amd/libgrout_hip.so
