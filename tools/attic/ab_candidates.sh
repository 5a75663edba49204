#!/bin/bash
# bench.py with gr_hip_batch_place over CANDS candidates each, alternating processes.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
for r in $(seq ${ROUNDS:-3}); do
  for c in ${CANDS:-6 12}; do
    timeout -k 10 300 python bench.py --candidates $c --no-cpu-baseline --no-host-path > $OUT/abc_$c$r.json 2> $OUT/abc.err
    s=$?; [ $s -eq 0 ] || { tail -3 $OUT/abc.err; exit $s; }
    python -c "import json; d=json.load(open('$OUT/abc_$c$r.json')); print(json.dumps({'candidates': $c, 'round': $r, 'value': d['value'], 'kernel_ms_avg': d['roofline']['kernel_ms_avg']}))" | tee -a $OUT/ab_candidates.jsonl
  done
done
