#!/bin/bash
# bench.py with calibrated vs plain batch placement, alternating processes
# (ROUNDS rounds), after the batch_alloc GPU test.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "batch_alloc" -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_balloc.log 2>&1
s=$?; grep -E "PASS|FAIL|Error|passed|failed|assert" $OUT/pytest_balloc.log | tail -8; [ $s -eq 0 ] || exit $s
for r in $(seq ${ROUNDS:-3}); do
  for p in calibrated plain; do
    timeout -k 10 300 python bench.py --placement $p --no-cpu-baseline --no-host-path > $OUT/abp_$p$r.json 2> $OUT/abp.err
    s=$?; [ $s -eq 0 ] || { tail -3 $OUT/abp.err; exit $s; }
    python -c "import json; d=json.load(open('$OUT/abp_$p$r.json')); print(json.dumps({'placement': '$p', 'round': $r, 'value': d['value'], 'kernel_ms_avg': d['roofline']['kernel_ms_avg']}))" | tee -a $OUT/ab_placement.jsonl
  done
done
