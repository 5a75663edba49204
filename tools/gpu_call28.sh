#!/bin/bash
# FIB format parity + A/B on the default ring
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "kernel_variants or live_fib or full_size" > $OUT/pytest_fmt.log 2>&1
s=$?; tail -15 $OUT/pytest_fmt.log; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python tools/variants.py --workload fullview64 --fib16 2,1,0 --nt 1 --wg 0 --ring 2 --rounds 4 --reps 5 > $OUT/var_fib.jsonl 2> $OUT/var_fib.err
s=$?; cat $OUT/var_fib.jsonl; tail -2 $OUT/var_fib.err; exit $s
