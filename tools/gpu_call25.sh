#!/bin/bash
# ring geometry sweep on the headline workload (one process, interleaved rounds)
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python tools/variants.py --workload fullview64 --fib16 1 --nt 1 --wg 0 --ring 2,9,10,11,12,7 --rounds 4 --reps 5 > $OUT/var_ring.jsonl 2> $OUT/var_ring.err
s=$?; cat $OUT/var_ring.jsonl; tail -3 $OUT/var_ring.err; exit $s
