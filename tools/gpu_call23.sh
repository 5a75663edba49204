#!/bin/bash
# narrow in-place stores: parity, then A/B of placements in one process
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { local s=$1; if [ "$s" -ne 0 ] && [ "$s" -ne 1 ]; then echo "FATAL $2 $s" | tee -a $OUT/steps.log; exit "$s"; fi; echo "$2 exit $s" | tee -a $OUT/steps.log; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "in_place or full_size" > $OUT/pytest_inplace.log 2>&1
s=$?; tail -12 $OUT/pytest_inplace.log; fatal $s pytest_inplace
timeout -k 10 300 python tools/variants.py --workload fullview64 --fib16 1 --nt 1 --wg 0 --ring 1 --place out,in,infull --rounds 5 --reps 5 > $OUT/var_place.jsonl 2> $OUT/var_place.err
s=$?; cat $OUT/var_place.jsonl; tail -3 $OUT/var_place.err; fatal $s var_place
timeout -k 10 300 python tools/variants.py --workload single64 --fib16 1 --nt 1 --wg 0 --ring 1 --place out,in --rounds 3 --reps 5 > $OUT/var_place1.jsonl 2> $OUT/var_place1.err
s=$?; cat $OUT/var_place1.jsonl; tail -3 $OUT/var_place1.err; fatal $s var_place1
exit 0
