#!/bin/bash
# narrow in-place stores with and without nontemporal hints
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { local s=$1; if [ "$s" -ne 0 ] && [ "$s" -ne 1 ]; then echo "FATAL $2 $s" | tee -a $OUT/steps.log; exit "$s"; fi; echo "$2 exit $s" | tee -a $OUT/steps.log; }
timeout -k 10 300 python tools/variants.py --workload fullview64 --fib16 1 --nt 0,1 --wg 0 --place out,in,infull --rounds 4 --reps 5 > $OUT/var_nt.jsonl 2> $OUT/var_nt.err
s=$?; cat $OUT/var_nt.jsonl; tail -3 $OUT/var_nt.err; fatal $s var_nt
exit 0
