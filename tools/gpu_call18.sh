#!/bin/bash
# parity (node shim, 9 ring geometries), geometry A/B
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { local s=$1; if [ "$s" -ne 0 ] && [ "$s" -ne 1 ]; then echo "FATAL $2 $s" | tee -a $OUT/steps.log; exit "$s"; fi; echo "$2 exit $s" | tee -a $OUT/steps.log; }
timeout -k 10 700 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
s=$?; tail -30 $OUT/pytest_gpu.log; fatal $s pytest_gpu
[ $s -ne 0 ] && exit 1
timeout -k 10 400 python tools/variants.py --nt 1 --wg 0 --fib16 1 --stats 1 --tile 256 --kernel 2 --ring 1,2,5,6,7,8 --rounds 5 > $OUT/variants.jsonl 2> $OUT/variants.err
fatal $? variants
cat $OUT/variants.jsonl
timeout -k 10 300 python tools/variants.py --workload single64 --nt 1 --wg 0 --fib16 1 --stats 1 --tile 256 --kernel 2 --ring 1,2,6,7,8 --rounds 3 > $OUT/variants_single.jsonl 2>> $OUT/variants.err
fatal $? variants_single
cat $OUT/variants_single.jsonl
exit 0
