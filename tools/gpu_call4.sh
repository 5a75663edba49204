#!/bin/bash
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { local s=$1; if [ "$s" -ne 0 ] && [ "$s" -ne 1 ]; then echo "FATAL $2 $s" | tee -a $OUT/steps.log; exit "$s"; fi; echo "$2 exit $s" | tee -a $OUT/steps.log; }
timeout -k 10 120 ./tools/ceiling > $OUT/ceiling.jsonl 2>&1
fatal $? ceiling
cat $OUT/ceiling.jsonl
timeout -k 10 300 python tools/variants.py --workload single64 --staging 0,1 --stats 1,0 --wg 0,4 --rounds 5 > $OUT/variants_single.jsonl 2> $OUT/variants.err
fatal $? variants_single
cat $OUT/variants_single.jsonl
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -k "mirror or golden" > $OUT/pytest_gpu.log 2>&1
fatal $? pytest_gpu
tail -5 $OUT/pytest_gpu.log
exit 0
