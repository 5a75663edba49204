#!/bin/bash
# after retiring the pipe kernel: parity, bench, batch-size sweep
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { local s=$1; if [ "$s" -ne 0 ] && [ "$s" -ne 1 ]; then echo "FATAL $2 $s" | tee -a $OUT/steps.log; exit "$s"; fi; echo "$2 exit $s" | tee -a $OUT/steps.log; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
s=$?; tail -20 $OUT/pytest_gpu.log; fatal $s pytest_gpu
[ $s -ne 0 ] && exit 1
timeout -k 10 300 python tools/batch_sweep.py > $OUT/batch_sweep.jsonl 2> $OUT/batch_sweep.err
fatal $? batch_sweep
cat $OUT/batch_sweep.jsonl
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
s=$?; cat $OUT/bench.json; fatal $s bench
exit 0
