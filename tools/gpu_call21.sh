#!/bin/bash
# in-place narrow stores: parity + A/B against out-of-place and whole-line stores
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { local s=$1; if [ "$s" -ne 0 ] && [ "$s" -ne 1 ]; then echo "FATAL $2 $s" | tee -a $OUT/steps.log; exit "$s"; fi; echo "$2 exit $s" | tee -a $OUT/steps.log; }
timeout -k 10 300 python -m pytest tests -m gpu -q -p no:cacheprovider -k "store_width or in_place or golden or corpus" > $OUT/pytest_gpu.log 2>&1
s=$?; tail -15 $OUT/pytest_gpu.log; fatal $s pytest_gpu
for w in fullview64 single64; do
timeout -k 10 300 python tools/variants.py --workload $w --fib16 1 --nt 1 --wg 0 --place out,in,infull --rounds 5 --reps 5 > $OUT/var_$w.jsonl 2> $OUT/var_$w.err
s=$?; cat $OUT/var_$w.jsonl; tail -3 $OUT/var_$w.err; fatal $s var_$w
done
exit 0
