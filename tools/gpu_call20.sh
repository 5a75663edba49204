#!/bin/bash
# IPv6 edge registrations + IPv6 bench line + headline bench
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { local s=$1; if [ "$s" -ne 0 ] && [ "$s" -ne 1 ]; then echo "FATAL $2 $s" | tee -a $OUT/steps.log; exit "$s"; fi; echo "$2 exit $s" | tee -a $OUT/steps.log; }
timeout -k 10 300 python -m pytest tests -m gpu -q -p no:cacheprovider -k "ip6 or fullview6 or mixed" > $OUT/pytest_gpu.log 2>&1
s=$?; tail -15 $OUT/pytest_gpu.log; fatal $s pytest_gpu
timeout -k 10 300 python bench.py --workload fullview6 --no-host-path > $OUT/bench_v6.json 2> $OUT/bench_v6.err
s=$?; cat $OUT/bench_v6.json; tail -5 $OUT/bench_v6.err; fatal $s bench_v6
timeout -k 10 300 python bench.py --no-host-path --no-cpu-baseline > $OUT/bench_v4.json 2> $OUT/bench_v4.err
s=$?; cat $OUT/bench_v4.json; fatal $s bench_v4
exit 0
