#!/bin/bash
# IPv6: parity with the 24-bit first level, then the IPv6 bench line
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "6 or corpus or golden" > $OUT/pytest_v6.log 2>&1
s=$?; grep -E "PASS|FAIL|Error|passed|failed|assert" $OUT/pytest_v6.log | tail -25; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python bench.py --workload fullview6 --no-cpu-baseline --no-host-path > $OUT/bench_fullview6.json 2> $OUT/bench_fullview6.err
s=$?; cat $OUT/bench_fullview6.json; tail -2 $OUT/bench_fullview6.err; exit $s
