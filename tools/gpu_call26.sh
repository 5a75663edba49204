#!/bin/bash
# cost of each FIB gather: measurement builds without the top / chunk gather
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
for h in 0 1 2; do
  make -B -j16 EXTRA_HIPFLAGS=-DFIB_HACK=$h grout_amd/libgrout_hip.so > $OUT/hack_build$h.log 2>&1 || exit 1
  timeout -k 10 200 python tools/variants.py --workload fullview64 --fib16 1 --nt 1 --wg 0 --ring 1,2 --rounds 4 --reps 5 > $OUT/var_hack$h.jsonl 2> $OUT/var_hack$h.err
  s=$?; echo "hack $h"; cat $OUT/var_hack$h.jsonl; [ $s -eq 0 ] || exit $s
done
