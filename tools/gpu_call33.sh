#!/bin/bash
# what the one FIB gather and the counters cost (measurement build without any FIB access)
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
for h in "" "-DFIB_HACK_NOGATHER"; do
  make -B -j16 EXTRA_HIPFLAGS="$h" grout_amd/libgrout_hip.so > $OUT/hack_build.log 2>&1 || exit 1
  for w in fullview64 single64; do
    timeout -k 10 200 python tools/variants.py --workload $w --fib16 2 --stats 1,0 --nt 1 --wg 0 --ring 2 --rounds 3 --reps 5 > $OUT/var_ng.jsonl 2> $OUT/var_ng.err
    s=$?; sed "s/^/[$h] /" $OUT/var_ng.jsonl; [ $s -eq 0 ] || exit $s
  done
done
