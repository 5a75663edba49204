#!/bin/bash
# chunk-gather cost against the chunk table's footprint (measurement builds)
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
for h in 0x7fffffff 0xfff 0x7ff 0xff 0x0; do
  make -B -j16 EXTRA_HIPFLAGS=-DFIB_HACK_MASK=$h grout_amd/libgrout_hip.so > $OUT/hack_build.log 2>&1 || exit 1
  timeout -k 10 200 python tools/variants.py --workload fullview64 --fib16 1 --nt 1 --wg 0 --ring 2 --rounds 3 --reps 5 > $OUT/var_mask$h.jsonl 2> $OUT/var_mask.err
  s=$?; echo "mask $h $(cat $OUT/var_mask$h.jsonl)"; [ $s -eq 0 ] || exit $s
done
