#!/bin/bash
# A/B prebuilt builds of one library on one box, through
# tools/node_graph_rate.py (ARGS: its options): LIB=graph (default) swaps
# tests/standin/libgrout_standin.so (the walk harness + the module library), LIB=hip libgrout_hip.so,
# with build/ab/<LIB>_<name>.so for each name in LIBS (default "old new"),
# alternating processes.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
L=${LIB:-graph}
cp grout_amd/libgrout_$L.so build/ab/${L}_cur.so
for r in 1 2 3; do
  for v in ${LIBS:-old new}; do
    cp build/ab/${L}_$v.so grout_amd/libgrout_$L.so
    timeout -k 10 150 python -u tools/node_graph_rate.py ${ARGS:---batch 15360 --depths 2 --rx-touch 0,1 --reps 2} \
      > $OUT/abg_$v$r.jsonl 2> $OUT/abg.err
    s=$?; sed "s/^/$v $r /" $OUT/abg_$v$r.jsonl; [ $s -eq 0 ] || { cp build/ab/${L}_cur.so grout_amd/libgrout_$L.so; exit $s; }
  done
done
cp build/ab/${L}_cur.so grout_amd/libgrout_$L.so
