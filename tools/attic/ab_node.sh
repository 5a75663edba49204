#!/bin/bash
# A/B prebuilt libgrout_hip.so builds (build/ab/<name>.so) on the node walk
# (tools/node_scale.py, staged lines), alternating processes.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
cp grout_amd/libgrout_hip.so build/ab/cur.so
for r in 1 2; do
  for v in ${LIBS:-old new}; do
    cp build/ab/$v.so grout_amd/libgrout_hip.so
    timeout -k 10 300 python tools/node_scale.py --mode staged --threads ${THREADS:-1,8} > $OUT/abn_$v$r.jsonl 2> $OUT/abn.err
    s=$?; echo "$v $r"; cat $OUT/abn_$v$r.jsonl; [ $s -eq 0 ] || { cp build/ab/cur.so grout_amd/libgrout_hip.so; exit $s; }
  done
done
cp build/ab/cur.so grout_amd/libgrout_hip.so
