#!/bin/bash
# host path with 32-byte line write-back over PCIe (experiment build) vs whole lines
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
cp grout_amd/libgrout_hip.so build/ab/cur.so
for v in old narrow old narrow; do
  cp build/ab/$v.so grout_amd/libgrout_hip.so
  GR_HIP_AB_OLD=1 timeout -k 10 300 python tools/host_path_ab.py > $OUT/hn_$v.jsonl 2> $OUT/hn.err
  s=$?; echo "$v"; grep '"host_direct": 1' $OUT/hn_$v.jsonl | tail -1; [ $s -eq 0 ] || { cp build/ab/cur.so grout_amd/libgrout_hip.so; tail -3 $OUT/hn.err; exit $s; }
done
cp build/ab/cur.so grout_amd/libgrout_hip.so
