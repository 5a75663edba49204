#!/bin/bash
# A/B prebuilt libgrout_graph.so builds (the grout node + walk harness) on one
# box: build/ab/graph_<name>.so for each name in LIBS (default "old new"),
# alternating processes, through tools/node_graph_rate.py (ARGS: its options).
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
cp grout_amd/libgrout_graph.so build/ab/graph_cur.so
for r in 1 2 3; do
  for v in ${LIBS:-old new}; do
    cp build/ab/graph_$v.so grout_amd/libgrout_graph.so
    timeout -k 10 150 python -u tools/node_graph_rate.py ${ARGS:---batch 15360 --depths 2 --rx-touch 0,1 --reps 2} \
      > $OUT/abg_$v$r.jsonl 2> $OUT/abg.err
    s=$?; sed "s/^/$v $r /" $OUT/abg_$v$r.jsonl; [ $s -eq 0 ] || { cp build/ab/graph_cur.so grout_amd/libgrout_graph.so; exit $s; }
  done
done
cp build/ab/graph_cur.so grout_amd/libgrout_graph.so
