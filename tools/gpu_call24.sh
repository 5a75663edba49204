#!/bin/bash
# memory-pattern ceilings at the headline size (tools/ceiling.hip)
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 120 ./tools/ceiling > $OUT/ceiling.jsonl 2>&1
s=$?; cat $OUT/ceiling.jsonl; exit $s
