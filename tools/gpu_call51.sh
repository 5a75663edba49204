#!/bin/bash
# Relative buffer placement: tools/offset_probe.py for the output lines, then metadata.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u tools/offset_probe.py --what out > $OUT/offset_out.jsonl 2> $OUT/offset.err || { tail $OUT/offset.err; exit 1; }
tail -1 $OUT/offset_out.jsonl
timeout -k 10 300 python -u tools/offset_probe.py --what meta --passes 1 > $OUT/offset_meta.jsonl 2>> $OUT/offset.err || { tail $OUT/offset.err; exit 1; }
tail -1 $OUT/offset_meta.jsonl
