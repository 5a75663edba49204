#!/bin/bash
# hipMalloc vs contiguous vs torch allocations of the batch (tools/contig_probe.py).
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u tools/contig_probe.py > $OUT/contig.jsonl 2> $OUT/contig.err || { tail $OUT/contig.err; exit 1; }
tail -1 $OUT/contig.jsonl
