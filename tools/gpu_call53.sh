#!/bin/bash
# Placement spread: torch sets, allocation kinds, then the sets again under
# a TCP UTCL1 (L1 TLB) counter pass to see whether slow sets translate more.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/placement_probe.py --sets 8 --passes 2 --steps 30 > $OUT/placement.jsonl 2> $OUT/placement.err || { tail $OUT/placement.err; exit 1; }
grep summary $OUT/placement.jsonl
timeout -k 10 400 python -u tools/contig_probe.py > $OUT/contig.jsonl 2> $OUT/contig.err || { tail $OUT/contig.err; exit 1; }
tail -1 $OUT/contig.jsonl
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_PERMISSION_MISS_sum --output-format csv -d $OUT/pmc_place -o run -- python3 tools/placement_probe.py --sets 8 --passes 1 --steps 5 > $OUT/pmc_place.jsonl 2> $OUT/pmc_place.err
s=$?; echo "pmc exit $s"; grep summary $OUT/pmc_place.jsonl; exit $s
