#!/bin/bash
# list the PMC counters rocprofv3 offers on gfx950 (names only)
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --list-avail > $OUT/pmc_list.txt 2>&1
s=$?; grep -oE "^[[:space:]]*(TA|TD|TCP|TCC|SQ|GRBM)_[A-Za-z0-9_]+" $OUT/pmc_list.txt | sort -u | tr -d ' ' > $OUT/pmc_names.txt; wc -l $OUT/pmc_names.txt; exit $s
