#!/bin/bash
# Placement spread under TCC EA counters: one --pmc pass per counter group.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum" \
	   "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum" \
	   "TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum" \
	   "TCC_EA0_RDREQ_GMI_32B_sum TCC_EA0_RDREQ_DRAM_32B_sum" \
	   "TCC_TAG_STALL_sum TCC_EA0_WRREQ_STALL_sum"; do
	timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_pl$i -o run -- python3 tools/placement_probe.py --sets 8 --passes 1 --steps 5 > $OUT/pmc_pl$i.jsonl 2> $OUT/pmc_pl$i.err
	s=$?; [ $s -ne 0 ] && { echo "pass $i exit $s"; tail -3 $OUT/pmc_pl$i.err; exit $s; }
	echo "== $grp"; python3 tools/pmc_place.py $OUT/pmc_pl$i
	i=$((i+1))
done
