#!/bin/bash
# Round-1 profile set for the default kernel (ring 2, DIR24_8 2-byte FIB):
# bench line, rocprofv3 kernel stats of the bench, PMC passes for HBM bytes.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { local s=$1; if [ "$s" -ne 0 ]; then echo "FATAL $2 $s" | tee -a $OUT/steps.log; exit "$s"; fi; echo "$2 exit $s" | tee -a $OUT/steps.log; }
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
fatal $? bench
cat $OUT/bench.json
rm -rf $OUT/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-host-path > $OUT/prof_bench.json 2> $OUT/prof.err
fatal $? rocprof
cat $OUT/prof_bench.json
head -2 $OUT/prof/run_kernel_stats.csv | cut -c1-200
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
	i=$((i+1))
	rm -rf $OUT/pmc_d_$i
	timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc_d_$i -o run -- python3 tools/pmc_run.py > $OUT/pmc_d_$i.log 2>&1
	fatal $? "pmc $set"
done
python tools/pmc_summary.py $OUT/pmc_d_* > $OUT/pmc_summary.json && python tools/pmc_traffic.py $OUT/pmc_summary.json gr_fwd4_ring fullview64 16777216 146 > $OUT/pmc_traffic.json
cat $OUT/pmc_summary.json $OUT/pmc_traffic.json
