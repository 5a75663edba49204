#!/bin/bash
# round-1 deliverables: bench line, rocprofv3 kernel trace of the bench, PMC traffic passes
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { local s=$1; if [ "$s" -ne 0 ] && [ "$s" -ne 1 ]; then echo "FATAL $2 $s" | tee -a $OUT/steps.log; exit "$s"; fi; echo "$2 exit $s" | tee -a $OUT/steps.log; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
s=$?; cat $OUT/bench.json; tail -3 $OUT/bench.err; fatal $s bench
[ $s -ne 0 ] && exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-path > $OUT/prof.log 2>&1
fatal $? rocprof_bench
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
	i=$((i+1))
	timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o run -- python3 tools/pmc_run.py > $OUT/pmc$i.log 2>&1
	fatal $? "pmc$i $set"
done
python tools/pmc_summary.py $OUT/pmc1 $OUT/pmc2 $OUT/pmc3 $OUT/pmc4 $OUT/pmc5 > $OUT/pmc_summary.json 2>&1
python tools/pmc_traffic.py $OUT/pmc_summary.json gr_fwd4_ring fullview64 16777216 > $OUT/pmc_traffic.json
cat $OUT/pmc_traffic.json
find $OUT/prof -name "*stats*"
exit 0
