#!/bin/bash
# parity tests, variant A/B, PMC passes, kernel trace of the bench
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { local s=$1; if [ "$s" -ne 0 ] && [ "$s" -ne 1 ]; then echo "FATAL $2 $s" | tee -a $OUT/steps.log; exit "$s"; fi; echo "$2 exit $s" | tee -a $OUT/steps.log; }

timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
fatal $? pytest_gpu
tail -15 $OUT/pytest_gpu.log

timeout -k 10 400 python tools/variants.py > $OUT/variants.jsonl 2> $OUT/variants.err
fatal $? variants
cat $OUT/variants.jsonl

rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true

i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
	i=$((i+1))
	timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o run -- python3 tools/pmc_run.py > $OUT/pmc$i.log 2>&1
	fatal $? "pmc$i $set"
done
python tools/pmc_summary.py $OUT/pmc1 $OUT/pmc2 $OUT/pmc3 $OUT/pmc4 $OUT/pmc5 > $OUT/pmc_summary.json 2>&1
cat $OUT/pmc_summary.json

timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
	python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $OUT/prof_bench.json 2> $OUT/prof.err
fatal $? rocprof_bench
cat $OUT/prof_bench.json
head -3 $OUT/prof/run_kernel_stats.csv
exit 0
