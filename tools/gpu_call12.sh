#!/bin/bash
# PMC passes: ring (wg 2, 3) and tile (wg 24) kernels on the full view, ring on single64
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { local s=$1; if [ "$s" -ne 0 ] && [ "$s" -ne 1 ]; then echo "FATAL $2 $s" | tee -a $OUT/steps.log; exit "$s"; fi; echo "$2 exit $s" | tee -a $OUT/steps.log; }
sets=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "GRBM_GUI_ACTIVE GRBM_COUNT")
for cfg in "ring2:--kernel 2 --wg 2 --stats 1 --nt 1" "ring3:--kernel 2 --wg 3 --stats 1 --nt 1" "tile24:--kernel 0 --wg 24 --stats 1 --nt 1" "ring2s:--kernel 2 --wg 2 --stats 1 --nt 1 --workload single64"; do
	name=${cfg%%:*}; opts=${cfg#*:}
	i=0
	for set in "${sets[@]}"; do
		i=$((i+1))
		timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc_${name}_$i -o run -- python3 tools/pmc_run.py --no-calib $opts > $OUT/pmc_${name}_$i.log 2>&1
		fatal $? "pmc $name $set"
	done
	python tools/pmc_summary.py $OUT/pmc_${name}_* > $OUT/pmc_${name}.json 2>&1
	cat $OUT/pmc_${name}.json
done
exit 0
