#!/bin/bash
# PMC: what the FIB gather costs in the memory pipeline (full view vs one route)
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
sets=("TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_PENDING_STALL_CYCLES_sum"
      "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
      "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"
      "TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_THRASHING_STALL_sum"
      "TCC_HIT_sum TCC_MISS_sum TCC_TAG_STALL_sum"
      "GRBM_GUI_ACTIVE GRBM_COUNT")
for w in fullview64 single64; do
  i=0
  for set in "${sets[@]}"; do
    i=$((i+1))
    rm -rf $OUT/pmc_${w}_$i
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc_${w}_$i -o run -- python3 tools/pmc_run.py --no-calib --workload $w > $OUT/pmc_${w}_$i.log 2>&1
    s=$?; [ $s -eq 0 ] || { echo "FATAL pmc $w $i $s"; tail -5 $OUT/pmc_${w}_$i.log; exit $s; }
  done
  python tools/pmc_summary.py $OUT/pmc_${w}_* > $OUT/pmc_tlb_$w.json
  python -c "import json; d=json.load(open('$OUT/pmc_tlb_$w.json')); print('$w', json.dumps(d.get('gr_fwd4_ring')))"
done
