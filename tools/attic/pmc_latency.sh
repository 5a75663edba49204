#!/bin/bash
# PMC passes behind DESIGN.md §6's account of the FIB gather: L1->L2 read
# latency and pending stalls (TCP), L2 hit / EA read latency (TCC), TA
# address stalls, on the full view and on the one-route stream (or the
# workloads given as arguments).
cd "$(dirname "$0")/.."
for wl in ${@:-fullview64 single64}; do
	bash tools/gpu_session.sh \
		"pmc:${wl}_tcp=TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum@--workload $wl --no-calib" \
		"pmc:${wl}_tcc=TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum@--workload $wl --no-calib" \
		"pmc:${wl}_ta=TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE@--workload $wl --no-calib" || exit $?
done
