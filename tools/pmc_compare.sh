#!/bin/bash
# SPDX-License-Identifier: BSD-3-Clause
# rocprofv3 --pmc passes (one process each, counter groups within the
# per-block limits) of tools/pmc_run.py for each workload given, into
# gpurun_out/pmc_cmp/<workload>/p<k>; summarise with
#   python3 tools/pmc_compare.py gpurun_out/pmc_cmp
# usage: tools/pmc_compare.sh single64 fullview64
#        PMC_GROUPS="3 5" tools/pmc_compare.sh span20:fullview64:--span-bits=20 ...
# (an item is a workload, or label:workload:extra pmc_run.py arguments)
set -e
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc_cmp
groups=(
  "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum"
  "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_WRREQ_LEVEL_sum"
  "TCC_BUSY_sum TCC_EA0_WRREQ_64B_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_128B_sum"
  "TCP_UTCL1_TRANSLATION_MISS_sum TCP_CLIENT_UTCL1_INFLIGHT_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_STALL_MULTI_MISS_sum"
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum"
  "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCC_LATENCY_FIFO_FULL_sum TCP_PENDING_STALL_CYCLES_sum"
  "SQ_INSTS_SMEM SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"
)
for item in "$@"; do
  IFS=: read -r label wl extra <<< "$item"
  wl=${wl:-$label}
  for k in ${PMC_GROUPS:-${!groups[@]}}; do
    timeout -s KILL 90 rocprofv3 --pmc ${groups[$k]} --output-format csv -d gpurun_out/pmc_cmp/$label/p$k -o run \
      -- python3 tools/pmc_run.py --workload $wl --reps 6 --no-calib $extra > gpurun_out/pmc_cmp/$label.p$k.log 2>&1
    echo "$label p$k done"
  done
done
