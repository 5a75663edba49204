#!/bin/bash
# SPDX-License-Identifier: BSD-3-Clause
# FETCH_SIZE and WRITE_SIZE, one rocprofv3 --pmc pass each (a process of its
# own), of tools/pmc_run.py for every bench workload, into
# gpurun_out/pmc_traffic/<workload>/{fetch,write}; then, here:
#   python tools/pmc_summary.py gpurun_out/pmc_traffic/<wl> > s.json
#   python tools/pmc_traffic.py s.json gr_fwd4_ring <wl> <batch> <B_pkt> "<source>"
set -e
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc_traffic
for wl in ${WORKLOADS:-fullview64 single64 imix fullview6 imix_frames}; do
  extra=""
  [ "$wl" = imix_frames ] && extra="--batch 4194304"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_traffic/$wl/$c -o run \
      -- python3 tools/pmc_run.py --workload $wl --reps 4 $extra > gpurun_out/pmc_traffic/$wl.$c.log 2>&1
    echo "$wl $c done"
  done
done
