// SPDX-License-Identifier: BSD-3-Clause
// Test stand-in under the name of modules/policy/datapath/nat_datapath.h: nat_verdict_t, snat44_process.
// The module files (grout_amd/module/) include grout's and DPDK's headers by
// their names; here those names lead to the stand-ins, in grout to the real ones.
#pragma once

#include "gr_datapath_min.h"
