// SPDX-License-Identifier: BSD-3-Clause
// Test stand-in under the name of modules/infra/datapath/rcu.h: gr_datapath_rcu.
// The module files (grout_amd/module/) include grout's and DPDK's headers by
// their names; here those names lead to the stand-ins, in grout to the real ones.
#pragma once

#include "gr_datapath_min.h"
