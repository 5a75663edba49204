// SPDX-License-Identifier: BSD-3-Clause
// Test stand-in under the name of modules/infra/control/nexthop.h (+ gr_nexthop.h): struct nexthop, nexthop_info_l3 / _group, the GR_EVENT_NEXTHOP_* events (PRE_DELETE: the control patch).
// The module files (grout_amd/module/) include grout's and DPDK's headers by
// their names; here those names lead to the stand-ins, in grout to the real ones.
#pragma once

#include "gr_control_min.h"
