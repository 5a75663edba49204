// SPDX-License-Identifier: BSD-3-Clause
// Test stand-in under the name of modules/ip/control/ip4.h (+ gr_ip4.h): GR_EVENT_IP_ROUTE_*, struct route4_event (moved there by the control patch).
// The module files (grout_amd/module/) include grout's and DPDK's headers by
// their names; here those names lead to the stand-ins, in grout to the real ones.
#pragma once

#include "gr_control_min.h"
