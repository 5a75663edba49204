// SPDX-License-Identifier: BSD-3-Clause
// Test stand-in under the name of modules/infra/control/iface.h (+ gr_infra.h): struct iface, iface_stats, iface_get_stats, iface_get_eth_addr, the GR_EVENT_IFACE_* events.
// The module files (grout_amd/module/) include grout's and DPDK's headers by
// their names; here those names lead to the stand-ins, in grout to the real ones.
#pragma once

#include "gr_control_min.h"
