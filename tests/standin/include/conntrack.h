// SPDX-License-Identifier: BSD-3-Clause
// Test stand-in under the name of modules/policy/control/conntrack.h: conn_key, conn_mbuf_data, gr_conn_parse_key, gr_conn_lookup.
// The module files (grout_amd/module/) include grout's and DPDK's headers by
// their names; here those names lead to the stand-ins, in grout to the real ones.
#pragma once

#include "gr_datapath_min.h"
