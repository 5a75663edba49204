// SPDX-License-Identifier: BSD-3-Clause
// Test stand-in under the name of modules/infra/datapath/eth.h: eth_domain_t, eth_input_mbuf_data, eth_output_mbuf_data.
// The module files (grout_amd/module/) include grout's and DPDK's headers by
// their names; here those names lead to the stand-ins, in grout to the real ones.
#pragma once

#include "gr_datapath_min.h"
