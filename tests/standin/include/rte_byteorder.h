// SPDX-License-Identifier: BSD-3-Clause
// Test stand-in under the name of DPDK rte_byteorder.h: RTE_BE16, rte_be16_t.
// The module files (grout_amd/module/) include grout's and DPDK's headers by
// their names; here those names lead to the stand-ins, in grout to the real ones.
#pragma once

#include "rte_graph_min.h"
