// SPDX-License-Identifier: BSD-3-Clause
// Test stand-in under the name of DPDK rte_graph.h: struct rte_node_register, rte_node_from_name, rte_graph_walk.
// The module files (grout_amd/module/) include grout's and DPDK's headers by
// their names; here those names lead to the stand-ins, in grout to the real ones.
#pragma once

#include "rte_graph_min.h"
