// SPDX-License-Identifier: BSD-3-Clause
// Test stand-in under the name of DPDK rte_graph_worker.h: struct rte_node, rte_node_enqueue, rte_node_enqueue_x1.
// The module files (grout_amd/module/) include grout's and DPDK's headers by
// their names; here those names lead to the stand-ins, in grout to the real ones.
#pragma once

#include "rte_graph_min.h"
