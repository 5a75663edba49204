// SPDX-License-Identifier: BSD-3-Clause
// Test stand-in under the name of modules/infra/control/graph.h: GR_NODE_CTX_TYPE, struct gr_node_info, GR_NODE_REGISTER, GR_DROP_REGISTER, gr_node_attach_parent.
// The module files (grout_amd/module/) include grout's and DPDK's headers by
// their names; here those names lead to the stand-ins, in grout to the real ones.
#pragma once

#include "gr_datapath_min.h"
