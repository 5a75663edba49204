// SPDX-License-Identifier: BSD-3-Clause
// Test stand-in under the name of main/event.h: event_subscribe, event_push (+ event_subscribe_internal / event_push_internal: the control patch).
// The module files (grout_amd/module/) include grout's and DPDK's headers by
// their names; here those names lead to the stand-ins, in grout to the real ones.
#pragma once

#include "gr_control_min.h"
