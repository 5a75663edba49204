// SPDX-License-Identifier: BSD-3-Clause
// Test stand-in under the name of libevent event2/event.h: evtimer_new / _add / _del, event_free.
// The module files (grout_amd/module/) include grout's and DPDK's headers by
// their names; here those names lead to the stand-ins, in grout to the real ones.
#pragma once

#include "../gr_control_min.h"
