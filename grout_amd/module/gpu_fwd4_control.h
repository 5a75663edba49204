// SPDX-License-Identifier: BSD-3-Clause
//
// gpu_fwd4_control.h -- the control-plane mirror of the fast path's grout
// module (gpu_fwd4_control.c): it follows grout's control plane through its
// events and keeps every GPU context's iface, nexthop, reta and FIB mirrors
// equal to grout's objects.
//
// It subscribes, at constructor time as grout's modules do, to
//   GR_EVENT_IFACE_POST_ADD / _POST_RECONFIG / _STATUS_UP / _STATUS_DOWN /
//     _MAC_CHANGE / _PRE_REMOVE / _REMOVE         (modules/infra/control/iface.c)
//   GR_EVENT_NEXTHOP_NEW / _UPDATE / _DELETE      (modules/infra/control/nexthop.c)
//   GR_EVENT_IP_ROUTE_ADD / _DEL                  (modules/ip/control/route.c)
//   GR_EVENT_IP6_ROUTE_ADD / _DEL                 (modules/ip6/control/route.c)
// with event_subscribe, and to the same nexthop and route events with
// event_subscribe_internal: integration/grout-gpu_fwd4-control.patch makes
// grout push those, through a channel no API client sees, where it changes
// an object without a public event (GR_NH_ORIGIN_INTERNAL nexthops and
// routes: every address's nexthop, every learned neighbour's /32 or /128;
// nexthop state changes by ARP/NDP resolution and ageing; group members
// dropped with a deleted nexthop).
//
// A nexthop is named on the GPU by a slot (1.., 0 = NULL), the mirror's dense
// index for the struct nexthop * grout's FIB holds (route.c:124-145); the slot
// is taken at the nexthop's first event and given back at its DELETE, which
// grout pushes after rte_rcu_qsbr_synchronize (modules/infra/control/nexthop.c:505-513), when no
// batch can name it any more. Route changes are published in batches
// (gpu_fwd4_fib4_commit at the control loop turn's end, every 4096 changes,
// and at GR_EVENT_NEXTHOP_PRE_DELETE, which the patch pushes before
// nexthop_destroy's synchronize), so a route is gone from every GPU before
// grout's synchronize for its nexthop starts.
#pragma once

#include <grout_hip.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct nexthop;

// The slot of a nexthop (0: not mirrored). No dereference of nh.
uint32_t gpu_fwd4_control_nh_slot(const struct nexthop *nh);

// What the mirror holds, as it pushed it to every context.
int gpu_fwd4_control_nh(uint32_t slot, struct gr_hip_nh *out); // -ENOENT: free slot
int gpu_fwd4_control_iface(uint16_t iface_id, struct gr_hip_iface *out); // -ENOENT: none
int gpu_fwd4_control_reta(uint32_t first, uint32_t *slots, uint32_t n);
// Routes in the mirror (host bits masked): the count, up to max written.
int gpu_fwd4_control_routes4(struct gr_hip_route4 *out, uint32_t max);
int gpu_fwd4_control_routes6(struct gr_hip_route6 *out, uint32_t max);

struct gpu_fwd4_control_stats {
	uint64_t events; // public events handled
	uint64_t internal; // internal events handled (the patch's channel)
	uint64_t commits; // FIB publications
	uint64_t errors; // fast-path calls that failed
	int first_error; // -errno of the first
	uint32_t slots_used; // nexthop slots held
	uint32_t reta_used; // reta entries held
	uint32_t routes4, routes6;
	uint32_t pending; // route changes in every context's RIB, not yet published
	uint64_t presync; // publications grout's wait for the datapath forced (see "publication")
	uint64_t unordered; // publications made while L3 nexthop changes were unpublished (0: never)
	uint64_t no_timer; // changes published at once: no timer on an event base (before attach)
};
void gpu_fwd4_control_stats(struct gpu_fwd4_control_stats *);

// Replay the mirror's whole state into context i (ifaces, nexthops, reta,
// every VRF's FIBs rebuilt and published), then clear its divergence
// (gpu_fwd4_resync): the recovery of a context a control call failed on.
int gpu_fwd4_control_replay(uint32_t i);

// Tests: forget everything (the contexts' state is the caller's to reset).
void gpu_fwd4_control_reset(void);

// Route changes are published in batches (gpu_fwd4_control.c,
// "publication"): a timer on the control thread's event base, which the
// module's init passes here, publishes what the event loop's turn gathered.
struct event_base;
void gpu_fwd4_control_attach(struct event_base *ev);
// Publish every route change gathered so far, now (every VRF's FIBs).
void gpu_fwd4_control_flush(void);

#ifdef __cplusplus
}
#endif
