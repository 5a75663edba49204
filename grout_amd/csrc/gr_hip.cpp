// SPDX-License-Identifier: BSD-3-Clause
//
// gr_hip.cpp -- implementation of the C ABI declared in include/grout_hip.h:
// device mirrors of grout's iface / nexthop objects, per-VRF device FIBs fed
// by the host RIB (fib4.c), queues (one HIP stream each, the analogue of one
// grout worker / RX queue) and the launches of the fused kernel.
//
// Control-plane updates are stream ordered: a control stream first waits for
// every queue's submitted work, then copies, then the caller returns once the
// copies are done. Submits issued after the call see the new state; in-flight
// kernels never see a half-updated table. That is the role of the RCU QSBR
// synchronisation grout performs around FIB changes (modules/ip/control/route.c:86-95,740-771).
#include <hip/hip_runtime.h>

#include "fib4.h"
#include "fib6.h"
#include "fwd4_kernel.h"
#include "gr_node_priv.h"

#include <algorithm>
#include <atomic>
#include <errno.h>
#include <mutex>
#include <shared_mutex>
#include <new>
#include <stdio.h>
#include <time.h>
#include <unistd.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

extern "C" hipError_t gr_fwd4_ring_launch(const fwd4_params *A, uint32_t grid, hipStream_t s, int variant, int cfg);
extern "C" int gr_fwd4_ring_occupancy(int variant, int cfg, uint32_t nhf_lds);
extern "C" hipError_t gr_fwd4_resident_launch(const fwd4_res_params *R, uint32_t rings, hipStream_t s);
extern "C" hipError_t gr_stats_collect_launch(void *d, void *out, uint32_t w, uint32_t pitch, uint32_t rows, int reset,
					      hipStream_t s);
extern "C" uint32_t gr_fwd4_ring_nhf_max(void);
extern "C" int gr_fwd4_resident_occupancy(void);
extern "C" int gr_fwd4_ring_ncfg(void);
#define RING_WG_PER_CU 2 // default workgroups per CU of the ring kernel (measured)


// GR_HIP_TRACE_ERRORS=1 in the environment: each failing HIP call named on
// stderr (file:line, the call, HIP's error string) before it is returned
#define HCK(expr)                                                                                  \
	do {                                                                                       \
		hipError_t e__ = (expr);                                                           \
		if (e__ != hipSuccess) {                                                           \
			(void)hipGetLastError();                                                   \
			if (getenv("GR_HIP_TRACE_ERRORS"))                                         \
				fprintf(stderr, "gr_hip: %s:%d: %s: %s\n", __FILE__, __LINE__, #expr, \
					hipGetErrorString(e__));                                   \
			return e__ == hipErrorOutOfMemory ? -ENOMEM : -EIO;                        \
		}                                                                                  \
	} while (0)

namespace {

constexpr uint32_t N_TIMED = 64;
constexpr uint32_t HOST_SLOTS = 3;
constexpr uint32_t HOST_CHUNK = 1u << 18; // packets per host-mode chunk

// Device FIB formats (gr_hip_tune "fib_format"); the 2-byte ones apply while
// every nexthop slot and tbl8 group index fits 15 bits, else FIB_FMT_24.
#define FIB_FMT_24 0 // DIR24_8, 4-byte entries (fib4.h encoding)
#define FIB_FMT_16_8_8 1 // DIR-16-8-8, 2-byte entries
#define FIB_FMT_24_W2 2 // DIR24_8, 2-byte entries

// One of a VRF's two device copies of its IPv4 FIB (FIB publication is
// double-buffered: launches read the published copy while a commit writes
// the other, see gr_hip_fib4_commit).
struct fib4_buf {
	uint32_t *d24 = nullptr; // 4-byte entries (fib4.h encoding)
	uint32_t *d8 = nullptr;
	// DIR-16-8-8 with 2-byte entries, used while every slot fits 15 bits:
	// top[65536] (u32: bit31 = chunk index, else the /16's entry), then
	// chunks of 256 2-byte /24 entries for the non-uniform /16s only.
	uint32_t *d16 = nullptr; // top, followed by the chunks
	uint16_t *d8_16 = nullptr;
	// DIR24_8 with 2-byte entries (bit15 = tbl8 group), same condition
	uint16_t *d24_16 = nullptr;
	int fmt = FIB_FMT_24; // format of the table it holds
	bool up = false; // holds a complete table in `fmt`

	void free_all() {
		hipFree(d24);
		hipFree(d8);
		hipFree(d16);
		hipFree(d8_16);
		hipFree(d24_16);
		*this = fib4_buf();
	}
};

// The same for the IPv6 trie: top[65536], group slots, skips (fib6.h).
struct fib6_buf {
	uint32_t *d6 = nullptr;
	uint32_t groups = 0; // group capacity
	bool up = false;

	void free_all() {
		hipFree(d6);
		*this = fib6_buf();
	}
};

struct vrf_fib {
	gr_fib4 *rib = nullptr;
	fib4_buf b4[2];
	int pub4 = 1; // the copy the current generation's views point at (the other is written)
	uint8_t sel4[2] = {1, 1}; // the copy each view generation points at
	// what b4[pub4 ^ 1] misses of the published table: tbl24 index ranges
	// (sorted, disjoint) and tbl8 groups (sorted), or everything
	std::vector<gr_fib4_range> pend24;
	std::vector<uint32_t> pend8;
	bool pend_all = true;
	// DIR-16-8-8 chunk assignment, shared by both copies (each dirty /16 is
	// rewritten into a copy before that copy is published)
	std::vector<int32_t> chunk_of; // per /16: chunk index or -1
	std::vector<uint32_t> chunk_free; // free chunk indexes (stack)
	uint32_t n_chunks = 0; // chunks in use
	uint32_t max_slot = 0; // highest nexthop slot ever routed (never decreases)
	uint32_t num_tbl8 = 0;

	const fib4_buf &pub() const {
		return b4[pub4];
	}
	bool uploaded() const {
		return b4[pub4].up;
	}
	void reset4() { // forget the IPv4 state only (device copies freed by the caller)
		rib = nullptr;
		b4[0] = fib4_buf();
		b4[1] = fib4_buf();
		pub4 = 1;
		sel4[0] = sel4[1] = 1;
		pend24.clear();
		pend8.clear();
		pend_all = true;
		chunk_of.clear();
		chunk_free.clear();
		n_chunks = 0;
		max_slot = 0;
		num_tbl8 = 0;
	}
	// IPv6: fib6.h trie, double-buffered the same way: what b6[pub6 ^ 1]
	// misses of the published image (first-level indexes, group slots, skip
	// nodes, sorted), or everything
	gr_fib6_t *rib6 = nullptr;
	fib6_buf b6[2];
	int pub6 = 1;
	uint8_t sel6[2] = {1, 1};
	std::vector<uint32_t> pend6[3];
	bool pend6_all = true;

	bool uploaded6() const {
		return b6[pub6].up;
	}
};

struct host_slot {
	hipStream_t s = nullptr;
	uint8_t *in = nullptr, *out = nullptr;
	gr_hip_pkt_meta *meta = nullptr;
	gr_hip_verdict *v = nullptr;
};

// What the resident kernel must have done (res_post): seq[j] on ring j of the
// queue's rings, j < k (each ring numbers its own batches).
#define RES_WMAX 8
struct res_mark {
	uint64_t seq[RES_WMAX] = {};
	uint32_t k = 0;
};

// One rte_graph node walk (gr_hip_node_start .. gr_hip_node_finish): its
// pinned staging, grown on demand, and the walk in flight.
struct node_slot {
	uint32_t cap = 0;
	uint8_t *lines = nullptr, *out = nullptr;
	gr_hip_pkt_meta *meta = nullptr;
	gr_hip_verdict *v = nullptr;
	void *d_lines = nullptr, *d_out = nullptr, *d_meta = nullptr, *d_v = nullptr; // their device addresses
	std::vector<uint32_t> pos; // where each mbuf is staged (gr_hip_node_layout)
	hipEvent_t done = nullptr; // recorded behind the walk's GPU work
	gr_hip_mbuf *m = nullptr;
	uint32_t n = 0, ns = 0, burst = 0;
	bool by_addr = false;
	bool sync = false; // finished at start already (staged copies, or nothing to send)
	int r = 0; // the GPU call's result when sync
	// the walk being appended (gr_hip_node_append): views and slots staged so
	// far, and whether the header lines are (not with "node_ptrs")
	bool open = false, lines_in = false;
	uint32_t na = 0, p = 0;
	// appended from the mbufs (gr_hip_node_append_mbufs): no views; the
	// mbufs (contiguous over the slot's appends) and the layout they are read with
	bool own = false;
	void *const *mb0 = nullptr;
	const gr_hip_mbuf_layout *lay = nullptr;
	bool kcount = false; // its kernel counts the per-iface counters (not the hand-back)
	bool resident = false; // posted to the resident kernel (res_post): done at `res`
	res_mark res;
	uint64_t t_post = 0; // when it was posted (host ns): its deadline starts there
};

} // namespace

// gr_hip_node_prof's clocks run (the "node_prof" knob): off by default, each
// read costs tens of nanoseconds per append
static std::atomic<bool> node_prof_on{false};

// a worker's own: on whole 128-byte line pairs, none shared with another
// worker's queue (the node writes its slots at every append)
struct alignas(128) gr_hip_queue {
	gr_hip_ctx *ctx;
	hipStream_t s;
	bool own_stream;
	hipEvent_t ev0[N_TIMED], ev1[N_TIMED];
	uint64_t n_launch; // timed launches
	uint64_t n_submit; // submits that could be timed (time_every sampling)
	bool always_timed; // every launch carries events, whatever the knobs (gr_hip_batch_place's probes)
	hipEvent_t quiesce;
	hipEvent_t retire; // recorded at every FIB publication: the launches that may read the unpublished copies
	uint64_t seen_serial; // the publication this queue's stream last waited for (ready_ev)
	hipEvent_t sync_ev; // host waits on the queue's streams (host_wait)
	gr_hip_iface_stats *d_stats; // [FWD4_STAT_SHARDS][max_ifaces]
	host_slot hs[HOST_SLOTS];
	// node walks in flight (gr_hip_node_start / _finish), a ring of GR_HIP_NODE_DEPTH
	node_slot nw[GR_HIP_NODE_DEPTH];
	uint32_t nw_head, nw_count;
	uint8_t *d_pad; // the zeroed line pad slots of a frames-by-address batch point at
	uint32_t *h_err, *d_err; // kernel error word (pinned, mapped): a workgroup gave up
	// per-iface counters of the node walks handed back (gr_hip_node_iface_stats):
	// what the kernels counted in d_stats for the walks launched with counters
	// (folded in through a pinned snapshot of d_stats), and what the host
	// hand-back counted for the others
	std::vector<gr_hip_iface_stats> node_if;
	std::vector<gr_hip_iface_stats> kern_seen; // d_stats totals folded into node_if so far
	gr_hip_iface_stats *snap = nullptr; // pinned [FWD4_STAT_SHARDS][snap_w] copy of d_stats
	void *snap_d = nullptr; // its device address (gr_stats_collect writes it)
	uint32_t snap_cap = 0, snap_w = 0; // ifaces per shard: allocated, in the copy in flight
	// gr_hip_queue_stats' read of every shard (pinned, as snap)
	gr_hip_iface_stats *rd = nullptr;
	void *rd_d = nullptr;
	uint32_t rd_cap = 0;
	hipEvent_t snap_ev = nullptr;
	bool snap_pending = false;
	uint64_t node_counted = 0, snap_counted = 0; // node walks launched with counters; covered by a snapshot
	// gr_hip_fwd4_host on pageable memory: the queue's own pinned copies
	// (grown on demand), which the CPU fills and drains around the pinned path
	uint8_t *pg_lines = nullptr, *pg_out = nullptr;
	gr_hip_pkt_meta *pg_meta = nullptr;
	gr_hip_verdict *pg_v = nullptr;
	uint32_t pg_cap = 0;
	int ring = -1; // the first of the resident kernel's res_w rings this queue posts to (-1: none yet)
	uint32_t res_w = 0; // how many (the context's res_w when they were taken)
	uint32_t res_inflight = 0; // its resident batches posted and not yet finished
	res_mark res_posted; // the last seq posted on each of its rings
	res_mark res_retire; // posted before the last FIB publication (retire_wait)
	// per ring of the queue: the last seq res_cancel retired unrun (read
	// without res_mu by the worker's node_finish)
	uint64_t res_cancelled[RES_WMAX] = {};
	// a resident batch the kernel would neither finish nor leave (res_cancel):
	// the GPU may still write the queue's node slots, so nothing of them is
	// used or freed again; every later node call fails (the node punts)
	bool dead = false;
	uint32_t res_polls = 0; // gr_hip_node_pending's polls of resident batches
	uint32_t res_rot = 0; // the helper ring the last rotated batch went to (knob "resident_rotate")
};

struct host_range { // gr_hip_host_register
	uintptr_t host, dev;
	size_t len;
	bool ours; // holds a reference on a registration of ours (hreg_global)
};

// hipHostRegister is process-wide: the runtime knows one registration of a
// range, whichever context asked. Every context that registers a range holds
// a reference here, and the last one out unregisters it, after waiting on the
// host for its own queues (gr_hip_host_unregister). Without the count, context
// A's unregister left context B's registry holding a device address the
// runtime no longer mapped (tools/hostreg_probe.py: B's address unchanged
// after A's hipHostUnregister, the runtime's attributes already "unregistered").
struct hreg_global {
	uintptr_t host, dev;
	size_t len;
	uint32_t refs;
};
static std::mutex g_hreg_mu;
static std::vector<hreg_global> g_hregs;

#define RES_MAX_DEV 64
// Rings held by queues, per device, over every context of the process: a
// resident launch's workgroups must all be co-resident (one per CU at its LDS
// size), or a ring no CU ever runs stalls its queue's batches (res_take).
static std::atomic<uint32_t> g_res_held[RES_MAX_DEV];

// The registration of ours that holds [p, p + len), or null (g_hreg_mu held).
static hreg_global *hreg_global_find(uintptr_t p, size_t len) {
	for (hreg_global &g : g_hregs)
		if (p >= g.host && p - g.host <= g.len && len <= g.len - (p - g.host))
			return &g;
	return nullptr;
}

// Drop a reference taken by gr_hip_host_register; the last unregisters.
static int hreg_global_put(uintptr_t p, size_t len) {
	std::lock_guard<std::mutex> gl(g_hreg_mu);
	for (size_t i = 0; i < g_hregs.size(); i++) {
		hreg_global &g = g_hregs[i];
		if (!(p >= g.host && p - g.host <= g.len && len <= g.len - (p - g.host)))
			continue;
		if (--g.refs == 0) {
			const hipError_t e = hipHostUnregister(reinterpret_cast<void *>(g.host));
			g_hregs.erase(g_hregs.begin() + (long)i);
			if (e != hipSuccess) {
				(void)hipGetLastError();
				return -EIO;
			}
		}
		return 0;
	}
	return -ENOENT;
}

struct gr_hip_ctx {
	int dev;
	uint32_t max_ifaces, max_nh;
	int n_cu;
	std::shared_mutex mu; // control-plane writers exclusive; submitters shared
	std::mutex fib_mu; // FIB writers (routes, commits), taken before mu
	hipStream_t ctl;
	std::vector<gr_hip_iface> ifaces;
	std::vector<gr_hip_nh> nh;
	std::vector<uint32_t> reta;
	std::vector<vrf_fib> vrfs;
	// Two generations of the RX views and of the table block a launch reads
	// (double-buffered FIB publication): a submit takes generation `gen`.
	uint32_t gen;
	std::vector<fwd4_rx> rx[2]; // host images of the device views
	std::vector<fwd4_adj> adj;
	uint32_t nh_hi; // highest nexthop slot ever set
	fwd4_rx *d_rx[2];
	fwd4_adj *d_adj;
	std::vector<fwd4_nhf> nhf; // fast adjacencies (host image)
	fwd4_nhf *d_nhf;
	std::vector<fwd4_nhf> nhf6; // the same for the IPv6 chain
	fwd4_nhf *d_nhf6;
	uint32_t v6_routes; // IPv6 routes on the device, all VRFs (stage nhf6 in LDS when > 0)
	std::vector<fwd4_rx6> rx6[2]; // IPv6 views and adjacencies (host images)
	// per generation: the trie every IPv6 RX view points at when they all
	// point at one (one VRF with IPv6 routes), which launches stage the
	// 2000::/4 first-level entries of in LDS; NULL otherwise
	const uint32_t *top6[2];
	std::vector<fwd4_adj6> adj6;
	fwd4_rx6 *d_rx6[2];
	fwd4_adj6 *d_adj6;
	uint32_t *d_reta;
	uint32_t d_reta_cap;
	uint32_t *d_vlan_keys;
	uint16_t *d_vlan_vals;
	uint32_t vlan_cap;
	std::vector<uint32_t> vlan_keys_h; // host image of the VLAN table (node hand-back counters)
	std::vector<uint16_t> vlan_vals_h;
	fwd4_edges edges;
	fwd4_tables *d_tables[2]; // device copy of what every launch reads, by generation
	std::vector<gr_hip_queue *> queues;
	// tuning knobs (gr_hip_tune)
	int nt; // FWD4_V_NT
	int stats_on;
	int wg_per_cu; // 0 = one tile per workgroup, N = persistent N per CU
	int fib_fmt; // FIB format when 2-byte entries fit (FIB_FMT_*)
	int ring_cfg; // ring geometry (fwd4_ring.hip ring_cfgN)
	int host_direct; // host path: the kernel reads / writes pinned host memory itself
	int node_ptrs; // node path: frames in registered memory are handed over by address
	uint32_t stage_min_tiles; // fast adjacencies staged in LDS only from this many tiles per workgroup
	int tile_order; // 0: workgroup b takes tiles b, b + G, ...; 1: one contiguous run each;
	                // 2: one region per XCD; 3: runs of tile_run tiles interleaved
	uint32_t tile_run; // tiles per run of tile order 3
	int alloc_contig; // large device arrays physically contiguous first (dev_alloc), default 1
	uint32_t spin_max; // ring waits: polls before giving up (0 = the kernel's default)
	std::atomic<int> fail_appends{0}; // tests: the next N gr_hip_node_append calls fail (-ENOMEM)
	int untimed; // measurements: no HIP events around launches (gr_hip_queue_kernel_ms sees none)
	uint32_t time_every; // HIP events around every N-th submit of a queue only (0, 1 = every one)
	int stats_copy; // gr_hip_queue_stats reads with a copy and resets with a memset (measurement only)
	int sync_check; // debugging: the host path waits after each step it enqueues and names a failing one
	std::atomic<int> host_path_last{-1}; // the path the last gr_hip_fwd4_host(_ex) took (GR_HIP_HOST_PATH_*)
	std::vector<host_range> hregs; // registered host memory, by host address
	// the resident kernel (knob "resident", see res_post): descriptor rings,
	// done and exited words (pinned host memory), its stream and launch state
	int res_on;
	uint32_t res_rings; // workgroups of a launch = rings (knob "resident_rings")
	uint32_t res_w; // rings (workgroups) per queue: each batch split over them (knob "resident_wgs")
	uint32_t res_ms; // lifetime of an idle workgroup (knob "resident_ms")
	uint32_t res_nap; // idle poll backoff ceiling, in s_sleep(8) units (knob "resident_nap")
	uint32_t res_tiles; // tiles per workgroup a batch is split into, up to the queue's rings (knob "resident_tiles")
	uint32_t res_split = 0; // at most this many of a queue's rings per batch (0: all; knob "resident_split")
	uint32_t res_budget = 32; // workgroups the busy queues' batches are split over together (knob "resident_budget"; 0: no cap)
	// a one-ring batch posted while the queue has others in flight runs on
	// the queue's next helper ring, its first ring only waking that one
	// (knob "resident_rotate", off by default; the grout node sets it when
	// more than one batch per graph is on the GPU, gpu_fwd4_conf.depth > 2)
	bool res_rotate = false;
	std::atomic<uint32_t> res_busy{0}; // queues with resident batches in flight
	fwd4_res_desc *res_desc;
	uint64_t *res_done, *res_exited;
	uint32_t *res_stop;
	uint32_t *res_taken_h; // [res_rings]: rings held by a queue, as the kernel reads it
	uint64_t *res_wake_d = nullptr; // [res_rings * RES_STRIDE], device memory: helpers' wake words
	fwd4_res_desc *res_desc_d; // their device addresses
	uint64_t *res_done_d, *res_exited_d;
	uint32_t *res_stop_d, *res_taken_d;
	hipStream_t res_s;
	hipEvent_t res_ev;
	std::atomic<bool> res_live; // launched, and not yet seen to have left
	uint64_t res_launch; // id of the last launch (0: none)
	std::vector<uint8_t> res_taken; // rings held by a queue
	std::mutex res_mu;
	uint32_t res_wait_ms = 500; // a resident batch not done after this is cancelled (knob "resident_wait_ms")
	uint32_t res_cap = 0; // rings this device can hold co-resident (res_setup; device-wide, g_res_held)
	// CUs no ring may take (knob "resident_reserve_cu"): a queue that finds no
	// ring launches per batch, and its launches need CUs the resident kernel
	// does not hold for its lifetime after the last batch
	uint32_t res_reserve_cu = 16;
	uint32_t res_held = 0; // rings this context's queues hold (counted in g_res_held)
	bool res_dead = false; // a launch that would not leave: no resident batch any more, its words never freed
	bool res_hold = false; // tests: no (re)launch while set (a kernel that stopped serving its rings)
	bool res_leave_fail = false; // tests: res_leave reports a launch that would not leave
	std::atomic<uint32_t> res_cancels{0}; // batches res_cancel retired unrun (knob read "resident_cancels")
	// FIB publication (see retire_wait): two pinned staging buffers used in
	// turn by the commits (fib_mu), each with the event of its last upload,
	// and per generation the event of the upload that made it complete
	uint8_t *stage[2];
	size_t stage_cap[2];
	hipEvent_t stage_ev[2];
	uint32_t stage_i;
	hipEvent_t ready_ev[2];
	uint64_t serial; // publications so far
	std::atomic<uint32_t> commit_us[3]; // the last commit: staging (host), enqueue (shared lock), publish (exclusive lock)
	std::mutex occ_mu; // the occupancy cache below (launches run concurrently)
	int occ_ring[8]; // by variant, of the last launch's geometry and staging ("occupancy")
	struct occ_entry {
		uint32_t staged; // fast adjacencies staged in LDS (IPv4 + IPv6)
		int cfg; // ring geometry
		int occ[8]; // workgroups per CU by variant, 0 = does not fit
	} occ_cache[4];
	uint32_t occ_n; // entries filled (round robin past 4)
};

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------

// Make the control stream wait for everything submitted on every queue.
static int res_wait(gr_hip_queue *q, const res_mark &m);
static void res_free(gr_hip_ctx *c);
static uint64_t now_ns_host();

static int quiesce(gr_hip_ctx *c) {
	for (gr_hip_queue *q : c->queues) {
		HCK(hipEventRecord(q->quiesce, q->s));
		HCK(hipStreamWaitEvent(c->ctl, q->quiesce, 0));
		if (const int r = res_wait(q, q->res_posted)) // its resident batches: on the host
			return r;
	}
	return 0;
}

static int h2d(gr_hip_ctx *c, void *dst, const void *src, size_t n) {
	if (n == 0)
		return 0;
	HCK(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, c->ctl));
	return 0;
}

static int ctl_sync(gr_hip_ctx *c) {
	HCK(hipStreamSynchronize(c->ctl));
	return 0;
}

// The host waits for what queue q enqueued on stream s, through an event:
// hipStreamSynchronize holds the stream for as long as it waits, which would
// hold up the FIB publication recording its retire event there from the
// control thread (measured: the publish step then took as long as the
// rest of the queue's work, 1-1.6 ms).
static int host_wait(gr_hip_queue *q, hipStream_t s) {
	HCK(hipEventRecord(q->sync_ev, s));
	HCK(hipEventSynchronize(q->sync_ev));
	return 0;
}

static const gr_hip_iface *iface_get(const gr_hip_ctx *c, uint32_t id) {
	if (id == GR_HIP_IFACE_ID_UNDEF || id >= c->max_ifaces || c->ifaces[id].id != id)
		return nullptr; // iface_from_id, iface.c:459-466
	return &c->ifaces[id];
}

// RX view of iface `id` in view generation `g`: iface_input's admin/mode
// edge (iface_input.c:88-97), eth_input's MAC (eth_input.c:62-68) and the
// copy of the VRF FIB that generation points at (modules/ip/control/route.c:51-61).
static fwd4_rx make_rx(const gr_hip_ctx *c, uint32_t id, uint32_t g) {
	fwd4_rx r;
	memset(&r, 0, sizeof(r));
	const gr_hip_iface *i = iface_get(c, id);
	if (i == nullptr)
		return r;
	r.id = (uint16_t)id;
	if (!(i->flags & GR_HIP_IFACE_F_UP))
		r.e_in = GR_HIP_E_IFACE_INPUT_ADMIN_DOWN;
	else
		r.e_in = i->mode < GR_HIP_IFACE_MODE_COUNT ? c->edges.mode[i->mode] : GR_HIP_E_IFACE_MODE_UNKNOWN;
	r.flags = (i->mac_ok ? FWD4_RX_MAC_OK : 0) | ((i->flags & GR_HIP_IFACE_F_SNAT_DYNAMIC) ? FWD4_RX_SNAT_DYN : 0)
		| (i->mode == GR_HIP_IFACE_MODE_VRF ? FWD4_RX_VLAN_DEMUX : 0);
	memcpy(r.mac, i->mac, 6);
	const gr_hip_iface *vrf = iface_get(c, i->vrf_id);
	if (vrf != nullptr && vrf->type == GR_HIP_IFACE_TYPE_VRF && c->vrfs[i->vrf_id].rib != nullptr
	    && c->vrfs[i->vrf_id].b4[c->vrfs[i->vrf_id].sel4[g]].up) {
		const fib4_buf &b = c->vrfs[i->vrf_id].b4[c->vrfs[i->vrf_id].sel4[g]];
		if (b.fmt == FIB_FMT_16_8_8) {
			r.tbl24 = b.d16;
			r.tbl8 = reinterpret_cast<const uint32_t *>(b.d8_16);
			r.flags |= FWD4_RX_FIB16;
		} else if (b.fmt == FIB_FMT_24_W2) {
			r.tbl24 = reinterpret_cast<const uint32_t *>(b.d24_16);
			r.tbl8 = reinterpret_cast<const uint32_t *>(b.d8_16);
			r.flags |= FWD4_RX_FIB24W2;
		} else {
			r.tbl24 = b.d24;
			r.tbl8 = b.d8;
		}
	}
	return r;
}

// IPv6 view of iface `id` in view generation `g`: the FIB6 of its VRF
// (get_fib6, modules/ip6/control/route.c:54-64).
static fwd4_rx6 make_rx6(const gr_hip_ctx *c, uint32_t id, uint32_t g) {
	fwd4_rx6 r = {nullptr, nullptr, nullptr};
	const gr_hip_iface *i = iface_get(c, id);
	if (i == nullptr)
		return r;
	const gr_hip_iface *vrf = iface_get(c, i->vrf_id);
	if (vrf != nullptr && vrf->type == GR_HIP_IFACE_TYPE_VRF && c->vrfs[i->vrf_id].rib6 != nullptr
	    && c->vrfs[i->vrf_id].b6[c->vrfs[i->vrf_id].sel6[g]].up) {
		const fib6_buf &b = c->vrfs[i->vrf_id].b6[c->vrfs[i->vrf_id].sel6[g]];
		r.top = b.d6;
		r.groups = b.d6 + GR_FIB6_TOP;
		r.skips = reinterpret_cast<const uint4 *>(b.d6 + GR_FIB6_TOP + (size_t)b.groups * GR_FIB6_GROUP);
	}
	return r;
}

// eth_output -> iface_output for a nexthop leaving through `oif`
// (eth_output.c:43-62, iface_output.c:75-108), shared by both AFs.
template <typename A>
static void fill_post(const gr_hip_ctx *c, const gr_hip_nh &nh, const gr_hip_iface *oif, A &a) {
	const fwd4_edges &E = c->edges;
	memcpy(a.dmac, nh.mac, 6);
	a.post_iface = oif->id;
	if (!oif->mac_ok) {
		a.e_post = GR_HIP_E_ETH_OUTPUT_NO_MAC;
		return;
	}
	memcpy(a.smac, oif->mac, 6);
	const gr_hip_iface *out = oif;
	if (oif->type == GR_HIP_IFACE_TYPE_VLAN) {
		out = iface_get(c, oif->parent_id);
		if (out == nullptr) {
			a.e_post = GR_HIP_E_IFACE_OUTPUT_VLAN_NO_PARENT;
			return;
		}
	}
	if (!(oif->flags & GR_HIP_IFACE_F_UP)) {
		a.e_post = GR_HIP_E_IFACE_OUTPUT_ADMIN_DOWN;
		return;
	}
	a.tx_if = oif->id;
	a.tx_par = out != oif ? out->id : 0;
	a.post_iface = out->id;
	a.e_post = out->type < 8 ? E.iout_type[out->type] : GR_HIP_E_IFACE_OUTPUT_INVAL_TYPE;
}

// IPv6 adjacency of nexthop `slot`: ip6_input's view (ip6_input.c:133-144)
// and ip6_output -> eth_output -> iface_output resolved for the nexthop
// (ip6_output.c:75-134), leaving the MTU and LINK destination checks.
static fwd4_adj6 make_adj6(const gr_hip_ctx *c, uint32_t slot) {
	const fwd4_edges &E = c->edges;
	const gr_hip_nh &nh = c->nh[slot];
	fwd4_adj6 a;
	memset(&a, 0, sizeof(a));
	a.type = nh.type;
	a.e_in = nh.type < 8 ? E.in6_nh[nh.type] : GR_HIP_EDGE_CHAIN;
	a.flags = ((nh.type == GR_HIP_NH_T_L3 && (nh.flags & GR_HIP_NH_F_LOCAL)) ? FWD4_ADJ_LOCAL : 0)
		| ((nh.flags & GR_HIP_NH_F_LINK) ? FWD4_ADJ_LINK : 0);
	memcpy(a.ipv6, nh.ipv6, 16);
	a.e_mid = a.e_post = GR_HIP_EDGE_CHAIN;
	uint8_t e = nh.type < 8 ? E.out6_nh[nh.type] : GR_HIP_EDGE_CHAIN;
	if (e != GR_HIP_EDGE_CHAIN) { // :85-87
		a.e_pre = e;
		return a;
	}
	const gr_hip_iface *oif = iface_get(c, nh.iface_id);
	if (oif == nullptr) { // :94-97
		a.e_pre = GR_HIP_E_IP6_OUTPUT_ERROR;
		return a;
	}
	a.e_pre = GR_HIP_EDGE_CHAIN;
	a.oif = oif->id;
	a.mtu = oif->mtu;
	e = oif->type < 8 ? E.out6_iface[oif->type] : GR_HIP_EDGE_CHAIN; // :106
	if (e != GR_HIP_EDGE_CHAIN)
		a.e_mid = e;
	else if (nh.state != GR_HIP_NH_S_REACHABLE) // :113-119
		a.e_mid = GR_HIP_E_IP6_HOLD;
	fill_post(c, nh, oif, a);
	return a;
}

// Adjacency of nexthop `slot`: the ip_input view (ip_input.c:156-187) and
// ip_output -> eth_output -> iface_output resolved for that nexthop
// (ip_output.c:87-152, eth_output.c:43-62, iface_output.c:75-108),
// leaving the packet-dependent MTU/DF and LINK destination checks.
static fwd4_adj make_adj(const gr_hip_ctx *c, uint32_t slot) {
	const fwd4_edges &E = c->edges;
	const gr_hip_nh &nh = c->nh[slot];
	fwd4_adj a;
	memset(&a, 0, sizeof(a));
	a.type = nh.type;
	a.e_in = nh.type < 8 ? E.in_nh[nh.type] : GR_HIP_EDGE_CHAIN;
	a.flags = ((nh.type == GR_HIP_NH_T_L3 && (nh.flags & GR_HIP_NH_F_LOCAL)) ? FWD4_ADJ_LOCAL : 0)
		| ((nh.flags & GR_HIP_NH_F_LINK) ? FWD4_ADJ_LINK : 0);
	a.ipv4 = nh.ipv4;
	a.n_members = nh.n_members;
	a.reta_size = nh.reta_size;
	a.reta_off = nh.reta_off;
	a.single = nh.single;
	a.e_mid = a.e_post = GR_HIP_EDGE_CHAIN;
	uint8_t e = nh.type < 8 ? E.out_nh[nh.type] : GR_HIP_EDGE_CHAIN;
	if (e != GR_HIP_EDGE_CHAIN) {
		a.e_pre = e;
		return a;
	}
	const gr_hip_iface *oif = iface_get(c, nh.iface_id);
	if (oif == nullptr) {
		a.e_pre = GR_HIP_E_IP_OUTPUT_ERROR;
		return a;
	}
	a.e_pre = GR_HIP_EDGE_CHAIN;
	a.oif = oif->id;
	a.mtu = oif->mtu;
	e = oif->type < 8 ? E.out_iface[oif->type] : GR_HIP_EDGE_CHAIN;
	if (oif->flags & (GR_HIP_IFACE_F_SNAT_STATIC | GR_HIP_IFACE_F_SNAT_DYNAMIC))
		a.e_mid = GR_HIP_E_IP_OUTPUT_SNAT;
	else if (e != GR_HIP_EDGE_CHAIN)
		a.e_mid = e;
	else if (nh.state != GR_HIP_NH_S_REACHABLE)
		a.e_mid = GR_HIP_E_IP_HOLD;
	fill_post(c, nh, oif, a);
	return a;
}

// Fast adjacency of a precomputed adjacency: filled only for the plain
// forward to a port (see fwd4_nhf), mtu = 0 otherwise.
static fwd4_nhf make_nhf(const fwd4_adj &a) {
	fwd4_nhf f;
	memset(&f, 0, sizeof(f));
	if (a.type == GR_HIP_NH_T_L3 && a.e_in == GR_HIP_EDGE_CHAIN && a.flags == 0 && a.e_pre == GR_HIP_EDGE_CHAIN
	    && a.e_mid == GR_HIP_EDGE_CHAIN && a.e_post == GR_HIP_E_PORT_OUTPUT && a.post_iface == a.oif
	    && a.tx_if == a.oif && a.tx_par == 0 && a.mtu != 0) {
		memcpy(f.dmac, a.dmac, 6);
		memcpy(f.smac, a.smac, 6);
		f.oif = a.oif;
		f.mtu = a.mtu;
	}
	return f;
}

// The IPv6 chain's fast adjacency (chain6): the same plain forward by the
// IPv6 edges (ip6_input / ip6_output registrations), mtu = 0 otherwise.
static fwd4_nhf make_nhf6(const fwd4_adj6 &a) {
	fwd4_nhf f;
	memset(&f, 0, sizeof(f));
	if (a.type == GR_HIP_NH_T_L3 && a.e_in == GR_HIP_EDGE_CHAIN && a.flags == 0 && a.e_pre == GR_HIP_EDGE_CHAIN
	    && a.e_mid == GR_HIP_EDGE_CHAIN && a.e_post == GR_HIP_E_PORT_OUTPUT && a.post_iface == a.oif
	    && a.tx_if == a.oif && a.tx_par == 0 && a.mtu != 0) {
		memcpy(f.dmac, a.dmac, 6);
		memcpy(f.smac, a.smac, 6);
		f.oif = a.oif;
		f.mtu = a.mtu;
	}
	return f;
}

// The trie all of generation g's IPv6 RX views share (NULL: none, or several).
static const uint32_t *common_top6(const gr_hip_ctx *c, uint32_t g) {
	const uint32_t *t = nullptr;
	for (const fwd4_rx6 &r : c->rx6[g]) {
		if (r.top == nullptr || r.top == t)
			continue;
		if (t != nullptr)
			return nullptr;
		t = r.top;
	}
	return t;
}

// Recompute and upload the RX views of generation g (IPv4 and IPv6, every
// iface) on the control stream; does not wait.
static int upload_rx(gr_hip_ctx *c, uint32_t g) {
	for (uint32_t i = 0; i < c->max_ifaces; i++) {
		c->rx[g][i] = make_rx(c, i, g);
		c->rx6[g][i] = make_rx6(c, i, g);
	}
	c->top6[g] = common_top6(c, g);
	HCK(hipMemcpyAsync(c->d_rx[g], c->rx[g].data(), sizeof(fwd4_rx) * c->max_ifaces, hipMemcpyHostToDevice, c->ctl));
	HCK(hipMemcpyAsync(c->d_rx6[g], c->rx6[g].data(), sizeof(fwd4_rx6) * c->max_ifaces, hipMemcpyHostToDevice,
			   c->ctl));
	return 0;
}

// Recompute and upload the RX views (both generations, all ifaces) and
// adjacencies [first, first+n) (n == 0: every slot up to nh_hi). Caller
// holds c->mu exclusively and has quiesced.
static int upload_views(gr_hip_ctx *c, bool rx, uint32_t first, uint32_t n, bool adj) {
	if (rx) {
		for (uint32_t g = 0; g < 2; g++) {
			int r = upload_rx(c, g);
			if (r)
				return r;
		}
	}
	if (adj) {
		if (n == 0) {
			first = 1;
			n = c->nh_hi;
		}
		for (uint32_t i = first; i < first + n; i++) {
			c->adj[i] = make_adj(c, i);
			c->nhf[i] = make_nhf(c->adj[i]);
			c->adj6[i] = make_adj6(c, i);
			c->nhf6[i] = make_nhf6(c->adj6[i]);
		}
		if (n) {
			HCK(hipMemcpyAsync(c->d_adj6 + first, &c->adj6[first], sizeof(fwd4_adj6) * n, hipMemcpyHostToDevice,
					   c->ctl));
			HCK(hipMemcpyAsync(c->d_adj + first, &c->adj[first], sizeof(fwd4_adj) * n, hipMemcpyHostToDevice, c->ctl));
			HCK(hipMemcpyAsync(c->d_nhf + first, &c->nhf[first], sizeof(fwd4_nhf) * n, hipMemcpyHostToDevice, c->ctl));
			HCK(hipMemcpyAsync(c->d_nhf6 + first, &c->nhf6[first], sizeof(fwd4_nhf) * n, hipMemcpyHostToDevice,
					   c->ctl));
		}
	}
	HCK(hipStreamSynchronize(c->ctl));
	return 0;
}

// Refresh the device-resident fwd4_tables (caller holds c->mu and has
// quiesced the queues); completes before returning.
static int upload_tables(gr_hip_ctx *c) {
	fwd4_tables t[2];
	memset(t, 0, sizeof(t));
	for (uint32_t g = 0; g < 2; g++) {
		t[g].rx = c->d_rx[g];
		t[g].adj = c->d_adj;
		t[g].nhf = c->d_nhf;
		t[g].nhf6 = c->d_nhf6;
		t[g].rx6 = c->d_rx6[g];
		t[g].adj6 = c->d_adj6;
		t[g].reta = c->d_reta;
		t[g].vlan_keys = c->d_vlan_keys;
		t[g].vlan_vals = c->d_vlan_vals;
		t[g].reta_cap = c->d_reta ? (uint32_t)c->reta.size() : 0;
		t[g].vlan_mask = c->vlan_cap ? c->vlan_cap - 1 : 0;
		t[g].max_ifaces = c->max_ifaces;
		t[g].max_nh = c->max_nh;
		t[g].edges = c->edges;
		HCK(hipMemcpyAsync(c->d_tables[g], &t[g], sizeof(t[g]), hipMemcpyHostToDevice, c->ctl));
	}
	HCK(hipStreamSynchronize(c->ctl));
	return 0;
}

static void set_default_edges(fwd4_edges *E) {
	// grout's default module set: ip_input.c:200-203, arp_input.c:62,
	// ip6_input.c:161, lacp_input.c:66-68, eth_input.c:115, xconnect.c:65,
	// bridge_input.c:124-125, vxlan_output.c:138, bond_output.c:250,
	// port_output.c:51, xvrf.c:63, ipip/datapath_out.c:91,
	// srv6_output.c:152, dnat44_static.c:102
	memset(E, 0, sizeof(*E));
	auto be = [](uint16_t h) { return (uint16_t)((h >> 8) | (h << 8)); };
	const struct {
		uint16_t t;
		uint8_t e;
	} types[] = {
		{0x0800, GR_HIP_EDGE_CHAIN},
		{0x0806, GR_HIP_E_ARP_INPUT},
		{0x86dd, GR_HIP_EDGE_CHAIN6},
		{0x8809, GR_HIP_E_LACP_INPUT},
	};
	for (auto &t : types) {
		E->eth_type_be[E->n_eth_types] = be(t.t);
		E->eth_type_edge[E->n_eth_types] = t.e;
		E->n_eth_types++;
	}
	E->mode[GR_HIP_IFACE_MODE_VRF] = GR_HIP_EDGE_CHAIN;
	E->mode[GR_HIP_IFACE_MODE_XC] = GR_HIP_E_XCONNECT;
	E->mode[GR_HIP_IFACE_MODE_BOND] = GR_HIP_EDGE_CHAIN;
	E->mode[GR_HIP_IFACE_MODE_BRIDGE] = GR_HIP_E_BRIDGE_INPUT;
	for (int i = 0; i < 8; i++) {
		E->in_nh[i] = GR_HIP_EDGE_CHAIN;
		E->out_nh[i] = GR_HIP_EDGE_CHAIN;
		E->out_iface[i] = GR_HIP_EDGE_CHAIN;
		E->iout_type[i] = GR_HIP_E_IFACE_OUTPUT_INVAL_TYPE;
	}
	for (int i = 0; i < 8; i++) {
		E->in6_nh[i] = GR_HIP_EDGE_CHAIN;
		E->out6_nh[i] = GR_HIP_EDGE_CHAIN;
		E->out6_iface[i] = GR_HIP_EDGE_CHAIN;
	}
	E->in6_nh[GR_HIP_NH_T_BLACKHOLE] = GR_HIP_E_IP6_BLACKHOLE; // ip6_input.c:163-164
	E->in6_nh[GR_HIP_NH_T_REJECT] = GR_HIP_E_IP6_ERROR_DEST_UNREACH;
	E->in6_nh[GR_HIP_NH_T_SR6_LOCAL] = GR_HIP_E_SR6_LOCAL; // srv6_local.c:481
	E->out6_nh[GR_HIP_NH_T_SR6_OUTPUT] = GR_HIP_E_SR6_OUTPUT; // srv6_output.c:153
	E->out6_iface[GR_HIP_IFACE_TYPE_VRF] = GR_HIP_E_XVRF; // xvrf.c:64
	E->in_nh[GR_HIP_NH_T_BLACKHOLE] = GR_HIP_E_IP_BLACKHOLE;
	E->in_nh[GR_HIP_NH_T_REJECT] = GR_HIP_E_IP_ERROR_DEST_UNREACH;
	E->in_nh[GR_HIP_NH_T_DNAT] = GR_HIP_E_DNAT44_STATIC;
	E->out_nh[GR_HIP_NH_T_SR6_OUTPUT] = GR_HIP_E_SR6_OUTPUT;
	E->out_iface[GR_HIP_IFACE_TYPE_VRF] = GR_HIP_E_XVRF;
	E->out_iface[GR_HIP_IFACE_TYPE_IPIP] = GR_HIP_E_IPIP_OUTPUT;
	E->iout_type[GR_HIP_IFACE_TYPE_PORT] = GR_HIP_E_PORT_OUTPUT;
	E->iout_type[GR_HIP_IFACE_TYPE_BOND] = GR_HIP_E_BOND_OUTPUT;
	E->iout_type[GR_HIP_IFACE_TYPE_VXLAN] = GR_HIP_E_VXLAN_OUTPUT;
	E->iout_type[GR_HIP_IFACE_TYPE_BRIDGE] = GR_HIP_E_BRIDGE_INPUT;
}

// ---------------------------------------------------------------------------
// lifetime
// ---------------------------------------------------------------------------

extern "C" int gr_hip_abi_version(void) {
	return GR_HIP_ABI_VERSION;
}

extern "C" const char *gr_hip_strerror(int err) {
	return strerror(err < 0 ? -err : err);
}

extern "C" int gr_hip_init(int dev, uint32_t max_ifaces, uint32_t max_nexthops, gr_hip_ctx_t **out) {
	if (out == nullptr || max_ifaces < 2 || max_ifaces > 65535 || max_nexthops == 0
	    || max_nexthops > GR_HIP_MAX_NEXTHOPS)
		return -EINVAL;
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
		(void)hipGetLastError();
		return -ENODEV;
	}
	if (dev < 0 || dev >= ndev)
		return -ENODEV;
	HCK(hipSetDevice(dev));
	gr_hip_ctx *c = new (std::nothrow) gr_hip_ctx();
	if (c == nullptr)
		return -ENOMEM;
	c->dev = dev;
	c->max_ifaces = max_ifaces;
	c->max_nh = max_nexthops;
	hipDeviceProp_t prop;
	if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
		delete c;
		return -EIO;
	}
	c->n_cu = prop.multiProcessorCount;
	c->ifaces.assign(max_ifaces, gr_hip_iface {});
	c->nh.assign((size_t)max_nexthops + 1, gr_hip_nh {});
	c->vrfs.assign(max_ifaces, vrf_fib {});
	c->gen = 0;
	for (uint32_t g = 0; g < 2; g++) {
		c->rx[g].assign(max_ifaces, fwd4_rx {});
		c->rx6[g].assign(max_ifaces, fwd4_rx6 {});
		c->top6[g] = nullptr;
	}
	c->adj.assign((size_t)max_nexthops + 1, fwd4_adj {});
	c->nhf.assign((size_t)max_nexthops + 1, fwd4_nhf {});
	c->nhf6.assign((size_t)max_nexthops + 1, fwd4_nhf {});
	c->v6_routes = 0;
	c->adj6.assign((size_t)max_nexthops + 1, fwd4_adj6 {});
	c->nh_hi = 0;
	set_default_edges(&c->edges);
	c->d_reta = nullptr;
	c->d_reta_cap = 0;
	c->d_vlan_keys = nullptr;
	c->d_vlan_vals = nullptr;
	c->vlan_cap = 0;
	int ret = -ENOMEM;
	if (hipStreamCreateWithFlags(&c->ctl, hipStreamNonBlocking) != hipSuccess)
		goto fail;
	for (uint32_t g = 0; g < 2; g++) {
		if (hipEventCreateWithFlags(&c->ready_ev[g], hipEventDisableTiming) != hipSuccess
		    || hipEventCreateWithFlags(&c->stage_ev[g], hipEventDisableTiming) != hipSuccess
		    || hipEventRecord(c->ready_ev[g], c->ctl) != hipSuccess // nothing to wait for yet
		    || hipEventRecord(c->stage_ev[g], c->ctl) != hipSuccess)
			goto fail;
		if (hipMalloc(&c->d_rx[g], sizeof(fwd4_rx) * max_ifaces) != hipSuccess
		    || hipMalloc(&c->d_rx6[g], sizeof(fwd4_rx6) * max_ifaces) != hipSuccess
		    || hipMalloc(&c->d_tables[g], sizeof(fwd4_tables)) != hipSuccess)
			goto fail;
		if (hipMemsetAsync(c->d_rx[g], 0, sizeof(fwd4_rx) * max_ifaces, c->ctl) != hipSuccess
		    || hipMemsetAsync(c->d_rx6[g], 0, sizeof(fwd4_rx6) * max_ifaces, c->ctl) != hipSuccess)
			goto fail;
	}
	if (hipMalloc(&c->d_nhf, sizeof(fwd4_nhf) * ((size_t)max_nexthops + 1)) != hipSuccess)
		goto fail;
	if (hipMalloc(&c->d_nhf6, sizeof(fwd4_nhf) * ((size_t)max_nexthops + 1)) != hipSuccess)
		goto fail;
	if (hipMalloc(&c->d_adj6, sizeof(fwd4_adj6) * ((size_t)max_nexthops + 1)) != hipSuccess)
		goto fail;
	if (hipMalloc(&c->d_adj, sizeof(fwd4_adj) * ((size_t)max_nexthops + 1)) != hipSuccess)
		goto fail;
	// every device write goes through the control stream: a plain hipMemset
	// runs on the null stream, which a non-blocking stream does not order with
	if (hipMemsetAsync(c->d_adj, 0, sizeof(fwd4_adj) * ((size_t)max_nexthops + 1), c->ctl) != hipSuccess
	    || hipMemsetAsync(c->d_nhf, 0, sizeof(fwd4_nhf) * ((size_t)max_nexthops + 1), c->ctl) != hipSuccess
	    || hipMemsetAsync(c->d_nhf6, 0, sizeof(fwd4_nhf) * ((size_t)max_nexthops + 1), c->ctl) != hipSuccess
	    || hipMemsetAsync(c->d_adj6, 0, sizeof(fwd4_adj6) * ((size_t)max_nexthops + 1), c->ctl) != hipSuccess)
		goto fail;
	c->nt = FWD4_V_NT; // measured faster on every kernel
	c->stats_on = 1;
	c->wg_per_cu = 0;
	c->fib_fmt = FIB_FMT_24_W2;
	c->ring_cfg = 2; // 16 waves: 2 loaders, 2 storers, 12 compute, 16 slots
	c->host_direct = 1; // measured 1.9x the staged copies
	c->node_ptrs = 0; // staged lines: faster than frames by address, more so with several workers
	c->tile_order = 0;
	c->tile_run = 16;
	c->stage_min_tiles = 4;
	c->res_on = 0;
	c->res_rings = 256; // 32 queues (worker graphs) of 8 rings; workgroups of rings no queue holds leave at once
	c->res_w = 8; // a batch uses up to 8 of them, fewer when many queues are busy (res_budget)
	c->res_ms = 50;
	c->res_nap = 16;
	c->res_tiles = 8; // RES_TILES_PER_WG (measured: DESIGN.md §3.3)
	c->spin_max = 0;
	c->untimed = 0;
	c->time_every = 1;
	c->alloc_contig = 1;
	for (int v = 0; v < 8; v++)
		c->occ_ring[v] = gr_fwd4_ring_occupancy(v, 0, 0);
	c->occ_n = 0;
	ret = -EIO;
	if (upload_tables(c) != 0)
		goto fail;
	*out = c;
	return 0;
fail:
	(void)hipGetLastError();
	gr_hip_fini(c);
	return ret;
}

extern "C" int gr_hip_fini(gr_hip_ctx_t *c) {
	if (c == nullptr)
		return -EINVAL;
	hipSetDevice(c->dev);
	while (!c->queues.empty())
		gr_hip_queue_destroy(c->queues.back());
	res_free(c);
	if (c->ctl)
		hipStreamSynchronize(c->ctl); // the last commits' uploads
	// (every queue is gone: nothing of this context reads them any more)
	for (const host_range &r : c->hregs)
		if (r.ours)
			hreg_global_put(r.host, r.len);
	c->hregs.clear();
	for (vrf_fib &v : c->vrfs) {
		gr_fib4_free(v.rib);
		gr_fib6_free(v.rib6);
		for (int k = 0; k < 2; k++) {
			v.b4[k].free_all();
			v.b6[k].free_all();
		}
	}
	for (uint32_t g = 0; g < 2; g++) {
		hipFree(c->d_rx[g]);
		hipFree(c->d_rx6[g]);
		hipFree(c->d_tables[g]);
	}
	hipFree(c->d_adj6);
	hipFree(c->d_adj);
	hipFree(c->d_nhf);
	hipFree(c->d_nhf6);
	hipFree(c->d_reta);
	hipFree(c->d_vlan_keys);
	hipFree(c->d_vlan_vals);
	for (int i = 0; i < 2; i++) {
		hipHostFree(c->stage[i]);
		if (c->stage_ev[i])
			hipEventDestroy(c->stage_ev[i]);
		if (c->ready_ev[i])
			hipEventDestroy(c->ready_ev[i]);
	}
	if (c->ctl)
		hipStreamDestroy(c->ctl);
	(void)hipGetLastError();
	delete c;
	return 0;
}

// ---------------------------------------------------------------------------
// edges
// ---------------------------------------------------------------------------

static bool edge_ok(uint8_t e) {
	return e == GR_HIP_EDGE_CHAIN || e < GR_HIP_E_COUNT;
}

extern "C" int gr_hip_edges_eth_type(gr_hip_ctx_t *c, uint16_t be_type, uint8_t edge) {
	if (c == nullptr || !(edge_ok(edge) || edge == GR_HIP_EDGE_CHAIN6))
		return -EINVAL;
	std::lock_guard<std::shared_mutex> l(c->mu);
	fwd4_edges &E = c->edges;
	for (uint32_t i = 0; i < E.n_eth_types; i++) {
		if (E.eth_type_be[i] == be_type) {
			E.eth_type_edge[i] = edge;
			hipSetDevice(c->dev);
			int r = quiesce(c);
			return r ? r : upload_tables(c); // only the table reads ether types
		}
	}
	if (E.n_eth_types >= FWD4_MAX_ETH_TYPES)
		return -ENOSPC;
	E.eth_type_be[E.n_eth_types] = be_type;
	E.eth_type_edge[E.n_eth_types] = edge;
	E.n_eth_types++;
	hipSetDevice(c->dev);
	int r = quiesce(c);
	return r ? r : upload_tables(c);
}

#define EDGE_SETTER(fn, field, limit)                                                              \
	extern "C" int fn(gr_hip_ctx_t *c, uint8_t key, uint8_t edge) {                            \
		if (c == nullptr || key >= (limit) || !edge_ok(edge))                              \
			return -EINVAL;                                                            \
		std::lock_guard<std::shared_mutex> l(c->mu);                                              \
		c->edges.field[key] = edge;                                                        \
		hipSetDevice(c->dev);                                                              \
		int r = quiesce(c);                                                                \
		if (r == 0)                                                                        \
			r = upload_views(c, true, 0, 0, true);                                     \
		return r ? r : upload_tables(c);                                                   \
	}
EDGE_SETTER(gr_hip_edges_iface_mode, mode, GR_HIP_IFACE_MODE_COUNT)
EDGE_SETTER(gr_hip_edges_ip_input_nh_type, in_nh, 8)
EDGE_SETTER(gr_hip_edges_ip_output_nh_type, out_nh, 8)
EDGE_SETTER(gr_hip_edges_ip_output_iface_type, out_iface, 8)
EDGE_SETTER(gr_hip_edges_iface_output_type, iout_type, 8)
EDGE_SETTER(gr_hip_edges_ip6_input_nh_type, in6_nh, 8)
EDGE_SETTER(gr_hip_edges_ip6_output_nh_type, out6_nh, 8)
EDGE_SETTER(gr_hip_edges_ip6_output_iface_type, out6_iface, 8)

extern "C" int gr_hip_edges_get(gr_hip_ctx_t *c, int table, uint16_t key) {
	if (c == nullptr)
		return -EINVAL;
	std::shared_lock<std::shared_mutex> l(c->mu);
	const fwd4_edges &E = c->edges;
	const uint8_t *t = nullptr;
	uint32_t lim = 8;
	switch (table) {
	case GR_HIP_EDGES_ETH_TYPE: {
		int e = GR_HIP_E_ETH_INPUT_UNKNOWN_TYPE; // l2l3_edges default (eth_input.c:24)
		for (uint32_t i = 0; i < E.n_eth_types; i++)
			if (E.eth_type_be[i] == key)
				e = E.eth_type_edge[i];
		return e;
	}
	case GR_HIP_EDGES_IFACE_MODE:
		t = E.mode;
		lim = GR_HIP_IFACE_MODE_COUNT;
		break;
	case GR_HIP_EDGES_IP_INPUT_NH_TYPE:
		t = E.in_nh;
		break;
	case GR_HIP_EDGES_IP_OUTPUT_NH_TYPE:
		t = E.out_nh;
		break;
	case GR_HIP_EDGES_IP_OUTPUT_IFACE_TYPE:
		t = E.out_iface;
		break;
	case GR_HIP_EDGES_IFACE_OUTPUT_TYPE:
		t = E.iout_type;
		break;
	case GR_HIP_EDGES_IP6_INPUT_NH_TYPE:
		t = E.in6_nh;
		break;
	case GR_HIP_EDGES_IP6_OUTPUT_NH_TYPE:
		t = E.out6_nh;
		break;
	case GR_HIP_EDGES_IP6_OUTPUT_IFACE_TYPE:
		t = E.out6_iface;
		break;
	default:
		return -EINVAL;
	}
	return key < lim ? t[key] : -EINVAL;
}

// ---------------------------------------------------------------------------
// devices
// ---------------------------------------------------------------------------

extern "C" int gr_hip_device_count(void) {
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess) {
		(void)hipGetLastError();
		return -ENODEV;
	}
	return n;
}

extern "C" int gr_hip_device_numa_node(int dev) {
	char bus[64];
	if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) {
		(void)hipGetLastError();
		return -ENODEV;
	}
	for (char *p = bus; *p; p++) // sysfs names are lower case
		if (*p >= 'A' && *p <= 'F')
			*p = (char)(*p - 'A' + 'a');
	char path[160];
	snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
	FILE *f = fopen(path, "r");
	if (f == nullptr)
		return -ENOENT;
	int node = -1;
	const int got = fscanf(f, "%d", &node);
	fclose(f);
	if (got != 1)
		return -EIO;
	return node < 0 ? 0 : node; // -1: no NUMA information (one node)
}

// ---------------------------------------------------------------------------
// mirrors
// ---------------------------------------------------------------------------

static int upload_vlans(gr_hip_ctx *c) {
	uint32_t n = 0;
	for (const gr_hip_iface &i : c->ifaces)
		n += i.id != 0 && i.type == GR_HIP_IFACE_TYPE_VLAN;
	uint32_t cap = 16;
	while (cap < 2 * n)
		cap *= 2;
	std::vector<uint32_t> keys(cap, 0);
	std::vector<uint16_t> vals(cap, 0);
	for (const gr_hip_iface &i : c->ifaces) {
		if (i.id == 0 || i.type != GR_HIP_IFACE_TYPE_VLAN)
			continue;
		uint32_t key = (((uint32_t)i.parent_id << 16) | i.vlan_id) + 1;
		uint32_t h = (key * 0x9e3779b1u) & (cap - 1);
		while (keys[h] != 0 && keys[h] != key)
			h = (h + 1) & (cap - 1);
		keys[h] = key;
		vals[h] = i.id;
	}
	if (cap != c->vlan_cap) {
		hipFree(c->d_vlan_keys);
		hipFree(c->d_vlan_vals);
		c->d_vlan_keys = nullptr;
		c->d_vlan_vals = nullptr;
		c->vlan_cap = 0;
		HCK(hipMalloc(&c->d_vlan_keys, cap * sizeof(uint32_t)));
		HCK(hipMalloc(&c->d_vlan_vals, cap * sizeof(uint16_t)));
		c->vlan_cap = cap;
	}
	int r = h2d(c, c->d_vlan_keys, keys.data(), cap * sizeof(uint32_t));
	if (r == 0)
		r = h2d(c, c->d_vlan_vals, vals.data(), cap * sizeof(uint16_t));
	if (r == 0)
		r = ctl_sync(c); // the vectors go out of scope
	if (r == 0) {
		c->vlan_keys_h = std::move(keys);
		c->vlan_vals_h = std::move(vals);
		r = upload_tables(c);
	}
	return r;
}

extern "C" int gr_hip_iface_set(gr_hip_ctx_t *c, const struct gr_hip_iface *ifs, uint32_t n) {
	if (c == nullptr || (ifs == nullptr && n))
		return -EINVAL;
	for (uint32_t i = 0; i < n; i++)
		if (ifs[i].id == 0 || ifs[i].id >= c->max_ifaces)
			return -EINVAL;
	std::lock_guard<std::shared_mutex> l(c->mu);
	hipSetDevice(c->dev);
	bool vlans = false;
	for (uint32_t i = 0; i < n; i++) {
		vlans |= ifs[i].type == GR_HIP_IFACE_TYPE_VLAN
			|| c->ifaces[ifs[i].id].type == GR_HIP_IFACE_TYPE_VLAN;
		c->ifaces[ifs[i].id] = ifs[i];
	}
	int r = quiesce(c);
	if (r == 0) // ifaces feed every RX view and every adjacency
		r = upload_views(c, true, 0, 0, true);
	if (r == 0 && (vlans || c->vlan_cap == 0))
		r = upload_vlans(c);
	return r;
}

extern "C" int gr_hip_iface_del(gr_hip_ctx_t *c, uint16_t id) {
	if (c == nullptr || id == 0 || id >= c->max_ifaces)
		return -EINVAL;
	std::lock_guard<std::shared_mutex> l(c->mu);
	hipSetDevice(c->dev);
	bool vlan = c->ifaces[id].type == GR_HIP_IFACE_TYPE_VLAN;
	c->ifaces[id] = gr_hip_iface {};
	int r = quiesce(c);
	if (r == 0)
		r = upload_views(c, true, 0, 0, true);
	if (r == 0 && vlan)
		r = upload_vlans(c);
	return r;
}

extern "C" int gr_hip_nh_set(gr_hip_ctx_t *c, uint32_t first, const struct gr_hip_nh *nh, uint32_t n) {
	if (c == nullptr || first == 0 || (nh == nullptr && n)
	    || (uint64_t)first + n > (uint64_t)c->max_nh + 1)
		return -EINVAL;
	std::lock_guard<std::shared_mutex> l(c->mu);
	hipSetDevice(c->dev);
	memcpy(&c->nh[first], nh, (size_t)n * sizeof(*nh));
	if (n && first + n - 1 > c->nh_hi)
		c->nh_hi = first + n - 1;
	int r = quiesce(c);
	if (r == 0 && n)
		r = upload_views(c, false, first, n, true);
	return r;
}

extern "C" int gr_hip_reta_set(gr_hip_ctx_t *c, uint32_t first, const uint32_t *slots, uint32_t n) {
	if (c == nullptr || (slots == nullptr && n) || (uint64_t)first + n > (1ull << 31))
		return -EINVAL;
	std::lock_guard<std::shared_mutex> l(c->mu);
	hipSetDevice(c->dev);
	if ((uint64_t)first + n > c->reta.size())
		c->reta.resize((size_t)first + n, 0);
	memcpy(&c->reta[first], slots, (size_t)n * sizeof(*slots));
	int r = quiesce(c);
	if (r != 0)
		return r;
	if (c->reta.size() > c->d_reta_cap) {
		uint32_t cap = c->d_reta_cap ? c->d_reta_cap : 4096;
		while (cap < c->reta.size())
			cap *= 2;
		uint32_t *d = nullptr;
		HCK(hipStreamSynchronize(c->ctl));
		HCK(hipMalloc(&d, (size_t)cap * sizeof(uint32_t)));
		HCK(hipMemsetAsync(d, 0, (size_t)cap * sizeof(uint32_t), c->ctl));
		hipFree(c->d_reta);
		c->d_reta = d;
		c->d_reta_cap = cap;
		r = h2d(c, c->d_reta, c->reta.data(), c->reta.size() * sizeof(uint32_t));
	} else {
		r = h2d(c, c->d_reta + first, &c->reta[first], (size_t)n * sizeof(uint32_t));
	}
	if (r == 0)
		r = ctl_sync(c);
	if (r == 0)
		r = upload_tables(c);
	return r;
}

// ---------------------------------------------------------------------------
// FIB
// ---------------------------------------------------------------------------

// FIB publication is double-buffered, the MI355X analogue of grout's RCU
// (rte_fib with an RCU QSBR variable, modules/ip/control/route.c:87-95, and
// rte_rcu_qsbr_synchronize before a FIB is freed, :766): every VRF keeps two
// device copies of its tables, and the context two generations of the RX
// views and table block a launch reads. A submit takes the current
// generation (under the shared lock, for microseconds), so each launch sees
// one table from its first packet to its last. A commit
//   1. with c->mu held shared (submitters keep going), stages what the
//      unpublished copy misses and the other generation's views in pinned
//      memory, and enqueues on the control stream: a wait for the launches
//      submitted before the previous publication (the only ones that can
//      still read that copy: `retire` events), the uploads, and the
//      generation's `ready_ev`;
//   2. publishes: flips the generation and records `retire` on every queue,
//      with c->mu held exclusively for a few microseconds.
// Nothing waits on the host: the first launch of each queue after a
// publication makes its stream wait for `ready_ev` (launch()), so the
// datapath sees the new table as soon as it is uploaded and the commit
// returns once the work is enqueued. Route adds and deletes only touch the
// host RIB (fib_mu).

static uint64_t now_ns_host() {
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return (uint64_t)t.tv_sec * 1000000000u + (uint64_t)t.tv_nsec;
}

static uint64_t now_us() {
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return (uint64_t)t.tv_sec * 1000000u + (uint64_t)t.tv_nsec / 1000u;
}

// Wait, on the control stream, for every launch submitted before the last
// publication.
static int retire_wait(gr_hip_ctx *c) {
	for (gr_hip_queue *q : c->queues) {
		HCK(hipStreamWaitEvent(c->ctl, q->retire, 0));
		if (const int r = res_wait(q, q->res_retire)) // resident batches posted before it: on the host
			return r;
	}
	return 0;
}

// Point generation g at every VRF's published copies (the caller then points
// it at the copy it writes).
static void views_follow_published(gr_hip_ctx *c, uint32_t g) {
	for (vrf_fib &v : c->vrfs) {
		v.sel4[g] = (uint8_t)v.pub4;
		v.sel6[g] = (uint8_t)v.pub6;
	}
}

static void count_v6(gr_hip_ctx *c);

// Step 2: flip to generation g, which the caller has written. Takes c->mu
// exclusively; `then` runs under it (the per-VRF published index).
template <typename F>
static int publish(gr_hip_ctx *c, uint32_t g, F then) {
	std::lock_guard<std::shared_mutex> l(c->mu);
	c->gen = g;
	c->serial++;
	then();
	count_v6(c);
	for (gr_hip_queue *q : c->queues) {
		HCK(hipEventRecord(q->retire, q->s));
		q->res_retire = q->res_posted;
	}
	return 0;
}

// Host staging for one commit's uploads: the bytes of every (destination,
// length) write packed into a pinned buffer, then one DMA per write on the
// control stream. Nothing is synchronised: the two staging buffers are used
// in turn, and a commit waits only until the one it takes is free again
// (the commit before last has uploaded).
struct stager {
	gr_hip_ctx *c;
	std::vector<uint8_t> buf;
	struct op {
		void *dst;
		size_t off, n;
	};
	std::vector<op> ops;

	explicit stager(gr_hip_ctx *c_) : c(c_) {}
	// room for `count` entries going to dst; valid until the next add
	template <typename E>
	E *add(E *dst, size_t count) {
		const size_t off = (buf.size() + 15) & ~(size_t)15;
		buf.resize(off + count * sizeof(E));
		ops.push_back({dst, off, count * sizeof(E)});
		return reinterpret_cast<E *>(buf.data() + off);
	}
	int flush() { // enqueue on the control stream
		if (buf.empty())
			return 0;
		const uint32_t i = c->stage_i ^= 1;
		HCK(hipEventSynchronize(c->stage_ev[i]));
		if (buf.size() > c->stage_cap[i]) {
			hipHostFree(c->stage[i]);
			c->stage[i] = nullptr;
			c->stage_cap[i] = 0;
			HCK(hipHostMalloc(reinterpret_cast<void **>(&c->stage[i]), buf.size(), hipHostMallocDefault));
			c->stage_cap[i] = buf.size();
		}
		memcpy(c->stage[i], buf.data(), buf.size());
		for (const op &o : ops)
			HCK(hipMemcpyAsync(o.dst, c->stage[i] + o.off, o.n, hipMemcpyHostToDevice, c->ctl));
		HCK(hipEventRecord(c->stage_ev[i], c->ctl));
		return 0;
	}
};

// Stage generation g's RX views (IPv4 and IPv6, every iface).
static void stage_rx(stager &st, gr_hip_ctx *c, uint32_t g) {
	for (uint32_t i = 0; i < c->max_ifaces; i++) {
		c->rx[g][i] = make_rx(c, i, g);
		c->rx6[g][i] = make_rx6(c, i, g);
	}
	c->top6[g] = common_top6(c, g);
	memcpy(st.add(c->d_rx[g], c->max_ifaces), c->rx[g].data(), sizeof(fwd4_rx) * c->max_ifaces);
	memcpy(st.add(c->d_rx6[g], c->max_ifaces), c->rx6[g].data(), sizeof(fwd4_rx6) * c->max_ifaces);
}

extern "C" int gr_hip_fib4_create(gr_hip_ctx_t *c, uint16_t vrf, uint32_t max_routes, uint32_t num_tbl8) {
	if (c == nullptr || vrf == 0 || vrf >= c->max_ifaces)
		return -EINVAL;
	std::lock_guard<std::mutex> f(c->fib_mu);
	std::lock_guard<std::shared_mutex> l(c->mu);
	hipSetDevice(c->dev);
	vrf_fib &v = c->vrfs[vrf];
	if (v.rib != nullptr)
		return -EEXIST;
	if (num_tbl8 == 0) // fib4_auto_tbl8, modules/ip/control/route.c:38-41
		num_tbl8 = max_routes / 500 < 256 ? 256 : max_routes / 500;
	v.rib = gr_fib4_new(max_routes, num_tbl8);
	if (v.rib == nullptr)
		return -ENOMEM;
	v.num_tbl8 = num_tbl8;
	// device copies are allocated by the commits, in the format they pick
	gr_fib4_dirty_clear(v.rib);
	return 0;
}

extern "C" int gr_hip_fib4_destroy(gr_hip_ctx_t *c, uint16_t vrf) {
	if (c == nullptr || vrf == 0 || vrf >= c->max_ifaces)
		return -EINVAL;
	std::lock_guard<std::mutex> f(c->fib_mu);
	std::lock_guard<std::shared_mutex> l(c->mu);
	hipSetDevice(c->dev);
	vrf_fib &v = c->vrfs[vrf];
	if (v.rib == nullptr)
		return -ENOENT;
	gr_fib4 *rib = v.rib;
	v.rib = nullptr; // make_rx() stops pointing at it
	int r = quiesce(c);
	if (r == 0)
		r = upload_views(c, true, 0, 0, false);
	if (r != 0) {
		v.rib = rib;
		return r;
	}
	v.b4[0].free_all();
	v.b4[1].free_all();
	gr_fib4_free(rib);
	v.reset4();
	return 0;
}

extern "C" int gr_hip_route4_add(gr_hip_ctx_t *c, const struct gr_hip_route4 *rt, uint32_t n, int replace) {
	if (c == nullptr || (rt == nullptr && n))
		return -EINVAL;
	std::lock_guard<std::mutex> f(c->fib_mu); // the host RIB only: launches go on
	for (uint32_t i = 0; i < n; i++) {
		if (rt[i].vrf_id == 0 || rt[i].vrf_id >= c->max_ifaces || rt[i].nh == 0
		    || rt[i].nh > c->max_nh)
			return -EINVAL;
		vrf_fib &v = c->vrfs[rt[i].vrf_id];
		if (v.rib == nullptr)
			return -ENONET;
		int r = gr_fib4_add(v.rib, __builtin_bswap32(rt[i].ip), rt[i].prefixlen, rt[i].nh, replace);
		if (r < 0)
			return r;
		if (rt[i].nh > v.max_slot)
			v.max_slot = rt[i].nh;
	}
	return 0;
}

extern "C" int gr_hip_route4_del(gr_hip_ctx_t *c, uint16_t vrf, uint32_t ip, uint8_t len) {
	if (c == nullptr || vrf == 0 || vrf >= c->max_ifaces)
		return -EINVAL;
	std::lock_guard<std::mutex> f(c->fib_mu);
	vrf_fib &v = c->vrfs[vrf];
	if (v.rib == nullptr)
		return -ENONET;
	return gr_fib4_del(v.rib, __builtin_bswap32(ip), len);
}

static uint16_t to16(uint32_t e) { // fib4.h 4-byte entry -> 2-byte entry
	return (uint16_t)((e & GR_FIB4_EXT) ? (0x8000u | (e & 0x7fffu)) : e);
}

// Sorted, disjoint union of sorted range lists; ranges less than `gap`
// entries apart are merged too (re-writing unchanged entries in between
// costs less than one more DMA).
static std::vector<gr_fib4_range> range_union(const std::vector<gr_fib4_range> &a,
					      const std::vector<gr_fib4_range> &b, uint32_t gap) {
	std::vector<gr_fib4_range> all(a);
	all.insert(all.end(), b.begin(), b.end());
	std::sort(all.begin(), all.end(), [](const gr_fib4_range &x, const gr_fib4_range &y) { return x.lo < y.lo; });
	std::vector<gr_fib4_range> out;
	for (const gr_fib4_range &r : all) {
		if (!out.empty() && (uint64_t)r.lo <= (uint64_t)out.back().hi + gap)
			out.back().hi = std::max(out.back().hi, r.hi);
		else
			out.push_back(r);
	}
	return out;
}

static std::vector<uint32_t> group_union(const std::vector<uint32_t> &a, const std::vector<uint32_t> &b) {
	std::vector<uint32_t> all(a);
	all.insert(all.end(), b.begin(), b.end());
	std::sort(all.begin(), all.end());
	all.erase(std::unique(all.begin(), all.end()), all.end());
	return all;
}

// Stage runs of tbl8 groups (sorted) of a host table converted entry by entry.
template <typename E, typename Conv>
static void stage_groups(stager &st, E *dev, const uint32_t *t8, const std::vector<uint32_t> &gs, Conv conv) {
	for (size_t i = 0; i < gs.size();) {
		size_t j = i + 1;
		while (j < gs.size() && gs[j] == gs[j - 1] + 1)
			j++;
		E *h = st.add(dev + (size_t)gs[i] * 256, (j - i) * 256);
		const uint32_t *src = t8 + (size_t)gs[i] * 256;
		for (size_t k = 0; k < (j - i) * 256; k++)
			h[k] = conv(src[k]);
		i = j;
	}
}

// Large device arrays (the FIB tables, batch buffers and their placement
// candidates) are asked of the driver physically contiguous first
// (hipDeviceMallocContiguous), which maps them with large fragments: the
// kernel's streams and gathers then translate fast whatever pages they land
// on. Plain allocations are placed at random in that respect, and a slow
// pairing of frames and output lines stalls on address translation (the
// L1 TLB's in-flight limit: TCP_UTCL1_STALL_INFLIGHT_MAX, DESIGN.md §6
// "placement"). hipMalloc when the driver cannot (or "alloc_contig" 0).
static hipError_t dev_alloc(const gr_hip_ctx *c, void **p, size_t sz) {
	if (c->alloc_contig) {
		if (hipExtMallocWithFlags(p, sz, hipDeviceMallocContiguous) == hipSuccess)
			return hipSuccess;
		(void)hipGetLastError();
	}
	return hipMalloc(p, sz);
}
#define fib_malloc(p, sz) dev_alloc(c, (void **)(p), (sz))

// Allocate the device arrays copy `b` needs in format `fmt`.
static int fib4_buf_alloc(gr_hip_ctx *c, fib4_buf &b, int fmt, uint32_t num_tbl8) {
	if (fmt != FIB_FMT_24 && b.d8_16 == nullptr)
		HCK(fib_malloc(&b.d8_16, sizeof(uint16_t) * 256 * (size_t)num_tbl8));
	if (fmt == FIB_FMT_24_W2 && b.d24_16 == nullptr)
		HCK(fib_malloc(&b.d24_16, sizeof(uint16_t) * GR_FIB4_TBL24_ENTRIES));
	if (fmt == FIB_FMT_16_8_8 && b.d16 == nullptr) // top + the worst case of one chunk per /16
		HCK(fib_malloc(&b.d16, sizeof(uint32_t) * 65536 + sizeof(uint16_t) * 256 * 65536));
	if (fmt == FIB_FMT_24 && b.d24 == nullptr) {
		HCK(fib_malloc(&b.d24, sizeof(uint32_t) * GR_FIB4_TBL24_ENTRIES));
		HCK(fib_malloc(&b.d8, sizeof(uint32_t) * 256 * (size_t)num_tbl8));
	}
	return 0;
}

// Stage the tbl24 ranges `rs` and tbl8 groups `gs` of the host table into
// copy `b` in format `fmt` (DIR-16-8-8: the /16s the ranges touch, chunk
// assignments updated on the way).
static void fib4_stage(stager &st, vrf_fib &v, fib4_buf &b, int fmt, const std::vector<gr_fib4_range> &rs,
		       const std::vector<uint32_t> &gs) {
	const uint32_t *t24 = gr_fib4_tbl24(v.rib);
	const uint32_t *t8 = gr_fib4_tbl8(v.rib);
	if (fmt == FIB_FMT_24_W2) {
		for (const gr_fib4_range &r : rs) {
			uint16_t *h = st.add(b.d24_16 + r.lo, r.hi - r.lo);
			for (uint32_t i = r.lo; i < r.hi; i++)
				h[i - r.lo] = to16(t24[i]);
		}
		stage_groups(st, b.d8_16, t8, gs, to16);
	} else if (fmt == FIB_FMT_16_8_8) {
		const size_t top_n = 65536, chunk_n = 256;
		uint16_t *chunks_dev = reinterpret_cast<uint16_t *>(b.d16 + top_n);
		// the /16s the ranges touch, as sorted disjoint runs
		std::vector<gr_fib4_range> ks;
		for (const gr_fib4_range &r : rs) {
			const uint32_t k_lo = r.lo >> 8, k_hi = (r.hi + 255) >> 8;
			if (!ks.empty() && k_lo <= ks.back().hi)
				ks.back().hi = std::max(ks.back().hi, k_hi);
			else
				ks.push_back({k_lo, k_hi});
		}
		std::vector<std::pair<uint32_t, uint32_t>> chunks; // (chunk, /16) rewritten
		for (const gr_fib4_range &kr : ks) {
			uint32_t *top = st.add(b.d16 + kr.lo, kr.hi - kr.lo);
			for (uint32_t k = kr.lo; k < kr.hi; k++) {
				const uint32_t *e = t24 + (size_t)k * 256;
				bool uniform = !(e[0] & GR_FIB4_EXT);
				for (uint32_t j = 1; uniform && j < 256; j++)
					uniform = e[j] == e[0];
				if (uniform) {
					top[k - kr.lo] = to16(e[0]);
					if (v.chunk_of[k] >= 0) {
						v.chunk_free.push_back((uint32_t)v.chunk_of[k]);
						v.chunk_of[k] = -1;
						v.n_chunks--;
					}
					continue;
				}
				if (v.chunk_of[k] < 0) {
					v.chunk_of[k] = (int32_t)v.chunk_free.back();
					v.chunk_free.pop_back();
					v.n_chunks++;
				}
				top[k - kr.lo] = 0x80000000u | (uint32_t)v.chunk_of[k];
				chunks.push_back({(uint32_t)v.chunk_of[k], k});
			}
		}
		std::sort(chunks.begin(), chunks.end());
		for (size_t i = 0; i < chunks.size();) { // runs of consecutive chunks
			size_t j = i + 1;
			while (j < chunks.size() && chunks[j].first == chunks[j - 1].first + 1)
				j++;
			uint16_t *h = st.add(chunks_dev + (size_t)chunks[i].first * chunk_n, (j - i) * chunk_n);
			for (size_t m = i; m < j; m++)
				for (uint32_t e = 0; e < chunk_n; e++)
					h[(m - i) * chunk_n + e] = to16(t24[(size_t)chunks[m].second * 256 + e]);
			i = j;
		}
		stage_groups(st, b.d8_16, t8, gs, to16);
	} else {
		for (const gr_fib4_range &r : rs)
			memcpy(st.add(b.d24 + r.lo, r.hi - r.lo), t24 + r.lo, (size_t)(r.hi - r.lo) * sizeof(uint32_t));
		stage_groups(st, b.d8, t8, gs, [](uint32_t e) { return e; });
	}
}

// Publish the VRF's IPv4 FIB as the host RIB holds it now: write the
// unpublished copy (what changed since it was last written: its pending
// list and this commit's dirty ranges, in the format the tables fit —
// 2-byte entries while every nexthop slot and tbl8 group index fits 15
// bits, else 4-byte), then flip (see the comment above retire_wait).
extern "C" int gr_hip_fib4_commit(gr_hip_ctx_t *c, uint16_t vrf) {
	if (c == nullptr || vrf == 0 || vrf >= c->max_ifaces)
		return -EINVAL;
	std::lock_guard<std::mutex> f(c->fib_mu);
	hipSetDevice(c->dev);
	vrf_fib &v = c->vrfs[vrf];
	if (v.rib == nullptr)
		return -ENONET;
	const uint64_t t0 = now_us();
	const bool fits16 = v.max_slot <= 0x7fff && v.num_tbl8 <= 0x8000;
	const int want = fits16 ? c->fib_fmt : FIB_FMT_24;
	const int w = v.pub4 ^ 1;
	fib4_buf &b = v.b4[w];
	// this commit's changes
	std::vector<gr_fib4_range> d24(4096);
	std::vector<uint32_t> d8(v.num_tbl8);
	int n24 = gr_fib4_dirty_tbl24(v.rib, d24.data(), (uint32_t)d24.size());
	int n8 = gr_fib4_dirty_tbl8(v.rib, d8.data(), v.num_tbl8);
	const bool d_all = n24 < 0 || n8 < 0;
	d24.resize(n24 < 0 ? 0 : (size_t)n24);
	d8.resize(n8 < 0 ? 0 : (size_t)n8);
	if (!d_all && d24.empty() && d8.empty() && v.uploaded() && v.pub().fmt == want)
		return 0; // nothing to publish
	const bool full = d_all || v.pend_all || !b.up || b.fmt != want;
	std::vector<gr_fib4_range> rs;
	std::vector<uint32_t> gs;
	if (full) {
		rs.push_back({0, GR_FIB4_TBL24_ENTRIES});
		gs.resize(v.num_tbl8);
		for (uint32_t g = 0; g < v.num_tbl8; g++)
			gs[g] = g;
	} else {
		rs = range_union(v.pend24, d24, 2048);
		gs = group_union(v.pend8, d8);
	}
	const uint32_t B = c->gen ^ 1; // the generation this commit writes
	int r;
	uint64_t t1 = t0;
	{
		std::shared_lock<std::shared_mutex> l(c->mu); // submitters go on
		r = fib4_buf_alloc(c, b, want, v.num_tbl8);
		if (r != 0)
			return r;
		if (want == FIB_FMT_16_8_8 && (v.chunk_of.empty() || (full && !(v.pub().up && v.pub().fmt == FIB_FMT_16_8_8)))) {
			// no copy uses the chunk assignment: start afresh
			v.chunk_of.assign(65536, -1);
			v.chunk_free.clear();
			for (uint32_t k = 0; k < 65536; k++)
				v.chunk_free.push_back(65535 - k);
			v.n_chunks = 0;
		}
		stager st(c);
		fib4_stage(st, v, b, want, rs, gs);
		b.fmt = want;
		b.up = true;
		views_follow_published(c, B);
		v.sel4[B] = (uint8_t)w;
		stage_rx(st, c, B);
		t1 = now_us();
		r = retire_wait(c); // no launch may still read copy w or generation B's views
		if (r == 0)
			r = st.flush();
		if (r == 0 && hipEventRecord(c->ready_ev[B], c->ctl) != hipSuccess) // launches of B wait for it
			r = -EIO;
		if (r != 0) {
			b.up = false; // half written: rewritten in full next time
			views_follow_published(c, B);
			return r;
		}
	}
	gr_fib4_dirty_clear(v.rib);
	const uint64_t t2 = now_us();
	r = publish(c, B, [&] {
		const bool old_up = v.pub().up;
		v.pub4 = w;
		// the copy just unpublished misses this commit's changes
		v.pend_all = d_all || !old_up;
		v.pend24 = std::move(d24);
		v.pend8 = std::move(d8);
	});
	const uint64_t t3 = now_us();
	c->commit_us[0].store((uint32_t)(t1 - t0), std::memory_order_relaxed);
	c->commit_us[1].store((uint32_t)(t2 - t1), std::memory_order_relaxed);
	c->commit_us[2].store((uint32_t)(t3 - t2), std::memory_order_relaxed);
	return r;
}

extern "C" int gr_hip_fib4_lookup_host(gr_hip_ctx_t *c, uint16_t vrf, uint32_t ip_be, uint32_t *nh) {
	if (c == nullptr || nh == nullptr || vrf == 0 || vrf >= c->max_ifaces)
		return -EINVAL;
	std::lock_guard<std::mutex> f(c->fib_mu);
	vrf_fib &v = c->vrfs[vrf];
	if (v.rib == nullptr)
		return -ENONET;
	*nh = gr_fib4_lookup(v.rib, __builtin_bswap32(ip_be));
	return 0;
}

extern "C" int gr_hip_fib4_info(gr_hip_ctx_t *c, uint16_t vrf, uint32_t *n_routes, uint32_t *tbl8_used, uint64_t *bytes) {
	if (c == nullptr || vrf == 0 || vrf >= c->max_ifaces)
		return -EINVAL;
	std::lock_guard<std::mutex> f(c->fib_mu);
	vrf_fib &v = c->vrfs[vrf];
	if (v.rib == nullptr)
		return -ENONET;
	if (n_routes)
		*n_routes = gr_fib4_n_routes(v.rib);
	if (tbl8_used)
		*tbl8_used = gr_fib4_tbl8_used(v.rib);
	const int fmt = v.pub().fmt;
	if (bytes) // device bytes a lookup can touch (the published copy)
		*bytes = fmt == FIB_FMT_16_8_8 ? 4ull * 65536 + 512ull * v.n_chunks + 512ull * v.num_tbl8
			 : fmt == FIB_FMT_24_W2 ? 2ull * GR_FIB4_TBL24_ENTRIES + 512ull * v.num_tbl8
						: 4ull * GR_FIB4_TBL24_ENTRIES + 1024ull * v.num_tbl8;
	return 0;
}

// ---------------------------------------------------------------------------
// FIB6
// ---------------------------------------------------------------------------

// addr6_linklocal_scope (modules/ip6/control/ip6.h:23-36): a link-local
// address is keyed with the iface id in bytes 2-3.
static void scope6(uint8_t out[16], const uint8_t ip[16], uint16_t iface_id) {
	memcpy(out, ip, 16);
	if (ip[0] == 0xfe && (ip[1] & 0xc0) == 0x80) {
		out[2] = (uint8_t)(iface_id >> 8);
		out[3] = (uint8_t)iface_id;
	}
}

// IPv6 routes published, all VRFs: the launches stage the IPv6 fast
// adjacencies in LDS only when there are some. Caller holds c->mu exclusively.
static void count_v6(gr_hip_ctx *c) {
	uint32_t n = 0;
	for (const vrf_fib &v : c->vrfs)
		if (v.rib6 != nullptr && v.uploaded6())
			n += gr_fib6_n_routes(v.rib6);
	c->v6_routes = n;
}

extern "C" int gr_hip_fib6_create(gr_hip_ctx_t *c, uint16_t vrf, uint32_t max_routes, uint32_t num_tbl8) {
	if (c == nullptr || vrf == 0 || vrf >= c->max_ifaces || max_routes == 0)
		return -EINVAL;
	std::lock_guard<std::mutex> f(c->fib_mu);
	std::lock_guard<std::shared_mutex> l(c->mu);
	vrf_fib &v = c->vrfs[vrf];
	if (v.rib6 != nullptr)
		return -EEXIST;
	v.rib6 = gr_fib6_new(max_routes, num_tbl8);
	return v.rib6 ? 0 : -ENOMEM;
}

extern "C" int gr_hip_fib6_destroy(gr_hip_ctx_t *c, uint16_t vrf) {
	if (c == nullptr || vrf == 0 || vrf >= c->max_ifaces)
		return -EINVAL;
	std::lock_guard<std::mutex> f(c->fib_mu);
	std::lock_guard<std::shared_mutex> l(c->mu);
	hipSetDevice(c->dev);
	vrf_fib &v = c->vrfs[vrf];
	if (v.rib6 == nullptr)
		return -ENOENT;
	gr_fib6_t *rib6 = v.rib6;
	v.rib6 = nullptr; // make_rx6() stops pointing at it
	int r = quiesce(c);
	if (r == 0)
		r = upload_views(c, true, 0, 0, false);
	if (r != 0) {
		v.rib6 = rib6;
		return r;
	}
	v.b6[0].free_all();
	v.b6[1].free_all();
	v.pub6 = 1;
	v.sel6[0] = v.sel6[1] = 1;
	for (auto &p : v.pend6)
		p.clear();
	v.pend6_all = true;
	gr_fib6_free(rib6);
	count_v6(c);
	return 0;
}

extern "C" int gr_hip_route6_add(gr_hip_ctx_t *c, const struct gr_hip_route6 *rt, uint32_t n, int replace) {
	if (c == nullptr || (rt == nullptr && n))
		return -EINVAL;
	std::lock_guard<std::mutex> f(c->fib_mu); // the host RIB only
	for (uint32_t i = 0; i < n; i++) {
		if (rt[i].vrf_id == 0 || rt[i].vrf_id >= c->max_ifaces || rt[i].nh == 0 || rt[i].nh > c->max_nh
		    || rt[i].prefixlen > 128)
			return -EINVAL;
		vrf_fib &v = c->vrfs[rt[i].vrf_id];
		if (v.rib6 == nullptr)
			return -ENONET;
		uint8_t key[16];
		scope6(key, rt[i].ip, rt[i].iface_id);
		int r = gr_fib6_add(v.rib6, key, rt[i].prefixlen, rt[i].nh, replace);
		if (r < 0)
			return r;
	}
	return 0;
}

extern "C" int gr_hip_route6_del(gr_hip_ctx_t *c, uint16_t vrf, uint16_t iface_id, const uint8_t ip[16], uint8_t len) {
	if (c == nullptr || vrf == 0 || vrf >= c->max_ifaces || ip == nullptr || len > 128)
		return -EINVAL;
	std::lock_guard<std::mutex> f(c->fib_mu);
	vrf_fib &v = c->vrfs[vrf];
	if (v.rib6 == nullptr)
		return -ENONET;
	uint8_t key[16];
	scope6(key, ip, iface_id);
	return gr_fib6_del(v.rib6, key, len);
}

// Sorted, duplicate-free union of two index lists.
static std::vector<uint32_t> index_union(const std::vector<uint32_t> &a, const std::vector<uint32_t> &b) {
	std::vector<uint32_t> all(a);
	all.insert(all.end(), b.begin(), b.end());
	std::sort(all.begin(), all.end());
	all.erase(std::unique(all.begin(), all.end()), all.end());
	return all;
}

// Stage runs of consecutive indexes of a host array of `unit`-element items
// into the same places of a device array.
template <typename E>
static void stage_runs(stager &st, E *dev, const E *host, size_t unit, const std::vector<uint32_t> &idx) {
	for (size_t i = 0; i < idx.size();) {
		size_t j = i + 1;
		while (j < idx.size() && idx[j] == idx[j - 1] + 1)
			j++;
		memcpy(st.add(dev + (size_t)idx[i] * unit, (j - i) * unit), host + (size_t)idx[i] * unit,
		       (j - i) * unit * sizeof(E));
		i = j;
	}
}

// Publish the VRF's IPv6 trie: bring the host image up to date along the
// paths the route changes touched (gr_fib6_build), write into the
// unpublished copy what it misses -- its pending lists (the previous
// commit's changes) and this commit's: first-level entries, 1 KiB group
// slots, skip nodes -- then flip like gr_hip_fib4_commit. The first commit
// into a copy writes it whole.
extern "C" int gr_hip_fib6_commit(gr_hip_ctx_t *c, uint16_t vrf) {
	if (c == nullptr || vrf == 0 || vrf >= c->max_ifaces)
		return -EINVAL;
	std::lock_guard<std::mutex> f(c->fib_mu);
	hipSetDevice(c->dev);
	vrf_fib &v = c->vrfs[vrf];
	if (v.rib6 == nullptr)
		return -ENONET;
	const uint64_t t0 = now_us();
	int r = gr_fib6_build(v.rib6);
	if (r < 0)
		return r;
	// this commit's changes
	std::vector<uint32_t> d[3];
	bool d_all = false;
	for (int k = 0; k < 3; k++) {
		const uint32_t *l = nullptr;
		uint32_t n = 0;
		const int all = gr_fib6_dirty(v.rib6, k, &l, &n);
		if (all < 0)
			return all;
		d_all |= all != 0;
		d[k].assign(l, l + n);
		std::sort(d[k].begin(), d[k].end());
	}
	if (!d_all && d[0].empty() && d[1].empty() && d[2].empty() && v.uploaded6())
		return 0; // nothing to publish
	const int w = v.pub6 ^ 1;
	fib6_buf &b = v.b6[w];
	const bool full = d_all || v.pend6_all || !b.up;
	const uint32_t B = c->gen ^ 1;
	uint64_t t1 = t0;
	{
		std::shared_lock<std::shared_mutex> l(c->mu); // submitters go on
		if (b.d6 == nullptr) { // sized for the VRF's group capacity once: top, group slots, skips
			const uint32_t cap = gr_fib6_max_groups(v.rib6);
			HCK(fib_malloc(&b.d6, ((size_t)GR_FIB6_TOP + (size_t)cap * GR_FIB6_GROUP) * sizeof(uint32_t)
						      + (size_t)cap * sizeof(gr_fib6_skip)));
			b.groups = cap;
		}
		gr_fib6_skip *d_skips = reinterpret_cast<gr_fib6_skip *>(b.d6 + GR_FIB6_TOP + (size_t)b.groups * GR_FIB6_GROUP);
		stager st(c);
		if (full) {
			const uint32_t groups = gr_fib6_groups_used(v.rib6), skips = gr_fib6_skips_used(v.rib6);
			memcpy(st.add(b.d6, GR_FIB6_TOP), gr_fib6_top(v.rib6), (size_t)GR_FIB6_TOP * sizeof(uint32_t));
			if (groups)
				memcpy(st.add(b.d6 + GR_FIB6_TOP, (size_t)groups * GR_FIB6_GROUP), gr_fib6_groups(v.rib6),
				       (size_t)groups * GR_FIB6_GROUP * sizeof(uint32_t));
			if (skips)
				memcpy(st.add(d_skips, skips), gr_fib6_skips(v.rib6), (size_t)skips * sizeof(gr_fib6_skip));
		} else {
			stage_runs(st, b.d6, gr_fib6_top(v.rib6), 1, index_union(v.pend6[0], d[0]));
			stage_runs(st, b.d6 + GR_FIB6_TOP, gr_fib6_groups(v.rib6), GR_FIB6_GROUP, index_union(v.pend6[1], d[1]));
			stage_runs(st, d_skips, gr_fib6_skips(v.rib6), 1, index_union(v.pend6[2], d[2]));
		}
		b.up = true;
		views_follow_published(c, B);
		v.sel6[B] = (uint8_t)w;
		stage_rx(st, c, B);
		t1 = now_us();
		r = retire_wait(c);
		if (r == 0)
			r = st.flush();
		if (r == 0 && hipEventRecord(c->ready_ev[B], c->ctl) != hipSuccess)
			r = -EIO;
		if (r != 0) {
			b.up = false; // half written: rewritten in full next time
			views_follow_published(c, B);
			return r;
		}
	}
	gr_fib6_dirty_clear(v.rib6);
	const uint64_t t2 = now_us();
	r = publish(c, B, [&] {
		const bool old_up = v.b6[v.pub6].up;
		v.pub6 = w;
		// the copy just unpublished misses this commit's changes
		v.pend6_all = d_all || !old_up;
		for (int k = 0; k < 3; k++)
			v.pend6[k] = std::move(d[k]);
	});
	const uint64_t t3 = now_us();
	c->commit_us[0].store((uint32_t)(t1 - t0), std::memory_order_relaxed);
	c->commit_us[1].store((uint32_t)(t2 - t1), std::memory_order_relaxed);
	c->commit_us[2].store((uint32_t)(t3 - t2), std::memory_order_relaxed);
	return r;
}

extern "C" int gr_hip_fib6_lookup_host(gr_hip_ctx_t *c, uint16_t vrf, uint16_t iface_id, const uint8_t ip[16],
				       uint32_t *nh) {
	if (c == nullptr || vrf == 0 || vrf >= c->max_ifaces || ip == nullptr || nh == nullptr)
		return -EINVAL;
	std::lock_guard<std::mutex> f(c->fib_mu);
	vrf_fib &v = c->vrfs[vrf];
	if (v.rib6 == nullptr)
		return -ENONET;
	uint8_t key[16];
	scope6(key, ip, iface_id);
	*nh = gr_fib6_lookup(v.rib6, key);
	return 0;
}

extern "C" int gr_hip_fib6_info(gr_hip_ctx_t *c, uint16_t vrf, uint32_t *n_routes, uint32_t *groups_used,
				uint64_t *bytes) {
	if (c == nullptr || vrf == 0 || vrf >= c->max_ifaces)
		return -EINVAL;
	std::lock_guard<std::mutex> f(c->fib_mu);
	vrf_fib &v = c->vrfs[vrf];
	if (v.rib6 == nullptr)
		return -ENONET;
	if (n_routes)
		*n_routes = gr_fib6_n_routes(v.rib6);
	if (groups_used)
		*groups_used = gr_fib6_groups_used(v.rib6);
	if (bytes) // device bytes a lookup can touch
		*bytes = 4ull * GR_FIB6_TOP + 1024ull * gr_fib6_groups_used(v.rib6)
			 + sizeof(gr_fib6_skip) * (uint64_t)gr_fib6_skips_used(v.rib6);
	return 0;
}

// ---------------------------------------------------------------------------
// queues and submits
// ---------------------------------------------------------------------------

extern "C" int gr_hip_queue_create(gr_hip_ctx_t *c, void *stream, gr_hip_queue_t **out) {
	if (c == nullptr || out == nullptr)
		return -EINVAL;
	std::lock_guard<std::shared_mutex> l(c->mu);
	hipSetDevice(c->dev);
	gr_hip_queue *q = new (std::nothrow) gr_hip_queue();
	if (q == nullptr)
		return -ENOMEM;
	q->ctx = c;
	q->own_stream = stream == nullptr;
	if (stream == nullptr) {
		if (hipStreamCreateWithFlags(&q->s, hipStreamNonBlocking) != hipSuccess) {
			delete q;
			return -EIO;
		}
	} else {
		q->s = (hipStream_t)stream;
	}
	for (uint32_t i = 0; i < N_TIMED; i++) {
		hipEventCreate(&q->ev0[i]);
		hipEventCreate(&q->ev1[i]);
	}
	hipEventCreateWithFlags(&q->quiesce, hipEventDisableTiming);
	hipEventCreateWithFlags(&q->retire, hipEventDisableTiming);
	hipEventCreateWithFlags(&q->sync_ev, hipEventDisableTiming);
	for (node_slot &w : q->nw)
		hipEventCreateWithFlags(&w.done, hipEventDisableTiming);
	hipEventRecord(q->retire, q->s); // nothing submitted yet
	if (hipHostMalloc(reinterpret_cast<void **>(&q->h_err), sizeof(uint32_t), hipHostMallocMapped) == hipSuccess) {
		*q->h_err = 0;
		if (hipHostGetDevicePointer(reinterpret_cast<void **>(&q->d_err), q->h_err, 0) != hipSuccess) {
			hipHostFree(q->h_err);
			q->h_err = q->d_err = nullptr;
		}
	}
	(void)hipGetLastError();
	size_t sb = sizeof(gr_hip_iface_stats) * FWD4_STAT_SHARDS * c->max_ifaces;
	if (hipMalloc(&q->d_stats, sb) != hipSuccess || hipMemsetAsync(q->d_stats, 0, sb, q->s) != hipSuccess) {
		(void)hipGetLastError();
		q->d_stats = nullptr;
	}
	try {
		q->node_if.assign(c->max_ifaces, gr_hip_iface_stats{0, 0, 0, 0});
		q->kern_seen.assign(c->max_ifaces, gr_hip_iface_stats{0, 0, 0, 0});
	} catch (...) {
		return -ENOMEM; // (not reached in practice: a few tens of KiB)
	}
	c->queues.push_back(q);
	*out = q;
	return 0;
}

extern "C" int gr_hip_queue_destroy(gr_hip_queue_t *q) {
	if (q == nullptr)
		return -EINVAL;
	gr_hip_ctx *c = q->ctx;
	hipSetDevice(c->dev);
	hipStreamSynchronize(q->s);
	for (host_slot &h : q->hs)
		if (h.s)
			hipStreamSynchronize(h.s);
	if (q->ring >= 0) {
		res_wait(q, q->res_posted); // its resident batches (retired past the deadline), then the rings are free again
		if (q->res_inflight > 0)
			c->res_busy.fetch_sub(1, std::memory_order_relaxed);
		std::lock_guard<std::mutex> rl(c->res_mu);
		if (!c->res_dead) {
			for (uint32_t j = 0; j < q->res_w; j++) {
				c->res_taken[(size_t)q->ring + j] = 0;
				__atomic_store_n(c->res_taken_h + q->ring + j, 0u, __ATOMIC_RELEASE);
			}
			g_res_held[c->dev].fetch_sub(q->res_w);
			c->res_held -= q->res_w;
		}
	}
	{
		// unlink first: a commit running on another thread reaches the
		// queue's stream and events through this list (quiesce(),
		// retire_wait(), publish()), under the lock; after this, none can
		std::lock_guard<std::shared_mutex> l(c->mu);
		for (size_t i = 0; i < c->queues.size(); i++) {
			if (c->queues[i] == q) {
				c->queues.erase(c->queues.begin() + (long)i);
				break;
			}
		}
	}
	// a commit may have made its control stream wait on q->retire / q->quiesce
	// just before the unlink: let that wait resolve before the events go
	hipStreamSynchronize(c->ctl);
	for (host_slot &h : q->hs) {
		if (h.s)
			hipStreamDestroy(h.s);
		hipFree(h.in);
		hipFree(h.out);
		hipFree(h.meta);
		hipFree(h.v);
	}
	for (uint32_t i = 0; i < N_TIMED; i++) {
		hipEventDestroy(q->ev0[i]);
		hipEventDestroy(q->ev1[i]);
	}
	hipEventDestroy(q->quiesce);
	hipEventDestroy(q->retire);
	hipEventDestroy(q->sync_ev);
	hipFree(q->d_stats);
	if (q->snap_ev != nullptr)
		hipEventDestroy(q->snap_ev);
	hipHostFree(q->snap);
	hipHostFree(q->rd);
	hipHostFree(q->h_err);
	hipHostFree(q->pg_lines);
	hipHostFree(q->pg_out);
	hipHostFree(q->pg_meta);
	hipHostFree(q->pg_v);
	for (node_slot &w : q->nw) {
		hipEventDestroy(w.done);
		if (q->dead) // a resident launch that would not leave may still write them: leaked
			continue;
		hipHostFree(w.lines);
		hipHostFree(w.out);
		hipHostFree(w.meta);
		hipHostFree(w.v);
	}
	hipFree(q->d_pad);
	if (q->own_stream)
		hipStreamDestroy(q->s);
	(void)hipGetLastError();
	delete q;
	return 0;
}

extern "C" void *gr_hip_queue_stream(gr_hip_queue_t *q) {
	return q ? (void *)q->s : nullptr;
}

// The device address of pinned (hipHostMalloc'd or registered) host memory,
// false for pageable memory.
static bool host_dev_ptr(const void *p, void **dp) {
	hipPointerAttribute_t a;
	if (hipPointerGetAttributes(&a, p) != hipSuccess) {
		(void)hipGetLastError();
		return false;
	}
	if (a.type != hipMemoryTypeHost || a.devicePointer == nullptr || a.hostPointer == nullptr)
		return false;
	*dp = static_cast<uint8_t *>(a.devicePointer) + (static_cast<const uint8_t *>(p) - static_cast<uint8_t *>(a.hostPointer));
	return true;
}

static int launch(gr_hip_queue *q, hipStream_t s, const gr_hip_batch *b, bool timed) {
	gr_hip_ctx *c = q->ctx;
	fwd4_params A{};
	A.in = static_cast<const uint8_t *>(b->in_frames);
	A.out = static_cast<uint8_t *>(b->out_lines);
	A.meta = b->meta;
	A.verdicts = b->verdicts;
	A.stats = q->d_stats;
	const uint32_t g = c->gen;
	A.T = c->d_tables[g]; // the generation published when this launch is enqueued
	// ... whose upload the stream waits for, once per publication (the
	// host's own streams of gr_hip_fwd4_host at every launch)
	if (s != q->s || q->seen_serial != c->serial) {
		HCK(hipStreamWaitEvent(s, c->ready_ev[g], 0));
		if (s == q->s)
			q->seen_serial = c->serial;
	}
	A.n = b->n;
	A.in_stride = b->in_stride;
	A.out_stride = b->out_stride;
	A.readable = (b->flags & GR_HIP_BATCH_F_LINES_ONLY) ? GR_HIP_LINE
		: (b->flags & GR_HIP_BATCH_F_FRAME_PTRS)    ? UINT32_MAX // whole frames
							    : b->in_stride;
	A.nhf_lds = 0;
	int stats = c->stats_on && q->d_stats != nullptr;
	uint32_t slot = (uint32_t)(q->n_launch % N_TIMED);
	// persistent: one resident round of workgroups, each walking 64-packet tiles
	int variant = (stats ? FWD4_V_STATS : 0) | c->nt | ((b->flags & GR_HIP_BATCH_F_FRAME_PTRS) ? FWD4_V_PTRS : 0);
	uint32_t tiles = (b->n + 63) / 64;
	// fast adjacencies staged in LDS: IPv4, and IPv6 when IPv6 routes exist,
	// as many as the geometry's LDS leaves room for (IPv6 given up first)
	uint32_t n4 = c->nh_hi < gr_fwd4_ring_nhf_max() ? c->nh_hi : gr_fwd4_ring_nhf_max();
	uint32_t n6 = c->v6_routes ? n4 : 0;
	// and 2000::/4 of the IPv6 trie's first level, when one VRF holds IPv6
	// routes (given up before the fast adjacencies; in 16-byte units below)
	uint32_t t6 = c->v6_routes && c->top6[g] != nullptr ? FWD4_TOP6_MAX : 0;
	// a launch too small to give each workgroup "stage_min_tiles" tiles reads
	// the adjacencies from the global tables: staging 32 KiB per workgroup
	// for a tile or two only adds to a small batch's latency
	{
		const uint32_t per = c->wg_per_cu > 0 ? (uint32_t)c->wg_per_cu : RING_WG_PER_CU;
		const uint32_t g0 = (uint32_t)c->n_cu * per;
		if ((uint64_t)tiles < (uint64_t)g0 * c->stage_min_tiles)
			n4 = n6 = t6 = 0;
	}
	int occ;
	{
		std::lock_guard<std::mutex> ol(c->occ_mu);
		const int cfg = c->ring_cfg;
		auto occ_of = [&](uint32_t staged) -> const gr_hip_ctx::occ_entry & {
			const uint32_t filled = c->occ_n < 4 ? c->occ_n : 4;
			for (uint32_t i = 0; i < filled; i++)
				if (c->occ_cache[i].staged == staged && c->occ_cache[i].cfg == cfg)
					return c->occ_cache[i];
			gr_hip_ctx::occ_entry &e = c->occ_cache[c->occ_n++ % 4];
			e.staged = staged;
			e.cfg = cfg;
			for (int v = 0; v < 8; v++)
				e.occ[v] = gr_fwd4_ring_occupancy(v, cfg, staged);
			return e;
		};
		const gr_hip_ctx::occ_entry *e = &occ_of(n4 + n6 + t6 / 4);
		if (e->occ[variant] <= 0 && t6) {
			t6 = 0;
			e = &occ_of(n4 + n6);
		}
		if (e->occ[variant] <= 0 && n6) {
			n6 = 0;
			e = &occ_of(n4);
		}
		if (e->occ[variant] <= 0 && n4) {
			n4 = 0;
			e = &occ_of(0);
		}
		occ = e->occ[variant];
		memcpy(c->occ_ring, e->occ, sizeof(c->occ_ring));
	}
	A.nhf_lds = n4;
	A.nhf6_lds = n6;
	A.top6 = t6 ? c->top6[g] : nullptr;
	A.top6_lds = t6;
	uint32_t per_cu = c->wg_per_cu > 0 ? (uint32_t)c->wg_per_cu : RING_WG_PER_CU;
	if (occ > 0 && per_cu > (uint32_t)occ)
		per_cu = (uint32_t)occ;
	uint32_t grid = (uint32_t)c->n_cu * per_cu;
	if (grid > tiles)
		grid = tiles;
	A.err = q->d_err;
	A.spin_max = c->spin_max;
	A.order = c->tile_order;
	A.chunk = 0;
	if (c->tile_order == 1)
		A.chunk = (tiles + grid - 1) / grid;
	if (c->tile_order == 2 && grid % 8 == 0)
		A.chunk = (tiles + 7) / 8;
	else if (c->tile_order == 2)
		A.order = 0;
	if (c->tile_order == 3)
		A.chunk = c->tile_run;
	// every `time_every`-th submit of the queue carries the event pair
	// (counted over every submit that could be timed, whatever the knobs)
	if (timed && !q->always_timed) {
		const uint64_t k = q->n_submit++;
		timed = !c->untimed && (c->time_every <= 1 || k % c->time_every == 0);
	}
	if (timed)
		HCK(hipEventRecord(q->ev0[slot], s));
	HCK(gr_fwd4_ring_launch(&A, grid, s, variant, c->ring_cfg));
	if (timed) {
		HCK(hipEventRecord(q->ev1[slot], s));
		q->n_launch++;
	}
	return 0;
}

// ---------------------------------------------------------------------------
// the resident kernel (knob "resident"; fwd4_ring.hip gr_fwd4_resident)
// ---------------------------------------------------------------------------
// A queue's node batches go to the context's resident kernel instead of a
// launch each. The queue holds res_w rings (descriptors in pinned host
// memory), each numbering its own batches; a batch goes to k of them
// (RES_TILES_PER_WG tiles each): its fwd4_params into each one's next
// descriptor, then that ring's seq, workgroup j < k taking tiles j, j + k, ...
// The kernel's workgroup for a ring stores the seq into the ring's done word
// once its tiles' results are in host memory; the batch is done when all k
// are (the node polls those words: loads, no runtime call, no hardware queue
// held per batch: DESIGN.md §6.3). Once no ring has finished a batch for the
// lifetime, a first ring sets the stop word and all leave after their batch; whoever then finds a batch
// waiting launches the kernel again, once every ring's exited word carries
// the last launch's id, so that one workgroup at most ever serves a ring.
// Posts wait for the FIB generation's upload on the host (launches make their
// stream wait); commits and quiesce wait, on the host, for the batches posted
// before them (retire_wait, quiesce).
#define RES_NDESC 8 // descriptors per ring (GR_HIP_NODE_DEPTH batches in flight at most)
static_assert(GR_HIP_NODE_DEPTH < RES_NDESC, "a ring's batches in flight fit its descriptors");
#define RES_STRIDE 8 // uint64_t per ring in the done / exited words: a 64-byte line each
#define RES_TILES_PER_WG 8 // default tiles per workgroup a batch is split into (knob "resident_tiles")
#define RES_LEAVE_NS (500ull * 1000000ull) // a launch told to stop has left within this, or is stuck

static uint64_t res_word(const uint64_t *w, int ring) {
	return __atomic_load_n(w + (size_t)ring * RES_STRIDE, __ATOMIC_ACQUIRE);
}

// Tell the live launch to stop and wait, bounded, until it is gone: every
// workgroup leaves after the batch it is running (whose waits are bounded).
// 0: gone (or faulted: it touches nothing more); -EDEADLK: still running
// past RES_LEAVE_NS (a workgroup no CU runs, or one that does not return).
static int res_leave(gr_hip_ctx *c) {
	if (c->res_leave_fail) // tests: as if a workgroup never left (the kernel itself is stopped by "resident_hold")
		return -EDEADLK;
	if (!c->res_live)
		return 0;
	__atomic_store_n(c->res_stop, 1u, __ATOMIC_RELEASE);
	const uint64_t t0 = now_ns_host();
	for (uint32_t spin = 0;; spin++) {
		const hipError_t e = hipEventQuery(c->res_ev);
		if (e == hipSuccess || e != hipErrorNotReady) {
			(void)hipGetLastError();
			break;
		}
		if (now_ns_host() - t0 > RES_LEAVE_NS)
			return -EDEADLK;
		if (spin > 64)
			usleep(20);
	}
	c->res_live = false;
	return 0;
}

static void res_free(gr_hip_ctx *c) {
	if (c->res_live && c->res_stop != nullptr && res_leave(c) != 0) {
		// still running: its rings and words stay allocated (leaked), the
		// kernel may still read and write them
		c->res_dead = true;
		c->res_desc = nullptr;
		c->res_done = c->res_exited = nullptr;
		c->res_stop = nullptr;
		c->res_taken_h = nullptr;
		c->res_wake_d = nullptr;
		c->res_ev = nullptr;
		c->res_s = nullptr;
		return;
	}
	if (c->res_ev != nullptr)
		hipEventDestroy(c->res_ev);
	if (c->res_s != nullptr)
		hipStreamDestroy(c->res_s);
	hipHostFree(c->res_desc);
	hipHostFree(c->res_done);
	hipHostFree(c->res_exited);
	hipHostFree(c->res_stop);
	hipHostFree(c->res_taken_h);
	hipFree(c->res_wake_d);
	c->res_wake_d = nullptr;
	c->res_taken_h = nullptr;
	c->res_ev = nullptr;
	c->res_s = nullptr;
	c->res_desc = nullptr;
	c->res_done = c->res_exited = nullptr;
	c->res_stop = nullptr;
	(void)hipGetLastError();
}

// The rings, their words and the kernel's stream, on first use (res_mu held).
static int res_setup(gr_hip_ctx *c) {
	if (c->res_desc != nullptr)
		return 0;
	const size_t nd = sizeof(fwd4_res_desc) * c->res_rings * RES_NDESC;
	const size_t nw = sizeof(uint64_t) * c->res_rings * RES_STRIDE;
	const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
	int least = 0, greatest = 0;
	hipDeviceGetStreamPriorityRange(&least, &greatest);
	if (hipHostMalloc(reinterpret_cast<void **>(&c->res_desc), nd, fl) != hipSuccess
	    || hipHostMalloc(reinterpret_cast<void **>(&c->res_done), nw, fl) != hipSuccess
	    || hipHostMalloc(reinterpret_cast<void **>(&c->res_exited), nw, fl) != hipSuccess
	    || hipHostMalloc(reinterpret_cast<void **>(&c->res_stop), 64, fl) != hipSuccess
	    || hipHostMalloc(reinterpret_cast<void **>(&c->res_taken_h), sizeof(uint32_t) * c->res_rings, fl) != hipSuccess
	    || hipHostGetDevicePointer(reinterpret_cast<void **>(&c->res_taken_d), c->res_taken_h, 0) != hipSuccess
	    || hipHostGetDevicePointer(reinterpret_cast<void **>(&c->res_desc_d), c->res_desc, 0) != hipSuccess
	    || hipHostGetDevicePointer(reinterpret_cast<void **>(&c->res_done_d), c->res_done, 0) != hipSuccess
	    || hipHostGetDevicePointer(reinterpret_cast<void **>(&c->res_exited_d), c->res_exited, 0) != hipSuccess
	    || hipHostGetDevicePointer(reinterpret_cast<void **>(&c->res_stop_d), c->res_stop, 0) != hipSuccess
	    || hipMalloc(reinterpret_cast<void **>(&c->res_wake_d), nw + 64) != hipSuccess // + the active word
	    // its own priority: a hardware queue of its own, not shared with the
	    // streams whose work would wait behind a resident launch
	    || hipStreamCreateWithPriority(&c->res_s, hipStreamNonBlocking, greatest) != hipSuccess
	    || hipEventCreateWithFlags(&c->res_ev, hipEventDisableTiming) != hipSuccess
	    // before the first launch, on its stream (no device-wide sync: another
	    // context's resident kernel may be running on this device)
	    || hipMemsetAsync(c->res_wake_d, 0, nw + 64, c->res_s) != hipSuccess) {
		(void)hipGetLastError();
		res_free(c);
		return -ENOMEM;
	}
	memset(c->res_desc, 0, nd);
	memset(c->res_done, 0, nw);
	memset(c->res_exited, 0, nw);
	memset(c->res_taken_h, 0, sizeof(uint32_t) * c->res_rings);
	*c->res_stop = 0;
	c->res_taken.assign(c->res_rings, 0);
	// how many rings the device runs at once: workgroups per CU at the
	// kernel's LDS size, times the CUs not reserved for other kernels
	const int occ = gr_fwd4_resident_occupancy();
	const int cus = c->n_cu - (int)c->res_reserve_cu;
	c->res_cap = occ > 0 && cus > 0 ? (uint32_t)(occ * cus) : 0;
	return 0;
}

// Launch the kernel when none runs (res_mu held). A launch that is leaving
// (stop set) is relaunched only once all its workgroups have left.
static int res_ensure(gr_hip_ctx *c) {
	if (c->res_hold) { // tests: the kernel stops serving its rings
		if (c->res_live)
			__atomic_store_n(c->res_stop, 1u, __ATOMIC_RELEASE);
		return 0;
	}
	if (c->res_live) {
		if (__atomic_load_n(c->res_stop, __ATOMIC_ACQUIRE) == 0)
			return 0;
		for (uint32_t r = 0; r < c->res_rings; r++)
			if (res_word(c->res_exited, (int)r) != c->res_launch)
				return 0; // still leaving: a later poll relaunches
		c->res_live = false;
	}
	__atomic_store_n(c->res_stop, 0u, __ATOMIC_RELEASE);
	fwd4_res_params R{};
	R.descs = c->res_desc_d;
	R.done = c->res_done_d;
	R.exited = c->res_exited_d;
	R.stop = c->res_stop_d;
	R.wake = c->res_wake_d;
	R.active = c->res_wake_d + (size_t)c->res_rings * RES_STRIDE;
	R.taken = c->res_taken_d;
	R.lifetime = (uint64_t)c->res_ms * 100000u; // s_memrealtime: 100 MHz
	R.launch_id = ++c->res_launch;
	R.ndesc = RES_NDESC;
	R.stride = RES_STRIDE;
	R.nap_max = c->res_nap;
	HCK(gr_fwd4_resident_launch(&R, c->res_rings, c->res_s));
	HCK(hipEventRecord(c->res_ev, c->res_s));
	c->res_live = true;
	return 0;
}

// A waiting batch and a kernel that left: launch it again.
static int res_kick(gr_hip_ctx *c) {
	if (!__atomic_load_n(c->res_stop, __ATOMIC_ACQUIRE) && c->res_live)
		return 0;
	std::lock_guard<std::mutex> l(c->res_mu);
	return res_ensure(c);
}

// A ring for queue q, on its first resident batch: false when none is free.
static bool res_take(gr_hip_queue *q) {
	if (q->ring >= 0)
		return true;
	gr_hip_ctx *c = q->ctx;
	std::lock_guard<std::mutex> l(c->res_mu);
	if (res_setup(c) != 0)
		return false;
	const uint32_t W = c->res_w;
	if (c->res_dead || (uint32_t)c->dev >= RES_MAX_DEV)
		return false;
	// co-residency: the device's rings held, over every context, stay within
	// what its CUs run at once; past that the queue launches per batch
	std::atomic<uint32_t> &held = g_res_held[c->dev];
	for (uint32_t h = held.load(); ;) {
		if (h + W > c->res_cap)
			return false;
		if (held.compare_exchange_weak(h, h + W))
			break;
	}
	bool got = false;
	for (uint32_t r = 0; r + W <= c->res_rings && !got; r += W) { // W consecutive rings, in groups of W
		// all W free: queues that took theirs under another "resident_wgs"
		// hold groups of another size
		bool free = true;
		for (uint32_t j = 0; j < W && free; j++)
			free = !c->res_taken[r + j];
		if (free) {
			for (uint32_t j = 0; j < W; j++) { // 1: the queue's first ring, 2: a helper
				c->res_taken[r + j] = 1;
				__atomic_store_n(c->res_taken_h + r + j, j == 0 ? 1u : 2u, __ATOMIC_RELEASE);
			}
			// a live launch's workgroups for these rings left at once: it
			// leaves, and the next batch launches one that serves them
			if (c->res_live)
				__atomic_store_n(c->res_stop, 1u, __ATOMIC_RELEASE);
			q->ring = (int)r;
			q->res_w = W;
			q->res_posted.k = W; // each ring's numbering goes on
			for (uint32_t j = 0; j < W; j++)
				q->res_posted.seq[j] = res_word(c->res_done, (int)(r + j));
			q->res_retire = q->res_posted;
			for (uint32_t j = 0; j < RES_WMAX; j++)
				q->res_cancelled[j] = 0;
			c->res_held += W;
			got = true;
		}
	}
	if (!got)
		held.fetch_sub(W);
	return got;
}

static bool res_is_done(const gr_hip_queue *q, const res_mark &m) {
	for (uint32_t j = 0; j < m.k; j++)
		if (res_word(q->ctx->res_done, q->ring + (int)j) < m.seq[j])
			return false;
	return true;
}

// Whether res_cancel retired any of m's descriptors unrun.
static bool res_was_cancelled(const gr_hip_queue *q, const res_mark &m) {
	for (uint32_t j = 0; j < m.k; j++)
		if (__atomic_load_n(&q->res_cancelled[j], __ATOMIC_ACQUIRE) >= m.seq[j])
			return true;
	return false;
}

// A batch past its deadline, or a launch that faulted (res_mu not held):
// make sure no workgroup ever runs it. The live launch is told to stop and
// waited for (res_leave); its workgroups finish the batch each is running,
// so once it is gone a ring whose done word is still below m's seq never
// started m there. Those descriptors are retired (seq cleared, the done word
// moved on by the host, so that a relaunch resumes after them) and recorded
// in res_cancelled: the walk's verdicts still hold the fill value there and
// its packets go back to grout's CPU nodes untouched. A launch that does not
// leave makes the context's resident kernel dead: -EDEADLK, and the caller
// must neither reuse nor free what the batch names (the node marks the queue
// dead). Returns 0 (m done after all), -ETIMEDOUT (retired), -EDEADLK.
static int res_cancel(gr_hip_queue *q, const res_mark &m) {
	gr_hip_ctx *c = q->ctx;
	std::lock_guard<std::mutex> l(c->res_mu);
	if (res_is_done(q, m))
		return 0;
	if (res_leave(c) != 0) {
		c->res_dead = true;
		q->dead = true;
		return -EDEADLK;
	}
	if (res_is_done(q, m))
		return 0; // it ran before the launch left
	for (uint32_t j = 0; j < m.k; j++) {
		const int ring = q->ring + (int)j;
		const uint64_t d = res_word(c->res_done, ring);
		if (d >= m.seq[j])
			continue;
		for (uint64_t sq = d + 1; sq <= m.seq[j]; sq++) {
			fwd4_res_desc &dd = c->res_desc[(size_t)ring * RES_NDESC + sq % RES_NDESC];
			if (__atomic_load_n(&dd.seq, __ATOMIC_ACQUIRE) == sq)
				__atomic_store_n(&dd.seq, 0ull, __ATOMIC_RELEASE);
		}
		__atomic_store_n(&q->res_cancelled[j], m.seq[j], __ATOMIC_RELEASE);
		__atomic_store_n(c->res_done + (size_t)ring * RES_STRIDE, m.seq[j], __ATOMIC_RELEASE);
	}
	c->res_cancels.fetch_add(1);
	return -ETIMEDOUT;
}

// Wait, on the host, until batch m is done: past `deadline` (host ns), or
// when the launch faulted, res_cancel decides (0, -ETIMEDOUT, -EDEADLK).
static int res_wait(gr_hip_queue *q, const res_mark &m, uint64_t deadline) {
	if (q->ring < 0 || res_is_done(q, m))
		return 0;
	gr_hip_ctx *c = q->ctx;
	if (c->res_dead)
		return res_was_cancelled(q, m) ? -ETIMEDOUT : -EDEADLK;
	for (uint32_t spin = 1; !res_is_done(q, m); spin++) {
		if ((spin & 1023) == 0) {
			if (res_kick(c) != 0)
				return res_cancel(q, m);
			const hipError_t e = hipEventQuery(c->res_ev);
			if (e != hipSuccess && e != hipErrorNotReady) {
				(void)hipGetLastError();
				const int r = res_cancel(q, m); // the faulted launch touches nothing more
				return r == -ETIMEDOUT ? -EIO : r;
			}
			if (now_ns_host() > deadline)
				return res_cancel(q, m);
		}
		__builtin_ia32_pause();
	}
	return 0;
}

static int res_wait(gr_hip_queue *q, const res_mark &m) {
	return res_wait(q, m, now_ns_host() + (uint64_t)q->ctx->res_wait_ms * 1000000ull);
}

// Post batch b (device addresses) on k of q's rings (RES_TILES_PER_WG tiles
// each, workgroup j < k taking tiles j, j + k, ...); *m receives what must be
// done for it. c->mu held shared.
static int res_post(gr_hip_queue *q, const gr_hip_batch *b, res_mark *m) {
	gr_hip_ctx *c = q->ctx;
	if (c->res_dead || q->dead)
		return -EIO;
	const uint32_t g = c->gen;
	if (q->seen_serial != c->serial) { // the generation's upload (launch(): a stream wait)
		HCK(hipEventSynchronize(c->ready_ev[g]));
		q->seen_serial = c->serial;
	}
	const uint32_t tiles = (b->n + 63) / 64;
	uint32_t k = (tiles + c->res_tiles - 1) / c->res_tiles;
	k = k < 1 ? 1 : k > q->res_w ? q->res_w : k;
	if (c->res_split != 0 && k > c->res_split)
		k = c->res_split;
	if (c->res_budget != 0) { // busy GPU: fewer workgroups per batch
		const uint32_t busy = c->res_busy.load(std::memory_order_relaxed) + (q->res_inflight == 0 ? 1 : 0);
		const uint32_t cap = c->res_budget / busy;
		k = k > cap ? (cap < 1 ? 1 : cap) : k;
	}
	// a batch of k rings behind others of the queue: on helper rings h ..
	// h + k - 1, so that it does not wait for them on the first ring(s),
	// which only wakes those (an empty share of its own; rings 1 .. h-1 are
	// waited for at their last posted batch, older ones, which leave before
	// this one anyway). h goes round 1 .. res_w - k.
	uint32_t h = 0;
	if (c->res_rotate && q->res_inflight > 0 && k < q->res_w) {
		const uint32_t span = q->res_w - k; // first rings of a group of k among the helpers
		q->res_rot = q->res_rot % span + 1;
		h = q->res_rot;
	}
	const uint32_t kpost = h ? h + k : k; // rings the batch's mark covers
	for (uint32_t j = 0; j < kpost; j++)
		if ((!h || j == 0 || j >= h)
		    && q->res_posted.seq[j] + 1 > res_word(c->res_done, q->ring + (int)j) + RES_NDESC)
			return -EBUSY; // (not reached: GR_HIP_NODE_DEPTH < RES_NDESC)
	fwd4_params A{};
	A.in = static_cast<const uint8_t *>(b->in_frames);
	A.out = static_cast<uint8_t *>(b->out_lines);
	A.meta = b->meta;
	A.verdicts = b->verdicts;
	A.T = c->d_tables[g];
	A.n = b->n;
	A.in_stride = b->in_stride;
	A.out_stride = b->out_stride;
	A.readable = (b->flags & GR_HIP_BATCH_F_LINES_ONLY) ? GR_HIP_LINE
		: (b->flags & GR_HIP_BATCH_F_FRAME_PTRS)    ? UINT32_MAX
							    : b->in_stride;
	A.spin_max = c->spin_max;
	A.err = q->d_err;
	A.wgs = k;
	A.ptrs = (b->flags & GR_HIP_BATCH_F_FRAME_PTRS) ? 1 : 0;
	if (h) {
		m->k = kpost;
		for (uint32_t j = 1; j < h; j++)
			m->seq[j] = q->res_posted.seq[j];
		// rings h .. h + k - 1: the batch split over k rings, workgroup j
		// taking tiles j, j + k, ... (helpers wake no one)
		uint64_t sh[RES_WMAX] = {};
		for (uint32_t j = 0; j < k; j++) {
			const uint32_t r = h + j;
			sh[j] = q->res_posted.seq[r] + 1;
			fwd4_res_desc &dh = c->res_desc[(size_t)(q->ring + (int)r) * RES_NDESC + sh[j] % RES_NDESC];
			A.wg0 = j;
			A.wgs = k;
			memcpy(&dh.A, &A, sizeof(A));
			memset(dh.helper_seq, 0, sizeof(dh.helper_seq));
			__atomic_store_n(&dh.seq, sh[j], __ATOMIC_RELEASE); // after A
			q->res_posted.seq[r] = sh[j];
			m->seq[r] = sh[j];
		}
		// the first ring: no tile of its own, wakes rings h .. h + k - 1 for it
		const uint64_t s0 = q->res_posted.seq[0] + 1;
		fwd4_res_desc &d0 = c->res_desc[(size_t)q->ring * RES_NDESC + s0 % RES_NDESC];
		A.n = 0;
		A.wg0 = 0;
		A.wgs = h + k;
		memcpy(&d0.A, &A, sizeof(A));
		memset(d0.helper_seq, 0, sizeof(d0.helper_seq));
		for (uint32_t j = 0; j < k; j++)
			d0.helper_seq[h + j - 1] = sh[j];
		__atomic_store_n(&d0.seq, s0, __ATOMIC_RELEASE);
		q->res_posted.seq[0] = s0;
		m->seq[0] = s0;
		if (q->res_inflight++ == 0)
			c->res_busy.fetch_add(1, std::memory_order_relaxed);
		return res_kick(c);
	}
	m->k = k;
	// the helpers first: the first ring's workgroup wakes them (fwd4_res_desc)
	for (uint32_t j = k; j-- > 0;) {
		const uint64_t seq = q->res_posted.seq[j] + 1;
		fwd4_res_desc &d = c->res_desc[(size_t)(q->ring + (int)j) * RES_NDESC + seq % RES_NDESC];
		A.wg0 = j;
		memcpy(&d.A, &A, sizeof(A));
		// the first ring's names its helpers' seqs; a helper's, none (a
		// workgroup that still holds the first ring's role from an older
		// grouping reads zeros here, which the kernel's max ignores)
		memset(d.helper_seq, 0, sizeof(d.helper_seq));
		if (j == 0)
			for (uint32_t h = 1; h < k; h++)
				d.helper_seq[h - 1] = m->seq[h];
		__atomic_store_n(&d.seq, seq, __ATOMIC_RELEASE); // after A
		q->res_posted.seq[j] = seq;
		m->seq[j] = seq;
	}
	if (q->res_inflight++ == 0)
		c->res_busy.fetch_add(1, std::memory_order_relaxed);
	return res_kick(c);
}

extern "C" int gr_hip_tune(gr_hip_ctx_t *c, const char *key, int value) {
	if (c == nullptr || key == nullptr)
		return -EINVAL;
	std::lock_guard<std::shared_mutex> l(c->mu);
	if (strcmp(key, "nt") == 0) {
		c->nt = value ? FWD4_V_NT : 0;
	} else if (strcmp(key, "stats") == 0) {
		c->stats_on = value != 0;
	} else if (strcmp(key, "wg_per_cu") == 0) {
		if (value < 0 || value > 32)
			return -EINVAL;
		c->wg_per_cu = value;
	} else if (strcmp(key, "fib_format") == 0) { // takes effect at the next commit
		if (value < FIB_FMT_24 || value > FIB_FMT_24_W2)
			return -EINVAL;
		c->fib_fmt = value;
	} else if (strcmp(key, "node_ptrs") == 0) {
		c->node_ptrs = value != 0;
	} else if (strcmp(key, "node_prof") == 0) { // process-wide: gr_hip_node_prof's clocks
		node_prof_on.store(value != 0);
	} else if (strcmp(key, "untimed") == 0) {
		c->untimed = value != 0;
	} else if (strcmp(key, "stats_copy") == 0) { // measurement: the counters read as in round 5
		c->stats_copy = value != 0;
	} else if (strcmp(key, "sync_check") == 0) { // debugging: host path steps waited for one by one
		c->sync_check = value != 0;
	} else if (strcmp(key, "host_path_last") == 0) { // read: 0 direct, 1 staged copies, 2 pageable
		return c->host_path_last.load();
	} else if (strcmp(key, "time_every") == 0) { // sample the launch timing: less event overhead
		if (value < 0 || value > 1024)
			return -EINVAL;
		c->time_every = (uint32_t)value;
		for (gr_hip_queue *q : c->queues) // the sampling restarts: submits 0, N, 2N ... from now
			q->n_submit = 0;
	} else if (strcmp(key, "fail_appends") == 0) { // tests: the node's staging failure path
		if (value < 0)
			return -EINVAL;
		c->fail_appends.store(value);
	} else if (strcmp(key, "spin_max") == 0) { // tests: make ring waits give up early
		if (value < 0)
			return -EINVAL;
		c->spin_max = (uint32_t)value;
	} else if (strcmp(key, "alloc_contig") == 0) { // later allocations only
		c->alloc_contig = value != 0;
	} else if (strcmp(key, "tile_order") == 0) {
		if (value < 0 || value > 3)
			return -EINVAL;
		c->tile_order = value;
	} else if (strcmp(key, "resident") == 0) { // node batches through the resident kernel (res_post)
		c->res_on = value != 0;
	} else if (strcmp(key, "resident_rings") == 0) { // before the first resident batch only
		if (value < 1 || value > 256 || c->res_desc != nullptr)
			return -EINVAL;
		c->res_rings = (uint32_t)value;
	} else if (strcmp(key, "resident_wgs") == 0) { // for queues that take their rings from then on
		if (value < 1 || value > RES_WMAX)
			return -EINVAL;
		c->res_w = (uint32_t)value;
	} else if (strcmp(key, "resident_tiles") == 0) {
		if (value < 1)
			return -EINVAL;
		c->res_tiles = (uint32_t)value;
	} else if (strcmp(key, "resident_budget") == 0) { // the next batches of every queue; 0: off
		if (value < 0)
			return -EINVAL;
		c->res_budget = (uint32_t)value;
	} else if (strcmp(key, "resident_split") == 0) { // the next batches of every queue
		if (value < 0 || value > RES_WMAX)
			return -EINVAL;
		c->res_split = (uint32_t)value;
	} else if (strcmp(key, "resident_nap") == 0) { // the next launch
		if (value < 1 || value > 64)
			return -EINVAL;
		c->res_nap = (uint32_t)value;
	} else if (strcmp(key, "resident_rotate") == 0) { // one-ring batches behind others go to the helper rings in turn
		c->res_rotate = value != 0;
	} else if (strcmp(key, "resident_rotating") == 0) { // read: "resident_rotate"
		return c->res_rotate ? 1 : 0;
	} else if (strcmp(key, "resident_wait_ms") == 0) { // a resident batch's deadline, from its post
		if (value < 1 || value > 60000)
			return -EINVAL;
		c->res_wait_ms = (uint32_t)value;
	} else if (strcmp(key, "resident_reserve_cu") == 0) { // before the first resident batch only
		if (value < 0 || value >= c->n_cu || c->res_desc != nullptr)
			return -EINVAL;
		c->res_reserve_cu = (uint32_t)value;
	} else if (strcmp(key, "resident_cap") == 0) { // read: rings the device holds co-resident (0: not set up)
		return (int)c->res_cap;
	} else if (strcmp(key, "resident_held") == 0) { // read: rings held on this device, every context
		return (uint32_t)c->dev < RES_MAX_DEV ? (int)g_res_held[c->dev].load() : 0;
	} else if (strcmp(key, "resident_cancels") == 0) { // read: batches retired unrun past their deadline
		return (int)c->res_cancels.load();
	} else if (strcmp(key, "resident_dead") == 0) { // read: a launch would not leave (no resident batches since)
		return c->res_dead ? 1 : 0;
	} else if (strcmp(key, "resident_hold") == 0) { // tests: the live launch leaves and is not relaunched (1) or is again (0)
		std::lock_guard<std::mutex> rl(c->res_mu);
		c->res_hold = value != 0;
		if (c->res_hold && c->res_live)
			__atomic_store_n(c->res_stop, 1u, __ATOMIC_RELEASE);
	} else if (strcmp(key, "resident_leave_fail") == 0) { // tests: the -EDEADLK path (with "resident_hold")
		c->res_leave_fail = value != 0;
	} else if (strcmp(key, "resident_ms") == 0) {
		if (value < 1 || value > 10000)
			return -EINVAL;
		c->res_ms = (uint32_t)value;
	} else if (strcmp(key, "resident_launches") == 0) { // read
		return (int)c->res_launch;
	} else if (strcmp(key, "resident_ring_count") == 0) { // read: "resident_rings"
		return (int)c->res_rings;
	} else if (strcmp(key, "resident_busy") == 0) { // read: queues with resident batches in flight
		return (int)c->res_busy.load();
	} else if (strcmp(key, "stage_min_tiles") == 0) {
		if (value < 0)
			return -EINVAL;
		c->stage_min_tiles = (uint32_t)value;
	} else if (strcmp(key, "tile_run") == 0) {
		if (value < 1 || value > 4096)
			return -EINVAL;
		c->tile_run = (uint32_t)value;
	} else if (strcmp(key, "host_direct") == 0) {
		c->host_direct = value != 0;
	} else if (strcmp(key, "fib_format_of") == 0) { // read: the format VRF `value` is on the device in
		if (value <= 0 || (uint32_t)value >= c->max_ifaces || c->vrfs[value].rib == nullptr
		    || !c->vrfs[value].uploaded())
			return -ENONET;
		return c->vrfs[value].pub().fmt;
	} else if (strcmp(key, "fib16") == 0) { // older key: 0 = 4-byte DIR24_8, else DIR-16-8-8
		c->fib_fmt = value ? FIB_FMT_16_8_8 : FIB_FMT_24;
	} else if (strcmp(key, "ring") == 0) { // ring geometry, fwd4_ring.hip ring_cfgN
		if (value < 0 || value >= gr_fwd4_ring_ncfg())
			return -EINVAL;
		c->ring_cfg = value;
	} else if (strncmp(key, "commit_us_", 10) == 0) { // read-only: the last IPv4 commit's phases
		const char *k = key + 10;
		const int i = strcmp(k, "stage") == 0 ? 0 : strcmp(k, "enqueue") == 0 ? 1 : strcmp(k, "publish") == 0 ? 2 : -1;
		if (i < 0)
			return -ENOENT;
		const uint32_t us = c->commit_us[i].load(std::memory_order_relaxed);
		return (int)(us > 0x7fffffffu ? 0x7fffffffu : us);
	} else if (strcmp(key, "occupancy") == 0) { // read-only: WGs/CU of the current variant
		return c->occ_ring[(c->stats_on ? FWD4_V_STATS : 0) | c->nt]; // as of the last launch
	} else {
		return -ENOENT;
	}
	return 0;
}

static int batch_ok(const gr_hip_batch *b) {
	if (b == nullptr)
		return -EINVAL;
	if (b->n == 0)
		return 0;
	if (b->flags & GR_HIP_BATCH_F_PREFIX32) { // 32-byte output prefixes, packed
		if (!b->out_lines || b->out_stride != GR_HIP_PREFIX || ((uintptr_t)b->out_lines & 15))
			return -EINVAL;
		gr_hip_batch full = *b;
		full.flags &= ~GR_HIP_BATCH_F_PREFIX32;
		full.out_stride = GR_HIP_LINE; // the other checks as for whole lines
		return batch_ok(&full);
	}
	if (b->flags & GR_HIP_BATCH_F_FRAME_PTRS) {
		// in_frames: n frame addresses; out_lines NULL = rewrite each frame in place
		if (!b->in_frames || !b->meta || !b->verdicts || ((uintptr_t)b->in_frames & 7)
		    || (b->out_lines && (b->out_stride < GR_HIP_LINE || (b->out_stride & 15)
					 || ((uintptr_t)b->out_lines & 15)))
		    || ((uintptr_t)b->meta & 7) || ((uintptr_t)b->verdicts & 7))
			return -EINVAL;
	} else {
		if (!b->in_frames || !b->out_lines || !b->meta || !b->verdicts)
			return -EINVAL;
		if (b->in_stride < GR_HIP_LINE || b->out_stride < GR_HIP_LINE || (b->in_stride & 15)
		    || (b->out_stride & 15) || ((uintptr_t)b->in_frames & 15) || ((uintptr_t)b->out_lines & 15)
		    || ((uintptr_t)b->meta & 7) || ((uintptr_t)b->verdicts & 7))
			return -EINVAL;
	}
	if (b->n > (1u << 31))
		return -E2BIG;
	return 1;
}

extern "C" int gr_hip_fwd4_submit(gr_hip_queue_t *q, const struct gr_hip_batch *b) {
	if (q == nullptr)
		return -EINVAL;
	int ok = batch_ok(b);
	if (ok <= 0)
		return ok;
	// enqueued entirely before a control-plane update's quiesce or entirely
	// after its upload: the update holds the lock exclusively (RCU analogue)
	std::shared_lock<std::shared_mutex> l(q->ctx->mu);
	return launch(q, q->s, b, true);
}

// After a sync: did a workgroup of a kernel on this queue give up a ring
// wait (its results are incomplete)? Reports it once.
static int q_check(gr_hip_queue *q) {
	if (q->h_err != nullptr && __atomic_load_n(q->h_err, __ATOMIC_ACQUIRE)) {
		__atomic_store_n(q->h_err, 0, __ATOMIC_RELEASE);
		return -ETIMEDOUT;
	}
	return 0;
}

extern "C" int gr_hip_queue_sync(gr_hip_queue_t *q) {
	if (q == nullptr)
		return -EINVAL;
	if (const int e_ = host_wait(q, q->s))
		return e_;
	return q_check(q);
}

extern "C" int gr_hip_queue_kernel_ms(gr_hip_queue_t *q, uint32_t n, float *ms, uint32_t *count) {
	if (q == nullptr || ms == nullptr)
		return -EINVAL;
	uint64_t avail = q->n_launch < N_TIMED ? q->n_launch : N_TIMED;
	if (n > avail)
		n = (uint32_t)avail;
	float total = 0;
	for (uint32_t k = 0; k < n; k++) {
		uint32_t slot = (uint32_t)((q->n_launch - 1 - k) % N_TIMED);
		HCK(hipEventSynchronize(q->ev1[slot]));
		float t = 0;
		HCK(hipEventElapsedTime(&t, q->ev0[slot], q->ev1[slot]));
		total += t;
	}
	*ms = total;
	if (count)
		*count = n;
	return 0;
}

// Knob "sync_check" (debugging): the host path waits for each step it has
// just enqueued on stream s, and a failing one is named on stderr (an
// asynchronous error otherwise surfaces at whatever call comes next: round 5's
// illegal address was reported by a copy).
#define SYNC_CHECK(c, s, what)                                                                    \
	do {                                                                                       \
		if ((c)->sync_check) {                                                             \
			const hipError_t e__ = hipStreamSynchronize(s);                            \
			if (e__ != hipSuccess) {                                                   \
				(void)hipGetLastError();                                           \
				fprintf(stderr, "gr_hip: sync_check: %s: %s\n", what, hipGetErrorString(e__)); \
				return -EIO;                                                       \
			}                                                                          \
		}                                                                                  \
	} while (0)

// Zero-copy host batch (the context's "host_direct"): the kernel's loaders
// and storers move the lines over PCIe themselves, both directions at once,
// no staging copies. Enqueues the launch on the queue's stream and sets
// *direct, or leaves it false when the buffers are not device-accessible
// pinned memory (the caller stages them). The caller holds c->mu shared.
static int host_direct_launch(gr_hip_queue *q, const void *lines, const gr_hip_pkt_meta *meta, uint32_t n,
			      void *out_lines, uint32_t out_stride, gr_hip_verdict *verdicts, bool *direct) {
	*direct = false;
	if (!q->ctx->host_direct)
		return 0;
	void *d_in, *d_meta, *d_out, *d_v;
	if (!host_dev_ptr(lines, &d_in) || !host_dev_ptr(meta, &d_meta) || !host_dev_ptr(out_lines, &d_out)
	    || !host_dev_ptr(verdicts, &d_v))
		return 0;
	const uint32_t oflags = out_stride == GR_HIP_PREFIX ? GR_HIP_BATCH_F_PREFIX32 : 0;
	gr_hip_batch b = {d_in, d_out, static_cast<const gr_hip_pkt_meta *>(d_meta), static_cast<gr_hip_verdict *>(d_v),
			  n, GR_HIP_LINE, out_stride, GR_HIP_BATCH_F_LINES_ONLY | oflags};
	const int r = launch(q, q->s, &b, true);
	*direct = r == 0;
	if (r == 0)
		SYNC_CHECK(q->ctx, q->s, "direct launch");
	return r;
}

// Pageable host memory: through the queue's own pinned copies, in chunks,
// the CPU copying in and out around the pinned path. Pageable pointers never
// reach the runtime's asynchronous copies (a pageable copy once reported an
// illegal address after earlier tests had registered and unregistered host
// memory: DESIGN.md §4).
#define PG_CHUNK (1u << 20)
static int host_pageable(gr_hip_queue *q, const void *lines, const gr_hip_pkt_meta *meta, uint32_t n,
			 void *out_lines, uint32_t out_stride, gr_hip_verdict *verdicts) {
	const uint32_t cap = n < PG_CHUNK ? n : PG_CHUNK;
	if (q->pg_cap < cap) {
		hipHostFree(q->pg_lines);
		hipHostFree(q->pg_out);
		hipHostFree(q->pg_meta);
		hipHostFree(q->pg_v);
		q->pg_lines = q->pg_out = nullptr;
		q->pg_meta = nullptr;
		q->pg_v = nullptr;
		q->pg_cap = 0;
		if (hipHostMalloc(reinterpret_cast<void **>(&q->pg_lines), (size_t)cap * GR_HIP_LINE, hipHostMallocDefault) != hipSuccess
		    || hipHostMalloc(reinterpret_cast<void **>(&q->pg_out), (size_t)cap * GR_HIP_LINE, hipHostMallocDefault) != hipSuccess
		    || hipHostMalloc(reinterpret_cast<void **>(&q->pg_meta), (size_t)cap * sizeof(gr_hip_pkt_meta), hipHostMallocDefault) != hipSuccess
		    || hipHostMalloc(reinterpret_cast<void **>(&q->pg_v), (size_t)cap * sizeof(gr_hip_verdict), hipHostMallocDefault) != hipSuccess) {
			(void)hipGetLastError();
			return -ENOMEM;
		}
		q->pg_cap = cap;
	}
	const uint8_t *in = static_cast<const uint8_t *>(lines);
	uint8_t *out = static_cast<uint8_t *>(out_lines);
	int r = 0;
	for (uint32_t off = 0; off < n; off += cap) {
		const uint32_t cnt = n - off < cap ? n - off : cap;
		memcpy(q->pg_lines, in + (size_t)off * GR_HIP_LINE, (size_t)cnt * GR_HIP_LINE);
		memcpy(q->pg_meta, meta + off, (size_t)cnt * sizeof(*meta));
		const int e = gr_hip_fwd4_host_ex(q, q->pg_lines, q->pg_meta, cnt, q->pg_out, out_stride, q->pg_v);
		if (e < 0 && e != -ETIMEDOUT)
			return e;
		if (e == -ETIMEDOUT) // verdicts of packets never reached read back as 0xff: reported once
			r = e;
		memcpy(out + (size_t)off * out_stride, q->pg_out, (size_t)cnt * out_stride);
		memcpy(verdicts + off, q->pg_v, (size_t)cnt * sizeof(*verdicts));
	}
	return r;
}

extern "C" int gr_hip_fwd4_host_ex(
	gr_hip_queue_t *q,
	const void *lines,
	const struct gr_hip_pkt_meta *meta,
	uint32_t n,
	void *out_lines,
	uint32_t out_stride,
	struct gr_hip_verdict *verdicts
) {
	if (q == nullptr)
		return -EINVAL;
	if (n == 0)
		return 0;
	if (!lines || !meta || !out_lines || !verdicts || (out_stride != GR_HIP_LINE && out_stride != GR_HIP_PREFIX))
		return -EINVAL;
	const uint32_t oflags = out_stride == GR_HIP_PREFIX ? GR_HIP_BATCH_F_PREFIX32 : 0;
	gr_hip_ctx *c = q->ctx;
	hipSetDevice(c->dev);
	void *dp;
	if (!host_dev_ptr(lines, &dp) || !host_dev_ptr(meta, &dp) || !host_dev_ptr(out_lines, &dp)
	    || !host_dev_ptr(verdicts, &dp)) {
		const int r = host_pageable(q, lines, meta, n, out_lines, out_stride, verdicts);
		c->host_path_last.store(GR_HIP_HOST_PATH_PAGEABLE);
		return r;
	}
	std::shared_lock<std::shared_mutex> l(c->mu); // see gr_hip_fwd4_submit
	bool direct = false;
	if (const int r = host_direct_launch(q, lines, meta, n, out_lines, out_stride, verdicts, &direct); r < 0)
		return r;
	c->host_path_last.store(direct ? GR_HIP_HOST_PATH_DIRECT : GR_HIP_HOST_PATH_STAGED);
	if (direct) {
		l.unlock(); // enqueued: the wait needs no lock (see gr_hip_node_start)
		if (const int e_ = host_wait(q, q->s))
			return e_;
		return q_check(q);
	}
	for (host_slot &h : q->hs) {
		if (h.s != nullptr)
			continue;
		HCK(hipStreamCreateWithFlags(&h.s, hipStreamNonBlocking));
		HCK(hipMalloc(&h.in, (size_t)HOST_CHUNK * GR_HIP_LINE));
		HCK(hipMalloc(&h.out, (size_t)HOST_CHUNK * GR_HIP_LINE));
		HCK(hipMalloc(&h.meta, (size_t)HOST_CHUNK * sizeof(gr_hip_pkt_meta)));
		HCK(hipMalloc(&h.v, (size_t)HOST_CHUNK * sizeof(gr_hip_verdict)));
	}
	// the chunks follow everything already submitted on the queue
	HCK(hipEventRecord(q->quiesce, q->s));
	for (host_slot &h : q->hs)
		HCK(hipStreamWaitEvent(h.s, q->quiesce, 0));
	const uint8_t *in = static_cast<const uint8_t *>(lines);
	uint8_t *out = static_cast<uint8_t *>(out_lines);
	uint32_t k = 0;
	for (uint32_t off = 0; off < n; off += HOST_CHUNK, k++) {
		host_slot &h = q->hs[k % HOST_SLOTS];
		uint32_t cnt = n - off < HOST_CHUNK ? n - off : HOST_CHUNK;
		HCK(hipMemcpyAsync(h.in, in + (size_t)off * GR_HIP_LINE, (size_t)cnt * GR_HIP_LINE,
				   hipMemcpyHostToDevice, h.s));
		SYNC_CHECK(c, h.s, "lines H2D");
		HCK(hipMemcpyAsync(h.meta, meta + off, (size_t)cnt * sizeof(*meta), hipMemcpyHostToDevice, h.s));
		SYNC_CHECK(c, h.s, "meta H2D");
		// verdicts of packets a kernel that gave up never reached read back as 0xff
		HCK(hipMemsetAsync(h.v, 0xff, (size_t)cnt * sizeof(*verdicts), h.s));
		SYNC_CHECK(c, h.s, "verdict fill");
		gr_hip_batch b = {h.in, h.out, h.meta, h.v, cnt, GR_HIP_LINE, out_stride, GR_HIP_BATCH_F_LINES_ONLY | oflags};
		int r = launch(q, h.s, &b, false);
		if (r < 0)
			return r;
		SYNC_CHECK(c, h.s, "staged launch");
		HCK(hipMemcpyAsync(out + (size_t)off * out_stride, h.out, (size_t)cnt * out_stride,
				   hipMemcpyDeviceToHost, h.s));
		SYNC_CHECK(c, h.s, "lines D2H");
		HCK(hipMemcpyAsync(verdicts + off, h.v, (size_t)cnt * sizeof(*verdicts), hipMemcpyDeviceToHost, h.s));
		SYNC_CHECK(c, h.s, "verdicts D2H");
	}
	for (host_slot &h : q->hs) {
		if (const int e_ = host_wait(q, h.s))
			return e_;
	}
	return q_check(q);
}

extern "C" int gr_hip_fwd4_host(gr_hip_queue_t *q, const void *lines, const struct gr_hip_pkt_meta *meta, uint32_t n,
				void *out_lines, struct gr_hip_verdict *verdicts) {
	return gr_hip_fwd4_host_ex(q, lines, meta, n, out_lines, GR_HIP_LINE, verdicts);
}

// Registered host memory (gr_hip_host_register): host -> device address.
static const host_range *hreg_find(const gr_hip_ctx *c, uintptr_t p) {
	for (const host_range &r : c->hregs)
		if (p - r.host < r.len)
			return &r;
	return nullptr;
}

// Every frame in registered memory and 16-byte aligned: their device
// addresses into ptrs[pos[i]].
template <class F> static bool host_dev_ptrs(gr_hip_ctx *c, uint32_t n, F frame, uint64_t *ptrs, const uint32_t *pos) {
	// the caller holds c->mu
	if (c->hregs.empty())
		return false;
	const host_range *hit = &c->hregs[0];
	for (uint32_t i = 0; i < n; i++) {
		const uintptr_t p = reinterpret_cast<uintptr_t>(frame(i));
		if ((p & 15) || (p - hit->host >= hit->len && (hit = hreg_find(c, p)) == nullptr))
			return false;
		ptrs[pos[i]] = hit->dev + (p - hit->host);
	}
	return true;
}

static bool host_dev_ptr_ok(gr_hip_ctx *c, const gr_hip_mbuf *m, uint32_t n, uint64_t *ptrs, const uint32_t *pos) {
	return host_dev_ptrs(c, n, [m](uint32_t i) { return m[i].frame; }, ptrs, pos);
}

extern "C" int gr_hip_host_register(gr_hip_ctx_t *c, void *ptr, size_t bytes) {
	if (c == nullptr || ptr == nullptr || bytes == 0)
		return -EINVAL;
	std::lock_guard<std::shared_mutex> l(c->mu);
	hipSetDevice(c->dev);
	const uintptr_t p = reinterpret_cast<uintptr_t>(ptr);
	for (const host_range &r : c->hregs)
		if (p < r.host + r.len && r.host < p + bytes)
			return -EEXIST;
	host_range r = {p, 0, bytes, false};
	void *dp = nullptr;
	std::lock_guard<std::mutex> gl(g_hreg_mu);
	if (hreg_global_find(p, bytes) != nullptr) { // registered by us for another context
		hreg_global *g = hreg_global_find(p, bytes);
		g->refs++;
		r.dev = g->dev + (p - g->host);
		r.ours = true;
	} else if (host_dev_ptr(ptr, &dp)) { // pinned by someone else (hipHostMalloc, torch pin_memory)
		r.dev = reinterpret_cast<uintptr_t>(dp);
	} else {
		HCK(hipHostRegister(ptr, bytes, hipHostRegisterMapped));
		if (hipHostGetDevicePointer(&dp, ptr, 0) != hipSuccess || dp == nullptr) {
			(void)hipGetLastError();
			hipHostUnregister(ptr);
			return -EFAULT;
		}
		r.dev = reinterpret_cast<uintptr_t>(dp);
		r.ours = true;
		g_hregs.push_back({p, r.dev, bytes, 1});
	}
	c->hregs.push_back(r);
	return 0;
}

extern "C" int gr_hip_host_unregister(gr_hip_ctx_t *c, void *ptr) {
	if (c == nullptr || ptr == nullptr)
		return -EINVAL;
	std::lock_guard<std::shared_mutex> l(c->mu);
	hipSetDevice(c->dev);
	for (size_t i = 0; i < c->hregs.size(); i++) {
		if (c->hregs[i].host != reinterpret_cast<uintptr_t>(ptr))
			continue;
		// no kernel of this context may still read it: quiesce() orders the
		// control stream after every queue's work (and waits for resident
		// batches on the host); the host then waits for that stream, before
		// the runtime unmaps the range (an unmapped range read by a kernel
		// still running is an illegal address)
		if (const int r = quiesce(c))
			return r;
		if (const int r = ctl_sync(c))
			return r;
		const host_range hr = c->hregs[i];
		c->hregs.erase(c->hregs.begin() + (long)i);
		return hr.ours ? hreg_global_put(hr.host, hr.len) : 0;
	}
	return -ENOENT;
}

extern "C" int gr_hip_host_dev_addr(gr_hip_ctx_t *c, const void *ptr, uint64_t *dev) {
	if (c == nullptr || dev == nullptr)
		return -EINVAL;
	std::shared_lock<std::shared_mutex> l(c->mu);
	const host_range *r = hreg_find(c, reinterpret_cast<uintptr_t>(ptr));
	if (r == nullptr)
		return -ENOENT;
	*dev = r->dev + (reinterpret_cast<uintptr_t>(ptr) - r->host);
	return 0;
}

// A kernel that gave up (-ETIMEDOUT) wrote each 64-packet tile's lines and
// verdicts together or not at all (the storer stores a whole tile once it
// took it): a verdict still holding the fill value was not processed, its
// frame is untouched. Those packets go back to grout's CPU nodes (PUNT).
#define NODE_V_FILL 0xff

static uint32_t node_unfinished(const gr_hip_pkt_meta *meta, uint32_t n, const uint32_t *pos, gr_hip_verdict *v) {
	uint32_t k = 0;
	for (uint32_t i = 0; i < n; i++) {
		gr_hip_verdict &x = v[pos[i]];
		if (x.edge != NODE_V_FILL)
			continue;
		x = gr_hip_verdict{GR_HIP_E_PUNT, 0, meta[pos[i]].iface, 0}; // the view's iface, as staged
		k++;
	}
	return k;
}

// The node's walk (include/grout_hip.h, "rte_graph node shim"): lay the
// graph walks out on 64-packet tiles, stage the mbufs' header lines (or
// frame addresses) into one of the queue's pinned walk slots and enqueue the
// GPU work (gr_hip_node_start); wait for it and hand the walk back with the
// context's iface / nexthop mirrors (gr_hip_node_finish). With two slots the
// GPU forwards one walk while the CPU stages the next.
// Measurement: nanoseconds spent in the parts of gr_hip_node_start, summed
// over every queue (gr_hip_node_prof).
// Each thread's own cell (no line shared between workers), summed when read.
struct alignas(128) node_prof_cell {
	std::atomic<uint64_t> ns[GR_HIP_NODE_PROF_COUNT]; // one writer: the cell's thread
	void add(int k, uint64_t d) {
		ns[k].store(ns[k].load(std::memory_order_relaxed) + d, std::memory_order_relaxed);
	}
};
static std::mutex node_prof_mu;
static std::vector<node_prof_cell *> node_prof_cells; // kept for the process's life (a few per worker thread)

static node_prof_cell &node_prof_ns() {
	thread_local node_prof_cell *cell = nullptr;
	if (cell == nullptr) {
		cell = new node_prof_cell();
		std::lock_guard<std::mutex> l(node_prof_mu);
		node_prof_cells.push_back(cell);
	}
	return *cell;
}

static inline uint64_t prof_now() {
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

extern "C" int gr_hip_node_prof(uint64_t *out, uint32_t n, int reset) {
	std::lock_guard<std::mutex> l(node_prof_mu);
	for (uint32_t k = 0; k < GR_HIP_NODE_PROF_COUNT; k++) {
		uint64_t v = 0;
		for (node_prof_cell *c : node_prof_cells)
			v += reset ? c->ns[k].exchange(0) : c->ns[k].load();
		if (out != nullptr && k < n)
			out[k] = v;
	}
	return GR_HIP_NODE_PROF_COUNT;
}

// Pinned staging for ns slots; the first `keep` staged lines and metadata
// survive (an append growing the walk being staged).
static int slot_grow(node_slot &w, uint32_t ns, uint32_t keep) {
	if (ns <= w.cap)
		return 0;
	uint32_t cap = w.cap ? w.cap : 1024;
	while (cap < ns)
		cap = cap > UINT32_MAX / 2 ? ns : cap * 2;
	uint8_t *lines = nullptr, *out = nullptr;
	gr_hip_pkt_meta *meta = nullptr;
	gr_hip_verdict *v = nullptr;
	// fine-grained (coherent): the resident kernel reads a slot while it runs,
	// past any kernel boundary, which is the only point where coarse-grained
	// host memory is made coherent (its frame pointers read stale otherwise)
	const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
	if (hipHostMalloc((void **)&lines, (size_t)cap * GR_HIP_LINE, fl) != hipSuccess
	    || hipHostMalloc((void **)&out, (size_t)cap * GR_HIP_PREFIX, fl) != hipSuccess
	    || hipHostMalloc((void **)&meta, (size_t)cap * sizeof(gr_hip_pkt_meta), fl) != hipSuccess
	    || hipHostMalloc((void **)&v, (size_t)cap * sizeof(gr_hip_verdict), fl) != hipSuccess) {
		(void)hipGetLastError();
		hipHostFree(lines);
		hipHostFree(out);
		hipHostFree(meta);
		hipHostFree(v);
		return -ENOMEM;
	}
	if (keep) {
		memcpy(lines, w.lines, (size_t)keep * GR_HIP_LINE);
		memcpy(meta, w.meta, (size_t)keep * sizeof(gr_hip_pkt_meta));
	}
	hipHostFree(w.lines);
	hipHostFree(w.out);
	hipHostFree(w.meta);
	hipHostFree(w.v);
	w.lines = lines;
	w.out = out;
	w.meta = meta;
	w.v = v;
	w.cap = cap;
	// looked up once here, not per walk (hipPointerGetAttributes is slow)
	if (!host_dev_ptr(w.lines, &w.d_lines) || !host_dev_ptr(w.out, &w.d_out) || !host_dev_ptr(w.meta, &w.d_meta)
	    || !host_dev_ptr(w.v, &w.d_v))
		w.d_lines = w.d_out = w.d_meta = w.d_v = nullptr; // not device-accessible: staged copies
	return 0;
}

// The slot the next walk is staged into.
static node_slot &open_slot(gr_hip_queue_t *q) {
	return q->nw[(q->nw_head + q->nw_count) % GR_HIP_NODE_DEPTH];
}

extern "C" int gr_hip_node_append(gr_hip_queue_t *q, const struct gr_hip_mbuf *m, uint32_t n, uint32_t burst) {
	if (q == nullptr || (n && m == nullptr))
		return -EINVAL;
	if (q->dead)
		return -EIO; // (res_cancel) its slots may still be written by the GPU
	if (q->nw_count == GR_HIP_NODE_DEPTH)
		return -EBUSY;
	node_slot &w = open_slot(q);
	if (!w.open) {
		w.open = true;
		w.own = false;
		w.na = w.p = 0;
		w.lines_in = !q->ctx->node_ptrs;
	} else if (w.own || (n && !(m[0].flags & GR_HIP_MBUF_F_WALK))) {
		return -EINVAL; // each append is a walk (or walks) of its own, of views
	}
	if (n == 0)
		return (int)w.p;
	if (q->ctx->fail_appends.load(std::memory_order_relaxed) > 0 && q->ctx->fail_appends.fetch_sub(1) > 0)
		return -ENOMEM; // as a failed slot_grow: the slot is left as it was
	const bool prof = node_prof_on.load(std::memory_order_relaxed);
	const uint64_t t_prof = prof ? prof_now() : 0;
	if (w.pos.size() < (size_t)w.na + n)
		w.pos.resize(std::max<size_t>((size_t)w.na + n, 2 * w.pos.size()));
	uint32_t *pos = w.pos.data() + w.na;
	const uint64_t p = gr_node_layout_from(m, n, burst, w.p, pos);
	if (p > INT32_MAX)
		return -E2BIG;
	if (p > w.cap) {
		hipSetDevice(q->ctx->dev);
		int r = slot_grow(w, (uint32_t)p, w.p);
		if (r < 0)
			return r;
	}
	int r = gr_node_stage_from(m, n, burst, pos, w.p, w.lines_in ? w.lines : nullptr, w.meta);
	if (r < 0)
		return r;
	w.na += n;
	w.p = (uint32_t)p;
	if (prof)
		node_prof_ns().add(GR_HIP_NODE_PROF_STAGE, prof_now() - t_prof);
	return (int)p;
}

extern "C" int gr_hip_node_append_mbufs(gr_hip_queue_t *q, void *const *mbufs, uint32_t n,
					const struct gr_hip_mbuf_layout *lay, uint32_t burst) {
	if (q == nullptr || lay == nullptr || (n && mbufs == nullptr))
		return -EINVAL;
	if (q->dead)
		return -EIO; // (res_cancel) its slots may still be written by the GPU
	if (q->nw_count == GR_HIP_NODE_DEPTH)
		return -EBUSY;
	node_slot &w = open_slot(q);
	if (!w.open) {
		w.open = true;
		w.own = true;
		w.na = w.p = 0;
		w.lines_in = !q->ctx->node_ptrs;
		w.mb0 = mbufs;
		w.lay = lay;
	} else if (!w.own || mbufs != w.mb0 + w.na || lay != w.lay) {
		return -EINVAL; // views were appended to this slot, or not the mbufs that follow
	}
	if (n == 0)
		return (int)w.p;
	if (q->ctx->fail_appends.load(std::memory_order_relaxed) > 0 && q->ctx->fail_appends.fetch_sub(1) > 0)
		return -ENOMEM; // as a failed slot_grow: the slot is left as it was
	const bool prof = node_prof_on.load(std::memory_order_relaxed);
	const uint64_t t_prof = prof ? prof_now() : 0;
	const uint64_t p = gr_node_walk_end(w.p, n, burst); // the cuts do not depend on the mbufs
	if (p > INT32_MAX)
		return -E2BIG;
	if (p > w.cap) {
		hipSetDevice(q->ctx->dev);
		int r = slot_grow(w, (uint32_t)p, w.p);
		if (r < 0)
			return r;
	}
	const size_t need = (size_t)w.na + n;
	if (w.pos.size() < need)
		w.pos.resize(std::max(need, 2 * w.pos.size()));
	gr_node_stage_mbufs(mbufs, n, lay, burst, w.p, w.pos.data() + w.na, w.lines_in ? w.lines : nullptr, w.meta);
	w.na += n;
	w.p = (uint32_t)p;
	if (prof)
		node_prof_ns().add(GR_HIP_NODE_PROF_STAGE, prof_now() - t_prof);
	return (int)p;
}

extern "C" int gr_hip_node_discard(gr_hip_queue_t *q) {
	if (q == nullptr)
		return -EINVAL;
	if (q->nw_count < GR_HIP_NODE_DEPTH)
		open_slot(q).open = false;
	return 0;
}

extern "C" int gr_hip_node_send(gr_hip_queue_t *q, struct gr_hip_mbuf *m, uint32_t n, uint32_t burst) {
	if (q == nullptr)
		return -EINVAL;
	if (q->dead)
		return -EIO; // (res_cancel) its slots may still be written by the GPU
	if (q->nw_count == GR_HIP_NODE_DEPTH)
		return -EBUSY;
	gr_hip_ctx *c = q->ctx;
	node_slot &w = open_slot(q);
	const bool was_open = w.open;
	w.open = false;
	const bool own = was_open && w.own; // appended from the mbufs: no views
	w.own = own;
	if ((own ? m != nullptr : n && m == nullptr) || !(was_open ? w.na == n : n == 0))
		return -EINVAL; // not what was appended
	uint32_t *pos = w.pos.data();
	uint64_t t_prof = prof_now();
	auto lap = [&](int k) {
		const uint64_t t = prof_now();
		node_prof_ns().add(k, t - t_prof);
		t_prof = t;
	};
	const uint32_t ns = was_open ? w.p : 0;
	w.m = m;
	w.n = n;
	w.ns = ns;
	w.burst = burst;
	w.by_addr = false;
	w.sync = true;
	w.r = 0;
	w.kcount = false;
	w.resident = false;
	if (n == 0) { // nothing to send: finishes at once
		q->nw_count++;
		return 0;
	}
	hipSetDevice(c->dev);
	if (q->d_pad == nullptr) { // the frame a pad slot points at (frames by address)
		HCK(hipMalloc((void **)&q->d_pad, GR_HIP_LINE));
		HCK(hipMemset(q->d_pad, 0, GR_HIP_LINE));
	}
	memset(w.v, NODE_V_FILL, (size_t)ns * sizeof(gr_hip_verdict));
	lap(GR_HIP_NODE_PROF_PREP);
	std::shared_lock<std::shared_mutex> lk(c->mu); // see gr_hip_fwd4_submit
	lap(GR_HIP_NODE_PROF_LOCK);
	int r;
	bool enqueued = false;
	uint64_t *ptrs = reinterpret_cast<uint64_t *>(w.lines);
	auto mbuf_frame = [&w](uint32_t i) { return gr_node_frame(w.mb0[i], w.lay); };
	w.by_addr = !w.lines_in && c->node_ptrs
		&& (own ? host_dev_ptrs(c, n, mbuf_frame, ptrs, pos) : host_dev_ptr_ok(c, m, n, ptrs, pos));
	if (w.by_addr) {
		// the frames are device-accessible: hand them over by address, the
		// kernel reads and rewrites them in place over PCIe
		for (uint32_t i = 0, next = 0; i <= n; i++) { // pads point at a zeroed device line
			const uint32_t at = i < n ? pos[i] : ns;
			for (; next < at; next++)
				ptrs[next] = reinterpret_cast<uint64_t>(q->d_pad);
			next = at + 1;
		}
		if (w.d_lines == nullptr)
			return -EFAULT;
		gr_hip_batch b = {w.d_lines, nullptr, static_cast<const gr_hip_pkt_meta *>(w.d_meta),
				  static_cast<gr_hip_verdict *>(w.d_v), ns, 0, 0,
				  GR_HIP_BATCH_F_LINES_ONLY | GR_HIP_BATCH_F_FRAME_PTRS};
		// after everything already submitted on the queue, like gr_hip_fwd4_host;
		// no timing events (the walk's own completion event is enough)
		if (c->res_on && res_take(q)) {
			w.t_post = now_ns_host();
			if ((r = res_post(q, &b, &w.res)) < 0)
				return r;
			w.resident = true;
		} else if ((r = launch(q, q->s, &b, false)) < 0) {
			return r;
		}
		enqueued = true;
	} else {
		if (!w.lines_in) { // "node_ptrs" on, but not every frame is registered: stage the lines now
			if (own) { // the lines only: the metadata is staged
				for (uint32_t i = 0, next = 0; i < n; next = pos[i] + 1, i++) {
					for (; next < pos[i]; next++) // a pad slot
						memset(w.lines + (size_t)next * GR_HIP_LINE, 0, GR_HIP_LINE);
					memcpy(w.lines + (size_t)pos[i] * GR_HIP_LINE, mbuf_frame(i), GR_HIP_LINE);
				}
			} else if ((r = gr_node_stage_from(m, n, burst, pos, 0, w.lines, w.meta)) < 0) {
				return r;
			}
			lap(GR_HIP_NODE_PROF_STAGE);
		}
		// the hand-back writes back at most the first 26 bytes: packed
		// 32-byte prefixes come back, not whole lines
		if (c->host_direct && w.d_lines != nullptr) {
			// zero-copy (see host_direct_launch), on the slot's device addresses
			gr_hip_batch b = {w.d_lines, w.d_out, static_cast<const gr_hip_pkt_meta *>(w.d_meta),
					  static_cast<gr_hip_verdict *>(w.d_v), ns, GR_HIP_LINE, GR_HIP_PREFIX,
					  GR_HIP_BATCH_F_LINES_ONLY | GR_HIP_BATCH_F_PREFIX32};
			if (c->res_on && res_take(q)) {
				w.t_post = now_ns_host();
				if ((r = res_post(q, &b, &w.res)) < 0)
					return r;
				w.resident = true;
			} else if ((r = launch(q, q->s, &b, false)) < 0) {
				return r;
			}
			enqueued = true;
		}
		lap(GR_HIP_NODE_PROF_LAUNCH);
		if (!enqueued) { // not device-accessible: staged copies, waited for here
			lk.unlock(); // gr_hip_fwd4_host takes it itself
			w.r = gr_hip_fwd4_host_ex(q, w.lines, w.meta, ns, w.out, GR_HIP_PREFIX, w.v);
		}
	}
	if (enqueued) {
		if (!w.resident)
			HCK(hipEventRecord(w.done, q->s));
		w.sync = false;
	}
	// the kernel counted the walk's packets per iface (launch's "stats" variant;
	// the resident kernel counts none: the hand-back does)
	w.kcount = c->stats_on && q->d_stats != nullptr && !w.resident;
	if (w.kcount)
		q->node_counted++;
	lap(GR_HIP_NODE_PROF_RECORD);
	// the lock covers the enqueue, not the wait: control-plane writers
	// (FIB publication) are not held behind the walk's GPU time
	q->nw_count++;
	return 0;
}

extern "C" int gr_hip_node_start(gr_hip_queue_t *q, struct gr_hip_mbuf *m, uint32_t n, uint32_t burst) {
	if (q == nullptr || (n && m == nullptr))
		return -EINVAL;
	if (q->nw_count == GR_HIP_NODE_DEPTH)
		return -EBUSY;
	gr_hip_node_discard(q); // the whole walk at once: append it, send it
	int r = gr_hip_node_append(q, m, n, burst);
	if (r < 0) {
		gr_hip_node_discard(q);
		return r;
	}
	return gr_hip_node_send(q, m, n, burst);
}

static int node_finish(gr_hip_queue_t *q, struct gr_hip_mbuf **mp, uint32_t *np, struct gr_hip_node_stats *stats,
		       struct gr_node_direct *direct) {
	if (q == nullptr)
		return -EINVAL;
	if (q->nw_count == 0)
		return -ENOENT;
	gr_hip_ctx *c = q->ctx;
	node_slot &w = q->nw[q->nw_head];
	q->nw_head = (q->nw_head + 1) % GR_HIP_NODE_DEPTH;
	q->nw_count--;
	if (mp != nullptr)
		*mp = w.m;
	if (np != nullptr)
		*np = w.n;
	if (w.n == 0)
		return 0;
	int r = w.r;
	if (direct != nullptr)
		direct->meta = w.own ? w.meta : nullptr; // no views: the hand-back reads the mbufs
	uint64_t t_prof = prof_now();
	if (!w.sync && w.resident) {
		r = res_wait(q, w.res, w.t_post + (uint64_t)c->res_wait_ms * 1000000ull);
		if (q->res_inflight > 0 && --q->res_inflight == 0)
			c->res_busy.fetch_sub(1, std::memory_order_relaxed);
		if (r == -EDEADLK)
			return r; // the GPU may still run it: nothing of the walk is touched (q->dead)
		// retired unrun (here or by a control-plane wait), or the launch
		// faulted: what was not reached is punted, like a give-up
		if (r == 0 && res_was_cancelled(q, w.res))
			r = -ETIMEDOUT;
		if (r == -EIO)
			r = -ETIMEDOUT;
		if (r == 0)
			r = q_check(q);
	} else if (!w.sync) {
		hipSetDevice(c->dev);
		HCK(hipEventSynchronize(w.done));
		// the queue's error word covers every kernel in flight on it: which
		// walk a give-up hit is read from the verdicts below
		r = q_check(q);
	}
	// appended from the mbufs: gr_hip_node_finish_mbufs hands it back. Refused
	// only once the GPU is done with it (above): a caller that drops the walk
	// here (a graph destroyed with a batch in flight) frees its mbufs next,
	// whose frames the kernel may be rewriting in place
	if (direct == nullptr && w.own)
		return -EINVAL;
	if (r < 0 && r != -ETIMEDOUT)
		return r;
	uint64_t t = prof_now();
	node_prof_ns().add(GR_HIP_NODE_PROF_FIN_WAIT, t - t_prof);
	// packets a kernel that gave up never reached go back to grout's CPU
	// nodes, the others are handed back as usual
	const uint32_t unfinished = r == 0 ? 0 : node_unfinished(w.meta, w.n, w.pos.data(), w.v); // 0: none gave up
	t_prof = prof_now();
	node_prof_ns().add(GR_HIP_NODE_PROF_FIN_SCAN, t_prof - t);
	{
		std::shared_lock<std::shared_mutex> lk(c->mu); // the hand-back reads the iface and nexthop mirrors
		const gr_node_vlans vl = {c->vlan_keys_h.data(), c->vlan_vals_h.data(), (uint32_t)c->vlan_keys_h.size()};
		// the per-iface counters: the kernel's (gr_hip_node_iface_stats folds
		// them in), or the hand-back's when the kernel ran without them
		r = gr_node_apply_ex(w.m, w.n, w.burst, w.pos.data(), w.by_addr ? nullptr : w.out, GR_HIP_PREFIX, w.v,
				     c->ifaces.data(), c->max_ifaces, c->nh.data(), (uint32_t)c->nh.size(), stats, &vl,
				     w.kcount ? nullptr : q->node_if.data(), (uint32_t)q->node_if.size(), direct);
	}
	node_prof_ns().add(GR_HIP_NODE_PROF_FIN_APPLY, prof_now() - t_prof);
	return r < 0 ? r : (int)unfinished;
}

extern "C" int gr_hip_node_finish(gr_hip_queue_t *q, struct gr_hip_mbuf **mp, uint32_t *np,
				  struct gr_hip_node_stats *stats) {
	return node_finish(q, mp, np, stats, nullptr);
}

extern "C" int gr_hip_node_finish_mbufs(gr_hip_queue_t *q, void *const *mbufs, const struct gr_hip_mbuf_layout *layout,
					uint8_t *edges, uint32_t *stale, struct gr_hip_node_stats *stats) {
	if (mbufs == nullptr || layout == nullptr || edges == nullptr)
		return -EINVAL;
	gr_node_direct d = {mbufs, layout, edges, 0, nullptr};
	const int r = node_finish(q, nullptr, nullptr, stats, &d);
	if (stale != nullptr)
		*stale = d.stale;
	return r;
}

// The d_stats totals of a complete snapshot (or of `all`, a whole copy
// [FWD4_STAT_SHARDS][max_ifaces]) folded into node_if: what the kernels
// counted since the last fold. (gr_hip_queue_stats' reset zeroes d_stats:
// the totals then restart below what was folded.)
static void kern_fold(gr_hip_queue_t *q, const gr_hip_iface_stats *all, uint32_t w, uint32_t pitch) {
	auto since = [](uint64_t now, uint64_t seen) { return now >= seen ? now - seen : now; };
	for (uint32_t i = 0; i < w; i++) {
		gr_hip_iface_stats t = {0, 0, 0, 0};
		for (uint32_t s = 0; s < FWD4_STAT_SHARDS; s++) {
			const gr_hip_iface_stats &x = all[(size_t)s * pitch + i];
			t.rx_packets += x.rx_packets;
			t.rx_bytes += x.rx_bytes;
			t.tx_packets += x.tx_packets;
			t.tx_bytes += x.tx_bytes;
		}
		gr_hip_iface_stats &seen = q->kern_seen[i], &acc = q->node_if[i];
		acc.rx_packets += since(t.rx_packets, seen.rx_packets);
		acc.rx_bytes += since(t.rx_bytes, seen.rx_bytes);
		acc.tx_packets += since(t.tx_packets, seen.tx_packets);
		acc.tx_bytes += since(t.tx_bytes, seen.tx_bytes);
		seen = t;
	}
}

// A pinned, coherent, device-mapped buffer of at least `n` counter entries
// (gr_stats_collect's destination), grown on demand.
static int stats_buf(gr_hip_iface_stats **h, void **d, uint32_t *cap, uint32_t n) {
	if (*cap >= n)
		return 0;
	hipHostFree(*h);
	*h = nullptr;
	*d = nullptr;
	*cap = 0;
	if (hipHostMalloc(reinterpret_cast<void **>(h), sizeof(gr_hip_iface_stats) * n,
			  hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess
	    || hipHostGetDevicePointer(d, *h, 0) != hipSuccess) {
		(void)hipGetLastError();
		hipHostFree(*h);
		*h = nullptr;
		*d = nullptr;
		return -ENOMEM;
	}
	*cap = n;
	return 0;
}

// Copy d_stats' first snap_w ifaces of every shard into the pinned snapshot
// behind the queue's work (gr_stats_collect: read at the memory side), and
// mark it pending.
static int snap_start(gr_hip_queue_t *q) {
	gr_hip_ctx *c = q->ctx;
	std::shared_lock<std::shared_mutex> lk(c->mu); // the iface mirror
	uint32_t w = 0; // the ifaces in use: ids below the highest one pushed
	for (uint32_t i = c->max_ifaces; i-- > 1;)
		if (c->ifaces[i].id != 0) {
			w = i + 1;
			break;
		}
	if (w == 0)
		w = 1;
	if (q->snap_ev == nullptr)
		HCK(hipEventCreateWithFlags(&q->snap_ev, hipEventDisableTiming));
	uint32_t cap = q->snap_cap * FWD4_STAT_SHARDS;
	if (const int r = stats_buf(&q->snap, &q->snap_d, &cap, w * FWD4_STAT_SHARDS))
		return q->snap_cap = 0, r;
	q->snap_cap = cap / FWD4_STAT_SHARDS;
	HCK(gr_stats_collect_launch(q->d_stats, q->snap_d, w, c->max_ifaces, FWD4_STAT_SHARDS, 0, q->s));
	HCK(hipEventRecord(q->snap_ev, q->s));
	q->snap_w = w;
	q->snap_pending = true;
	q->snap_counted = q->node_counted;
	return 0;
}

extern "C" int gr_hip_node_iface_stats(gr_hip_queue_t *q, struct gr_hip_iface_stats *st, uint32_t max, int reset) {
	if (q == nullptr || (st == nullptr && max))
		return -EINVAL;
	// the kernels' counts: a snapshot of d_stats behind the walks launched so
	// far, folded when it has landed (a poll). With no walk in flight the
	// counts are final: wait for the snapshot, so that the result is exact
	// (a housekeeping tick with walks on the GPU reports them at a later one).
	if (q->d_stats != nullptr && (q->snap_pending || q->snap_counted != q->node_counted)) {
		const bool idle = q->nw_count == 0;
		hipSetDevice(q->ctx->dev);
		for (int pass = 0; pass < 2; pass++) {
			if (q->snap_pending) {
				if (idle)
					HCK(hipEventSynchronize(q->snap_ev));
				const hipError_t e = idle ? hipSuccess : hipEventQuery(q->snap_ev);
				if (e == hipSuccess) {
					kern_fold(q, q->snap, q->snap_w, q->snap_w);
					q->snap_pending = false;
				} else if (e != hipErrorNotReady) {
					return -EIO;
				}
				(void)hipGetLastError();
			}
			if (q->snap_pending || q->snap_counted == q->node_counted)
				break;
			if (const int r = snap_start(q))
				return r;
			if (!idle)
				break; // folded at a later call
		}
	}
	const uint32_t m = max < q->node_if.size() ? max : (uint32_t)q->node_if.size();
	if (m)
		memcpy(st, q->node_if.data(), (size_t)m * sizeof(*st));
	if (max > m)
		memset(st + m, 0, (size_t)(max - m) * sizeof(*st));
	if (reset)
		std::fill(q->node_if.begin(), q->node_if.end(), gr_hip_iface_stats{0, 0, 0, 0});
	return 0;
}

extern "C" int gr_hip_node_pending(gr_hip_queue_t *q, int *ready) {
	if (q == nullptr)
		return -EINVAL;
	if (ready != nullptr) {
		*ready = 0;
		if (q->nw_count) {
			const node_slot &w = q->nw[q->nw_head];
			if (w.sync) {
				*ready = 1;
			} else if (w.resident) { // a load of the ring's done word; a kernel that left is relaunched
				gr_hip_ctx *c = q->ctx;
				if (res_is_done(q, w.res)) {
					*ready = 1;
				} else if (c->res_dead || res_kick(c) != 0) {
					return -EIO; // node_finish sorts it out (res_wait, res_cancel)
				} else if ((++q->res_polls & 255) == 0) {
					// bounded like res_wait: past the batch's deadline, or a
					// launch that faulted, node_finish cancels it
					const hipError_t e = hipEventQuery(c->res_ev);
					if (e != hipSuccess && e != hipErrorNotReady) {
						(void)hipGetLastError();
						return -EIO;
					}
					if (now_ns_host() - w.t_post > (uint64_t)c->res_wait_ms * 1000000ull)
						return -ETIMEDOUT;
				}
			} else {
				hipSetDevice(q->ctx->dev);
				const hipError_t e = hipEventQuery(w.done);
				if (e == hipSuccess)
					*ready = 1;
				else if (e != hipErrorNotReady)
					return -EIO;
				(void)hipGetLastError();
			}
		}
	}
	return (int)q->nw_count;
}

extern "C" int gr_hip_node_process(gr_hip_queue_t *q, struct gr_hip_mbuf *m, uint32_t n, uint32_t burst,
				   struct gr_hip_node_stats *stats) {
	if (q == nullptr || (n && m == nullptr))
		return -EINVAL;
	if (n == 0)
		return 0;
	if (q->nw_count)
		return -EBUSY; // finish the pipelined walks first
	const int r = gr_hip_node_start(q, m, n, burst);
	if (r < 0)
		return r;
	return gr_hip_node_finish(q, nullptr, nullptr, stats);
}

// Every shard's counters of every iface into q->rd ([FWD4_STAT_SHARDS][max_ifaces]),
// behind all the queue's work, read at the memory side (gr_stats_collect; with
// `reset` zeroed by the same atomics: no memset whose zeroes an XCD's L2 might
// hold). Node walks' counts not folded yet go to node_if first.
static int stats_collect_all(gr_hip_queue *q, bool reset) {
	gr_hip_ctx *c = q->ctx;
	if (q->d_stats == nullptr)
		return -ENOMEM;
	hipSetDevice(c->dev);
	if (const int e_ = host_wait(q, q->s))
		return e_;
	for (host_slot &h : q->hs)
		if (h.s)
			if (const int e_ = host_wait(q, h.s))
				return e_;
	if (const int r = stats_buf(&q->rd, &q->rd_d, &q->rd_cap, FWD4_STAT_SHARDS * c->max_ifaces))
		return r;
	const size_t bytes = sizeof(gr_hip_iface_stats) * FWD4_STAT_SHARDS * c->max_ifaces;
	if (c->stats_copy) { // measurement only (tools/stats_read_probe.py): round 5's copy and memset
		HCK(hipMemcpy(q->rd, q->d_stats, bytes, hipMemcpyDeviceToHost));
		if (reset)
			HCK(hipMemsetAsync(q->d_stats, 0, bytes, q->s));
	} else {
		HCK(gr_stats_collect_launch(q->d_stats, q->rd_d, c->max_ifaces, c->max_ifaces, FWD4_STAT_SHARDS,
					    reset ? 1 : 0, q->s));
		if (const int e_ = host_wait(q, q->s))
			return e_;
	}
	if (reset) {
		// node walks' counts not folded yet go to node_if before the zeroing
		// (a queue of node walks and plain submits at once reports both there)
		if (q->snap_counted != q->node_counted || q->snap_pending) {
			kern_fold(q, q->rd, c->max_ifaces, c->max_ifaces);
			q->snap_pending = false;
			q->snap_counted = q->node_counted;
		}
		std::fill(q->kern_seen.begin(), q->kern_seen.end(), gr_hip_iface_stats{0, 0, 0, 0});
	}
	return 0;
}

extern "C" int gr_hip_queue_stats_shards(gr_hip_queue_t *q, struct gr_hip_iface_stats *st, uint32_t w, int reset) {
	if (q == nullptr || (st == nullptr && w))
		return -EINVAL;
	if (const int r = stats_collect_all(q, reset != 0))
		return r;
	const uint32_t mi = q->ctx->max_ifaces, m = w < mi ? w : mi;
	for (uint32_t s = 0; s < FWD4_STAT_SHARDS; s++) {
		memcpy(st + (size_t)s * w, q->rd + (size_t)s * mi, (size_t)m * sizeof(*st));
		if (w > m)
			memset(st + (size_t)s * w + m, 0, (size_t)(w - m) * sizeof(*st));
	}
	return FWD4_STAT_SHARDS;
}

extern "C" int gr_hip_queue_stats(gr_hip_queue_t *q, struct gr_hip_iface_stats *st, uint32_t max, int reset) {
	if (q == nullptr || (st == nullptr && max))
		return -EINVAL;
	gr_hip_ctx *c = q->ctx;
	if (const int r = stats_collect_all(q, reset != 0))
		return r;
	uint32_t m = max < c->max_ifaces ? max : c->max_ifaces;
	memset(st, 0, (size_t)max * sizeof(*st));
	for (uint32_t s = 0; s < FWD4_STAT_SHARDS; s++) {
		for (uint32_t i = 0; i < m; i++) {
			const gr_hip_iface_stats &x = q->rd[(size_t)s * c->max_ifaces + i];
			st[i].rx_packets += x.rx_packets;
			st[i].rx_bytes += x.rx_bytes;
			st[i].tx_packets += x.tx_packets;
			st[i].tx_bytes += x.tx_bytes;
		}
	}
	return 0;
}

// ---------------------------------------------------------------------------
// memory helpers
// ---------------------------------------------------------------------------

extern "C" int gr_hip_dev_alloc(gr_hip_ctx_t *c, size_t bytes, void **p) {
	if (c == nullptr || p == nullptr)
		return -EINVAL;
	hipSetDevice(c->dev);
	HCK(hipMalloc(p, bytes));
	return 0;
}

extern "C" int gr_hip_dev_free(gr_hip_ctx_t *c, void *p) {
	if (c == nullptr)
		return -EINVAL;
	HCK(hipFree(p));
	return 0;
}

extern "C" int gr_hip_batch_alloc(gr_hip_ctx_t *c, uint32_t n, uint32_t in_stride, gr_hip_batch *b) {
	if (c == nullptr || b == nullptr || n == 0 || n > (1u << 31) || in_stride < GR_HIP_LINE || (in_stride & 15))
		return -EINVAL;
	hipSetDevice(c->dev);
	const size_t sizes[4] = {(size_t)n * in_stride, (size_t)n * GR_HIP_LINE, (size_t)n * 8, (size_t)n * 8};
	void *p[4] = {nullptr, nullptr, nullptr, nullptr};
	for (int k = 0; k < 4; k++)
		if (dev_alloc(c, &p[k], sizes[k]) != hipSuccess || hipMemset(p[k], 0, sizes[k]) != hipSuccess) {
			(void)hipGetLastError();
			for (void *q : p)
				if (q)
					hipFree(q);
			return -ENOMEM;
		}
	b->in_frames = p[0];
	b->out_lines = p[1];
	b->meta = static_cast<gr_hip_pkt_meta *>(p[2]);
	b->verdicts = static_cast<gr_hip_verdict *>(p[3]);
	b->n = n;
	b->in_stride = in_stride;
	b->out_stride = GR_HIP_LINE;
	b->flags = 0;
	return 0;
}

// Kernel time of batch t on the probe queue q: 3 warm-up launches, 6 timed
// (the first `warm` extra launches bring the clock up before any probe).
static int place_time(gr_hip_queue *q, const gr_hip_batch &t, float *ms, int warm = 0) {
	constexpr int TIMED = 6;
	for (int i = 0; i < warm + 3 + TIMED; i++) {
		const int r = gr_hip_fwd4_submit(q, &t);
		if (r)
			return r;
	}
	uint32_t cnt = 0; // the last TIMED launches
	const int r = gr_hip_queue_kernel_ms(q, TIMED, ms, &cnt);
	return r ? r : cnt == TIMED ? 0 : -EIO; // the probes must all be timed
}

// Up to `candidates` more device buffers of `bytes` each (fewer when memory
// runs short), after `cur`. With "alloc_contig" the candidates alternate
// between plain and physically contiguous allocations: which kind lands in
// the fast translation class differs from box to box.
static std::vector<void *> place_alloc(const gr_hip_ctx *c, void *cur, size_t bytes, uint32_t candidates) {
	std::vector<void *> v{cur};
	for (uint32_t k = 0; k < candidates; k++) {
		void *o = nullptr;
		if ((c->alloc_contig && k % 2 == 0 ? hipMalloc(&o, bytes) : dev_alloc(c, &o, bytes)) != hipSuccess) {
			(void)hipGetLastError();
			break;
		}
		v.push_back(o);
	}
	return v;
}

extern "C" int gr_hip_batch_place(gr_hip_ctx_t *c, gr_hip_batch *b, uint32_t candidates) {
	const bool prefix = b != nullptr && (b->flags & GR_HIP_BATCH_F_PREFIX32);
	if (c == nullptr || b == nullptr || b->out_lines == nullptr
	    || b->out_stride != (prefix ? (uint32_t)GR_HIP_PREFIX : (uint32_t)GR_HIP_LINE) || candidates > 16
	    || (b->flags & GR_HIP_BATCH_F_FRAME_PTRS))
		return -EINVAL;
	int r = batch_ok(b);
	if (r <= 0)
		return r ? r : -EINVAL;
	hipSetDevice(c->dev);
	if (candidates == 0)
		return 0;
	gr_hip_queue_t *q = nullptr;
	if ((r = gr_hip_queue_create(c, nullptr, &q)) != 0)
		return r;
	// no counters on this queue: the probe launches run the counter-less
	// kernel variant, so they neither count nor show up as the counted one
	hipStreamSynchronize(q->s);
	hipFree(q->d_stats);
	q->d_stats = nullptr;
	q->always_timed = true; // "untimed" / "time_every" do not apply to the probes
	// 1. the output lines: candidates against the current buffer
	std::vector<void *> outs = place_alloc(c, b->out_lines, (size_t)b->n * b->out_stride, candidates);
	size_t pick = 0;
	float best = 0;
	for (size_t k = 0; k < outs.size() && r == 0; k++) {
		gr_hip_batch t = *b;
		t.out_lines = outs[k];
		float ms = 0;
		if ((r = place_time(q, t, &ms, k == 0 ? 32 : 0)) == 0 && (k == 0 || ms < best)) {
			best = ms;
			pick = k;
		}
	}
	// 2. the frames, against the lines just kept: each candidate gets a
	// copy of the batch's frames (the pair decides)
	const size_t in_b = (size_t)b->n * b->in_stride;
	std::vector<void *> ins{const_cast<void *>(b->in_frames)};
	size_t pick_in = 0;
	if (r == 0) {
		ins = place_alloc(c, const_cast<void *>(b->in_frames), in_b, candidates);
		for (size_t k = 1; k < ins.size() && r == 0; k++) {
			if (hipMemcpyAsync(ins[k], b->in_frames, in_b, hipMemcpyDeviceToDevice, q->s) != hipSuccess) {
				(void)hipGetLastError();
				r = -EIO;
				break;
			}
			gr_hip_batch t = *b;
			t.in_frames = ins[k];
			t.out_lines = outs[pick];
			float ms = 0;
			if ((r = place_time(q, t, &ms)) == 0 && ms < best) {
				best = ms;
				pick_in = k;
			}
		}
	}
	if (r == 0)
		r = gr_hip_queue_sync(q);
	gr_hip_queue_destroy(q);
	if (r)
		pick = pick_in = 0; // keep the batch as it was
	for (size_t k = 0; k < outs.size(); k++)
		if (k != pick)
			hipFree(outs[k]);
	for (size_t k = 0; k < ins.size(); k++)
		if (k != pick_in)
			hipFree(ins[k]);
	b->out_lines = outs[pick];
	b->in_frames = ins[pick_in];
	return r;
}

extern "C" int gr_hip_batch_free(gr_hip_ctx_t *c, gr_hip_batch *b) {
	if (c == nullptr || b == nullptr)
		return -EINVAL;
	hipSetDevice(c->dev);
	for (const void *p : {b->in_frames, static_cast<const void *>(b->out_lines), static_cast<const void *>(b->meta),
			      static_cast<const void *>(b->verdicts)})
		if (p)
			hipFree(const_cast<void *>(p));
	memset(b, 0, sizeof(*b));
	return 0;
}

extern "C" int gr_hip_host_alloc(gr_hip_ctx_t *c, size_t bytes, void **p) {
	if (c == nullptr || p == nullptr)
		return -EINVAL;
	hipSetDevice(c->dev);
	HCK(hipHostMalloc(p, bytes, hipHostMallocDefault));
	return 0;
}

extern "C" int gr_hip_host_free(gr_hip_ctx_t *c, void *p) {
	if (c == nullptr)
		return -EINVAL;
	HCK(hipHostFree(p));
	return 0;
}

extern "C" int gr_hip_memcpy_h2d(gr_hip_ctx_t *c, void *dst, const void *src, size_t n) {
	if (c == nullptr)
		return -EINVAL;
	hipSetDevice(c->dev);
	HCK(hipMemcpy(dst, src, n, hipMemcpyHostToDevice));
	return 0;
}

extern "C" int gr_hip_memcpy_d2h(gr_hip_ctx_t *c, void *dst, const void *src, size_t n) {
	if (c == nullptr)
		return -EINVAL;
	hipSetDevice(c->dev);
	HCK(hipMemcpy(dst, src, n, hipMemcpyDeviceToHost));
	return 0;
}
