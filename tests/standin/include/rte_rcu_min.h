// SPDX-License-Identifier: BSD-3-Clause
//
// rte_rcu_min.h -- a stand-in for DPDK's QSBR RCU (lib/rcu, rte_rcu_qsbr.h in
// DPDK 25.11, which grout pins: subprojects/dpdk-25.11.wrap), so that the
// fast path's grout node can be held to grout's reader contract here, where
// DPDK is not installed. Only the names, argument meanings and the semantics
// grout relies on follow DPDK; the implementation is this repo's:
//
//   * readers are thread ids < max_threads, registered once; a registered
//     reader is offline until rte_rcu_qsbr_thread_online();
//   * a writer's rte_rcu_qsbr_start() takes a new token; rte_rcu_qsbr_check()
//     is done once every registered reader that is online has reported a
//     quiescent state (rte_rcu_qsbr_quiescent) at or after that token, or
//     went offline;
//   * rte_rcu_qsbr_synchronize() = start + check(wait), what grout's control
//     plane calls before freeing an object the datapath may still read
//     (modules/infra/control/nexthop.c:505, iface.c:712, route.c:764).
//
// grout's worker registers its lcore id, goes online when it picks up a graph
// and reports quiescent every 256 graph walks
// (modules/infra/datapath/main_loop.c:408,441,464).
#pragma once

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTE_QSBR_THRID_INVALID 0xffffffffu
#define RTE_QSBR_CNT_THR_OFFLINE 0
#define RTE_QSBR_CNT_INIT 1

struct rte_rcu_qsbr_cnt {
	uint64_t cnt; // last token seen by the reader; RTE_QSBR_CNT_THR_OFFLINE when offline
	uint32_t registered;
} __attribute__((aligned(64)));

struct rte_rcu_qsbr {
	uint64_t token __attribute__((aligned(64))); // the writers' counter
	uint32_t max_threads;
	uint32_t num_threads; // registered readers
	struct rte_rcu_qsbr_cnt qsbr_cnt[] __attribute__((aligned(64)));
};

size_t rte_rcu_qsbr_get_memsize(uint32_t max_threads);
// 0, or -EINVAL (DPDK: 1 + rte_errno).
int rte_rcu_qsbr_init(struct rte_rcu_qsbr *v, uint32_t max_threads);
int rte_rcu_qsbr_thread_register(struct rte_rcu_qsbr *v, unsigned int thread_id);
int rte_rcu_qsbr_thread_unregister(struct rte_rcu_qsbr *v, unsigned int thread_id);

// The reader starts reading shared data: everything it reads from now on is
// protected against writers that start after this point.
static inline void rte_rcu_qsbr_thread_online(struct rte_rcu_qsbr *v, unsigned int thread_id) {
	const uint64_t t = __atomic_load_n(&v->token, __ATOMIC_RELAXED);
	__atomic_store_n(&v->qsbr_cnt[thread_id].cnt, t, __ATOMIC_RELAXED);
	// the reader's later loads of shared data must not pass the store
	__atomic_thread_fence(__ATOMIC_SEQ_CST);
}

// The reader holds no reference to shared data any more.
static inline void rte_rcu_qsbr_thread_offline(struct rte_rcu_qsbr *v, unsigned int thread_id) {
	__atomic_store_n(&v->qsbr_cnt[thread_id].cnt, (uint64_t)RTE_QSBR_CNT_THR_OFFLINE, __ATOMIC_RELEASE);
}

// The reader holds no reference taken before this point.
static inline void rte_rcu_qsbr_quiescent(struct rte_rcu_qsbr *v, unsigned int thread_id) {
	const uint64_t t = __atomic_load_n(&v->token, __ATOMIC_ACQUIRE);
	__atomic_store_n(&v->qsbr_cnt[thread_id].cnt, t, __ATOMIC_RELEASE);
}

uint64_t rte_rcu_qsbr_start(struct rte_rcu_qsbr *v);
// 1 when every online reader has passed token t; with wait, spins until then.
int rte_rcu_qsbr_check(struct rte_rcu_qsbr *v, uint64_t t, bool wait);
// thread_id: the caller's own reader id (reports quiescent after the start),
// or RTE_QSBR_THRID_INVALID for a thread that is not a reader.
void rte_rcu_qsbr_synchronize(struct rte_rcu_qsbr *v, unsigned int thread_id);

#ifdef __cplusplus
}
#endif
