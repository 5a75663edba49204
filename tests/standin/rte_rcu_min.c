// SPDX-License-Identifier: BSD-3-Clause
//
// rte_rcu_min.c -- the QSBR stand-in behind rte_rcu_min.h.
#include "rte_rcu_min.h"

#include <errno.h>
#include <sched.h>
#include <string.h>

size_t rte_rcu_qsbr_get_memsize(uint32_t max_threads) {
	return sizeof(struct rte_rcu_qsbr) + (size_t)max_threads * sizeof(struct rte_rcu_qsbr_cnt);
}

int rte_rcu_qsbr_init(struct rte_rcu_qsbr *v, uint32_t max_threads) {
	if (v == NULL || max_threads == 0)
		return -EINVAL;
	memset(v, 0, rte_rcu_qsbr_get_memsize(max_threads));
	v->token = RTE_QSBR_CNT_INIT;
	v->max_threads = max_threads;
	return 0;
}

int rte_rcu_qsbr_thread_register(struct rte_rcu_qsbr *v, unsigned int thread_id) {
	if (v == NULL || thread_id >= v->max_threads)
		return -EINVAL;
	struct rte_rcu_qsbr_cnt *c = &v->qsbr_cnt[thread_id];
	if (__atomic_exchange_n(&c->registered, 1u, __ATOMIC_ACQ_REL) == 0)
		__atomic_fetch_add(&v->num_threads, 1u, __ATOMIC_RELAXED);
	return 0;
}

int rte_rcu_qsbr_thread_unregister(struct rte_rcu_qsbr *v, unsigned int thread_id) {
	if (v == NULL || thread_id >= v->max_threads)
		return -EINVAL;
	struct rte_rcu_qsbr_cnt *c = &v->qsbr_cnt[thread_id];
	__atomic_store_n(&c->cnt, (uint64_t)RTE_QSBR_CNT_THR_OFFLINE, __ATOMIC_RELEASE);
	if (__atomic_exchange_n(&c->registered, 0u, __ATOMIC_ACQ_REL) != 0)
		__atomic_fetch_sub(&v->num_threads, 1u, __ATOMIC_RELAXED);
	return 0;
}

uint64_t rte_rcu_qsbr_start(struct rte_rcu_qsbr *v) {
	return __atomic_add_fetch(&v->token, 1, __ATOMIC_RELEASE);
}

int rte_rcu_qsbr_check(struct rte_rcu_qsbr *v, uint64_t t, bool wait) {
	for (uint32_t i = 0; i < v->max_threads; i++) {
		const struct rte_rcu_qsbr_cnt *c = &v->qsbr_cnt[i];
		for (;;) {
			if (!__atomic_load_n(&c->registered, __ATOMIC_ACQUIRE))
				break;
			const uint64_t n = __atomic_load_n(&c->cnt, __ATOMIC_ACQUIRE);
			if (n == RTE_QSBR_CNT_THR_OFFLINE || n >= t)
				break;
			if (!wait)
				return 0;
			sched_yield();
		}
	}
	return 1;
}

void rte_rcu_qsbr_synchronize(struct rte_rcu_qsbr *v, unsigned int thread_id) {
	const uint64_t t = rte_rcu_qsbr_start(v);
	if (thread_id != RTE_QSBR_THRID_INVALID) // the caller's own read side is past
		rte_rcu_qsbr_quiescent(v, thread_id);
	rte_rcu_qsbr_check(v, t, true);
}
