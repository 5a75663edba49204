// SPDX-License-Identifier: BSD-3-Clause
//
// node_mt.c -- the node walk from K C threads (tools/node_pipeline.py
// --driver c): no Python between the library calls, so that depth 1
// (gr_hip_node_process per flush) and depth 2 (gr_hip_node_start of flush i,
// gr_hip_node_finish of flush i-1) are compared on the library alone.
//
//   cc -O2 -pthread -shared -fPIC -Iinclude -o tools/libnode_mt.so tools/node_mt.c -Lgrout_amd -lgrout_hip
#include <grout_hip.h>

#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <time.h>

struct job {
	gr_hip_queue_t *q;
	struct gr_hip_mbuf *m;
	uint32_t n, flush;
	int depth;
	int err;
	pthread_barrier_t *bar;
};

static int walk(struct job *j) {
	int r;
	if (j->depth < 2) {
		for (uint32_t o = 0; o < j->n; o += j->flush) {
			const uint32_t k = j->n - o < j->flush ? j->n - o : j->flush;
			if ((r = gr_hip_node_process(j->q, j->m + o, k, 64, NULL)) < 0)
				return r;
		}
		return 0;
	}
	for (uint32_t o = 0; o < j->n; o += j->flush) {
		const uint32_t k = j->n - o < j->flush ? j->n - o : j->flush;
		if ((r = gr_hip_node_start(j->q, j->m + o, k, 64)) < 0)
			return r;
		if (o && (r = gr_hip_node_finish(j->q, NULL, NULL, NULL)) < 0)
			return r;
	}
	r = gr_hip_node_finish(j->q, NULL, NULL, NULL);
	return r < 0 ? r : 0;
}

static void *run(void *arg) {
	struct job *j = arg;
	pthread_barrier_wait(j->bar);
	j->err = walk(j);
	pthread_barrier_wait(j->bar);
	return NULL;
}

// One round: every thread walks its mbufs once, between two barriers.
// Returns 0 and the round's wall time, or the first thread's -errno.
int node_mt_round(gr_hip_queue_t **queues, struct gr_hip_mbuf **mbufs, uint32_t threads, uint32_t n, uint32_t flush,
		  int depth, double *seconds) {
	if (threads == 0 || threads > 64 || flush == 0)
		return -EINVAL;
	pthread_barrier_t bar;
	pthread_barrier_init(&bar, NULL, threads + 1);
	struct job jobs[64];
	pthread_t th[64];
	for (uint32_t i = 0; i < threads; i++) {
		jobs[i] = (struct job) {queues[i], mbufs[i], n, flush, depth, 0, &bar};
		pthread_create(&th[i], NULL, run, &jobs[i]);
	}
	struct timespec a, b;
	pthread_barrier_wait(&bar);
	clock_gettime(CLOCK_MONOTONIC, &a);
	pthread_barrier_wait(&bar);
	clock_gettime(CLOCK_MONOTONIC, &b);
	int err = 0;
	for (uint32_t i = 0; i < threads; i++) {
		pthread_join(th[i], NULL);
		if (jobs[i].err < 0 && err == 0)
			err = jobs[i].err;
	}
	pthread_barrier_destroy(&bar);
	*seconds = (double)(b.tv_sec - a.tv_sec) + (double)(b.tv_nsec - a.tv_nsec) * 1e-9;
	return err;
}
