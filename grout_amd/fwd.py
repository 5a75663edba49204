# SPDX-License-Identifier: BSD-3-Clause
"""Python handle on the HIP fast path (thin layer over include/grout_hip.h).

Mirrors the way grout's control plane drives the datapath: objects are
pushed with iface/nexthop/route calls (modules/infra/control/*.c,
modules/ip/control/route.c) and packets are handed over in batches per
queue (one queue per RX queue / worker, modules/infra/control/worker.c).
Every call goes to libgrout_hip.so; there is no CPU fallback.
"""
import ctypes

import numpy as np

from . import abi
from .abi import check, ptr


class FastPath:
    def __init__(self, dev=0, max_ifaces=1024, max_nexthops=1 << 17):
        self.lib = abi.hip()
        h = ctypes.c_void_p()
        check("gr_hip_init", self.lib.gr_hip_init(dev, max_ifaces, max_nexthops, ctypes.byref(h)))
        self.h = h
        self.max_ifaces = max_ifaces
        self.max_nexthops = max_nexthops
        self.queues = []

    @classmethod
    def borrow(cls, handle, max_ifaces=1024, max_nexthops=1 << 17):
        """Wrap a context created elsewhere (e.g. by the grout node's module,
        gpu_fwd4_hip_ctx()) without owning it: close() leaves it alive."""
        self = cls.__new__(cls)
        self.lib = abi.hip()
        self.h = ctypes.c_void_p(handle)
        self.max_ifaces = max_ifaces
        self.max_nexthops = max_nexthops
        self.queues = []
        self._borrowed = True
        return self

    def close(self):
        if self.h:
            for q in self.queues:
                q._h = None
            if not getattr(self, "_borrowed", False):
                self.lib.gr_hip_fini(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- objects -------------------------------------------------------------
    def set_ifaces(self, ifaces):
        a = np.ascontiguousarray(ifaces[ifaces["id"] != 0], dtype=abi.IFACE_DT)
        check("gr_hip_iface_set", self.lib.gr_hip_iface_set(self.h, ptr(a), len(a)))

    def del_iface(self, iface_id):
        check("gr_hip_iface_del", self.lib.gr_hip_iface_del(self.h, iface_id))

    def set_nexthops(self, nh, first=1):
        a = np.ascontiguousarray(nh, dtype=abi.NH_DT)
        check("gr_hip_nh_set", self.lib.gr_hip_nh_set(self.h, first, ptr(a), len(a)))

    def set_reta(self, reta, first=0):
        a = np.ascontiguousarray(reta, dtype=np.uint32)
        if len(a):
            check("gr_hip_reta_set", self.lib.gr_hip_reta_set(self.h, first, ptr(a), len(a)))

    def fib_create(self, vrf_id, max_routes=1 << 16, num_tbl8=0):
        check("gr_hip_fib4_create", self.lib.gr_hip_fib4_create(self.h, vrf_id, max_routes, num_tbl8))

    def fib_destroy(self, vrf_id):
        check("gr_hip_fib4_destroy", self.lib.gr_hip_fib4_destroy(self.h, vrf_id))

    def route_add(self, routes, replace=False):
        a = np.ascontiguousarray(routes, dtype=abi.ROUTE_DT)
        check("gr_hip_route4_add", self.lib.gr_hip_route4_add(self.h, ptr(a), len(a), 1 if replace else 0))

    def route_del(self, vrf_id, ip_host, prefixlen):
        be = int.from_bytes(int(ip_host).to_bytes(4, "big"), "little")
        check("gr_hip_route4_del", self.lib.gr_hip_route4_del(self.h, vrf_id, be, prefixlen))

    def fib_commit(self, vrf_id):
        check("gr_hip_fib4_commit", self.lib.gr_hip_fib4_commit(self.h, vrf_id))

    def fib6_create(self, vrf_id, max_routes=1 << 16, num_groups=0):
        check("gr_hip_fib6_create", self.lib.gr_hip_fib6_create(self.h, vrf_id, max_routes, num_groups))

    def fib6_destroy(self, vrf_id):
        check("gr_hip_fib6_destroy", self.lib.gr_hip_fib6_destroy(self.h, vrf_id))

    def route6_add(self, routes, replace=False):
        a = np.ascontiguousarray(routes, dtype=abi.ROUTE6_DT)
        check("gr_hip_route6_add", self.lib.gr_hip_route6_add(self.h, ptr(a), len(a), 1 if replace else 0))

    def route6_del(self, vrf_id, ip16, prefixlen, iface_id=0):
        a = np.frombuffer(bytes(ip16), np.uint8).copy()
        check("gr_hip_route6_del", self.lib.gr_hip_route6_del(self.h, vrf_id, iface_id, ptr(a), prefixlen))

    def fib6_commit(self, vrf_id):
        check("gr_hip_fib6_commit", self.lib.gr_hip_fib6_commit(self.h, vrf_id))

    def fib6_lookup(self, vrf_id, ip16, iface_id=0):
        out = ctypes.c_uint32()
        a = np.frombuffer(bytes(ip16), np.uint8).copy()
        check("gr_hip_fib6_lookup_host", self.lib.gr_hip_fib6_lookup_host(self.h, vrf_id, iface_id, ptr(a),
                                                                          ctypes.byref(out)))
        return out.value

    def fib6_info(self, vrf_id):
        n, u, b = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint64()
        check("gr_hip_fib6_info", self.lib.gr_hip_fib6_info(self.h, vrf_id, ctypes.byref(n), ctypes.byref(u),
                                                            ctypes.byref(b)))
        return dict(routes=n.value, groups_used=u.value, dev_bytes=b.value)

    def fib_lookup(self, vrf_id, ip_host):
        out = ctypes.c_uint32()
        be = int.from_bytes(ip_host.to_bytes(4, "big"), "little")
        check("gr_hip_fib4_lookup_host", self.lib.gr_hip_fib4_lookup_host(self.h, vrf_id, be, ctypes.byref(out)))
        return out.value

    def fib_info(self, vrf_id):
        n, u, b = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint64()
        check("gr_hip_fib4_info", self.lib.gr_hip_fib4_info(self.h, vrf_id, ctypes.byref(n), ctypes.byref(u), ctypes.byref(b)))
        return dict(routes=n.value, tbl8_used=u.value, dev_bytes=b.value)

    def tune(self, key, value=0):
        return check("gr_hip_tune", self.lib.gr_hip_tune(self.h, key.encode(), value))

    def load(self, topo):
        """Push a grout_amd.topology.Topology (ifaces, nexthops, reta, FIBs)."""
        self.set_ifaces(topo.ifaces)
        if topo.n_nh:
            self.set_nexthops(topo.nh[1:topo.n_nh + 1], first=1)
        self.set_reta(topo.reta)
        routes = topo.route_array()
        for vrf_id, (max_routes, num_tbl8) in topo.fibs.items():
            self.fib_create(vrf_id, max_routes, num_tbl8)
        if len(routes):
            self.route_add(routes)
        for vrf_id in topo.fibs:
            self.fib_commit(vrf_id)
        routes6 = topo.route6_array()
        for vrf_id, (max_routes, num_groups) in topo.fibs6.items():
            self.fib6_create(vrf_id, max_routes, num_groups)
        if len(routes6):
            self.route6_add(routes6)
        for vrf_id in topo.fibs6:
            self.fib6_commit(vrf_id)

    def batch_alloc(self, n, in_stride=64):
        """Zeroed device buffers of an n-packet batch (gr_hip_batch_alloc); -> abi.Batch."""
        b = abi.Batch()
        check("gr_hip_batch_alloc", self.lib.gr_hip_batch_alloc(self.h, n, in_stride, ctypes.byref(b)))
        return b

    def batch_place(self, b, candidates=6):
        """gr_hip_batch_place: re-place b's output lines by timing candidates."""
        check("gr_hip_batch_place", self.lib.gr_hip_batch_place(self.h, ctypes.byref(b), candidates))

    def batch_free(self, b):
        check("gr_hip_batch_free", self.lib.gr_hip_batch_free(self.h, ctypes.byref(b)))

    def queue(self, stream=None):
        q = Queue(self, stream)
        self.queues.append(q)
        return q


def shared_stream(device):
    """A created torch stream, made torch's current one on `device`, for a
    queue that shares the stream with torch work (copies, reductions). The
    null stream cannot be shared: gr_hip_queue_create(NULL) makes a private
    non-blocking stream that does not order against it."""
    import torch
    s = torch.cuda.Stream(device)
    torch.cuda.set_stream(s)
    return s.cuda_stream


class Queue:
    def __init__(self, fp, stream=None):
        self.fp = fp
        self.lib = fp.lib
        if stream is not None and int(stream) == 0:
            raise ValueError("the null stream cannot be shared with a queue (NULL = private stream); "
                             "pass grout_amd.fwd.shared_stream(device)")
        h = ctypes.c_void_p()
        check("gr_hip_queue_create", self.lib.gr_hip_queue_create(fp.h, stream, ctypes.byref(h)))
        self._h = h
        self._walks = []  # mbuf arrays of the node walks in flight (node_start .. node_finish)

    @property
    def stream(self):
        return self.lib.gr_hip_queue_stream(self._h)

    def submit(self, in_frames, out_lines, meta, verdicts, n, in_stride=64, out_stride=64, lines_only=False,
               prefix32=False):
        """Enqueue the fused kernel on device buffers (torch tensors / pointers).
        prefix32: out_lines gets packed 32-byte prefixes (GR_HIP_BATCH_F_PREFIX32)."""
        flags = (abi.BATCH_F_LINES_ONLY if lines_only else 0) | (abi.BATCH_F_PREFIX32 if prefix32 else 0)
        b = abi.Batch(ptr(in_frames), ptr(out_lines), ptr(meta), ptr(verdicts), n, in_stride,
                      abi.PREFIX if prefix32 else out_stride, flags)
        check("gr_hip_fwd4_submit", self.lib.gr_hip_fwd4_submit(self._h, ctypes.byref(b)))

    def sync(self):
        check("gr_hip_queue_sync", self.lib.gr_hip_queue_sync(self._h))

    def kernel_ms(self, n):
        ms, cnt = ctypes.c_float(), ctypes.c_uint32()
        check("gr_hip_queue_kernel_ms", self.lib.gr_hip_queue_kernel_ms(self._h, n, ctypes.byref(ms), ctypes.byref(cnt)))
        return ms.value, cnt.value

    def forward_host(self, lines, meta, out_lines=None, verdicts=None):
        """Host-memory path: header lines + metadata in host memory."""
        n = len(meta)
        lines = np.ascontiguousarray(lines)
        meta = np.ascontiguousarray(meta, dtype=abi.META_DT)
        if out_lines is None:
            out_lines = np.empty((n, abi.LINE), dtype=np.uint8)
        if verdicts is None:
            verdicts = np.empty(n, dtype=abi.VERDICT_DT)
        check("gr_hip_fwd4_host", self.lib.gr_hip_fwd4_host(self._h, ptr(lines), ptr(meta), n, ptr(out_lines), ptr(verdicts)))
        return out_lines, verdicts

    def node_process(self, mbufs, burst=64):
        """The rte_graph node's walk over host mbuf views (abi.MBUF_DT, frame
        pointers into host memory): stage, forward, hand back in place.
        Returns the per-node counters of this call (abi.NODE_STATS_DT)."""
        assert mbufs.dtype == abi.MBUF_DT and mbufs.flags["C_CONTIGUOUS"]
        ns = np.zeros(1, dtype=abi.NODE_STATS_DT)
        r = check("gr_hip_node_process", self.lib.gr_hip_node_process(self._h, ptr(mbufs), len(mbufs), burst,
                                                                     ptr(ns)))
        self.unfinished = r  # mbufs handed back as PUNT because a kernel gave up
        return ns[0]

    def node_start(self, mbufs, burst=64):
        """First half of node_process: stage and enqueue without waiting.
        The mbufs belong to the queue until the matching node_finish()."""
        assert mbufs.dtype == abi.MBUF_DT and mbufs.flags["C_CONTIGUOUS"]
        check("gr_hip_node_start", self.lib.gr_hip_node_start(self._h, ptr(mbufs), len(mbufs), burst))
        self._walks.append(mbufs)  # keeps the views alive while the GPU works on them

    def node_finish(self):
        """Wait for the oldest started walk and hand it back; returns (the
        mbuf array it was started with, per-node counters)."""
        ns = np.zeros(1, dtype=abi.NODE_STATS_DT)
        pm, pn = ctypes.c_void_p(), ctypes.c_uint32()
        r = check("gr_hip_node_finish", self.lib.gr_hip_node_finish(self._h, ctypes.byref(pm), ctypes.byref(pn),
                                                                   ptr(ns)))
        m = self._walks.pop(0)
        assert pn.value == len(m) and (len(m) == 0 or pm.value == m.ctypes.data)
        self.unfinished = r
        return m, ns[0]

    def node_pending(self):
        """(walks in flight, whether the oldest one's GPU work is done)."""
        ready = ctypes.c_int()
        n = check("gr_hip_node_pending", self.lib.gr_hip_node_pending(self._h, ctypes.byref(ready)))
        return n, bool(ready.value)

    def stats(self, reset=False):
        """Per-iface counters the queue's kernels accumulated on the device."""
        st = np.zeros(self.fp.max_ifaces, dtype=abi.STATS_DT)
        check("gr_hip_queue_stats", self.lib.gr_hip_queue_stats(self._h, ptr(st), len(st), 1 if reset else 0))
        return st

    def stats_shards(self, w, reset=False):
        """The same counters per shard, (64, w) of abi.STATS_DT: workgroup b of
        a launch counts into shard b % 64 (gr_hip_queue_stats_shards)."""
        st = np.zeros(64 * w, dtype=abi.STATS_DT)
        check("gr_hip_queue_stats_shards", self.lib.gr_hip_queue_stats_shards(self._h, ptr(st), w, 1 if reset else 0))
        return st.reshape(64, w)

    def node_iface_stats(self, reset=False):
        """Per-iface counters of the node walks (the kernels' counts, or the
        hand-back's with "stats" off; what the grout node folds into grout's
        iface_stats)."""
        st = np.zeros(self.fp.max_ifaces, dtype=abi.STATS_DT)
        check("gr_hip_node_iface_stats", self.lib.gr_hip_node_iface_stats(self._h, ptr(st), len(st),
                                                                         1 if reset else 0))
        return st

    def close(self):
        if self._h:
            self.lib.gr_hip_queue_destroy(self._h)
            self._h = None
