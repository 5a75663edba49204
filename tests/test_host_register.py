# SPDX-License-Identifier: BSD-3-Clause
"""Host memory registered with gr_hip_host_register, unregistered, and used
again (round 5's illegal-address fault).

What tools/hostreg_probe.py measured on the box: after hipHostUnregister the
runtime reports the range as unregistered at once (hipPointerGetAttributes,
hipHostGetDevicePointer), also when the allocator hands the same virtual
address out again; but a second context that had registered the same range
kept the first context's device address in its registry after the first
unregistered it. The library now counts registrations process-wide (the last
context out unregisters) and waits on the host for a context's queues before
a range is unmapped. These tests pin each step: which path gr_hip_fwd4_host_ex
takes ("host_path_last"), and parity with the oracle on each."""
import ctypes

import numpy as np
import pytest

import oracle
from golden_util import fresh_fastpath_state, topo_for
from grout_amd import abi
from grout_amd import synth as S

pytestmark = pytest.mark.gpu

DIRECT, STAGED, PAGEABLE = 0, 1, 2


class _Attr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def _runtime_registered(p):
    """hipPointerGetAttributes' view of host address p: True when pinned."""
    hip = ctypes.CDLL("libamdhip64.so")
    a = _Attr()
    if hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p)) != 0:
        hip.hipGetLastError()
        return False
    return a.type == 1


def _our_addr(fp, p):
    d = ctypes.c_uint64()
    r = fp.lib.gr_hip_host_dev_addr(fp.h, ctypes.c_void_p(p), ctypes.byref(d))
    return r if r < 0 else d.value


class _Bufs:
    """One numpy allocation holding a batch's lines, metadata, prefixes out
    and verdicts, each 4 KiB-aligned inside it."""

    def __init__(self, n):
        sizes = [n * abi.LINE, n * 8, n * abi.PREFIX, n * 8]
        offs, o = [], 0
        for sz in sizes:
            offs.append(o)
            o += (sz + 4095) & ~4095
        self.mem = np.zeros(o + 4096, np.uint8)
        base = (-self.mem.ctypes.data) & 4095
        self.base = self.mem.ctypes.data + base
        self.nbytes = o
        self.views = [self.mem[base + off:base + off + sz] for off, sz in zip(offs, sizes)]

    def run(self, fp, q, fr, me, o):
        n = len(me)
        lines, meta, out, v = self.views
        lines[:] = np.ascontiguousarray(fr).reshape(-1)
        meta[:] = me.view(np.uint8)
        out[:] = 0
        v[:] = 0
        abi.check("gr_hip_fwd4_host_ex", fp.lib.gr_hip_fwd4_host_ex(
            q._h, lines.ctypes.data, meta.ctypes.data, n, out.ctypes.data, abi.PREFIX, v.ctypes.data))
        assert np.array_equal(o[1], v.view(abi.VERDICT_DT))
        assert np.array_equal(o[0][:, :32], out.reshape(n, abi.PREFIX))
        return fp.tune("host_path_last")


def _case(fastpath, n=(1 << 16) + 7):
    tf = topo_for("fullview")
    fresh_fastpath_state(fastpath, tf)
    fr, me = S.stream(n, 0x4E6, routes=tf.route_array())
    return fr, me, oracle.Oracle(tf).process(fr, me, lines_only=True)


def test_register_unregister_reuse(fastpath):
    """Register, forward (the kernel reads and writes the buffers over PCIe),
    unregister, forward again from the same buffers (now pageable: the CPU
    copies them through the queue's pinned buffers), then free them, allocate
    anew at what is likely the same address and forward from that: the path
    each time as expected, every result the oracle's."""
    fr, me, o = _case(fastpath)
    L = fastpath.lib
    q = fastpath.queue()
    try:
        for sync_check in (0, 1):  # and once with every step waited for and checked
            fastpath.tune("sync_check", sync_check)
            b = _Bufs(len(me))
            assert b.run(fastpath, q, fr, me, o) == PAGEABLE
            abi.check("register", L.gr_hip_host_register(fastpath.h, ctypes.c_void_p(b.base), b.nbytes))
            assert _runtime_registered(b.base)
            assert b.run(fastpath, q, fr, me, o) == DIRECT
            abi.check("unregister", L.gr_hip_host_unregister(fastpath.h, ctypes.c_void_p(b.base)))
            assert not _runtime_registered(b.base)
            assert _our_addr(fastpath, b.base) == -2  # -ENOENT
            assert b.run(fastpath, q, fr, me, o) == PAGEABLE
            va = b.base
            del b
            b2 = _Bufs(len(me))  # the allocator may hand the same range back
            assert not _runtime_registered(b2.base), b2.base == va
            assert b2.run(fastpath, q, fr, me, o) == PAGEABLE
            del b2
    finally:
        fastpath.tune("sync_check", 0)
        q.close()


def test_registration_shared_by_two_contexts(fastpath):
    """Two contexts register one range; the first unregisters. The range stays
    registered for the second (the runtime still maps it, and the second's
    address for it is still the runtime's), the second still forwards from it
    directly; only the second's unregister unmaps it."""
    from grout_amd.fwd import FastPath
    fr, me, o = _case(fastpath, n=4096 + 3)
    tf = topo_for("fullview")
    other = FastPath(0)
    st = {}
    try:
        fresh_fastpath_state(other, tf, st)
        b = _Bufs(len(me))
        p = ctypes.c_void_p(b.base)
        abi.check("register A", fastpath.lib.gr_hip_host_register(fastpath.h, p, b.nbytes))
        abi.check("register B", other.lib.gr_hip_host_register(other.h, p, b.nbytes))
        dev_b = _our_addr(other, b.base)
        assert dev_b == _our_addr(fastpath, b.base) and dev_b > 0
        abi.check("unregister A", fastpath.lib.gr_hip_host_unregister(fastpath.h, p))
        assert _runtime_registered(b.base)  # B's reference keeps it
        assert _our_addr(other, b.base) == dev_b
        qb = other.queue()
        try:
            assert b.run(other, qb, fr, me, o) == DIRECT
        finally:
            qb.close()
        abi.check("unregister B", other.lib.gr_hip_host_unregister(other.h, p))
        assert not _runtime_registered(b.base)
        # registered by A, then context B destroyed with its own reference
        abi.check("register A", fastpath.lib.gr_hip_host_register(fastpath.h, p, b.nbytes))
        abi.check("register B", other.lib.gr_hip_host_register(other.h, p, b.nbytes))
    finally:
        other.close()
    assert _runtime_registered(b.base)  # A's reference
    abi.check("unregister A", fastpath.lib.gr_hip_host_unregister(fastpath.h, p))
    assert not _runtime_registered(b.base)
