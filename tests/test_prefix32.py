# SPDX-License-Identifier: BSD-3-Clause
"""GR_HIP_BATCH_F_PREFIX32: the output is each packet's first 32 bytes, packed.

It rests on one property of grout's chain: no node on the path writes past
byte 31 of the frame. eth_output writes bytes 0-13 (eth_output.c:49-60),
ip_forward the TTL (22) and checksum (24-25) (ip_forward.c:29-32),
ip6_forward the hop limit (21), iface_output only mbuf fields
(iface_output.c:81-86). The CPU test checks that property on the oracle over
every committed fixture; the GPU tests check the packed prefixes against the
oracle's lines."""
import numpy as np
import pytest

import oracle
import scenarios as SC
from golden_util import fresh_fastpath_state, load, run_gpu, topo_for
from grout_amd import abi
from grout_amd import synth as S
from grout_amd import topology as T


@pytest.mark.parametrize("name", ["corpus", "eth_cache", "single", "fullview", "fullview6", "imix"])
def test_path_never_writes_past_byte_31(name):
    g = load(name)
    fr, out = g["frames"], g["out"]
    assert np.array_equal(out[:, 32:64], fr[:, 32:64]), name
    # ...while the first 32 bytes do change for forwarded packets
    fwd = g["verdicts"]["edge"] == abi.EDGE["port_output"]
    if fwd.any():
        assert (out[fwd, :32] != fr[fwd, :32]).any(axis=1).all(), name


def _run_prefix(fp, topo, frames, meta, placed=False):
    import torch
    fresh_fastpath_state(fp, topo)
    dev = torch.device("cuda")
    n = len(meta)
    fin = torch.from_numpy(np.ascontiguousarray(frames).reshape(-1)).to(dev)
    me = torch.from_numpy(np.ascontiguousarray(meta).view(np.uint8)).to(dev)
    out = torch.zeros(n * abi.PREFIX, dtype=torch.uint8, device=dev)
    v = torch.zeros(n * 8, dtype=torch.uint8, device=dev)
    q = fp.queue()
    q.stats(reset=True)
    q.submit(fin, out, me, v, n, in_stride=frames.shape[1], prefix32=True)
    q.sync()
    st = q.stats(reset=True)
    q.close()
    return out.cpu().numpy().reshape(n, abi.PREFIX), v.cpu().numpy().view(abi.VERDICT_DT), st


@pytest.mark.gpu
def test_prefix32_corpus(fastpath):
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    o_lines, o_v, o_st = oracle.Oracle(t).process(fr, me)
    p, v, st = _run_prefix(fastpath, t, fr, me)
    bad = np.nonzero(o_v != v)[0]
    assert len(bad) == 0, [(lab[i], o_v[i], v[i]) for i in bad[:6]]
    badl = np.nonzero((o_lines[:, :32] != p).any(axis=1))[0]
    assert len(badl) == 0, [lab[i] for i in badl[:6]]
    assert np.array_equal(o_st, st)


@pytest.mark.gpu
def test_prefix32_fullview_ragged(fastpath):
    """Full view, a ragged size, and the packed prefixes against whole lines
    of the same launch."""
    tf = topo_for("fullview")
    n = (1 << 20) + 37
    fr, me = S.stream(n, 0x32F1, routes=tf.route_array())
    o = oracle.Oracle(tf).process(fr, me)
    p, v, st = _run_prefix(fastpath, tf, fr, me)
    assert np.array_equal(o[1], v)
    assert np.array_equal(o[0][:, :32], p)
    assert np.array_equal(o[2], st)
    lines, v2, _ = run_gpu(fastpath, tf, fr, me)
    assert np.array_equal(lines[:, :32], p) and np.array_equal(v2, v)


@pytest.mark.gpu
def test_prefix32_batch_place(fastpath):
    """gr_hip_batch_place with packed prefixes: candidates sized n x 32."""
    import ctypes
    tf = topo_for("fullview")
    fresh_fastpath_state(fastpath, tf)
    n = 1 << 18
    fr, me = S.stream(n, 0x32F2, routes=tf.route_array())
    b = fastpath.batch_alloc(n)
    L = fastpath.lib
    abi.check("h2d", L.gr_hip_memcpy_h2d(fastpath.h, b.in_frames, fr.ctypes.data, fr.nbytes))
    abi.check("h2d", L.gr_hip_memcpy_h2d(fastpath.h, b.meta, me.ctypes.data, me.nbytes))
    try:
        b.flags = abi.BATCH_F_PREFIX32
        b.out_stride = abi.PREFIX
        fastpath.batch_place(b, 3)
        q = fastpath.queue()
        abi.check("submit", L.gr_hip_fwd4_submit(q._h, ctypes.byref(b)))
        q.sync()
        q.close()
        p = np.empty((n, abi.PREFIX), dtype=np.uint8)
        v = np.empty(n, dtype=abi.VERDICT_DT)
        abi.check("d2h", L.gr_hip_memcpy_d2h(fastpath.h, p.ctypes.data, b.out_lines, p.nbytes))
        abi.check("d2h", L.gr_hip_memcpy_d2h(fastpath.h, v.ctypes.data, b.verdicts, v.nbytes))
        o = oracle.Oracle(tf).process(fr, me)
        assert np.array_equal(o[1], v)
        assert np.array_equal(o[0][:, :32], p)
    finally:
        fastpath.batch_free(b)


@pytest.mark.gpu
def test_prefix32_rejects_bad_batches(fastpath):
    """The flag needs out_lines with stride 32: a whole-line stride or
    in-place rewrite (no out_lines) is refused before any launch."""
    import ctypes
    import torch
    dev = torch.device("cuda")
    buf = torch.zeros(1 << 16, dtype=torch.uint8, device=dev)
    p = buf.data_ptr()
    q = fastpath.queue()
    try:
        for out, stride in ((p, 64), (0, 32), (p + 8, 32)):
            b = abi.Batch(p, out, p, p, 64, 64, stride, abi.BATCH_F_PREFIX32)
            assert fastpath.lib.gr_hip_fwd4_submit(q._h, ctypes.byref(b)) == -22, (out - p if out else 0, stride)
    finally:
        q.close()


@pytest.mark.gpu
def test_prefix32_host_path(fastpath):
    """gr_hip_fwd4_host_ex with 32-byte prefixes back, on pinned host memory
    (the kernel's own PCIe loads and stores) and on pageable memory (staged
    chunk copies): the same prefixes and verdicts as the oracle."""
    import torch
    tf = topo_for("fullview")
    fresh_fastpath_state(fastpath, tf)
    n = (1 << 19) + 5  # two chunks of the staged path and a ragged end
    fr, me = S.stream(n, 0x32F3, routes=tf.route_array())
    o = oracle.Oracle(tf).process(fr, me, lines_only=True)
    q = fastpath.queue()
    try:
        for pinned in (True, False):
            mk = (lambda a: torch.from_numpy(a).pin_memory()) if pinned else torch.from_numpy
            h_in, h_me = mk(np.ascontiguousarray(fr)), mk(me.view(np.uint8).copy())
            h_out = mk(np.zeros(n * abi.PREFIX, dtype=np.uint8))
            h_v = mk(np.zeros(n * 8, dtype=np.uint8))
            abi.check("gr_hip_fwd4_host_ex", fastpath.lib.gr_hip_fwd4_host_ex(
                q._h, h_in.data_ptr(), h_me.data_ptr(), n, h_out.data_ptr(), abi.PREFIX, h_v.data_ptr()))
            assert np.array_equal(o[1], h_v.numpy().view(abi.VERDICT_DT)), pinned
            assert np.array_equal(o[0][:, :32], h_out.numpy().reshape(n, abi.PREFIX)), pinned
    finally:
        q.close()
