# SPDX-License-Identifier: BSD-3-Clause
"""Helpers shared by the golden and GPU parity tests."""
import functools
import os

import numpy as np

import scenarios as SC
from grout_amd import abi
from grout_amd import topology as T

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


@functools.lru_cache(maxsize=None)
def _fullview():
    return T.config_fullview()


@functools.lru_cache(maxsize=None)
def _fullview6():
    return T.config_fullview6()


def topo_for(name):
    if name in ("corpus", "eth_cache"):
        return SC.corpus_topology()[0]
    if name == "single":
        return T.config_single_route()
    if name == "fullview6":
        return _fullview6()
    return _fullview()


_loaded = {}


def fresh_fastpath_state(fp, topo, state=None):
    """(Re)load topo into the shared FastPath (or into `fp` with its own
    `state` dict): clear the old objects first."""
    st = _loaded if state is None else state
    key = id(topo)
    if st.get("key") == key:
        return
    st.pop("topo", None)
    st.pop("key", None)
    # wipe previous state: FIBs, ifaces, nexthops (popped first, so that one
    # failure does not cascade into every later test)
    for vrf in st.pop("fibs", []):
        fp.fib_destroy(vrf)
    for vrf in st.pop("fibs6", []):
        fp.fib6_destroy(vrf)
    for i in st.pop("ifaces", []):
        fp.del_iface(int(i))
    fp.set_nexthops(np.zeros(fp.max_nexthops, dtype=abi.NH_DT), first=1)
    fp.load(topo)
    st.update(key=key, fibs=list(topo.fibs), fibs6=list(topo.fibs6), ifaces=list(topo.live_ifaces()["id"]),
                   topo=topo)


def run_gpu(fp, topo, frames, meta, lines_only=False, inplace=False, q=None):
    """Device-resident path through the C ABI; returns (lines, verdicts, stats)."""
    import torch
    fresh_fastpath_state(fp, topo)
    dev = torch.device("cuda")
    if q is None:
        if "q" not in _loaded:
            from grout_amd.fwd import shared_stream
            _loaded["q"] = fp.queue(shared_stream(dev))
        q = _loaded["q"]
    n = len(meta)
    stride = frames.shape[1]
    fin = torch.from_numpy(np.ascontiguousarray(frames).reshape(-1)).to(dev)
    me = torch.from_numpy(np.ascontiguousarray(meta).view(np.uint8)).to(dev)
    out = fin if inplace else torch.zeros(n * abi.LINE, dtype=torch.uint8, device=dev)
    v = torch.zeros(n * 8, dtype=torch.uint8, device=dev)
    q.stats(reset=True)
    q.submit(fin, out, me, v, n, in_stride=stride, out_stride=stride if inplace else abi.LINE,
             lines_only=lines_only)
    q.sync()
    lines = out.cpu().numpy().reshape(n, -1)[:, :abi.LINE].copy()
    verdicts = v.cpu().numpy().view(abi.VERDICT_DT).copy()
    st = q.stats(reset=True)
    return lines, verdicts, st
