# SPDX-License-Identifier: BSD-3-Clause
"""Host-memory path rates (PCIe-inclusive): staged chunk copies vs the kernel
reading / writing pinned host memory directly (gr_hip_tune host_direct), on
the headline workload's header lines. One JSON line per mode and batch."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath

    topo = T.config_fullview()
    fp = FastPath(0)
    fp.load(topo)
    nmax = 1 << 23
    fr, me = S.stream(nmax, S.SEED_GPU_BASE, routes=topo.route_array())
    h_in = torch.from_numpy(fr.reshape(-1)).pin_memory()
    h_me = torch.from_numpy(me.view(np.uint8)).pin_memory()
    h_out = torch.empty(nmax * abi.LINE, dtype=torch.uint8).pin_memory()
    h_v = torch.empty(nmax * 8, dtype=torch.uint8).pin_memory()
    q = fp.queue()
    ref = None
    for n in (1 << 16, 1 << 20, nmax):
        for direct in (0, 1):
            fp.tune("host_direct", direct)
            fn = fp.lib.gr_hip_fwd4_host
            args = (q._h, h_in.data_ptr(), h_me.data_ptr(), n, h_out.data_ptr(), h_v.data_ptr())
            abi.check("gr_hip_fwd4_host", fn(*args))
            reps = max(3, (1 << 24) // n)
            t0 = time.perf_counter()
            for _ in range(reps):
                abi.check("gr_hip_fwd4_host", fn(*args))
            dt = (time.perf_counter() - t0) / reps
            if n == nmax:
                h = (int(h_out.view(torch.int64).sum()), int(h_v.view(torch.int64).sum()))
                ref = h if ref is None else ref
                assert h == ref, ("outputs differ between modes", h, ref)
            print(json.dumps({"batch": n, "host_direct": direct, "us": round(dt * 1e6, 1),
                              "mpps": round(n / dt / 1e6, 1),
                              "GBps_per_dir": round(n * (abi.LINE + 8) / dt / 1e9, 1)}), flush=True)
    # the rte_graph node's whole walk (gr_hip_node_process): stage the lines
    # from the mbufs on the CPU, forward, hand back onto the mbufs
    n = 1 << 21
    bufs = np.zeros((n, 256), dtype=np.uint8)  # mbuf data rooms (frame at offset 0)
    bufs[:, :64] = fr[:n]
    mb = np.zeros(n, dtype=abi.MBUF_DT)
    mb["frame"] = bufs.ctypes.data + np.arange(n, dtype=np.uint64) * 256
    mb["pkt_len"] = me["pkt_len"][:n]
    mb["data_len"] = me["pkt_len"][:n]
    mb["data_off"] = 128
    mb["rss"] = me["rss"][:n]
    mb["iface"] = me["iface"][:n]
    fp.tune("host_direct", 1)
    abi.check("gr_hip_host_register", fp.lib.gr_hip_host_register(fp.h, bufs.ctypes.data, bufs.nbytes))
    for mode in ("staged", "frame_ptrs"):
        fp.tune("node_ptrs", 1 if mode == "frame_ptrs" else 0)
        m = mb.copy()
        q.node_process(m)
        dt = []
        for _ in range(4):
            m[:] = mb
            bufs[:, :64] = fr[:n]
            t1 = time.perf_counter()
            q.node_process(m)
            dt.append(time.perf_counter() - t1)
        d = float(np.median(dt))
        print(json.dumps({"node_process_batch": n, "mode": mode, "us": round(d * 1e6, 1),
                          "mpps": round(n / d / 1e6, 1), "cpu_threads": 1}), flush=True)
    fp.tune("node_ptrs", 1)
    abi.check("gr_hip_host_unregister", fp.lib.gr_hip_host_unregister(fp.h, bufs.ctypes.data))
    fp.tune("host_direct", 1)
    q.close()
    fp.close()


if __name__ == "__main__":
    main()
