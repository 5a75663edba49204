"""Is the bench's run-to-run spread buffer placement or box state?

One process, one FIB, one host stream; SETS fresh device allocations of the
batch (input lines, metadata, output lines, verdicts), all kept alive so each
gets its own physical pages. Passes go round-robin over the sets, timing
STEPS launches per set with the queue's HIP events. If the kernel time
follows the set across passes, placement matters; if it follows the pass
(time), it is the box's clock state.

    python tools/placement_probe.py [--sets 8] [--passes 3] [--steps 50]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=8)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--workload", default="fullview64", choices=["fullview64", "single64"])
    ap.add_argument("--orders", default="0", help="tile_order values to time per set, e.g. 0,1")
    ap.add_argument("--fib-reloads", type=int, default=0, help="also re-create the FIB this many times (pass 0 set)")
    a = ap.parse_args()
    import torch
    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath, shared_stream

    dev = torch.device("cuda", 0)
    fp = FastPath(0)
    n = a.batch
    if a.workload == "single64":
        topo = T.config_single_route()
        frames, meta = S.stream(n, 0x67721000, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    else:
        topo = T.config_fullview()
        frames, meta = S.stream(n, 0x67721000, routes=topo.route_array())
    fp.load(topo)
    sets = []
    for _ in range(a.sets):
        d_in = torch.from_numpy(frames.reshape(-1)).to(dev)
        d_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
        d_out = torch.empty(n * abi.LINE, dtype=torch.uint8, device=dev)
        d_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
        sets.append((d_in, d_meta, d_out, d_v))
    torch.cuda.synchronize()
    q = fp.queue(shared_stream(dev))

    def run(s, steps):
        d_in, d_meta, d_out, d_v = sets[s]
        for _ in range(steps):
            q.submit(d_in, d_out, d_meta, d_v, n, in_stride=abi.LINE, out_stride=abi.LINE)
        torch.cuda.synchronize()
        ms, cnt = q.kernel_ms(steps)
        return ms / max(cnt, 1)

    for s in range(a.sets):
        run(s, 5)
    orders = [int(x) for x in a.orders.split(",")]
    res_o = np.zeros((a.passes, a.sets, len(orders)))
    t0 = time.time()
    for p in range(a.passes):
        for s in range(a.sets):
            for oi, o in enumerate(orders):
                fp.tune("tile_order", o)
                res_o[p, s, oi] = run(s, a.steps)
                print(json.dumps({"pass": p, "set": s, "tile_order": o, "kernel_ms": round(res_o[p, s, oi], 4),
                                  "t": round(time.time() - t0, 2)}), flush=True)
    fp.tune("tile_order", orders[0])
    res = res_o[:, :, 0]
    # which buffer carries it: every mix of the fastest and slowest set's four buffers
    by_set = res.mean(axis=0)
    fast, slow = int(by_set.argmin()), int(by_set.argmax())
    roles = ["in", "meta", "out", "v"]
    mix = []
    for code in range(16):
        pick = [slow if code >> r & 1 else fast for r in range(4)]
        d_in, d_meta, d_out, d_v = (sets[pick[r]][r] for r in range(4))
        for _ in range(3):
            q.submit(d_in, d_out, d_meta, d_v, n, in_stride=abi.LINE, out_stride=abi.LINE)
        for _ in range(a.steps):
            q.submit(d_in, d_out, d_meta, d_v, n, in_stride=abi.LINE, out_stride=abi.LINE)
        torch.cuda.synchronize()
        ms, cnt = q.kernel_ms(a.steps)
        mix.append({"slow_set_for": [roles[r] for r in range(4) if code >> r & 1], "kernel_ms": round(ms / cnt, 4)})
        print(json.dumps(mix[-1]), flush=True)
    print(json.dumps({"addrs": [[hex(t.data_ptr()) for t in st] for st in sets]}), flush=True)
    fib = []
    for r in range(a.fib_reloads):
        fp.fib_destroy(T.VRF_MAIN)
        fp.fib6_destroy(T.VRF_MAIN)
        fp.load(topo)
        fib.append(round(run(0, a.steps), 4))
        print(json.dumps({"fib_reload": r, "set": 0, "kernel_ms": fib[-1]}), flush=True)
    by_pass = res.mean(axis=1)
    print(json.dumps({"summary": True, "sets": a.sets, "passes": a.passes, "steps": a.steps,
                      "set_mean_ms": [round(x, 4) for x in by_set], "pass_mean_ms": [round(x, 4) for x in by_pass],
                      "spread_across_sets": round(float(by_set.max() - by_set.min()), 4),
                      "spread_across_passes": round(float(by_pass.max() - by_pass.min()), 4),
                      "within_set_std": round(float(res.std(axis=0).mean()), 4), "fib_reload_ms": fib,
                      "by_order": {o: {"set_mean_ms": [round(x, 4) for x in res_o[:, :, oi].mean(axis=0)],
                                       "mean": round(float(res_o[:, :, oi].mean()), 4)}
                                   for oi, o in enumerate(orders)}}))
    fp.close()


if __name__ == "__main__":
    main()
