# SPDX-License-Identifier: BSD-3-Clause
"""The multi-GPU path (replicas) on CPU with gloo, world size 2.

Each rank builds its FIB replica and its own RX stream (seed 0x67721000 +
rank), forwards it through the oracle as the CPU stand-in for its GPU, and
the job is aggregated exactly as bench.py does: barrier, max-over-ranks
clock, whole-job rate. No collective touches packet data."""
import os
import socket
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import oracle
    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.replicas import Replicas

    rep = Replicas("gloo")
    topo = T.config_single_route()
    frames, meta = S.stream(4096, rep.seed(), dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    o = oracle.Oracle(topo)
    rep.barrier()
    t0 = time.perf_counter()
    lines, v, st = o.process(frames, meta)
    if rank == 1:
        time.sleep(0.05)  # the slow replica must set the job's clock
    rep.barrier()
    el = time.perf_counter() - t0
    tmax = rep.max_over_ranks(el)
    digests = rep.gather_objects(int(np.frombuffer(lines.tobytes(), np.uint64).sum() % (1 << 61)))
    mpps = rep.aggregate_mpps(len(meta), 1, tmax)
    out.put(dict(rank=rank, seed=rep.seed(), el=el, tmax=tmax, digests=digests, mpps=mpps,
                 fwd=int((v["edge"] == abi.EDGE["port_output"]).sum()), n=len(meta)))
    rep.close()


def test_two_replicas_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda d: d["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r["seed"] for r in res] == [0x67721000, 0x67721001]
    assert res[0]["tmax"] == res[1]["tmax"] >= max(r["el"] for r in res) - 1e-9
    assert res[1]["el"] >= 0.05
    # independent streams: different packets, every packet forwarded on each
    assert res[0]["digests"][0] != res[0]["digests"][1]
    assert all(r["fwd"] == r["n"] for r in res)
    # whole-job rate = all ranks' packets over the slowest clock
    assert abs(res[0]["mpps"] - 2 * 4096 / res[0]["tmax"] / 1e6) < 1e-9


@pytest.mark.gpu
def test_bench_two_ranks_on_the_gpu():
    """The driver's N>1 command, on the box's one GPU: torch.distributed.run
    starts two bench.py ranks, each forwards its own stream on its own FIB
    replica through libgrout_hip.so (GR_BENCH_SHARE_GPU=1: both on device 0,
    gloo for the barrier and the clock, since RCCL refuses two ranks on one
    GPU), and rank 0 alone prints the whole-job line."""
    import json
    import subprocess
    import sys
    env = dict(os.environ, GR_BENCH_SHARE_GPU="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "4", "--warmup", "2", "--workload", "single64", "--batch", str(1 << 20), "--placement", "plain",
           "--settle-ms", "5", "--no-plain", "--no-prefix-leg", "--no-cpu-baseline", "--no-host-path"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 4 and d["warmup"] == 2 and d["scaling"] == "weak"
    assert d["config"]["batch_pkts_per_gpu"] == 1 << 20
    assert d["config"]["forwarded_frac"] == 1.0  # every packet of rank 0's stream left by port_output
    # whole-job rate: both ranks' packets over the slowest rank's clock
    assert abs(d["value"] - 2 * (1 << 20) * 4 / (d["ms_per_step"] * 4 / 1e3) / 1e6) < 0.01 * d["value"]
