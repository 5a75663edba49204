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


# A rank of the spawn path: what bench.py's ranks do around the GPU step
# (gloo barrier, own clock, max-over-ranks clock, per-rank report), with the
# oracle as the CPU stand-in for the rank's GPU; rank 0 prints the job's line.
_CHILD = """
import json, os, sys, time
sys.path.insert(0, {root!r})
import numpy as np
import oracle
from grout_amd import abi, replicas
from grout_amd import synth as S, topology as T
fail = int(os.environ.get("GR_TEST_FAIL_RANK", "-1"))
rep = replicas.Replicas("gloo")
if rep.rank == fail:
    sys.exit(3)
topo = T.config_single_route()
frames, meta = S.stream(2048, rep.seed(), dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
o = oracle.Oracle(topo)
rep.barrier()
t0 = time.perf_counter()
lines, v, st = o.process(frames, meta)
own = time.perf_counter() - t0
rep.barrier()
tmax = rep.max_over_ranks(time.perf_counter() - t0)
ranks = rep.gather_objects(dict(rank=rep.rank, local=rep.local, seed=rep.seed(), own=own,
                                fwd=int((v["edge"] == abi.EDGE["port_output"]).sum())))
if rep.rank == 0:
    print(json.dumps(dict(n_gpus=rep.world, value=rep.aggregate_mpps(len(meta), 1, tmax), ranks=ranks)), flush=True)
rep.close()
"""


def test_spawn_ranks_gloo(capfd):
    """replicas.spawn (bench.py --gpus N without a launcher): N fresh rank
    processes with RANK/LOCAL_RANK/WORLD_SIZE set, gloo rendezvous, one line
    from rank 0 carrying every rank's report, exit status 0."""
    import json
    import sys
    sys.path.insert(0, ROOT)
    from grout_amd import replicas
    rc = replicas.spawn(3, ["-c", _CHILD.format(root=ROOT)])
    out = capfd.readouterr().out
    assert rc == 0
    lines = [x for x in out.splitlines() if x.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), out  # gloo's chatter kept off stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 3
    assert [r["rank"] for r in d["ranks"]] == [0, 1, 2] and [r["local"] for r in d["ranks"]] == [0, 1, 2]
    assert [r["seed"] for r in d["ranks"]] == [0x67721000 + g for g in range(3)]
    assert all(r["fwd"] == 2048 for r in d["ranks"])


def test_spawn_failing_rank_ends_the_job(capfd):
    """A rank that fails takes the job down: the others (blocked at the
    rendezvous or a barrier) are terminated and its status is the job's."""
    import sys
    sys.path.insert(0, ROOT)
    from grout_amd import replicas
    env = dict(os.environ, GR_TEST_FAIL_RANK="1")
    t0 = time.time()
    rc = replicas.spawn(2, ["-c", _CHILD.format(root=ROOT)], env=env)
    assert rc == 3
    assert time.time() - t0 < 60
    assert not [x for x in capfd.readouterr().out.splitlines() if x.startswith("{")]


def test_bench_world_must_match_gpus():
    """Under a launcher, WORLD_SIZE != --gpus is refused before any GPU call."""
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "3"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 2 and "WORLD_SIZE=2 but --gpus 3" in r.stderr


def test_bench_spawns_its_ranks():
    """bench.py --gpus 2 with no launcher starts two ranks itself; here (no
    GPU) each rank reaches the device check after the gloo rendezvous and
    exits 2, which is the job's status."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 2, r.stderr[-2000:]
    # the first rank out takes the other down, which may not get to say so
    assert "rank 0 wants device 0" in r.stderr or "rank 1 wants device 1" in r.stderr


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


@pytest.mark.gpu
def test_bench_spawns_two_ranks_on_the_gpu():
    """The driver's N>1 command without a launcher: bench.py --gpus 2 starts
    both ranks itself on config 3 (full view); one line, n_gpus 2, both
    ranks' own rates and kernel times, and -- after the final barrier, rank
    0 alone -- the PCIe-inclusive host path and the CPU baseline (a short
    sample here), as on the driver's N>1 lines."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["GR_BENCH_SHARE_GPU"] = "1"
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--workload", "fullview64", "--batch", str(1 << 22),
           "--steps", "8", "--warmup", "2", "--settle-ms", "20", "--no-prefix-leg", "--cpu-seconds", "0.3",
           "--cpu-threads", "4"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]  # only the line on stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and [x["rank"] for x in d["ranks"]] == [0, 1]
    assert all(x["mpps"] > 0 and x["kernel_ms_avg"] > 0 and x["forwarded_frac"] > 0.999 for x in d["ranks"])
    assert "frac_plain" in d["roofline"]
    assert d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["cores"] == 4 and d["cpu_baseline"]["ranks_idle"] == 1
    assert d["host_path"]["mpps"] > 0
