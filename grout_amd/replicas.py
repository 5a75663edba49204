# SPDX-License-Identifier: BSD-3-Clause
"""One process per GPU, replicas only.

grout shards by RX queue (modules/infra/control/worker.c:424-481): packets are
independent, so every GPU owns its own RX stream and a full FIB replica and
no data crosses GPUs. torch.distributed over gloo (host memory, CPU) is used
only for the start/stop barrier, the max-over-ranks clock and the per-rank
report of the benchmark, never on the data path: there is no exchange step, so
no RCCL communicator is created.

Two ways in: under a launcher (torch.distributed.run sets WORLD_SIZE, RANK,
LOCAL_RANK, MASTER_*), or `spawn()`: the parent starts one fresh child process
per GPU before it makes any GPU call, the way grout's main process starts one
worker thread per lcore (worker.c:59-66), and exits with their status.
"""
import os
import signal
import socket
import subprocess
import sys
import time

from . import synth


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn(n, argv, env=None, poll_s=0.05):
    """Run `python argv...` as n ranks (RANK = LOCAL_RANK = 0..n-1,
    WORLD_SIZE = n, rendezvous on 127.0.0.1) and return the job's exit status:
    0 when every rank exited 0, else the first failing rank's status (a signal
    as 128 + signo). A failing rank takes the others down: the rest would wait
    forever at the next barrier. Must be called before this process touches a
    GPU: the children initialise their own device."""
    if n < 1:
        raise ValueError("spawn: n >= 1")
    base = dict(os.environ if env is None else env)
    base.update(WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                MASTER_PORT=str(free_port()))
    procs = []

    def stop(signo, _frame):  # a limit on the parent ends the ranks too
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        raise SystemExit(128 + signo)

    old = {s: signal.signal(s, stop) for s in (signal.SIGTERM, signal.SIGINT)}
    try:
        for r in range(n):
            e = dict(base, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
            procs.append(subprocess.Popen([sys.executable] + list(argv), env=e))
        status = 0
        live = set(range(n))
        while live:
            for r in sorted(live):
                rc = procs[r].poll()
                if rc is None:
                    continue
                live.discard(r)
                if rc != 0 and status == 0:
                    status = 128 - rc if rc < 0 else rc
                    for o in live:  # the others would block at the next barrier
                        procs[o].send_signal(signal.SIGTERM)
            if live:
                time.sleep(poll_s)
        return status
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for s, h in old.items():
            signal.signal(s, h)


class Replicas:
    def __init__(self, backend="gloo"):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        self.backend = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # gloo announces its connections on fd 1, where rank 0's JSON
            # line goes: stdout points at stderr for the rendezvous
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group(backend, rank=self.rank, world_size=self.world)
            finally:
                os.dup2(saved, 1)
                os.close(saved)
            self.dist = dist
            self.backend = backend

    def seed(self, base=synth.SEED_GPU_BASE):
        """RX stream seed of this replica: 0x67721000 + g."""
        return base + self.rank

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max_over_ranks(self, x):
        """Max of a float over the ranks (the slowest replica sets the clock)."""
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather_objects(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def aggregate_mpps(self, pkts_per_rank_per_step, steps, seconds_max):
        """Whole-job rate: all ranks' packets over the slowest rank's time."""
        return self.world * pkts_per_rank_per_step * steps / seconds_max / 1e6

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()
            self.dist = None


def numa_cpus(node):
    """The CPUs of NUMA node `node` this process may use (empty if unknown)."""
    try:
        spec = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
    except OSError:
        return set()
    cpus = set()
    for part in spec.split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return cpus & set(os.sched_getaffinity(0))


def bind_to_numa(node):
    """Pin this rank's threads to its GPU's NUMA node (grout puts the workers
    of a port on the port's socket, worker.c:424-481). Returns the node the
    rank now runs on, or None when the node is unknown or has no usable CPU."""
    if node is None or node < 0:
        return None
    cpus = numa_cpus(node)
    if not cpus:
        return None
    os.sched_setaffinity(0, cpus)
    return node


def cpu_numa_node():
    """NUMA node of the CPU this thread runs on now (None if unreadable)."""
    try:
        cpu = int(open("/proc/self/stat").read().rsplit(")", 1)[1].split()[36])
    except (OSError, ValueError, IndexError):
        return None
    base = f"/sys/devices/system/cpu/cpu{cpu}"
    try:
        for name in os.listdir(base):
            if name.startswith("node") and name[4:].isdigit():
                return int(name[4:])
    except OSError:
        pass
    return None
