# SPDX-License-Identifier: BSD-3-Clause
"""One process per GPU, replicas only.

grout shards by RX queue (modules/infra/control/worker.c:424-481): packets are
independent, so every GPU owns its own RX stream and a full FIB replica and
no data crosses GPUs. torch.distributed (RCCL on GPUs, gloo on CPU tests) is
used only for the start/stop barrier and the max-over-ranks clock of the
benchmark, never on the data path.
"""
import os

from . import synth


class Replicas:
    def __init__(self, backend=None):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            kw = {}
            if backend == "nccl":
                kw["device_id"] = torch.device("cuda", self.local)
            dist.init_process_group(backend, rank=self.rank, world_size=self.world, **kw)
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
        dev = torch.device("cuda", self.local) if self.backend == "nccl" else torch.device("cpu")
        t = torch.tensor([x], dtype=torch.float64, device=dev)
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
