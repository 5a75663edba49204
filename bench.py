# SPDX-License-Identifier: BSD-3-Clause
"""Headline benchmark: Mpps of IPv4 forwarding, 64 B packets, ~1M-route FIB,
device-resident, per MI355X (BASELINE.json `metric`, config 3).

A step is one pass of the fused forwarding kernel over one batch of
synthetic packets already resident in HBM (default 2^24 packets, 64-byte
slots): iface_input .. iface_output for every packet, header lines written
out of place so every step sees the same input. Multi-GPU runs are replicas
(one independent RX stream and FIB replica per GPU, no collective on the data
path; torch.distributed over gloo is used only for the barrier, the
max-over-ranks clock and the per-rank report), so scaling is weak.

    python bench.py [--gpus N] [--steps K] [--warmup W]

--gpus N > 1 without a launcher: this process starts N fresh rank processes
itself (grout_amd.replicas.spawn) before any GPU call and exits with their
status. Under torch.distributed.run, WORLD_SIZE must equal --gpus.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# algorithmic HBM bytes per packet: line in, metadata in, one
# FIB entry (2 or 4 bytes by device format), line out, verdict out
def host_cpus():
    """The CPUs the CPU baseline may use: the process's cpuset, and the
    cgroup's CPU-time quota (cgroup v2 cpu.max) when one is set: a box's 16
    cores are a share of a larger host, which is why the baseline varies by box."""
    out = {"allowed": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()}
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        out["quota_cpus"] = None if quota == "max" else round(int(quota) / int(period), 2)
    except (OSError, ValueError):
        out["quota_cpus"] = None
    return out


def cgroup_cpu_stat():
    """The cgroup's CPU accounting (cgroup v2 cpu.stat): with a CPU-time quota
    (cpu.max), `throttled_usec` grows when the process's threads together
    exceed it, which slows busy pinned workers whatever their CPUs."""
    try:
        return {k: int(v) for k, v in (l.split() for l in open("/sys/fs/cgroup/cpu.stat"))}
    except (OSError, ValueError):
        return {}


def _cpu_sysfs(cpu, leaf):
    try:
        return open(f"/sys/devices/system/cpu/cpu{cpu}/{leaf}").read().strip()
    except OSError:
        return None


def cpu_placement(n, policy="spread"):
    """CPUs for n pinned workers, or None (the i-th allowed CPU each).
    "spread": one hardware thread per physical core, the cores taken round
    robin over the L3 domains (a Zen CCD: 8 cores, one L3 and one link to
    memory), socket by socket; a grout deployment spreads its lcores the same
    way. "socket": the same over the L3 domains of one socket (the first
    allowed CPU's: the workers' staging memory and the GPU's link stay on
    it). None when the topology is unreadable or has fewer cores than n."""
    if policy not in ("spread", "socket") or not hasattr(os, "sched_getaffinity"):
        return None
    domains = {}
    for c in sorted(os.sched_getaffinity(0)):
        sib = _cpu_sysfs(c, "topology/thread_siblings_list")
        if sib is None:
            return None
        first = int(sib.replace("-", ",").split(",")[0])
        if first != c:
            continue  # an SMT sibling of a core already listed
        pkg = _cpu_sysfs(c, "topology/physical_package_id") or "0"
        l3 = _cpu_sysfs(c, "cache/index3/id") or pkg
        domains.setdefault((int(pkg), int(l3)), []).append(c)
    if policy == "socket" and domains:
        first = min(domains)[0]
        domains = {k: v for k, v in domains.items() if k[0] == first}
    order, lists = [], [domains[k] for k in sorted(domains)]
    for i in range(max((len(x) for x in lists), default=0)):
        order += [x[i] for x in lists if i < len(x)]
    return order[:n] if len(order) >= n else None


def b_pkt(fib_entry_bytes, out_bytes=64):
    return 64 + 8 + fib_entry_bytes + out_bytes + 8
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E spec peak


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=None,
                   help="packets per step per GPU (default 2^24; 2^22 for imix_frames, 8 GiB of 2 KiB slots)")
    p.add_argument("--workload", default="fullview64",
                   choices=["fullview64", "single64", "imix", "imix_frames", "fullview6"])
    p.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                   help="gr_hip_tune knobs set before the FIB load, e.g. v6_shortcut=1 (repeatable)")
    p.add_argument("--slot", type=int, default=2240,
                   help="imix_frames: bytes per frame slot (2240 = grout's mbuf object: 128 B rte_mbuf + "
                        "64 B priv + 2048 B data room, mempool.c:57-100)")
    p.add_argument("--placement", default="calibrated", choices=["calibrated", "plain"],
                   help="calibrated: batch buffers from gr_hip_batch_alloc, output lines re-placed by gr_hip_batch_place over "
                        "--candidates allocations; plain: torch allocations")
    p.add_argument("--candidates", type=int, default=8)
    p.add_argument("--no-plain", action="store_true",
                   help="skip the same measurement on plain torch allocations (value_plain_placement)")
    p.add_argument("--time-every", type=int, default=4,
                   help="HIP events around every N-th launch only (the kernel time is their average; "
                        "each event pair costs ~7 us of stream time)")
    p.add_argument("--output", default="line", choices=["line", "prefix32"],
                   help="line: each packet's whole 64-byte header line written back (BASELINE.md's 148 B); prefix32: "
                        "packed 32-byte prefixes, every byte the path changes (GR_HIP_BATCH_F_PREFIX32)")
    p.add_argument("--no-prefix-leg", action="store_true",
                   help="skip the same measurement with packed 32-byte output prefixes (prefix32 in the line)")
    p.add_argument("--settle-ms", type=float, default=100.0,
                   help="before the --warmup steps of each leg, run the same step untimed for this long: after the "
                        "idle gap of the stream upload the GPU takes ~20-40 launches to reach its steady clock "
                        "(tools/clock_probe.py); the forwarding plane's throughput is its steady-state rate")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-host-path", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=6.0, help="wall time of the CPU baseline sample")
    p.add_argument("--cpu-threads", type=int, default=16, help="host cores of the box share (16)")
    return p.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    from grout_amd import replicas

    # N GPUs = N replicas, one process each. Without a launcher the parent
    # starts them itself, before anything here touches a GPU, and exits with
    # their status; under one (torch.distributed.run) the world must be --gpus
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(replicas.spawn(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        log(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}: one rank per GPU, the two must agree")
        sys.exit(2)

    import torch

    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath, shared_stream

    # GR_BENCH_SHARE_GPU=1: a rehearsal of the N>1 path on a one-GPU box,
    # every rank on device 0; the driver's runs never set it. Barrier, clock
    # and report go over gloo either way (no collective on the data path)
    share = os.environ.get("GR_BENCH_SHARE_GPU") == "1"
    rep = replicas.Replicas("gloo")
    world, rank = rep.world, rep.rank
    local = 0 if share else rep.local
    if local >= torch.cuda.device_count():
        log(f"bench.py: rank {rank} wants device {local}, {torch.cuda.device_count()} visible")
        sys.exit(2)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    gpu_numa = abi.hip().gr_hip_device_numa_node(local)
    # the CPUs this process may use before the rank binds to its GPU's socket:
    # the CPU baseline gets them back (a box's whole share, not one socket's)
    own_cpus = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None
    bound = replicas.bind_to_numa(gpu_numa)  # this rank's host threads on its GPU's socket

    # ---- control plane: topology + FIB replica on this GPU
    t0 = time.time()
    if args.workload == "single64":
        topo = T.config_single_route()
        routes, dst_range = None, (T.ip4("16.1.0.0"), T.ip4("16.1.255.255"))
        workload = "config2: 64B synthetic burst, 1-route FIB"
    elif args.workload == "fullview6":
        topo = T.config_fullview6()
        routes, dst_range = None, None
        workload = ("IPv6: 64B synthetic burst, 200k-route IPv6 full view (fib_inject -6, "
                    "smoke/fib6_fullview_manualtest.sh sizing)")
    else:
        topo = T.config_fullview()
        routes, dst_range = topo.route_array(), None
        workload = {"fullview64": "config3: 64B synthetic burst, 1M-route full-view FIB (fib_inject)",
                    "imix": "config4: IMIX 64/570/1518 synthetic burst, full-view FIB, header lines staged",
                    "imix_frames": ("config4: IMIX 64/570/1518 synthetic burst, full-view FIB, whole frames "
                                    f"resident in {args.slot}-byte mbuf-like slots")}[args.workload]
    fp = FastPath(local)
    tune = dict(kv.split("=", 1) for kv in args.tune)
    for k, v in tune.items():
        fp.tune(k, int(v))
    fp.load(topo)
    info = fp.fib6_info(T.VRF_MAIN) if args.workload == "fullview6" else fp.fib_info(T.VRF_MAIN)
    log(f"[rank {rank}] topology + FIB loaded in {time.time() - t0:.1f}s: {info}")

    # ---- synthetic RX stream of this GPU (seed 0x67721000 + g)
    n = args.batch or (1 << 22 if args.workload == "imix_frames" else 1 << 24)
    seed = rep.seed()
    imix = args.workload == "imix"
    prefix32 = args.output == "prefix32"
    out_bytes = abi.PREFIX if prefix32 else abi.LINE
    in_stride = args.slot if args.workload == "imix_frames" else abi.LINE
    t0 = time.time()

    def make_stream(s):
        if args.workload == "fullview6":
            r6 = topo.route6_array()
            return S.stream6(n, s, r6[r6["prefixlen"] < 128])
        return S.stream(n, s, routes=routes, dst_range=dst_range, imix=imix or in_stride > abi.LINE,
                        lines_only=imix, stride=in_stride)

    def h2d(dst, src):
        src = np.ascontiguousarray(src)
        abi.check("gr_hip_memcpy_h2d", fp.lib.gr_hip_memcpy_h2d(fp.h, dst, src.ctypes.data, src.nbytes))

    frames, meta = make_stream(seed)
    batch = None
    if args.placement == "calibrated":
        # gr_hip_batch_alloc + gr_hip_batch_place: the output lines' pages are
        # picked among --candidates allocations by timing them over a batch of
        # the same workload drawn with ANOTHER seed; the
        # measured stream is then loaded into the placed buffers
        batch = fp.batch_alloc(n, in_stride)
        cf, cm = make_stream(seed ^ 0xCA11B)
        h2d(batch.in_frames, cf)
        h2d(batch.meta, cm)
        del cf, cm
        if imix:
            batch.flags = abi.BATCH_F_LINES_ONLY
        if prefix32:
            batch.flags |= abi.BATCH_F_PREFIX32
            batch.out_stride = abi.PREFIX
        fp.batch_place(batch, args.candidates)
        batch.flags = 0
        h2d(batch.in_frames, frames)
        h2d(batch.meta, meta)
        d_in, d_out, d_meta, d_v = batch.in_frames, batch.out_lines, batch.meta, batch.verdicts
    else:
        d_in = torch.from_numpy(frames.reshape(-1)).to(dev)
        d_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
        d_out = torch.empty(n * out_bytes, dtype=torch.uint8, device=dev)
        d_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    log(f"[rank {rank}] {n} packets generated and resident in {time.time() - t0:.1f}s")

    q = fp.queue(shared_stream(dev))
    every = max(1, min(args.time_every, args.steps))
    settle_launches = []  # per leg

    def measure(bufs, steps, warmup, prefix=None):
        """warmup + steps launches on `bufs`; -> (max-over-ranks seconds of the
        timed steps, kernel ms summed over the timed launches, their count)."""
        d_in_, d_out_, d_meta_, d_v_ = bufs
        pfx = prefix32 if prefix is None else prefix

        def step():
            q.submit(d_in_, d_out_, d_meta_, d_v_, n, in_stride=in_stride, out_stride=abi.LINE, lines_only=imix,
                     prefix32=pfx)

        # settle: the same step, untimed, until the GPU has been busy for
        # --settle-ms (its clock ramps up over the first tens of ms after idle)
        fp.tune("untimed", 1)
        t_settle, settled = time.perf_counter(), 0
        while time.perf_counter() - t_settle < args.settle_ms / 1e3:
            for _ in range(8):
                step()
            settled += 8
            torch.cuda.synchronize()
        fp.tune("untimed", 0)
        settle_launches.append(settled)
        fp.tune("time_every", every)  # every `every`-th submit of the queue carries events (count restarts)

        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        q.sync()  # raises if a kernel gave up a ring wait (-ETIMEDOUT)
        rep.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        own = time.perf_counter() - t0  # this replica's own clock
        rep.barrier()
        el = time.perf_counter() - t0
        q.sync()
        # setting time_every restarted the queue's count: submits 0, every,
        # 2 * every ... of warmup + steps carried events
        timed = sum(1 for i in range(warmup, warmup + steps) if i % every == 0)
        ms, cnt = q.kernel_ms(timed)
        fp.tune("time_every", 1)
        measure.own = own
        return rep.max_over_ranks(el), ms, cnt

    tmax, kern_ms, kcount = measure((d_in, d_out, d_meta, d_v), args.steps, args.warmup)
    own_s = measure.own

    if batch is not None:
        vh = np.empty(n, dtype=abi.VERDICT_DT)
        abi.check("gr_hip_memcpy_d2h", fp.lib.gr_hip_memcpy_d2h(fp.h, vh.ctypes.data, d_v, vh.nbytes))
        edges = np.bincount(vh["edge"], minlength=abi.E_COUNT)
        fp.batch_free(batch)
    else:
        edges = torch.bincount(d_v.view(n, 8)[:, 0].long(), minlength=abi.E_COUNT).cpu().numpy()
    fwd_frac = float(edges[abi.EDGE["port_output"]]) / n
    value = rep.aggregate_mpps(n, args.steps, tmax)
    avg_kernel_s = kern_ms / max(kcount, 1) / 1e3
    if args.workload == "fullview6":
        entry = 4  # fib6.h trie entries
    else:
        entry = 4 if fp.tune("fib_format_of", T.VRF_MAIN) == 0 else 2
    B_PKT = b_pkt(entry, out_bytes)
    achieved = n * B_PKT / avg_kernel_s / 1e9

    # HBM bytes per launch from PMC counters cannot be read from inside this
    # process: they come from separate rocprofv3 --pmc passes of the same
    # workload (tools/pmc_traffic.py), named with the file and run they came from
    traffic, traffic_src = None, None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        try:
            pm = json.load(open(tf))
            for e in pm if isinstance(pm, list) else [pm]:
                if e.get("workload") == args.workload and e.get("batch") == n and e.get("bytes_per_pkt") == B_PKT:
                    traffic = e.get("hbm_bytes_per_launch")
                    traffic_src = f"profiles/pmc_traffic.json <- {e.get('source', '?')}"
        except (OSError, ValueError, AttributeError):
            traffic, traffic_src = None, None

    # the same measurement on gr_hip_batch_alloc's buffers without placement
    # (physically contiguous allocations, "alloc_contig"): what a deployment
    # gets with no timing at start-up, in the same run
    contig = None
    if batch is not None and not args.no_plain:
        cb = fp.batch_alloc(n, in_stride)
        h2d(cb.in_frames, frames)
        h2d(cb.meta, meta)
        torch.cuda.synchronize()
        ct, cms, ccnt = measure((cb.in_frames, cb.out_lines, cb.meta, cb.verdicts), args.steps, args.warmup)
        contig = {"value": round(rep.aggregate_mpps(n, args.steps, ct), 1),
                  "ms_per_step": round(ct / args.steps * 1e3, 4),
                  "kernel_ms_avg": round(cms / max(ccnt, 1), 4),
                  "note": "gr_hip_batch_alloc buffers (physically contiguous), no placement timing"}
        fp.batch_free(cb)

    # the same measurement on plain torch allocations of the same stream:
    # the placement's share of `value`, in the same run
    plain = None
    if batch is not None and not args.no_plain:
        p_in = torch.from_numpy(frames.reshape(-1)).to(dev)
        p_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
        p_out = torch.empty(n * out_bytes, dtype=torch.uint8, device=dev)
        p_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        pt, pms, pcnt = measure((p_in, p_out, p_meta, p_v), args.steps, args.warmup)
        plain = {"value": round(rep.aggregate_mpps(n, args.steps, pt), 1),
                 "ms_per_step": round(pt / args.steps * 1e3, 4),
                 "kernel_ms_avg": round(pms / max(pcnt, 1), 4)}
        del p_in, p_meta, p_out, p_v

    # the same stream with packed 32-byte output prefixes (GR_HIP_BATCH_F_PREFIX32:
    # every byte the path changes; bytes 32-63 of a frame never change), on
    # plain allocations: what a deployment that writes back only the changed
    # bytes gets. Reported beside `value`, which keeps whole lines
    pfx_leg = None
    if not prefix32 and not args.no_prefix_leg and not imix:
        x_in = torch.from_numpy(frames.reshape(-1)).to(dev)
        x_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
        x_out = torch.empty(n * abi.PREFIX, dtype=torch.uint8, device=dev)
        x_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        xt, xms, xcnt = measure((x_in, x_out, x_meta, x_v), args.steps, args.warmup, prefix=True)
        xb = b_pkt(entry, abi.PREFIX)
        xk = xms / max(xcnt, 1)
        pfx_leg = {"value": round(rep.aggregate_mpps(n, args.steps, xt), 1),
                   "ms_per_step": round(xt / args.steps * 1e3, 4), "kernel_ms_avg": round(xk, 4),
                   "bytes_per_pkt": xb, "frac": round(n * xb / (xk / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if xk else None,
                   "placement": "plain torch allocations",
                   "note": "out_lines = packed 32-byte prefixes (GR_HIP_BATCH_F_PREFIX32), same verdicts and "
                           "changed bytes as whole lines"}
        del x_in, x_meta, x_out, x_v

    # every replica's own figures, next to the whole-job line: its GPU, the
    # NUMA node of its GPU and of the CPU it ran on, its own clock and kernel
    props = torch.cuda.get_device_properties(local)
    pci = None
    if hasattr(props, "pci_bus_id"):
        pci = f"{getattr(props, 'pci_domain_id', 0):04x}:{props.pci_bus_id:02x}:{getattr(props, 'pci_device_id', 0):02x}"
    mine = {"rank": rank, "device": local, "pci": pci, "gpu_numa": gpu_numa, "cpu_numa": replicas.cpu_numa_node(),
            "bound_to_gpu_numa": bound is not None, "mpps": round(n * args.steps / own_s / 1e6, 1),
            "ms_per_step": round(own_s / args.steps * 1e3, 4), "kernel_ms_avg": round(avg_kernel_s * 1e3, 4),
            "frac": round(achieved / HBM_PEAK_GBS, 4), "forwarded_frac": round(fwd_frac, 6),
            **({"kernel_ms_avg_plain": plain["kernel_ms_avg"]} if plain is not None else {})}
    ranks = rep.gather_objects(mine)

    result = {
        "metric": "Mpps IPv4 forward, 64B pkts, ~1M-route FIB (device-resident), 1/8 GPU",
        "value": round(value, 1),
        "unit": "Mpps",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle": {"ms": args.settle_ms, "launches": settle_launches[0] if settle_launches else 0,
                   "note": "untimed launches of the same step before the warmup steps of each leg: the GPU's "
                           "steady clock after the stream upload's idle gap"},
        "ms_per_step": round(tmax / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/u32 integer",
        "data": "synthetic (fib_inject route set, seeded 64B UDP stream per GPU)",
        "config": {
            "workload": workload,
            "batch_pkts_per_gpu": n,
            "routes": int(info["routes"]),
            **({"trie_groups_used": int(info["groups_used"])} if "groups_used" in info
               else {"tbl8_groups_used": int(info["tbl8_used"])}),
            "parallelism": f"replicas x{world} (one RX stream + FIB replica per GPU, no collective)"
            + (" [rehearsal: all ranks on one GPU]" if share else ""),
            "forwarded_frac": round(fwd_frac, 6),
            **({"tune": {k: int(v) for k, v in tune.items()}} if tune else {}),
            "occupancy_wg_per_cu": fp.tune("occupancy"),
            "placement": (f"calibrated: output lines, then frames = fastest of {args.candidates + 1} allocations "
                          "each (gr_hip_batch_alloc's, then plain and physically contiguous in turn), timed over a "
                          "batch of this workload drawn with another seed (gr_hip_batch_place)"
                          if batch is not None else "plain torch allocations"),
            "output": ("packed 32-byte header prefixes (every byte the path changes; GR_HIP_BATCH_F_PREFIX32)"
                       if prefix32 else "whole 64-byte header lines"),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "bytes_per_pkt": B_PKT,
            "kernel_ms_avg": round(avg_kernel_s * 1e3, 4),
            "kernel_launches_timed": kcount,
        },
    }
    if args.workload == "imix_frames":
        # the frame head is one 64-byte line of a 2 KiB slot: HBM moves it as a
        # 128-byte granule, so the bytes this layout must move per packet are
        # 64 more than the algorithmic figure
        floor = B_PKT + 64
        result["roofline"]["bytes_per_pkt_granule_floor"] = floor
        result["roofline"]["frac_at_granule_floor"] = round(n * floor / avg_kernel_s / 1e9 / HBM_PEAK_GBS, 4)
    if plain is not None:
        result["value_plain_placement"] = plain["value"]
        result["plain_placement"] = plain
        # the conservative figure: the same kernel on plain torch allocations
        if plain["kernel_ms_avg"]:
            result["roofline"]["frac_plain"] = round(n * B_PKT / (plain["kernel_ms_avg"] / 1e3) / 1e9 / HBM_PEAK_GBS,
                                                     4)
        result["roofline"]["kernel_ms_avg_plain"] = plain["kernel_ms_avg"]
    if contig is not None:
        result["contiguous_unplaced"] = contig
        if contig["kernel_ms_avg"]:
            result["roofline"]["frac_contiguous_unplaced"] = round(
                n * B_PKT / (contig["kernel_ms_avg"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
    if world > 1:
        result["ranks"] = ranks
    if pfx_leg is not None:
        result["prefix32"] = pfx_leg
    if args.workload == "fullview6":
        result["metric"] = "Mpps IPv6 forward, 64B pkts, 200k-route IPv6 view (device-resident) [non-headline]"
    elif args.workload != "fullview64":
        result["metric"] = result["metric"] + f" [non-headline workload: {args.workload}]"

    # every rank's GPU legs are done: after this barrier rank 0 alone goes on,
    # with the host-memory path on its own GPU and the CPU baseline on the
    # host's cores (N > 1 lines carry both too; the other ranks are idle)
    rep.barrier()
    if rank != 0:
        q.close()
        fp.close()
        rep.close()
        return

    # ---- host-memory path (PCIe-inclusive): reported, never `value`
    if not args.no_host_path:
        hn = min(n, 1 << 23)
        lines = torch.from_numpy(np.ascontiguousarray(frames[:hn, :abi.LINE]).reshape(-1)).pin_memory()
        hmeta = torch.from_numpy(meta[:hn].view(np.uint8)).pin_memory()
        hout = torch.empty(hn * abi.LINE, dtype=torch.uint8).pin_memory()
        hv = torch.empty(hn * 8, dtype=torch.uint8).pin_memory()
        hq = fp.queue()
        import ctypes
        fn = fp.lib.gr_hip_fwd4_host
        fn(hq._h, lines.data_ptr(), hmeta.data_ptr(), hn, hout.data_ptr(), hv.data_ptr())
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            r = fn(hq._h, lines.data_ptr(), hmeta.data_ptr(), hn, hout.data_ptr(), hv.data_ptr())
            abi.check("gr_hip_fwd4_host", r)
        ht = (time.perf_counter() - t0) / reps
        # packed 32-byte prefixes back (gr_hip_fwd4_host_ex): 40 B per packet D2H
        fx = fp.lib.gr_hip_fwd4_host_ex
        abi.check("gr_hip_fwd4_host_ex", fx(hq._h, lines.data_ptr(), hmeta.data_ptr(), hn, hout.data_ptr(),
                                            abi.PREFIX, hv.data_ptr()))
        t0 = time.perf_counter()
        for _ in range(reps):
            abi.check("gr_hip_fwd4_host_ex", fx(hq._h, lines.data_ptr(), hmeta.data_ptr(), hn, hout.data_ptr(),
                                                abi.PREFIX, hv.data_ptr()))
        hx = (time.perf_counter() - t0) / reps
        hq.close()
        del ctypes
        result["host_path"] = {
            "mpps": round(hn / ht / 1e6, 1),
            "pkts": hn,
            "h2d_bytes_per_pkt": abi.LINE + 8,
            "d2h_bytes_per_pkt": abi.LINE + 8,
            "mpps_prefix32": round(hn / hx / 1e6, 1),
            "note": ("header lines + metadata in pinned host memory; the kernel reads and writes them over "
                     "PCIe itself (host_direct), H2D and D2H concurrent; mpps_prefix32: 32-byte prefixes back "
                     "(gr_hip_fwd4_host_ex), 40 B per packet D2H"),
        }

    # ---- CPU baseline: the oracle restatement on this host's cores
    # (SURVEY.md §8d): pinned workers on one shared FIB (grout's layout: one
    # rte_fib per VRF for every worker), each starting at its own offset of
    # the sample, each warmed up by one untimed pass over the whole sample
    # before the timed part, one core per L3 domain in turn (cpu_placement);
    # the same leg packed on the first allowed CPUs beside it. The single-core
    # leg is the 16-core leg's worker 0
    # alone: same CPU, offset, warm-up, shared FIB and packet count, in the
    # same call; beside them the 16 workers with a FIB copy each on THP
    # (slower on the boxes measured: 16 tables of 128 MiB leave L3)
    if not args.no_cpu_baseline:
        import oracle
        if own_cpus is not None:  # unbound: the box's whole CPU share (cpu_placement picks from it)
            os.sched_setaffinity(0, own_cpus)
        o = oracle.Oracle(topo)
        cf, cm = frames[: 1 << 20].copy(), meta[: 1 << 20].copy()
        threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        allowed = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
        packed = allowed[:threads] if len(allowed) >= threads else None  # worker i on the i-th allowed CPU
        spread = cpu_placement(threads, "spread")  # one core per L3 domain in turn
        cpus = spread or packed
        one = cpus[:1] if cpus else None
        m0, _ = o.bench(cf, cm, 1, 1 << 20, fib_copy=False, cpus=one)  # sizes the timed parts
        per_thread = max(1 << 20, int(m0 * 1e6 * args.cpu_seconds))
        m1, _ = o.bench(cf, cm, 1, per_thread, fib_copy=False, cpus=one)
        cs0 = cgroup_cpu_stat()
        tS = time.perf_counter()
        mS, _ = o.bench(cf, cm, threads, per_thread, fib_copy=False, cpus=cpus)
        tS = time.perf_counter() - tS
        cs1 = cgroup_cpu_stat()
        m1b, _ = o.bench(cf, cm, 1, per_thread, fib_copy=False, cpus=one)  # after, same CPU
        mP = None
        if spread and packed and spread != packed:  # the same leg on the first allowed CPUs
            mP, _ = o.bench(cf, cm, threads, per_thread, fib_copy=False, cpus=packed)
        mN, _ = o.bench(cf, cm, threads, per_thread, cpus=cpus)
        single = (m1 + m1b) / 2

        def l3_domains(cs):
            return len({_cpu_sysfs(c, "cache/index3/id") for c in cs}) if cs else None
        # value: the better of the two placements, both measured in this call
        # (which one wins depends on the box's other load)
        best, best_name = (mP, "packed") if mP is not None and mP > mS else (mS, "spread")
        result["cpu_baseline"] = {
            "value": round(best, 2),
            "unit": "Mpps",
            "cores": threads,
            "kind": "port",
            "placement": best_name,
            "single_core_mpps": round(single, 2),
            "single_core_mpps_before_after": [round(m1, 2), round(m1b, 2)],
            "per_core_mpps": round(best / threads, 2),
            "per_core_over_single": round(best / threads / single, 3),
            "spread_mpps": round(mS, 2),
            "spread_per_core_over_single": round(mS / threads / single, 3),
            "l3_domains": l3_domains(cpus),
            # the same workers packed on the first allowed CPUs (fewer L3
            # domains: they share each CCD's L3 and its link to memory)
            "packed_mpps": round(mP, 2) if mP is not None else None,
            "packed_per_core_over_single": round(mP / threads / single, 3) if mP is not None else None,
            "packed_l3_domains": l3_domains(packed) if mP is not None else None,
            "fib_copy_mpps": round(mN, 2),
            # the cgroup's CPU-time quota over the multi-core leg: throttled
            # time is time the pinned workers were stopped by the quota, not
            # slowed by their own work (the process has other threads too)
            "quota_throttled_ms": round((cs1.get("throttled_usec", 0) - cs0.get("throttled_usec", 0)) / 1e3, 1)
            if cs0 and cs1 else None,
            "quota_throttled_periods": (cs1.get("nr_throttled", 0) - cs0.get("nr_throttled", 0)) if cs0 and cs1 else None,
            "multi_core_leg_s": round(tS, 2),
            "cpus": cpus,
            "host_cpus": host_cpus(),
            "ranks_idle": world - 1,  # the other replicas had finished (final barrier)
            "sample": (f"oracle C restatement of grout's node chain (bursts of 64, "
                       f"{'per-length prefix hash LPM6' if args.workload == 'fullview6' else 'DIR24_8 8-byte entries'}), "
                       f"{threads} pinned threads on one shared FIB (grout's layout: one rte_fib per VRF), "
                       f"each starting at its own offset of the same 1M-packet prefix of this stream, warmed up "
                       f"by one pass over it, then {per_thread} packets each timed; single_core_mpps: worker 0 "
                       f"alone (same CPU, offset, warm-up, shared FIB, packets), before and after the "
                       f"{threads}-core leg; value: the better of spread_mpps (one core per L3 domain in turn, as grout "
                       f"spreads its lcores) and packed_mpps (the first {threads} allowed CPUs); "
                       f"fib_copy_mpps: the {threads} workers with a FIB copy each on THP"),
        }
        o.close()

    print(json.dumps(result), flush=True)
    q.close()
    fp.close()
    rep.close()


if __name__ == "__main__":
    main()
