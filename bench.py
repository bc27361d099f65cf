"""Benchmark: simulated packets/sec of the network.Config enforcement path (BASELINE.json metric).

Default workload (BASELINE.json configs[2]): storm-style random all-to-all traffic
over 10,000 instances per GPU, heterogeneous LinkShape (latency/jitter/loss/dup/corrupt/reorder/
bandwidth), Poisson(0.5) packets per instance per 1 µs tick.  One step = one pass of the hot path
over one window of `--window` ticks of offered traffic that is already resident in HBM (generated
on the device before the timed region): filter -> netem -> HTB (k_sim), routing by destination
shard, RCCL all-to-all (N > 1), per-destination delivery sort.  The same line carries an
`at_1M_peers` object: the C4 gossip flood over 1,000,000 peers in total (split over the N GPUs),
so both halves of BASELINE.json's metric ("at 10k & 1M peers") are measured in one run.

`--workload gossip` (C4, BASELINE.json configs[3]): flood of 64 messages over --peers instances per
GPU, degree 8, 1 KiB, L~U[5,50] ms, loss 1 %.  A step is one 5 ms window: forwards of the previous
window's receipts generated on the device, then the hot path.
`--workload epochs` (C5, configs[4]): 100,000 instances per GPU, C3 shapes and traffic at
lambda 0.2, 1,000-tick epochs; a step reshapes 10 % of the instances (batched ConfigureNetwork),
runs the epoch and passes the `epoch-k` barrier (counters summed over ranks on the device).

Launch: N = 1 runs directly.  `--gpus N` with N > 1 and no WORLD_SIZE in the environment starts N
ranks itself (torch.distributed.run, one process per GPU) from this parent, which never touches
the GPU; under an external launcher WORLD_SIZE must equal --gpus.  The storm headline is
BASELINE.json configs[2] at every N: 10,000 instances in total, split over the ranks (strong
scaling); at N > 1 the line also carries `weak_per_gpu`, the same storm with 10,000 instances per
rank.  The 1M-peer gossip is 1,000,000 peers in total at every N.  Cross-shard deliveries are
exchanged by the engine's RCCL all-to-all.
"""
import argparse
import ctypes
import hashlib
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "simulated packets/sec (whole node) at 10k & 1M peers; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

# Algorithmic HBM bytes of k_sim: per offered packet 16 B record read + 1 B verdict
# write; per scheduled record 24 B delivery write; per source 64 B params + 32 B state read + 32 B
# state write + 16 B CSR offsets + 4 B emit count; plus the netem queue state the kernel actually
# carries between windows through HBM (16 B per queued item, 8 B per departing item, loaded and
# stored once per fused group: tgsim_debug_carry_bytes), reported apart as carry_bytes.  The r02
# basis charged the per-window model of that carry (queue_state_bytes: a load and a store at every
# window), which rewards re-streaming; it is kept as frac_modeled_restream.
B_OFFERED, B_SCHEDULED, B_SOURCE = 17, 24, 148
REC = 24  # sizeof(tgsim_delivery), the record an exchange moves


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None, help="timed steps (default: storm 30, epochs 30, gossip 70 windows)")
    p.add_argument("--warmup", type=int, default=None, help="untimed steps (default: 3; gossip: 0)")
    p.add_argument("--workload", default="storm", choices=["storm", "gossip", "epochs", "bridge"])
    p.add_argument("--peers", type=int, default=0,
                   help="storm: instances in total, split over the GPUs (configs[2]; at N > 1 a second run with "
                        "this many per GPU is reported as weak_per_gpu); gossip/epochs/bridge: instances per GPU "
                        "(default: storm 10,000; gossip 125,000; epochs 100,000)")
    p.add_argument("--floods", type=int, default=64, help="gossip: flood messages")
    p.add_argument("--flood-gap", type=int, default=1000, help="gossip: ticks between flood starts")
    p.add_argument("--lam", type=float, default=None,
                   help="packets per us per source (default: storm 0.5, storm --shapes open 0.008, epochs 0.2)")
    p.add_argument("--window", type=int, default=2000, help="ticks (1 us) per step")
    p.add_argument("--settle-ms", type=float, default=120.0,
                   help="untimed simulated time before warm-up so every netem queue is in its sustained "
                        "storm state (> max latency + jitter = 110 ms); queues start empty otherwise")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=min(16, os.cpu_count() or 1),
                   help="threads of the all-core CPU oracle leg (the GPU box's CPU share is 16)")
    p.add_argument("--queue-limit", type=int, default=0, help="netem limit (0 = netlink default 1000)")
    p.add_argument("--shapes", default="storm", choices=["storm", "open", "fixed"],
                   help="storm: C3 heterogeneous shapes; open: C3 shapes at 1 Gbit/s driven below capacity "
                        "(the sub-capacity variant); fixed: L=5 ms, no jitter/loss/reorder (probe)")
    p.add_argument("--sharded", action="store_true",
                   help="use the engine's exchange (tgsim_comm_*) even at one rank; there it is the single-shard "
                        "step (nothing to route) unless TGSIM_COMM_ROUTE1=1 keeps the routed N>1 path")
    p.add_argument("--exact-exchange", action="store_true",
                   help="sharded storm: exchange exact record counts every step instead of fixed-size chunks")
    p.add_argument("--no-1m", action="store_true",
                   help="storm: skip the at_1M_peers gossip run that accompanies the headline line")
    p.add_argument("--no-variants", action="store_true",
                   help="storm: skip the at_subcapacity and at_epochs runs that accompany the headline line")
    p.add_argument("--gossip-1m-peers", type=int, default=1_000_000,
                   help="total peers of the at_1M_peers run (split over the ranks)")
    p.add_argument("--launch-check", action="store_true",
                   help="launcher self-test: every rank reports RANK/WORLD_SIZE and exits before any GPU call")
    a = p.parse_args(argv)
    if not a.peers:
        a.peers = {"storm": 10_000, "gossip": 125_000, "epochs": 100_000, "bridge": 1000}[a.workload]
    if a.workload in ("epochs", "bridge"):
        a.lam, a.window = 0.2, 1000
    if a.lam is None:
        from testground_amd.workloads import STORM_OPEN_LAMBDA
        a.lam = STORM_OPEN_LAMBDA if a.shapes == "open" else 0.5
    if a.workload == "gossip":
        a.window = 5000
    if a.steps is None:
        a.steps = {"gossip": 70, "epochs": 30, "bridge": 200}.get(a.workload, 30)  # storm: amortizes the pipeline fill and drain
    if a.warmup is None:
        a.warmup = 0 if a.workload == "gossip" else 3
    return a


# ------------------------------------------------------------------------------------------------
# Launcher: the driver may call `bench.py --gpus N` bare; ranks are then started from here, before
# anything initializes HIP in this process (a GPU-initialized process must never exec).
def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(n: int, argv, port: int):
    """torch.distributed.run command that starts n ranks of this script with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve()), *argv]


def launch_decision(gpus: int, env) -> str:
    """'run' (this process is a rank), 'spawn' (start gpus ranks) or an error message."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "spawn" if gpus > 1 else "run"
    if int(ws) != gpus:
        return f"bench.py: WORLD_SIZE={ws} but --gpus {gpus}; launch one rank per GPU (--nproc-per-node {gpus})"
    return "run"


def spawn_ranks(n: int, argv) -> int:
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["TGSIM_BENCH_LAUNCHED"] = "1"
    return subprocess.run(launch_command(n, argv, free_port()), env=env).returncode


# ------------------------------------------------------------------------------------------------
def kernel_sha16() -> str:
    return hashlib.sha256((ROOT / "testground_amd" / "csrc" / "tgsim_kernels.hip").read_bytes()).hexdigest()[:16]


def cpu_baseline(a, workload, peers_total, lam, window, cpu_seconds, shapes=None):
    """The CPU oracle (a 'port' of the reference semantics) timed on this host, on a bounded sample
    of the same workload: single thread, plus (storm/epochs) one oracle shard per thread."""
    from testground_amd import abi, workloads
    from testground_amd.build import build_oracle
    from testground_amd.engine import CABIEngine

    lib = ctypes.CDLL(str(build_oracle()))
    abi.declare(lib, "tgo_")
    busy, steps = 0.0, 0
    if workload == "gossip":  # closed loop: needs every peer, so the sample is a smaller flood
        n = min(peers_total, 20_000)

        def gleg(seconds):
            """The flood over n instances on one oracle engine, stepped for ~seconds of step time."""
            e = CABIEngine(lib, "tgo_", n, lookahead_ns=workloads.GOSSIP_MIN_LAT)
            workloads.configure_gossip(e, n)
            e.gossip_init(n_floods=a.floods, degree=8, msg_len=1024, start_gap_ticks=a.flood_gap, start_tick=0)
            busy, steps = 0.0, 0
            while busy < seconds and steps < 400:
                t0 = time.perf_counter()
                e.gen_gossip(window)
                e.step(window)
                busy += time.perf_counter() - t0
                steps += 1
                e.drain()
            return e.stats()["offered"], busy, steps

        pkts, busy, steps = gleg(cpu_seconds)
        sample = (f"oracle/tgoracle.c, the same flood over {n} instances ({a.floods} floods, degree 8), "
                  f"{steps} windows of {window} ticks incl. forward generation, {pkts} packets, {busy:.1f} s")
        one = {"value": pkts / busy, "unit": "packets/s", "cores": 1, "kind": "port", "sample": sample}
        if a.cpu_threads <= 1:
            return one
        # all-core leg: the closed loop cannot be split without an exchange, so every thread runs its
        # own replica of the flood (ctypes drops the GIL); the sum of the per-thread rates
        from concurrent.futures import ThreadPoolExecutor

        t = a.cpu_threads
        w0 = time.perf_counter()
        with ThreadPoolExecutor(t) as ex:
            res = list(ex.map(lambda _: gleg(cpu_seconds / 2), range(t)))
        wall = time.perf_counter() - w0
        return {"value": sum(p / b for p, b, _ in res), "unit": "packets/s", "cores": t, "kind": "port",
                "sample": (f"oracle/tgoracle.c, {t} threads, each an independent replica of the flood over "
                           f"{n} instances ({a.floods} floods, degree 8) for ~{cpu_seconds / 2:.0f} s of step "
                           f"time; {sum(p for p, _, _ in res)} packets, {wall:.1f} s wall"),
                "single_thread": one}
    sample_src = min(1000, peers_total)
    shapes = shapes or a.shapes

    def leg(lo, hi, seconds):
        """One oracle shard [lo, hi) of the same workload stepped for ~seconds of step time."""
        e = CABIEngine(lib, "tgo_", peers_total, shard=(lo, hi))
        workloads.configure_storm(e, peers_total, open_links=shapes == "open")
        busy, steps = 0.0, 0
        while busy < seconds:
            if workload == "epochs" and steps:
                plan = workloads.epoch_plan(peers_total, steps)  # (ahead of the timing, as on the GPU leg)
                r0 = time.perf_counter()
                workloads.epoch_reshape(e, peers_total, steps, plan=plan)
                busy += time.perf_counter() - r0
            e.gen_storm(lam, window)
            t0 = time.perf_counter()
            e.step(window)
            busy += time.perf_counter() - t0
            steps += 1
            e.drain()
        return e.stats()["offered"], busy, steps

    pkts, busy, steps = leg(0, sample_src, cpu_seconds)
    sample = (f"oracle/tgoracle.c, sources 0..{sample_src - 1} of the {peers_total}-instance {workload} "
              f"workload, lambda={lam}, {steps} windows of {window} ticks, {pkts} packets, {busy:.1f} s")
    if a.cpu_threads > 1:  # all-core leg: one oracle shard per thread (ctypes drops the GIL)
        from concurrent.futures import ThreadPoolExecutor

        t = a.cpu_threads
        per = max(1, min(sample_src, peers_total // t))
        w0 = time.perf_counter()
        with ThreadPoolExecutor(t) as ex:
            res = list(ex.map(lambda k: leg(k * per, (k + 1) * per, cpu_seconds / 2), range(t)))
        wall = time.perf_counter() - w0
        # each thread's packets over its own stepping time; the sum is the all-core rate
        rate = sum(p / b for p, b, _ in res)
        return {"value": rate, "unit": "packets/s", "cores": t, "kind": "port",
                "sample": (f"oracle/tgoracle.c, {t} threads, thread k steps sources "
                           f"[{per}k, {per}(k+1)) of the {peers_total}-instance {workload} workload "
                           f"(lambda={lam}, windows of {window} ticks) for ~{cpu_seconds / 2:.0f} s; "
                           f"{sum(p for p, _, _ in res)} packets, {wall:.1f} s wall"),
                "single_thread": {"value": pkts / busy, "cores": 1, "sample": sample}}
    return {"value": pkts / busy, "unit": "packets/s", "cores": 1, "kind": "port", "sample": sample}


def load_pmc(workload, window, peers, lam, shapes="storm", kind="k_sim"):
    """HBM traffic of k_sim (kind "delivery": of the delivery kernels) from the committed PMC passes
    (rocprofv3 cannot run inside the bench).  Reported only when the file was collected on the same
    kernel source (sha of tgsim_kernels.hip) and the same workload configuration; the line names the
    file and its provenance either way."""
    tag = workload if workload != "storm" or shapes == "storm" else f"storm_{shapes}"
    f = ROOT / "profiles" / (f"pmc_{kind}.json" if tag == "storm" else f"pmc_{kind}_{tag}.json")
    src = {"file": str(f.relative_to(ROOT)), "kernel_sha16_now": kernel_sha16()}
    if not f.exists():
        return None, dict(src, status="absent")
    try:
        pmc = json.loads(f.read_text())
    except Exception:
        return None, dict(src, status="unreadable")
    src.update({k: pmc.get(k) for k in ("kernel_sha16", "commit", "peers", "lam", "window")})
    if pmc.get("kernel_sha16") != src["kernel_sha16_now"]:
        return None, dict(src, status="stale: collected on another k_sim source")
    want_shapes = shapes if workload == "storm" else workload  # gossip/epochs have their own shapes
    if (pmc.get("window") != window or pmc.get("peers") != peers
            or (workload != "gossip" and pmc.get("lam", lam) != lam) or pmc.get("shapes", "storm") != want_shapes):
        return None, dict(src, status="other configuration")
    return pmc.get("hbm_bytes_per_launch"), dict(src, status="matches this kernel and configuration")


WORKLOAD_NAMES = {
    "storm": "C3 storm: random all-to-all, heterogeneous LinkShape (BASELINE.json configs[2])",
    "storm_open": "C3 storm, sub-capacity variant: C3 shapes with every link at 1 Gbit/s, lambda 0.008 "
                  "(no netem queue at its limit)",
    "gossip": "C4 gossip flood: degree 8, 1 KiB, L~U[5,50] ms, loss 1 % (BASELINE.json configs[3])",
    "epochs": "C5 epochs: C3 traffic at lambda 0.2, 10 % reshaped per 1,000-tick epoch, barrier per epoch "
              "(BASELINE.json configs[4])",
    "bridge": "C6 bridge: real payloads (U[64,512] B) through the native packet bridge, 16 datagrams per "
              "instance per 1 ms window to random peers, L~U[1,10] ms, J~U[0,1] ms, loss/dup/corrupt 1 %, 1 Gbit/s",
}


def run_bridge(a, world, rank, local, dist, want_cpu):
    """C6: datagrams with payloads through tgsim_bridge_* (send -> engine step -> payload matching
    -> per-destination FIFOs -> receive into the caller's buffers), one bridge of --peers instances
    per rank (independent replicas).  The payloads live in host memory, so this line is host-inclusive
    by construction: it measures the whole datagram path a plan's packets take, not the kernel."""
    import numpy as np
    import torch

    from testground_amd import bridge as br
    from testground_amd import workloads
    from testground_amd.engine import Engine

    n, window = a.peers, 1000
    eng = Engine(n, device=local, lookahead_ns=window * 1000)
    workloads.configure_bridge(eng, n)
    b = br.NativeBridge(eng, n, window)
    src, dst, data, off = workloads.bridge_traffic(n)
    msgs = np.empty(4 * len(src), dtype=br.MSG_DTYPE)
    buf = np.empty(4 * len(data) + (1 << 20), dtype=np.uint8)
    got = [0, 0]

    def one():
        b.send_many(src, dst, data, off)
        b.step()
        while True:
            k = b.recv_into(msgs, buf)
            got[0] += k
            got[1] += int(msgs["len"][:k].sum()) if k else 0
            if k < len(msgs):
                break

    for _ in range(20 + a.warmup):  # past the largest latency + jitter: the FIFOs are in steady state
        one()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
        torch.cuda.synchronize()
    got[:] = [0, 0]
    t0 = time.perf_counter()
    for _ in range(a.steps):
        one()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    s = eng.stats()
    b.close()
    eng.close()
    if dist:
        t = torch.tensor([el, float(got[0]), float(got[1])], dtype=torch.float64)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        el, delivered, nbytes = float(mx[0]), float(t[1]), float(t[2])
    else:
        delivered, nbytes = float(got[0]), float(got[1])
    if rank != 0:
        return None
    res = {
        "metric": "datagrams/s delivered with payloads through the native packet bridge",
        "value": delivered / el, "unit": "datagrams/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": el * 1e3 / a.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8 payloads, u32/u64 records",
        "data": "synthetic (host-generated datagrams, fixed per-window pattern)",
        "config": {"workload": WORKLOAD_NAMES["bridge"], "peers_per_gpu": n, "peers_total": n * world,
                   "window_ticks": window, "tick_ns": 1000, "datagrams_sent_per_step": len(src) * world,
                   "parallelism": f"independent replicas x{world}"},
        "sent_per_s": len(src) * world * a.steps / el,
        "payload_bytes_per_s": nbytes / el,
        "engine_by_verdict": s["by_verdict"],
        "roofline": None,
        "cpu_baseline": None,
    }
    if world == 1 and want_cpu:
        res["cpu_baseline"] = cpu_bridge_baseline(n, window, a.cpu_seconds)
        res["cpu_baseline"]["gpu_over_cpu"] = res["value"] / res["cpu_baseline"]["value"]
    return res


def cpu_bridge_baseline(n, window, seconds):
    """The Python PacketBridge over the CPU oracle, same instances, shapes and send pattern."""
    from testground_amd import abi, workloads
    from testground_amd.bridge import PacketBridge
    from testground_amd.build import build_oracle
    from testground_amd.engine import CABIEngine

    lib = ctypes.CDLL(str(build_oracle()))
    abi.declare(lib, "tgo_")
    e = CABIEngine(lib, "tgo_", n, lookahead_ns=window * 1000)
    workloads.configure_bridge(e, n)
    b = PacketBridge(e, n, window)
    src, dst, data, off = workloads.bridge_traffic(n)
    items = [(int(s), int(d), data[int(off[i]):int(off[i + 1])]) for i, (s, d) in enumerate(zip(src, dst))]
    got, steps, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for s, d, p in items:
            b.send(s, d, p)
        b.step()
        got += sum(len(b.recv(p)) for p in range(n))
        steps += 1
    el = time.perf_counter() - t0
    return {"value": got / el, "unit": "datagrams/s", "cores": 1, "kind": "port",
            "sample": f"testground_amd/bridge.py PacketBridge over oracle/tgoracle.c, {n} instances, "
                      f"{steps} windows of {len(items)} sends ({el:.1f} s, including the fill of the first windows)"}


def shard_bounds(peers, world, split):
    """(instances in total, contiguous source ranges of the ranks): `peers` per rank, or with split
    `peers` in total, split evenly (contiguous source partition)."""
    total = peers if split else peers * world
    return total, [r * total // world for r in range(world)] + [total]


# The host process group only carries the bench's own bookkeeping (the RCCL id broadcast, barriers,
# the max/sum of the timed results); every data-path collective is the engine's own RCCL communicator
# (tgsim_comm_*).  A gloo group keeps each process at ONE RCCL communicator: a second one (torch's
# NCCL group) would double RCCL's streams and buffers on a box with 4 hardware queues per process.
HOST_GROUP_BACKEND = "gloo"


def init_host_group(world):
    """The bench's host process group (gloo, over 127.0.0.1)."""
    import torch.distributed as dist

    if world == 1 and "MASTER_PORT" not in os.environ:
        # one rank started without a launcher (--sharded): an in-process store, no TCP port to
        # race for (a probed free port was once taken before the store bound it: EADDRINUSE)
        dist.init_process_group(HOST_GROUP_BACKEND, store=dist.HashStore(), rank=0, world_size=1)
    else:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group(HOST_GROUP_BACKEND)
    return dist


T_START = time.perf_counter()


def progress(msg):
    """A progress line on stderr (the JSON line alone goes to stdout): a long default run keeps
    writing, so that a watchdog on the GPU box never takes it for a hung run."""
    print(f"bench [{time.perf_counter() - T_START:7.1f} s] {msg}", file=sys.stderr, flush=True)


def runs_cpu_baseline(rank, want_cpu):
    """North star: the oracle is timed 'on the box's own host cores in the same run' beside the GPU
    line at every world size; rank 0 runs it (after the timed region, the other ranks wait)."""
    return want_cpu and rank == 0


def headline_plan(a, world):
    """What the default line measures at this world size (bench.py --launch-check prints it)."""
    total, bounds = shard_bounds(a.peers, world, a.workload == "storm")
    plan = {"workload": a.workload, "peers_total": total, "bounds": bounds,
            "scaling": "strong" if a.workload == "storm" and world > 1 else "weak"}
    if a.workload == "storm" and world > 1:
        plan["weak_per_gpu_peers_total"] = shard_bounds(a.peers, world, False)[0]
    if a.workload == "storm" and not a.no_1m:
        plan["at_1M_peers_total"] = shard_bounds(a.gossip_1m_peers, world, True)[0]
    if a.workload == "storm" and not a.no_variants:
        plan["at_subcapacity_total"] = shard_bounds(a.peers, world, True)[0]
        plan["at_epochs_total"] = shard_bounds(100_000, world, True)[0]
    plan["cpu_baseline_ranks"] = [r for r in range(world) if runs_cpu_baseline(r, not a.no_cpu)]
    return plan


def run_workload(a, workload, peers, steps, warmup, window, lam, world, rank, local, dist, want_cpu,
                 split=False, shapes=None):
    """Builds one engine shard on this rank, brings the workload to its timed state, times `steps`
    steps (barrier + synchronize on both sides, max over ranks) and returns the rank-0 result object
    (None on the other ranks).  `peers` instances per rank (weak scaling), or with split=True
    `peers` instances in total, split evenly over the ranks (strong scaling)."""
    import numpy as np
    import torch

    from testground_amd import abi, workloads
    from testground_amd.engine import Engine
    from testground_amd.network import configs_array

    sharded = dist is not None
    shapes = shapes or a.shapes
    peers_total, bounds = shard_bounds(peers, world, split)
    lo, hi = bounds[rank], bounds[rank + 1]
    peers = hi - lo  # this rank's sources
    kw = dict(lookahead_ns=workloads.GOSSIP_MIN_LAT) if workload == "gossip" else {}
    # the sub-capacity storm's 0.12-ms windows: HIP timing events around every window cost 2-5 % of
    # it, so its simulate and delivery spans are sampled every 8th window (the windows
    # of a settled storm are alike); the engine reads these when it is created
    sample = {k: "8" for k in ("TGSIM_SIM_TIMING", "TGSIM_DV_TIMING")
              if workload == "storm" and shapes == "open" and k not in os.environ}
    os.environ.update(sample)
    try:
        eng = Engine(peers_total, shard=(lo, hi), device=local, flags=abi.OPT_DISCARD_DELIVERIES,
                     queue_limit=a.queue_limit, **kw)
    finally:
        for k in sample:
            del os.environ[k]
    timing_every = int(os.environ.get("TGSIM_SIM_TIMING", sample.get("TGSIM_SIM_TIMING", "1")))
    t_setup = time.perf_counter()
    if workload == "gossip":
        workloads.configure_gossip(eng, peers_total)
    elif shapes in ("storm", "open"):
        workloads.configure_storm(eng, peers_total, open_links=shapes == "open")
    else:
        eng.configure_batch(np.arange(peers_total), configs_array(np.full(peers_total, 5_000_000), routing_policy=2))
    stepper = None
    if sharded:  # the engine's own RCCL exchange (tgsim_comm_*), as a Go host would drive it
        from testground_amd.shard import CommStepper
        stepper = CommStepper(eng, bounds, device="cpu")  # the id crosses the gloo host group
    step = eng.step if stepper is None else stepper.step
    epoch = [0]
    plans = {}  # epochs: each epoch's reshape as its plan asks for it, computed before the timed loop
    host_s = {"step": 0.0, "reshape": 0.0, "signal": 0.0, "barrier": 0.0}  # epochs: host time per call

    def timed(name, fn, *args):
        t = time.perf_counter()
        r = fn(*args)
        host_s[name] += time.perf_counter() - t
        return r

    def reshape(k):
        workloads.epoch_reshape(eng, peers_total, k, plan=plans.pop(k, None))

    def one_step():
        if workload == "gossip":
            eng.gen_gossip(window)
            step(window)
        elif workload == "epochs":  # traffic pre-generated; reshape + epoch + barrier
            k = epoch[0]
            if stepper is None:
                # as the sharded step below: epoch k+1's ConfigureNetwork calls are staged on the
                # host while epoch k simulates (the step is asynchronous) and take effect at the
                # next step; epoch 0 runs on the initial configs
                timed("step", step, window)
                timed("reshape", reshape, k + 1)
            else:
                # the sharded step waits for its records, so epoch k+1's ConfigureNetwork calls
                # are staged on the host while epoch k simulates (epoch k's were staged during
                # epoch k-1); staged configs take effect at the next launch, after the barrier below
                stepper.step(window, between=lambda: reshape(k + 1))
            state, rnd = workloads.epoch_state(k)
            timed("signal", eng.signal_async, state, peers)  # K7: the count stays on the device
            ok = timed("barrier", stepper.barrier if stepper else eng.barrier_poll, state, rnd * peers_total)
            if not ok:
                raise RuntimeError(f"barrier epoch-{k} did not release")
            epoch[0] += 1
        else:
            step(window)

    if workload == "gossip":
        # two empty windows, untimed: the step's buffers are allocated and first touched here, not
        # in the timed flood; the floods start at the next window
        for _ in range(2):
            step(window)
        eng.gossip_init(n_floods=a.floods, degree=8, msg_len=1024, start_gap_ticks=a.flood_gap)
        settle = 0  # a flood is a transient by nature: the timed windows cover it from the start
    else:
        settle = int(a.settle_ms * 1000 / window + 0.999)
        if workload == "epochs":  # the plan's reshape requests of the warm-up and timed epochs, ahead
            plans.update({k: workloads.epoch_plan(peers_total, k) for k in range(settle + 1, settle + warmup + steps + 2)})
        for _ in range(settle):  # untimed: bring every netem queue to its sustained state
            eng.gen_storm(lam, window)
            one_step()
        for _ in range(warmup + steps):
            eng.gen_storm(lam, window)  # inputs resident in HBM before the timed region

    def run_steps(n):
        if stepper is not None and workload == "storm" and a.exact_exchange:
            for _ in range(n):
                stepper.step(window)
        elif stepper is not None and workload == "storm":  # pre-generated: simulate one step ahead
            # slotted exchange: groups of TGSIM_SHARD_FUSE (4) windows per launch and per all-to-all
            # (A/B at one rank: 1 27.5, 4 30.4, 8 27.7-28.6 G pkt/s: larger groups lengthen the
            # pipeline drain); TGSIM_FUSE is the single engine's group size (default 8, tgsim_step_n)
            stepper.run(n, window, fuse=int(os.environ.get("TGSIM_SHARD_FUSE", "4")))
        elif workload == "storm":  # pre-generated windows, up to TGSIM_FUSE (8) per launch (tgsim_step_n)
            eng.step_n(window, n)
        else:
            for _ in range(n):
                one_step()

    # the pipelined run's fixed-size chunks are sized by the engine from the largest per-rank count
    # the settle windows exchanged (max over ranks, x1.25 + 4096); an overflow fails the run
    run_steps(warmup)
    eng.drain()
    setup_s = time.perf_counter() - t_setup
    for k in host_s:
        host_s[k] = 0.0
    s0 = eng.stats()
    x0 = stepper.exchanged_records if stepper is not None else 0
    eng.sim_kernel_ms(reset=True)
    eng.delivery_kernel_ms(reset=True)
    c0 = eng.carry_bytes()
    k0 = eng.bucket_records()
    # the device is idle before the barrier (the engine's own communicator and torch's never have
    # collectives in flight at once), and again after it (the barrier's kernel)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(steps)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    s1 = eng.stats()
    offered = s1["offered"] - s0["offered"]
    scheduled = s1["scheduled"] - s0["scheduled"]
    verd = np.array([s1["by_verdict"][k] - s0["by_verdict"][k] for k in abi.VERDICT_NAMES], dtype=np.float64)
    exch = (stepper.exchanged_records - x0) if stepper is not None else 0
    sim_ms, n_launch = eng.sim_kernel_ms()
    dv_ms, n_dv = eng.delivery_kernel_ms()
    if dist:
        t = torch.tensor([el, float(offered), float(scheduled), float(exch), *verd], dtype=torch.float64)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        el = float(mx[0])
        offered_all, scheduled_all, exch_all = float(t[1]), float(t[2]), float(t[3])
        verd_all = t[4:].numpy()
    else:
        offered_all, scheduled_all, exch_all, verd_all = float(offered), float(scheduled), 0.0, verd
    extra = {}
    if workload == "epochs":  # where the host's time per epoch goes
        extra["host_us_per_epoch"] = {k: v * 1e6 / max(1, steps) for k, v in host_s.items()}
    if workload == "gossip":
        reached = eng.gossip_reached()
        if dist:
            r = torch.as_tensor(reached.astype(np.int64))
            dist.all_reduce(r)
            reached = r.numpy()
        extra = {"floods": a.floods, "flood_gap_ticks": a.flood_gap,
                 "reached_min_frac": float(reached.min()) / peers_total,
                 "sim_ms_covered": (warmup + steps) * window / 1000}
    qbytes = s1["queue_state_bytes"] - s0["queue_state_bytes"]
    carry = eng.carry_bytes() - c0
    bkt = eng.bucket_records() - k0
    slot_cap = stepper.slot_cap if stepper is not None else None
    n_dst_rank = hi - lo
    eng.close()
    del eng, stepper
    cpu = None
    progress(f"{workload} ({shapes if workload == 'storm' else workload}, {peers_total} peers): "
             f"{offered_all / el / 1e9:.3f} G pkt/s, {el * 1e3 / steps:.4f} ms/step")
    if runs_cpu_baseline(rank, want_cpu):  # the oracle on this host's cores, beside the line at every N
        cpu = cpu_baseline(a, workload, peers_total, lam, window,
                           a.cpu_seconds if workload == "storm" else a.cpu_seconds / 2, shapes=shapes)
        progress(f"{workload} CPU baseline: {cpu['value'] / 1e6:.1f} M pkt/s")
    if dist:  # the other ranks wait here for rank 0's CPU legs before the next collective
        torch.cuda.synchronize()
        dist.barrier()
    if rank != 0:
        return None
    base = (B_OFFERED * offered + B_SCHEDULED * scheduled) / max(1, steps) + B_SOURCE * peers
    carry_w, model_w = carry / max(1, steps), qbytes / max(1, steps)
    per_launch = base + carry_w
    gbs = (lambda b: b / (sim_ms * 1e-3) / 1e9) if sim_ms > 0 else (lambda b: None)
    achieved = gbs(per_launch)
    frac_of = lambda b: (gbs(b) / HBM_PEAK_GBS) if sim_ms > 0 else None  # noqa: E731
    traffic, traffic_src = load_pmc(workload, window, peers, lam, shapes)
    tot_v = max(1.0, float(verd_all.sum()))
    res = {
        "metric": METRIC,
        "value": offered_all / el,
        "unit": "packets/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": el * 1e3 / steps,
        "higher_is_better": True,
        "scaling": "strong" if split and world > 1 else "weak",
        "vs_baseline": None,
        "dtype": "u32/u64 integer",
        "data": f"synthetic (device-generated {workload} traffic, Philox-keyed)",
        "config": dict({"workload": WORKLOAD_NAMES["storm_open" if workload == "storm" and shapes == "open"
                                                   else workload],
                        "peers_per_gpu": peers, "peers_total": peers_total,
                        **({} if workload == "gossip" else {"lambda_per_tick": lam}), "tick_ns": 1000, "window_ticks": window, "settle_sim_ms": settle * window / 1000,
                        "shapes": shapes if workload == "storm" else workload,
                        "queue_limit": a.queue_limit or 1000, "packets_per_step": offered_all / steps,
                        "parallelism": f"peer-sharded x{world}" + (" (RCCL exchange path)" if sharded else ""),
                        **({"exchange": "slotted" if slot_cap else "exact", "slot_cap_records_per_rank": slot_cap,
                            "exchanged_bytes_per_step": (exch_all * REC / steps)} if sharded else {})}, **extra),
        # what the packets/s hides: the verdict mix of the timed offered packets (originals + clones)
        # and the rate of records that went through netem + HTB and were given a delivery time
        "scheduled_per_s": scheduled_all / el,
        "verdict_mix": {k: float(v) / tot_v for k, v in zip(abi.VERDICT_NAMES, verd_all)},
        "setup_s": setup_s,
        "roofline": {"bound": "hbm", "kernel": "k_sim_fused (dense generated windows, a fused dispatch's time divided by its "
                                               "windows) | k_sim (other dense steps) | k_sim_sparse + k_sim_multi + k_sim_list (sparse steps)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                     "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": per_launch, "carry_bytes": carry_w,
                     "frac_without_carry": frac_of(base), "queue_state_bytes_modeled": model_w,
                     "frac_modeled_restream": frac_of(base + model_w),
                     "kernel_ms_avg": sim_ms, "launches": n_launch, "timed_every_nth_window": timing_every,
                     "per": "window (one step of --window ticks; a fused dispatch counts each of its windows)"},
        "cpu_baseline": None,
    }
    if dv_ms > 0 and n_dv:
        # the delivery (K5) on its own stream: histogram scan (8 B count read, 8 B offset and 8 B
        # cursor written, 8 B cleared per destination, 8 B offsets re-read by the sort), then per
        # record 24 B read from the emit region + 24 B scattered + 24 B read + 24 B written in
        # destination order; per source its 4 B emit count and 8 B offset (local delivery).  A
        # record the simulate kernel wrote straight into its destination's bucket (sparse windows)
        # is only read from there and written in destination order: 48 B
        recs_w = scheduled / max(1, steps)
        bkt_w = min(recs_w, bkt / max(1, steps))
        dv_bytes = 96 * (recs_w - bkt_w) + 48 * bkt_w + 40 * n_dst_rank + 12 * peers
        dv_traffic, dv_src = load_pmc(workload, window, peers, lam, shapes, kind="delivery")
        dv_gbs = dv_bytes / (dv_ms * 1e-3) / 1e9
        res["roofline"]["delivery"] = {
            "kernel": "k_scan_* + k_local_scatter_ls / k_local_scatter (or k_dst_hist/k_dst_scatter) + k_dst_sort_bkt "
                      "(bucketed sparse windows) / k_dst_sort_flat / k_dst_sort_wide",
            "achieved": dv_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": dv_gbs / HBM_PEAK_GBS,
            "algorithmic_bytes_per_window": dv_bytes, "records_per_window": recs_w,
            "bucketed_records_per_window": bkt_w, "span_ms_avg": dv_ms,
            "windows": n_dv, "traffic": dv_traffic, "traffic_source": dv_src,
            "note": "span from the first delivery kernel to the sort on the delivery stream (HIP events), "
                    "including the time its kernels wait for CU slots beside the next simulate kernel"}
    if cpu is not None:
        res["cpu_baseline"] = cpu
        cpu["gpu_over_cpu"] = res["value"] / cpu["value"]
        cpu["timed_on"] = f"rank 0's host cores, in the same run (world size {world})"
        import shutil
        missing = [t for t in ("docker", "tc") if shutil.which(t) is None]
        # the reference's local:docker sidecar + netem path is timed only where it runs
        res["cpu_baseline"]["reference_docker_netem"] = (
            f"not available on this host ({', '.join(missing)} absent)" if missing else "present, not timed by bench.py")
    return res


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    decision = launch_decision(a.gpus, os.environ)
    if decision == "spawn":
        sys.exit(spawn_ranks(a.gpus, argv))
    if decision != "run":
        print(decision, file=sys.stderr)
        sys.exit(2)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.launch_check:
        # the host group is created exactly as a measured run creates it (gloo touches no GPU)
        dist = init_host_group(world)
        backend = dist.get_backend()
        dist.barrier()
        dist.destroy_process_group()
        line = json.dumps({"rank": rank, "world": world, "local_rank": local, "gpus": a.gpus,
                           "launched_by_bench": os.environ.get("TGSIM_BENCH_LAUNCHED") == "1",
                           "host_group": backend, "headline": headline_plan(a, world)})
        os.write(1, (line + "\n").encode())  # one write: the ranks share the pipe
        return
    # the one JSON line goes to the original stdout; everything else (RCCL's version banner, library
    # chatter) is sent to stderr so that the line stays the only thing on stdout
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    import torch

    torch.cuda.set_device(local)
    dist = None
    if world > 1 or a.sharded:
        dist = init_host_group(world)
    if a.workload == "bridge":
        res = run_bridge(a, world, rank, local, dist, want_cpu=not a.no_cpu)
    else:
        # storm (configs[2]: "10k instances, 1/2/4/8 GPUs"): the headline is --peers instances in
        # total, split over the ranks; the weak-scaling run (--peers per GPU) rides along at N > 1
        res = run_workload(a, a.workload, a.peers, a.steps, a.warmup, a.window, a.lam, world, rank, local, dist,
                           want_cpu=not a.no_cpu, split=a.workload == "storm")
        if a.workload == "storm" and world > 1:
            w = run_workload(a, "storm", a.peers, a.steps, a.warmup, a.window, a.lam, world, rank, local, dist,
                             want_cpu=False)
            if res is not None:
                res["weak_per_gpu"] = {k: w[k] for k in ("value", "unit", "ms_per_step", "steps", "scaling", "config",
                                                         "scheduled_per_s", "roofline")}
    if a.workload == "storm" and not a.no_1m:
        # the 1M-peer half of the metric: C4 gossip over 1M peers in total, split over the ranks
        g = run_workload(a, "gossip", a.gossip_1m_peers, 70, 0, 5000, a.lam, world, rank, local, dist,
                         want_cpu=not a.no_cpu, split=True)
        if res is not None:
            res["at_1M_peers"] = {k: g[k] for k in ("value", "unit", "ms_per_step", "steps", "config",
                                                    "scheduled_per_s", "verdict_mix", "setup_s", "roofline",
                                                    "cpu_baseline")}
            res["at_1M_peers"]["scaling"] = "strong (1M peers in total, split over the GPUs)"
    if a.workload == "storm" and not a.no_variants:
        # the rest of BASELINE.json's configs on the same line, each with its own roofline and CPU
        # baseline: the sub-capacity storm (C3's shapes at 1 Gbit/s below
        # capacity: the variant that exercises delay, HTB and delivery at rate) and C5's epochs
        from testground_amd.workloads import STORM_OPEN_LAMBDA
        keys = ("value", "unit", "ms_per_step", "steps", "warmup", "config", "scheduled_per_s", "verdict_mix",
                "setup_s", "roofline", "cpu_baseline")
        sub = run_workload(a, "storm", a.peers, 30, 3, 2000, STORM_OPEN_LAMBDA, world, rank, local, dist,
                           want_cpu=not a.no_cpu, split=True, shapes="open")
        # 30 timed epochs, not 10: ten ~1.1-ms epochs made a 12-ms timed region that one host stall
        # halved (9.7 against 17.3 G pkt/s, profiles/r05/epochs_steps/)
        ep = run_workload(a, "epochs", 100_000, 30, 3, 1000, 0.2, world, rank, local, dist,
                          want_cpu=not a.no_cpu, split=True)
        if res is not None:
            res["at_subcapacity"] = dict({k: sub[k] for k in keys},
                                         scaling="strong (10,000 instances in total, split over the GPUs)")
            res["at_epochs"] = dict({k: ep[k] for k in keys},
                                    scaling="strong (100,000 instances in total, split over the GPUs)")
    if res is not None:
        os.write(json_fd, (json.dumps(res) + "\n").encode())
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
