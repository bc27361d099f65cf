"""Benchmark: simulated packets/sec of the network.Config enforcement path (BASELINE.json metric).

Default workload (BASELINE.json configs[2]): storm-style random all-to-all traffic
over 10,000 instances per GPU, heterogeneous LinkShape (latency/jitter/loss/dup/corrupt/reorder/
bandwidth), Poisson(0.5) packets per instance per 1 µs tick.  One step = one pass of the hot path
over one window of `--window` ticks of offered traffic that is already resident in HBM (generated
on the device before the timed region): filter -> netem -> HTB (k_sim), routing by destination
shard, RCCL all-to-all (N > 1), per-destination delivery sort.

`--workload gossip` (C4, BASELINE.json configs[3]): flood of 64 messages over --peers instances per
GPU (125,000 per GPU = 1M at 8 GPUs), degree 8, 1 KiB, L~U[5,50] ms, loss 1 %.  A step is one 5 ms
window: forwards of the previous window's receipts generated on the device, then the hot path.
`--workload epochs` (C5, configs[4]): 100,000 instances per GPU, C3 shapes and traffic at
lambda 0.2, 1,000-tick epochs; a step reshapes 10 % of the instances (batched ConfigureNetwork),
runs the epoch and passes the `epoch-k` barrier (counters summed over ranks).

N = 1 runs directly; N > 1 is launched by torch.distributed.run, one rank per GPU, each rank owning
--peers instances (weak scaling), cross-shard deliveries exchanged with all_to_all_single (RCCL).
"""
import argparse
import ctypes
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "simulated packets/sec (whole node) at 10k & 1M peers; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

# Algorithmic HBM bytes of k_sim: per offered packet 16 B record read + 1 B verdict
# write; per scheduled record 24 B delivery write; per source 64 B params + 32 B state read + 32 B
# state write + 16 B CSR offsets + 4 B emit count; plus the netem queue state each source carries
# across steps (16 B per queued item, 8 B per departing item, loaded at step start and stored at
# step end: the engine's queue_state_bytes counter).
B_OFFERED, B_SCHEDULED, B_SOURCE = 17, 24, 148


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None, help="timed steps (default: storm 30, epochs 10, gossip 70 windows)")
    p.add_argument("--warmup", type=int, default=None, help="untimed steps (default: 3; gossip: 0)")
    p.add_argument("--workload", default="storm", choices=["storm", "gossip", "epochs"])
    p.add_argument("--peers", type=int, default=0,
                   help="instances per GPU (default: storm 10,000; gossip 125,000; epochs 100,000)")
    p.add_argument("--floods", type=int, default=64, help="gossip: flood messages")
    p.add_argument("--flood-gap", type=int, default=1000, help="gossip: ticks between flood starts")
    p.add_argument("--lam", type=float, default=0.5)
    p.add_argument("--window", type=int, default=2000, help="ticks (1 us) per step")
    p.add_argument("--settle-ms", type=float, default=120.0,
                   help="untimed simulated time before warm-up so every netem queue is in its sustained "
                        "storm state (> max latency + jitter = 110 ms); queues start empty otherwise")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=min(16, os.cpu_count() or 1),
                   help="threads of the all-core CPU oracle leg (the GPU box's CPU share is 16)")
    p.add_argument("--queue-limit", type=int, default=0, help="netem limit (0 = netlink default 1000)")
    p.add_argument("--shapes", default="storm", choices=["storm", "fixed"],
                   help="storm: C3 heterogeneous shapes; fixed: L=5 ms, no jitter/loss/reorder (probe)")
    p.add_argument("--sharded", action="store_true",
                   help="use the peer-sharded step (RCCL exchange) even at one rank, to time the N>1 path")
    p.add_argument("--exact-exchange", action="store_true",
                   help="sharded storm: exchange exact record counts every step instead of fixed-size chunks")
    a = p.parse_args()
    if not a.peers:
        a.peers = {"storm": 10_000, "gossip": 125_000, "epochs": 100_000}[a.workload]
    if a.workload == "epochs":
        a.lam, a.window = 0.2, 1000
    if a.workload == "gossip":
        a.window = 5000
    if a.steps is None:
        a.steps = {"gossip": 70, "epochs": 10}.get(a.workload, 30)  # storm: amortizes the pipeline fill and drain
    if a.warmup is None:
        a.warmup = 0 if a.workload == "gossip" else 3
    return a


def cpu_baseline(a, peers_total):
    """The CPU oracle (a 'port' of the reference semantics) timed on this host, single thread, on a
    bounded sample of the same workload."""
    from testground_amd import abi, workloads
    from testground_amd.build import build_oracle
    from testground_amd.engine import CABIEngine

    lib = ctypes.CDLL(str(build_oracle()))
    abi.declare(lib, "tgo_")
    busy, steps = 0.0, 0
    if a.workload == "gossip":  # closed loop: needs every peer, so the sample is a smaller flood
        n = min(peers_total, 20_000)
        e = CABIEngine(lib, "tgo_", n, lookahead_ns=workloads.GOSSIP_MIN_LAT)
        workloads.configure_gossip(e, n)
        e.gossip_init(n_floods=a.floods, degree=8, msg_len=1024, start_gap_ticks=a.flood_gap, start_tick=0)
        while busy < a.cpu_seconds and steps < 400:
            t0 = time.perf_counter()
            e.gen_gossip(a.window)
            e.step(a.window)
            busy += time.perf_counter() - t0
            steps += 1
            e.drain()
        pkts = e.stats()["offered"]
        sample = (f"oracle/tgoracle.c, the same flood over {n} instances ({a.floods} floods, degree 8), "
                  f"{steps} windows of {a.window} ticks incl. forward generation, {pkts} packets, {busy:.1f} s")
    else:
        sample_src = min(1000, peers_total)

        def leg(lo, hi, seconds):
            """One oracle shard [lo, hi) of the same workload stepped for ~seconds of step time."""
            e = CABIEngine(lib, "tgo_", peers_total, shard=(lo, hi))
            workloads.configure_storm(e, peers_total)
            busy, steps = 0.0, 0
            while busy < seconds:
                if a.workload == "epochs" and steps:
                    r0 = time.perf_counter()
                    workloads.epoch_reshape(e, peers_total, steps)
                    busy += time.perf_counter() - r0
                e.gen_storm(a.lam, a.window)
                t0 = time.perf_counter()
                e.step(a.window)
                busy += time.perf_counter() - t0
                steps += 1
                e.drain()
            return e.stats()["offered"], busy, steps

        pkts, busy, steps = leg(0, sample_src, a.cpu_seconds)
        sample = (f"oracle/tgoracle.c, sources 0..{sample_src - 1} of the {peers_total}-instance {a.workload} "
                  f"workload, lambda={a.lam}, {steps} windows of {a.window} ticks, {pkts} packets, {busy:.1f} s")
        if a.cpu_threads > 1:  # all-core leg: one oracle shard per thread (ctypes drops the GIL)
            from concurrent.futures import ThreadPoolExecutor

            t = a.cpu_threads
            per = max(1, min(sample_src, peers_total // t))
            w0 = time.perf_counter()
            with ThreadPoolExecutor(t) as ex:
                res = list(ex.map(lambda k: leg(k * per, (k + 1) * per, a.cpu_seconds / 2), range(t)))
            wall = time.perf_counter() - w0
            # each thread's packets over its own stepping time; the sum is the all-core rate
            rate = sum(p / b for p, b, _ in res)
            return {"value": rate, "unit": "packets/s", "cores": t, "kind": "port",
                    "sample": (f"oracle/tgoracle.c, {t} threads, thread k steps sources "
                               f"[{per}k, {per}(k+1)) of the {peers_total}-instance {a.workload} workload "
                               f"(lambda={a.lam}, windows of {a.window} ticks) for ~{a.cpu_seconds / 2:.0f} s; "
                               f"{sum(p for p, _, _ in res)} packets, {wall:.1f} s wall"),
                    "single_thread": {"value": pkts / busy, "cores": 1, "sample": sample}}
    return {"value": pkts / busy, "unit": "packets/s", "cores": 1, "kind": "port", "sample": sample}


def load_pmc(a):
    f = ROOT / "profiles" / ("pmc_k_sim.json" if a.workload == "storm" else f"pmc_k_sim_{a.workload}.json")
    if not f.exists():
        return None
    try:
        pmc = json.loads(f.read_text())
    except Exception:
        return None
    if pmc.get("window") == a.window and pmc.get("peers") == a.peers and pmc.get("lam", a.lam) == a.lam:
        return pmc.get("hbm_bytes_per_launch")
    return None


WORKLOAD_NAMES = {
    "storm": "C3 storm: random all-to-all, heterogeneous LinkShape (BASELINE.json configs[2])",
    "gossip": "C4 gossip flood: degree 8, 1 KiB, L~U[5,50] ms, loss 1 % (BASELINE.json configs[3])",
    "epochs": "C5 epochs: C3 traffic at lambda 0.2, 10 % reshaped per 1,000-tick epoch, barrier per epoch "
              "(BASELINE.json configs[4])",
}


def main():
    a = parse()
    # the one JSON line goes to the original stdout; everything else (RCCL's version banner, library
    # chatter) is sent to stderr so that the line stays the only thing on stdout
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch

    from testground_amd import abi, workloads
    from testground_amd.engine import Engine
    from testground_amd.network import configs_array

    torch.cuda.set_device(local)
    dist = None
    sharded = world > 1 or a.sharded
    if sharded:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        import torch.distributed as dist
        from testground_amd.shard import init_rccl
        init_rccl(torch.device("cuda", local))
    peers_total = a.peers * world
    lo, hi = rank * a.peers, (rank + 1) * a.peers
    kw = dict(lookahead_ns=workloads.GOSSIP_MIN_LAT) if a.workload == "gossip" else {}
    eng = Engine(peers_total, shard=(lo, hi), device=local, flags=abi.OPT_DISCARD_DELIVERIES,
                 queue_limit=a.queue_limit, **kw)
    if a.workload == "gossip":
        workloads.configure_gossip(eng, peers_total)
    elif a.shapes == "storm":
        workloads.configure_storm(eng, peers_total)
    else:
        eng.configure_batch(np.arange(peers_total), configs_array(np.full(peers_total, 5_000_000), routing_policy=2))
    bounds = [r * a.peers for r in range(world)] + [peers_total]
    stepper = None
    if sharded:
        from testground_amd.shard import ShardedStepper
        stepper = ShardedStepper(eng, bounds, device=f"cuda:{local}")
    step = eng.step if stepper is None else stepper.step
    barrier = None if stepper is None else stepper.barrier
    epoch = [0]

    def one_step():
        if a.workload == "gossip":
            eng.gen_gossip(a.window)
            step(a.window)
        elif a.workload == "epochs":  # traffic pre-generated; reshape + epoch + barrier
            k = epoch[0]
            if stepper is None:
                if k:
                    workloads.epoch_reshape(eng, peers_total, k)
                step(a.window)  # asynchronous: the next reshape's host work overlaps this k_sim
            else:
                # the sharded step waits for its records, so epoch k+1's ConfigureNetwork calls
                # are staged on the host while epoch k simulates (epoch k's were staged during
                # epoch k-1); staged configs take effect at the next launch, after the barrier below
                stepper.step(a.window, between=lambda: workloads.epoch_reshape(eng, peers_total, k + 1))
            state, rnd = workloads.epoch_state(k)
            eng.signal(state, a.peers)
            ok = barrier(state, rnd * peers_total) if barrier else eng.barrier_poll(state, rnd * peers_total)
            if not ok:
                raise RuntimeError(f"barrier epoch-{k} did not release")
            epoch[0] += 1
        else:
            step(a.window)

    if a.workload == "gossip":
        # two empty windows, untimed: the step's buffers (two emit regions, sized for a full netem
        # queue per source: ~64 GB at 1M peers) are allocated and first touched here, not in the
        # timed flood; the floods start at the next window
        for _ in range(2):
            step(a.window)
        eng.gossip_init(n_floods=a.floods, degree=8, msg_len=1024, start_gap_ticks=a.flood_gap)
        settle = 0  # a flood is a transient by nature: the timed windows cover it from the start
    else:
        settle = int(a.settle_ms * 1000 / a.window + 0.999)
        for _ in range(settle):  # untimed: bring every netem queue to its sustained state
            eng.gen_storm(a.lam, a.window)
            one_step()
        for _ in range(a.warmup + a.steps):
            eng.gen_storm(a.lam, a.window)  # inputs resident in HBM before the timed region
    def run_steps(n):
        if stepper is not None and a.workload == "storm":  # pre-generated: simulate one step ahead
            stepper.run(n, a.window)
        else:
            for _ in range(n):
                one_step()

    if stepper is not None and a.workload == "storm" and not a.exact_exchange:
        # fixed-size exchange for the pipelined run: per-rank chunks sized from the largest count
        # the settle steps exchanged (max over ranks) plus a margin; an overflow fails the run
        m = torch.tensor([stepper.max_count], dtype=torch.int64, device=f"cuda:{local}")
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        stepper.slot_cap = int(int(m.item()) * 1.25) + 4096
    run_steps(a.warmup)
    eng.drain()
    s0 = eng.stats()
    eng.sim_kernel_ms(reset=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(a.steps)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    s1 = eng.stats()
    offered = s1["offered"] - s0["offered"]
    scheduled = s1["scheduled"] - s0["scheduled"]
    sim_ms, n_launch = eng.sim_kernel_ms()
    if dist:
        t = torch.tensor([el, float(offered)], dtype=torch.float64, device="cuda")
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        el = float(mx[0])
        offered_all = float(t[1])
    else:
        offered_all = float(offered)
    extra = {}
    if a.workload == "gossip":
        reached = eng.gossip_reached()
        if dist:
            r = torch.as_tensor(reached.astype(np.int64), device="cuda")
            dist.all_reduce(r)
            reached = r.cpu().numpy()
        extra = {"floods": a.floods, "flood_gap_ticks": a.flood_gap,
                 "reached_min_frac": float(reached.min()) / peers_total,
                 "sim_ms_covered": (a.warmup + a.steps) * a.window / 1000}
    if rank != 0:
        dist.destroy_process_group()
        return
    qbytes = s1["queue_state_bytes"] - s0["queue_state_bytes"]
    per_launch = (B_OFFERED * offered + B_SCHEDULED * scheduled + qbytes) / max(1, a.steps) + B_SOURCE * a.peers
    achieved = per_launch / (sim_ms * 1e-3) / 1e9 if sim_ms > 0 else None
    res = {
        "metric": METRIC,
        "value": offered_all / el,
        "unit": "packets/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": el * 1e3 / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32/u64 integer",
        "data": f"synthetic (device-generated {a.workload} traffic, Philox-keyed)",
        "config": dict({"workload": WORKLOAD_NAMES[a.workload],
                        "peers_per_gpu": a.peers, "peers_total": peers_total, "lambda_per_tick": a.lam,
                        "tick_ns": 1000, "window_ticks": a.window, "settle_sim_ms": settle * a.window / 1000,
                        "shapes": a.shapes if a.workload == "storm" else a.workload,
                        "queue_limit": a.queue_limit or 1000, "packets_per_step": offered_all / a.steps,
                        "parallelism": f"peer-sharded x{world}" + (" (RCCL exchange path)" if sharded else ""),
                        **({"exchange": "slotted" if stepper.slot_cap else "exact",
                            "slot_cap_records": stepper.slot_cap} if stepper is not None else {})}, **extra),
        "roofline": {"bound": "hbm", "kernel": "k_sim", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                     "traffic": load_pmc(a), "algorithmic_bytes_per_launch": per_launch,
                     "kernel_ms_avg": sim_ms, "launches": n_launch},
        "cpu_baseline": None,
    }
    if world == 1 and not a.no_cpu:
        res["cpu_baseline"] = cpu_baseline(a, peers_total)
        res["cpu_baseline"]["gpu_over_cpu"] = res["value"] / res["cpu_baseline"]["value"]
        import shutil
        missing = [t for t in ("docker", "tc") if shutil.which(t) is None]
        # the reference's local:docker sidecar + netem path is timed only where it runs
        res["cpu_baseline"]["reference_docker_netem"] = (
            f"not available on this host ({', '.join(missing)} absent)" if missing else "present, not timed by bench.py")
    os.write(json_fd, (json.dumps(res) + "\n").encode())
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
