"""World-size-2 `gloo` run of the sharded step (testground_amd/shard.py) on CPU: each rank owns half
of the sources (an oracle shard), records are exchanged with all_to_all, and the result must equal
a single engine over all sources, step by step: verdicts per shard and deliveries per destination.
Device-generated workloads: C3 storm, C4 gossip (receipts feed the next window) and C5 epochs
(reshaping every epoch, barrier counters summed over the ranks with all_reduce)."""
import ctypes
import os
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from testground_amd import abi, workloads
from testground_amd.build import build_oracle
from testground_amd.engine import CABIEngine

N, STEPS, WINDOW, LAM = 200, 3, 1500, 0.5


def _oracle(n, **kw):
    lib = ctypes.CDLL(str(build_oracle()))
    abi.declare(lib, "tgo_")
    return CABIEngine(lib, "tgo_", n, **kw)


def _window(eng, workload, k, step, barrier=None):
    """Runs window k of `workload` on eng with the given step function (sharded or single)."""
    if workload == "storm":
        if k == 0:
            workloads.configure_storm(eng, N)
        eng.gen_storm(LAM, WINDOW)
        step(WINDOW)
    elif workload == "gossip":
        if k == 0:
            workloads.configure_gossip(eng, N)
            eng.gossip_init(n_floods=4, degree=8, msg_len=1024, start_gap_ticks=900, start_tick=0)
        w = workloads.gossip_window_ticks(eng)
        eng.gen_gossip(w)
        step(w)
    else:  # C5 epochs: reshaping + barrier reduced over the ranks
        if k == 0:
            workloads.configure_storm(eng, N)
        lo, hi = eng.shard
        workloads.run_epoch(eng, N, k, hi - lo, step=step, barrier=barrier)


def _kw(workload):
    return dict(lookahead_ns=workloads.GOSSIP_MIN_LAT) if workload == "gossip" else {}


def _rank(rank, world, port, outdir, workload="storm", steps=STEPS):
    import torch.distributed as dist

    from testground_amd.shard import ShardedStepper, shard_bounds

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = shard_bounds(N, world)
    eng = _oracle(N, shard=(b[rank], b[rank + 1]), **_kw(workload))
    st = ShardedStepper(eng, b, device="cpu")
    for k in range(steps):
        _window(eng, workload, k, st.step, st.barrier)
        np.save(os.path.join(outdir, f"v{rank}_{k}.npy"), eng.verdicts())
        np.save(os.path.join(outdir, f"d{rank}_{k}.npy"), eng.drain())
    dist.destroy_process_group()


@pytest.mark.parametrize("workload,steps,min_pkts",
                         [("storm", STEPS, 10_000), ("gossip", 16, 100), ("epochs", 4, 10_000)])
def test_two_rank_gloo_equals_single_engine(workload, steps, min_pkts):
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rank, args=(world, 29600 + os.getpid() % 300 + 7 * ["storm", "gossip", "epochs"].index(workload), d,
                                        workload, steps), nprocs=world, start_method="spawn", join=True)
        ref = _oracle(N, **_kw(workload))
        for k in range(steps):
            _window(ref, workload, k, ref.step)
            v = np.concatenate([np.load(os.path.join(d, f"v{r}_{k}.npy")) for r in range(world)])
            dl = np.concatenate([np.load(os.path.join(d, f"d{r}_{k}.npy")) for r in range(world)])
            vr, dr = ref.verdicts(), ref.drain()
            assert len(v) == len(vr) and (v == vr).all(), f"step {k}: verdicts"
            total = total + len(v) if k else len(v)
            assert len(dl) == len(dr) and (dl == dr).all(), f"step {k}: deliveries"
        assert total > min_pkts


def _rank_pipelined(rank, world, port, outdir, steps):
    import torch.distributed as dist

    from testground_amd.shard import ShardedStepper, shard_bounds

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = shard_bounds(N, world)
    eng = _oracle(N, shard=(b[rank], b[rank + 1]))
    workloads.configure_storm(eng, N)
    for _ in range(steps):  # every window pre-generated: the stepper simulates one step ahead
        eng.gen_storm(LAM, WINDOW)
    ShardedStepper(eng, b, device="cpu").run(steps, WINDOW)
    np.save(os.path.join(outdir, f"d{rank}.npy"), eng.drain())
    np.save(os.path.join(outdir, f"s{rank}.npy"), np.array([eng.stats()["offered"], eng.stats()["scheduled"]]))
    dist.destroy_process_group()


def test_two_rank_pipelined_run_equals_single_engine():
    world, steps = 2, 4
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rank_pipelined, args=(world, 29950 + os.getpid() % 40, d, steps), nprocs=world,
                           start_method="spawn", join=True)
        ref = _oracle(N)
        workloads.configure_storm(ref, N)
        per_step = []
        for _ in range(steps):
            ref.gen_storm(LAM, WINDOW)
            ref.step(WINDOW)
            per_step.append(ref.drain())
        dr = np.concatenate(per_step)
        s = sum(np.load(os.path.join(d, f"s{r}.npy")) for r in range(world))
        st = ref.stats()
        assert list(s) == [st["offered"], st["scheduled"]]
        # each rank's drain is its destinations' deliveries, step after step
        lo_hi = [(0, N // 2), (N // 2, N)]
        for r, (lo, hi) in enumerate(lo_hi):
            dl = np.load(os.path.join(d, f"d{r}.npy"))
            want = np.concatenate([x[(x["dst"] >= lo) & (x["dst"] < hi)] for x in per_step])
            assert len(dl) == len(want) and (dl == want).all(), f"rank {r}"
        assert len(dr) > 5_000
