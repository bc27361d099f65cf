"""The sharded step on one GPU with a world of one rank, against the single-engine step: identical
verdicts and deliveries, open loop (storm) and closed loop (gossip, whose receipts feed the next
window).  Every test runs the exchanges: the engine's own (CommStepper over tgsim_comm_*: its RCCL
communicator, exchange stream and buffers, what bench.py and a Go host use; at one rank the
single-shard step, or with TGSIM_COMM_ROUTE1=1 the routed path) and the torch.distributed one over
the split-phase ABI (ShardedStepper)."""
import os

import numpy as np
import pytest

from testground_amd import workloads as wl
from testground_amd.engine import Engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl():
    import torch
    import torch.distributed as dist

    torch.cuda.init()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    from testground_amd.shard import init_rccl

    init_rccl(torch.device("cuda", 0), rank=0, world_size=1)
    yield dist
    dist.destroy_process_group()


class RoutedCommStepper:
    """CommStepper at one rank with TGSIM_COMM_ROUTE1=1: the routed N > 1 path (routing kernels, the
    delivery reading the routed records in place) instead of the single-shard step."""

    def __new__(cls, *args, **kw):
        from testground_amd.shard import CommStepper

        os.environ["TGSIM_COMM_ROUTE1"] = "1"  # read by tgsim_comm_init
        try:
            return CommStepper(*args, **kw)
        finally:
            del os.environ["TGSIM_COMM_ROUTE1"]


@pytest.fixture(params=["engine", "engine-routed", "torch"])
def Stepper(request, rccl):
    from testground_amd.shard import CommStepper, ShardedStepper

    return {"engine": CommStepper, "engine-routed": RoutedCommStepper, "torch": ShardedStepper}[request.param]


def test_stepper_storm_equals_step(Stepper):

    n = 300
    ref, sh = Engine(n), Engine(n)
    for e in (ref, sh):
        wl.configure_storm(e, n)
    st = Stepper(sh, [0, n], device="cuda:0")
    for k in range(6):
        ref.gen_storm(0.5, 1500)
        sh.gen_storm(0.5, 1500)
        ref.step(1500)
        st.step(1500)
        assert (sh.verdicts() == ref.verdicts()).all(), f"step {k}"
        d_sh, d_ref = sh.drain(), ref.drain()
        assert len(d_sh) == len(d_ref) and (d_sh == d_ref).all(), f"step {k}"


def test_stepper_gossip_equals_step(Stepper):

    n = 1500
    ref = Engine(n, lookahead_ns=wl.GOSSIP_MIN_LAT)
    sh = Engine(n, lookahead_ns=wl.GOSSIP_MIN_LAT)
    for e in (ref, sh):
        wl.configure_gossip(e, n)
        e.gossip_init(n_floods=8, degree=8, msg_len=1024, start_gap_ticks=300, start_tick=0)
    st = Stepper(sh, [0, n], device="cuda:0")
    w = wl.gossip_window_ticks(ref)
    for k in range(25):
        ref.gen_gossip(w)
        ref.step(w)
        sh.gen_gossip(w)
        st.step(w)
        d_sh, d_ref = sh.drain(), ref.drain()
        assert len(d_sh) == len(d_ref) and (d_sh == d_ref).all(), f"window {k}"
    assert (sh.gossip_reached() == ref.gossip_reached()).all()


def test_stepper_pipelined_run_equals_step(Stepper):
    """run(): step k+1's k_sim launched before step k's exchange and delivery."""

    n, steps = 2000, 8
    ref, sh = Engine(n), Engine(n)
    for e in (ref, sh):
        wl.configure_storm(e, n)
    for _ in range(steps):
        sh.gen_storm(0.5, 1000)
    Stepper(sh, [0, n], device="cuda:0").run(steps, 1000)
    want = []
    for _ in range(steps):
        ref.gen_storm(0.5, 1000)
        ref.step(1000)
        want.append(ref.drain())
    want = np.concatenate(want)
    got = sh.drain()
    assert len(got) == len(want) > 10_000 and (got == want).all()
    s, r = sh.stats(), ref.stats()
    assert (s["offered"], s["scheduled"], s["by_verdict"]) == (r["offered"], r["scheduled"], r["by_verdict"])


def test_stepper_epochs_staged_reshape_equals_step(Stepper):
    """C5 through the stepper as bench.py runs it: epoch k+1's reshape staged on the host while
    epoch k simulates (between=), the barrier summed on the host group; the same verdicts,
    deliveries and barrier releases as reshaping before each single-engine step."""

    n, ticks = 3000, 800
    ref, sh = Engine(n), Engine(n)
    for e in (ref, sh):
        wl.configure_storm(e, n)
    st = Stepper(sh, [0, n], device="cuda:0")
    for k in range(5):
        if k:
            wl.epoch_reshape(ref, n, k)
        ref.gen_storm(0.2, ticks)
        sh.gen_storm(0.2, ticks)
        ref.step(ticks)
        st.step(ticks, between=lambda: wl.epoch_reshape(sh, n, k + 1))
        state, rnd = wl.epoch_state(k)
        ref.signal(state, n)
        sh.signal(state, n)
        assert ref.barrier_poll(state, rnd * n) and st.barrier(state, rnd * n)
        assert not st.barrier(state, rnd * n + 1)
        assert (sh.verdicts() == ref.verdicts()).all(), f"epoch {k}"
        d_sh, d_ref = sh.drain(), ref.drain()
        assert len(d_sh) == len(d_ref) > 0 and (d_sh == d_ref).all(), f"epoch {k}"


def test_stepper_slotted_run_equals_step(Stepper):
    """run() with fixed-size exchange chunks (slot_cap): the host only enqueues, never reads a count;
    the same deliveries and statistics as the single-engine steps."""

    n, steps = 2000, 8
    ref, sh = Engine(n), Engine(n)
    for e in (ref, sh):
        wl.configure_storm(e, n)
    for _ in range(steps):
        sh.gen_storm(0.5, 1000)
    st = Stepper(sh, [0, n], device="cuda:0", slot_cap=400_000)
    assert st.run(steps, 1000) == -1
    want = []
    for _ in range(steps):
        ref.gen_storm(0.5, 1000)
        ref.step(1000)
        want.append(ref.drain())
    want = np.concatenate(want)
    got = sh.drain()
    assert len(got) == len(want) > 10_000 and (got == want).all()
    s, r = sh.stats(), ref.stats()
    assert (s["offered"], s["scheduled"], s["by_verdict"]) == (r["offered"], r["scheduled"], r["by_verdict"])


def test_stepper_slotted_overflow_fails(Stepper):
    """A chunk too small for a step's records is an error (-ENOSPC), never a silent loss.  At one
    rank the engine's own exchange routes nothing (tgsim_comm_run is the single-shard tgsim_step_n),
    so no chunk can overflow there: the run equals the single engine instead."""
    from testground_amd.engine import EngineError
    from testground_amd.shard import CommStepper

    n = 500
    sh, ref = Engine(n), Engine(n)
    for e in (sh, ref):
        wl.configure_storm(e, n)
        for _ in range(3):
            e.gen_storm(0.5, 1000)
    if Stepper is CommStepper:  # (RoutedCommStepper routes, and overflows below)
        Stepper(sh, [0, n], device="cuda:0", slot_cap=16).run(3, 1000)
        ref.step_n(1000, 3)
        got, want = sh.drain(), ref.drain()
        assert len(got) == len(want) > 1000 and (got == want).all()
        assert sh.comm_info()["exchanged_records"] == 0
        return
    with pytest.raises(EngineError, match="slot capacity"):
        Stepper(sh, [0, n], device="cuda:0", slot_cap=16).run(3, 1000)
        sh.sync()
