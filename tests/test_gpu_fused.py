"""Fused windows (tgsim_step_n, k_sim_fused): several windows in one launch, a source's window k + 1
starting as soon as its window k has handed its netem queue, departure ring and state over (sc1
write-through stores, a per-source completion word, sc1 loads).  The bar is the same as for
tgsim_step: bit-exact against the CPU oracle, and bit-exact against the unfused engine at the full
C3 size, where the hand-off is exercised under load on every source."""
import numpy as np
import pytest

from testground_amd import workloads as wl
from testground_amd.engine import Engine

from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

try:  # torch ships its own HIP runtime: let it initialise first when both share a process
    import torch

    if torch.cuda.is_available():
        torch.cuda.init()
except ImportError:  # pragma: no cover
    torch = None


def _fused(e):
    return int(e._fn("debug_fused_windows")(e._h))


def test_step_n_equals_oracle(make_oracle, monkeypatch):
    """Storm windows through step_n (10, 3 and 5 per call: fused 4 + 4 + 2, 3, 4 + 1) against the oracle stepping one by one, with
    a reshaping between two calls (configuration applies from the next group's first window)."""
    n, ticks = 600, 300
    monkeypatch.setenv("TGSIM_FUSE", "4")  # groups of at most four windows (read at engine creation)
    g, c = Engine(n), make_oracle(n)
    for e in (g, c):
        wl.configure_storm(e, n)
    for part, k in enumerate((10, 3, 5)):
        if part == 2:
            for e in (g, c):
                wl.epoch_reshape(e, n, 1)
        for e in (g, c):
            for _ in range(k):
                e.gen_storm(0.5, ticks)
            e.step_n(ticks, k)
        assert_same(g, c, f"step_n part {part}")
    assert _fused(g) == 17, "4 + 4 + 2, 3, then 4 + one window alone (a group needs two)"


def test_step_n_full_storm_equals_step():
    """C3 at full size (10,000 sources, 2,000-tick windows): 8 fused windows equal 8 tgsim_step
    calls bit for bit (verdicts of the last window, every delivery, the statistics)."""
    n, ticks = 10_000, 2000
    a, b = Engine(n), Engine(n)
    for e in (a, b):
        wl.configure_storm(e, n)
        for _ in range(3):  # queues fill: the hand-off then carries ~1,000 items per source
            e.gen_storm(0.5, ticks)
            e.step(ticks)
        e.drain()
        for _ in range(8):
            e.gen_storm(0.5, ticks)
    for _ in range(8):
        a.step(ticks)
    b.step_n(ticks, 8)
    assert _fused(b) == 8 and _fused(a) == 0
    v, d = assert_same(b, a, "fused vs unfused")
    assert len(v) > 9_000_000 and len(d) > 1_000_000
    assert b.stats()["queue_state_bytes"] > 8 * 100_000_000


def test_step_n_falls_back_when_not_fusable(make_oracle):
    """Host-submitted packets and sparse windows take the per-window path, with the same results."""
    n, ticks = 300, 400
    g, c = Engine(n), make_oracle(n)
    for e in (g, c):
        wl.configure_storm(e, n)
        for _ in range(2):
            e.gen_storm(0.05, ticks)  # 20 packets per source: sparse windows
        e.step_n(ticks, 2)
    assert _fused(g) == 0
    assert_same(g, c, "sparse windows through step_n")


def test_step_n_after_sparse_fifo_windows(make_oracle):
    """FIFO sources (fixed latency; no jitter, reordering or duplication) in sparse windows: the
    sparse kernel serves the sorted queue's prefix and appends behind its tail in place, moving the
    queue's head slot instead of the items.  Dense windows after them run fused, whose bounded loads
    read every queue from slot 0 (k_unrotate compacts them first).  Every window equals the oracle."""
    from testground_amd.network import configs_array

    n = 300
    g, c = Engine(n), make_oracle(n)
    for e in (g, c):
        e.configure_batch(np.arange(n), configs_array(np.full(n, 3_000_000), routing_policy=2))
    for k in range(6):  # ~20 packets per source and window, ~60 queued: sparse, FIFO
        for e in (g, c):
            e.gen_storm(0.02, 1000)
            e.step(1000)
        assert_same(g, c, f"sparse FIFO window {k}")
    model = g.stats()["queue_state_bytes"]
    # (with ~60 queued items the first chunk is all of a queue: what stays in place is the store)
    assert g.carry_bytes() < 0.8 * model, "the FIFO path left the queues in place"
    for e in (g, c):
        for _ in range(4):
            e.gen_storm(0.5, 400)  # 200 packets per source: dense, fused
        e.step_n(400, 4)
    assert _fused(g) == 4
    assert_same(g, c, "fused windows after in-place queues")


def test_three_shards_fused_slotted_exchange_equal_one():
    """The fused slotted layout (tgsim_step_sim_launch_slotted_n: rank-major chunks, window-minor;
    tgsim_deliver_slotted_n_async) over three shards on one GPU, the chunks swapped by hand as the
    fixed-size all-to-all would: three fused windows deliver exactly what one engine delivers over
    three tgsim_step calls, window after window."""
    import torch

    n, bounds, ticks, g = 600, [0, 150, 420, 600], 400, 3
    ref = Engine(n)
    shards = [Engine(n, shard=(bounds[r], bounds[r + 1])) for r in range(3)]
    for e in [ref] + shards:
        wl.configure_storm(e, n)
        for _ in range(g):
            e.gen_storm(0.5, ticks)
    want = []
    for _ in range(g):
        ref.step(ticks)
        want.append(ref.drain())
    want = np.concatenate(want)
    cap = 40_000
    chunk = (cap + 1) * 24
    bufs = []
    for r, s in enumerate(shards):
        buf = torch.zeros(3 * g * chunk, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        s.step_sim_launch_slotted_n(ticks, g, bounds, buf.data_ptr(), cap)
        s.step_sim_release()
        s.sync()
        assert _fused(s) == g
        bufs.append(buf)
    for k, s in enumerate(shards):  # rank k receives chunks [k * g, (k + 1) * g) of every sender
        inbound = torch.cat([b[k * g * chunk:(k + 1) * g * chunk] for b in bufs])
        torch.cuda.synchronize()
        s.deliver_slotted_n_async(inbound.data_ptr(), 3, g, cap)
        s.sync()
    # each shard's drain is its destinations' deliveries window after window; the single engine's is
    # every destination's, window after window
    got = [s.drain() for s in shards]
    for r in range(3):
        lo, hi = bounds[r], bounds[r + 1]
        mine = want[(want["dst"] >= lo) & (want["dst"] < hi)]
        assert len(got[r]) == len(mine) > 1000
        assert (got[r] == mine).all()
    s_ref = ref.stats()
    tot = [s.stats() for s in shards]
    assert sum(t["offered"] for t in tot) == s_ref["offered"]
    assert sum(t["scheduled"] for t in tot) == s_ref["scheduled"]


@pytest.mark.parametrize("exchange", ["engine", "torch"])
def test_stepper_fused_slotted_run_equals_step(exchange):
    """Sharded run(fuse=4) at one rank, through the engine's own exchange (tgsim_comm_run) and the
    torch.distributed one: groups of four windows per launch and per exchange, the same deliveries
    and statistics as the single-engine steps."""
    import os

    import torch
    import torch.distributed as dist

    from testground_amd.shard import CommStepper, ShardedStepper, init_rccl

    torch.cuda.init()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29534")
    init_rccl(torch.device("cuda", 0), rank=0, world_size=1)
    try:
        n, steps = 2000, 10
        ref, sh = Engine(n), Engine(n)
        for e in (ref, sh):
            wl.configure_storm(e, n)
        for _ in range(steps):
            sh.gen_storm(0.5, 1000)
        cls = CommStepper if exchange == "engine" else ShardedStepper
        st = cls(sh, [0, n], device="cuda:0", slot_cap=400_000)
        assert st.run(steps, 1000, fuse=4) == -1
        assert _fused(sh) == steps  # 4 + 4 + 2
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
    finally:
        dist.destroy_process_group()
