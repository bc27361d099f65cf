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
