"""a routed step asks tgsim_sim_capacity for the next window's emit layout before
it launches the window, and the sparse-or-dense choice that call makes is kept for the launch.  The
kept choice must advance the dense streak exactly as a fresh one does, so that a run pushed to the
dense kernel by deferrals (here: correlated draws, which k_sim_sparse always hands to k_sim_list)
still re-measures the sparse kernels every 64th window.  The windows stay equal to the oracle's."""
import numpy as np
import pytest

from testground_amd import abi
from testground_amd import network as nw
from testground_amd.engine import Engine

pytestmark = pytest.mark.gpu

try:  # torch ships its own HIP runtime: let it initialise first when both share a process
    import torch

    if torch.cuda.is_available():
        torch.cuda.init()
except ImportError:  # pragma: no cover
    torch = None


def test_capacity_query_keeps_the_sparse_remeasure(make_oracle):
    n, window, lam, steps = 2000, 2000, 0.002, 140  # ~4 packets per source and window: sparse
    g = Engine(n, flags=abi.OPT_DISCARD_DELIVERIES)
    c = make_oracle(n, flags=abi.OPT_DISCARD_DELIVERIES)
    cfg = nw.configs_array(np.full(n, 5 * nw.Millisecond), np.full(n, 2 * nw.Millisecond), np.full(n, 1 << 30),
                           loss=1.0, duplicate=2.0)
    cfg["shape"]["duplicate_corr"] = 25.0  # correlated duplicate draws: every busy source is deferred
    g.configure_batch(np.arange(n), cfg)
    c.configure_batch(np.arange(n), cfg)
    for _ in range(steps):
        for e in (g, c):
            e.gen_storm(lam, window)
            assert e.sim_capacity() > 0
            e.step(window)
    sparse = int(g._fn("debug_sparse_windows")(g._h))
    # dense after the first deferrals, and back to the sparse kernels at least once per 64 windows
    assert 3 <= sparse <= 20, sparse
    assert g.stats() == c.stats()
