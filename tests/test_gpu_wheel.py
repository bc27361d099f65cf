"""GPU parity of the carried netem state's HBM layout (round 6): the departure ring kept circular in HBM
(a window loads only its head and writes only what it appends) and the timing wheel (far items parked
in per-source buckets by eligibility time).  Neither changes a result: every window is
bit-exact with the oracle (verdicts, deliveries in drain order, statistics) through the paths that
touch parked items -- reshaping that changes a link's delay range (the wheel takes a new bucket
width), disconnects (flush of a source's parked items, purge of parked items towards a removed
peer), sparse windows after dense ones (k_sim_sparse defers a source with parked items to k_sim_list,
which takes them all back) and fused groups (k_sim_fused hands the wheel from window to window)."""
import numpy as np
import pytest

from testground_amd import network as nw
from testground_amd import workloads as wl
from testground_amd.engine import Engine

from test_gpu_parity import assert_same, both

pytestmark = pytest.mark.gpu

try:  # torch ships its own HIP runtime: let it initialise first when both share a process
    import torch

    if torch.cuda.is_available():
        torch.cuda.init()
except ImportError:  # pragma: no cover
    torch = None


def test_wheel_reshape_disconnect_purge(make_oracle):
    """Storm shapes driven into their sustained state, then a quarter of the links reshaped to three
    times their latency (a delay range the wheel's buckets no longer span: kept items, a rebuild) and
    back, then 5 % of the peers disconnected (their own parked items flushed, parked items towards
    them purged) and reconnected."""
    n, window, lam = 600, 2000, 0.3
    g, c = both(make_oracle, n)
    wl.configure_storm(g, n)
    wl.configure_storm(c, n)
    rng = np.random.default_rng(11)
    sh = wl.storm_shape_arrays(n)
    sel = rng.choice(n, n // 4, replace=False)
    gone = rng.choice(n, n // 20, replace=False)
    for k in range(72):
        if k in (40, 52):
            f = 3 if k == 40 else 1
            cfg = nw.configs_array(sh["latency_ns"][sel] * f, sh["jitter_ns"][sel], sh["bandwidth_bps"][sel],
                                   sh["loss"][sel], sh["corrupt"][sel], sh["reorder"][sel], sh["duplicate"][sel],
                                   routing_policy=2)
            g.configure_batch(sel, cfg)
            c.configure_batch(sel, cfg)
        if k in (58, 64):
            for i in gone:
                cfg = nw.Config(Network="default", Enable=k == 64, Default=wl.storm_shapes(n)[int(i)])
                g.configure(int(i), cfg)
                c.configure(int(i), cfg)
        g.gen_storm(lam, window)
        c.gen_storm(lam, window)
        g.step(window)
        c.step(window)
        assert_same(g, c, f"window {k}")
    s = g.stats()
    assert s["flushed"] > 0 and s["lost_in_flight"] > 0
    # the far items did stay parked: the bytes moved are well below the per-window model
    assert g.carry_bytes() < 0.5 * s["queue_state_bytes"], (g.carry_bytes(), s["queue_state_bytes"])


def test_wheel_dense_then_sparse_windows(make_oracle):
    """Dense windows park far items; the sparse windows that follow (few packets per source, the
    automatic kernel choice) defer every source with parked items to k_sim_list, which takes them
    back into the heap array; dense again at the end."""
    n = 300
    g, c = both(make_oracle, n)
    cfg = nw.configs_array(np.full(n, 30 * nw.Millisecond), np.full(n, 8 * nw.Millisecond), np.full(n, 1 << 30),
                           loss=1.0, duplicate=1.0, corrupt=1.0, reorder=1.0)
    g.configure_batch(np.arange(n), cfg)
    c.configure_batch(np.arange(n), cfg)
    for k in range(50):
        lam = 0.05 if k < 20 or k >= 42 else 0.002  # 100 vs 4 packets per source and window
        g.gen_storm(lam, 2000)
        c.gen_storm(lam, 2000)
        g.step(2000)
        c.step(2000)
        assert_same(g, c, f"window {k}")


@pytest.mark.parametrize("diag", [False, True], ids=["plain", "stamps-and-timing"])
def test_wheel_fused_groups(make_oracle, monkeypatch, diag):
    """Generated windows fused eight per launch (k_sim_fused: the wheel's counts, header and items
    cross between windows of one launch by the write-through hand-off) after a settle in single
    windows; two groups, equal to the oracle's eight-window steps.  With the diagnostics on (in-kernel
    stamps, timing events around every launch) the results are the same."""
    if diag:
        for k in ("TGSIM_STAMPS", "TGSIM_SIM_TIMING", "TGSIM_DV_TIMING"):
            monkeypatch.setenv(k, "1")
    n, window = 1000, 2000
    g, c = both(make_oracle, n)
    wl.configure_storm(g, n)
    wl.configure_storm(c, n)
    for k in range(30):
        g.gen_storm(0.5, window)
        c.gen_storm(0.5, window)
        g.step(window)
        c.step(window)
    assert_same(g, c, "settled")
    for grp in range(2):
        for _ in range(8):
            g.gen_storm(0.5, window)
            c.gen_storm(0.5, window)
        g.step_n(window, 8)
        c.step_n(window, 8)
        dg, dc = g.drain(), c.drain()
        assert len(dg) == len(dc) and (dg == dc).all(), f"group {grp}"
        assert g.stats() == c.stats(), f"group {grp}"


def test_compact_emit_long_jittered_queues_default_knobs(make_oracle):
    """a sparse window of 90,000 sources (the compact emit layout: classic regions
    past 2 GiB) whose jittered queues hold 300-400 items, so k_sim_sparse defers them to k_sim_list.
    With default knobs the list claims emit-pool space only for the items due before the horizon plus
    two per offered packet, so the pool suffices (no sticky -ENOSPC) and every window equals the oracle."""
    n, window = 90_000, 2000
    g, c = both(make_oracle, n)
    cfg = nw.configs_array(np.full(n, 50 * nw.Millisecond), np.full(n, 20 * nw.Millisecond), np.full(n, 1 << 30),
                           loss=0.5, duplicate=0.5)
    g.configure_batch(np.arange(n), cfg)
    c.configure_batch(np.arange(n), cfg)
    for k in range(28):
        g.gen_storm(0.008, window)  # 16 packets per source and window: sparse
        c.gen_storm(0.008, window)
        g.step(window)
        c.step(window)
        if k >= 26:
            assert_same(g, c, f"window {k}")
        else:
            g.drain(), c.drain()
    assert g.stats() == c.stats()
