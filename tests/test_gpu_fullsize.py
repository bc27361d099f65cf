"""C4 at BASELINE.json's full size (configs[3]: 1,000,000 peers, degree 8, 64 floods): the oracle
cannot step a million peers in test time, so the full-size run is checked through properties that
do not depend on size:

* two different simulate paths agree bit for bit on every window of the flood: the register-only
  k_sim_sparse (+ k_sim_list for the sources it defers), which the bench runs, and the LDS-queue
  k_sim (TGSIM_SPARSE=0) — verdicts, every delivery in order, every statistic;
* the flood reaches (almost) every peer, the same peers on both paths, and every window's
  deliveries come out ordered by destination, then (time, source, sequence, clone first);
* the statistics add up: every offered packet has exactly one verdict, clones counted apart.

The small-size version of the same loop is bit-exact against the oracle
(test_gpu_parity.test_gossip_gpu_equals_oracle)."""
import numpy as np
import pytest

from testground_amd import abi
from testground_amd import workloads as wl
from testground_amd.engine import Engine

pytestmark = pytest.mark.gpu

try:  # torch ships its own HIP runtime: let it initialise first when both share a process
    import torch

    if torch.cuda.is_available():
        torch.cuda.init()
except ImportError:  # pragma: no cover
    torch = None


def _ordered(d):
    """Deliveries sorted by (dst, t_ns, src, seq, clone first): the delivery order
    (oracle/tgoracle.c cmp_del), checked pairwise over neighbours (vectorized)."""
    if len(d) < 2:
        return True
    a, b = d[:-1], d[1:]
    ca, cb = (a["flags"] & abi.FLAG_DUP) == 0, (b["flags"] & abi.FLAG_DUP) == 0
    le = (a["seq"] < b["seq"]) | ((a["seq"] == b["seq"]) & (ca <= cb))
    le = (a["src"] < b["src"]) | ((a["src"] == b["src"]) & le)
    le = (a["t_ns"] < b["t_ns"]) | ((a["t_ns"] == b["t_ns"]) & le)
    le = (a["dst"] < b["dst"]) | ((a["dst"] == b["dst"]) & le)
    return bool(le.all())


def test_gossip_1m_sparse_equals_dense(monkeypatch):
    n, windows = 1_000_000, 70
    engines = []
    for mode in ("1", "0"):  # read at engine creation
        monkeypatch.setenv("TGSIM_SPARSE", mode)
        e = Engine(n, lookahead_ns=wl.GOSSIP_MIN_LAT)
        wl.configure_gossip(e, n)
        engines.append(e)
    monkeypatch.delenv("TGSIM_SPARSE")
    sp, de = engines
    w = wl.gossip_window_ticks(sp)
    for e in engines:
        e.gossip_init(n_floods=64, degree=8, msg_len=1024, start_gap_ticks=1000, start_tick=0)
    peak = 0
    for k in range(windows):
        for e in engines:
            e.gen_gossip(w)
            e.step(w)
        v, vd = sp.verdicts(), de.verdicts()
        assert len(v) == len(vd) and np.array_equal(v, vd), f"window {k}: verdicts differ"
        d, dd = sp.drain(), de.drain()
        assert len(d) == len(dd) and np.array_equal(d.view(np.uint8), dd.view(np.uint8)), f"window {k}: deliveries differ"
        assert sp.stats() == de.stats(), f"window {k}"
        peak = max(peak, len(v))
        if k % 7 == 3:
            assert _ordered(d), f"window {k}: deliveries out of order"
        if k % 10 == 9:
            print(f"window {k + 1}: {len(v)} packets, {len(d)} deliveries", flush=True)
    assert peak > 5_000_000  # the flood's peak offers ~7-10 M packets per window
    rs, rd = sp.gossip_reached(), de.gossip_reached()
    assert (rs == rd).all() and (rs > 0.99 * n).all()
    st = sp.stats()
    by = st["by_verdict"]
    assert sum(by.values()) == st["offered"] + st["cloned"]
    assert by["scheduled"] > 0.98 * st["offered"] and st["scheduled"] > 0
    assert set(k for k, x in by.items() if x) <= {"scheduled", "loss"}, by


def test_epochs_100k_two_shards_equal_one():
    """C5 at full size (configs[4]: 100,000 instances, 10 % reshaped per 1,000-tick epoch): one
    engine and two uneven shards whose records are exchanged by hand (the all-to-all's data
    movement) agree bit for bit, epoch after epoch — verdicts, every delivery, the offered and
    scheduled counts — and each shard's barrier releases with its own peers' signals."""
    from test_gpu_parity import _manual_sharded_step

    n, bounds = 100_000, [0, 40_000, 100_000]
    ref = Engine(n)
    shards = [Engine(n, shard=(bounds[r], bounds[r + 1])) for r in range(2)]
    for e in [ref] + shards:
        wl.configure_storm(e, n)
    for k in range(4):
        wl.run_epoch(ref, n, k, n)
        for e in shards:
            if k:
                wl.epoch_reshape(e, n, k)
            e.gen_storm(wl.EPOCH_LAMBDA, wl.EPOCH_TICKS)
        _manual_sharded_step(shards, bounds, wl.EPOCH_TICKS)
        state, rnd = wl.epoch_state(k)
        for r, e in enumerate(shards):
            e.signal_async(state, bounds[r + 1] - bounds[r])
            assert e.barrier_poll(state, rnd * (bounds[r + 1] - bounds[r]))
        v_ref = ref.verdicts()
        v_sh = np.concatenate([e.verdicts() for e in shards])
        assert len(v_ref) > 15_000_000 and np.array_equal(v_sh, v_ref), f"epoch {k}: verdicts differ"
        d_ref = ref.drain()
        d_sh = np.concatenate([e.drain() for e in shards])
        assert len(d_sh) == len(d_ref) > 100_000, f"epoch {k}"
        assert np.array_equal(d_sh.view(np.uint8), d_ref.view(np.uint8)), f"epoch {k}: deliveries differ"
        assert _ordered(d_ref)
        print(f"epoch {k}: {len(v_ref)} packets, {len(d_ref)} deliveries", flush=True)
    s_ref, s_sh = ref.stats(), [e.stats() for e in shards]
    for key in ("offered", "scheduled", "cloned", "corrupted", "bytes_scheduled"):
        assert sum(s[key] for s in s_sh) == s_ref[key], key
    assert ref.barrier_poll(wl.epoch_state(3)[0], n)
