"""GPU parity: the HIP engine (libtgsim.so, through its C ABI) against the CPU oracle on identical
inputs.  Integer/byte work, so the bar is bit-exact: per-packet verdict bytes, every delivery record
(time, src, dst, seq, len, flags) in drain order, and the statistics counters."""
import ipaddress

import numpy as np
import pytest

from testground_amd import abi
from testground_amd import network as nw
from testground_amd import workloads as wl
from testground_amd.engine import Engine, packets

pytestmark = pytest.mark.gpu

try:  # torch ships its own HIP runtime: let it initialise first when both share a process
    import torch

    if torch.cuda.is_available():
        torch.cuda.init()
except ImportError:  # pragma: no cover
    torch = None


def assert_same(gpu, cpu, what=""):
    vg, vc = gpu.verdicts(), cpu.verdicts()
    assert len(vg) == len(vc), what
    bad = np.nonzero(vg != vc)[0]
    assert len(bad) == 0, f"{what}: {len(bad)} verdicts differ, first at {bad[:5]}: gpu {vg[bad[:5]]} cpu {vc[bad[:5]]}"
    dg, dc = gpu.drain(), cpu.drain()
    assert len(dg) == len(dc), f"{what}: {len(dg)} vs {len(dc)} deliveries"
    if len(dg):
        neq = np.nonzero(dg != dc)[0]
        assert len(neq) == 0, f"{what}: deliveries differ at {neq[:5]}: gpu {dg[neq[:3]]} cpu {dc[neq[:3]]}"
    sg, sc = gpu.stats(), cpu.stats()
    assert sg == sc, what
    return vg, dg


def both(make_oracle, n, **kw):
    return Engine(n, **kw), make_oracle(n, **kw)


def random_packets(rng, n_peers, n, n_ticks, ext_frac=0.0, seq_base=None):
    src = rng.integers(0, n_peers, n)
    dst = (src + 1 + rng.integers(0, n_peers - 1, n)) % n_peers
    if ext_frac:
        dst = np.where(rng.random(n) < ext_frac, abi.EXTERNAL, dst)
    pk = np.zeros(n, dtype=abi.PKT_DTYPE)
    pk["src"], pk["dst"] = src, dst
    pk["len"] = rng.integers(40, 1500, n)
    pk["tick"] = rng.integers(0, n_ticks, n)
    # unique per-source sequence numbers
    order = np.lexsort((pk["tick"], src))
    seq = np.empty(n, dtype=np.uint32)
    counts = np.bincount(src, minlength=n_peers)
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    ranks = np.arange(n) - starts[src[order]]
    base = seq_base if seq_base is not None else np.zeros(n_peers, dtype=np.uint32)
    seq[order] = ranks + base[src[order]]
    base += counts.astype(np.uint32)
    pk["seq"] = seq
    return pk


def test_storm_generator_and_step(make_oracle):
    """C3 at small scale: device-generated storm traffic, heterogeneous shapes, three steps."""
    n = 257
    g, c = both(make_oracle, n)
    wl.configure_storm(g, n)
    wl.configure_storm(c, n)
    for step in range(3):
        g.gen_storm(0.5, 1500)
        c.gen_storm(0.5, 1500)
        g.step(1500)
        c.step(1500)
        v, d = assert_same(g, c, f"storm step {step}")
        assert len(v) > 100_000
    s = g.stats()
    assert s["by_verdict"]["queue_full"] > 0 and s["by_verdict"]["loss"] > 0 and s["cloned"] > 0


def test_host_packets_all_features(make_oracle):
    """Correlated dup/corrupt/reorder, jitter, bandwidth, rules, disconnects, external traffic."""
    n = 96
    rng = np.random.default_rng(3)
    g, c = both(make_oracle, n, queue_limit=64)
    for i in range(n):
        s = nw.LinkShape(Latency=int(rng.integers(0, 20)) * nw.Millisecond,
                         Jitter=int(rng.integers(0, 5)) * nw.Millisecond,
                         Bandwidth=int(rng.choice([0, 1 << 20, 10**7, 10**8])),
                         Loss=float(rng.uniform(0, 10)), Duplicate=float(rng.uniform(0, 20)),
                         DuplicateCorr=float(rng.choice([0, 25.0])), Corrupt=float(rng.uniform(0, 20)),
                         CorruptCorr=float(rng.choice([0, 40.0])), Reorder=float(rng.choice([0, 10.0])),
                         ReorderCorr=float(rng.choice([0, 30.0])))
        rules = []
        if i % 5 == 0:
            for j in rng.integers(0, n, 6):
                rules.append(nw.LinkRule(Subnet=(str(ipaddress.IPv4Address(wl.peer_ip(int(j)))), 32),
                                         LinkShape=nw.LinkShape(Filter=nw.FilterAction(int(rng.integers(1, 3))))))
            rules.append(nw.LinkRule(Subnet="16.0.0.64/27", LinkShape=nw.LinkShape(Filter=nw.FilterAction.Reject)))
        pol = nw.RoutingPolicyType.AllowAll if i % 3 == 0 else nw.RoutingPolicyType.DenyAll
        cfg = nw.Config(Network="default", Enable=(i % 17 != 5), Default=s, Rules=rules, RoutingPolicy=pol)
        g.configure(i, cfg)
        c.configure(i, cfg)
    seq = np.zeros(n, dtype=np.uint32)
    for step in range(4):
        pk = random_packets(rng, n, 60_000, 4000, ext_frac=0.02, seq_base=seq)
        g.submit(pk)
        c.submit(pk)
        g.step(4000)
        c.step(4000)
        assert_same(g, c, f"host step {step}")


@pytest.mark.parametrize("queue_limit,lookahead", [(1000, 0), (32, 0), (200, 300_000)])
def test_window_edge_shapes(make_oracle, queue_limit, lookahead):
    """Uncorrelated shapes that stress the windowed netem/HTB resolution of k_sim: zero and
    sub-tick latency, jitter larger than the latency (delays clamped to 0, items eligible at once),
    heavy reorder and duplication, every bandwidth class, bursts of packets in one tick, and
    sequence numbers that are not monotone across ticks (ties in e resolved by seq)."""
    n = 128
    rng = np.random.default_rng(11 + queue_limit)
    g, c = both(make_oracle, n, queue_limit=queue_limit, lookahead_ns=lookahead)
    lat = [0, 50 * nw.Microsecond, 1 * nw.Millisecond, 20 * nw.Millisecond]
    for i in range(n):
        L = lat[i % 4]
        J = [0, L // 2, 2 * L, 5 * nw.Millisecond][(i // 4) % 4]
        s = nw.LinkShape(Latency=L, Jitter=J,
                         Bandwidth=int([0, 1 << 20, 10**7, 10**8, 10**9][(i // 16) % 5]),
                         Reorder=float([0, 5, 50][(i // 3) % 3]), Duplicate=float([0, 20][(i // 7) % 2]),
                         Loss=float([0, 5][(i // 11) % 2]), Corrupt=float([0, 10][(i // 5) % 2]))
        cfg = nw.Config(Network="default", Enable=True, Default=s)
        g.configure(i, cfg)
        c.configure(i, cfg)
    for step in range(3):
        m = 150_000
        src = rng.integers(0, n, m)
        pk = np.zeros(m, dtype=abi.PKT_DTYPE)
        pk["src"] = src
        pk["dst"] = (src + 1 + rng.integers(0, n - 1, m)) % n
        pk["len"] = rng.integers(40, 1500, m)
        # bursty ticks: a third of the packets land on 20 ticks
        tick = rng.integers(0, 2000, m)
        burst = rng.random(m) < 0.33
        tick[burst] = rng.choice(rng.integers(0, 2000, 20), burst.sum())
        pk["tick"] = tick
        pk["seq"] = rng.permutation(m).astype(np.uint32) + np.uint32(step * m)  # unique, not monotone
        g.submit(pk)
        c.submit(pk)
        g.step(2000)
        c.step(2000)
        assert_same(g, c, f"edge shapes step {step}")
    st = g.stats()
    assert st["by_verdict"]["queue_full"] > 0 and st["cloned"] > 0


def test_mid_run_reconfiguration(make_oracle):
    """C5-style: reshape a subset between steps, including the netem quirks (corrupt persists when
    re-set to 0, correlation state re-randomised) and a re-address (reconnect)."""
    n = 64
    rng = np.random.default_rng(5)
    g, c = both(make_oracle, n)
    shapes = wl.storm_shapes(n, 99)
    for i, s in enumerate(shapes):
        s.Corrupt, s.CorruptCorr, s.DuplicateCorr = 5.0, 20.0, 10.0
        for e in (g, c):
            e.configure(i, nw.Config(Network="default", Enable=True, Default=s))
    seq = np.zeros(n, dtype=np.uint32)
    for epoch in range(5):
        pk = random_packets(rng, n, 30_000, 3000, seq_base=seq)
        g.submit(pk)
        c.submit(pk)
        g.step(3000)
        c.step(3000)
        assert_same(g, c, f"epoch {epoch}")
        for i in rng.choice(n, n // 10, replace=False):
            s = wl.storm_shapes(1, int(rng.integers(1 << 30)))[0]
            ip = wl.peer_ip(int(i)) + 1000 if epoch == 2 else None
            cfg = nw.Config(Network="default", Enable=True, Default=s,
                            IPv4=(str(ipaddress.IPv4Address(ip)), 16) if ip else None)
            g.configure(int(i), cfg)
            c.configure(int(i), cfg)


@pytest.mark.parametrize("case", ["drop", "reject", "accept"])
def test_splitbrain_1k(make_oracle, case):
    """C2: 1000 instances, all 999,000 ordered pairs, request + reply."""
    n = 1000
    g, c = both(make_oracle, n)
    ok_g, art_g = wl.run_splitbrain(g, n, case)
    ok_c, art_c = wl.run_splitbrain(c, n, case)
    for k in ("v_req", "d_req", "v_rep", "d_rep"):
        assert len(art_g[k]) == len(art_c[k]) and (art_g[k] == art_c[k]).all(), k
    assert (ok_g == ok_c).all()
    assert (ok_g == wl.splitbrain_expected(n, case)).all()


def test_pingpong_rtt_windows_gpu():
    """C1 on the GPU: RTT within pingpong.go:185 / :195 windows."""
    e = Engine(2, lookahead_ns=1_000_000)
    for i in (0, 1):
        e.configure(i, wl.pingpong_config(100 * nw.Millisecond))
    rtt, now = wl.pingpong_round(e, 0, 0)
    assert all(200 * nw.Millisecond <= r <= 215 * nw.Millisecond for r in rtt), rtt
    for i in (0, 1):
        e.configure(i, wl.pingpong_config(10 * nw.Millisecond, "latency-reduced"))
    rtt2, _ = wl.pingpong_round(e, now + 100_000, 10)
    assert all(20 * nw.Millisecond <= r <= 35 * nw.Millisecond for r in rtt2), rtt2


def test_two_shards_equal_one(make_oracle):
    """Sharding sources over two engines (step_sim -> exchange -> deliver) gives the single-engine
    result: same verdicts per shard and the same delivered multiset per destination."""
    n = 300
    half = 150
    ref = Engine(n)
    shards = [Engine(n, shard=(0, half)), Engine(n, shard=(half, n))]
    wl.configure_storm(ref, n)
    for s in shards:
        wl.configure_storm(s, n)
    rng = np.random.default_rng(9)
    seq = np.zeros(n, dtype=np.uint32)
    pk = random_packets(rng, n, 200_000, 5000, seq_base=seq)
    ref.submit(pk)
    ref.step(5000)
    v_ref = ref.verdicts()
    d_ref = ref.drain()
    outs = []
    for k, s in enumerate(shards):
        lo, hi = (0, half) if k == 0 else (half, n)
        s.submit(pk[(pk["src"] >= lo) & (pk["src"] < hi)])
        buf = torch.empty(s.sim_capacity() * 24, dtype=torch.uint8, device="cuda")
        cnt = s.step_sim(5000, [0, half, n], buf.data_ptr(), s.sim_capacity())
        outs.append((buf, cnt))
    for k, s in enumerate(shards):
        parts = []
        for j, (buf, cnt) in enumerate(outs):
            off = int(cnt[:k].sum()) * 24
            parts.append(buf[off: off + int(cnt[k]) * 24])
        inbound = torch.cat(parts)
        torch.cuda.current_stream().synchronize()  # torch.cat ran on torch's stream
        s.deliver(inbound.data_ptr(), inbound.numel() // 24)
    d_sh = np.concatenate([s.drain() for s in shards])
    assert len(d_sh) == len(d_ref)
    assert (np.sort(d_sh, order=["dst", "t_ns", "src", "seq", "flags"]) ==
            np.sort(d_ref, order=["dst", "t_ns", "src", "seq", "flags"])).all()
    assert (d_sh == d_ref).all()  # drain order is (dst, t, src, seq, clone-first) on each shard
    v_sh = [s.verdicts() for s in shards]
    for k, (lo, hi) in enumerate([(0, half), (half, n)]):
        sel = (pk["src"] >= lo) & (pk["src"] < hi)
        assert (v_sh[k] == v_ref[sel]).all()


def test_full_size_storm_properties():
    """C3 at full size (10,000 instances): conservation and ordering invariants."""
    n = 10_000
    e = Engine(n)
    wl.configure_storm(e, n)
    e.gen_storm(0.5, 2000)
    e.step(2000)
    v = e.verdicts()
    d = e.drain()
    s = e.stats()
    assert s["offered"] == len(v) > 9_000_000
    assert sum(s["by_verdict"].values()) == len(v) + int(((v >> 4) != abi.V_NONE).sum())
    assert s["scheduled"] == len(d)
    assert (np.diff(d["dst"].astype(np.int64)) >= 0).all()
    same = d["dst"][1:] == d["dst"][:-1]
    assert (d["t_ns"][1:][same] >= d["t_ns"][:-1][same]).all()


def _manual_sharded_step(shards, bounds, window):
    """step_sim on every shard, exchange through device buffers, deliver (one GPU, no collective)."""
    outs = []
    torch.cuda.current_stream().synchronize()  # the engines run on their own streams (shard.py)
    for s in shards:
        buf = torch.empty(max(1, s.sim_capacity()) * 24, dtype=torch.uint8, device="cuda")
        cnt = s.step_sim(window, bounds, buf.data_ptr(), s.sim_capacity())
        outs.append((buf, cnt))
    for k, s in enumerate(shards):
        parts = [buf[int(cnt[:k].sum()) * 24: int(cnt[:k + 1].sum()) * 24] for buf, cnt in outs]
        inbound = torch.cat(parts)
        torch.cuda.current_stream().synchronize()  # torch.cat ran on torch's stream
        s.deliver(inbound.data_ptr(), inbound.numel() // 24)


def test_gossip_gpu_equals_oracle(make_oracle):
    """C4 at small scale: device-generated floods whose receipts drive the next window; every
    window's verdicts and deliveries, and the per-flood reach, bit-exact with the oracle."""
    n, floods = 3000, 16
    g, c = both(make_oracle, n, lookahead_ns=wl.GOSSIP_MIN_LAT)
    for e in (g, c):
        wl.configure_gossip(e, n)
        e.gossip_init(n_floods=floods, degree=8, msg_len=1024, start_gap_ticks=500, start_tick=0)
    w = wl.gossip_window_ticks(g)
    total = 0
    for k in range(40):
        g.gen_gossip(w)
        c.gen_gossip(w)
        g.step(w)
        c.step(w)
        v, _ = assert_same(g, c, f"gossip window {k}")
        total += len(v)
    rg, rc = g.gossip_reached(), c.gossip_reached()
    assert (rg == rc).all() and (rg > 0.99 * n).all()
    assert total == 8 * int(rg.sum())  # every reached peer forwarded once (floods drained)
    # the sparse windows wrote records straight into destination buckets, and the
    # destinations that received more than a bucket holds took the rest through the slot scatter
    b, sched = g.bucket_records(), g.stats()["scheduled"]
    assert 0 < b < sched, (b, sched)


@pytest.mark.parametrize("knobs", [{"TGSIM_DST_BKT": "0"}, {"TGSIM_DST_SLOT": "0"}, {"TGSIM_EMIT_SETS": "2"},
                                   {"TGSIM_STAMPS": "1", "TGSIM_SIM_TIMING": "1", "TGSIM_DV_TIMING": "1"}],
                         ids=["slot-scatter", "cursor-scatter", "two-sets", "diagnostics-on"])
def test_gossip_delivery_layouts_equal_oracle(make_oracle, monkeypatch, knobs):
    """The delivery layouts the engine can be switched to for A/B runs (read at
    tgsim_create) give the default's results: every window bit-exact with the oracle, at a size
    where destinations overflow their buckets."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    n, floods = 2000, 16
    g, c = both(make_oracle, n, lookahead_ns=wl.GOSSIP_MIN_LAT)
    for e in (g, c):
        wl.configure_gossip(e, n)
        e.gossip_init(n_floods=floods, degree=8, msg_len=1024, start_gap_ticks=500, start_tick=0)
    w = wl.gossip_window_ticks(g)
    for k in range(30):
        g.gen_gossip(w)
        c.gen_gossip(w)
        g.step(w)
        c.step(w)
        assert_same(g, c, f"gossip window {k} ({knobs})")
    assert (g.gossip_reached() == c.gossip_reached()).all()
    if "TGSIM_DST_BKT" in knobs or "TGSIM_DST_SLOT" in knobs:
        assert g.bucket_records() == 0


def test_gossip_two_shards_equal_one():
    """C4 sharded: receipts are folded on the destination's shard and forwarded from there."""
    n, floods, half = 2000, 8, 1000
    ref = Engine(n, lookahead_ns=wl.GOSSIP_MIN_LAT)
    shards = [Engine(n, shard=(0, half), lookahead_ns=wl.GOSSIP_MIN_LAT),
              Engine(n, shard=(half, n), lookahead_ns=wl.GOSSIP_MIN_LAT)]
    for e in [ref] + shards:
        wl.configure_gossip(e, n)
        e.gossip_init(n_floods=floods, degree=8, msg_len=1024, start_gap_ticks=300, start_tick=0)
    w = wl.gossip_window_ticks(ref)
    for k in range(30):
        ref.gen_gossip(w)
        ref.step(w)
        for s in shards:
            s.gen_gossip(w)
        _manual_sharded_step(shards, [0, half, n], w)
        d_sh = np.concatenate([s.drain() for s in shards])
        d_ref = ref.drain()
        assert len(d_sh) == len(d_ref) and (d_sh == d_ref).all(), f"window {k}"
        v_sh = np.concatenate([s.verdicts() for s in shards])
        assert (v_sh == ref.verdicts()).all(), f"window {k}"
    assert (shards[0].gossip_reached() + shards[1].gossip_reached() == ref.gossip_reached()).all()


def test_epochs_reshaping_and_barriers(make_oracle):
    """C5 at small scale: 10 % of the peers get a fresh shape every epoch, all peers pass the
    epoch barrier; every epoch bit-exact with the oracle."""
    n = 2000
    g, c = both(make_oracle, n)
    for e in (g, c):
        wl.configure_storm(e, n)
    for k in range(6):
        for e in (g, c):
            wl.run_epoch(e, n, k, n)
        v, _ = assert_same(g, c, f"epoch {k}")
        assert len(v) > 300_000
    assert g.barrier_poll(wl.epoch_state(5)[0], n) and not g.barrier_poll(wl.epoch_state(6)[0], 1)


def test_full_size_storm_rates():
    """C3 at full size: the netem event rates the engine produced match the configured shapes
    (loss, duplicate within +-0.5 pp of the offered-weighted mean of the per-instance rates)."""
    n = 10_000
    e = Engine(n)
    wl.configure_storm(e, n)
    e.gen_storm(0.5, 2000)
    e.step(2000)
    v = e.verdicts()
    shapes = wl.storm_shape_arrays(n)
    s = e.stats()
    offered = s["offered"]
    # every instance offers Poisson(0.5) per tick: weights equal in expectation
    loss_exp = float(np.mean(shapes["loss"])) / 100
    dup_exp = float(np.mean(shapes["duplicate"])) / 100
    lost_orig = int(((v & 15) == abi.V_LOSS).sum())
    cloned = int(((v >> 4) != abi.V_NONE).sum())
    # loss on an original happens only without a duplicate event: P = loss * (1 - dup)
    assert abs(lost_orig / offered - loss_exp * (1 - dup_exp)) <= 0.005
    assert abs(cloned / offered - dup_exp * (1 - loss_exp)) <= 0.005


def test_edge_inputs(make_oracle):
    """Empty and ragged inputs, extreme values: steps with no packets at all, one peer sending
    everything, the last tick of a window, zero- and maximum-length packets, the maximum netem
    limit (1024) filled from empty in one burst, external traffic from a disconnected source,
    a latency past the 2^32 us clamp (link.go:143-151), and 1-tick steps."""
    n = 50
    g, c = both(make_oracle, n, queue_limit=1024)
    shapes = [nw.LinkShape(), nw.LinkShape(Latency=5 * nw.Millisecond, Bandwidth=1 << 20),
              nw.LinkShape(Latency=(1 << 33) * nw.Microsecond), nw.LinkShape(Jitter=3 * nw.Millisecond),
              nw.LinkShape(Latency=1, Loss=100.0), nw.LinkShape(Duplicate=100.0, Reorder=100.0)]
    for i in range(n):
        cfg = nw.Config(Network="default", Enable=(i != 7), Default=shapes[i % len(shapes)],
                        RoutingPolicy=nw.RoutingPolicyType.AllowAll if i % 2 else nw.RoutingPolicyType.DenyAll)
        g.configure(i, cfg)
        c.configure(i, cfg)
    seq = np.zeros(n, dtype=np.uint32)

    def run(pk, ticks, what):
        if pk is not None:
            g.submit(pk)
            c.submit(pk)
        g.step(ticks)
        c.step(ticks)
        assert_same(g, c, what)

    run(None, 1000, "empty step")
    run(None, 1, "empty 1-tick step")
    # one source, 3000 packets in one tick: the 1024 queue fills, the rest are QUEUE_FULL
    m = 3000
    pk = np.zeros(m, dtype=abi.PKT_DTYPE)
    pk["src"], pk["dst"], pk["len"], pk["tick"] = 1, 2, 1500, 999
    pk["seq"] = np.arange(m)
    run(pk, 1000, "burst into the max limit")
    # ragged: every source a different count, lengths 0 and 65535, externals, disconnected source
    rng = np.random.default_rng(21)
    parts = []
    for s in range(n):
        k = int(s * 3 % 17)
        if not k:
            continue
        p = np.zeros(k, dtype=abi.PKT_DTYPE)
        p["src"] = s
        p["dst"] = np.where(rng.random(k) < 0.2, abi.EXTERNAL, (s + 1 + rng.integers(0, n - 1, k)) % n)
        p["len"] = rng.choice([0, 1, 65535], k)
        p["tick"] = np.sort(rng.integers(0, 5, k))
        p["seq"] = seq[s] + np.arange(k) + 10_000
        seq[s] += k
        parts.append(p)
    run(np.concatenate(parts), 5, "ragged 5-tick step")
    for w in (1, 7, 1):
        run(None, w, f"empty {w}-tick step after traffic")
    st = g.stats()
    bv = st["by_verdict"]
    assert bv["queue_full"] > 0 and bv["disconnected"] > 0 and bv["external"] > 0 and bv["no_route"] > 0


def _ks_uniform(x, lo, hi):
    x = np.sort((np.asarray(x, dtype=np.float64) - lo) / (hi - lo))
    cdf = np.arange(1, len(x) + 1) / len(x)
    return max(np.max(cdf - x), np.max(x - (cdf - 1 / len(x))))


def test_full_size_latency_distribution():
    """Statistical parity on the GPU at scale (north_star: KS <= 0.02 on latency, loss +-0.5 pp):
    1,000 instances in four LinkShape groups, 100 packets each, sparse enough that the netem limit
    is never reached and unlimited bandwidth (HTB passes at e).  Each group's delays follow
    netem's uniform U[L-J, L+J) (no distribution table, link.go:169-179) and its loss rate is the
    configured percentage."""
    n, per, gap = 1000, 100, 700
    groups = [(20, 5, 1.0), (50, 10, 3.0), (5, 0, 0.0), (80, 20, 2.0)]  # L ms, J ms, loss %
    e = Engine(n)
    for i in range(n):
        L, J, loss = groups[i % 4]
        e.configure(i, nw.Config(Network="default", Enable=True, Default=nw.LinkShape(
            Latency=L * nw.Millisecond, Jitter=J * nw.Millisecond, Loss=loss)))
    half = per // 2  # ticks are u16 within a step: two steps of 50 packets per instance
    src = np.repeat(np.arange(n, dtype=np.uint32), half)
    vs = []
    for c in range(2):
        idx = np.tile(np.arange(half, dtype=np.uint32), n)
        pk = np.zeros(n * half, dtype=abi.PKT_DTYPE)
        pk["src"], pk["seq"], pk["len"] = src, idx + c * half, 200
        pk["dst"] = (src + 1 + ((idx + c * half) * 7919) % (n - 1)) % n
        pk["tick"] = idx * gap
        e.submit(pk)
        e.step(half * gap)
        vs.append(e.verdicts() & 15)
    v = np.concatenate(vs)
    src = np.concatenate([src, src])
    assert not (v == abi.V_QUEUE_FULL).any()
    for _ in range(2):
        e.step(60_000)  # past the largest L + J
    d = e.drain()
    d = d[(d["flags"] & abi.FLAG_DUP) == 0]
    delays = d["t_ns"].astype(np.int64) - d["seq"].astype(np.int64) * gap * 1000
    for g, (L, J, loss) in enumerate(groups):
        mine = (d["src"] % 4) == g
        x = delays[mine]
        lo, hi = (L - J) * 1e6, (L + J) * 1e6
        if J == 0:
            assert (x == L * 1_000_000).all()
        else:
            assert x.min() >= lo and x.max() < hi
            assert _ks_uniform(x, lo, hi) <= 0.02, f"group {g}"
        sent = np.asarray(src % 4 == g)
        lost = int((v[sent] == abi.V_LOSS).sum())
        assert abs(lost / int(sent.sum()) - loss / 100) <= 0.005, f"group {g}"


def test_three_shards_slotted_exchange_equal_one():
    """The slotted layout (tgsim_step_sim_launch_slotted / tgsim_deliver_slotted_async) over three
    shards on one GPU, the chunks swapped by hand as the fixed-size all-to-all would: the same
    deliveries and verdicts as one engine.  Rank edges, count headers and empty slots are all
    exercised (one chunk per rank pair, slot_cap well above every count)."""
    n, bounds = 300, [0, 90, 210, 300]
    ref = Engine(n)
    shards = [Engine(n, shard=(bounds[r], bounds[r + 1])) for r in range(3)]
    for e in [ref] + shards:
        wl.configure_storm(e, n)
    rng = np.random.default_rng(21)
    pk = random_packets(rng, n, 150_000, 5000, seq_base=np.zeros(n, dtype=np.uint32))
    ref.submit(pk)
    ref.step(5000)
    v_ref, d_ref = ref.verdicts(), ref.drain()
    cap = 60_000
    chunk = (cap + 1) * 24
    bufs = []
    for r, s in enumerate(shards):
        s.submit(pk[(pk["src"] >= bounds[r]) & (pk["src"] < bounds[r + 1])])
        buf = torch.zeros(3 * chunk, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        s.step_sim_launch_slotted(5000, bounds, buf.data_ptr(), cap)
        s.step_sim_release()
        s.sync()
        bufs.append(buf)
    for k, s in enumerate(shards):
        inbound = torch.cat([b[k * chunk:(k + 1) * chunk] for b in bufs])
        torch.cuda.synchronize()
        s.deliver_slotted_async(inbound.data_ptr(), 3, cap)
        s.sync()
    d_sh = np.concatenate([s.drain() for s in shards])
    assert len(d_sh) == len(d_ref) > 2000
    assert (d_sh == d_ref).all()
    for r, s in enumerate(shards):
        sel = (pk["src"] >= bounds[r]) & (pk["src"] < bounds[r + 1])
        assert (s.verdicts() == v_ref[sel]).all()


@pytest.mark.parametrize("mode", ["0", "1"])
def test_sparse_and_dense_kernels_agree(make_oracle, monkeypatch, mode):
    """The same steps through the dense k_sim (TGSIM_SPARSE=0) and through k_sim_sparse + k_sim_list
    (TGSIM_SPARSE=1: open queues in the register-only kernel, the rest deferred to the worklist):
    bit-exact with the oracle either way, on a mix of sparse and dense, correlated and plain
    senders."""
    monkeypatch.setenv("TGSIM_SPARSE", mode)
    n = 201
    rng = np.random.default_rng(41)
    g, c = both(make_oracle, n, queue_limit=300, lookahead_ns=200_000)
    shapes = wl.storm_shapes(n, 3)
    for i, s in enumerate(shapes):
        if i % 7 == 0:
            s.DuplicateCorr, s.CorruptCorr = 30.0, 20.0
        s.Latency = int(rng.integers(0, 8)) * nw.Millisecond
        for e in (g, c):
            e.configure(i, nw.Config(Network="default", Enable=True, Default=s))
    seq = np.zeros(n, dtype=np.uint32)
    for step in range(5):
        # a few heavy senders, many light ones
        heavy = rng.random(n) < 0.1
        m = 20_000
        src = np.where(rng.random(m) < 0.7, rng.choice(np.nonzero(heavy)[0], m), rng.integers(0, n, m))
        pk = np.zeros(m, dtype=abi.PKT_DTYPE)
        pk["src"] = src
        pk["dst"] = (src + 1 + rng.integers(0, n - 1, m)) % n
        pk["len"] = rng.integers(40, 1500, m)
        pk["tick"] = rng.integers(0, 3000, m)
        order = np.lexsort((pk["tick"], src))
        counts = np.bincount(src, minlength=n)
        starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
        sq = np.empty(m, dtype=np.uint32)
        sq[order] = np.arange(m) - starts[src[order]] + seq[src[order]]
        seq += counts.astype(np.uint32)
        pk["seq"] = sq
        g.submit(pk)
        c.submit(pk)
        g.step(3000)
        c.step(3000)
        assert_same(g, c, f"mode {mode} step {step}")


def test_sparse_long_queues(make_oracle, monkeypatch):
    """Sparse windows whose netem queues grow to 300-600 items (30-60 ms of latency, 2-ms windows of
    ~20 packets): k_sim_sparse serves them from registers while they fit (256 queued items), then
    defers them to k_sim_list; bit-exact with the oracle window by window."""
    monkeypatch.setenv("TGSIM_SPARSE", "1")
    n = 65
    rng = np.random.default_rng(7)
    g, c = both(make_oracle, n)
    for i in range(n):
        s = nw.LinkShape(Latency=int(rng.integers(30, 61)) * nw.Millisecond, Jitter=int(rng.integers(0, 3)) * nw.Millisecond,
                         Bandwidth=1 << 30, Loss=1.0, Duplicate=2.0, Corrupt=1.0)
        for e in (g, c):
            e.configure(i, nw.Config(Network="default", Enable=True, Default=s))
    seq = np.zeros(n, dtype=np.uint32)
    for step in range(40):
        m = 20 * n
        src = rng.integers(0, n, m)
        pk = np.zeros(m, dtype=abi.PKT_DTYPE)
        pk["src"] = src
        pk["dst"] = (src + 1 + rng.integers(0, n - 1, m)) % n
        pk["len"] = rng.integers(40, 1500, m)
        pk["tick"] = rng.integers(0, 2000, m)
        order = np.lexsort((pk["tick"], src))
        counts = np.bincount(src, minlength=n)
        starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
        sq = np.empty(m, dtype=np.uint32)
        sq[order] = np.arange(m) - starts[src[order]] + seq[src[order]]
        seq += counts.astype(np.uint32)
        pk["seq"] = sq
        g.submit(pk)
        c.submit(pk)
        g.step(2000)
        c.step(2000)
        assert_same(g, c, f"step {step}")
    # the queues did grow past the 128 items held in registers (state bytes: ~16 B x 2 per item)
    assert g.stats()["queue_state_bytes"] > 40 * n * 32 * 128 // 2


@pytest.mark.parametrize("latency_ms", [0, 3])
def test_flat_sort_hot_destinations(make_oracle, latency_ms):
    """The flattened per-destination sort (k_dst_sort_flat: sparse windows, up to 48 records per
    destination on average) with segments longer than its 64-record staging (three hot
    destinations take ~30 % of the traffic: sorted whole by the wave holding their first record),
    segments that straddle chunk boundaries, and duplicates whose delivery time equals their
    original's (no latency, no rate limit: the clone-first tie rule); bit-exact with the oracle in
    drain order."""
    n = 200
    rng = np.random.default_rng(11)
    g, c = both(make_oracle, n)
    for i in range(n):
        s = nw.LinkShape(Latency=latency_ms * nw.Millisecond, Duplicate=20.0, Loss=2.0, Corrupt=1.0)
        for e in (g, c):
            e.configure(i, nw.Config(Network="default", Enable=True, Default=s))
    seq = np.zeros(n, dtype=np.uint32)
    for step in range(5):
        m = 20 * n
        src = rng.integers(0, n, m)
        hot = rng.random(m) < 0.3
        dst = np.where(hot, rng.integers(0, 3, m), (src + 1 + rng.integers(0, n - 1, m)) % n)
        dst = np.where(dst == src, (src + 1) % n, dst)
        pk = np.zeros(m, dtype=abi.PKT_DTYPE)
        pk["src"], pk["dst"] = src, dst
        pk["len"] = rng.integers(40, 1500, m)
        pk["tick"] = rng.integers(0, 2000, m)
        order = np.lexsort((pk["tick"], src))
        counts = np.bincount(src, minlength=n)
        starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
        sq = np.empty(m, dtype=np.uint32)
        sq[order] = np.arange(m) - starts[src[order]] + seq[src[order]]
        seq += counts.astype(np.uint32)
        pk["seq"] = sq
        g.submit(pk)
        c.submit(pk)
        g.step(2000)
        c.step(2000)
        _, d = assert_same(g, c, f"latency {latency_ms} ms step {step}")
        if latency_ms == 0 or step >= 2:  # the hot segments exceed 64 records
            assert np.bincount(d["dst"], minlength=n)[:3].min() > 64


def test_multi_round_fifo_sources(make_oracle, monkeypatch):
    """k_sim_multi's own parity case.  FIFO links (no jitter, duplicates or reordering)
    offered 150-300 packets per window each, so k_sim_sparse hands every such source to k_sim_multi
    (more than 64 offered packets), whose rounds of 64 candidates go behind the queue tail and whose
    due prefix runs past 256 items.  Every 10th source reorders (5 %) and every 10th + 4 duplicates
    (3 %): their queue stops being FIFO partway through the candidates, after k_sim_multi already
    wrote some behind the tail, and they go on to k_sim_list.  Bit-exact with the oracle, window by
    window, with a high netem limit."""
    monkeypatch.setenv("TGSIM_SPARSE", "1")
    n = 60
    rng = np.random.default_rng(23)
    g, c = both(make_oracle, n, queue_limit=1024)
    for i in range(n):
        s = nw.LinkShape(Latency=int(rng.integers(1, 6)) * nw.Millisecond, Bandwidth=1 << 30, Loss=1.0,
                         Reorder=5.0 if i % 10 == 3 else 0.0, Duplicate=3.0 if i % 10 == 7 else 0.0)
        for e in (g, c):
            e.configure(i, nw.Config(Network="default", Enable=True, Default=s))
    seq = np.zeros(n, dtype=np.uint32)
    for step in range(12):
        per = rng.integers(150, 301, n)
        src = np.repeat(np.arange(n), per)
        m = len(src)
        pk = np.zeros(m, dtype=abi.PKT_DTYPE)
        pk["src"] = src
        pk["dst"] = (src + 1 + rng.integers(0, n - 1, m)) % n
        pk["len"] = rng.integers(40, 1500, m)
        pk["tick"] = rng.integers(0, 4000, m)
        order = np.lexsort((pk["tick"], src))
        counts = np.bincount(src, minlength=n)
        starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
        sq = np.empty(m, dtype=np.uint32)
        sq[order] = np.arange(m) - starts[src[order]] + seq[src[order]]
        seq += counts.astype(np.uint32)
        pk["seq"] = sq
        g.submit(pk)
        c.submit(pk)
        g.step(4000)
        c.step(4000)
        _, d = assert_same(g, c, f"step {step}")
        assert len(d) > 0


@pytest.mark.parametrize("reserve", [1, 8])
def test_compact_emit_layout(make_oracle, monkeypatch, reserve):
    """the compact emit layout (sparse windows keep 2 records per offered packet
    plus `reserve` per source in place; a source that serves more of its old queue claims the rest
    from the window's pool), forced on small windows with a tiny reserve so that most sources use the
    pool, through k_sim_sparse, k_sim_multi and k_sim_list; bit-exact with the oracle."""
    monkeypatch.setenv("TGSIM_SPARSE", "1")
    monkeypatch.setenv("TGSIM_EMIT_COMPACT", "2")
    monkeypatch.setenv("TGSIM_EMIT_R", str(reserve))
    n = 80
    rng = np.random.default_rng(31)
    g, c = both(make_oracle, n, queue_limit=1024)
    for i in range(n):
        # latency longer than a window: old queue items are served next to a few new ones; every 8th
        # source offers > 64 packets (k_sim_multi), every 10th + 3 duplicates (k_sim_list)
        s = nw.LinkShape(Latency=int(rng.integers(3, 9)) * nw.Millisecond, Bandwidth=1 << 30, Loss=1.0,
                         Duplicate=3.0 if i % 10 == 3 else 0.0)
        for e in (g, c):
            e.configure(i, nw.Config(Network="default", Enable=True, Default=s))
    seq = np.zeros(n, dtype=np.uint32)
    for step in range(14):
        burst = step % 4 == 0  # bursts, then quiet windows that serve the queued items
        per = np.where(np.arange(n) % 8 == 0, rng.integers(100, 200, n), rng.integers(20, 60, n)) if burst \
            else rng.integers(0, 4, n)
        src = np.repeat(np.arange(n), per)
        m = len(src)
        pk = np.zeros(m, dtype=abi.PKT_DTYPE)
        pk["src"] = src
        pk["dst"] = (src + 1 + rng.integers(0, n - 1, m)) % n
        pk["len"] = rng.integers(40, 1500, m)
        pk["tick"] = rng.integers(0, 2000, m)
        order = np.lexsort((pk["tick"], src))
        counts = np.bincount(src, minlength=n)
        starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
        sq = np.empty(m, dtype=np.uint32)
        sq[order] = np.arange(m) - starts[src[order]] + seq[src[order]]
        seq += counts.astype(np.uint32)
        pk["seq"] = sq
        g.submit(pk)
        c.submit(pk)
        g.step(2000)
        c.step(2000)
        assert_same(g, c, f"reserve {reserve} step {step}")


def test_compact_emit_pool_overflow_fails(monkeypatch):
    """A compact window whose sources need more pool than it holds fails loudly (-ENOSPC at the
    next call), never silently: records past a region with no pool space are not delivered."""
    import errno

    from testground_amd.engine import EngineError

    monkeypatch.setenv("TGSIM_SPARSE", "1")
    monkeypatch.setenv("TGSIM_EMIT_COMPACT", "2")
    monkeypatch.setenv("TGSIM_EMIT_R", "1")
    monkeypatch.setenv("TGSIM_EMIT_POOL", "0")
    n = 40
    g = Engine(n)
    for i in range(n):
        g.configure(i, nw.Config(Network="default", Enable=True,
                                 Default=nw.LinkShape(Latency=5 * nw.Millisecond, Bandwidth=1 << 30)))
    seq = np.zeros(n, dtype=np.uint32)
    with pytest.raises(EngineError) as ei:
        for step in range(6):
            per = np.full(n, 30) if step == 0 else np.zeros(n, dtype=np.int64)
            src = np.repeat(np.arange(n), per)
            pk = np.zeros(len(src), dtype=abi.PKT_DTYPE)
            pk["src"], pk["dst"] = src, (src + 1) % n
            pk["len"], pk["tick"] = 100, 0
            pk["seq"] = np.arange(len(src)) - np.repeat(np.concatenate([[0], np.cumsum(per)[:-1]]), per) + seq[src]
            seq += per.astype(np.uint32)
            g.submit(pk)
            g.step(2000)
        g.sync()
    assert ei.value.code == -errno.ENOSPC and "emit pool" in str(ei.value)
    g.close()
