"""Synthetic equivalents of the reference's network workloads (SURVEY §8(d) C1–C3).

Each driver talks to an engine-shaped object (``Engine`` or any ``CABIEngine``), so the same
driver runs the HIP engine on the GPU and, in the tests, the CPU oracle with identical inputs.

  C1 pingpong    plans/network/pingpong.go:16-201 (RTT windows :185, :195)
  C2 splitbrain  plans/splitbrain/main.go:60-186 (expectErrors :50-58)
  C3 storm       plans/benchmarks/storm.go:31-197, random all-to-all with heterogeneous shapes
  C4 gossip      SURVEY §8(d): 1M-peer flood, degree 8, 1 KiB messages, L~U[5,50] ms, loss 1 %
  C5 epochs      SURVEY §8(d): C3 traffic, mid-run reshaping of 10 % of peers per epoch, barriers

A reaction to a delivery at time d (reply, echo, forward) is offered at tick floor(d/tick) + 1.
"""
from __future__ import annotations

import ipaddress
from typing import Dict, List, Tuple

import numpy as np

from . import abi
from .network import Config, FilterAction, LinkRule, LinkShape, Millisecond, RoutingPolicyType, configs_array

SEED = 0x7E576A0D00000001


# ---------------------------------------------------------------------------------------------
# C3: storm — heterogeneous LinkShape per instance.
def storm_shape_arrays(n_peers: int, seed: int = SEED) -> Dict[str, np.ndarray]:
    """L~U[1,100] ms, J~U[0,10] ms, Loss~U[0,5] %, Dup/Corrupt/Reorder~U[0,1] %,
    Bw in {1,10,100,1000} Mbit/s, correlations 0."""
    rng = np.random.default_rng(seed & 0xFFFFFFFF)
    lat = rng.integers(1 * Millisecond, 100 * Millisecond + 1, n_peers)
    jit = rng.integers(0, 10 * Millisecond + 1, n_peers)
    loss = rng.uniform(0, 5, n_peers).astype(np.float32)
    dup = rng.uniform(0, 1, n_peers).astype(np.float32)
    cor = rng.uniform(0, 1, n_peers).astype(np.float32)
    reo = rng.uniform(0, 1, n_peers).astype(np.float32)
    bw = rng.choice(np.array([1, 10, 100, 1000], dtype=np.int64) * 1_000_000, n_peers)
    return dict(latency_ns=lat, jitter_ns=jit, bandwidth_bps=bw, loss=loss, duplicate=dup, corrupt=cor,
                reorder=reo)


def storm_shapes(n_peers: int, seed: int = SEED) -> List[LinkShape]:
    a = storm_shape_arrays(n_peers, seed)
    return [LinkShape(Latency=int(a["latency_ns"][i]), Jitter=int(a["jitter_ns"][i]),
                      Bandwidth=int(a["bandwidth_bps"][i]), Loss=float(a["loss"][i]),
                      Duplicate=float(a["duplicate"][i]), Corrupt=float(a["corrupt"][i]),
                      Reorder=float(a["reorder"][i]))
            for i in range(n_peers)]


def storm_configs(n_peers: int, seed: int = SEED, open_links: bool = False) -> np.ndarray:
    """The storm shapes as tgsim_config records (RoutingPolicy DenyAll), for configure_batch.
    open_links: the sub-capacity variant, every link at 1 Gbit/s (latency, jitter, loss, dup,
    corrupt, reorder unchanged), driven at STORM_OPEN_LAMBDA so no netem queue reaches its limit."""
    a = storm_shape_arrays(n_peers, seed)
    if open_links:
        a["bandwidth_bps"] = np.full(n_peers, 1_000_000_000, dtype=np.int64)
    return configs_array(routing_policy=2, **a)


# Sub-capacity C3: 0.008 packets per us per source of U[64,1500] B is ~50 Mbit/s offered against
# 1 Gbit/s, and the netem queue holds lambda * (L + J) <= 0.008 * 110,000 us = 880 items at the very
# worst shape (~440 on average) against the limit of 1,000: the delay, HTB and delivery path is
# exercised, not the full-queue ballot.
STORM_OPEN_LAMBDA = 0.008


def configure_storm(eng, n_peers: int, seed: int = SEED, open_links: bool = False) -> None:
    eng.configure_batch(np.arange(n_peers), storm_configs(n_peers, seed, open_links))


# ---------------------------------------------------------------------------------------------
# C2: splitbrain.
REGION_A, REGION_B, REGION_C = 0, 1, 2


def splitbrain_regions(n: int) -> np.ndarray:
    """seq = i + 1 (SignalEntry is 1-based), region = seq % 3 (splitbrain/main.go:84-87)."""
    return (np.arange(n) + 1) % 3


def expect_errors(case: str, ra: int, rb: int) -> bool:
    """splitbrain/main.go:50-58."""
    if case == "accept" or ra == REGION_C or rb == REGION_C:
        return False
    return (ra == REGION_A and rb == REGION_B) or (ra == REGION_B and rb == REGION_A)


def peer_ip(i: int, subnet_base: int = 16 << 24) -> int:
    return subnet_base + 2 + i


def configure_splitbrain(eng, n: int, case: str) -> np.ndarray:
    action = {"drop": FilterAction.Drop, "reject": FilterAction.Reject, "accept": FilterAction.Accept}[case]
    region = splitbrain_regions(n)
    b_peers = np.nonzero(region == REGION_B)[0]
    for i in np.nonzero(region == REGION_A)[0]:
        rules = [LinkRule(Subnet=(str(ipaddress.IPv4Address(peer_ip(int(p)))), 32),
                          LinkShape=LinkShape(Filter=action)) for p in b_peers]
        eng.configure(int(i), Config(Network="default", Enable=True, Rules=rules,
                                     CallbackState=f"reconfigured{i}", CallbackTarget=1))
    return region


def run_splitbrain(eng, n: int, case: str, pkt_len: int = 66, gap: int = 8) -> Tuple[np.ndarray, Dict]:
    """Every instance contacts every other instance once, sequentially (one request every `gap`
    ticks, as the plan's `for _, p := range nodes { httpclient.Get(...) }`, main.go:159-175), and
    every delivered request is answered.  Replies run in a second window on the same relative time
    axis (reply tick = floor(d / tick) + 1).  Returns ok[i, j] = request i->j and its reply j->i
    both delivered, plus the step artifacts."""
    region = configure_splitbrain(eng, n, case)
    src, dst = np.nonzero(~np.eye(n, dtype=bool))
    k = dst - (dst > src)  # per-source request index 0..n-2
    req = np.zeros(len(src), dtype=abi.PKT_DTYPE)
    req["src"], req["dst"], req["len"] = src, dst, pkt_len
    req["seq"], req["tick"] = k, k * gap
    span = (n - 1) * gap
    t0 = eng.stats()["now_tick"]
    eng.submit(req)
    eng.step(span)
    v_req = eng.verdicts()
    d_req = eng.drain()
    tick = eng.tick_ns
    rep = np.zeros(len(d_req), dtype=abi.PKT_DTYPE)
    rep["src"], rep["dst"], rep["len"] = d_req["dst"], d_req["src"], pkt_len
    rep["seq"] = (n - 1) + d_req["src"]  # fresh per-source sequence numbers
    rep["tick"] = (d_req["t_ns"] // tick + 1) - t0
    eng.submit(rep)
    eng.step(span + 2)
    v_rep = eng.verdicts()
    d_rep = eng.drain()
    ok = np.zeros((n, n), dtype=bool)
    ok[d_rep["dst"], d_rep["src"]] = True  # reply j->i delivered to i => i->j round trip ok
    return ok, {"region": region, "v_req": v_req, "d_req": d_req, "v_rep": v_rep, "d_rep": d_rep}


def splitbrain_expected(n: int, case: str) -> np.ndarray:
    region = splitbrain_regions(n)
    exp = np.zeros((n, n), dtype=bool)
    for i in range(n):
        for j in range(n):
            if i != j:
                exp[i, j] = not expect_errors(case, int(region[i]), int(region[j]))
    return exp


# ---------------------------------------------------------------------------------------------
# C1: ping-pong (2 instances).
def pingpong_config(latency_ns: int, callback: str = "network-configured", ipv4=None) -> Config:
    """pingpong.go:29-42 (and :61-65 for the re-addressing)."""
    return Config(Network="default", Enable=True, IPv4=ipv4,
                  Default=LinkShape(Latency=latency_ns, Bandwidth=1 << 20),
                  CallbackState=callback, RoutingPolicy=RoutingPolicyType.DenyAll)


def pingpong_round(eng, start_tick: int, seq0: int, pkt_len: int = 66, chunk: int = 1000,
                   max_ticks: int = 2_000_000) -> Tuple[List[int], int]:
    """One pingPong() exchange (pingpong.go:116-183): both sides write their id at start_tick,
    echo the other's id on receipt, and stop when their own id comes back.  The engine must have
    lookahead >= chunk ticks.  Returns (rtt_ns per instance, next free tick)."""
    tick = eng.tick_ns
    now = eng.stats()["now_tick"]
    assert now <= start_tick
    if start_tick > now:
        eng.step(start_tick - now)
        eng.drain()
        now = start_tick
    pending: List[tuple] = [(0, 1, seq0, pkt_len, 0), (1, 0, seq0, pkt_len, 0)]  # (src,dst,seq,len,abs tick)
    pending = [(s, d, q, l, start_tick) for (s, d, q, l, _) in pending]
    rtt = [None, None]
    while None in rtt and now - start_tick < max_ticks:
        window = [p for p in pending if now <= p[4] < now + chunk]
        pending = [p for p in pending if p[4] >= now + chunk]
        if window:
            arr = np.array([(s, d, q, l, t - now) for (s, d, q, l, t) in window], dtype=abi.PKT_DTYPE)
            eng.submit(arr)
        eng.step(chunk)
        now += chunk
        for r in eng.drain():
            dst, src, t = int(r["dst"]), int(r["src"]), int(r["t_ns"])
            react = t // tick + 1
            if int(r["seq"]) == seq0:  # the other's id arrived: echo it back
                pending.append((dst, src, seq0 + 1 + dst, pkt_len, react))
            elif rtt[dst] is None:  # own id came back
                rtt[dst] = t - start_tick * tick
    return rtt, now


# ---------------------------------------------------------------------------------------------
# C4: gossip flood.  The engine generates and consumes the traffic on the device
# (tgsim_gossip_init / tgsim_gen_gossip); this module only shapes the peers and runs windows.
GOSSIP_MIN_LAT = 5 * Millisecond


def gossip_shapes(n_peers: int, seed: int = SEED) -> Tuple[np.ndarray, float]:
    """Per-peer latency L~U[5,50] ms in whole microseconds (what toMicroseconds keeps), loss 1 %."""
    rng = np.random.default_rng((seed >> 32) & 0xFFFFFFFF)
    lat_us = rng.integers(5_000, 50_001, n_peers)
    return lat_us * 1000, 1.0


def configure_gossip(eng, n_peers: int, seed: int = SEED) -> None:
    lat, loss = gossip_shapes(n_peers, seed)
    eng.configure_batch(np.arange(n_peers), configs_array(lat, loss=loss))


def gossip_window_ticks(eng) -> int:
    """The largest window whose receipts are all known before the next window: the engine serves
    items eligible before T_end + lookahead, so lookahead = window = the minimum latency."""
    return GOSSIP_MIN_LAT // eng.tick_ns


def gossip_run(eng, n_windows: int, window: int, collect: bool = True):
    """Runs n_windows gossip windows; returns per-window (verdicts, deliveries) when collect."""
    out = []
    for _ in range(n_windows):
        eng.gen_gossip(window)
        eng.step(window)
        if collect:
            out.append((eng.verdicts(), eng.drain()))
    return out


# ---------------------------------------------------------------------------------------------
# C5: epochs of C3 traffic with mid-run reshaping and a barrier per epoch.
EPOCH_TICKS = 1000
EPOCH_LAMBDA = 0.2
EPOCH_RESHAPE_FRAC = 0.1


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)).astype(np.uint64)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def epoch_selection(n_peers: int, epoch: int, frac: float = EPOCH_RESHAPE_FRAC, seed: int = SEED) -> np.ndarray:
    """Peers reshaped at the start of `epoch` (hash-selected, ~frac of all peers)."""
    with np.errstate(over="ignore"):
        x = _splitmix64(np.arange(n_peers, dtype=np.uint64) ^ np.uint64((seed ^ (epoch << 40)) & (2**64 - 1)))
    return np.nonzero((x >> np.uint64(32)) < np.uint64(int(frac * 2**32)))[0].astype(np.uint32)


def epoch_plan(n_peers: int, epoch: int, seed: int = SEED) -> Tuple[np.ndarray, np.ndarray]:
    """What epoch `epoch`'s plan asks for: the reshaped peers and their fresh C3-style configs."""
    sel = epoch_selection(n_peers, epoch, seed=seed)
    return sel, storm_configs(len(sel), (seed + 0x1000 * (epoch + 1)) & 0xFFFFFFFF)


def epoch_reshape(eng, n_peers: int, epoch: int, seed: int = SEED, plan=None) -> int:
    """Fresh C3-style shapes for the epoch's selected peers; every shard receives every call.
    plan: epoch_plan's output computed ahead (the bench keeps the plan's own work out of the timed
    loop, as it does the traffic; the ConfigureNetwork calls stay in it)."""
    sel, cfg = plan if plan is not None else epoch_plan(n_peers, epoch, seed)
    eng.configure_batch(sel, cfg)
    return len(sel)


def epoch_state(epoch: int) -> Tuple[int, int]:
    """Sync state id of barrier `epoch-k` and the round of that id (epochs cycle over 1024 of the
    engine's sync counters, so a long run keeps reusing the same few)."""
    return epoch % 1024, epoch // 1024 + 1


def run_epoch(eng, n_peers: int, epoch: int, n_local: int, step=None, barrier=None,
              lam: float = EPOCH_LAMBDA, ticks: int = EPOCH_TICKS, seed: int = SEED) -> None:
    """One C5 epoch: reshape (from epoch 1), traffic window, then every local peer signals
    `epoch-k` and the barrier must release with all n_peers signals (summed over shards)."""
    if epoch:
        epoch_reshape(eng, n_peers, epoch, seed)
    eng.gen_storm(lam, ticks)
    (step or eng.step)(ticks)
    state, rnd = epoch_state(epoch)
    eng.signal_async(state, n_local)
    ok = barrier(state, rnd * n_peers) if barrier else eng.barrier_poll(state, rnd * n_peers)
    if not ok:
        raise RuntimeError(f"barrier epoch-{epoch} did not release")


# ---------------------------------------------------------------------------------------------
# C6: bridge — real payloads through the native packet bridge: every
# instance sends BRIDGE_PER_WINDOW datagrams per window to random peers.
BRIDGE_PER_WINDOW = 16


def bridge_shape_arrays(n_peers: int, seed: int = SEED) -> Dict[str, np.ndarray]:
    """L~U[1,10] ms, J~U[0,1] ms, loss/dup/corrupt 1 %, 1 Gbit/s."""
    rng = np.random.default_rng((seed >> 16) & 0xFFFFFFFF)
    return dict(latency_ns=rng.integers(1 * Millisecond, 10 * Millisecond + 1, n_peers),
                jitter_ns=rng.integers(0, 1 * Millisecond + 1, n_peers),
                bandwidth_bps=np.full(n_peers, 1_000_000_000, dtype=np.int64),
                loss=np.full(n_peers, 1.0, np.float32), duplicate=np.full(n_peers, 1.0, np.float32),
                corrupt=np.full(n_peers, 1.0, np.float32))


def configure_bridge(eng, n_peers: int, seed: int = SEED) -> None:
    eng.configure_batch(np.arange(n_peers), configs_array(**bridge_shape_arrays(n_peers, seed)))


def bridge_traffic(n_peers: int, per_instance: int = BRIDGE_PER_WINDOW, seed: int = SEED):
    """One window of sends: (src, dst, payload bytes, offsets); payloads of U[64,512] bytes."""
    rng = np.random.default_rng(seed & 0xFFFF)
    src = np.repeat(np.arange(n_peers, dtype=np.uint32), per_instance)
    dst = ((src + 1 + rng.integers(0, n_peers - 1, len(src))) % n_peers).astype(np.uint32)
    lens = rng.integers(64, 513, len(src))
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    return src, dst, rng.bytes(int(off[-1])), off
