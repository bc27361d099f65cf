"""Pins the CPU oracle (oracle/tgoracle.c) before it is trusted as the GPU checker.

Known answers come from (a) Random123's published Philox4x32-10 vectors, (b) the reference's own
end-to-end assertions: ping-pong RTT windows (plans/network/pingpong.go:185, :195), the splitbrain
reachability matrix (plans/splitbrain/main.go:50-58), the sidecar's config contract
(pkg/sidecar/docker_network.go:52-55, link.go:143-217, route.go:102-117), and (c) the analytic
netem distributions (uniform jitter, Bernoulli loss) that the reference's kernel path samples.
"""
import ctypes as C
import math

import numpy as np
import pytest

from testground_amd import abi
from testground_amd import network as nw
from testground_amd import workloads as wl
from testground_amd.engine import EngineError, packets

# Random123 kat_vectors, philox4x32 10 rounds: (ctr, key) -> out
PHILOX_KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_philox_known_answers(oracle_lib):
    out = (C.c_uint32 * 4)()
    for ctr, key, want in PHILOX_KAT:
        oracle_lib.tgo_philox4x32_10((C.c_uint32 * 4)(*ctr), (C.c_uint32 * 2)(*key), out)
        assert tuple(out) == want


def test_unit_conversions(oracle_lib):
    lib = oracle_lib
    lib.tgo_to_microseconds.restype = C.c_uint32
    lib.tgo_to_microseconds.argtypes = [C.c_int64]
    lib.tgo_time2tick.restype = C.c_uint32
    lib.tgo_time2tick.argtypes = [C.c_uint32]
    lib.tgo_percentage2u32.restype = C.c_uint32
    lib.tgo_percentage2u32.argtypes = [C.c_float]
    # link.go:143-151
    assert lib.tgo_to_microseconds(100 * nw.Millisecond) == 100_000
    assert lib.tgo_to_microseconds(1999) == 1  # truncation
    assert lib.tgo_to_microseconds(nw.Hour * 2) == 0xFFFFFFFF  # clamp "~1 hour"
    # psched: 15.625 ticks/us, 64 ns/tick: 100 ms -> 100,000,000 ns; 1 us -> 960 ns
    assert lib.tgo_time2tick(100_000) * 64 == 100_000_000
    assert lib.tgo_time2tick(1) * 64 == 960
    assert lib.tgo_percentage2u32(100.0) == 0xFFFFFFFF
    assert lib.tgo_percentage2u32(0.0) == 0
    assert lib.tgo_percentage2u32(50.0) == 0x80000000
    assert abs(lib.tgo_percentage2u32(1.0) - 0.01 * 2**32) < 2**32 * 1e-6


def compiled(oracle_lib, shape):
    out = (C.c_uint64 * 13)()
    oracle_lib.tgo_compile_shape(C.byref(nw.shape_to_c(shape)), out)
    return list(out)


def test_htb_compile_pingpong_shape(oracle_lib):
    c = compiled(oracle_lib, nw.LinkShape(Latency=100 * nw.Millisecond, Bandwidth=1 << 20))
    lat, sigma, rate, mult, shift, burst = c[:6]
    assert lat == 100_000_000 and sigma == 0
    assert rate == (1 << 20) // 8
    cost66 = (66 * mult) >> shift
    assert abs(cost66 - 66e9 / 131072) <= 1  # psched_l2t_ns ~ len * NSEC_PER_SEC / rate
    assert abs(burst - 1600e9 / 131072) < 64 * 16  # (rate/hz + mtu) bytes at rate, tick-rounded


def test_pingpong_rtt_windows(make_oracle):
    """plans/network/pingpong.go:185 (200-215 ms at 100 ms) and :195 (20-35 ms at 10 ms)."""
    e = make_oracle(2, lookahead_ns=1_000_000)
    for i in (0, 1):
        e.configure(i, wl.pingpong_config(100 * nw.Millisecond))
    rtt, now = wl.pingpong_round(e, start_tick=0, seq0=0)
    assert all(200 * nw.Millisecond <= r <= 215 * nw.Millisecond for r in rtt), rtt
    for i in (0, 1):
        e.configure(i, wl.pingpong_config(10 * nw.Millisecond, "latency-reduced"))
    rtt2, _ = wl.pingpong_round(e, start_tick=now + 100_000, seq0=10)
    assert all(20 * nw.Millisecond <= r <= 35 * nw.Millisecond for r in rtt2), rtt2


@pytest.mark.parametrize("case", ["drop", "reject", "accept"])
def test_splitbrain_matrix(make_oracle, case):
    """plans/splitbrain/main.go:50-58: A<->B unreachable for drop/reject, all reachable for accept."""
    n = 60
    e = make_oracle(n)
    ok, art = wl.run_splitbrain(e, n, case)
    exp = wl.splitbrain_expected(n, case)
    assert (ok == exp).all()
    v = art["v_req"] & 15
    region = art["region"]
    src, dst = np.nonzero(~np.eye(n, dtype=bool))
    ab = (region[src] == wl.REGION_A) & (region[dst] == wl.REGION_B)
    want = {"drop": abi.V_BLACKHOLE, "reject": abi.V_PROHIBIT, "accept": abi.V_SCHEDULED}[case]
    assert (v[ab] == want).all()
    assert (v[~ab] == abi.V_SCHEDULED).all()


def test_config_contract(make_oracle):
    e = make_oracle(4)
    with pytest.raises(EngineError, match="unsupported network: bogus"):
        e.configure(0, nw.Config(Network="bogus", Enable=True))
    # Enable=false disconnects; shape/rules are not applied (docker_network.go:65-75)
    e.configure(1, nw.Config(Network="default", Enable=False))
    # external traffic: denied by default / DenyAll, allowed with AllowAll (route.go:102-117)
    e.configure(2, nw.Config(Network="default", Enable=True, RoutingPolicy=nw.RoutingPolicyType.AllowAll))
    # a Drop rule whose prefix carries host bits is rejected by the FIB (EINVAL)
    with pytest.raises(EngineError, match="invalid argument"):
        e.configure(3, nw.Config(Network="default", Enable=True,
                                 Rules=[nw.LinkRule(Subnet=("16.0.0.5", 24), LinkShape=nw.LinkShape(Filter=nw.FilterAction.Drop))]))
    e.submit(packets([(0, 1, 0, 100, 0), (1, 0, 0, 100, 0), (0, abi.EXTERNAL, 1, 100, 0),
                      (2, abi.EXTERNAL, 0, 100, 0), (3, 0, 0, 100, 0)]))
    e.step(10)
    v = e.verdicts() & 15
    assert list(v) == [abi.V_DISCONNECTED, abi.V_DISCONNECTED, abi.V_NO_ROUTE, abi.V_EXTERNAL, abi.V_SCHEDULED]


def test_rules_are_cumulative_and_accept_deletes(make_oracle):
    e = make_oracle(8)
    ip5 = str(__import__("ipaddress").IPv4Address(wl.peer_ip(5)))
    drop = nw.LinkShape(Filter=nw.FilterAction.Drop)
    rej = nw.LinkShape(Filter=nw.FilterAction.Reject)
    e.configure(0, nw.Config(Network="default", Enable=True, Rules=[nw.LinkRule(Subnet="16.0.0.0/29", LinkShape=drop)]))
    e.configure(0, nw.Config(Network="default", Enable=True, Rules=[nw.LinkRule(Subnet=(ip5, 32), LinkShape=rej)]))
    e.submit(packets([(0, d, d, 64, 0) for d in range(1, 8)]))
    e.step(1)
    v = list(e.verdicts() & 15)
    # ips .3.. .7 are inside 16.0.0.0/29 -> blackhole, except .7 (peer 5) -> longest prefix reject
    assert v == [abi.V_BLACKHOLE] * 4 + [abi.V_PROHIBIT] + [abi.V_SCHEDULED] * 2
    e.configure(0, nw.Config(Network="default", Enable=True, Rules=[nw.LinkRule(Subnet="16.0.0.0/29", LinkShape=nw.LinkShape())]))
    e.submit(packets([(0, d, 10 + d, 64, 0) for d in range(1, 8)]))
    e.step(1)
    v = list(e.verdicts() & 15)
    assert v == [abi.V_SCHEDULED] * 4 + [abi.V_PROHIBIT] + [abi.V_SCHEDULED] * 2


def _ks_uniform(x, lo, hi):
    x = np.sort((np.asarray(x, dtype=np.float64) - lo) / (hi - lo))
    n = len(x)
    cdf = np.arange(1, n + 1) / n
    return max(np.max(cdf - x), np.max(x - (cdf - 1 / n)))


def test_netem_distributions(make_oracle):
    """Latency ~ U[L-J, L+J) (KS <= 0.02) and loss within +-0.5 pp of the configured rate."""
    n_pk = 40_000
    e = make_oracle(2, queue_limit=1000)
    shape = nw.LinkShape(Latency=50 * nw.Millisecond, Jitter=10 * nw.Millisecond, Loss=3.0)
    e.configure(0, nw.Config(Network="default", Enable=True, Default=shape))
    # one packet per 65 ticks keeps the 1000-packet netem queue below its limit at <= 60 ms delay
    lost, sent, per, gap = 0, 0, 1000, 65
    for chunk in range(n_pk // per):
        pk = np.zeros(per, dtype=abi.PKT_DTYPE)
        pk["src"], pk["dst"], pk["len"] = 0, 1, 100
        pk["seq"] = np.arange(per) + chunk * per
        pk["tick"] = np.arange(per) * gap
        e.submit(pk)
        e.step(per * gap)
        v = e.verdicts() & 15
        lost += int((v == abi.V_LOSS).sum())
        sent += len(v)
        assert not (v == abi.V_QUEUE_FULL).any()
    e.step(65_000)
    d = e.drain()
    d = d[(d["flags"] & abi.FLAG_DUP) == 0]
    offer_t = d["seq"].astype(np.int64) * gap * 1000
    delays = d["t_ns"].astype(np.int64) - offer_t
    L, J = 50e6, 10e6
    assert delays.min() >= L - J and delays.max() < L + J
    assert _ks_uniform(delays, L - J, L + J) <= 0.02
    assert abs(lost / sent - 0.03) <= 0.005


def test_configure_batch_equals_sequential(make_oracle):
    """tgsim_configure_batch is n tgsim_configure calls: the vectorised records give the same run as
    per-instance Config objects, and a failing record reports its peer and the reference's error."""
    import ctypes

    from testground_amd import network as nw
    from testground_amd import workloads as wl
    n = 120
    a, b = make_oracle(n), make_oracle(n)
    for i, s in enumerate(wl.storm_shapes(n)):
        a.configure(i, nw.Config(Network="default", Enable=True, Default=s,
                                 RoutingPolicy=nw.RoutingPolicyType.DenyAll))
    wl.configure_storm(b, n)
    for e in (a, b):
        e.gen_storm(0.5, 800)
        e.step(800)
    assert (a.verdicts() == b.verdicts()).all() and (a.drain() == b.drain()).all()
    bogus = ctypes.create_string_buffer(b"bogus")
    recs = nw.configs_array([1000, 2000])
    recs["network"][1] = ctypes.addressof(bogus)
    with pytest.raises(Exception, match="peer 7.*unsupported network: bogus"):
        b.configure_batch([3, 7], recs)


@pytest.mark.parametrize("bw,gap_ticks", [(1 << 20, 5000), (10 ** 7, 500), (10 ** 8, 50)])
def test_htb_rate(make_oracle, bw, gap_ticks):
    """Bandwidth (link.go:156-167 -> HTB class rate = Bandwidth/8 B/s): a source offered about
    twice its rate delivers at the configured rate, within 0.5 %, once its burst is spent."""
    e = make_oracle(2)
    e.configure(0, nw.Config(Network="default", Enable=True,
                             Default=nw.LinkShape(Latency=1 * nw.Millisecond, Bandwidth=bw)))
    length = 1250
    step_ticks = 50_000  # 50 ms per step, 12 steps
    per = step_ticks // gap_ticks
    for k in range(12):
        pk = np.zeros(per, dtype=abi.PKT_DTYPE)
        pk["src"], pk["dst"], pk["len"] = 0, 1, length
        pk["seq"] = np.arange(per) + k * per
        pk["tick"] = np.arange(per) * gap_ticks
        e.submit(pk)
        e.step(step_ticks)
    d = e.drain()
    t = np.sort(d["t_ns"].astype(np.int64))
    t = t[t >= 200_000_000]  # steady state: the queue backlog has absorbed the burst
    rate = (len(t) - 1) * length * 8 / ((t[-1] - t[0]) * 1e-9)
    assert abs(rate / bw - 1) <= 0.005, (bw, rate)


def test_netem_event_rates(make_oracle):
    """Duplicate, corrupt and reorder rates within +-0.5 pp of the configured percentages
    (link.go:169-179: the only netem attributes the sidecar sets besides delay and loss)."""
    n_pk, per, gap = 60_000, 1000, 65
    e = make_oracle(2, queue_limit=1000)
    shape = nw.LinkShape(Latency=10 * nw.Millisecond, Duplicate=4.0, Corrupt=6.0, Reorder=8.0)
    e.configure(0, nw.Config(Network="default", Enable=True, Default=shape))
    clones = 0
    for chunk in range(n_pk // per):
        pk = np.zeros(per, dtype=abi.PKT_DTYPE)
        pk["src"], pk["dst"], pk["len"] = 0, 1, 100
        pk["seq"] = np.arange(per) + chunk * per
        pk["tick"] = np.arange(per) * gap
        e.submit(pk)
        e.step(per * gap)
        v = e.verdicts()
        assert not ((v & 15) == abi.V_QUEUE_FULL).any()
        clones += int(((v >> 4) != abi.V_NONE).sum())
    e.step(20_000)
    d = e.drain()
    orig = d[(d["flags"] & abi.FLAG_DUP) == 0]
    assert len(orig) == n_pk
    assert abs(clones / n_pk - 0.04) <= 0.005
    assert abs(float((d["flags"] & abi.FLAG_CORRUPT != 0).mean()) - 0.06) <= 0.005
    delay = orig["t_ns"].astype(np.int64) - orig["seq"].astype(np.int64) * gap * 1000
    # reordered (sent at once) or delayed by L, plus at most the HTB serialisation behind items
    # served at the same instant (100 B at the unlimited class rate of 2^32-1 B/s: 23 ns each)
    now = delay < 1000
    assert (now | ((delay >= 10_000_000) & (delay < 10_001_000))).all(), np.unique(delay)
    assert abs(float(now.mean()) - 0.08) <= 0.005
