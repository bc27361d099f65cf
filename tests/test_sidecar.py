"""The reference's sidecar tests (pkg/sidecar/sidecar_test.go:19-93), restated over the Python mirror,
plus the same flows over SimNetwork: the CPU oracle here, the HIP engine in the gpu variant."""
import threading

import numpy as np
import pytest

from testground_amd import abi
from testground_amd import network as nw
from testground_amd import sidecar as sc
from testground_amd import workloads as wl


def _run(reactor, ctx):
    t = threading.Thread(target=reactor.Handle, args=(ctx, sc.handler), daemon=True)
    t.start()
    return t


def test_network_initialize():
    """sidecar_test.go:20-37: the handler configures the default network exactly once at init."""
    r = sc.MockReactor()
    ctx = sc.Context(timeout=10)
    t = _run(r, ctx)
    sc.NetClient(r.Client, r.RunEnv, r.Hostname).WaitNetworkInitialized(ctx)
    assert len(r.Network.Configured) == 1
    ctx.cancel()
    t.join(5)


def test_network_configured_fails_misconfigured():
    """sidecar_test.go:40-60: a config without CallbackState is rejected with the exact message."""
    r = sc.MockReactor()
    ctx = sc.Context(timeout=10)
    t = _run(r, ctx)
    c = sc.NetClient(r.Client, r.RunEnv, r.Hostname)
    c.WaitNetworkInitialized(ctx)
    with pytest.raises(ValueError, match="^failed to configure network; no callback state provided$"):
        c.ConfigureNetwork(ctx, nw.Config())
    ctx.cancel()
    t.join(5)


def test_network_configured():
    """sidecar_test.go:63-93: a well-formed config reaches the Network unmodified."""
    r = sc.MockReactor()
    ctx = sc.Context(timeout=10)
    t = _run(r, ctx)
    c = sc.NetClient(r.Client, r.RunEnv, r.Hostname)
    c.WaitNetworkInitialized(ctx)
    cfg = nw.Config(Network="default", Enable=True, CallbackState="reconfigured",
                    Default=nw.LinkShape(Latency=nw.Hour))
    before = sc.snapshot(cfg)
    c.ConfigureNetwork(ctx, cfg)
    assert len(r.Network.Configured) == 2
    assert r.Network.Active["default"] == before == cfg
    ctx.cancel()
    t.join(5)


def _sim_flow(engine, n=3):
    """SimReactor over an engine: every instance's handler runs; instance 0 installs a Drop rule for
    instance 1 through network.Client, the callback barrier releases, and the data path obeys."""
    r = sc.SimReactor(engine, n)
    ctx = sc.Context(timeout=30)
    r.Handle(ctx, sc.handler)
    c0 = r.net_client(0)
    c0.WaitNetworkInitialized(ctx)
    import ipaddress
    cfg = nw.Config(Network="default", Enable=True, CallbackState="rules-installed", CallbackTarget=1,
                    Default=nw.LinkShape(Latency=10 * nw.Millisecond),
                    Rules=[nw.LinkRule(Subnet=(str(ipaddress.IPv4Address(wl.peer_ip(1))), 32),
                                       LinkShape=nw.LinkShape(Filter=nw.FilterAction.Drop))])
    c0.ConfigureNetwork(ctx, cfg)
    with pytest.raises(TimeoutError):  # the sidecar rejects an unknown network: no callback comes
        r.net_client(2).ConfigureNetwork(sc.Context(timeout=0.5),
                                         nw.Config(Network="bogus", Enable=True, CallbackState="never"))
    ctx.cancel()
    r.Close()
    # the handler's states went through the engine's sync counters (K7)
    assert isinstance(r.Client, sc.EngineSyncClient)
    assert engine.barrier_poll(r.Client.state_id(sc.NET_INIT_STATE), n)
    assert not engine.barrier_poll(r.Client.state_id(sc.NET_INIT_STATE), n + 1)
    assert engine.barrier_poll(r.Client.state_id("rules-installed"), 1)
    assert any("failed to update network bogus: " in str(e) and "unsupported network: bogus" in str(e)
               for e in r.errors), r.errors
    engine.submit(np.array([(0, 1, 0, 100, 0), (0, 2, 1, 100, 0)], dtype=abi.PKT_DTYPE))
    engine.step(20_000)
    v = engine.verdicts() & 15
    d = engine.drain()
    assert list(v) == [abi.V_BLACKHOLE, abi.V_SCHEDULED]
    assert len(d) == 1 and d[0]["dst"] == 2 and d[0]["t_ns"] == 10 * nw.Millisecond


def test_sim_network_over_oracle(make_oracle):
    _sim_flow(make_oracle(3))


@pytest.mark.gpu
def test_sim_network_over_engine():
    from testground_amd.engine import Engine
    _sim_flow(Engine(3))


def test_publish_delivers_a_copy():
    """sdk-go serialises published payloads: a publisher changing its object afterwards does not
    change what subscribers (or the sidecar, via ConfigureNetwork) see."""
    from testground_amd import network as nw
    from testground_amd.sidecar import Context, SyncClient

    c = SyncClient()
    cfg = nw.Config(Network="default", Enable=True, Default=nw.LinkShape(Latency=5))
    c.Publish(Context(), "t", cfg)
    cfg.Default.Latency = 99
    assert c.Subscribe(Context(), "t").get_nowait().Default.Latency == 5


def test_configure_network_passes_a_copy_to_the_sidecar():
    import threading

    from testground_amd import network as nw
    from testground_amd.sidecar import Context, MockReactor, NetClient, handler

    r = MockReactor()
    ctx = Context(timeout=10)
    t = threading.Thread(target=r.Handle, args=(ctx, handler), daemon=True)
    t.start()
    nc = NetClient(r.Client, r.RunEnv, r.Hostname)
    nc.WaitNetworkInitialized(ctx)
    cfg = nw.Config(Network="default", Enable=True, Default=nw.LinkShape(Latency=7), CallbackState="a")
    nc.ConfigureNetwork(ctx, cfg)
    cfg.Default.Latency = 1234
    assert r.Network.Active["default"].Default.Latency == 7
    ctx.cancel()
    t.join(5)


def test_engine_sync_client_beyond_engine_slots(make_oracle):
    """More distinct states than the engine holds (one callback state per instance): the extra
    states live in the client's in-memory counters; a sharded client refuses them clearly."""
    import pytest

    from testground_amd.sidecar import Context, EngineSyncClient

    e = make_oracle(2)
    c = EngineSyncClient(e, n_slots=1024)
    ctx = Context()
    for i in range(1100):
        assert c.SignalEntry(ctx, f"reconfigured{i}") == 1
    assert c.SignalEntry(ctx, "reconfigured1099") == 2
    c.Barrier(ctx, "reconfigured1099", 2)
    assert c._reached("reconfigured5", 1) and not c._reached("reconfigured5", 2)
    sharded = EngineSyncClient(e, n_slots=2, reduce=lambda sid, t: True)
    sharded.SignalEntry(ctx, "a")
    sharded.SignalEntry(ctx, "b")
    with pytest.raises(RuntimeError, match="engine sync counters"):
        sharded.SignalEntry(ctx, "c")
